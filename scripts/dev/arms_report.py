"""Summarise gpurun_out/arm<i>_<round>.log (scripts/gpu/ab_convs_multi.sh): median ms per (layer, pass) per arm."""
import glob
import re
import statistics
import sys
from collections import defaultdict

t = defaultdict(lambda: defaultdict(list))
for f in glob.glob("gpurun_out/arm*_*.log"):
    arm = int(re.search(r"arm(\d+)_", f).group(1))
    for line in open(f):
        m = re.match(r"(\w+)\s+(fwd|dgrad|wgrad)\s+ours\s+([\d.]+) ms", line)
        if m:
            t[(m.group(1), m.group(2))][arm].append(float(m.group(3)))
arms = sorted({a for v in t.values() for a in v})
names = sys.argv[1:] or [f"arm{a}" for a in arms]
print("layer  pass   " + " ".join(f"{n:>12s}" for n in names))
tot = defaultdict(float)
for k in sorted(t):
    meds = [statistics.median(t[k][a]) for a in arms]
    for a, m in zip(arms, meds):
        tot[a] += m
    print(f"{k[0]:6s} {k[1]:6s} " + " ".join(f"{m:12.3f}" for m in meds))
print("total         " + " ".join(f"{tot[a]:12.3f}" for a in arms))

b = defaultdict(list)
import json  # noqa: E402
for f in glob.glob("gpurun_out/barm*_*.log"):
    arm = int(re.search(r"barm(\d+)_", f).group(1))
    for line in open(f):
        if line.startswith("{"):
            b[arm].append(json.loads(line)["value"])
for a in sorted(b):
    nm = names[a] if a < len(names) else f"arm{a}"
    print(f"bench {nm:>12s} img/s " + " ".join(f"{v:.1f}" for v in sorted(b[a])) + f"  median {statistics.median(b[a]):.1f}")
