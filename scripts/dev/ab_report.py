"""Summarise gpurun_out/ab_*.log: per (layer, pass) median ms old vs new, and the bench medians."""
import glob
import json
import re
import statistics
from collections import defaultdict

t = defaultdict(lambda: defaultdict(list))
for f in glob.glob("gpurun_out/ab_old_*.log") + glob.glob("gpurun_out/ab_new_*.log"):
    side = "old" if "ab_old_" in f else "new"
    for line in open(f):
        m = re.match(r"(\w+)\s+(fwd|dgrad|wgrad)\s+ours\s+([\d.]+) ms", line)
        if m:
            t[(m.group(1), m.group(2))][side].append(float(m.group(3)))
tot = {"old": 0.0, "new": 0.0}
for k in sorted(t):
    o, n = statistics.median(t[k]["old"]), statistics.median(t[k]["new"])
    tot["old"] += o
    tot["new"] += n
    print(f"{k[0]:4s} {k[1]:6s} old {o:7.3f} new {n:7.3f}  {100 * (n / o - 1):+6.1f}%")
print(f"total old {tot['old']:.3f} new {tot['new']:.3f} ({100 * (tot['new'] / max(tot['old'], 1e-9) - 1):+.1f}%)")
b = defaultdict(list)
for f in glob.glob("gpurun_out/ab_bench_*.log"):
    side = "old" if "_old_" in f else "new"
    for line in open(f):
        if line.startswith("{"):
            b[side].append(json.loads(line)["value"])
print("bench img/s old", sorted(b["old"]), "new", sorted(b["new"]))
