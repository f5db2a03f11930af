"""Register / spill report of one HIP source for gfx950: python scripts/dev/regs.py <file.hip> [name-filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-x", "hip", "-c", src, "-o", "/tmp/_regs.o", "-O3",
                    "-std=c++17", "-I" + src.rsplit("/", 1)[0], "-Rpass-analysis=kernel-resource-usage"],
                   capture_output=True, text=True)
cur = None
info = {}
for line in r.stderr.splitlines():
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        info[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z /\[\]]+): (\S+)", line)
    if m and cur:
        info[cur][m.group(1).strip()] = m.group(2)
for k, v in info.items():
    if flt in k:
        print(f"{k[:90]:90s} vgpr {v.get('VGPRs')} agpr {v.get('AGPRs')} spill {v.get('VGPRs Spill')} "
              f"scratch {v.get('ScratchSize [bytes/lane]')} occ {v.get('Occupancy [waves/SIMD]')}")
