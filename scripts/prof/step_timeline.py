"""Per-step kernel timeline from a rocprofv3 kernel trace CSV.

usage: python scripts/prof/step_timeline.py <run_kernel_trace.csv> [marker-kernel]
Splits the trace into steps at each launch of the marker kernel (default: the
fused SGD kernel, the last kernel of a step), prints the last full step's
kernels in order with duration, gap before it and grid size, plus totals.
"""
import csv
import re
import sys


def short(name):
    name = re.sub(r"\(.*", "", name)
    name = name.replace("void ", "").replace("can::", "")
    return name[:60]


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "sgd_momentum"
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    if len(ends) < 2:
        print("not enough steps"); return
    step = rows[ends[-2] + 1: ends[-1] + 1]
    t0 = int(step[0]["Start_Timestamp"])
    prev_end = int(rows[ends[-2]]["End_Timestamp"])
    busy = 0
    agg = {}
    for r in step:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        d = (e - s) / 1e3
        busy += d
        gap = (s - prev_end) / 1e3
        prev_end = e
        n = short(r["Kernel_Name"])
        agg[n] = agg.get(n, 0) + d
        print(f"{(s - t0) / 1e3:9.1f} {d:8.1f} us gap {gap:6.1f}  grid {int(r['Grid_Size_X']) // max(1, int(r['Workgroup_Size_X'])):6d}x{r['Workgroup_Size_X']:>4}  {n}")
    span = (int(step[-1]["End_Timestamp"]) - t0) / 1e3
    print(f"\nstep span {span:.1f} us, kernel busy {busy:.1f} us, idle {span - busy:.1f} us, {len(step)} kernels")
    for n, d in sorted(agg.items(), key=lambda x: -x[1]):
        print(f"{d:9.1f} us {100 * d / busy:5.1f}%  {n}")


if __name__ == "__main__":
    main()
