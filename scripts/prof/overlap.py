"""Step-level concurrency summary of a kernel trace: span, busy per stream, chip-idle time (no kernel running),
and time with 2+ kernels resident.  usage: overlap.py <kernel_trace.csv> [marker=sgd_momentum]"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "sgd_momentum"
    rows = list(csv.DictReader(open(path)))
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    step = rows[idx[-2] + 1: idx[-1] + 1]
    busy = defaultdict(float)
    ev = []
    for r in step:
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        busy[r["Stream_Id"]] += (b - a) / 1e3
        ev += [(a, 1), (b, -1)]
    ev.sort()
    t0, t1 = ev[0][0], ev[-1][0]
    depth, last, idle, multi = 0, t0, 0, 0
    for t, d in ev:
        if depth == 0:
            idle += t - last
        elif depth >= 2:
            multi += t - last
        depth += d
        last = t
    print(f"span {(t1 - t0) / 1e3:.1f} us  kernels {len(step)}  busy/stream " +
          " ".join(f"{k}:{v:.1f}" for k, v in sorted(busy.items())) +
          f"  chip-idle {idle / 1e3:.1f} us  2+ kernels {multi / 1e3:.1f} us")


if __name__ == "__main__":
    main()
