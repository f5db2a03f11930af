"""Export a rocprofv3 SQLite (rocpd) result database to the CSV files the other profile scripts read.

usage: python scripts/prof/rocpd_to_csv.py <results.db> <out_prefix>
writes <out_prefix>_kernel_trace.csv (one row per dispatch, rocprofv3 --output-format csv column names)
and <out_prefix>_kernel_stats.csv (per kernel name: calls, total / average / min / max ns, share).
rocprofv3 on this image writes only the database unless --output-format csv is given.
"""
import csv
import sqlite3
import sys


def main():
    db, prefix = sys.argv[1], sys.argv[2]
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end, grid_x, workgroup_x, stream_id, lds_size, vgpr_count, "
                     "accum_vgpr_count from kernels order by start").fetchall()
    with open(prefix + "_kernel_trace.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Grid_Size_X", "Workgroup_Size_X",
                    "Stream_Id", "LDS_Block_Size", "VGPR_Count", "Accum_VGPR_Count"])
        w.writerows(rows)
    agg = {}
    for name, s, e, *_ in rows:
        d = e - s
        a = agg.setdefault(name, [0, 0, d, d])
        a[0] += 1; a[1] += d; a[2] = min(a[2], d); a[3] = max(a[3], d)
    tot = sum(a[1] for a in agg.values()) or 1
    with open(prefix + "_kernel_stats.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, (n, t, mn, mx) in sorted(agg.items(), key=lambda x: -x[1][1]):
            w.writerow([name, n, t, f"{t / n:.1f}", f"{100 * t / tot:.2f}", mn, mx])
    print(f"{len(rows)} dispatches, {len(agg)} kernels, {tot / 1e6:.3f} ms kernel time")


if __name__ == "__main__":
    main()
