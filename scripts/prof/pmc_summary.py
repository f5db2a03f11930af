"""Summarise a rocprofv3 --pmc counter_collection.csv: mean of each counter per kernel.

usage: python scripts/prof/pmc_summary.py <run_counter_collection.csv> [name-filter]
Prints kernel, dispatches, counters (and L2 hit rate / effective clock when present).
"""
import csv
import re
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    per = defaultdict(lambda: defaultdict(list))
    dur = {}
    for r in rows:
        name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("can::", "")
        if filt not in name:
            continue
        key = (name, r["Dispatch_Id"])
        per[name][r["Counter_Name"]].append((r["Dispatch_Id"], float(r["Counter_Value"])))
        if "End_Timestamp" in r:
            dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    for name, cs in per.items():
        out = {c: sum(v for _, v in vals) / len(vals) for c, vals in cs.items()}
        n = len(next(iter(cs.values())))
        extra = ""
        if "TCC_HIT_sum" in out and "TCC_MISS_sum" in out:
            extra += f" L2hit={out['TCC_HIT_sum'] / max(1.0, out['TCC_HIT_sum'] + out['TCC_MISS_sum']):.3f}"
        if "GRBM_GUI_ACTIVE" in out:
            ds = [dur[(name, d)] for d, _ in cs["GRBM_GUI_ACTIVE"] if (name, d) in dur]
            if ds:
                extra += f" clk={out['GRBM_GUI_ACTIVE'] / 8 / (sum(ds) / len(ds)) / 1e9:.2f}GHz"
        print(f"{name[:48]:48s} n={n:3d} " + " ".join(f"{c}={v:.4g}" for c, v in out.items()) + extra)


if __name__ == "__main__":
    main()
