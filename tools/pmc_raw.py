"""Mean per dispatch of every rocprofv3 counter, per kernel.

    python tools/pmc_raw.py <pmc_dir> [--width N]   (kernel-name characters kept, default 48)
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d, width=48):
    agg = defaultdict(lambda: defaultdict(float))
    names, times = {}, {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            k = int(r["Dispatch_Id"])
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            names[k] = r["Kernel_Name"].split("(")[0][:width]
            times[k] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    per = defaultdict(list)
    for k in sorted(agg):
        per[names[k]].append((agg[k], times[k]))
    for name, rows in per.items():
        n = len(rows)
        c = {key: sum(r[0].get(key, 0.0) for r in rows) / n for key in rows[0][0]}
        t = sum(r[1] for r in rows) / n
        print(f"{name} n={n} t={t * 1e6:.1f}us " + " ".join(f"{k}={v:.4g}" for k, v in sorted(c.items())))


if __name__ == "__main__":
    w = int(sys.argv[sys.argv.index("--width") + 1]) if "--width" in sys.argv else 48
    main(sys.argv[1], w)
