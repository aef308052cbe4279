"""Turn rocprofv3 --pmc CSVs into HBM bytes per launch (profiles/traffic.json).

    python tools/pmc_traffic.py <fetch_dir> <write_dir> [--out profiles/traffic.json]

Counters (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE are in KiB and
come from separate passes (TCC slots).  On gfx950 FETCH_SIZE reads 1/2 of the
bytes of a wide coalesced stream; the guide says to calibrate on a known byte
count, so the probe's first dispatch copies exactly 1 GiB and the read
correction factor is 1 GiB / (FETCH_SIZE of that copy).  WRITE_SIZE is exact
for 16-B-per-lane stores; its own calibration factor is reported too.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def read_counters(d, counter):
    rows = []
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                rows.append((int(row.get("Dispatch_Id", 0)), row["Kernel_Name"],
                             float(row["Counter_Value"])))
    # sum over dimension instances of one dispatch
    agg = defaultdict(float)
    names = {}
    for did, name, val in rows:
        agg[did] += val
        names[did] = name
    return [(did, names[did], agg[did]) for did in sorted(agg)]


def per_kernel(rows, key):
    vals = [v for _, n, v in rows if key in n]
    return sum(vals) / len(vals) if vals else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--config", default="sceneflow")
    ap.add_argument("--out", default="profiles/traffic.json")
    a = ap.parse_args()
    fr = read_counters(a.fetch_dir, "FETCH_SIZE")
    wr = read_counters(a.write_dir, "WRITE_SIZE")
    GiB = float(1 << 30)
    cal_f = [v for _, n, v in fr if "build" not in n and "lookup" not in n and v * 1024 > GiB / 4]
    cal_w = [v for _, n, v in wr if "build" not in n and "lookup" not in n and v * 1024 > GiB / 4]
    kf = GiB / (cal_f[0] * 1024) if cal_f else 2.0
    kw = GiB / (cal_w[0] * 1024) if cal_w else 1.0
    res = {}
    for kname, key in (("build", "build_"), ("lookup", "lookup_kernel"),
                       ("lookup_chain", "lookup_chain_kernel"), ("lookup_pair", "lookup_pair_kernel"),
                       ("lookup_bwd", "lookup_bwd_pre_kernel"),
                       ("lookup_bwd_pair", "lookup_bwd_pair_kernel")):
        f = per_kernel(fr, key)
        w = per_kernel(wr, key)
        if f is None or w is None:
            continue
        res[f"{kname}_fetch_bytes_raw"] = f * 1024
        res[f"{kname}_write_bytes_raw"] = w * 1024
        res[f"{kname}_bytes"] = f * 1024 * kf + w * 1024 * kw
    res["fetch_calibration"] = kf
    res["write_calibration"] = kw
    res["note"] = ("per-launch HBM-side bytes: FETCH_SIZE*1024*fetch_calibration + "
                   "WRITE_SIZE*1024*write_calibration; calibration = 1 GiB torch clone in the "
                   "same process (MI355X_MICROARCH.md §HBM). Infinity-Cache hits are counted.")
    out = {}
    if os.path.exists(a.out):
        with open(a.out) as fh:
            out = json.load(fh)
    out[a.config] = res
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
