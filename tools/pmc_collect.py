"""rocprofv3 --pmc runs of bench.py -> profiles/pmc.json (per config, per kernel).

    python tools/pmc_collect.py <config> <fetch_dir> <write_dir> <sq_dir> [--out profiles/pmc.json]
                                [--tag r03]

The three directories come from three separate passes of the SAME command
(``bench.py --config <config> --pmc-calibrate ...``: the counters do not fit
one pass), e.g.

    rocprofv3 --pmc FETCH_SIZE -d <fetch_dir> -- python3 bench.py --config sceneflow --pmc-calibrate ...
    rocprofv3 --pmc WRITE_SIZE -d <write_dir> -- python3 bench.py ...
    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES -d <sq_dir> -- ...

so every entry describes a kernel exactly as bench.py launches it for that
config.  Per kernel (name without "void " and the argument list) and per
dispatch on average:
  hbm_bytes  = FETCH_SIZE * 1024 * fetch_cal + WRITE_SIZE * 1024 * write_cal,
             the calibration factors from the 1 GiB torch clone that
             --pmc-calibrate runs first (MI355X_MICROARCH.md §HBM: FETCH_SIZE
             reads 1/2 of a wide coalesced stream on gfx950);
  mfma_util  = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs * GRBM_GUI_ACTIVE / 8);
  clock_ghz  = GRBM_GUI_ACTIVE / 8 / duration.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def kernel_key(name):
    name = name.strip()
    if name.startswith("void "):
        name = name[5:]
    depth, out = 0, []
    for ch in name:            # drop the argument list, keep template arguments
        if ch == "(" and depth == 0:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out.append(ch)
    return "".join(out).strip()


def read(d):
    """{dispatch: (kernel, {counter: value summed over instances}, seconds)}"""
    rows = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as fh:
            for r in csv.DictReader(fh):
                k = int(r["Dispatch_Id"])
                name, cnt, t = rows.get(k, (kernel_key(r["Kernel_Name"]), defaultdict(float), 0.0))
                cnt[r["Counter_Name"]] += float(r["Counter_Value"])
                t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
                rows[k] = (name, cnt, t)
    return rows


def per_kernel(rows, counter):
    acc = defaultdict(list)
    for name, cnt, t in rows.values():
        if counter in cnt:
            acc[name].append((cnt[counter], t))
    return acc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config")
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("sq_dir")
    ap.add_argument("--out", default="profiles/pmc.json")
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    GiB = float(1 << 30)
    fr = per_kernel(read(a.fetch_dir), "FETCH_SIZE")
    wr = per_kernel(read(a.write_dir), "WRITE_SIZE")
    sq = read(a.sq_dir)

    def cal(table):
        # the clone: the first non-rc:: kernel moving at least 1/4 GiB
        for name, vals in table.items():
            if not name.startswith("rc::") and vals and vals[0][0] * 1024 > GiB / 4:
                return GiB / (vals[0][0] * 1024)
        return None
    kf, kw = cal(fr) or 2.0, cal(wr) or 1.0
    res = {}
    for name in sorted(set(fr) | set(wr)):
        if not name.startswith("rc::"):
            continue
        f = [v for v, _ in fr.get(name, [])]
        w = [v for v, _ in wr.get(name, [])]
        e = {"dispatches": max(len(f), len(w))}
        if f:
            e["fetch_bytes_raw"] = sum(f) / len(f) * 1024
        if w:
            e["write_bytes_raw"] = sum(w) / len(w) * 1024
        if f and w:
            e["hbm_bytes"] = e["fetch_bytes_raw"] * kf + e["write_bytes_raw"] * kw
        res[name] = e
    mf = defaultdict(list)
    for name, cnt, t in sq.values():
        if name.startswith("rc::") and "SQ_VALU_MFMA_BUSY_CYCLES" in cnt and cnt.get("GRBM_GUI_ACTIVE"):
            cyc = cnt["GRBM_GUI_ACTIVE"] / 8
            mf[name].append((cnt["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cyc), cyc / t / 1e9 if t else None, t))
    for name, vals in mf.items():
        e = res.setdefault(name, {})
        e["mfma_util"] = sum(v[0] for v in vals) / len(vals)
        clk = [v[1] for v in vals if v[1]]
        e["clock_ghz"] = sum(clk) / len(clk) if clk else None
        e["us_profiled"] = sum(v[2] for v in vals) / len(vals) * 1e6
    out = {}
    if os.path.exists(a.out):
        with open(a.out) as fh:
            out = json.load(fh)
    out[a.config] = {"kernels": res, "fetch_calibration": kf, "write_calibration": kw,
                     "tag": a.tag,
                     "note": "per dispatch of bench.py --config %s under rocprofv3 --pmc (three passes); "
                             "hbm_bytes = FETCH_SIZE*1024*fetch_cal + WRITE_SIZE*1024*write_cal "
                             "(1 GiB clone calibration); mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / "
                             "(1024 SIMDs x GRBM_GUI_ACTIVE/8)" % a.config}
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    for name, e in res.items():
        print(a.config, name, json.dumps(e))


if __name__ == "__main__":
    main()
