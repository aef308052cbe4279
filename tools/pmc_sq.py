"""Summarise rocprofv3 SQ counters per kernel (mean per dispatch).

    python tools/pmc_sq.py <pmc_dir>

Derived: effective clock = GRBM_GUI_ACTIVE/8 XCDs / kernel time; MFMA
utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x GRBM_GUI_ACTIVE/8); wave-
cycle split from SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY (all in
quad-cycles, MI355X_MICROARCH.md 'rocprofv3 PMC slots')."""
import csv
import glob
import os
import sys
from collections import defaultdict

SIMDS = 256 * 4


def main(d, json_out=None):
    agg = defaultdict(lambda: defaultdict(float))
    names, times = {}, {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            k = int(r["Dispatch_Id"])
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            names[k] = r["Kernel_Name"].split("(")[0][:48]
            times[k] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    per = defaultdict(list)
    for k in sorted(agg):
        per[names[k]].append((agg[k], times[k]))
    util = {}
    for name, rows in per.items():
        n = len(rows)
        c = {key: sum(r[0].get(key, 0.0) for r in rows) / n for key in rows[0][0]}
        t = sum(r[1] for r in rows) / n
        gui = c.get("GRBM_GUI_ACTIVE", 0.0) / 8
        line = f"{name:48s} n={n} t={t*1e6:8.1f}us"
        if gui and t:
            line += f" clk={gui / t / 1e9:5.2f}GHz"
            if c.get("SQ_VALU_MFMA_BUSY_CYCLES"):
                u = c['SQ_VALU_MFMA_BUSY_CYCLES'] / (SIMDS * gui)
                line += f" mfma_util={u:.3f}"
                util[name] = {"mfma_util": u, "clock_ghz": gui / t / 1e9, "us": t * 1e6,
                              "dispatches": n}
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        if wc:
            line += (f" wait={c.get('SQ_WAIT_ANY', 0) / wc:.2f} wait_inst={c.get('SQ_WAIT_INST_ANY', 0) / wc:.2f}"
                     f" active={c.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f}")
        if c.get("SQ_WAVES"):
            line += f" waves={c['SQ_WAVES']:.0f}"
        print(line)


    if json_out:
        import json
        with open(json_out, "w") as fh:
            json.dump({"note": "SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE/8), "
                               "rocprofv3 --pmc pass over tools/probe.py", "kernels": util},
                      fh, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
