"""Where the record build's time goes: interleaved build
timings at the KITTI config of the row build (shadowed levels 0 and 2), the
record build, and the dev-library ablations of the record build
(RAFTCORR_REC_MODE: 1 records gathered not stored, 2 stored into 8
L2-resident image rows, 3 piece images only, 4 neither, 5 the loader waves gather and store, 6 non-temporal record stores).

    python tools/records_build_ablate.py [--reps 7] [--batch B]
"""
import argparse
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from raft_stereo_amd import CorrBlock1D, _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--batch", type=int, default=0)
    a = ap.parse_args()
    B, D, H, W1, W2, L, r, iters, _ = bench.CONFIGS["kitti"]
    B = a.batch or B
    dev = torch.device("cuda", 0)
    variants = [("rows", "rows", 0), ("records", "records", 0)] + \
        [(f"rec_mode{m}", "records", m) for m in (1, 2, 3, 4, 5, 6)]
    t = {n: [] for n, _, _ in variants}
    with torch.no_grad(), _lib.dev_library():
        f1, f2, _ = bench.make_inputs((B, D, H, W1, W2, L, r, 1, None), dev, seed=1, dtype=torch.bfloat16)
        # the loader-emission variant writes the product's records
        recs = {}
        for mode in (0, 5, 6):
            os.environ["RAFTCORR_REC_MODE"] = str(mode)
            recs[mode] = CorrBlock1D(f1, f2, num_levels=L, radius=r, layout="records")._records
        same5 = all(bool(torch.equal(recs[0].view(torch.int16), recs[m].view(torch.int16))) for m in (5, 6))
        del recs
        for _ in range(a.reps):
            for name, lay, mode in variants:
                os.environ["RAFTCORR_REC_MODE"] = str(mode)
                e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                torch.cuda._sleep(5_000_000)
                e[0].record()
                blk = CorrBlock1D(f1, f2, num_levels=L, radius=r, channels_last=True, layout=lay)
                e[1].record()
                torch.cuda.synchronize()
                t[name].append(e[0].elapsed_time(e[1]) * 1e3)
                del blk
        os.environ.pop("RAFTCORR_REC_MODE", None)
    print(json.dumps({"B": B, "modes5_6_records_equal": same5, "build_us": {n: statistics.median(v) for n, v in t.items()},
                      "min_us": {n: min(v) for n, v in t.items()}}), flush=True)


if __name__ == "__main__":
    main()
