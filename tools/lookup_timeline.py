"""Per-wave timeline of the pair lookup (dev probe, libraftcorr_dev.so).

    python tools/lookup_timeline.py [--config sceneflow]

Runs the stamped diagnostic build (RAFTCORR_LOOKUP_VARIANT=210,
lookup_pair_stamped_kernel) on the bench workload and prints, over all
waves, the distribution (min / p10 / p50 / p90 / max, microseconds) of each
phase -- loads issued, span 0 wait, pair-0 math, span 2 wait, pair-2 math,
store drain -- and of the absolute start / data-ready / end times relative to
the first wave's start.  The diagnostic build's waits forbid some overlaps,
so its total is not the product's time; the shares and spreads are the point.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from raft_stereo_amd import CorrBlock1D, _lib  # noqa: E402


def q(a):
    return [round(float(np.percentile(a, p)), 2) for p in (0, 10, 50, 90, 100)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="sceneflow")
    a = ap.parse_args()
    cfg = bench.CONFIGS[a.config]
    B, D, H, W1, W2, L, r, iters, _ = cfg
    dev = torch.device("cuda", 0)
    f1, f2, coords = bench.make_inputs(cfg, dev, seed=1)
    P = B * H * W1
    nw = (P + 255) // 256 * 4
    dbg = torch.zeros(nw * 8, dtype=torch.int64, device=dev)
    res = {}
    with torch.no_grad(), _lib.dev_library() as lib:
        lib.rc_dev_set_dbg.argtypes = [ctypes.c_void_p]
        lib.rc_dev_set_dbg.restype = None
        blk = CorrBlock1D(f1, f2, num_levels=L, radius=r)
        os.environ["RAFTCORR_LOOKUP_VARIANT"] = "210"
        lib.rc_dev_set_dbg(dbg.data_ptr())
        for it in range(4):            # the last of 4 back-to-back launches
            blk(coords[it])
        torch.cuda.synchronize()
        lib.rc_dev_set_dbg(None)
        os.environ["RAFTCORR_LOOKUP_VARIANT"] = "0"
    t = dbg.view(nw, 8).cpu().numpy()
    st = t[:, :7].astype(np.float64) * 0.01            # 100 MHz -> microseconds
    st -= st[:, 0].min()
    names = ["issue", "wait_span0", "math_pair0", "wait_span2", "math_pair2", "store_drain"]
    for k, n in enumerate(names):
        res[n] = q(st[:, k + 1] - st[:, k])
    res["abs_start"] = q(st[:, 0])
    res["abs_span0_ready"] = q(st[:, 2])
    res["abs_pair0_done"] = q(st[:, 3])
    res["abs_end"] = q(st[:, 6])
    res["note"] = "us, [min, p10, p50, p90, max] over waves; diagnostic build (not the product's time)"
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
