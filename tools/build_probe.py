"""Isolated launches of the bf16 build kernels for rocprofv3 counter runs
(dev library; kernels of different RAFTCORR_BUILD_MODE values carry
different template names).

    python tools/build_probe.py [--config kitti] [--iters 3] [--modes 0,32,40,44,47]

Launches a calibration copy (1 GiB read + 1 GiB written), then --iters
builds per mode.  Aggregate with tools/pmc_raw.py --width 120.
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from raft_stereo_amd import CorrBlock1D, _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="kitti")
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--modes", default="0,32,40,44,47")
    a = ap.parse_args()
    cfg = bench.CONFIGS[a.config]
    B, D, H, W1, W2, L, r, iters, _ = cfg
    dev = torch.device("cuda", 0)
    dt = torch.bfloat16 if a.config in bench.BF16_CONFIGS else torch.float32
    with torch.no_grad():
        big = torch.randn(1 << 28, device=dev)
        cal = big.clone()   # calibration: 1 GiB read + 1 GiB write
        del big, cal
        f1, f2, _ = bench.make_inputs(cfg, dev, seed=1, dtype=dt)
        with _lib.dev_library():
            for m in [x for x in a.modes.split(",") if x]:
                os.environ["RAFTCORR_BUILD_MODE"] = m
                for _ in range(a.iters):
                    CorrBlock1D(f1, f2, num_levels=L, radius=r)
                torch.cuda.synchronize()
        os.environ["RAFTCORR_BUILD_MODE"] = "0"


if __name__ == "__main__":
    main()
