"""Isolated builds for rocprofv3 counter runs: N split-bf16 builds
(rc::build_split_kernel) then N exact fp32 builds (rc::build_f32_ring_kernel)
of bench.py's workload.

    python tools/build_probe_split.py [--config sceneflow] [--iters 4]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from raft_stereo_amd import CorrBlock1D  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="sceneflow")
    ap.add_argument("--iters", type=int, default=4)
    a = ap.parse_args()
    B, D, H, W1, W2, L, r, iters, _ = bench.CONFIGS[a.config]
    ll = a.config in bench.LOW_LATENCY_CONFIGS
    with torch.no_grad():
        f1, f2, _ = bench.make_inputs(bench.CONFIGS[a.config], torch.device("cuda", 0), seed=1)
        for exact in (False, True):
            for _ in range(a.iters):
                CorrBlock1D(f1, f2, num_levels=L, radius=r, low_latency=ll, exact_f32=exact)
        torch.cuda.synchronize()
    print("probe done")


if __name__ == "__main__":
    main()
