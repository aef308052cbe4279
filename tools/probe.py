"""Isolated launches of the corr kernels for rocprofv3 counter runs.

    python tools/probe.py [--config sceneflow] [--iters N]

Launches, in order: a calibration copy (torch clone of a 1 GiB fp32 tensor:
exactly 1 GiB read + 1 GiB written), N builds (rc::build_f32_ring_kernel), N
CorrBlock1D lookups (rc::lookup_pair_kernel for 4 fp32 levels), N per-level lookups
(rc::lookup_kernel), N level-1 chain lookups (rc::lookup_chain_kernel), N lookup backwards
(rc::lookup_bwd_pre_kernel) of bench.py's workload.  tools/pmc_traffic.py turns
the per-dispatch FETCH_SIZE / WRITE_SIZE into bytes per launch.
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from raft_stereo_amd import CorrBlock1D  # noqa: E402
from raft_stereo_amd import corr as rcorr  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="sceneflow")
    ap.add_argument("--iters", type=int, default=4)
    ap.add_argument("--pyr-dtype", default="f32", choices=["f32", "bf16"])
    ap.add_argument("--dev-variants", default="",
                    help="also run N lookups per RAFTCORR_LOOKUP_VARIANT value through "
                         "libraftcorr_dev.so (their kernels carry distinct template names)")
    a = ap.parse_args()
    cfg = bench.CONFIGS[a.config]
    B, D, H, W1, W2, L, r, iters, _ = cfg
    dev = torch.device("cuda", 0)
    pdt = torch.float32 if a.pyr_dtype == "f32" else torch.bfloat16
    with torch.no_grad():
        big = torch.randn(1 << 28, device=dev)
        cal = big.clone()   # calibration: 1 GiB read + 1 GiB write
        del cal
        # a bf16 pyramid comes from bf16 fmaps, as in bench.py (the ring kernel)
        f1, f2, coords = bench.make_inputs(cfg, dev, seed=1, dtype=pdt)
        blk = None
        for _ in range(a.iters):
            blk = CorrBlock1D(f1, f2, num_levels=L, radius=r, pyramid_dtype=pdt)
        for it in range(a.iters):
            blk(coords[it % iters])        # rc::lookup_chain_kernel (fp32) / lookup_kernel
        for it in range(a.iters):          # the per-level kernel on the same pyramid
            rcorr.lookup(blk.corr_pyramid, coords[it % iters], L, r)
        if pdt == torch.float32 and L in (3, 4):   # the level-1 chain kernel (levels 0-1 given)
            lv = blk.corr_pyramid[:2] + [None] * (L - 2)
            for it in range(a.iters):
                rcorr.lookup_chain(lv, coords[it % iters], L, r)
        if pdt == torch.float32:           # rc::lookup_bwd_pre_kernel (one per lookup call)
            P = B * H * W1
            go = torch.randn(B, L * (2 * r + 1), H, W1, device=dev)
            for pair in (False, True):     # lookup_bwd_pre_kernel, lookup_bwd_pair_kernel
                grads = rcorr.grad_buffers(P, [W2 >> i for i in range(L)], dev, pair=pair)
                for it in range(a.iters):
                    rcorr.lookup_backward(grads, coords[it % iters], go, L, r)
                for _ in range(2):         # rc::volume_bwd_kernel (fp32 MFMA)
                    rcorr.build_backward(f1, f2, grads)
        if a.dev_variants:
            from raft_stereo_amd import _lib
            with _lib.dev_library():
                for v in a.dev_variants.split(","):
                    os.environ["RAFTCORR_LOOKUP_VARIANT"] = v
                    for it in range(a.iters):
                        blk(coords[it % iters])
                os.environ["RAFTCORR_LOOKUP_VARIANT"] = "0"
        torch.cuda.synchronize()
    print("probe done")


if __name__ == "__main__":
    main()
