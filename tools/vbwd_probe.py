"""Volume backward (rc_corr_build_backward) timing split (dev probe).

    python tools/vbwd_probe.py [--config sceneflow] [--rounds 7]

Through libraftcorr_dev.so, interleaved in one process, on the bench
workload's pair-layout gradients: the split-bf16 kernel whole, its dF1 tiles
only and its dF2 tiles only (RAFTCORR_VBWD_ONLY = 1 / 2: timing only, the
other gradient is left unwritten), the dF2 tiles' G^T staged by scattered
loads instead of G rows (RAFTCORR_VBWD_VARIANT = 2), and the exact fp32
kernel.  Median
microseconds per launch.
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
from raft_stereo_amd import _lib  # noqa: E402
from raft_stereo_amd import corr as rcorr  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="sceneflow")
    ap.add_argument("--rounds", type=int, default=7)
    a = ap.parse_args()
    cfg = bench.CONFIGS[a.config]
    B, D, H, W1, W2, L, r, iters, _ = cfg
    dev = torch.device("cuda", 0)
    f1, f2, _ = bench.make_inputs(cfg, dev, seed=1)
    P = B * H * W1
    widths = [W2 >> i for i in range(L)]
    grads = rcorr.grad_buffers(P, widths, dev, pair=True)
    g = torch.Generator(device=dev).manual_seed(5)
    for t in grads:
        if t is not None:
            t.copy_(torch.randn(t.shape, device=dev, generator=g))
    # (RAFTCORR_VBWD_ONLY, exact_f32, RAFTCORR_VBWD_VARIANT)
    variants = {"split": ("0", False, "0"), "split_dF1_only": ("1", False, "0"),
                "split_dF2_only": ("2", False, "0"), "split_scattered_GT": ("0", False, "2"),
                "split_scattered_GT_dF2_only": ("2", False, "2"), "exact": ("0", True, "0")}
    times = {k: [] for k in variants}
    with _lib.dev_library():
        for rd in range(a.rounds + 1):
            for k, (only, exact, var) in variants.items():
                os.environ["RAFTCORR_VBWD_ONLY"] = only
                os.environ["RAFTCORR_VBWD_VARIANT"] = var
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                rcorr.build_backward(f1, f2, grads, exact_f32=exact)
                e1.record()
                torch.cuda.synchronize()
                if rd:
                    times[k].append(e0.elapsed_time(e1) * 1e3)
        os.environ["RAFTCORR_VBWD_ONLY"] = "0"
        os.environ["RAFTCORR_VBWD_VARIANT"] = "0"
    print(json.dumps({"config": a.config, **{k: round(statistics.median(v), 1) for k, v in times.items()}}))


if __name__ == "__main__":
    main()
