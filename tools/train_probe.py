"""Autograd train step through CorrBlock1D: wall time vs GPU time (dev probe).

    python tools/train_probe.py [--config sceneflow] [--reps 7]

For the deferred lookup backward (the pair-layout default) and the per-call
backward (grad_deferred=False), prints the median wall time of a synchronised
step and the GPU time between two events bracketing it, and the same for the
forward alone -- a wall time well above the GPU time means the step is bound
by host-side launch work, not by the kernels.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from raft_stereo_amd import CorrBlock1D  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="sceneflow")
    ap.add_argument("--reps", type=int, default=7)
    a = ap.parse_args()
    cfg = bench.CONFIGS[a.config]
    B, D, H, W1, W2, L, r, iters, _ = cfg
    dev = torch.device("cuda", 0)
    f1, f2, coords = bench.make_inputs(cfg, dev, seed=1)
    g = torch.Generator().manual_seed(99)
    gouts = [torch.randn(B, L * (2 * r + 1), H, W1, generator=g).to(dev) for _ in range(2)]
    gl = [gouts[it % 2] for it in range(iters)]
    fa = f1.detach().clone().requires_grad_(True)
    fb = f2.detach().clone().requires_grad_(True)

    def step(deferred, backward=True):
        blk = CorrBlock1D(fa, fb, num_levels=L, radius=r, grad_deferred=deferred)
        outs = [blk(coords[it]) for it in range(iters)]
        if backward:
            torch.autograd.backward(outs, gl)

    res = {}
    for name, fn in (("fwd_only", lambda: step(None, False)), ("deferred", lambda: step(None)),
                     ("per_call", lambda: step(False))):
        fn()
        torch.cuda.synchronize()
        wall, gpu = [], []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            wall.append((time.perf_counter() - t0) * 1e3)
            gpu.append(e0.elapsed_time(e1))
        wall.sort()
        gpu.sort()
        res[name] = {"wall_ms": round(wall[len(wall) // 2], 3), "gpu_ms": round(gpu[len(gpu) // 2], 3)}
        print(name, res[name], flush=True)
    # Peak device memory of one step: the loss multiplies every
    # lookup output by a weight, so each call's output gradient is a fresh
    # tensor (as in the network) that the deferred state keeps until the build
    # node, where the per-call backward frees it after its own call.
    for name, deferred in (("mem_deferred", None), ("mem_per_call", False)):
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        base = torch.cuda.memory_allocated()
        torch.cuda.reset_peak_memory_stats()
        blk = CorrBlock1D(fa, fb, num_levels=L, radius=r, grad_deferred=deferred)
        loss = sum((blk(coords[it]) * gl[it]).sum() for it in range(iters))
        loss.backward()
        torch.cuda.synchronize()
        res[name] = {"peak_above_inputs_MB": round((torch.cuda.max_memory_allocated() - base) / 1e6, 1)}
        print(name, res[name], flush=True)
        del blk, loss
    print(json.dumps(res))


if __name__ == "__main__":
    main()
