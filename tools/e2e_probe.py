"""Whole-network timing at config 2 under different PyTorch execution settings
(encoders/GRU stay PyTorch ops; only how they run changes).

    python tools/e2e_probe.py [--steps 2]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pkgload  # noqa: E402

pkgload.load()
from raft_stereo_amd.network import RAFTStereo, StereoArgs  # noqa: E402


def run(mixed, benchmark, channels_last, steps, B=8, H=540, W=960, iters=32):
    torch.backends.cudnn.benchmark = benchmark
    torch.manual_seed(0)
    args = StereoArgs(mixed_precision=mixed)
    args.autocast_dtype = torch.bfloat16
    model = RAFTStereo(args).eval().cuda()
    if channels_last:
        model = model.to(memory_format=torch.channels_last)
    g = torch.Generator().manual_seed(1234)
    img1 = (torch.rand(B, 3, H, W, generator=g) * 255).cuda()
    img2 = torch.roll(img1, -8, dims=-1)
    with torch.no_grad():
        model(img1, img2, iters=iters)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            model(img1, img2, iters=iters)
        torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    return {"mixed_bf16": mixed, "miopen_benchmark": benchmark, "channels_last": channels_last,
            "ms_per_batch": dt * 1e3, "pairs_per_s": B / dt}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()
    for mixed, bench, cl in [(False, False, False), (False, True, False), (True, False, False),
                             (True, True, False), (True, True, True)]:
        print(json.dumps(run(mixed, bench, cl, a.steps)), flush=True)


if __name__ == "__main__":
    main()
