"""Small-problem lookup latency (dev probe): the level-parallel per-level
kernel (rc_corr_lookup below kLevelParP pixels) vs the pool-chain kernel
CorrBlock1D uses by default, on the realtime config (bench.py CONFIGS).
Prints median µs per launch and checks the outputs are bit-identical.

    python tools/levelpar_probe.py [--config realtime] [--reps 20]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from raft_stereo_amd import CorrBlock1D  # noqa: E402
from raft_stereo_amd import corr as rcorr  # noqa: E402


def timed(fn, coords, reps):
    ts = []
    for _ in range(reps):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(coords) + 1)]
        torch.cuda._sleep(1_000_000)
        ev[0].record()
        for k, c in enumerate(coords):
            fn(c)
            ev[k + 1].record()
        torch.cuda.synchronize()
        ts += [ev[k].elapsed_time(ev[k + 1]) * 1e3 for k in range(len(coords))]
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="realtime")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    cfg = bench.CONFIGS[a.config]
    B, D, H, W1, W2, L, r, iters, _ = cfg
    dev = torch.device("cuda", 0)
    f1, f2, coords = bench.make_inputs(cfg, dev, seed=1)
    res = {"config": a.config, "P": B * H * W1}
    with torch.no_grad():
        blk = CorrBlock1D(f1, f2, num_levels=L, radius=r)
        pyr = blk.corr_pyramid
        same = all(torch.equal(blk(c).view(torch.int32), rcorr.lookup(pyr, c, L, r).view(torch.int32))
                   for c in coords)
        res["bit_identical"] = same
        res["chain_us"] = round(timed(blk, coords, a.reps), 2)
        res["levelpar_us"] = round(timed(lambda c: rcorr.lookup(pyr, c, L, r), coords, a.reps), 2)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
