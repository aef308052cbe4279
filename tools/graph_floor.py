"""Per-node floor of a replayed HIP graph on this GPU (dev probe, realtime config).

    python tools/graph_floor.py [--reps 200]

Captures (a) 8 one-element torch kernels, (b) the realtime config's 7 lookups
alone (pyramid built outside the graph), (c) its build alone, (d) build + 7
lookups (bench.py --graph's step), and times back-to-back replays with events
on the capturing stream.  (a) is the cost of a graph node that does no memory
work: the floor under any 8-kernel realtime step.
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


def replay_us(fn, reps):
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    torch.cuda.synchronize()
    for _ in range(10):
        g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    a = ap.parse_args()
    cfg = bench.CONFIGS["realtime"]
    B, D, H, W1, W2, L, r, iters, _ = cfg
    dev = torch.device("cuda", 0)
    f1, f2, coords = bench.make_inputs(cfg, dev, seed=1)
    x = torch.zeros(1, device=dev)
    res = {}
    with torch.no_grad():
        def tiny():
            for _ in range(8):
                x.add_(1.0)
        res["tiny_x8_us"] = replay_us(tiny, a.reps)
        blk = CorrBlock1D(f1, f2, num_levels=L, radius=r, low_latency=True)

        def lookups():
            for it in range(iters):
                blk(coords[it])
        res["lookups_x7_us"] = replay_us(lookups, a.reps)

        def build():
            CorrBlock1D(f1, f2, num_levels=L, radius=r, low_latency=True)
        res["build_us"] = replay_us(build, a.reps)

        def step():
            b = CorrBlock1D(f1, f2, num_levels=L, radius=r, low_latency=True)
            for it in range(iters):
                b(coords[it])
        res["step_us"] = replay_us(step, a.reps)
    res["tiny_per_node_us"] = res["tiny_x8_us"] / 8
    res["lookup_per_node_us"] = res["lookups_x7_us"] / iters
    print(json.dumps({k: round(v, 2) for k, v in res.items()}))


if __name__ == "__main__":
    main()
