"""Interleaved A/B of the realtime config's graph-replayed step (dev probe).

    python tools/realtime_ab.py [--rounds 15] [--reps 100] VAR=val[,VAR=val] ...

Captures bench.py --config realtime --graph's step (CorrBlock1D build + 7
lookups) once with the product library and once per argument with the dev
library and those RAFTCORR_* knobs set at capture time (a launch is chosen
when it is captured), checks every variant's lookup outputs bit for bit
against the product's, then replays the graphs round-robin: per round each
graph ``reps`` times back to back between two events.  Prints the median
microseconds per step of each.
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from raft_stereo_amd import CorrBlock1D, _lib  # noqa: E402


def capture(f1, f2, coords, L, r, iters):
    outs = []

    def step():
        b = CorrBlock1D(f1, f2, num_levels=L, radius=r, low_latency=True)
        outs[:] = [b(coords[it]) for it in range(iters)]
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    torch.cuda.synchronize()
    return g, outs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=15)
    ap.add_argument("--reps", type=int, default=100)
    ap.add_argument("variants", nargs="*")
    a = ap.parse_args()
    cfg = bench.CONFIGS["realtime"]
    B, D, H, W1, W2, L, r, iters, _ = cfg
    dev = torch.device("cuda", 0)
    f1, f2, coords = bench.make_inputs(cfg, dev, seed=1)
    graphs = {}
    with torch.no_grad():
        graphs["product"] = capture(f1, f2, coords, L, r, iters)
        for v in a.variants:
            env = dict(kv.split("=") for kv in v.split(","))
            old = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            try:
                with _lib.dev_library():
                    graphs[v] = capture(f1, f2, coords, L, r, iters)
            finally:
                for k, val in old.items():
                    if val is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = val
    for name, (g, outs) in graphs.items():
        g.replay()
    torch.cuda.synchronize()
    ref = graphs["product"][1]
    same = {name: all(torch.equal(x.nan_to_num(7.0), y.nan_to_num(7.0)) for x, y in zip(outs, ref))
            for name, (g, outs) in graphs.items()}
    times = {name: [] for name in graphs}
    for _ in range(a.rounds):
        for name, (g, _o) in graphs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(a.reps):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) * 1e3 / a.reps)
    res = {name: {"median_us": round(sorted(t)[len(t) // 2], 2), "min_us": round(min(t), 2),
                  "bit_identical": same[name]} for name, t in times.items()}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
