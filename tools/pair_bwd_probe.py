"""A/B of the pair lookup backward's schedule (dev probe, libraftcorr_dev.so).

    python tools/pair_bwd_probe.py [--config sceneflow] [--variants 0,21,23]

RAFTCORR_LOOKUP_BWD_VARIANT on the pair layout (radius 4, 4 levels):
0 product (both pairs' loads up front, 190 VGPRs, 2 waves/SIMD), 21 / 22
occupancy floors 3 / 4 (spills), 23 pairs in sequence (122 VGPRs, 4
waves/SIMD), 24 = 23 with the floor.  Checks bit-identity of the gradient
buffers after 3 calls, then times interleaved rounds of 8 calls.
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from raft_stereo_amd import _lib  # noqa: E402
from raft_stereo_amd import corr as rcorr  # noqa: E402

_lib.dev_library().__enter__()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="sceneflow")
    ap.add_argument("--variants", default="0,21,23")
    ap.add_argument("--rounds", type=int, default=7)
    a = ap.parse_args()
    cfg = bench.CONFIGS[a.config]
    B, D, H, W1, W2, L, r, iters, _ = cfg
    dev = torch.device("cuda", 0)
    _, _, coords = bench.make_inputs(cfg, dev, seed=1, dtype=torch.float32)
    g = torch.Generator().manual_seed(9)
    go = torch.randn(B, L * (2 * r + 1), H, W1, generator=g).to(dev)
    P, widths = B * H * W1, [W2 >> i for i in range(L)]
    vs = [int(x) for x in a.variants.split(",") if x]
    outs = {}
    for v in vs:
        os.environ["RAFTCORR_LOOKUP_BWD_VARIANT"] = str(v)
        gv = rcorr.grad_buffers(P, widths, dev, pair=True)
        for k in range(3):
            rcorr.lookup_backward(gv, coords[k], go, L, r)
        outs[v] = gv
    for v in vs[1:]:
        for i in (0, 2):
            assert torch.equal(outs[v][i], outs[vs[0]][i]), ("variant", v, i)
    print("bit-identical", vs, flush=True)
    del outs
    gp = rcorr.grad_buffers(P, widths, dev, pair=True)
    res = {}
    for rnd in range(a.rounds):
        c = coords[rnd % iters]
        for v in vs:
            os.environ["RAFTCORR_LOOKUP_BWD_VARIANT"] = str(v)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(9)]
            torch.cuda._sleep(2_000_000)
            ev[0].record()
            for k in range(8):
                rcorr.lookup_backward(gp, c, go, L, r)
                ev[k + 1].record()
            torch.cuda.synchronize()
            res.setdefault(f"v{v}", []).extend(ev[k].elapsed_time(ev[k + 1]) * 1e3 for k in range(8))
    print(json.dumps({k: round(sorted(t)[len(t) // 2], 2) for k, t in res.items()}))


if __name__ == "__main__":
    main()
