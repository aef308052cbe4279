"""Where a middle rank's per-conv RowShardedStereo.forward spends its time
(config 4, 1984x2880, 32 iterations, exchanges replaced by zero rows as in
tools/shard_probe.py --perconv): encoders with per-module halos
(_perconv_state), the corr build on own rows +- 4, and the GRU loop, for
N = 1, 2, 4, 8 -- to locate the per-rank overhead that does not shrink with N.

    python tools/perconv_phases.py [--iters 32]
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
from raft_stereo_amd.shard import RowShardedStereo  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=32)
    ap.add_argument("--H", type=int, default=1984)
    ap.add_argument("--W", type=int, default=2880)
    ap.add_argument("--only", type=int, default=0, help="one N only (e.g. under rocprofv3)")
    ap.add_argument("--no-side", action="store_true", help="RowShardedStereo(side_stream=False)")
    ap.add_argument("--no-fuse", action="store_true", help="RowShardedStereo(fuse_zr=False)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = RAFTStereo(StereoArgs()).eval().to(dev)
    g = torch.Generator().manual_seed(1234)
    img1 = (torch.rand(1, 3, a.H, a.W, generator=g) * 255).to(dev)
    img2 = torch.roll(img1, -8, dims=-1)
    out = {}
    with torch.no_grad():
        for N in ((a.only,) if a.only else (1, 2, 4, 8)):
            rs = RowShardedStereo(model, N // 2, N, side_stream=not a.no_side, fuse_zr=not a.no_fuse)
            rs._fake_xchg = True
            acc = {"encoders": 0.0, "corr_build": 0.0}
            st0, cb0 = rs._perconv_state, model.corr_block

            def state(*args, **kw):
                torch.cuda.synchronize()
                t = time.perf_counter()
                r = st0(*args, **kw)
                torch.cuda.synchronize()
                acc["encoders"] += time.perf_counter() - t
                return r

            def block(*args, **kw):
                torch.cuda.synchronize()
                t = time.perf_counter()
                r = cb0(*args, **kw)
                torch.cuda.synchronize()
                acc["corr_build"] += time.perf_counter() - t
                return r

            rs._perconv_state = state
            model.corr_block = block
            try:
                rs.forward(img1, img2, iters=a.iters)          # warm-up (MIOpen finds its kernels)
                torch.cuda.synchronize()
                torch.cuda._sleep(1000)       # delimiter in a kernel trace: the timed reps follow
                torch.cuda.synchronize()
                acc = {"encoders": 0.0, "corr_build": 0.0}
                reps = 3
                t = time.perf_counter()
                for _ in range(reps):
                    rs.forward(img1, img2, iters=a.iters)
                torch.cuda.synchronize()
                total = (time.perf_counter() - t) / reps
            finally:
                model.corr_block = cb0
            o = {k: v / reps * 1e3 for k, v in acc.items()}
            o["total"] = total * 1e3
            o["gru_loop"] = o["total"] - o["encoders"] - o["corr_build"]
            out[N] = o
            print(N, json.dumps({k: round(v, 2) for k, v in o.items()}), flush=True)
    if 1 in out:
        ideal = {N: {k: round(out[1][k] / N, 2) for k in out[1]} for N in out}
        print(json.dumps({"per_N_ms": out, "ideal_from_N1": ideal}, indent=1))


if __name__ == "__main__":
    main()
