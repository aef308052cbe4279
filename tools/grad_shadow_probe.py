"""Which gradient levels pay for an RC_SHADOW copy (dev probe).

    python tools/grad_shadow_probe.py [--config sceneflow] [--reps 3]

For each setting (none, level 0, level 2, both) times, on the launch stream:
the zeroing of the gradient buffers, the 32 lookup backwards (median per
call) and the build backward; prints them and their sum, and checks that the
fmap gradients agree with the unshadowed ones (summation order differs).
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from raft_stereo_amd import corr as rcorr  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="sceneflow")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--settings", default="none,l0,l2,l0+l2")
    a = ap.parse_args()
    B, D, H, W1, W2, L, r, iters, _ = bench.CONFIGS[a.config]
    dev = torch.device("cuda", 0)
    f1, f2, coords = bench.make_inputs(bench.CONFIGS[a.config], dev, seed=1, dtype=torch.float32)
    g = torch.Generator(device=dev).manual_seed(3)
    T = 2 * r + 1
    gos = [torch.randn(B, L * T, H, W1, device=dev, generator=g) for _ in range(4)]
    P = B * H * W1
    widths = [W2 >> i for i in range(L)]
    res = {"config": a.config}
    ref = None
    want = set(a.settings.split(","))
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    for name, sh in (("none", ()), ("l0", (0,)), ("l2", (2,)), ("l0+l2", (0, 2))):
        if name not in want:
            continue
        zt, lt, bt = [], [], []
        for _ in range(a.reps):
            torch.cuda._sleep(2_000_000)
            e = [ev() for _ in range(iters + 3)]
            e[0].record()
            grads = rcorr.grad_buffers(P, widths, dev, pair=True, shadow=sh)
            e[1].record()
            for k in range(iters):
                rcorr.lookup_backward(grads, coords[k], gos[k % 4], L, r)
                e[2 + k].record()
            df1, df2 = rcorr.build_backward(f1, f2, grads)
            e[2 + iters].record()
            torch.cuda.synchronize()
            zt.append(e[0].elapsed_time(e[1]) * 1e3)
            lt += [e[1 + k].elapsed_time(e[2 + k]) * 1e3 for k in range(iters)]
            bt.append(e[1 + iters].elapsed_time(e[2 + iters]) * 1e3)
            del grads
        med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
        z, l, b = med(zt), med(lt), med(bt)
        out = {"zero_us": round(z, 1), "lookup_bwd_us": round(l, 2), "build_bwd_us": round(b, 1),
               "total_us": round(z + iters * l + b, 1)}
        if ref is None:
            ref = (df1, df2)
        else:
            out["df_rel_err"] = max(float((x - y).norm() / y.norm()) for x, y in zip((df1, df2), ref))
        res[name] = out
        print(name, out, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
