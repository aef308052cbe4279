"""A/B of the row-major vs disparity-major ("sheared") pyramid for the lookup.

    python tools/shear_probe.py [--config sceneflow] [--reps 20]

Builds the product (row-major) pyramid with CorrBlock1D, re-lays it out as
S_i[b,h][k][w1] (k = (w1>>i) - j + W_i - 1, see csrc/lookup_sheared.hip) with
torch indexing, and times both lookups on three disparity fields:
  random: coords_grid - U[0,64) per pixel (the bench's field);
  smooth: coords_grid - a smooth field in [0,64) (bilinear from a 9x16 grid);
  zero:   coords_grid (flow_init = 0, the first iteration).
Checks that both layouts give bit-identical results.
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from raft_stereo_amd import CorrBlock1D, coords_grid  # noqa: E402
from raft_stereo_amd import _lib  # noqa: E402


def smooth_disp(B, H, W, g, lo=0.0, hi=64.0, grid=(9, 16)):
    c = torch.rand(B, 1, *grid, generator=g) * (hi - lo) + lo
    return F.interpolate(c, size=(H, W), mode="bilinear", align_corners=True)[:, 0]


def make_coords(kind, B, H, W1, n, seed):
    base = coords_grid(B, H, W1)
    out = []
    for it in range(n):
        g = torch.Generator().manual_seed(seed * 100 + it)
        c = base.clone()
        if kind == "random":
            c[:, 0] -= torch.rand(B, H, W1, generator=g) * 64.0
        elif kind == "slant":
            # planar surfaces: d = a + b*w + c*h, |b|, |c| <= 0.25 px/px, clipped to [0, 64)
            a0 = torch.rand(B, 1, 1, generator=g) * 32 + 16
            bw = (torch.rand(B, 1, 1, generator=g) - 0.5) * 0.5
            ch = (torch.rand(B, 1, 1, generator=g) - 0.5) * 0.5
            w = torch.arange(W1).view(1, 1, W1) - W1 / 2
            h = torch.arange(H).view(1, H, 1) - H / 2
            c[:, 0] -= (a0 + bw * w + ch * h).clamp(0, 63.9) + torch.rand(B, H, W1, generator=g) * 0.25
        elif kind == "smooth":
            c[:, 0] -= smooth_disp(B, H, W1, g) + (torch.rand(B, H, W1, generator=g) - 0.5) * 0.5
        out.append(c.cuda())
    return out


def shear(pyr, B, H, W1, L, ldw):
    levels, K = [], []
    for i in range(L):
        Wi = pyr[i].shape[-1]
        C = pyr[i].reshape(B * H, W1, Wi)
        Ki = Wi + ((W1 - 1) >> i)
        S = torch.zeros(B * H, Ki, ldw, device=C.device)
        w1 = torch.arange(W1, device=C.device)
        j = torch.arange(Wi, device=C.device)
        kk = (w1 >> i)[:, None] - j[None, :] + Wi - 1
        S[:, kk, w1[:, None].expand(W1, Wi)] = C
        levels.append(S)
        K.append(Ki)
    return levels, K


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="sceneflow")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    B, D, H, W1, W2, L, r, iters, _ = bench.CONFIGS[a.config]
    lib = _lib.dev_library().__enter__()   # the prototype lives in the dev build only
    fn = lib.rc_dev_lookup_sheared
    fn.restype = ctypes.c_int
    vp, ci, cl = ctypes.c_void_p, ctypes.c_int, ctypes.c_long
    fn.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(ci), ctypes.POINTER(cl), cl, ci, ci, vp, cl,
                   ci, ci, ci, vp, vp]
    ldw = (W1 + 63) // 64 * 64
    res = {}
    with torch.no_grad():
        g = torch.Generator().manual_seed(0)
        f1 = torch.randn(B, D, H, W1, generator=g).cuda()
        f2 = torch.randn(B, D, H, W2, generator=g).cuda()
        blk = CorrBlock1D(f1, f2, num_levels=L, radius=r)
        S, K = shear(blk.corr_pyramid, B, H, W1, L, ldw)
        out = torch.empty(B, L * (2 * r + 1), H, W1, device="cuda")
        stream = torch.cuda.current_stream().cuda_stream

        def sheared(c):
            rc = fn(_lib.ptr_array([t.data_ptr() for t in S]),
                    _lib.int_array([t.shape[-1] for t in blk.corr_pyramid[:L]]),
                    _lib.long_array(K), ldw, L, r, c.data_ptr(), 2 * H * W1, B, H, W1,
                    out.data_ptr(), stream)
            assert rc == 0, rc
            return out

        variants = [("rows", blk, "0"), ("rows_unrolled", blk, "4"),
                    ("sheared", sheared, "0"), ("sheared_unrolled", sheared, "3")]
        for kind in ("random", "smooth", "slant", "zero"):
            cs = make_coords(kind, B, H, W1, 4, seed=3)
            for c in cs:
                os.environ["RAFTCORR_LOOKUP_VARIANT"] = "0"
                ref = blk(c).clone()
                for name, f, v in variants:
                    os.environ["RAFTCORR_LOOKUP_VARIANT"] = v
                    got = f(c)
                    assert torch.equal(ref, got), (kind, name, (ref - got).abs().max().item())
            for name, f, v in variants:
                os.environ["RAFTCORR_LOOKUP_VARIANT"] = v
                for _ in range(3):
                    f(cs[0])
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.reps + 1)]
                ev[0].record()
                for k in range(a.reps):
                    f(cs[k % len(cs)])
                    ev[k + 1].record()
                torch.cuda.synchronize()
                ts = [ev[k].elapsed_time(ev[k + 1]) * 1e3 for k in range(a.reps)]
                res[f"{kind}_{name}"] = {"median_us": statistics.median(ts), "min_us": min(ts)}
        alg = bench.lookup_bytes(B * H * W1, L, r)
        print(json.dumps({"config": a.config, "ldw": ldw, "K": K,
                          "sheared_MB": sum(t.numel() * 4 for t in S) / 1e6,
                          "alg_bytes": alg, "results": res}))


if __name__ == "__main__":
    main()
