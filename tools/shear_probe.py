"""A/B of the row-major pair lookup (the product) vs the disparity-major
("sheared") pair lookup.

    python tools/shear_probe.py [--config sceneflow] [--reps 7]

Builds the product pyramid (levels 0 and 2 stored) with CorrBlock1D, re-lays
levels 0 and 2 out as S_i[b,h][k][w1] (k = (w1>>i) - j + W_i - 1) with torch
indexing, and times both lookups -- the same pair arithmetic and Markstein
division, bit-identical outputs (checked) -- on five disparity fields, 32
launches each, interleaved:
  random: coords_grid - U[0,64) per pixel (the bench's field);
  smooth: coords_grid - a smooth field in [0,64) (bilinear from a 9x16 grid);
  slant:  planar surfaces, |slope| <= 0.25 px/px;
  zero:   coords_grid (flow_init = 0, the first iteration);
  net:    coords1 of network.RAFTStereo's iterations at 540x960 (tools/lookup_probe.py).
(Round 1's sheared prototype -- all four levels stored, one window per level
-- is in profiles/r01/shear_probe.log.)
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
sys.path.insert(0, os.path.join(ROOT, "tools"))
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


def shear_pair(pyr, B, H, W1):
    """Levels 0 and 2 of the product pyramid as S_i[b,h][k][w1] (the sheared
    pair kernel's layout, csrc/lookup.hip lookup_sheared_pair_kernel)."""
    out, K = [], []
    for i in (0, 2):
        Wi = pyr[i].shape[-1]
        C = pyr[i].reshape(B * H, W1, Wi)
        Ki = Wi + ((W1 - 1) >> i)
        S = torch.zeros(B * H, Ki, W1, device=C.device)
        w1 = torch.arange(W1, device=C.device)
        j = torch.arange(Wi, device=C.device)
        kk = (w1 >> i)[:, None] - j[None, :] + Wi - 1
        S[:, kk, w1[:, None].expand(W1, Wi)] = C
        out.append(S.contiguous())
        K.append(Ki)
    return out, K


def product_main(a):
    """--product: CorrBlock1D(layout="rows") against layout="disparity"
    (the product path, RC_LAYOUT_DISPARITY) with the product library only:
    the build alone (event-timed after a device-side sleep, as bench.py
    times it), the 32 lookups of each field, and whole steps (build + 32
    lookups), interleaved, medians; every lookup checked bit for bit."""
    B, D, H, W1, W2, L, r, iters, _ = bench.CONFIGS[a.config]
    res = {}
    with torch.no_grad():
        g = torch.Generator().manual_seed(0)
        f1 = torch.randn(B, D, H, W1, generator=g).cuda()
        f2 = torch.randn(B, D, H, W2, generator=g).cuda()
        layouts = ("rows", "disparity")
        mk = {lay: (lambda lay=lay: CorrBlock1D(f1, f2, num_levels=L, radius=r, layout=lay)) for lay in layouts}
        blocks = {lay: mk[lay]() for lay in layouts}
        bt = {lay: [] for lay in layouts}
        for _ in range(a.reps):
            for lay in layouts:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda._sleep(3_000_000)
                e0.record()
                mk[lay]()
                e1.record()
                torch.cuda.synchronize()
                bt[lay].append(e0.elapsed_time(e1) * 1e3)
        res["build_us"] = {lay: statistics.median(bt[lay]) for lay in layouts}
        print("build", {k: round(v, 1) for k, v in res["build_us"].items()}, flush=True)
        for kind in ("random", "smooth", "slant", "zero", "net"):
            if kind == "net":
                from lookup_probe import net_coords
                cs = net_coords(B, H, W1, iters, torch.device("cuda", 0))
            else:
                cs = make_coords(kind, B, H, W1, iters, seed=3)
            for c in cs[:4]:
                assert torch.equal(blocks["rows"](c), blocks["disparity"](c)), kind
            per = {lay: [] for lay in layouts}
            step = {lay: [] for lay in layouts}
            for _ in range(a.reps):
                for lay in layouts:
                    ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(cs) + 1)]
                    torch.cuda._sleep(3_000_000)
                    ev[0].record()
                    for k, c in enumerate(cs):
                        blocks[lay](c)
                        ev[k + 1].record()
                    torch.cuda.synchronize()
                    per[lay] += [ev[k].elapsed_time(ev[k + 1]) * 1e3 for k in range(len(cs))]
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    torch.cuda._sleep(3_000_000)
                    e0.record()
                    blk = mk[lay]()
                    for c in cs:
                        blk(c)
                    e1.record()
                    torch.cuda.synchronize()
                    step[lay].append(e0.elapsed_time(e1))
            res[kind] = {lay: {"lookup_us": statistics.median(per[lay]),
                               "step_ms": statistics.median(step[lay])} for lay in layouts}
            print(kind, {lay: {k: round(v, 3) for k, v in res[kind][lay].items()} for lay in layouts},
                  flush=True)
        alg = bench.lookup_bytes(B * H * W1, L, r)
        print(json.dumps({"config": a.config, "mode": "product", "alg_bytes": alg, "bit_identical": True,
                          "disparity_MB": sum(t.numel() * 4 for t in blocks["disparity"]._sheared.values()) / 1e6,
                          "results": res}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="sceneflow")
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--product", action="store_true",
                    help="CorrBlock1D layout='rows' vs 'disparity' (product library), builds and steps")
    a = ap.parse_args()
    if a.product:
        return product_main(a)
    B, D, H, W1, W2, L, r, iters, _ = bench.CONFIGS[a.config]
    lib = _lib.dev_library().__enter__()   # the sheared kernel lives in the dev build only
    fn = lib.rc_dev_lookup_sheared_pair
    fn.restype = ctypes.c_int
    vp, ci, cl = ctypes.c_void_p, ctypes.c_int, ctypes.c_long
    fn.argtypes = [vp, vp, cl, cl, cl, ctypes.POINTER(ci), vp, cl, ci, ci, ci, vp, vp]
    res = {}
    with torch.no_grad():
        g = torch.Generator().manual_seed(0)
        f1 = torch.randn(B, D, H, W1, generator=g).cuda()
        f2 = torch.randn(B, D, H, W2, generator=g).cuda()
        blk = CorrBlock1D(f1, f2, num_levels=L, radius=r)
        assert blk.levels_stored == [0, 2]
        S, K = shear_pair(blk.corr_pyramid, B, H, W1)
        widths = _lib.int_array([W2 >> i for i in range(4)])
        out = torch.empty(B, L * (2 * r + 1), H, W1, device="cuda")
        stream = torch.cuda.current_stream().cuda_stream

        def sheared(c):
            rc = fn(S[0].data_ptr(), S[1].data_ptr(), K[0], K[1], W1, widths, c.data_ptr(),
                    2 * H * W1, B, H, W1, out.data_ptr(), stream)
            assert rc == 0, rc
            return out

        variants = [("product_pair", blk), ("sheared_pair", sheared)]
        for kind in ("random", "smooth", "slant", "zero", "net"):
            if kind == "net":
                from lookup_probe import net_coords
                cs = net_coords(B, H, W1, iters, torch.device("cuda", 0))
            else:
                cs = make_coords(kind, B, H, W1, iters, seed=3)
            for c in cs[:4]:
                ref = blk(c).clone()
                got = sheared(c)
                assert torch.equal(ref, got), (kind, (ref - got).abs().max().item())
            per = {n: [] for n, _ in variants}
            for _ in range(a.reps):                  # interleaved: one 32-launch sequence each
                for name, f in variants:
                    ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(cs) + 1)]
                    torch.cuda._sleep(3_000_000)
                    ev[0].record()
                    for k, c in enumerate(cs):
                        f(c)
                        ev[k + 1].record()
                    torch.cuda.synchronize()
                    per[name] += [ev[k].elapsed_time(ev[k + 1]) * 1e3 for k in range(len(cs))]
            for name, _ in variants:
                res[f"{kind}_{name}"] = {"median_us": statistics.median(per[name]), "min_us": min(per[name])}
            print(kind, {n: round(res[f"{kind}_{n}"]["median_us"], 2) for n, _ in variants}, flush=True)
        alg = bench.lookup_bytes(B * H * W1, L, r)
        print(json.dumps({"config": a.config, "K": K, "sheared_MB": sum(t.numel() * 4 for t in S) / 1e6,
                          "alg_bytes": alg, "bit_identical": True, "results": res}))


if __name__ == "__main__":
    main()
