"""How the lookup's time depends on WHERE its coordinates point (dev probe).

    python tools/lookup_probe.py [--config sceneflow] [--reps 5]

The block's default lookup (the pair kernel for 4 fp32 levels), the
level-1 chain kernel and the per-level lookup are event-timed per launch, 32 launches back to back like the bench, under coordinate
distributions that differ only in locality:
  bench   coords_grid - U[0,64) per pixel, a fresh draw per launch (bench.py);
  same    one bench draw reused by all 32 launches (upper bound on re-use);
  row     x ~ U[0, W) anywhere in the row, fresh per launch: the working set
          is the whole pyramid, so the Infinity Cache cannot help;
  smooth  a smooth disparity field (neighbouring pixels similar), fresh phase
          per launch;
  net     the coords1 of each iteration of network.RAFTStereo (seeded random
          weights, default args) on a 540x960 textured pair whose right image
          is the left one shifted by 16 px: the field the update block feeds the
          lookup (smooth, with the network's own structure).
With --dev-variants the listed RAFTCORR_LOOKUP_VARIANT values (dev library)
are checked bit for bit against the product kernel and timed on the fields of
--dev-fields (default: bench).
Prints median microseconds per launch and algorithmic GB/s for each.
"""
import argparse
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from raft_stereo_amd import CorrBlock1D, coords_grid  # noqa: E402
from raft_stereo_amd import corr as rcorr  # noqa: E402


def coords_sets(B, H, W1, W2, n, kind, dev):
    grid = coords_grid(B, H, W1)
    out = []
    for it in range(n):
        g = torch.Generator().manual_seed(1000 + it)
        c = grid.clone()
        if kind == "bench" or kind == "same":
            c[:, 0] -= torch.rand(B, H, W1, generator=g) * 64.0
        elif kind == "row":
            c[:, 0] = torch.rand(B, H, W1, generator=g) * (W2 - 1)
        elif kind == "smooth":
            ph = float(torch.rand(1, generator=g)) * 6.28
            w = torch.arange(W1).float().view(1, 1, W1)
            h = torch.arange(H).float().view(1, H, 1)
            d = 32 + 24 * torch.sin(w / 17.0 + ph) * torch.cos(h / 13.0 + ph)
            c[:, 0] -= d + 0.37
        elif kind == "net":
            return net_coords(B, H, W1, n, dev)
        out.append(c.to(dev))
        if kind == "same":
            out = out * n
            break
    return out


def net_coords(B, H, W1, n, dev):
    """coords1 of n RAFTStereo iterations at (4H, 4W1) (n_downsample = 2)."""
    from raft_stereo_amd.network import RAFTStereo, StereoArgs
    rec = []

    class Recording(CorrBlock1D):
        def __call__(self, coords):
            rec.append(coords.clone())
            return super().__call__(coords)

    torch.manual_seed(0)
    model = RAFTStereo(StereoArgs(), corr_block=Recording).eval().to(dev)
    g = torch.Generator().manual_seed(7)
    tex = torch.nn.functional.interpolate(torch.rand(B, 3, H, W1, generator=g), scale_factor=4,
                                          mode="bilinear", align_corners=False)
    img1 = (tex * 255).to(dev)
    img2 = torch.roll(img1, -16, dims=-1)
    with torch.no_grad():
        model(img1, img2, iters=n)
    torch.cuda.synchronize()
    return rec[:n]


def time_seq(fn, coords, reps):
    ts = []
    for _ in range(reps):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(coords) + 1)]
        torch.cuda._sleep(3_000_000)
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
    ap.add_argument("--config", default="sceneflow")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--dev-variants", default="",
                    help="RAFTCORR_LOOKUP_VARIANT values to time on the bench coords "
                         "(libraftcorr_dev.so)")
    ap.add_argument("--dev-fields", default="bench",
                    help="coordinate fields the dev variants are timed on (comma list)")
    ap.add_argument("--only-dev", action="store_true",
                    help="time only the dev variants, default kernel only")
    a = ap.parse_args()
    B, D, H, W1, W2, L, r, iters, _ = bench.CONFIGS[a.config]
    dev = torch.device("cuda", 0)
    dt = torch.bfloat16 if a.config in bench.BF16_CONFIGS else torch.float32
    f1, f2, _ = bench.make_inputs(bench.CONFIGS[a.config], dev, seed=1, dtype=dt)
    P = B * H * W1
    lbytes = bench.lookup_bytes(P, L, r)
    res = {"config": a.config, "P": P, "alg_bytes": lbytes}
    with torch.no_grad():
        blk = CorrBlock1D(f1, f2, num_levels=L, radius=r)
        pyr = blk.corr_pyramid
        for kind in (() if a.only_dev else ("bench", "same", "row", "smooth", "net")):
            cs = coords_sets(B, H, W1, W2, iters, kind, dev)
            l1 = pyr[:2] + [None] * (L - 2)
            for name, fn in (("default", blk), ("chain_l1", lambda c: rcorr.lookup_chain(l1, c, L, r)),
                             ("per_level", lambda c: rcorr.lookup(pyr, c, L, r))):
                us = time_seq(fn, cs, a.reps)
                res[f"{kind}/{name}"] = {"us": round(us, 2),
                                         "alg_GBps": round(lbytes / (us * 1e-6) / 1e9, 1)}
        if a.dev_variants:
            from raft_stereo_amd import _lib
            l1 = pyr[:2] + [None] * (L - 2)
            for kind in a.dev_fields.split(","):
                cs = coords_sets(B, H, W1, W2, iters, kind, dev)
                ref_out = None
                vs = ["0"] + a.dev_variants.split(",")
                with _lib.dev_library():
                    for v in vs:
                        os.environ["RAFTCORR_LOOKUP_VARIANT"] = v
                        o = blk(cs[0])
                        torch.cuda.synchronize()
                        if ref_out is None:
                            ref_out = o.clone()
                        res[f"{kind}/dev{v}/bit_identical"] = bool(torch.equal(
                            torch.nan_to_num(o, nan=7.25), torch.nan_to_num(ref_out, nan=7.25)))
                    # interleaved: one 32-launch sequence per variant per round
                    per = {v: [] for v in vs}
                    for _ in range(a.reps):
                        for v in vs:
                            os.environ["RAFTCORR_LOOKUP_VARIANT"] = v
                            per[v].append(time_seq(blk, cs, 1))
                    for v in vs:
                        us = sorted(per[v])[len(per[v]) // 2]
                        res[f"{kind}/dev{v}/default"] = {
                            "us": round(us, 2), "alg_GBps": round(lbytes / (us * 1e-6) / 1e9, 1)}
                os.environ["RAFTCORR_LOOKUP_VARIANT"] = "0"
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
