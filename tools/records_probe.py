"""A/B of the bf16 pair lookup (the product: levels 0 and 2 each from the
better of two half-line-shifted copies, two 128-B lines per pixel) vs the
record layout (one line per pixel; dev prototype).

    python tools/records_probe.py [--config kitti] [--reps 7] [--batch B]

Builds the product CorrBlock1D (bf16 pyramid, channels-last output), re-lays a
no-shadow build's levels 0 and 2 out as records with torch strided views (no
kernel of its own yet), checks that the record lookup equals the product bit
for bit on the bench field and on special coordinates (NaN, +-inf, huge and
edge values), and times both in interleaved 32-launch sequences.  Also
reports the bytes of each layout (the build cost the records would add).
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402
from raft_stereo_amd import CorrBlock1D  # noqa: E402
from raft_stereo_amd import _lib  # noqa: E402
from raft_stereo_amd import corr as rcorr  # noqa: E402

M0 = -8          # first record's level-1 centre (a multiple of 4)
# slots -> (G level-1 centres per record, level-2 slots, level-0 slots)
GEOM = {64: (8, 26, 38), 128: (32, 38, 86)}


def records(pyr, P, W0, W2l, NR, slots):
    """(P, NR, slots) bf16: slots [0, n2) level-2 elements (G/2) r + M0/2 - 10 + j,
    slots [n2, n2 + n0) level-0 elements 2 G r + 2 M0 - 10 + j (zeros off the
    row and in any padding slots)."""
    G, n2s, n0s = GEOM[slots]
    L0 = pyr[0].reshape(P, -1)[:, :W0]
    L2 = pyr[2].reshape(P, -1)[:, :W2l]
    o0, o2 = -(2 * M0 - 10), -(M0 // 2 - 10)          # row offsets of element 0
    n0 = 2 * G * (NR - 1) + n0s + o0
    n2 = (G // 2) * (NR - 1) + n2s + o2
    Lp0 = torch.zeros(P, max(n0, o0 + W0), dtype=L0.dtype, device=L0.device)
    Lp0[:, o0:o0 + W0] = L0
    Lp2 = torch.zeros(P, max(n2, o2 + W2l), dtype=L2.dtype, device=L2.device)
    Lp2[:, o2:o2 + W2l] = L2
    rec = torch.zeros(P, NR, slots, dtype=L0.dtype, device=L0.device)
    rec[:, :, n2s:n2s + n0s] = Lp0.as_strided((P, NR, n0s), (Lp0.stride(0), 2 * G, 1))
    rec[:, :, :n2s] = Lp2.as_strided((P, NR, n2s), (Lp2.stride(0), G // 2, 1))
    del Lp0, Lp2
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="kitti")
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--slots", default="64,128", help="record sizes to time (bf16 elements: 64 or 128)")
    a = ap.parse_args()
    B, D, H, W1, W2, L, r, iters, _ = bench.CONFIGS[a.config]
    B = a.batch or B
    assert L == 4 and r == 4
    lib = _lib.dev_library().__enter__()
    fn = lib.rc_dev_lookup_records
    fn.restype = ctypes.c_int
    vp, ci, cl = ctypes.c_void_p, ctypes.c_int, ctypes.c_long
    fn.argtypes = [vp, ci, ci, ci, ctypes.POINTER(ci), vp, cl, ci, ci, ci, vp, vp]
    P = B * H * W1
    W1lvl = W2 >> 1
    slot_list = [int(v) for v in a.slots.split(",") if v]
    NRs = {sl: (W1lvl + r + 3 - M0) // GEOM[sl][0] + 1 for sl in slot_list}   # cover m1 up to W_1 + R + 3
    dev = torch.device("cuda", 0)
    res = {"config": a.config, "B": B, "NR": NRs, "M0": M0}
    with torch.no_grad():
        cfg = (B, D, H, W1, W2, L, r, iters, None)
        f1, f2, cs = bench.make_inputs(cfg, dev, seed=1, dtype=torch.bfloat16)
        blk = CorrBlock1D(f1, f2, num_levels=L, radius=r, channels_last=True)
        pyr = rcorr.build_pyramid(f1, f2, 3, torch.bfloat16, skip=(1,))
        recs = {sl: records(pyr, P, W2, W2 >> 2, NRs[sl], sl) for sl in slot_list}
        del pyr
        res["record_MB"] = {sl: t.numel() * 2 / 1e6 for sl, t in recs.items()}
        res["rows_shadowed_MB"] = sum(2 * t.numel() * 2 for t in (blk._levels[0], blk._levels[2])) / 1e6
        widths = _lib.int_array([W2 >> i for i in range(4)])
        out = torch.empty(B, L * (2 * r + 1), H, W1, device=dev).contiguous(memory_format=torch.channels_last)
        stream = torch.cuda.current_stream().cuda_stream

        def rec_lookup_for(sl):
            def f(c):
                rc = fn(recs[sl].data_ptr(), NRs[sl], M0, sl, widths, c.data_ptr(), 2 * H * W1, B, H, W1,
                        out.data_ptr(), stream)
                assert rc == 0, rc
                return out
            return f

        from test_corr_gpu import special_coords
        g = torch.Generator().manual_seed(5)
        checks = list(cs[:3]) + [special_coords(B, H, W1, W2, g).to(dev)]
        x = checks[-1][:, 0].clone()
        # no subnormal x: the prototype has no memory fallback (finish_pair's
        # path for a broken span relation, which only a subnormal x takes)
        x[(x.abs() < 1e-30) & (x != 0)] = 0.25
        x.view(-1)[100:400] = torch.linspace(-90, W2 + 90, 300, device=dev)   # both row edges
        checks[-1][:, 0] = x
        for sl in slot_list:
            for c in checks:
                ref = blk(c).clone()
                got = rec_lookup_for(sl)(c)
                same = torch.equal(ref.nan_to_num(7.0).view(torch.int32), got.nan_to_num(7.0).view(torch.int32))
                if not same:
                    d = (ref.nan_to_num(7.0) - got.nan_to_num(7.0)).abs()
                    print("MISMATCH", sl, d.max().item(), int((d > 0).sum()), flush=True)
                assert same
        res["bit_identical"] = True
        variants = [("product", blk)] + [(f"records{sl}", rec_lookup_for(sl)) for sl in slot_list]
        per = {n: [] for n, _ in variants}
        for _ in range(a.reps):
            for name, f in variants:
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(cs) + 1)]
                torch.cuda._sleep(3_000_000)
                ev[0].record()
                for k, c in enumerate(cs):
                    f(c)
                    ev[k + 1].record()
                torch.cuda.synchronize()
                per[name] += [ev[k].elapsed_time(ev[k + 1]) * 1e3 for k in range(len(cs))]
        res["lookup_us"] = {n: {"median": statistics.median(v), "min": min(v)} for n, v in per.items()}
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
