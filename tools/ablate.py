"""Interleaved A/B timing of kernel variants in ONE process (guide §5.4 rule 24).

    python tools/ablate.py [--config sceneflow] [--rounds 7]

Variants are dev-only env knobs read per launch by libraftcorr_dev.so (the
-DRAFTCORR_DEV build; the product library has none): RAFTCORR_BUILD_MODE
(volume.hip) and RAFTCORR_LOOKUP_VARIANT (lookup.hip).
Prints median / min microseconds per launch for each variant.
"""
import argparse
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from raft_stereo_amd import CorrBlock1D  # noqa: E402
from raft_stereo_amd import _lib  # noqa: E402
from raft_stereo_amd import corr as rcorr  # noqa: E402

_lib.dev_library().__enter__()   # every call of this tool goes to the knob-enabled build


def time_launches(fn, n):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
    torch.cuda._sleep(2_000_000)   # let the host queue all n launches first
    ev[0].record()
    for k in range(n):
        fn()
        ev[k + 1].record()
    torch.cuda.synchronize()
    return [ev[k].elapsed_time(ev[k + 1]) * 1e3 for k in range(n)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="sceneflow")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--build-modes", default="0,32,8,4,2,1,3")
    ap.add_argument("--lookup-variants", default="0,1,3")
    ap.add_argument("--staggers", default="", help="RAFTCORR_STAGGER values to try with mode 64")
    ap.add_argument("--chain", action="store_true",
                    help="time rc_corr_lookup_chain vs the per-level rc_corr_lookup")
    ap.add_argument("--bwd", action="store_true",
                    help="time the backward kernels")
    ap.add_argument("--bwd-variants", default="0,1,7",
                    help="RAFTCORR_LOOKUP_BWD_VARIANT values (0 product, 1 per-level waits, 3 capped occupancy, 4/5 prefetch 1/2 levels ahead, 6 grad_out loaded per level, 7 non-temporal grad_out loads)")
    ap.add_argument("--vbwd-variants", default="0",
                    help="RAFTCORR_VBWD_VARIANT values for the pair-layout volume backward (--bwd)")
    ap.add_argument("--convc1", action="store_true",
                    help="also time lookup+convc1+relu fused vs separate (MIOpen 1x1 conv)")
    a = ap.parse_args()
    cfg = bench.CONFIGS[a.config]
    B, D, H, W1, W2, L, r, iters, _ = cfg
    dev = torch.device("cuda", 0)
    res = {}
    bf16 = a.config in bench.BF16_CONFIGS
    with torch.no_grad():
        f1, f2, coords = bench.make_inputs(cfg, dev, seed=1,
                                           dtype=torch.bfloat16 if bf16 else torch.float32)
        ref_blk = CorrBlock1D(f1, f2, num_levels=L, radius=r)
        ref_out = ref_blk(coords[0])
        bm = [int(x) for x in a.build_modes.split(",") if x]
        lv = [int(x) for x in a.lookup_variants.split(",") if x]
        for m in bm:  # warm + correctness of product-equivalent modes
            os.environ["RAFTCORR_BUILD_MODE"] = str(m)
            blk = CorrBlock1D(f1, f2, num_levels=L, radius=r)
            if m in (0, 4, 5, 36, 128, 49, 50, 52, 53):
                for i in range(L + 1):
                    assert torch.equal(blk.corr_pyramid[i], ref_blk.corr_pyramid[i]), (m, i)
        os.environ["RAFTCORR_BUILD_MODE"] = "0"
        for v in lv:
            os.environ["RAFTCORR_LOOKUP_VARIANT"] = str(v)
            out = ref_blk(coords[0])
            assert torch.equal(out, ref_out), v
        stg = [int(x) for x in a.staggers.split(",") if x]
        for rnd in range(a.rounds):
            for m in bm:
                os.environ["RAFTCORR_BUILD_MODE"] = str(m)
                t = time_launches(lambda: CorrBlock1D(f1, f2, num_levels=L, radius=r), 3)
                res.setdefault(f"build_mode{m}", []).extend(t)
            for sv in stg:
                os.environ["RAFTCORR_BUILD_MODE"] = "64"
                os.environ["RAFTCORR_STAGGER"] = str(sv)
                t = time_launches(lambda: CorrBlock1D(f1, f2, num_levels=L, radius=r), 3)
                res.setdefault(f"build_stagger{sv}", []).extend(t)
            os.environ.pop("RAFTCORR_STAGGER", None)
            os.environ["RAFTCORR_BUILD_MODE"] = "0"
            for v in lv:
                os.environ["RAFTCORR_LOOKUP_VARIANT"] = str(v)
                t = time_launches(lambda: rcorr.lookup(ref_blk.corr_pyramid, coords[rnd % iters], L, r), 8)
                res.setdefault(f"lookup_v{v}", []).extend(t)
        if a.chain:
            os.environ["RAFTCORR_LOOKUP_VARIANT"] = "105"   # non-temporal stores: same values
            assert torch.equal(rcorr.lookup_chain(ref_blk.corr_pyramid, coords[0], L, r), ref_out)
            os.environ["RAFTCORR_LOOKUP_VARIANT"] = "0"
            for rnd in range(a.rounds):
                c = coords[rnd % iters]
                t = time_launches(lambda: rcorr.lookup_chain(ref_blk.corr_pyramid, c, L, r), 8)
                res.setdefault("lookup_chain", []).extend(t)
                t = time_launches(lambda: rcorr.lookup(ref_blk.corr_pyramid, c, L, r), 8)
                res.setdefault("lookup_perlevel", []).extend(t)
                for v in (101, 102, 103, 104, 105):   # no stores / no loads / loads only / math only / NT stores
                    os.environ["RAFTCORR_LOOKUP_VARIANT"] = str(v)
                    t = time_launches(lambda: rcorr.lookup_chain(ref_blk.corr_pyramid, c, L, r), 8)
                    res.setdefault(f"lookup_chain_v{v}", []).extend(t)
                os.environ["RAFTCORR_LOOKUP_VARIANT"] = "0"
        if a.bwd:
            P = B * H * W1
            widths = [W2 >> i for i in range(L)]
            g = torch.Generator().manual_seed(9)
            go = torch.randn(B, L * (2 * r + 1), H, W1, generator=g).to(dev)
            gper = rcorr.grad_buffers(P, widths, dev)
            bv = [int(x) for x in a.bwd_variants.split(",") if x]
            vv = [int(x) for x in a.vbwd_variants.split(",") if x]
            # bit-identity of the variants: same accumulation from the same start
            outs = {}
            for v in bv:
                os.environ["RAFTCORR_LOOKUP_BWD_VARIANT"] = str(v)
                gv = rcorr.grad_buffers(P, widths, dev)
                for k in range(3):
                    rcorr.lookup_backward(gv, coords[k], go, L, r)
                outs[v] = gv
            for v in bv[1:]:
                for i in range(L):
                    assert torch.equal(outs[v][i], outs[bv[0]][i]), ("bwd variant", v, i)
            del outs
            for rnd in range(a.rounds):
                c = coords[rnd % iters]
                for v in bv:
                    os.environ["RAFTCORR_LOOKUP_BWD_VARIANT"] = str(v)
                    t = time_launches(lambda: rcorr.lookup_backward(gper, c, go, L, r), 8)
                    res.setdefault(f"lookup_bwd_v{v}", []).extend(t)
                os.environ["RAFTCORR_LOOKUP_BWD_VARIANT"] = "0"
                t = time_launches(lambda: rcorr.build_backward(f1, f2, gper), 2)
                res.setdefault("volume_bwd", []).extend(t)
                for nl in (1, 2):   # fewer levels to fold on load (what a pre-folded G would cost)
                    for v in vv:
                        os.environ["RAFTCORR_VBWD_VARIANT"] = str(v)
                        t = time_launches(lambda: rcorr.build_backward(f1, f2, gper[:nl]), 2)
                        res.setdefault(f"volume_bwd_nlev{nl}_v{v}", []).extend(t)
                    os.environ["RAFTCORR_VBWD_VARIANT"] = "0"
            # the pair layout (the training default): RAFTCORR_VBWD_VARIANT values
            gpair = rcorr.grad_buffers(P, widths, dev, pair=True)
            for k in range(3):
                rcorr.lookup_backward(gpair, coords[k], go, L, r)
            ref_v = None
            for v in vv:
                os.environ["RAFTCORR_VBWD_VARIANT"] = str(v)
                o = rcorr.build_backward(f1, f2, gpair)
                if ref_v is None:
                    ref_v = o
                else:
                    assert all(torch.equal(x, y) for x, y in zip(o, ref_v)), ("vbwd variant", v)
            for rnd in range(a.rounds):
                for v in vv:
                    os.environ["RAFTCORR_VBWD_VARIANT"] = str(v)
                    t = time_launches(lambda: rcorr.build_backward(f1, f2, gpair), 2)
                    res.setdefault(f"volume_bwd_pair_v{v}", []).extend(t)
            os.environ["RAFTCORR_VBWD_VARIANT"] = "0"
        if a.convc1:
            conv = torch.nn.Conv2d(L * (2 * r + 1), 64, 1).to(dev)
            base = ref_blk.lookup_convc1(coords[0], conv.weight, conv.bias)
            os.environ["RAFTCORR_CONV_VARIANT"] = "1"   # one level at a time: same values
            assert torch.equal(ref_blk.lookup_convc1(coords[0], conv.weight, conv.bias), base)
            os.environ["RAFTCORR_CONV_VARIANT"] = "0"
            for rnd in range(a.rounds):
                c = coords[rnd % iters]
                t = time_launches(lambda: ref_blk.lookup_convc1(c, conv.weight, conv.bias), 8)
                res.setdefault("convc1_fused", []).extend(t)
                os.environ["RAFTCORR_CONV_VARIANT"] = "1"
                t = time_launches(lambda: ref_blk.lookup_convc1(c, conv.weight, conv.bias), 8)
                res.setdefault("convc1_fused_perlevel", []).extend(t)
                os.environ["RAFTCORR_CONV_VARIANT"] = "0"
                t = time_launches(lambda: torch.relu(conv(ref_blk(c))), 8)
                res.setdefault("convc1_separate", []).extend(t)
    out = {k: {"median_us": statistics.median(v), "min_us": min(v), "n": len(v)} for k, v in res.items()}
    print(json.dumps({"config": a.config, "results": out}, indent=1))


if __name__ == "__main__":
    main()
