"""Interleaved A/B timing of the fp32 volume kernels in ONE process.

    python tools/build_ablate.py [--config sceneflow] [--rounds 9] [--modes 0,1,2,4,7]

Variants: 'exact' (rc::build_f32_ring_kernel, RC_BUILD_EXACT_F32) and the
split-bf16 kernel (rc::build_split_kernel) under the dev library's
RAFTCORR_SPLIT_MODE ablation flags: 0 product, 1 no operand loads, 2 no
epilogue stores, 4 no MFMAs (sums combine; timing only, wrong values); a
variant NAME=VALUE sets that dev knob instead (e.g. RAFTCORR_SPLIT_RING=85).
Prints the median / min microseconds per launch of each variant.
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

_lib.dev_library().__enter__()


def time_launches(fn, n):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
    torch.cuda._sleep(2_000_000)
    ev[0].record()
    for k in range(n):
        fn()
        ev[k + 1].record()
    torch.cuda.synchronize()
    return [ev[k].elapsed_time(ev[k + 1]) * 1e3 for k in range(n)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="sceneflow")
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--per", type=int, default=4)
    ap.add_argument("--modes", default="0,1,2,4,3,6,7")
    a = ap.parse_args()
    cfg = bench.CONFIGS[a.config]
    B, D, H, W1, W2, L, r, iters, _ = cfg
    dev = torch.device("cuda", 0)
    ll = a.config in bench.LOW_LATENCY_CONFIGS
    # RAFTCORR_SPLIT_MODE values of the split kernel (dev library)
    variants = ["exact"] + [m if "=" in m else int(m) for m in a.modes.split(",") if m]
    res = {str(v): [] for v in variants}
    with torch.no_grad():
        f1, f2, _ = bench.make_inputs(cfg, dev, seed=1)

        knobs = {kv.split("=")[0] for m in variants if isinstance(m, str) and "=" in m
                 for kv in m.split("+")}

        def run(v):
            for k in knobs:
                os.environ.pop(k, None)
            if v == "exact":
                os.environ["RAFTCORR_SPLIT_MODE"] = "0"
                return lambda: CorrBlock1D(f1, f2, num_levels=L, radius=r, low_latency=ll, exact_f32=True)
            if isinstance(v, str):   # NAME=VALUE[+NAME=VALUE]: dev knobs over the product mode
                os.environ["RAFTCORR_SPLIT_MODE"] = "0"
                for kv in v.split("+"):
                    k, val = kv.split("=")
                    os.environ[k] = val
            else:
                os.environ["RAFTCORR_SPLIT_MODE"] = str(v)
            return lambda: CorrBlock1D(f1, f2, num_levels=L, radius=r, low_latency=ll)
        ref = None
        for v in variants:
            blk = run(v)()
            if v == 0:
                ref = [t.clone() for t in blk.corr_pyramid[:4]]
        # variants with math and stores (no 1/2/4 ablation bits) must
        # reproduce the product bit for bit
        for v in variants:
            if ((isinstance(v, int) and v and not (v & 7)) or isinstance(v, str) and "=" in v
                    and "MODE=" not in v) and ref is not None:
                got = run(v)().corr_pyramid[:4]
                res.setdefault("bit_identical", {})[str(v)] = all(
                    bool(torch.equal(x, y)) for x, y in zip(got, ref))
                res.setdefault("norm_err_vs_0", {})[str(v)] = max(
                    float((x - y).abs().max() / y.abs().max()) for x, y in zip(got, ref))
        for _ in range(a.rounds):
            for v in variants:
                fn = run(v)
                res[str(v)] += time_launches(fn, a.per)
        os.environ["RAFTCORR_SPLIT_MODE"] = "0"
        for k in knobs:
            os.environ.pop(k, None)
    ident = res.pop("bit_identical", {})
    nerr = res.pop("norm_err_vs_0", {})
    out = {k: {"median_us": statistics.median(x), "min_us": min(x)} for k, x in res.items()}
    for k, v in ident.items():
        out[k]["bit_identical"] = v
        out[k]["norm_err_vs_mode0"] = nerr[k]
    flops = bench.volume_flops(B, D, H, W1, W2)
    for k, v in out.items():
        v["fp32_equiv_tflops"] = flops / (v["median_us"] * 1e-6) / 1e12
    print(json.dumps({"config": a.config, "variants": out,
                      "legend": "exact = fp32 MFMA ring; split modes (build_split_kernel): 0 "
                                "product, 1 no loads, 2 no stores, 4 no MFMA (sums combine); NAME=VALUE a dev knob"}, indent=1))


if __name__ == "__main__":
    main()
