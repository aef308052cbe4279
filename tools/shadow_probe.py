"""Which stored levels pay for an RC_SHADOW copy (dev probe).

    python tools/shadow_probe.py [--config sceneflow|kitti] [--reps 5]

For each shadow setting (none, level 0, level 2, both) the CorrBlock1D build
and the 32 bench lookups are event-timed on the launch stream; prints build
µs, median lookup µs and the corr-path step = build + iters x lookup.
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from raft_stereo_amd import CorrBlock1D  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="sceneflow")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--row-align", type=int, default=16,
                    help="row stride granule of the stored levels in bytes (corr._ROW_ALIGN_BYTES)")
    ap.add_argument("--settings", default="none,l0,l2,l0+l2")
    ap.add_argument("--channels-last", action="store_true", help="NHWC lookup output")
    ap.add_argument("--dev-variant", default="",
                    help="RAFTCORR_LOOKUP_VARIANT for the lookups (libraftcorr_dev.so)")
    a = ap.parse_args()
    if a.dev_variant:
        from raft_stereo_amd import _lib
        _lib.dev_library().__enter__()
        os.environ["RAFTCORR_LOOKUP_VARIANT"] = a.dev_variant
    from raft_stereo_amd import corr as rcorr
    rcorr._ROW_ALIGN_BYTES = a.row_align
    cfg = bench.CONFIGS[a.config]
    B, D, H, W1, W2, L, r, iters, _ = cfg
    dev = torch.device("cuda", 0)
    dt = torch.bfloat16 if a.config in bench.BF16_CONFIGS else torch.float32
    f1, f2, coords = bench.make_inputs(cfg, dev, seed=1, dtype=dt)
    res = {"config": a.config, "row_align": a.row_align}
    want = set(a.settings.split(","))
    with torch.no_grad():
        for name, sh in (("none", ()), ("l0", (0,)), ("l2", (2,)), ("l0+l2", (0, 2))):
            if name not in want:
                continue
            bt, lt = [], []
            for _ in range(a.reps):
                torch.cuda._sleep(2_000_000)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                blk = CorrBlock1D(f1, f2, num_levels=L, radius=r, shadow=sh,
                                  channels_last=a.channels_last)
                e1.record()
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(iters + 1)]
                ev[0].record()
                for k in range(iters):
                    blk(coords[k])
                    ev[k + 1].record()
                torch.cuda.synchronize()
                assert blk._shadow == frozenset(sh)
                bt.append(e0.elapsed_time(e1) * 1e3)
                lt += [ev[k].elapsed_time(ev[k + 1]) * 1e3 for k in range(iters)]
                del blk
            bt.sort()
            lt.sort()
            b, l = bt[len(bt) // 2], lt[len(lt) // 2]
            res[name] = {"build_us": round(b, 1), "lookup_us": round(l, 2),
                         "step_us": round(b + iters * l, 1)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
