"""A/B of the bf16 pyramid layouts at the KITTI config:
the product rows (levels 0 and 2 each with its half-line-shifted shadow copy,
two 128-B lines per pixel per lookup) vs the record layout (RC_LAYOUT_RECORDS:
one line per pixel, 1.8x the build's bytes).

    python tools/records_probe.py [--config kitti] [--reps 5] [--batch B]

Checks bit-identity of the lookups (bench field and special coordinates),
then times, interleaved, per layout: the build alone, one lookup (median
launch) and the whole corr step (build + 32 lookups, the bench's step).
"""
import argparse
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="kitti")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=0)
    a = ap.parse_args()
    B, D, H, W1, W2, L, r, iters, _ = bench.CONFIGS[a.config]
    B = a.batch or B
    dev = torch.device("cuda", 0)
    cfg = (B, D, H, W1, W2, L, r, iters, None)
    res = {"config": a.config, "B": B}
    layouts = ("rows", "records")
    with torch.no_grad():
        f1, f2, cs = bench.make_inputs(cfg, dev, seed=1, dtype=torch.bfloat16)
        mk = {lay: (lambda lay=lay: CorrBlock1D(f1, f2, num_levels=L, radius=r, channels_last=True, layout=lay))
              for lay in layouts}
        from test_corr_gpu import special_coords
        g = torch.Generator().manual_seed(5)
        blocks = {lay: mk[lay]() for lay in layouts}
        for c in list(cs[:3]) + [special_coords(B, H, W1, W2, g).to(dev)]:
            x, y = (blocks[lay](c) for lay in layouts)
            assert torch.equal(x.contiguous().view(torch.int32), y.contiguous().view(torch.int32))
        res["bit_identical"] = True
        res["MB"] = {"rows_shadowed": sum(2 * t.numel() * 2 for t in (blocks["rows"]._levels[0],
                                                                       blocks["rows"]._levels[2])) / 1e6,
                     "records": blocks["records"]._records.numel() * 2 / 1e6}
        del blocks
        t = {lay: {"build": [], "lookup": [], "step": []} for lay in layouts}
        for _ in range(a.reps):
            for lay in layouts:
                # build alone (device sleep first: no host gap inside the events)
                e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                torch.cuda._sleep(5_000_000)
                e[0].record()
                blk = mk[lay]()
                e[1].record()
                torch.cuda.synchronize()
                t[lay]["build"].append(e[0].elapsed_time(e[1]) * 1e3)
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(cs) + 1)]
                torch.cuda._sleep(5_000_000)
                ev[0].record()
                for k, c in enumerate(cs):
                    blk(c)
                    ev[k + 1].record()
                torch.cuda.synchronize()
                t[lay]["lookup"] += [ev[k].elapsed_time(ev[k + 1]) * 1e3 for k in range(len(cs))]
                del blk
                # the bench's step: build + iters lookups, wall time
                torch.cuda.synchronize()
                s0 = torch.cuda.Event(enable_timing=True)
                s1 = torch.cuda.Event(enable_timing=True)
                s0.record()
                for _k in range(3):
                    blk = mk[lay]()
                    for c in cs:
                        blk(c)
                    del blk
                s1.record()
                torch.cuda.synchronize()
                t[lay]["step"].append(s0.elapsed_time(s1) * 1e3 / 3)
        res["us"] = {lay: {k: statistics.median(v) for k, v in d.items()} for lay, d in t.items()}
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
