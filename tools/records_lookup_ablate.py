"""Where the record lookup's time goes: interleaved
32-launch sequences at the KITTI config of the record lookup and its
dev-library timing modes (RAFTCORR_REC_LOOKUP: 1 no output stores, 2 no
record loads, 3 record loads only, 4 the cooperative whole-record fetch
into LDS (the product since r06o), 5 / 6 that without output stores / loads
only, 9 per-lane chunk loads, 10 two 64-pixel groups per wave).

    python tools/records_lookup_ablate.py [--reps 5] [--batch B]
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
from raft_stereo_amd import CorrBlock1D, _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--modes", default="0,1,2,3,4,5,6")
    a = ap.parse_args()
    B, D, H, W1, W2, L, r, iters, _ = bench.CONFIGS["kitti"]
    B = a.batch or B
    dev = torch.device("cuda", 0)
    modes = [int(m) for m in a.modes.split(",")]
    t = {m: [] for m in modes}
    with torch.no_grad(), _lib.dev_library():
        f1, f2, cs = bench.make_inputs((B, D, H, W1, W2, L, r, iters, None), dev, seed=1, dtype=torch.bfloat16)
        blk = CorrBlock1D(f1, f2, num_levels=L, radius=r, channels_last=True, layout="records")
        # the cooperative variants (modes 4, 10) return the product's output bit for bit
        from test_corr_gpu import special_coords
        g = torch.Generator().manual_seed(7)
        same4 = True
        for c in (cs[0], special_coords(B, H, W1, W2, g).to(dev)):
            os.environ["RAFTCORR_REC_LOOKUP"] = "0"
            ref = blk(c).clone()
            for m in ("4", "10"):
                os.environ["RAFTCORR_REC_LOOKUP"] = m
                got = blk(c)
                same4 &= bool(torch.equal(ref.contiguous().view(torch.int32), got.contiguous().view(torch.int32)))
        for _ in range(a.reps):
            for m in modes:
                os.environ["RAFTCORR_REC_LOOKUP"] = str(m)
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(cs) + 1)]
                torch.cuda._sleep(3_000_000)
                ev[0].record()
                for k, c in enumerate(cs):
                    blk(c)
                    ev[k + 1].record()
                torch.cuda.synchronize()
                t[m] += [ev[k].elapsed_time(ev[k + 1]) * 1e3 for k in range(len(cs))]
        os.environ.pop("RAFTCORR_REC_LOOKUP", None)
    print(json.dumps({"B": B, "coop_bit_identical": same4, "lookup_us": {m: statistics.median(v) for m, v in t.items()}}), flush=True)


if __name__ == "__main__":
    main()
