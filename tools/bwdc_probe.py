"""Deferred lookup backward (rc_corr_lookup_backward_calls) A/B (dev probe).

    python tools/bwdc_probe.py [--config sceneflow] [--rounds 7]

Variant 3 = compact rows (each lane keeps only the range its calls touch;
the product), 1 = whole rows, software-pipelined, 2 = whole rows, two read-modify-writes
per call, no overlap (RAFTCORR_BWDC_VARIANT), through libraftcorr_dev.so,
interleaved in one process on the bench workload (32 calls, one output
gradient per call).  Prints median microseconds per launch and whether the
two write the same gradient rows bit for bit.
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
from raft_stereo_amd import _lib  # noqa: E402
from raft_stereo_amd import corr as rcorr  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="sceneflow")
    ap.add_argument("--rounds", type=int, default=7)
    a = ap.parse_args()
    cfg = bench.CONFIGS[a.config]
    B, D, H, W1, W2, L, r, iters, _ = cfg
    dev = torch.device("cuda", 0)
    _, _, coords = bench.make_inputs(cfg, dev, seed=1)
    g = torch.Generator().manual_seed(99)
    gl = [torch.randn(B, L * (2 * r + 1), H, W1, generator=g).to(dev) for _ in range(iters)]
    P = B * H * W1
    widths = [W2 >> i for i in range(L)]
    bufs = {v: rcorr.grad_buffers(P, widths, dev, pair=True, zero=False) for v in (3, 1, 2)}
    times = {3: [], 1: [], 2: []}
    with _lib.dev_library():
        for rd in range(a.rounds + 1):
            for v in (3, 1, 2):
                os.environ["RAFTCORR_BWDC_VARIANT"] = str(v)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                rcorr.lookup_backward_calls(bufs[v], coords[:iters], gl, L, r, overwrite=True)
                e1.record()
                torch.cuda.synchronize()
                if rd:
                    times[v].append(e0.elapsed_time(e1) * 1e3)
        os.environ["RAFTCORR_BWDC_VARIANT"] = "0"
    same = all(torch.equal(x, y) and torch.equal(x, z)
               for x, y, z in zip(bufs[3], bufs[1], bufs[2]) if x is not None)
    print(json.dumps({"config": a.config, "calls": iters,
                      "compact_us": statistics.median(times[3]),
                      "whole_row_pipelined_us": statistics.median(times[1]),
                      "whole_row_unpipelined_us": statistics.median(times[2]), "bit_identical": same}))


if __name__ == "__main__":
    main()
