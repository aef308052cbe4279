"""Whole-network time at BASELINE configs[1] (B=8, 540x960, 32 iterations)
under PyTorch/MIOpen settings that leave the ops unchanged (dev probe):
default, MIOpen algorithm search (torch.backends.cudnn.benchmark), and the
fused coords step.  Prints one JSON line.

    python tools/e2e_settings_probe.py [--steps 3]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def run(variant, steps):
    torch.backends.cudnn.benchmark = variant.get("benchmark", False)
    cfg = bench.CONFIGS["sceneflow"]
    t0 = time.perf_counter()
    r = bench.e2e_pairs_per_s(cfg, torch.device("cuda", 0), steps, 2, fuse_step=variant.get("fuse", False),
                              mixed=variant.get("mixed", False))
    r["wall_s"] = time.perf_counter() - t0
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    out = {}
    for name, v in (("default", {}), ("benchmark", {"benchmark": True}),
                    ("benchmark+fuse_step", {"benchmark": True, "fuse": True}),
                    ("default_again", {})):
        r = run(v, a.steps)
        out[name] = {"ms_per_batch": r["ms_per_batch"], "pairs_per_s": r["pairs_per_s"], "wall_s": r["wall_s"]}
        print(name, out[name], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
