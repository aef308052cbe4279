"""Achievable HBM rate for the lookup's access pattern: random 128-byte lines.

    python tools/line_probe.py

The chain lookup reads ~3.5 random 128-B lines per pixel
from a pyramid far larger than the Infinity Cache and writes its output as a
coalesced stream.  This probe times the same two components in isolation on
the same device: (a) a gather of random 128-B rows (one index per row, rows
drawn uniformly from a 512 MB table) and (b) a plain coalesced copy, and
prints the GB/s of each.  The lookup's physical rate (PMC bytes / time) is
compared against (a) in DESIGN.md.
"""
import json

import torch


def timed(fn, reps=10):
    for _ in range(2):
        fn()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    ev[0].record()
    for k in range(reps):
        fn()
        ev[k + 1].record()
    torch.cuda.synchronize()
    ts = sorted(ev[k].elapsed_time(ev[k + 1]) for k in range(reps))
    return ts[len(ts) // 2] * 1e-3


def main():
    dev = torch.device("cuda", 0)
    rows_total = (512 << 20) // 128                 # 512 MB table of 128-B rows
    table = torch.randn(rows_total, 32, device=dev)
    res = {}
    for n_rows in (1 << 20, 1 << 21):               # 128 MB / 256 MB gathered
        idx = torch.randint(0, rows_total, (n_rows,), device=dev)
        out = torch.empty(n_rows, 32, device=dev)
        t = timed(lambda: torch.index_select(table, 0, idx, out=out))
        moved = n_rows * 128 * 2 + n_rows * 8        # rows read + written + indices
        res[f"gather_{n_rows * 128 >> 20}MB"] = {"us": t * 1e6, "GBps": moved / t / 1e9,
                                                 "read_GBps": n_rows * 128 / t / 1e9}
    src = torch.randn(64 << 20, device=dev)
    dst = torch.empty_like(src)
    t = timed(lambda: dst.copy_(src))
    res["copy_256MB"] = {"us": t * 1e6, "GBps": 2 * src.numel() * 4 / t / 1e9}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
