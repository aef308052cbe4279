"""Cost model of the lookup's access shape (dev probe, libraftcorr_dev.so).

    python tools/gather_probe.py

rc_dev_gather_probe (csrc/probe.hip): one lane per "pixel", K 16-B loads per
lane into the lane's own row, no tap math.  Cases vary the number of loads,
how many of them are predicated off, whether they are consecutive (a span,
~K*16/128 + 1 lines) or scattered (K lines), how many lanes share a line, and
whether the table is HBM-sized or cache-resident.  Prints median us per
launch, requests/s and distinct-line estimates.
"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pkgload  # noqa: E402

pkgload.load()
from raft_stereo_amd import _lib  # noqa: E402


def main():
    lib = _lib.dev_library().__enter__()
    fn = lib.rc_dev_gather_probe
    fn.restype = ctypes.c_int
    vp, ci, cll = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong
    fn.argtypes = [vp, cll, ci, ci, ci, ci, ci, ctypes.c_uint, cll, vp, vp]
    dev = torch.device("cuda", 0)
    lanes = 259200
    big = torch.randn(lanes * 240, device=dev)                    # 249 MB, level-0 sized
    wide = torch.randn(lanes // 8 * 2048 + 2048, device=dev)      # rows of 2048 floats
    small = torch.randn(2048 * 240, device=dev)                   # 2 MB: L2-resident
    out = torch.empty(lanes, device=dev)
    stream = torch.cuda.current_stream().cuda_stream

    def run(table, nrows, row, mode, G, K, oob, reps=12):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
        for _ in range(2):
            assert fn(table.data_ptr(), nrows, row, mode, G, K, oob, 1, lanes, out.data_ptr(), stream) == 0
        torch.cuda._sleep(2_000_000)
        ev[0].record()
        for k in range(reps):
            assert fn(table.data_ptr(), nrows, row, mode, G, K, oob, 7 + k, lanes, out.data_ptr(),
                      stream) == 0
            ev[k + 1].record()
        torch.cuda.synchronize()
        ts = sorted(ev[k].elapsed_time(ev[k + 1]) * 1e3 for k in range(reps))
        return ts[len(ts) // 2]

    cases = {
        "span16": (big, lanes, 240, 0, 1, 16, 0),
        "span16_oob8": (big, lanes, 240, 0, 1, 16, 8),
        "span16_oob12": (big, lanes, 240, 0, 1, 16, 12),
        "span12": (big, lanes, 240, 0, 1, 12, 0),
        "span8": (big, lanes, 240, 0, 1, 8, 0),
        "span4": (big, lanes, 240, 0, 1, 4, 0),
        "scatter16": (big, lanes, 240, 1, 1, 16, 0),
        "scatter8": (big, lanes, 240, 1, 1, 8, 0),
        "scatter4": (big, lanes, 240, 1, 1, 4, 0),
        "span16_small": (small, 2048, 240, 0, 1, 16, 0),
        "scatter16_small": (small, 2048, 240, 1, 1, 16, 0),
        "span8_small": (small, 2048, 240, 0, 1, 8, 0),
        "shared_g2_k8": (wide, lanes // 8, 2048, 2, 2, 8, 0),
        "shared_g4_k8": (wide, lanes // 8, 2048, 2, 4, 8, 0),
        "shared_g8_k8": (wide, lanes // 8, 2048, 2, 8, 8, 0),
    }
    res = {}
    for name, (t, nrows, row, mode, G, K, oob) in cases.items():
        us = run(t, nrows, row, mode, G, K, oob)
        req = lanes * (K - oob)
        res[name] = {"us": round(us, 2), "Greq_per_s": round(req / us / 1e3, 1),
                     "wave_instr_per_us_per_cu": round(lanes / 64 * K / us / 256, 2)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
