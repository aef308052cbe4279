"""Dev probe: do 16-B buffer loads honour 2-B-misaligned offsets, into VGPRs
and by LDS DMA?  (libraftcorr_dev.so, rc_dev_align_probe.)

    python tools/align_probe.py
"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pkgload  # noqa: E402

pkgload.load()
from raft_stereo_amd import _lib  # noqa: E402


def main():
    lib = ctypes.CDLL(_lib.DEV_LIB_PATH)
    src = torch.arange(64 * 64 + 64, dtype=torch.int32).to(torch.uint8).cuda()   # byte b = b & 255
    for mode, name in ((0, "vgpr b128"), (1, "lds-dma b128"), (2, "lds-dma b32")):
        out = torch.zeros(5 * 64 * 4, dtype=torch.int32, device="cuda")
        rc = lib.rc_dev_align_probe(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                    mode, None)
        torch.cuda.synchronize()
        o = out.cpu().view(5, 64, 4).numpy().view("uint8").reshape(5, 64, 16)
        s = src.cpu().numpy()
        for sh in range(5):
            ok = all((o[sh, l] == s[64 * l + 2 * sh: 64 * l + 2 * sh + 16]).all() for l in range(64))
            first = list(o[sh, 1])
            print(f"{name:13s} shift {2 * sh} B: {'exact' if ok else 'WRONG'}  lane1 bytes {first}  rc={rc}")


if __name__ == "__main__":
    main()
