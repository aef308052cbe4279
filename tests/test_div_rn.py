"""Exhaustive device check of the sampler's fast correctly-rounded division.

The lookup kernels compute xn = 2x/(W-1) - 1 (model.py:271) with rc::div_rn
(raft-stereo_amd/csrc/common.h): Markstein's correction of a*RN(1/b) instead of
the IEEE division sequence.  Bit-exact lookups need RN(a/b) exactly, so this
test compares div_rn with IEEE division bit for bit on the GPU for every
divisor b = W-1 in [1, 8192] and every fp32 numerator with
2^-30 <= |a| < 2^15 -- the whole range where the quotient can reach the
sampler's output (common.h explains why the rest cannot) -- and for a sample
of wider divisors over their own a-range.
"""
import ctypes
import os

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "native", "_build", "libdivcheck.so")


def _lib():
    if not os.path.exists(LIB):
        raise RuntimeError(f"{LIB} missing: run __graft_entry__.build()")
    lib = ctypes.CDLL(LIB)
    lib.divcheck.argtypes = [ctypes.c_int] * 4 + [ctypes.POINTER(ctypes.c_ulonglong),
                                                  ctypes.POINTER(ctypes.c_uint * 3)]
    lib.divcheck.restype = ctypes.c_int
    return lib


def test_divcheck_library_exports():
    lib = _lib()
    assert hasattr(lib, "divcheck")


@pytest.mark.gpu
def test_div_rn_matches_ieee_division_exhaustively():
    import torch
    assert torch.cuda.is_available()
    lib = _lib()
    total = 0
    for b_lo in range(1, 8193, 1024):
        count = ctypes.c_ulonglong(0)
        first = (ctypes.c_uint * 3)()
        rc = lib.divcheck(b_lo, b_lo + 1023, -30, 15, ctypes.byref(count), ctypes.byref(first))
        assert rc == 0, f"divcheck launch failed: hipError {rc}"
        assert count.value == 0, (f"div_rn differs from IEEE division {count.value} times in "
                                  f"b=[{b_lo},{b_lo + 1023}], first b={first[1]} a=0x{first[2]:08x}")
        total += 1024 * 2 * 45 * (1 << 23)
    # wider rows: sampled divisors up to 2^20, numerators up to 2^22
    for b in (8193, 12345, 16383, 16384, 32767, 65535, 99991, 131071, 524287, 1048575):
        count = ctypes.c_ulonglong(0)
        first = (ctypes.c_uint * 3)()
        rc = lib.divcheck(b, b, -30, 22, ctypes.byref(count), ctypes.byref(first))
        assert rc == 0, f"divcheck launch failed: hipError {rc}"
        assert count.value == 0, (f"div_rn differs from IEEE division {count.value} times at "
                                  f"b={b}, first a=0x{first[2]:08x}")
        total += 2 * 52 * (1 << 23)
    print(f"checked {total:.3e} quotients")
