"""RC_LAYOUT_RECORDS geometry on the host (no GPU): for every level-0 width
the record build accepts (64 < W2 <= 320), every radius 1..4 and a dense
sweep of fp32 coordinates across and beyond the row, the elements the pair
kernel's exact-span predicate reads for a pixel (tap_span in lookup.hip, the
taps of levels 2k and 2k+1 of model.py:297-316) lie inside the slots of ITS
level in the record the lookup picks (floor(x/2) clamped to the records'
range) -- so no chunk ever mixes in the other level's slots or misses a tap.
Also the C-ABI's refusals of the flag, which happen before any launch."""
import ctypes

import numpy as np
import pytest

import raft_stereo_amd  # noqa: F401  (registered by conftest)
from raft_stereo_amd import _lib

f32 = np.float32
M0 = -8


def rec_e0(r):
    return 16 * r + 2 * M0 - 10


def rec_e2(r):
    return 4 * r + M0 // 2 - 10


def tap_span(xl, W, R):
    """lookup.hip tap_span: the exact element range [f, l] the taps read
    (the reference's normalise / unnormalise round trip in fp32)."""
    Wm1 = f32(W - 1)
    half = f32(Wm1 / f32(2))

    def rt(v):
        q = (f32(2) * v) / Wm1                  # correctly rounded fp32 quotient (div_rn)
        return ((q - f32(1)) + f32(1)) * half

    pa = rt(f32(-R) + xl)
    pb = rt(f32(R) + xl)
    f = np.maximum(np.floor(pa).astype(np.int64), 0)
    l = np.minimum(np.floor(pb).astype(np.int64) + 1, W - 1)
    return f, l


@pytest.mark.parametrize("R", [1, 2, 3, 4])
def test_record_spans_fit_their_slots(R):
    for W2 in range(65, 321):
        W = [W2 >> l for l in range(4)]
        NR = _lib.rec_count(W2)
        x = np.concatenate([np.arange(-100.0, W2 + 100.0, 0.125, dtype=np.float64),
                            [-1e-45, 1e-45, -0.0, 3.0e-39]]).astype(f32)
        m1 = np.floor(x / f32(2)).astype(np.int64)
        r = (np.clip(m1, M0, M0 + 8 * NR - 1) - M0) >> 3
        for lo, first, nslots in ((0, rec_e0(r), 38), (2, rec_e2(r), 26)):
            xlo = x / f32(1 << lo)
            xhi = x / f32(2 << lo)
            inwin = (xhi > -(R + 4)) & (xhi < W[lo + 1] + R + 4)
            f0, l0 = tap_span(xlo, W[lo], R)
            f1, l1 = tap_span(xhi, W[lo + 1], R)
            e_lo = np.where(f0 <= l0, f0, 1 << 30)
            e_hi = np.where(f0 <= l0, l0, -1)
            e_lo = np.where(f1 <= l1, np.minimum(e_lo, 2 * f1), e_lo)
            e_hi = np.where(f1 <= l1, np.maximum(e_hi, 2 * l1 + 1), e_hi)
            read = inwin & (e_lo <= e_hi)
            ok = (e_lo >= first) & (e_hi < first + nslots)
            bad = read & ~ok
            assert not bad.any(), (W2, R, lo, x[bad][:5])


def test_rec_count_matches_header():
    import re
    text = open(_lib.HEADER).read()
    m = re.search(r"#define RC_REC_COUNT\(W2\)\s+(.+)", text)
    expr = m.group(1)
    for W2 in (65, 100, 240, 311, 320, 1000):
        assert eval(expr.replace("W2", str(W2))) == _lib.rec_count(W2)
    m = re.search(r"#define RC_LAYOUT_RECORDS\s+(0x[0-9a-fA-F]+)", text)
    assert m and int(m.group(1), 16) == _lib.RC_LAYOUT_RECORDS
    assert _lib.rec_count(311) == 22


def test_records_flag_validation():
    """The build refuses everything outside the record kernel before any
    launch (B = 0 shapes return after validation), and the entry points that
    do not serve the layout refuse the flag."""
    L = _lib.lib()
    f = lambda a: ctypes.c_void_p(a)  # noqa: E731
    RB = _lib.RC_BF16 | _lib.RC_LAYOUT_RECORDS

    def build(dt=_lib.RC_BF16, pdt=RB, D=256, W2=311, nbuf=3, ptrs=None):
        p = ptrs if ptrs is not None else _lib.ptr_array([f(0x1000), None, None])
        return L.rc_corr_build(f(0x2000), f(0x3000), dt, 0, D, 4, 311, W2, p, None, nbuf, pdt, None)

    assert build() == _lib.RC_OK
    assert build(dt=_lib.RC_F32) == _lib.RC_EUNSUPPORTED
    assert build(pdt=_lib.RC_F32 | _lib.RC_LAYOUT_RECORDS) == _lib.RC_EUNSUPPORTED
    assert build(pdt=RB | _lib.shadow_level(0)) == _lib.RC_EUNSUPPORTED
    assert build(nbuf=1, ptrs=_lib.ptr_array([f(0x1000)])) == _lib.RC_EUNSUPPORTED
    assert build(ptrs=_lib.ptr_array([f(0x1000), None, f(0x4000)])) == _lib.RC_EUNSUPPORTED
    assert build(W2=64) == _lib.RC_EUNSUPPORTED
    assert build(W2=321) == _lib.RC_EUNSUPPORTED
    assert build(D=224) == _lib.RC_EUNSUPPORTED
    assert build(pdt=RB | _lib.RC_LAYOUT_DISPARITY) == _lib.RC_EINVAL
    assert L.rc_last_error()
    ptrs = _lib.ptr_array([f(0x1000), None, None, None])
    w = _lib.int_array([311, 155, 77, 38])
    assert L.rc_corr_lookup(ptrs, w, None, RB, 4, 4, f(0x2000), 0, 1, 1, 311, f(0x3000), None) == \
        _lib.RC_EUNSUPPORTED
    assert L.rc_corr_lookup_conv(ptrs, w, None, RB, 4, 4, f(0x2000), 0, 1, 1, 311, f(0x4000), None, 4, 1,
                                 f(0x3000), None) == _lib.RC_EUNSUPPORTED
    assert L.rc_corr_lookup_step(ptrs, w, None, RB, 4, 4, 0, f(0x2000), None, f(0x3000), f(0x5000), 1, 1, 311,
                                 f(0x4000), None) == _lib.RC_EUNSUPPORTED
    # the chain lookup: 4 bf16 levels, no shadow, records only in pyr[0]
    chain = lambda p, dt, lv=4: L.rc_corr_lookup_chain(p, w, None, dt, lv, 4, f(0x2000), 0, 1, 1, 311,  # noqa: E731
                                                       f(0x3000), None)
    assert chain(ptrs, _lib.RC_F32 | _lib.RC_LAYOUT_RECORDS) == _lib.RC_EUNSUPPORTED
    assert chain(ptrs, RB | _lib.shadow_level(0)) == _lib.RC_EUNSUPPORTED
    assert chain(_lib.ptr_array([f(0x1000), None, f(0x4000), None]), RB) == _lib.RC_EINVAL
    assert chain(ptrs, RB, lv=2) == _lib.RC_EUNSUPPORTED


@pytest.mark.parametrize("W2", [65, 130, 240, 311, 320])
def test_records_level_gathers_the_documented_geometry(W2):
    """corr.records_level (the corr_pyramid gather of layout="records") on a
    CPU tensor laid out by the header's definition, written here directly:
    record r, slot s < 26 = level-2 element 4r - 14 + s, slot s >= 26 =
    level-0 element 16r - 26 + (s - 26), zeros off the row."""
    import torch
    from raft_stereo_amd import corr as rcorr
    P, NR = 5, _lib.rec_count(W2)
    g = torch.Generator().manual_seed(W2)
    l0 = torch.randn(P, W2, generator=g).to(torch.bfloat16)
    l2 = torch.randn(P, W2 >> 2, generator=g).to(torch.bfloat16)
    rec = torch.zeros(P, NR, 64, dtype=torch.bfloat16)
    for r in range(NR):
        for s in range(64):
            if s < 26:
                e, src, W = rec_e2(r) + s, l2, W2 >> 2
            else:
                e, src, W = rec_e0(r) + s - 26, l0, W2
            if 0 <= e < W:
                rec[:, r, s] = src[:, e]
    got0 = rcorr.records_level(rec, 0, W2).reshape(P, -1)
    got2 = rcorr.records_level(rec, 2, W2).reshape(P, -1)
    assert torch.equal(got0.view(torch.int16), l0.view(torch.int16))
    assert torch.equal(got2.view(torch.int16), l2.view(torch.int16))
