"""The C-ABI library loads, exports every symbol include/raftcorr.h declares,
and its host-side validation behaves -- no GPU needed (nothing launches)."""
import ctypes
import re

import pytest

import raft_stereo_amd  # noqa: F401  (registered by conftest)
from raft_stereo_amd import _lib


def declared_symbols():
    text = open(_lib.HEADER).read()
    return sorted(set(re.findall(r"^(?:int|const char \*)\s*(rc_\w+)\s*\(", text, re.M)))


def test_header_and_binding_agree():
    assert declared_symbols() == sorted(_lib.SIGNATURES)


def test_library_exports_all_symbols():
    dll = _lib.lib()
    for name in declared_symbols():
        assert hasattr(dll, name), name
    assert dll.rc_abi_version() == _lib.ABI_VERSION


def test_defines_match():
    text = open(_lib.HEADER).read()
    for name in ["RC_F32", "RC_BF16", "RC_OK", "RC_EINVAL", "RC_EUNSUPPORTED", "RC_EHIP",
                 "RC_MAX_LEVELS", "RC_ABI_VERSION"]:
        m = re.search(rf"#define {name}\s+(\d+)", text)
        assert m, name
        ours = getattr(_lib, name if name != "RC_ABI_VERSION" else "ABI_VERSION")
        assert int(m.group(1)) == ours, name


def _build(**kw):
    args = dict(f1=None, f2=None, dt=0, B=1, D=8, H=1, W1=8, W2=8, pyr=None, nbuf=1, pdt=0)
    args.update(kw)
    ptrs = _lib.ptr_array([None] * max(args["nbuf"], 1)) if args["pyr"] is None else args["pyr"]
    return _lib.lib().rc_corr_build(args["f1"], args["f2"], args["dt"], args["B"], args["D"],
                                    args["H"], args["W1"], args["W2"], ptrs, None, args["nbuf"],
                                    args["pdt"], None)


@pytest.mark.parametrize("kw,code", [
    (dict(nbuf=0), _lib.RC_EINVAL),
    (dict(nbuf=9), _lib.RC_EINVAL),
    (dict(W2=8, nbuf=5), _lib.RC_EINVAL),      # level 4 of width 0 (model.py:294 raises)
    (dict(D=0), _lib.RC_EINVAL),
    (dict(dt=7), _lib.RC_EINVAL),
    (dict(pdt=5), _lib.RC_EINVAL),
    (dict(), _lib.RC_EINVAL),                   # null feature maps
])
def test_build_validation(kw, code):
    assert _build(**kw) == code
    assert _lib.lib().rc_last_error()


def test_build_empty_is_noop():
    assert _build(B=0) == _lib.RC_OK


def test_lookup_validation():
    L = _lib.lib()
    ptrs = _lib.ptr_array([None])
    w = _lib.int_array([8])
    assert L.rc_corr_lookup(ptrs, w, None, 0, 0, 4, None, 0, 1, 1, 8, None, None) == _lib.RC_EINVAL
    assert L.rc_corr_lookup(ptrs, w, None, 0, 1, 9, None, 0, 1, 1, 8, None, None) == _lib.RC_EUNSUPPORTED
    assert L.rc_corr_lookup(ptrs, w, None, 3, 1, 4, None, 0, 1, 1, 8, None, None) == _lib.RC_EINVAL
    assert L.rc_corr_lookup(ptrs, w, None, 0, 1, 4, None, 0, 0, 1, 8, None, None) == _lib.RC_OK
    # misaligned level pointer is rejected before any launch
    bad = _lib.ptr_array([ctypes.c_void_p(0x1004)])
    assert L.rc_corr_lookup(bad, w, None, 0, 1, 4, ctypes.c_void_p(0x2000), 0, 1, 1, 8,
                            ctypes.c_void_p(0x3000), None) == _lib.RC_EINVAL
    assert b"aligned" in L.rc_last_error()
    # a row stride below the width is rejected
    good = _lib.ptr_array([ctypes.c_void_p(0x1000)])
    assert L.rc_corr_lookup(good, w, _lib.long_array([7]), 0, 1, 4, ctypes.c_void_p(0x2000), 0, 1,
                            1, 8, ctypes.c_void_p(0x3000), None) == _lib.RC_EINVAL


def test_pool_validation():
    L = _lib.lib()
    assert L.rc_corr_pool(None, 1, None, 1, 4, 1, 0, None) == _lib.RC_EINVAL
    assert L.rc_corr_pool(None, 8, None, 4, 0, 8, 0, None) == _lib.RC_OK
    assert L.rc_corr_pool(None, 7, None, 4, 0, 8, 0, None) == _lib.RC_EINVAL   # ld_in < W_in


def test_shadow_flag_and_offset_match_header():
    """RC_SHADOW (ABI v5): the flag value and RC_SHADOW_OFFSET agree with the
    binding's helper; the copy sits half a 128-B line after a line boundary."""
    text = open(_lib.HEADER).read()
    m = re.search(r"#define RC_SHADOW\s+(0x[0-9a-fA-F]+)", text)
    assert m and int(m.group(1), 16) == _lib.RC_SHADOW
    for rows, ld, es in [(1, 4, 4), (259200, 240, 4), (259200, 60, 4), (1870976, 312, 2), (3, 8, 2)]:
        off = _lib.shadow_offset(rows, ld, es)
        assert off % 128 == 64 and off >= rows * ld * es and off - rows * ld * es < 192


def test_shadow_window_validation():
    """A level whose primary + shadow copy exceed the pair kernel's 4 GiB of
    32-bit buffer offsets is refused before any launch."""
    L = _lib.lib()
    ptrs = _lib.ptr_array([ctypes.c_void_p(0x1000), None, ctypes.c_void_p(0x2000), None])
    w = _lib.int_array([1024, 512, 256, 128])
    rc = L.rc_corr_lookup_chain(ptrs, w, None, _lib.RC_F32 | _lib.RC_SHADOW, 4, 4,
                                ctypes.c_void_p(0x3000), 0, 1, 1000, 1000, ctypes.c_void_p(0x4000), None)
    assert rc == _lib.RC_EUNSUPPORTED and b"4 GiB" in L.rc_last_error()
    # the same request without the flag passes validation up to the launch
    # (not attempted here: H*W1 rows of fake pointers) -- only the flag differs
    assert _build(pdt=_lib.RC_F32 | _lib.RC_SHADOW, B=0) == _lib.RC_OK


def test_channels_last_flag_needs_pair_layout():
    """RC_OUT_CHANNELS_LAST is served by the pair kernel only: a 3-level
    (level-1 chain) request with it is refused before any launch."""
    L = _lib.lib()
    text = open(_lib.HEADER).read()
    m = re.search(r"#define RC_OUT_CHANNELS_LAST\s+(0x[0-9a-fA-F]+)", text)
    assert m and int(m.group(1), 16) == _lib.RC_OUT_CHANNELS_LAST
    ptrs = _lib.ptr_array([ctypes.c_void_p(0x1000), ctypes.c_void_p(0x2000), None])
    w = _lib.int_array([64, 32, 16])
    rc = L.rc_corr_lookup_chain(ptrs, w, None, _lib.RC_F32 | _lib.RC_OUT_CHANNELS_LAST, 3, 4,
                                ctypes.c_void_p(0x3000), 0, 1, 2, 64, ctypes.c_void_p(0x4000), None)
    assert rc == _lib.RC_EUNSUPPORTED and b"pair" in L.rc_last_error()


def test_grad_shadow_flag_validation():
    """RC_SHADOW_LEVEL bits on the backward entry points:
    levels 0 and 2 of the 4-level pair layout only, refused before any launch."""
    L = _lib.lib()
    f = lambda a: ctypes.c_void_p(a)  # noqa: E731
    w = _lib.int_array([64, 32, 16, 8])
    pair = _lib.ptr_array([f(0x1000), None, f(0x2000), None])
    full = _lib.ptr_array([f(0x1000), f(0x2000), f(0x3000), f(0x5000)])
    args = lambda ptrs, lv: (ptrs, w, None, lv, 4, f(0x7000), 0, 1, 2, 64, f(0x8000), None)  # noqa: E731
    for ptrs, lv in ((full, 4 | _lib.shadow_level(0)), (pair, 4 | _lib.shadow_level(1)),
                     (_lib.ptr_array([f(0x1000), None]), 2 | _lib.shadow_level(0))):
        assert L.rc_corr_lookup_backward(*args(ptrs, lv)) == _lib.RC_EUNSUPPORTED
        assert b"RC_SHADOW" in L.rc_last_error()
    bb = lambda ptrs, lv: L.rc_corr_build_backward(  # noqa: E731
        f(0x1000), f(0x2000), _lib.RC_F32, 1, 32, 2, 64, 64, ptrs, None, lv, f(0x3000), f(0x4000), None)
    assert bb(full, 4 | _lib.shadow_level(0)) == _lib.RC_EUNSUPPORTED
    assert bb(_lib.ptr_array([f(0x1000), None, f(0x2000)]), 3 | _lib.shadow_level(1)) == _lib.RC_EUNSUPPORTED
    assert b"RC_SHADOW" in L.rc_last_error()
    from raft_stereo_amd import corr as rcorr
    with pytest.raises(ValueError):
        rcorr.grad_buffers(16, [64, 32], "cpu", pair=True, shadow=(0,))
    with pytest.raises(ValueError):
        rcorr.grad_buffers(16, [64, 32, 16, 8], "cpu", pair=True, shadow=(1,))


def test_pyr_dtype_flag_bits_validated():
    """RC_OUT_CHANNELS_LAST on an entry point that cannot honour it
    is refused (RC_EUNSUPPORTED), and unknown flag bits are RC_EINVAL, on every
    entry point that takes a pyr_dtype -- before any launch."""
    L = _lib.lib()
    f = lambda a: ctypes.c_void_p(a)  # noqa: E731
    ptrs = _lib.ptr_array([f(0x1000)])
    w = _lib.int_array([8])
    cl = _lib.RC_F32 | _lib.RC_OUT_CHANNELS_LAST
    junk = _lib.RC_F32 | 0x400000
    for dt, code in ((cl, _lib.RC_EUNSUPPORTED), (junk, _lib.RC_EINVAL)):
        assert L.rc_corr_lookup(ptrs, w, None, dt, 1, 4, f(0x2000), 0, 1, 1, 8, f(0x3000), None) == code
        assert L.rc_corr_lookup_conv(ptrs, w, None, dt, 1, 4, f(0x2000), 0, 1, 1, 8, f(0x4000), None, 4,
                                     1, f(0x3000), None) == code
        assert _build(pdt=dt, B=0) == code
        assert L.rc_corr_pool(None, 8, None, 4, 0, 8, dt, None) == code
        assert L.rc_last_error()
    two = _lib.ptr_array([f(0x1000), None])
    w2 = _lib.int_array([64, 32])
    for fn in ("rc_corr_lookup_chain",):
        assert getattr(L, fn)(two, w2, None, junk, 2, 4, f(0x2000), 0, 1, 1, 64, f(0x3000),
                              None) == _lib.RC_EINVAL
    assert L.rc_corr_lookup_step(two, w2, None, junk, 2, 4, 1, f(0x2000), None, f(0x3000), f(0x5000),
                                 1, 1, 64, f(0x4000), None) == _lib.RC_EINVAL


def test_build_backward_exact_flag():
    """ABI v8: rc_corr_build_backward takes RC_BUILD_EXACT_F32 in fmap_dtype
    (the exact fp32 MFMA kernel instead of the split-bf16 one); any other
    dtype or flag bit is refused before a launch.  B = 0 returns after the
    dtype check without touching memory."""
    L = _lib.lib()
    f = lambda a: ctypes.c_void_p(a)  # noqa: E731
    g = _lib.ptr_array([f(0x1000)])
    bb = lambda dt, B: L.rc_corr_build_backward(  # noqa: E731
        f(0x1000), f(0x2000), dt, B, 32, 2, 64, 64, g, None, 1, f(0x3000), f(0x4000), None)
    assert bb(_lib.RC_F32 | _lib.RC_BUILD_EXACT_F32, 0) == _lib.RC_OK
    assert bb(_lib.RC_F32, 0) == _lib.RC_OK
    assert bb(_lib.RC_BF16, 0) == _lib.RC_EUNSUPPORTED
    assert bb(_lib.RC_F32 | 0x400000, 0) == _lib.RC_EUNSUPPORTED
    assert L.rc_last_error()


def test_backward_entry_points_reject_unknown_flag_bits():
    """bits of ``levels`` above the level count and the
    RC_SHADOW_LEVEL byte, other than RC_GRAD_OVERWRITE on
    rc_corr_lookup_backward_calls, are RC_EINVAL before any launch (they used
    to be dropped silently)."""
    L = _lib.lib()
    f = lambda a: ctypes.c_void_p(a)  # noqa: E731
    w = _lib.int_array([64, 32, 16, 8])
    pair = _lib.ptr_array([f(0x1000), None, f(0x2000), None])
    junk = 4 | 0x100000
    assert L.rc_corr_lookup_backward(pair, w, None, junk, 4, f(0x7000), 0, 1, 2, 64, f(0x8000),
                                     None) == _lib.RC_EINVAL
    assert b"flag" in L.rc_last_error()
    xs = _lib.ptr_array([f(0x7000)])
    gos = _lib.ptr_array([f(0x8000)])
    cbs = _lib.long_array([0])
    calls = lambda lv: L.rc_corr_lookup_backward_calls(  # noqa: E731
        pair, w, None, lv, 4, 1, xs, cbs, 1, 2, 64, gos, None)
    assert calls(junk) == _lib.RC_EINVAL and b"flag" in L.rc_last_error()
    assert calls(junk | _lib.RC_GRAD_OVERWRITE) == _lib.RC_EINVAL
    # the documented flag itself is accepted up to the point of validation
    # (no calls: RC_GRAD_OVERWRITE with n_calls == 0 is its own RC_EINVAL)
    assert L.rc_corr_lookup_backward_calls(pair, w, None, 4 | _lib.RC_GRAD_OVERWRITE, 4, 0, None, None,
                                           1, 2, 64, None, None) == _lib.RC_EINVAL
    assert b"no calls" in L.rc_last_error()


def test_disparity_layout_flag_validation():
    """RC_LAYOUT_DISPARITY (ABI v9): the header's value and RC_SHEAR_ROWS
    agree with the binding; only rc_corr_build and rc_corr_lookup_chain take
    it, and only for the fp32 pair layout on the split build -- every other
    request is refused before any launch (B = 0: nothing is touched)."""
    text = open(_lib.HEADER).read()
    m = re.search(r"#define RC_LAYOUT_DISPARITY\s+(0x[0-9a-fA-F]+)", text)
    assert m and int(m.group(1), 16) == _lib.RC_LAYOUT_DISPARITY
    assert "#define RC_SHEAR_ROWS(W2, W1, l) (((W2) >> (l)) + (((W1) - 1) >> (l)))" in text
    assert _lib.shear_rows(240, 240, 0) == 479 and _lib.shear_rows(240, 240, 2) == 119
    L = _lib.lib()
    f = lambda a: ctypes.c_void_p(a)  # noqa: E731
    D = _lib.RC_F32 | _lib.RC_LAYOUT_DISPARITY
    one = _lib.ptr_array([f(0x1000)])
    w1 = _lib.int_array([64])
    assert L.rc_corr_lookup(one, w1, None, D, 1, 4, f(0x2000), 0, 0, 1, 64, f(0x3000), None) == \
        _lib.RC_EUNSUPPORTED
    assert b"RC_LAYOUT_DISPARITY" in L.rc_last_error()
    assert L.rc_corr_lookup_conv(one, w1, None, D, 1, 4, f(0x2000), 0, 0, 1, 64, f(0x4000), None, 4, 1,
                                 f(0x3000), None) == _lib.RC_EUNSUPPORTED
    assert L.rc_corr_pool(None, 8, None, 4, 0, 8, D, None) == _lib.RC_EUNSUPPORTED
    pair = _lib.ptr_array([f(0x1000), None, f(0x2000), None])
    w4 = _lib.int_array([64, 32, 16, 8])
    assert L.rc_corr_lookup_step(pair, w4, None, D, 4, 4, 1, f(0x2000), None, f(0x3000), f(0x5000),
                                 0, 1, 64, f(0x4000), None) == _lib.RC_EUNSUPPORTED
    chain = lambda ptrs, w, dt, lv, r=4: L.rc_corr_lookup_chain(  # noqa: E731
        ptrs, w, None, dt, lv, r, f(0x2000), 0, 0, 1, 64, f(0x3000), None)
    assert chain(pair, w4, D, 4) == _lib.RC_OK                              # B = 0, accepted
    three = _lib.ptr_array([f(0x1000), f(0x2000), None])
    assert chain(three, _lib.int_array([64, 32, 16]), D, 3) == _lib.RC_EUNSUPPORTED
    assert chain(pair, w4, _lib.RC_BF16 | _lib.RC_LAYOUT_DISPARITY, 4) == _lib.RC_EUNSUPPORTED
    assert chain(pair, w4, D | _lib.RC_OUT_CHANNELS_LAST, 4) == _lib.RC_EUNSUPPORTED
    assert chain(pair, w4, D | _lib.shadow_level(2), 4) == _lib.RC_EUNSUPPORTED
    ld = _lib.long_array([64, 32, 64])
    b3 = _lib.ptr_array([f(0x1000), None, f(0x2000)])
    build = lambda **kw: L.rc_corr_build(  # noqa: E731
        f(0x1000), f(0x2000), kw.get("dt", 0), 0, 8, 1, kw.get("W1", 64), 64, kw.get("pyr", b3),
        kw.get("ld", ld), kw.get("nbuf", 3), kw.get("pdt", D), None)
    assert build() == _lib.RC_OK                                            # B = 0, accepted
    assert build(dt=_lib.RC_BF16) == _lib.RC_EUNSUPPORTED
    assert build(pdt=D | _lib.RC_BUILD_EXACT_F32) == _lib.RC_EUNSUPPORTED
    assert build(nbuf=2, pyr=_lib.ptr_array([f(0x1000), f(0x2000)])) == _lib.RC_EUNSUPPORTED
    assert build(pyr=_lib.ptr_array([f(0x1000), f(0x3000), f(0x2000)])) == _lib.RC_EUNSUPPORTED
    assert build(W1=62) == _lib.RC_EUNSUPPORTED
    assert build(ld=None) == _lib.RC_EINVAL
    assert build(ld=_lib.long_array([60, 32, 64])) == _lib.RC_EINVAL      # < W1
