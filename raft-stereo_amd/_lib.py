"""ctypes binding of libraftcorr.so (include/raftcorr.h).

The library is built in-tree by ``__graft_entry__.build()`` (or ``make -C
raft-stereo_amd/csrc``) into ``raft-stereo_amd/_build/``.  Loading fails
loudly when it is missing -- the product path has no CPU fallback.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_build", "libraftcorr.so")
# Same sources built with -DRAFTCORR_DEV: A/B knobs + ablation kernels
# (tools/ablate.py and the variant bit-identity tests only; never the product).
DEV_LIB_PATH = os.path.join(_HERE, "_build", "libraftcorr_dev.so")
HEADER = os.path.join(os.path.dirname(_HERE), "include", "raftcorr.h")

RC_F32, RC_BF16 = 0, 1
RC_OK, RC_EINVAL, RC_EUNSUPPORTED, RC_EHIP = 0, 1, 2, 3
RC_MAX_LEVELS = 8
ABI_VERSION = 10
RC_SHADOW = 0xFF00  # pyr_dtype flags: every stored level carries a line-phase shadow copy
RC_OUT_CHANNELS_LAST = 0x10000   # pyr_dtype flag: NHWC lookup output (pair kernel)
RC_BUILD_EXACT_F32 = 0x20000     # rc_corr_build flag: exact fp32 MFMA kernel instead of the split-bf16 one
RC_GRAD_OVERWRITE = 0x40000      # rc_corr_lookup_backward_calls flag: write the sum, do not add
RC_LAYOUT_DISPARITY = 0x80000    # rc_corr_build / rc_corr_lookup_chain: disparity-major levels 0, 2 (ABI v9)
RC_LAYOUT_RECORDS = 0x100000     # rc_corr_build / _lookup_chain / _lookup_step: bf16 levels 0, 2 as records (ABI v10)
RC_REC_SLOTS, RC_REC_BYTES = 64, 128


def rec_count(W2):
    """RC_REC_COUNT: 128-B records per pixel row of the record layout."""
    return (((W2 >> 1) + 15) >> 3) + 1


def shear_rows(W2, W1, l):
    """RC_SHEAR_ROWS: rows (diagonals) per image row of disparity-major level l."""
    return (W2 >> l) + ((W1 - 1) >> l)


def shadow_level(l):
    """RC_SHADOW_LEVEL(l): pyr_dtype flag for a shadow copy of level l only."""
    return 0x100 << l


def shadow_offset(rows, ld, esize):
    """RC_SHADOW_OFFSET: bytes from a stored level's base to its shadow copy."""
    return -(-(rows * ld * esize) // 128) * 128 + 64

# name -> (restype, argtypes); must match include/raftcorr.h exactly.
_vp, _i, _l = ctypes.c_void_p, ctypes.c_int, ctypes.c_long
SIGNATURES = {
    "rc_abi_version": (_i, []),
    "rc_last_error": (ctypes.c_char_p, []),
    "rc_corr_build": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _i,
                           ctypes.POINTER(_vp), ctypes.POINTER(_l), _i, _i, _vp]),
    "rc_corr_pool": (_i, [_vp, _l, _vp, _l, _l, _i, _i, _vp]),
    "rc_corr_lookup": (_i, [ctypes.POINTER(_vp), ctypes.POINTER(_i), ctypes.POINTER(_l), _i, _i,
                            _i, _vp, _l, _i, _i, _i, _vp, _vp]),
    "rc_corr_lookup_conv": (_i, [ctypes.POINTER(_vp), ctypes.POINTER(_i), ctypes.POINTER(_l), _i,
                                 _i, _i, _vp, _l, _i, _i, _i, _vp, _vp, _i, _i, _vp, _vp]),
    "rc_corr_lookup_chain": (_i, [ctypes.POINTER(_vp), ctypes.POINTER(_i), ctypes.POINTER(_l), _i,
                                  _i, _i, _vp, _l, _i, _i, _i, _vp, _vp]),
    "rc_corr_lookup_step": (_i, [ctypes.POINTER(_vp), ctypes.POINTER(_i), ctypes.POINTER(_l), _i,
                                 _i, _i, _i, _vp, _vp, _vp, _vp, _i, _i, _i, _vp, _vp]),
    "rc_corr_lookup_backward": (_i, [ctypes.POINTER(_vp), ctypes.POINTER(_i), ctypes.POINTER(_l),
                                     _i, _i, _vp, _l, _i, _i, _i, _vp, _vp]),
    "rc_corr_lookup_backward_calls": (_i, [ctypes.POINTER(_vp), ctypes.POINTER(_i), ctypes.POINTER(_l),
                                           _i, _i, _i, ctypes.POINTER(_vp), ctypes.POINTER(_l), _i, _i,
                                           _i, ctypes.POINTER(_vp), _vp]),
    "rc_convex_upsample": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _vp, _vp]),
    "rc_corr_build_backward": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _i, ctypes.POINTER(_vp),
                                    ctypes.POINTER(_l), _i, _vp, _vp, _vp]),
}

_lib = None
_dev = None
_active = None      # set while dev_library() is active


class CorrLibError(RuntimeError):
    pass


def _open(path):
    if not os.path.exists(path):
        raise CorrLibError(
            f"raft_stereo_amd: HIP library missing at {path}; build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'`")
    dll = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(dll, name)
        fn.restype = res
        fn.argtypes = args
    if dll.rc_abi_version() != ABI_VERSION:
        raise CorrLibError(f"raft_stereo_amd: ABI version mismatch in {path}")
    return dll


def lib():
    """Load (once) and return the CDLL; raise if the HIP library is absent."""
    global _lib
    if _active is not None:
        return _active
    if _lib is None:
        _lib = _open(LIB_PATH)
    return _lib


class _DevLibrary:
    """``with _lib.dev_library():`` routes every call to libraftcorr_dev.so
    (the knob-enabled A/B build) for the duration of the block."""

    def __enter__(self):
        global _dev, _active
        if _dev is None:
            _dev = _open(DEV_LIB_PATH)
        self._prev, _active = _active, _dev
        return _dev

    def __exit__(self, *exc):
        global _active
        _active = self._prev
        return False


dev_library = _DevLibrary


def check(rc, what):
    if rc != RC_OK:
        msg = lib().rc_last_error().decode(errors="replace")
        if rc == RC_EINVAL:
            raise ValueError(f"{what}: {msg}")
        raise CorrLibError(f"{what} failed (rc={rc}): {msg}")


def ptr_array(ptrs):
    return (ctypes.c_void_p * len(ptrs))(*ptrs)


def int_array(vals):
    return (ctypes.c_int * len(vals))(*vals)


def long_array(vals):
    return (ctypes.c_long * len(vals))(*vals)
