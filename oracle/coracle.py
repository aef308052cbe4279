"""ctypes wrapper for oracle/corr_oracle.c (TEST INFRASTRUCTURE ONLY).

Numpy in, numpy out.  See corr_oracle.c for the reference lines each function
restates.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libcorr_oracle.so")
_lib = None

_f32p = ctypes.POINTER(ctypes.c_float)


def build():
    """Compile corr_oracle.c into oracle/_build (gcc; no GPU needed)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        lib = ctypes.CDLL(_LIB_PATH)
        lib.oracle_corr_volume.argtypes = [_f32p, _f32p] + [ctypes.c_int] * 5 + [_f32p]
        lib.oracle_corr_pool.argtypes = [_f32p, ctypes.c_long, ctypes.c_int, _f32p]
        lib.oracle_corr_lookup.argtypes = [
            ctypes.POINTER(_f32p), ctypes.POINTER(ctypes.c_int), ctypes.c_int,
            ctypes.c_int, _f32p, ctypes.c_long, ctypes.c_int, ctypes.c_int,
            ctypes.c_int, _f32p]
        lib.oracle_corr_lookup_backward.argtypes = lib.oracle_corr_lookup.argtypes
        lib.oracle_corr_build_backward.argtypes = (
            [_f32p, _f32p] + [ctypes.c_int] * 5 + [ctypes.POINTER(_f32p), ctypes.c_int,
                                                   _f32p, _f32p, _f32p])
        _lib = lib
    return _lib


def _p(a):
    return a.ctypes.data_as(_f32p)


def corr_volume(f1, f2):
    """(B,D,H,W1),(B,D,H,W2) fp32 -> (B,H,W1,1,W2) fp32 (model.py:318-326)."""
    f1 = np.ascontiguousarray(f1, np.float32)
    f2 = np.ascontiguousarray(f2, np.float32)
    B, D, H, W1 = f1.shape
    W2 = f2.shape[3]
    out = np.empty((B, H, W1, 1, W2), np.float32)
    _load().oracle_corr_volume(_p(f1), _p(f2), B, D, H, W1, W2, _p(out))
    return out


def corr_pool(level):
    """(P, W) -> (P, W//2): one avg_pool2d([1,2]) step (model.py:294)."""
    level = np.ascontiguousarray(level, np.float32).reshape(level.shape[0], -1)
    P, W = level.shape
    out = np.empty((P, W // 2), np.float32)
    _load().oracle_corr_pool(_p(level), P, W, _p(out))
    return out


def corr_pyramid(f1, f2, num_levels):
    """num_levels+1 levels, each (P, W_l) (model.py:284-295)."""
    vol = corr_volume(f1, f2)
    B, H, W1, _, W2 = vol.shape
    pyr = [vol.reshape(B * H * W1, W2)]
    for _ in range(num_levels):
        pyr.append(corr_pool(pyr[-1]))
    return pyr


def corr_lookup(pyramid, coords, num_levels, radius):
    """pyramid: list of (P, W_l); coords (B,2,H,W1) -> (B, L(2r+1), H, W1)."""
    coords = np.ascontiguousarray(coords, np.float32)
    B, _, H, W1 = coords.shape
    levels = [np.ascontiguousarray(pyramid[i], np.float32).reshape(B * H * W1, -1)
              for i in range(num_levels)]
    ptrs = (_f32p * num_levels)(*[_p(l) for l in levels])
    widths = (ctypes.c_int * num_levels)(*[l.shape[1] for l in levels])
    out = np.empty((B, num_levels * (2 * radius + 1), H, W1), np.float32)
    _load().oracle_corr_lookup(ptrs, widths, num_levels, radius, _p(coords),
                               2 * H * W1, B, H, W1, _p(out))
    return out


def corr_lookup_backward(widths, coords, grad_out, num_levels, radius, grads=None):
    """Accumulate the lookup's pyramid gradients: returns a list of (P, W_l)
    (``grads`` to keep accumulating over several lookup calls)."""
    coords = np.ascontiguousarray(coords, np.float32)
    grad_out = np.ascontiguousarray(grad_out, np.float32)
    B, _, H, W1 = coords.shape
    P = B * H * W1
    if grads is None:
        grads = [np.zeros((P, widths[i]), np.float32) for i in range(num_levels)]
    ptrs = (_f32p * num_levels)(*[_p(g) for g in grads])
    wid = (ctypes.c_int * num_levels)(*widths[:num_levels])
    _load().oracle_corr_lookup_backward(ptrs, wid, num_levels, radius, _p(coords), 2 * H * W1,
                                        B, H, W1, _p(grad_out))
    return grads


def fold_grads(grads):
    """Total gradient of every pyramid level: each level's own gradient plus
    the pooling backward of the coarser total (model.py:294)."""
    tot = [g.copy() for g in grads]
    for i in range(len(grads) - 2, -1, -1):
        Wc = tot[i + 1].shape[1]
        tot[i][:, :2 * Wc] += np.repeat(tot[i + 1] * np.float32(0.5), 2, axis=1)
    return tot


def corr_build_backward(f1, f2, grads):
    """(d fmap1, d fmap2) from the per-level pyramid gradients (fp64 GEMMs)."""
    f1 = np.ascontiguousarray(f1, np.float32)
    f2 = np.ascontiguousarray(f2, np.float32)
    B, D, H, W1 = f1.shape
    W2 = f2.shape[3]
    grads = [np.ascontiguousarray(g, np.float32) for g in grads]
    scratch = np.empty((B * H * W1, W2), np.float32)
    df1, df2 = np.empty_like(f1), np.empty_like(f2)
    ptrs = (_f32p * len(grads))(*[_p(g) for g in grads])
    _load().oracle_corr_build_backward(_p(f1), _p(f2), B, D, H, W1, W2, ptrs, len(grads),
                                       _p(scratch), _p(df1), _p(df2))
    return df1, df2
