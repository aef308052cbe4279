"""Helpers to read tests/golden/*.npz (fixtures made by make_golden.py)."""
import glob
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as fh:
        return json.load(fh)


def files(kind):
    return sorted(glob.glob(os.path.join(GOLDEN, f"{kind}_*.npz")))


def load(path):
    z = np.load(path)  # allow_pickle=False (default)
    return {k: z[k] for k in z.files}


def same(a, b):
    """Bitwise-equal values (NaN == NaN, -0 == +0)."""
    return np.array_equal(a, b, equal_nan=True)


def norm_err(a, ref):
    """max|a-ref| / max|ref| -- the SURVEY §8d tolerance metric."""
    a = np.asarray(a, np.float64)
    ref = np.asarray(ref, np.float64)
    return float(np.abs(a - ref).max() / max(np.abs(ref).max(), 1e-30))


def rel_l2(a, ref):
    a = np.asarray(a, np.float64)
    ref = np.asarray(ref, np.float64)
    return float(np.linalg.norm(a - ref) / max(np.linalg.norm(ref), 1e-30))


def stereo_pair(B, H, W, seed, shift=6):
    """Synthetic stereo pair (CPU torch generator, so the same bits on every
    x86 host): right = left shifted by ``shift`` px plus noise.  Used by
    make_golden.py and by the tests that regenerate a golden's images."""
    import torch
    g = torch.Generator().manual_seed(seed)
    left = torch.rand(B, 3, H, W + shift, generator=g) * 255.0
    right = left[..., :W].clone()
    left = left[..., shift:].contiguous()
    right = (right + torch.randn(B, 3, H, W, generator=g) * 2.0).clamp(0, 255)
    return left, right


def image_digest(*imgs):
    import hashlib
    h = hashlib.sha256()
    for t in imgs:
        h.update(t.contiguous().numpy().tobytes())
    return h.hexdigest()
