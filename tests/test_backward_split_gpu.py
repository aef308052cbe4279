"""Volume backward on split-bf16 MFMA (ABI v8): the two
GEMMs of rc_corr_build_backward with every fp32 operand split exactly into
three bf16 pieces, six bf16 products per fp32 product.

Reference: model.py:324 (einsum) and :326 (/sqrt(D)) differentiated, with
avg_pool2d's backward (:294) folded into the level-0 gradient.  Parity: the
fp64-GEMM C oracle (coracle.corr_build_backward) within the fp32 contract
(max|d|/max|ref| <= 1e-4, rel-L2 <= 1e-5), and no worse than twice the exact
fp32 MFMA kernel's own error against the same oracle (RC_BUILD_EXACT_F32)."""
import numpy as np
import pytest
import torch

from golden_util import norm_err, rel_l2
from oracle import coracle
from raft_stereo_amd import CorrBlock1D
from raft_stereo_amd import corr as rcorr

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

SHAPES = [
    # B, D, H, W1, W2, layout (pair4 | pair2 | level2)
    (2, 256, 3, 240, 240, "pair4"),      # config-2 widths and depth
    (1, 256, 2, 720, 720, "pair4"),      # config-4 width (6 tiles per GEMM row)
    (1, 64, 2, 160, 160, "pair2"),       # realtime width, 2 levels -> 1 gradient level
    (2, 100, 2, 96, 132, "level2"),      # D not a multiple of 32, W1 != W2
    (1, 8, 3, 36, 40, "pair4"),          # tiny: one partial 32-k step
]


def level_grads(P, widths, layout, g):
    """Random level gradients in the layout's buffers, and the same values as
    the per-level list the oracle folds."""
    dev = torch.device(DEV)
    if layout == "level2":
        bufs = rcorr.grad_buffers(P, widths[:2], dev)
        per_level = []
        for t in bufs:
            v = torch.randn(t.shape, generator=g)
            t.copy_(v)
            per_level.append(v.numpy())
        return bufs, per_level
    L = 4 if layout == "pair4" else 2
    bufs = rcorr.grad_buffers(P, widths[:L], dev, pair=True)
    per_level = []
    for lvl in range(L):
        if bufs[lvl] is None:                 # folded level: zero in the oracle's list
            per_level.append(np.zeros((P, widths[lvl]), np.float32))
            continue
        v = torch.randn(bufs[lvl].shape, generator=g)
        bufs[lvl].copy_(v)
        per_level.append(v.numpy())
    return bufs, per_level


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_split_volume_backward_vs_oracle_and_exact(shape):
    B, D, H, W1, W2, layout = shape
    g = torch.Generator().manual_seed(B * D + H * W1 + W2)
    f1 = torch.randn(B, D, H, W1, generator=g)
    f2 = torch.randn(B, D, H, W2, generator=g)
    widths = [W2 >> i for i in range(4)]
    P = B * H * W1
    bufs, per_level = level_grads(P, widths, layout, g)
    r1, r2 = coracle.corr_build_backward(f1.numpy(), f2.numpy(), per_level)
    s1, s2 = rcorr.build_backward(f1.to(DEV), f2.to(DEV), bufs)
    e1, e2 = rcorr.build_backward(f1.to(DEV), f2.to(DEV), bufs, exact_f32=True)
    for got, ex, ref in ((s1, e1, r1), (s2, e2, r2)):
        got, ex = got.cpu().numpy(), ex.cpu().numpy()
        es, ee = norm_err(got, ref), norm_err(ex, ref)
        ls, le = rel_l2(got, ref), rel_l2(ex, ref)
        assert es <= 1e-4 and ls <= 1e-5, (es, ls)
        assert es <= 2 * ee + 1e-7 and ls <= 2 * le + 1e-8, (es, ee, ls, le)
        assert not np.array_equal(got, ex) or D <= 8   # the split path really ran


def test_split_volume_backward_through_autograd_exact_flag():
    """CorrBlock1D(exact_f32=True) takes the exact fp32 kernels forward AND
    backward; the default block's fmap gradients agree with it to the fp32
    contract."""
    g = torch.Generator().manual_seed(3)
    B, D, H, W1, W2, L, r = 1, 64, 2, 64, 64, 4, 4
    f1 = torch.randn(B, D, H, W1, generator=g)
    f2 = torch.randn(B, D, H, W2, generator=g)
    x = torch.arange(W1).float().view(1, 1, 1, W1) - torch.rand(B, 1, H, W1, generator=g) * 30
    c = torch.cat([x, torch.zeros_like(x)], 1).to(DEV)
    go = torch.randn(B, L * (2 * r + 1), H, W1, generator=g).to(DEV)
    grads = {}
    for exact in (False, True):
        a = f1.to(DEV).requires_grad_(True)
        b = f2.to(DEV).requires_grad_(True)
        (CorrBlock1D(a, b, num_levels=L, radius=r, exact_f32=exact)(c) * go).sum().backward()
        grads[exact] = (a.grad.cpu().numpy(), b.grad.cpu().numpy())
    for x_, y_ in zip(grads[False], grads[True]):
        assert norm_err(x_, y_) <= 1e-5 and rel_l2(x_, y_) <= 1e-6
        assert not np.array_equal(x_, y_)


def test_split_volume_backward_dev_variant2_equals_product():
    """Dev A/B variant RAFTCORR_VBWD_VARIANT=2 (G^T staged by the non-k-major
    mapping, buffer loads) computes the product's dF1 / dF2 bit for bit
    (its buffer-load staging used the k-major mapping)."""
    import os
    from raft_stereo_amd import _lib
    B, D, H, W1, W2 = 2, 256, 2, 240, 240
    g = torch.Generator().manual_seed(21)
    f1 = torch.randn(B, D, H, W1, generator=g).to(DEV)
    f2 = torch.randn(B, D, H, W2, generator=g).to(DEV)
    bufs, _ = level_grads(B * H * W1, [W2 >> i for i in range(4)], "pair4", g)
    ref = rcorr.build_backward(f1, f2, bufs)
    with _lib.dev_library():
        try:
            os.environ["RAFTCORR_VBWD_VARIANT"] = "2"
            got = rcorr.build_backward(f1, f2, bufs)
        finally:
            os.environ["RAFTCORR_VBWD_VARIANT"] = "0"
    for x_, y_ in zip(got, ref):
        assert torch.equal(x_, y_)
