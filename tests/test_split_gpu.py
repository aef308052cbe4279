"""The split-bf16 fp32 volume (csrc/volume_split.hip, the fp32 default since
ABI v6) against the C oracle's fp64 volume and against the exact fp32 MFMA
kernel (RC_BUILD_EXACT_F32) -- model.py:318-326 (volume) and :284-295
(pyramid).

Bar (SURVEY §8d fp32 contract): max|d|/max|ref| <= 1e-4 and rel-L2 <= 1e-5
per tensor.  The split kernel is also held to the exact kernel's own error:
its error against fp64 must not exceed twice the fp32 MFMA kernel's (or
1e-6), i.e. it is an fp32-accurate volume, not a reduced-precision one.
Pooled levels are bit-exact from the level below (avg_pool2d's fp32 ops).
"""
import numpy as np
import pytest
import torch

from golden_util import norm_err, rel_l2, same
from oracle import coracle
from raft_stereo_amd import CorrBlock1D
from raft_stereo_amd import corr as rcorr

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

SHAPES = [
    # B, D, H, W1, W2
    (2, 256, 3, 240, 240),      # config 2 rows: fragment tails at 240
    (1, 256, 2, 160, 160),      # config 5 rows
    (1, 256, 2, 720, 720),      # config 4 rows
    (1, 256, 2, 311, 311),      # odd width, not a multiple of 4
    (2, 40, 3, 37, 45),         # D % 32 != 0, W1 != W2
    (1, 8, 2, 16, 130),
    (1, 33, 1, 129, 17),
    (3, 64, 5, 64, 64),
    (1, 96, 3, 224, 224),       # tiles of 7 fragments: wave blocks of 4 + 3 inside the row
    (1, 64, 2, 96, 176),        # 6 / 11 fragments: tiles of 6 and of 6 + 5
    (1, 64, 2, 144, 400),       # 9 / 25 fragments: the 8-wave kernel's tiles of 9 and of 13 + 12
]


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_split_volume_vs_oracle_and_exact(shape):
    B, D, H, W1, W2 = shape
    g = torch.Generator().manual_seed(31 * B + D + H + W1 + W2)
    f1 = torch.randn(B, D, H, W1, generator=g)
    f2 = torch.randn(B, D, H, W2, generator=g)
    ref = coracle.corr_volume(f1.numpy(), f2.numpy())
    with torch.no_grad():
        sp = CorrBlock1D.corr(f1.to(DEV), f2.to(DEV)).cpu().numpy()
        ex = CorrBlock1D.corr(f1.to(DEV), f2.to(DEV), exact_f32=True).cpu().numpy()
    e_sp, e_ex = norm_err(sp, ref), norm_err(ex, ref)
    l_sp, l_ex = rel_l2(sp, ref), rel_l2(ex, ref)
    print(f"{shape}: split {e_sp:.2e}/{l_sp:.2e}  exact-f32 {e_ex:.2e}/{l_ex:.2e}")
    assert e_sp <= 1e-4 and l_sp <= 1e-5
    assert e_ex <= 1e-4 and l_ex <= 1e-5
    assert e_sp <= max(2 * e_ex, 1e-6) and l_sp <= max(2 * l_ex, 1e-6)


@pytest.mark.parametrize("levels,W", [(2, 240), (3, 240), (4, 240), (7, 240), (4, 160), (4, 224),
                                      (5, 208)], ids=lambda v: str(v))
def test_split_pyramid_levels_pool_bitexact(levels, W):
    """Every stored level (eager build: all num_levels+1, incl. levels past the
    5 the epilogue fuses) equals avg_pool2d of the level below bit for bit,
    and level 0 is within the fp32 bound -- incl. widths whose balanced tiles
    have fewer than 8 fragments (160: 5 + 5, 224: 7 + 7, 208: 7 + 6)."""
    B, D, H = 2, 64, 3
    g = torch.Generator().manual_seed(400 + levels)
    f1 = torch.randn(B, D, H, W, generator=g)
    f2 = torch.randn(B, D, H, W, generator=g)
    with torch.no_grad():
        blk = CorrBlock1D(f1.to(DEV), f2.to(DEV), num_levels=levels, radius=2, lazy_levels=False)
        pyr = [t.reshape(t.shape[0], -1).cpu().numpy() for t in blk.corr_pyramid]
    ref0 = coracle.corr_volume(f1.numpy(), f2.numpy()).reshape(B * H * W, W)
    assert norm_err(pyr[0], ref0) <= 1e-4 and rel_l2(pyr[0], ref0) <= 1e-5
    for l in range(1, levels + 1):
        assert same(pyr[l], coracle.corr_pool(pyr[l - 1])), f"level {l}"


def test_split_pair_layout_with_shadows_and_lookup():
    """The product default (levels 0 + 2 stored, level-2 shadow) through the
    split kernel: the pair lookup equals the per-level lookup on the
    materialised pyramid bit for bit, and the oracle's sampler."""
    B, D, H, W = 2, 256, 4, 240
    g = torch.Generator().manual_seed(77)
    f1 = torch.randn(B, D, H, W, generator=g).to(DEV)
    f2 = torch.randn(B, D, H, W, generator=g).to(DEV)
    x = torch.arange(W).float().view(1, 1, 1, W) - torch.rand(B, 1, H, W, generator=g) * 64
    coords = torch.cat([x, torch.zeros_like(x)], 1).to(DEV)
    with torch.no_grad():
        blk = CorrBlock1D(f1, f2)
        assert blk.levels_stored == [0, 2] and 2 in blk._shadow
        out = blk(coords)
        ref = rcorr.lookup(blk.corr_pyramid, coords, 4, 4)
        pyr = [t.reshape(t.shape[0], -1).cpu().numpy() for t in blk.corr_pyramid[:4]]
    assert torch.equal(out, ref)
    assert same(out.cpu().numpy(), coracle.corr_lookup(pyr, coords.cpu().numpy(), 4, 4))


def test_split_special_values():
    """Zeros, subnormals, large and tiny magnitudes stay within the fp32 bound
    (the three pieces are exact for every finite fp32 below 3.39e38)."""
    B, D, H, W = 1, 64, 2, 96
    g = torch.Generator().manual_seed(5)
    f1 = torch.randn(B, D, H, W, generator=g) * torch.logspace(-20, 20, W).view(1, 1, 1, W)
    f2 = torch.randn(B, D, H, W, generator=g)
    f1[0, :, 0, :8] = 0.0
    f2[0, :3, 1, :] = 1e-40
    ref = coracle.corr_volume(f1.numpy(), f2.numpy())
    with torch.no_grad():
        sp = CorrBlock1D.corr(f1.to(DEV), f2.to(DEV)).cpu().numpy()
    # per w1 row (magnitudes differ by 40 decades across rows)
    for w1 in range(W):
        r, s = ref[:, :, w1], sp[:, :, w1]
        if np.abs(r).max() > 0:
            assert norm_err(s, r) <= 1e-5, w1


def test_split_nonfinite_fmaps_pinned():
    """Non-finite fmap entries (model.py:324-326 on +-inf / NaN inputs).

    The exact fp32 kernel (exact_f32=True / RC_BUILD_EXACT_F32) reproduces
    the reference's pattern: +-inf where an inf meets finite values, NaN where
    a NaN is involved or infinities of both signs meet.  The split-bf16 default
    is PINNED to a documented difference: an
    inf operand splits into pieces (inf, NaN, NaN), so every entry the
    reference makes +-inf comes out NaN.  Everything the reference keeps
    finite stays finite and within the fp32 bound, and the non-finite SET is
    the reference's in both kernels.  (A guard that zeroes the tail pieces of a
    non-finite head cannot fix it: the head then meets zero tail pieces of the
    other operand in the h*m' and h*l' products, and inf * 0 is NaN on the
    MFMA as anywhere.)"""
    B, D, H, W = 1, 64, 3, 96
    g = torch.Generator().manual_seed(11)
    f1 = torch.randn(B, D, H, W, generator=g)
    f2 = torch.randn(B, D, H, W, generator=g)
    f1[0, 5, 0, 7] = float("inf")
    f1[0, 9, 1, 20] = float("-inf")
    f1[0, 2, 2, 33] = float("nan")
    f2[0, 17, 0, 50] = float("inf")
    f2[0, 17, 1, 60] = float("-inf")
    f1[0, 30, 1, 20] = float("inf")          # row w1=20 of h=1 meets +inf and -inf: NaN
    ref = coracle.corr_volume(f1.numpy(), f2.numpy())
    with torch.no_grad():
        sp = CorrBlock1D.corr(f1.to(DEV), f2.to(DEV)).cpu().numpy()
        ex = CorrBlock1D.corr(f1.to(DEV), f2.to(DEV), exact_f32=True).cpu().numpy()
    fin = np.isfinite(ref)
    assert (~fin).sum() > 0 and np.isnan(ref).sum() > 0 and np.isinf(ref).sum() > 0
    for got in (ex, sp):
        assert np.array_equal(np.isfinite(got), fin)
        assert norm_err(got[fin], ref[fin]) <= 1e-4
    # exact kernel: the reference's infinities (sign included) and NaNs
    assert np.array_equal(np.isnan(ex), np.isnan(ref))
    assert np.array_equal(ex[np.isinf(ref)], ref[np.isinf(ref)])
    # split default: NaN wherever the reference is non-finite (the pinned difference)
    assert np.isnan(sp[~fin]).all()
    # CorrBlock1D(check_finite=True): the non-finite fmaps are
    # detected, a RuntimeWarning names the switch, and the block is the exact
    # kernel's bit for bit (levels and lookups); finite fmaps keep the split
    # default (bit for bit the default block)
    c = torch.zeros(B, 2, H, W)
    c[:, 0] = torch.arange(W, dtype=torch.float32) - 3.25
    with torch.no_grad():
        with pytest.warns(RuntimeWarning, match="non-finite"):
            chk = CorrBlock1D(f1.to(DEV), f2.to(DEV), num_levels=2, check_finite=True,
                              layout="disparity")
        exb = CorrBlock1D(f1.to(DEV), f2.to(DEV), num_levels=2, exact_f32=True)
        assert chk.layout == "rows"
        for u, v in zip(chk.corr_pyramid, exb.corr_pyramid):
            assert torch.equal(u.view(torch.int32), v.view(torch.int32))
        assert torch.equal(chk(c.to(DEV)).view(torch.int32), exb(c.to(DEV)).view(torch.int32))
        g1, g2 = torch.randn(B, D, H, W, generator=g), torch.randn(B, D, H, W, generator=g)
        import warnings
        with warnings.catch_warnings():
            warnings.simplefilter("error")
            fine = CorrBlock1D(g1.to(DEV), g2.to(DEV), num_levels=2, check_finite=True)
        dflt = CorrBlock1D(g1.to(DEV), g2.to(DEV), num_levels=2)
        for u, v in zip(fine.corr_pyramid, dflt.corr_pyramid):
            assert torch.equal(u.view(torch.int32), v.view(torch.int32))
