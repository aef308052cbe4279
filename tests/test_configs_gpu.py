"""Parity at the BASELINE configs the earlier suites did not run at size
(VERDICT r2 "What's missing" 1-2, "What's weak" 1):

* config 4, Middlebury (B=1, D=256, 496x720 fmaps, fp32): the product default
  block (level-2 shadow copy only) and the same block with the 1.03 GB level
  0 shadowed too, where the pair kernel's 32-bit window covers 2 GB plus the
  gap;
* config 5, realtime (B=1, D=256, 120x160, 3 levels, r=4,
  ``low_latency=True``): every pixel against the C oracle;
* config 3's product default at per-GPU B=16 (bf16 fmaps, bf16 pyramid; the
  291 MB bf16 level 0 is larger than the Infinity Cache, so it is shadowed).

Reference lines: model.py:284-295 (pyramid), :297-316 (lookup), :318-326
(volume).  Tolerances: fp32 volume max|d|/max|ref| <= 1e-4 and rel-L2 <= 1e-5
(SURVEY §8d); a bf16-stored level vs the fp64 oracle on the bf16-rounded
inputs <= 1e-2 / rel-L2 <= 5e-3; lookups bit-exact given the same pyramid.
"""
import numpy as np
import pytest
import torch

from golden_util import norm_err, rel_l2, same
from oracle import coracle
from raft_stereo_amd import CorrBlock1D
from raft_stereo_amd import corr as rcorr

from test_corr_gpu import special_coords
from test_fullsize_gpu import oracle_row_levels, sampled_rows

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def bench_coords(B, H, W1, W2, g):
    """coords_grid - U[0,64) (the bench's distribution) with every 97th pixel
    moved anywhere in [-12, W2+12) and the special values of special_coords."""
    x = special_coords(B, H, W1, W2, g)[:, :1].contiguous()
    x.view(-1)[::97] = torch.randint(-12, W2 + 12, x.view(-1)[::97].shape, generator=g).float()
    return torch.cat([x, torch.zeros_like(x)], 1)


@pytest.mark.parametrize("shadow", [None, (0, 2)], ids=["default", "l0+l2"])
def test_config4_middlebury_fullsize(shadow):
    """Config 4 through the product default (levels 0 and 2 stored, level 2
    with its shadow copy) and with level 0 shadowed as well (a 2 GB window):
    48 sampled rows of levels 0-1 vs the C oracle, every
    row of levels 1-4 bit-exact against the oracle's pooling of the level
    below, and the pair lookup over all 357,120 pixels bit-exact against the
    per-level kernel on the materialised pyramid and, on 8 image rows, against
    the C oracle's sampler."""
    B, D, H, W = 1, 256, 496, 720
    g = torch.Generator().manual_seed(4044)
    f1 = torch.randn(B, D, H, W, generator=g)
    f2 = torch.randn(B, D, H, W, generator=g)
    coords = bench_coords(B, H, W, W, g)
    with torch.no_grad():
        blk = CorrBlock1D(f1.to(DEV), f2.to(DEV), num_levels=4, radius=4, shadow=shadow)
        assert blk._chain and blk.levels_stored == [0, 2]
        assert blk._shadow == frozenset(shadow or (2,))
        out = blk(coords.to(DEV))
        pyr = blk.corr_pyramid
        ref = rcorr.lookup(pyr, coords.to(DEV), 4, 4)
        torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int32), ref.view(torch.int32)), "pair lookup != per-level lookup"
    lv = [pyr[l].reshape(H, W, -1) for l in range(2)]
    f1n, f2n = f1.numpy(), f2.numpy()
    worst = 0.0
    for b, h in sampled_rows(B, H, 48, 41):
        rl = oracle_row_levels(f1n, f2n, b, h, 2)
        for l in range(2):
            got = lv[l][h].cpu().numpy()
            e = norm_err(got, rl[l])
            worst = max(worst, e)
            assert e <= 1e-4 and rel_l2(got, rl[l]) <= 1e-5, (h, l, e)
    for l in range(1, 5):
        below = pyr[l - 1].reshape(pyr[l - 1].shape[0], -1).cpu().numpy()
        got = pyr[l].reshape(pyr[l].shape[0], -1).cpu().numpy()
        assert same(got, coracle.corr_pool(below)), f"level {l}"
        del below, got
    rows = [0, 1, 137, 248, 300, 411, 494, 495]
    for h in rows:
        sl = slice(h * W, (h + 1) * W)
        lvls = [t.reshape(t.shape[0], -1)[sl].cpu().numpy() for t in pyr[:4]]
        oc = coracle.corr_lookup(lvls, coords[:, :, h:h + 1].numpy(), 4, 4)
        assert same(out[:, :, h:h + 1].cpu().numpy(), oc), f"row {h}"
    print(f"config-4 full-size: worst normalised volume error {worst:.2e} over 48 rows")


@pytest.mark.parametrize("low_latency", [True, False], ids=["low_latency", "default"])
def test_config5_realtime_every_pixel(low_latency):
    """Config 5 (B=1, D=256, 120x160, 3 levels, r=4): the whole pyramid vs the
    C oracle (volume within the fp32 bound, pooled levels bit-exact from our
    level 0), every pixel of the lookup bit-exact against the oracle's
    sampler, and the fused loop step (rc_corr_lookup_step) equal to the plain
    lookup at the updated coordinates."""
    B, D, H, W = 1, 256, 120, 160
    g = torch.Generator().manual_seed(5055)
    f1 = torch.randn(B, D, H, W, generator=g)
    f2 = torch.randn(B, D, H, W, generator=g)
    coords = bench_coords(B, H, W, W, g)
    with torch.no_grad():
        blk = CorrBlock1D(f1.to(DEV), f2.to(DEV), num_levels=3, radius=4, low_latency=low_latency)
        out = blk(coords.to(DEV)).cpu().numpy()
        pyr = [t.reshape(t.shape[0], -1).cpu().numpy() for t in blk.corr_pyramid]
    ref = coracle.corr_pyramid(f1.numpy(), f2.numpy(), 3)
    assert norm_err(pyr[0], ref[0]) <= 1e-4 and rel_l2(pyr[0], ref[0]) <= 1e-5
    for l in range(1, 4):
        assert same(pyr[l], coracle.corr_pool(pyr[l - 1])), f"level {l}"
    assert same(out, coracle.corr_lookup(pyr, coords.numpy(), 3, 4))
    # the fused loop step: coords1 + delta (y ignored), then the lookup there
    d = torch.randn(coords.shape, generator=g) * 3
    c1 = coords.clone().to(DEV)
    with torch.no_grad():
        corr, new, flow = blk.lookup_step(c1, d.to(DEV))
    moved = coords.clone()
    moved[:, 0] += d[:, 0]
    assert same(new.cpu().numpy(), moved.numpy())
    assert same(corr.cpu().numpy(), coracle.corr_lookup(pyr, moved.numpy(), 3, 4))


def test_config3_default_b16_shadowed_level0():
    """Config 3's product default at per-GPU B=16 (global 64 over 4 GPUs):
    bf16 fmaps, bf16 pyramid of levels 0 and 2, both shadowed (the bf16 level 0
    is 291 MB).  Pair lookup over all 467,744 pixels bit-exact against the
    per-level kernel on the materialised pyramid; 16 sampled rows of level 0
    vs the oracle on the bf16-rounded inputs within the bf16 bound."""
    B, D, H, W = 16, 256, 94, 311
    g = torch.Generator().manual_seed(3316)
    f1 = torch.randn(B, D, H, W, generator=g).bfloat16()
    f2 = torch.randn(B, D, H, W, generator=g).bfloat16()
    coords = bench_coords(B, H, W, W, g)
    with torch.no_grad():
        blk = CorrBlock1D(f1.to(DEV), f2.to(DEV), num_levels=4, radius=4)
        assert blk.pyramid_dtype == torch.bfloat16 and blk.levels_stored == [0, 2]
        assert blk._shadow == frozenset({0, 2})
        out = blk(coords.to(DEV))
        ref = rcorr.lookup(blk.corr_pyramid, coords.to(DEV), 4, 4)
        torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int32), ref.view(torch.int32))
    lvl0 = blk.corr_pyramid[0].reshape(B, H, W, W)
    f1n, f2n = f1.float().numpy(), f2.float().numpy()
    for b, h in sampled_rows(B, H, 16, 33):
        rl = oracle_row_levels(f1n, f2n, b, h, 1)[0]
        got = lvl0[b, h].float().cpu().numpy()
        assert norm_err(got, rl) <= 1e-2 and rel_l2(got, rl) <= 5e-3, (b, h)


LEVELPAR_SHAPES = [
    # B, D, H, W1, W2, L, r: 1-2 levels and radii > 4, which the launcher routes
    # to the level-parallel kernel below 64K pixels
    (1, 16, 3, 50, 50, 1, 4),
    (1, 16, 2, 64, 70, 1, 7),
    (2, 16, 3, 40, 45, 2, 5),
    (1, 32, 2, 96, 96, 2, 8),
    (1, 16, 2, 61, 64, 3, 6),
    (1, 16, 2, 90, 90, 4, 8),
]


@pytest.mark.parametrize("shape", LEVELPAR_SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_levelpar_shapes_vs_oracle(shape):
    """low_latency blocks with 1-4 levels and radius 4-8 bit-exact against the
    C oracle's sampler on their own pyramid, incl. NaN/inf/subnormal x."""
    B, D, H, W1, W2, L, r = shape
    g = torch.Generator().manual_seed(7000 + sum(shape))
    f1 = torch.randn(B, D, H, W1, generator=g).to(DEV)
    f2 = torch.randn(B, D, H, W2, generator=g).to(DEV)
    coords = special_coords(B, H, W1, W2, g)
    with torch.no_grad():
        blk = CorrBlock1D(f1, f2, num_levels=L, radius=r, low_latency=True)
        out = blk(coords.to(DEV)).cpu().numpy()
        pyr = [t.reshape(t.shape[0], -1).cpu().numpy() for t in blk.corr_pyramid[:L]]
    assert same(out, coracle.corr_lookup(pyr, coords.numpy(), L, r))
