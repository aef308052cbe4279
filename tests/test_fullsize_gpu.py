"""Parity at BASELINE sizes.

The build's full-size grids (config 2: B=8, 135x240, D=256 -> 8*135*2*2 =
4,320 workgroups through the XCD remap of volume.hip, with 4320 % 8 == 0; the
bf16 config-3 shape 94x311 has partial tiles on both axes) are checked
against the C oracle on sampled (b, h) rows -- the oracle's fp64 volume for
every (b, h) row at this size would take minutes -- and through
size-independent properties over ALL rows: pooled levels equal avg_pool2d of
the kernel's own level below bit for bit, and the chain lookup equals the
per-level lookup bit for bit.

Tolerances: fp32 volume max|d|/max|ref| <= 1e-4 and rel-L2 <= 1e-5; bf16
inputs vs the oracle on bf16-rounded inputs <= 1e-5 (fp32 pyramid); lookup
bit-exact given the same pyramid.
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


def sampled_rows(B, H, n, seed):
    g = np.random.default_rng(seed)
    rows = {(0, 0), (B - 1, H - 1), (0, H - 1), (B - 1, 0)}
    while len(rows) < n:
        rows.add((int(g.integers(B)), int(g.integers(H))))
    return sorted(rows)


def oracle_row_levels(f1, f2, b, h, nlev):
    """Oracle levels 0..nlev-1 of image row (b, h): (W1, W2 >> l) each."""
    vol = coracle.corr_volume(np.ascontiguousarray(f1[b:b + 1, :, h:h + 1]),
                              np.ascontiguousarray(f2[b:b + 1, :, h:h + 1]))
    lv = [vol.reshape(f1.shape[3], -1)]
    for _ in range(1, nlev):
        lv.append(coracle.corr_pool(lv[-1]))
    return lv


def np_level(t):
    return t.reshape(t.shape[0], -1).cpu().numpy()


@pytest.mark.parametrize("lazy", [True, False], ids=["lazy", "eager"])
def test_config2_build_fullsize_vs_oracle(lazy):
    """Config 2 (B=8, D=256, 135x240): 4,320 workgroups.  64 sampled rows of
    levels 0-1 vs the C oracle; every row of every level bit-exact against
    avg_pool2d of the level below (model.py:318-326, :284-295)."""
    B, D, H, W = 8, 256, 135, 240
    g = torch.Generator().manual_seed(2024)
    f1 = torch.randn(B, D, H, W, generator=g)
    f2 = torch.randn(B, D, H, W, generator=g)
    with torch.no_grad():
        blk = CorrBlock1D(f1.to(DEV), f2.to(DEV), num_levels=4, radius=4, lazy_levels=lazy)
        pyr = blk.corr_pyramid
        torch.cuda.synchronize()
    for l in range(1, 5):
        # the oracle's avg_pool2d step (model.py:294) of OUR level below, all rows
        assert same(np_level(pyr[l]), coracle.corr_pool(np_level(pyr[l - 1]))), f"level {l}"
    lv = [pyr[l].reshape(B, H, W, -1) for l in range(2)]
    f1n, f2n = f1.numpy(), f2.numpy()
    worst = 0.0
    for b, h in sampled_rows(B, H, 64, 7):
        ref = oracle_row_levels(f1n, f2n, b, h, 2)
        for l in range(2):
            got = lv[l][b, h].cpu().numpy()
            e = norm_err(got, ref[l])
            worst = max(worst, e)
            assert e <= 1e-4 and rel_l2(got, ref[l]) <= 1e-5, (b, h, l, e)
    print(f"config-2 full-size build: worst normalised error {worst:.2e} over 64 rows")


def test_config2_chain_lookup_fullsize_bitexact():
    """Config 2's whole P = 259,200 pixels: the chain lookup (product default)
    equals the per-level lookup over the materialised pyramid bit for bit,
    and a sample of pixels equals the C oracle's sampler bit for bit."""
    B, D, H, W = 8, 256, 135, 240
    g = torch.Generator().manual_seed(77)
    f1 = torch.randn(B, D, H, W, generator=g).to(DEV)
    f2 = torch.randn(B, D, H, W, generator=g).to(DEV)
    x = torch.arange(W).float().view(1, 1, 1, W) - torch.rand(B, 1, H, W, generator=g) * 64
    x.view(-1)[::997] = torch.randint(-12, W + 12, x.view(-1)[::997].shape, generator=g).float()
    coords = torch.cat([x, torch.zeros_like(x)], 1).to(DEV)
    with torch.no_grad():
        blk = CorrBlock1D(f1, f2, num_levels=4, radius=4)
        assert blk._chain
        out = blk(coords)
        ref = rcorr.lookup(blk.corr_pyramid, coords, 4, 4)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    rows = slice(0, 240 * 64)                      # the first 64 image rows of batch 0
    pyr = [t.reshape(t.shape[0], -1)[rows].cpu().numpy() for t in blk.corr_pyramid[:4]]
    oc = coracle.corr_lookup(pyr, coords[:1, :, :64].cpu().numpy(), 4, 4)
    assert same(out[:1, :, :64].cpu().numpy(), oc)


def test_config3_bf16_build_fullsize_vs_oracle():
    """Config 3 per-GPU shape at 8 GPUs (B=8, 94x311, bf16 fmaps, bf16 MFMA):
    level 0 of sampled rows vs the oracle on the bf16-rounded inputs
    (fp32 pyramid: <= 1e-5 normalised) -- partial tiles on both axes."""
    B, D, H, W = 8, 256, 94, 311
    g = torch.Generator().manual_seed(3)
    f1 = torch.randn(B, D, H, W, generator=g).bfloat16()
    f2 = torch.randn(B, D, H, W, generator=g).bfloat16()
    with torch.no_grad():
        blk = CorrBlock1D(f1.to(DEV), f2.to(DEV), num_levels=4, radius=4,
                          pyramid_dtype=torch.float32)
        lvl0 = blk.corr_pyramid[0].reshape(B, H, W, W)
    f1n, f2n = f1.float().numpy(), f2.float().numpy()
    for b, h in sampled_rows(B, H, 24, 9):
        ref = oracle_row_levels(f1n, f2n, b, h, 1)[0]
        got = lvl0[b, h].cpu().numpy()
        assert norm_err(got, ref) <= 1e-5, (b, h)


def test_validation_errors_are_python_errors():
    """Host-side validation: CPU weight / bias / delta / out and a
    short bias raise before any launch; convex_upsample refuses gradients."""
    from raft_stereo_amd.upsample import convex_upsample
    g = torch.Generator().manual_seed(1)
    f = torch.randn(1, 16, 2, 40, generator=g).to(DEV)
    blk = CorrBlock1D(f, f, num_levels=4, radius=4)
    c = torch.zeros(1, 2, 2, 40, device=DEV)
    w = torch.randn(64, 36, 1, 1, device=DEV)
    with torch.no_grad():
        with pytest.raises(RuntimeError):
            blk.lookup_convc1(c, w.cpu())
        with pytest.raises(RuntimeError):
            blk.lookup_convc1(c, w, torch.zeros(63, device=DEV))
        with pytest.raises(RuntimeError):
            blk.lookup_convc1(c, w, torch.zeros(64))
        with pytest.raises(RuntimeError):
            blk.lookup_step(c, torch.zeros(1, 2, 2, 40))
        with pytest.raises(RuntimeError):
            blk.lookup_step(c, None, out=torch.zeros(1, 2, 2, 40))
    flow = torch.randn(1, 1, 4, 4, device=DEV, requires_grad=True)
    mask = torch.randn(1, 9 * 16, 4, 4, device=DEV)
    with pytest.raises(RuntimeError):
        convex_upsample(flow, mask, 4)
    with torch.no_grad():
        assert convex_upsample(flow, mask, 4).shape == (1, 1, 16, 16)
