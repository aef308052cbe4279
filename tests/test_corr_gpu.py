"""Parity of the HIP path (through the C-ABI, via the drop-in CorrBlock1D)
against the reference goldens and the C oracle.

Tolerances (written here as the contract):
  * fp32 volume: max|d|/max|ref| <= 1e-4 and rel-L2 <= 1e-5;
  * pooling: bit-exact given the same level-0 values;
  * lookup: bit-exact given the same pyramid (NaN == NaN);
  * bf16 pyramid vs the fp32 oracle: max|d|/max|ref| <= 1e-2, rel-L2 <= 5e-3.
"""
import os
import numpy as np
import pytest
import torch

from golden_util import files, load, norm_err, rel_l2, same
from oracle import coracle
from raft_stereo_amd import CorrBlock1D
from raft_stereo_amd import _lib
from raft_stereo_amd import corr as rcorr

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
VOL_TOL, VOL_L2 = 1e-4, 1e-5


def cu(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def pyr_np(blk):
    return [t.reshape(t.shape[0], -1).float().cpu().numpy() for t in blk.corr_pyramid]


@pytest.mark.parametrize("path", files("volume") + files("lookup"), ids=lambda p: p.split("/")[-1])
def test_build_vs_golden(path):
    z = load(path)
    L = int(z["num_levels"])
    with torch.no_grad():
        blk = CorrBlock1D(cu(z["fmap1"]), cu(z["fmap2"]), num_levels=L, radius=4)
    got = pyr_np(blk)
    assert len(got) == L + 1
    assert norm_err(got[0], z["level0"]) <= VOL_TOL
    assert rel_l2(got[0], z["level0"]) <= VOL_L2
    for i in range(L):
        # fused epilogue pooling == avg_pool2d of OUR level i, bit for bit
        assert same(got[i + 1], coracle.corr_pool(got[i])), f"level {i + 1}"
        if f"level{i + 1}" in z:
            assert norm_err(got[i + 1], z[f"level{i + 1}"]) <= VOL_TOL


@pytest.mark.parametrize("path", files("lookup"), ids=lambda p: p.split("/")[-1])
def test_lookup_vs_golden_bitexact(path):
    """Feed the reference's own pyramid; the HIP lookup must match bit for bit."""
    z = load(path)
    L, r = int(z["num_levels"]), int(z["radius"])
    pyr = [cu(z[f"level{i}"]).view(z[f"level{i}"].shape[0], 1, 1, -1) for i in range(L)]
    out = rcorr.lookup(pyr, cu(z["coords"]), L, r).cpu().numpy()
    assert out.shape == z["out"].shape
    bad = ~((out == z["out"]) | (np.isnan(out) & np.isnan(z["out"])))
    assert not bad.any(), f"{bad.sum()} mismatches"


@pytest.mark.parametrize("path", files("lookup"), ids=lambda p: p.split("/")[-1])
def test_end_to_end_vs_golden(path):
    """Build + lookup from the fmaps (volume within tolerance -> lookup too)."""
    z = load(path)
    L, r = int(z["num_levels"]), int(z["radius"])
    with torch.no_grad():
        blk = CorrBlock1D(cu(z["fmap1"]), cu(z["fmap2"]), num_levels=L, radius=r)
        out = blk(cu(z["coords"])).cpu().numpy()
    fin = np.isfinite(z["out"])
    assert np.array_equal(np.isnan(out), np.isnan(z["out"]))
    assert norm_err(out[fin], z["out"][fin]) <= VOL_TOL
    # and bit-exact against the oracle lookup of OUR pyramid
    ref = coracle.corr_lookup(pyr_np(blk)[:L], z["coords"], L, r)
    assert same(out, ref)


SHAPES = [
    # B, D, H, W1, W2, L, r
    (1, 256, 3, 64, 64, 4, 4),
    (2, 256, 2, 240, 240, 4, 4),    # config-2 row width
    (1, 256, 2, 311, 311, 4, 4),    # config-3 width (W % 4 != 0)
    (1, 128, 2, 720, 720, 4, 4),    # config-4 width
    (1, 37, 3, 37, 53, 4, 3),       # D % 4 != 0, W1 != W2, odd widths
    (3, 64, 1, 130, 129, 3, 4),     # realtime-style 3 levels, tile tails
    (1, 16, 1, 20, 600, 7, 2),      # 8 pyramid buffers: fused (7) + pool kernel
    (1, 32, 2, 33, 64, 2, 8),       # radius 8
    (1, 32, 2, 40, 50, 1, 1),       # single level, radius 1
]


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_random_vs_oracle(shape):
    B, D, H, W1, W2, L, r = shape
    g = torch.Generator().manual_seed(sum(shape))
    f1 = torch.randn(B, D, H, W1, generator=g)
    f2 = torch.randn(B, D, H, W2, generator=g)
    x = torch.arange(W1).float().view(1, 1, 1, W1) - torch.rand(B, 1, H, W1, generator=g) * 64
    x[..., ::7] = torch.randint(-10, W2 + 10, x[..., ::7].shape, generator=g).float()
    coords = torch.cat([x, torch.randn(B, 1, H, W1, generator=g)], 1)
    with torch.no_grad():
        blk = CorrBlock1D(f1.to(DEV), f2.to(DEV), num_levels=L, radius=r)
        out = blk(coords.to(DEV)).cpu().numpy()
    got = pyr_np(blk)
    ref = coracle.corr_pyramid(f1.numpy(), f2.numpy(), L)
    assert [a.shape for a in got] == [a.shape for a in ref]
    assert norm_err(got[0], ref[0]) <= VOL_TOL and rel_l2(got[0], ref[0]) <= VOL_L2
    for i in range(L):
        assert same(got[i + 1], coracle.corr_pool(got[i]))
    assert same(out, coracle.corr_lookup(got[:L], coords.numpy(), L, r))


def test_corr_staticmethod():
    z = load(files("volume")[0])
    with torch.no_grad():
        c = CorrBlock1D.corr(cu(z["fmap1"]), cu(z["fmap2"]))
    B, D, H, W1 = z["fmap1"].shape
    assert c.shape == (B, H, W1, 1, z["fmap2"].shape[3])
    assert norm_err(c.reshape(-1, c.shape[-1]).cpu().numpy(), z["level0"]) <= VOL_TOL


def test_bf16_pyramid_tolerance():
    z = load(files("lookup")[1])
    L, r = int(z["num_levels"]), int(z["radius"])
    with torch.no_grad():
        blk = CorrBlock1D(cu(z["fmap1"]), cu(z["fmap2"]), num_levels=L, radius=r,
                          pyramid_dtype=torch.bfloat16)
        out = blk(cu(z["coords"])).cpu().numpy()
    assert blk.corr_pyramid[0].dtype == torch.bfloat16
    assert norm_err(out, z["out"]) <= 1e-2 and rel_l2(out, z["out"]) <= 5e-3


def test_bf16_fmaps_accepted():
    z = load(files("volume")[1])
    with torch.no_grad():
        blk = CorrBlock1D(cu(z["fmap1"]).bfloat16(), cu(z["fmap2"]).bfloat16(), num_levels=4)
    got = pyr_np(blk)
    assert norm_err(got[0], z["level0"]) <= 1e-2


def test_errors_mirror_reference():
    f = torch.randn(1, 8, 2, 16, device=DEV)
    with pytest.raises(RuntimeError):
        CorrBlock1D(f, torch.randn(1, 8, 2, 9, device=DEV), num_levels=4)  # 9 >> 4 == 0
    with pytest.raises(RuntimeError):
        CorrBlock1D(f, torch.randn(1, 8, 3, 16, device=DEV))                # H mismatch
    blk = CorrBlock1D(f, f, num_levels=2, radius=2)
    with pytest.raises(RuntimeError):
        blk(torch.zeros(1, 2, 2, 15, device=DEV))                          # wrong W1
    with pytest.raises(RuntimeError):
        blk(torch.zeros(1, 2, 2, 16, device=DEV, dtype=torch.float64))     # dtype
    fg = f.clone().requires_grad_(True)
    conv = torch.nn.Conv2d(18, 8, 1).to(DEV)
    with pytest.raises(RuntimeError, match="inference-only"):
        CorrBlock1D(fg, fg, num_levels=2, radius=4).lookup_convc1(
            torch.zeros(1, 2, 2, 16, device=DEV), conv.weight, conv.bias)


CHAIN_SHAPES = [
    # B, D, H, W1, W2, L, r
    (2, 64, 3, 240, 240, 4, 4),
    (1, 32, 2, 311, 311, 4, 4),     # odd widths: 311/155/77/38
    (1, 16, 3, 45, 45, 4, 3),
    (1, 16, 2, 60, 61, 3, 4),       # 3 levels: span start at even offsets
    (2, 8, 2, 33, 130, 3, 2),
    (1, 8, 2, 20, 16, 4, 1),        # W2 = 16: level 3 of width 2
    (1, 16, 2, 50, 50, 2, 4),       # 2 levels: the pair kernel on level 0 alone
    (2, 8, 2, 33, 61, 2, 2),
    (1, 8, 3, 70, 77, 4, 2),        # odd level-2 width (19), level 3 of 9
]


def special_coords(B, H, W1, W2, g):
    x = torch.arange(W1).float().view(1, 1, 1, W1) - torch.rand(B, 1, H, W1, generator=g) * 64
    x[..., ::6] = torch.randint(-30, W2 + 30, x[..., ::6].shape, generator=g).float()
    x[..., 1::9] = x[..., 1::9] / 7.0 - 3.0
    flat = x.reshape(-1)
    vals = [float("nan"), float("inf"), -float("inf"), 1e30, -1e30, 0.0, -0.0, 1e-45, -1e-45,
            -2.8e-45, 3.0e-39, -3.0e-39, -1e-40, W2 - 1.0, W2 + 3.999, -4.5, -33.0, -35.0]
    flat[:len(vals)] = torch.tensor(vals)
    return torch.cat([flat.view(B, 1, H, W1), torch.zeros(B, 1, H, W1)], 1)


@pytest.mark.parametrize("shape", CHAIN_SHAPES, ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("stored", ["default", "level1", "level2"])
def test_chain_lookup_bitexact(shape, stored):
    """rc_corr_lookup_chain == the per-level lookup == the oracle, bit for bit,
    incl. NaN/inf/subnormal x, for each pool-chain kernel: the block's default
    (levels 0+2 stored -> pair kernel for 2/4 levels; 0+1 for 3), levels 0+1
    only (the level-1 chain kernel) and levels 0+2 only (the pair kernel)."""
    B, D, H, W1, W2, L, r = shape
    if stored == "level1" and L < 3 or stored == "level2" and L not in (2, 4):
        pytest.skip("kernel not defined for this level count")
    g = torch.Generator().manual_seed(900 + sum(shape))
    f1 = torch.randn(B, D, H, W1, generator=g).to(DEV)
    f2 = torch.randn(B, D, H, W2, generator=g).to(DEV)
    coords = special_coords(B, H, W1, W2, g)
    with torch.no_grad():
        blk = CorrBlock1D(f1, f2, num_levels=L, radius=r)
        assert blk._chain
        if stored == "default":
            a = blk(coords.to(DEV)).cpu().numpy()
        else:
            keep = {"level1": (0, 1), "level2": (0, 2)}[stored]
            lv = [t if i in keep else None for i, t in enumerate(blk.corr_pyramid[:L])]
            a = rcorr.lookup_chain(lv, coords.to(DEV), L, r).cpu().numpy()
        b = rcorr.lookup(blk.corr_pyramid, coords.to(DEV), L, r).cpu().numpy()
    assert same(a, b)
    assert same(a, coracle.corr_lookup(pyr_np(blk)[:L], coords.numpy(), L, r))


def test_chain_block_stores_two_levels():
    """An fp32 block with 2-4 levels stores the two levels its chain kernel
    reads (0+2, or 0+1 for 3 levels); the others appear on first read of
    corr_pyramid."""
    f = torch.randn(1, 8, 2, 64, device=DEV)
    with torch.no_grad():
        assert CorrBlock1D(f, f, num_levels=4).levels_stored == [0, 2]
        assert CorrBlock1D(f, f, num_levels=3).levels_stored == [0, 1]
        assert CorrBlock1D(f, f, num_levels=2).levels_stored == [0]
        blk = CorrBlock1D(f, f, num_levels=4)
        assert len(blk.corr_pyramid) == 5 and blk.levels_stored == [0, 1, 2, 3, 4]


def test_chain_not_used_for_other_levels():
    f = torch.randn(1, 8, 2, 64, device=DEV)
    with torch.no_grad():
        assert CorrBlock1D(f, f, num_levels=4, pyramid_dtype=torch.bfloat16)._chain
        assert not CorrBlock1D(f, f, num_levels=3, pyramid_dtype=torch.bfloat16)._chain
        assert not CorrBlock1D(f, f, num_levels=1)._chain
        assert not CorrBlock1D(f, f, num_levels=5, radius=2)._chain
        assert not CorrBlock1D(f, f, num_levels=4, radius=5)._chain


def bf16_pool_np(level):
    """avg_pool2d([1,2]) of a bf16 level in fp32, rounded to bf16 (RNE), as
    PyTorch computes it on bf16 tensors."""
    t = torch.from_numpy(np.ascontiguousarray(level)).bfloat16().float()
    Wo = t.shape[1] // 2
    pm = (t[:, 0:2 * Wo:2] + t[:, 1:2 * Wo:2]) * 0.5
    return pm.bfloat16().float().numpy()


BF16_PAIR_SHAPES = [
    # B, D, H, W1, W2, L, r
    (2, 64, 3, 240, 240, 4, 4),
    (1, 32, 2, 311, 311, 4, 4),     # config-3 width: odd level widths
    (1, 16, 3, 45, 45, 4, 3),
    (1, 16, 2, 50, 50, 2, 4),
    (1, 8, 2, 20, 16, 4, 1),
]


@pytest.mark.parametrize("shape", BF16_PAIR_SHAPES, ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("fmap_dt", [torch.bfloat16, torch.float32], ids=["bf16in", "f32in"])
def test_bf16_pair_lookup_bitexact(shape, fmap_dt):
    """bf16 pyramid (config 3): every level is the bf16 pool of the level
    below as stored (the build epilogue, rc_corr_pool and avg_pool2d on bf16
    agree), and the pair kernel (levels 0 and 2 read, 1 and 3 derived and
    rounded) equals the per-level lookup over the materialised bf16 pyramid
    bit for bit, NaN/inf/subnormal coords included."""
    B, D, H, W1, W2, L, r = shape
    g = torch.Generator().manual_seed(700 + sum(shape))
    f1 = torch.randn(B, D, H, W1, generator=g).to(DEV, fmap_dt)
    f2 = torch.randn(B, D, H, W2, generator=g).to(DEV, fmap_dt)
    coords = special_coords(B, H, W1, W2, g).to(DEV)
    with torch.no_grad():
        blk = CorrBlock1D(f1, f2, num_levels=L, radius=r, pyramid_dtype=torch.bfloat16)
        eager = CorrBlock1D(f1, f2, num_levels=L, radius=r, pyramid_dtype=torch.bfloat16,
                            lazy_levels=False)
        assert blk._chain and blk.levels_stored == ([0, 2] if L == 4 else [0])
        a = blk(coords)
        pyr = blk.corr_pyramid
        b = rcorr.lookup(pyr, coords, L, r)
        c = eager(coords)
    assert same(a.cpu().numpy(), b.cpu().numpy())
    assert same(a.cpu().numpy(), c.cpu().numpy())
    lv = pyr_np(blk)
    le = pyr_np(eager)
    for i in range(L + 1):
        assert same(lv[i], le[i]), f"lazy vs fused epilogue, level {i}"
        if i:
            assert same(lv[i], bf16_pool_np(lv[i - 1])), f"level {i} != bf16 pool of level {i - 1}"


def test_repeat_launches_deterministic():
    g = torch.Generator().manual_seed(3)
    f1 = torch.randn(2, 64, 4, 96, generator=g).to(DEV)
    f2 = torch.randn(2, 64, 4, 96, generator=g).to(DEV)
    c = (torch.arange(96).float().view(1, 1, 1, 96) - 10 * torch.rand(2, 1, 4, 96, generator=g))
    c = torch.cat([c, c], 1).to(DEV)
    with torch.no_grad():
        outs = [CorrBlock1D(f1, f2)(c) for _ in range(5)]
    for o in outs[1:]:
        assert torch.equal(o, outs[0])


BF16_SHAPES = [
    (1, 256, 2, 64, 64, 4, 4),
    (2, 256, 2, 311, 311, 4, 4),    # config-3 width: rows not 16-B aligned
    (1, 96, 3, 40, 57, 3, 3),       # D % 32 != 0, odd W2
    (1, 37, 2, 24, 33, 4, 2),
    # bf16-fmap ring kernel: 4 waves along w2 x 3 w2 tiles, 6 w1 tiles
    (1, 64, 2, 700, 720, 4, 4),
    (1, 256, 1, 150, 130, 3, 4),    # 3 waves along w2; idle waves in the last w1 tile
    (1, 40, 2, 100, 100, 4, 2),     # 2 waves along w2, D % 32 != 0
]


@pytest.mark.parametrize("shape", BF16_SHAPES, ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("mode", ["bf16in_f32pyr", "bf16in_bf16pyr", "f32in_bf16pyr"])
def test_bf16_mma_vs_oracle(shape, mode):
    """bf16 MFMA kernel vs the fp64-accumulated oracle on bf16-rounded inputs.
    Tolerances: fp32 pyramid 1e-5 normalised (only the summation order
    differs: bf16 products are exact in fp32); bf16 pyramid 8e-3 normalised
    (one bf16 rounding of each stored value)."""
    B, D, H, W1, W2, L, r = shape
    g = torch.Generator().manual_seed(7 + sum(shape))
    f1 = torch.randn(B, D, H, W1, generator=g)
    f2 = torch.randn(B, D, H, W2, generator=g)
    f1r, f2r = f1.bfloat16().float(), f2.bfloat16().float()   # what the kernel multiplies
    x = torch.arange(W1).float().view(1, 1, 1, W1) - torch.rand(B, 1, H, W1, generator=g) * 40
    coords = torch.cat([x, torch.zeros_like(x)], 1)
    in_dt = torch.float32 if mode.startswith("f32in") else torch.bfloat16
    pyr_dt = torch.bfloat16 if mode.endswith("bf16pyr") else torch.float32
    with torch.no_grad():
        blk = CorrBlock1D(f1.to(DEV, in_dt), f2.to(DEV, in_dt), num_levels=L, radius=r,
                          pyramid_dtype=pyr_dt)
        out = blk(coords.to(DEV)).cpu().numpy()
    assert blk.corr_pyramid[0].dtype == pyr_dt
    got = pyr_np(blk)
    ref = coracle.corr_pyramid(f1r.numpy(), f2r.numpy(), L)
    tol = 1e-5 if pyr_dt == torch.float32 else 8e-3
    for i in range(L + 1):
        assert norm_err(got[i], ref[i]) <= tol, f"level {i}"
    if pyr_dt == torch.float32:
        for i in range(L):
            assert same(got[i + 1], coracle.corr_pool(got[i]))
    # the lookup reads the stored (bf16 or fp32) pyramid exactly
    assert same(out, coracle.corr_lookup(got[:L], coords.numpy(), L, r))


@pytest.mark.parametrize("pyr_dt", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_lookup_large_p_vs_oracle(pyr_dt):
    """P above the small-problem threshold takes the 256-thread runtime-level
    kernel; check it (random pyramid, padded rows, random coords incl. OOB)."""
    B, H, W1, W2, L, r = 3, 135, 240, 240, 4, 4            # P = 97200 * ... see below
    B = 6                                                  # P = 194400 > 131072
    g = torch.Generator().manual_seed(11)
    P = B * H * W1
    pyr = []
    for l in range(L):
        Wl = W2 >> l
        buf = torch.randn(P, Wl + 3, generator=g).to(pyr_dt)   # padded rows (stride Wl+3)
        pyr.append(buf.to(DEV)[:, :Wl].unsqueeze(1).unsqueeze(1))
    x = torch.arange(W1).float().view(1, 1, 1, W1) - torch.rand(B, 1, H, W1, generator=g) * 64
    x[..., ::11] = torch.randint(-20, W2 + 20, x[..., ::11].shape, generator=g).float()
    coords = torch.cat([x, torch.zeros_like(x)], 1)
    with torch.no_grad():
        out = rcorr.lookup(pyr, coords.to(DEV), L, r).cpu().numpy()
    ref = coracle.corr_lookup([t.reshape(P, -1).float().cpu().numpy() for t in pyr],
                              coords.numpy(), L, r)
    assert same(out, ref)


EDGE_SHAPES = [
    # B, D, H, W1, W2, L, r
    (1, 1, 1, 1, 16, 4, 4),       # D = 1, a single pixel
    (2, 3, 1, 5, 2, 1, 1),        # W2 = 2, one level
    (1, 8, 5, 1, 64, 6, 3),       # W1 = 1, 7 pyramid buffers
    (1, 64, 1, 129, 128, 7, 2),   # 8 buffers: 7 fused + 1 pool-kernel level
    (3, 16, 2, 67, 67, 2, 5),     # odd everything, radius 5
]


@pytest.mark.parametrize("shape", EDGE_SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_edge_shapes_vs_oracle(shape):
    B, D, H, W1, W2, L, r = shape
    g = torch.Generator().manual_seed(101 + sum(shape))
    f1 = torch.randn(B, D, H, W1, generator=g)
    f2 = torch.randn(B, D, H, W2, generator=g)
    x = torch.rand(B, 1, H, W1, generator=g) * (W2 + 8) - 4
    coords = torch.cat([x, torch.randn(B, 1, H, W1, generator=g)], 1)
    with torch.no_grad():
        blk = CorrBlock1D(f1.to(DEV), f2.to(DEV), num_levels=L, radius=r)
        out = blk(coords.to(DEV)).cpu().numpy()
    got = pyr_np(blk)
    ref = coracle.corr_pyramid(f1.numpy(), f2.numpy(), L)
    assert [a.shape for a in got] == [a.shape for a in ref]
    assert norm_err(got[0], ref[0]) <= VOL_TOL
    for i in range(L):
        assert same(got[i + 1], coracle.corr_pool(got[i]))
    assert same(out, coracle.corr_lookup(got[:L], coords.numpy(), L, r))


def test_empty_inputs():
    """B = 0 / H = 0: empty outputs of the right shapes, nothing launched."""
    for B, H in ((0, 3), (2, 0)):
        f = torch.randn(B, 8, H, 16, device=DEV)
        blk = CorrBlock1D(f, f, num_levels=2, radius=2)
        assert [t.shape for t in blk.corr_pyramid] == [(0, 1, 1, 16), (0, 1, 1, 8), (0, 1, 1, 4)]
        out = blk(torch.zeros(B, 2, H, 16, device=DEV))
        assert out.shape == (B, 10, H, 16)


def test_noncontiguous_coords_and_fmaps():
    """Strided coords (e.g. a view of a larger tensor) and non-contiguous fmaps
    give the same result as their contiguous copies."""
    g = torch.Generator().manual_seed(5)
    f1 = torch.randn(2, 32, 4, 48, generator=g).to(DEV)
    f2 = torch.randn(2, 32, 48, 4, generator=g).to(DEV).transpose(2, 3)   # non-contiguous
    big = torch.randn(2, 5, 4, 48, generator=g).to(DEV) * 10 + 20
    coords = big[:, 1:3]                                                    # strided view
    with torch.no_grad():
        a = CorrBlock1D(f1, f2, num_levels=3, radius=3)(coords)
        b = CorrBlock1D(f1, f2.contiguous(), num_levels=3, radius=3)(coords.contiguous())
    assert torch.equal(a, b)


@pytest.mark.parametrize("L", [1, 2, 3, 4, 5])
@pytest.mark.parametrize("r", [1, 2, 3, 4, 6, 8])
def test_levels_radius_grid(L, r):
    g = torch.Generator().manual_seed(L * 10 + r)
    B, D, H, W1, W2 = 1, 16, 2, 40, 96
    f1 = torch.randn(B, D, H, W1, generator=g)
    f2 = torch.randn(B, D, H, W2, generator=g)
    x = torch.rand(B, 1, H, W1, generator=g) * 110 - 7
    coords = torch.cat([x, torch.zeros_like(x)], 1)
    with torch.no_grad():
        blk = CorrBlock1D(f1.to(DEV), f2.to(DEV), num_levels=L, radius=r)
        out = blk(coords.to(DEV)).cpu().numpy()
    got = pyr_np(blk)
    assert same(out, coracle.corr_lookup(got[:L], coords.numpy(), L, r))


@pytest.mark.parametrize("L,r,pyr_dt,bias,relu", [
    (4, 4, torch.float32, True, True), (3, 4, torch.float32, True, True),
    (2, 3, torch.float32, False, False), (4, 4, torch.bfloat16, True, True)])
def test_lookup_convc1_vs_separate(L, r, pyr_dt, bias, relu):
    """Fused lookup+convc1(+ReLU) vs our lookup followed by torch's 1x1 conv
    (fp32).  Tolerance 1e-5 normalised: only the 1x1 conv's summation order
    differs (k ascending fmaf chain vs the library's GEMM)."""
    g = torch.Generator().manual_seed(31 * L + r)
    B, D, H, W1, W2 = 2, 64, 5, 96, 96
    f1 = torch.randn(B, D, H, W1, generator=g).to(DEV)
    f2 = torch.randn(B, D, H, W2, generator=g).to(DEV)
    x = torch.arange(W1).float().view(1, 1, 1, W1) - torch.rand(B, 1, H, W1, generator=g) * 30
    coords = torch.cat([x, torch.zeros_like(x)], 1).to(DEV)
    conv = torch.nn.Conv2d(L * (2 * r + 1), 64, 1, bias=bias).to(DEV)
    with torch.no_grad():
        blk = CorrBlock1D(f1, f2, num_levels=L, radius=r, pyramid_dtype=pyr_dt)
        fused = blk.lookup_convc1(coords, conv.weight, conv.bias, relu=relu)
        ref = conv(blk(coords))
        if relu:
            ref = torch.relu(ref)
    assert fused.shape == ref.shape
    assert norm_err(fused.cpu().numpy(), ref.cpu().numpy()) <= 1e-5


def test_lookup_convc1_prefetch_bit_identical(monkeypatch):
    """The default fused kernel issues every level's loads up front; the
    one-level-at-a-time kernel (RAFTCORR_CONV_VARIANT=1) does the same
    arithmetic: identical bits, NaN / inf / out-of-range coords included."""
    g = torch.Generator().manual_seed(4242)
    B, D, H, W1, W2, L, r = 2, 32, 3, 130, 130, 4, 4
    f1 = torch.randn(B, D, H, W1, generator=g).to(DEV)
    f2 = torch.randn(B, D, H, W2, generator=g).to(DEV)
    x = torch.arange(W1).float().view(1, 1, 1, W1) - torch.rand(B, 1, H, W1, generator=g) * 60
    x[..., ::7] = torch.randint(-20, W2 + 20, x[..., ::7].shape, generator=g).float()
    x[0, 0, 0, :5] = torch.tensor([float("nan"), float("inf"), -float("inf"), 1e30, -1e30])
    coords = torch.cat([x, torch.zeros_like(x)], 1).to(DEV)
    conv = torch.nn.Conv2d(L * (2 * r + 1), 64, 1).to(DEV)
    with torch.no_grad():
        blk = CorrBlock1D(f1, f2, num_levels=L, radius=r)
        a = blk.lookup_convc1(coords, conv.weight, conv.bias)
        monkeypatch.setenv("RAFTCORR_CONV_VARIANT", "1")
        with _lib.dev_library():
            b = blk.lookup_convc1(coords, conv.weight, conv.bias)
    assert torch.equal(a.nan_to_num(nan=7.0), b.nan_to_num(nan=7.0))


@pytest.mark.parametrize("shape", [(2, 64, 3, 240, 240, 4, 4), (1, 32, 2, 311, 311, 3, 3),
                                   (1, 16, 2, 45, 61, 4, 2)], ids=lambda s: "x".join(map(str, s)))
def test_lazy_levels_equal_fused_epilogue(shape):
    """Default fp32 blocks write two levels in the build (0+2, or 0+1 for 3
    levels) and pool the others on first access to corr_pyramid; the eager
    build writes every level in the fused epilogue.  Same values bit for bit,
    same lookups."""
    B, D, H, W1, W2, L, r = shape
    g = torch.Generator().manual_seed(1234 + sum(shape))
    f1 = torch.randn(B, D, H, W1, generator=g).to(DEV)
    f2 = torch.randn(B, D, H, W2, generator=g).to(DEV)
    coords = special_coords(B, H, W1, W2, g).to(DEV)
    with torch.no_grad():
        lazy = CorrBlock1D(f1, f2, num_levels=L, radius=r)
        eager = CorrBlock1D(f1, f2, num_levels=L, radius=r, lazy_levels=False)
        stored = lazy.levels_stored
        assert len(stored) == 2 and eager.levels_stored == list(range(L + 1))
        a, b = lazy(coords), eager(coords)
        assert lazy.levels_stored == stored            # the lookup did not need the others
    assert same(a.cpu().numpy(), b.cpu().numpy())
    pl, pe = pyr_np(lazy), pyr_np(eager)
    assert len(pl) == len(pe) == L + 1
    for i in range(L + 1):
        assert lazy.corr_pyramid[i].shape == eager.corr_pyramid[i].shape
        assert same(pl[i], pe[i]), f"level {i}"


@pytest.mark.parametrize("L,r,pyr_dt", [(4, 4, torch.float32), (3, 3, torch.float32),
                                        (2, 4, torch.float32), (4, 4, torch.bfloat16)])
def test_lookup_step_matches_unfused(L, r, pyr_dt):
    """rc_corr_lookup_step == the loop's PyTorch ops
    (coords1 + delta with delta[:,1] = 0; flow = coords1 - coords_grid) and
    the plain lookup at the new coords, bit for bit; also in place."""
    g = torch.Generator().manual_seed(40 + L + r)
    B, D, H, W1, W2 = 2, 32, 5, 96, 96
    f1 = torch.randn(B, D, H, W1, generator=g).to(DEV)
    f2 = torch.randn(B, D, H, W2, generator=g).to(DEV)
    c0 = rcorr.coords_grid(B, H, W1).to(DEV)
    c1 = c0.clone()
    c1[:, 0] -= (torch.rand(B, H, W1, generator=g) * 30).to(DEV)
    delta = (torch.randn(B, 2, H, W1, generator=g) * 3).to(DEV)
    with torch.no_grad():
        blk = CorrBlock1D(f1, f2, num_levels=L, radius=r, pyramid_dtype=pyr_dt)
        corr, new, flow = blk.lookup_step(c1, delta)
        d = delta.clone()
        d[:, 1] = 0.0
        ref_new = c1 + d
        assert torch.equal(new, ref_new)
        assert torch.equal(flow, ref_new - c0)
        assert same(corr.cpu().numpy(), blk(ref_new).cpu().numpy())
        # first iteration (no delta) and in-place update
        corr0, new0, flow0 = blk.lookup_step(c1)
        assert torch.equal(new0, c1) and torch.equal(flow0, c1 - c0)
        assert same(corr0.cpu().numpy(), blk(c1).cpu().numpy())
        buf = c1.clone()
        corr2, new2, _ = blk.lookup_step(buf, delta, out=buf)
        assert new2.data_ptr() == buf.data_ptr() and torch.equal(buf, ref_new)
        assert same(corr2.cpu().numpy(), corr.cpu().numpy())


RING_SHAPES = [
    # B, D, H, W1, W2, L  (L + 1 = 7 buffers: every level in the fused epilogue)
    (1, 64, 2, 130, 200, 6),
    (2, 32, 2, 67, 311, 6),
    (1, 48, 3, 311, 311, 6),
]


@pytest.mark.parametrize("shape", RING_SHAPES, ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("pyr_dt", [torch.float32, torch.bfloat16], ids=["f32pyr", "bf16pyr"])
def test_bf16_ring_epilogue_all_levels(shape, pyr_dt, monkeypatch):
    """bf16 fmaps take the LDS-DMA ring kernel, whose epilogue pools levels
    1-6 in registers (lane-local, xor-16, xor-32, fragment pairs).  Eager
    build of 7 levels: level 0 vs the oracle, every level i >= 1 == the pool
    of level i-1 as stored (corr_pool / bf16 avg_pool2d) bit for bit, and the
    per-wave bf16 kernel (dev library, RAFTCORR_BUILD_MODE=32) gives the same
    bits."""
    B, D, H, W1, W2, L = shape
    g = torch.Generator().manual_seed(99 + sum(shape))
    f1 = torch.randn(B, D, H, W1, generator=g).bfloat16()
    f2 = torch.randn(B, D, H, W2, generator=g).bfloat16()
    with torch.no_grad():
        blk = CorrBlock1D(f1.to(DEV), f2.to(DEV), num_levels=L, radius=2, pyramid_dtype=pyr_dt,
                          lazy_levels=False)
        got = pyr_np(blk)
    ref = coracle.corr_pyramid(f1.float().numpy(), f2.float().numpy(), 0)[0]
    assert norm_err(got[0], ref) <= (1e-5 if pyr_dt == torch.float32 else 8e-3)
    for i in range(1, L + 1):
        want = coracle.corr_pool(got[i - 1]) if pyr_dt == torch.float32 else bf16_pool_np(got[i - 1])
        assert same(got[i], want), f"level {i}"
    # the product assertions above always run; the per-wave variant
    # comparison below only where the dev library was pushed
    if not os.path.exists(_lib.DEV_LIB_PATH):
        return
    monkeypatch.setenv("RAFTCORR_BUILD_MODE", "32")
    with torch.no_grad(), _lib.dev_library():
        old = pyr_np(CorrBlock1D(f1.to(DEV), f2.to(DEV), num_levels=L, radius=2,
                                 pyramid_dtype=pyr_dt, lazy_levels=False))
    for i in range(L + 1):
        assert same(got[i], old[i]), f"ring vs per-wave kernel, level {i}"
