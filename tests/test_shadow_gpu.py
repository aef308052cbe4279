"""RC_SHADOW (ABI v5): the pair layout's stored levels carry a
copy shifted by half a 128-B line, and the pair lookup reads each pixel's
span from whichever copy it touches fewer lines in.  The values are the
same, so every result must be bit-identical to the unshadowed block's --
the reference-parity tests (test_chain_lookup_bitexact, the golden and
oracle tests) run through the shadowed default as well."""
import numpy as np
import pytest
import torch

from raft_stereo_amd import CorrBlock1D, _lib
from raft_stereo_amd import corr as rcorr

from test_corr_gpu import CHAIN_SHAPES, BF16_PAIR_SHAPES, special_coords

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def whole_allocation(t):
    """The flat buffer behind a level view (primary copy + shadow copy)."""
    st = t.untyped_storage()
    es = t.element_size()
    return torch.tensor([], dtype=t.dtype, device=t.device).set_(st, 0, (st.nbytes() // es,), (1,))


def shadow_view(t):
    """(P, W) view of the RC_SHADOW copy of level view t (P, 1, 1, W)."""
    P, W = t.shape[0], t.shape[-1]
    ld = rcorr._row_stride(t)
    es = t.element_size()
    off = _lib.shadow_offset(P, ld, es)
    assert off % es == 0
    flat = whole_allocation(t)
    assert flat.numel() * es >= off + P * ld * es
    return flat[off // es: off // es + P * ld].view(P, ld)[:, :W]


def pair_shapes():
    f32 = [(s, torch.float32) for s in CHAIN_SHAPES if s[5] in (2, 4)]
    b16 = [(s, torch.bfloat16) for s in BF16_PAIR_SHAPES]
    return f32 + b16


def ids(p):
    s, dt = p
    return "x".join(map(str, s)) + ("-bf16" if dt == torch.bfloat16 else "-f32")


@pytest.mark.parametrize("case", pair_shapes(), ids=ids)
def test_shadow_lookup_bit_identical(case):
    """Shadowed block == unshadowed block bit for bit (NaN/inf/subnormal
    coords included), and every stored level's shadow holds its values."""
    (B, D, H, W1, W2, L, r), dt = case
    g = torch.Generator().manual_seed(1300 + B * H + W1 + W2)
    f1 = torch.randn(B, D, H, W1, generator=g).to(DEV)
    f2 = torch.randn(B, D, H, W2, generator=g).to(DEV)
    coords = special_coords(B, H, W1, W2, g).to(DEV)
    with torch.no_grad():
        sh = CorrBlock1D(f1, f2, num_levels=L, radius=r, pyramid_dtype=dt, shadow=True)
        ns = CorrBlock1D(f1, f2, num_levels=L, radius=r, pyramid_dtype=dt, shadow=False)
        assert sh._shadow == frozenset(sh.levels_stored) and not ns._shadow
        assert torch.equal(sh(coords).view(torch.int32), ns(coords).view(torch.int32))
        for l in sh.levels_stored:
            prim = sh._levels[l].reshape(sh._levels[l].shape[0], -1)
            assert torch.equal(shadow_view(sh._levels[l]).view(torch.int16 if dt == torch.bfloat16 else torch.int32),
                               prim.view(torch.int16 if dt == torch.bfloat16 else torch.int32)), f"level {l}"
        # the fused loop step reads the same copies
        c1 = coords.clone()
        d = torch.randn(c1.shape, generator=g).to(DEV)
        a = sh.lookup_step(c1, d)
        b = ns.lookup_step(c1, d)
        for x, y in zip(a, b):
            assert torch.equal(x.view(torch.int32), y.view(torch.int32))


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_shadow_copies_are_both_read(dt):
    """Poisoning one copy of a stored level changes some pixels' outputs of
    the two levels it serves, poisoning the other copy changes other pixels:
    each lane picks one copy per span, and both copies are in use."""
    # bf16 at W = 240 would have level-2 rows of exactly one 128-B line (60
    # elements padded to 64): every span fits the primary, no shadow is read
    B, D, H = 2, 32, 4
    W = 240 if dt == torch.float32 else 311
    g = torch.Generator().manual_seed(77)
    f1 = torch.randn(B, D, H, W, generator=g).to(DEV)
    f2 = torch.randn(B, D, H, W, generator=g).to(DEV)
    x = torch.arange(W).float().view(1, 1, 1, W) - torch.rand(B, 1, H, W, generator=g) * 64
    coords = torch.cat([x, torch.zeros_like(x)], 1).to(DEV)
    T = 9
    with torch.no_grad():
        blk = CorrBlock1D(f1, f2, num_levels=4, radius=4, pyramid_dtype=dt, shadow=True)
        ref = blk(coords)
        for l in (0, 2):
            lvl = blk._levels[l]
            saved = whole_allocation(lvl).clone()
            bad = {}
            for poison in ("shadow", "primary"):
                v = shadow_view(lvl) if poison == "shadow" else lvl.view(lvl.shape[0], -1)
                v.fill_(float("nan"))
                out = blk(coords)[:, l * T:(l + 2) * T]
                bad[poison] = torch.isnan(out).any(1)
                whole_allocation(lvl).copy_(saved)
            a, b = bad["shadow"], bad["primary"]
            assert a.any() and b.any(), f"level {l}: both copies are read"
            assert not (a & b).any(), f"level {l}: one copy per span"
        assert torch.equal(blk(coords).view(torch.int32), ref.view(torch.int32))


@pytest.mark.parametrize("cfg", ["sceneflow", "kitti8"])
def test_shadow_fullsize_bit_identical(cfg):
    """Config 2 (B=8, 135x240, fp32) and config 3's shape (B=8, 94x311, bf16):
    shadowed == unshadowed over every pixel, bench coordinates."""
    B, D, H, W, dt = {"sceneflow": (8, 256, 135, 240, torch.float32),
                      "kitti8": (8, 256, 94, 311, torch.bfloat16)}[cfg]
    g = torch.Generator().manual_seed(5)
    f1 = torch.randn(B, D, H, W, generator=g).to(DEV, dt)
    f2 = torch.randn(B, D, H, W, generator=g).to(DEV, dt)
    x = torch.arange(W).float().view(1, 1, 1, W) - torch.rand(B, 1, H, W, generator=g) * 64
    coords = torch.cat([x, torch.zeros_like(x)], 1).to(DEV)
    with torch.no_grad():
        dflt = CorrBlock1D(f1, f2)
        sh = CorrBlock1D(f1, f2, shadow=True)
        ns = CorrBlock1D(f1, f2, shadow=False)
        # default levels: level 2 always, level 0 once it
        # outgrows the 256 MiB Infinity Cache (here 237 / 139 MiB: not yet)
        assert dflt._shadow == frozenset({2})
        assert sh._shadow == frozenset({0, 2})
        ref = ns(coords).view(torch.int32)
        assert torch.equal(sh(coords).view(torch.int32), ref)
        assert torch.equal(dflt(coords).view(torch.int32), ref)
