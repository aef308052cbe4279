"""CorrBlock1D(low_latency=True): the levels a lookup reads (0 .. L-1) stored,
the top one pooled when corr_pyramid is read; per-level lookup that gives
each level its own wave below 64K pixels (lookup_levelpar_kernel).
Same values bit for bit as the default block (pair / chain kernels), incl.
NaN/inf/subnormal coords and the fused loop step updating coords in place
(the kernel's block barrier orders the coords reads before the writes)."""
import numpy as np
import pytest
import torch

from raft_stereo_amd import CorrBlock1D

from test_corr_gpu import CHAIN_SHAPES, special_coords

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("shape", CHAIN_SHAPES, ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_low_latency_bit_identical(shape, dt):
    B, D, H, W1, W2, L, r = shape
    if dt == torch.bfloat16 and L == 3:
        pytest.skip("bf16 pyramids use the pair layout (2 or 4 levels) by default")
    g = torch.Generator().manual_seed(2100 + B * H + W1 + W2)
    f1 = torch.randn(B, D, H, W1, generator=g).to(DEV)
    f2 = torch.randn(B, D, H, W2, generator=g).to(DEV)
    coords = special_coords(B, H, W1, W2, g).to(DEV)
    with torch.no_grad():
        ref = CorrBlock1D(f1, f2, num_levels=L, radius=r, pyramid_dtype=dt)
        ll = CorrBlock1D(f1, f2, num_levels=L, radius=r, pyramid_dtype=dt, low_latency=True)
        assert not ll._chain and ll.levels_stored == list(range(L))
        assert torch.equal(ll(coords).view(torch.int32), ref(coords).view(torch.int32))
        assert ll.levels_stored == list(range(L))       # the lookup did not pool the top level
        d = torch.randn(coords.shape, generator=g).to(DEV)
        c_ref, c_ll = coords.clone(), coords.clone()
        a = ref.lookup_step(c_ref, d, out=c_ref)        # in place
        b = ll.lookup_step(c_ll, d, out=c_ll)
        for u, v in zip(a, b):
            assert torch.equal(u.view(torch.int32), v.view(torch.int32))
        assert torch.equal(c_ref.view(torch.int32), c_ll.view(torch.int32))
        # every level, the lazily pooled top one included, equals the default
        # block's (and the eager build's) bit for bit
        eager = CorrBlock1D(f1, f2, num_levels=L, radius=r, pyramid_dtype=dt, low_latency=True,
                            lazy_levels=False)
        assert eager.levels_stored == list(range(L + 1))
        iv = torch.int16 if dt == torch.bfloat16 else torch.int32
        for u, v, w in zip(ref.corr_pyramid, ll.corr_pyramid, eager.corr_pyramid):
            assert torch.equal(u.contiguous().view(iv), v.contiguous().view(iv))
            assert torch.equal(v.contiguous().view(iv), w.contiguous().view(iv))
        assert len(ll.corr_pyramid) == L + 1


# below 64K pixels every rc_corr_lookup with 1-4 levels takes the
# level-parallel kernel, whatever the radius (1-8); shapes the chain / pair
# kernels never served (1 level, radius > 4) against the C oracle, bit for bit.
LEVELPAR_EXTRA = [
    # B, D, H, W1, W2, L, r
    (1, 16, 2, 40, 48, 1, 3),
    (1, 16, 2, 33, 64, 1, 8),
    (2, 8, 2, 30, 64, 2, 6),
    (1, 16, 3, 45, 90, 3, 5),
    (1, 8, 2, 50, 128, 4, 7),
]


@pytest.mark.parametrize("shape", LEVELPAR_EXTRA, ids=lambda s: "x".join(map(str, s)))
def test_levelpar_levels_radius_vs_oracle(shape):
    from oracle import coracle
    from raft_stereo_amd import corr as rcorr
    B, D, H, W1, W2, L, r = shape
    g = torch.Generator().manual_seed(sum(shape) + 99)
    f1 = torch.randn(B, D, H, W1, generator=g).to(DEV)
    f2 = torch.randn(B, D, H, W2, generator=g).to(DEV)
    c = special_coords(B, H, W1, W2, g)
    with torch.no_grad():
        blk = CorrBlock1D(f1, f2, num_levels=L, radius=r, low_latency=True)
        pyr = [t.reshape(t.shape[0], -1) for t in blk.corr_pyramid[:L]]
        a = blk(c.to(DEV)).cpu().numpy()
        b = rcorr.lookup(blk.corr_pyramid, c.to(DEV), L, r).cpu().numpy()
    ref = coracle.corr_lookup([t.cpu().numpy() for t in pyr], c.numpy(), L, r)
    assert np.array_equal(a, ref, equal_nan=True)
    assert np.array_equal(b, ref, equal_nan=True)
