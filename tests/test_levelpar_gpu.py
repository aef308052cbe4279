"""CorrBlock1D(low_latency=True): every level stored, per-level lookup that
gives each level its own wave below 64K pixels (lookup_levelpar_kernel).
Same values bit for bit as the default block (pair / chain kernels), incl.
NaN/inf/subnormal coords and the fused loop step updating coords in place
(the kernel's block barrier orders the coords reads before the writes)."""
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
        assert not ll._chain and ll.levels_stored == list(range(L + 1))
        assert torch.equal(ll(coords).view(torch.int32), ref(coords).view(torch.int32))
        d = torch.randn(coords.shape, generator=g).to(DEV)
        c_ref, c_ll = coords.clone(), coords.clone()
        a = ref.lookup_step(c_ref, d, out=c_ref)        # in place
        b = ll.lookup_step(c_ll, d, out=c_ll)
        for u, v in zip(a, b):
            assert torch.equal(u.view(torch.int32), v.view(torch.int32))
        assert torch.equal(c_ref.view(torch.int32), c_ll.view(torch.int32))
