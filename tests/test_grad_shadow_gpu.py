"""RC_SHADOW gradient copies: the pair lookup backward adds
each pixel's span into whichever copy of the level-0 / level-2 gradient it
touches fewer 128-B lines in, and the build backward sums the two copies.
Only the order of additions changes, so gradients agree with the unshadowed
buffers to fp32 rounding; both copies must receive spans."""
import pytest
import torch

from raft_stereo_amd import CorrBlock1D, _lib
from raft_stereo_amd import corr as rcorr

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def copy_views(buf):
    """(primary, shadow) (P, ld) views of a gradient level with a shadow."""
    P, W = buf.shape
    ld = buf.stride(0)
    st = buf.untyped_storage()
    flat = torch.tensor([], dtype=torch.float32, device=buf.device).set_(st, 0, (st.nbytes() // 4,), (1,))
    off = _lib.shadow_offset(P, ld, 4) // 4
    return flat[:P * ld].view(P, ld)[:, :W], flat[off:off + P * ld].view(P, ld)[:, :W]


@pytest.mark.parametrize("shape", [(2, 32, 6, 240, 240, 4), (1, 64, 5, 311, 311, 4), (2, 32, 3, 97, 130, 3)])
@pytest.mark.parametrize("sh", [(0,), (2,), (0, 2)], ids=["l0", "l2", "l0l2"])
def test_grad_shadow_matches_unshadowed(shape, sh):
    B, D, H, W1, W2, r = shape
    g = torch.Generator().manual_seed(B * W1 + H + r)
    f1 = torch.randn(B, D, H, W1, generator=g).to(DEV)
    f2 = torch.randn(B, D, H, W2, generator=g).to(DEV)
    P, T, L = B * H * W1, 2 * r + 1, 4
    widths = [W2 >> i for i in range(L)]
    out = {}
    for name, s in (("ref", ()), ("sh", sh)):
        grads = rcorr.grad_buffers(P, widths, DEV, pair=True, shadow=s)
        gg = torch.Generator().manual_seed(9)
        for _ in range(5):
            x = torch.arange(W1).float().view(1, 1, 1, W1) - torch.rand(B, 1, H, W1, generator=gg) * 48
            coords = torch.cat([x, torch.zeros_like(x)], 1).to(DEV)
            go = torch.randn(B, L * T, H, W1, generator=gg).to(DEV)
            rcorr.lookup_backward(grads, coords, go, L, r)
        out[name] = (grads, rcorr.build_backward(f1, f2, grads))
    (gr, (a1, a2)), (gs, (b1, b2)) = out["ref"], out["sh"]
    for x, y in ((b1, a1), (b2, a2)):
        assert float((x - y).norm() / y.norm()) < 1e-6
    for l in (0, 2):
        if l in sh:
            prim, shad = copy_views(gs[l])
            # rows of exactly one aligned line (W2 = 130: level 2 is 32 floats)
            # never straddle, so their spans all stay in the primary
            one_line = gs[l].stride(0) * 4 == 128
            assert prim.abs().sum() > 0 and (one_line or shad.abs().sum() > 0), \
                f"level {l}: both copies receive spans"
            torch.testing.assert_close(prim + shad, gr[l], rtol=1e-5, atol=1e-5)
        else:
            torch.testing.assert_close(gs[l], gr[l], rtol=0, atol=0)


def test_grad_shadow_autograd_block():
    """CorrBlock1D(grad_shadow=(0, 2)) through autograd == grad_shadow=()."""
    B, D, H, W = 2, 32, 4, 200
    g = torch.Generator().manual_seed(4)
    f1 = torch.randn(B, D, H, W, generator=g).to(DEV)
    f2 = torch.randn(B, D, H, W, generator=g).to(DEV)
    x = torch.arange(W).float().view(1, 1, 1, W) - torch.rand(B, 1, H, W, generator=g) * 40
    coords = torch.cat([x, torch.zeros_like(x)], 1).to(DEV)
    res = []
    for s in ((), (0, 2)):
        a = f1.clone().requires_grad_()
        b = f2.clone().requires_grad_()
        blk = CorrBlock1D(a, b, grad_shadow=s)
        assert blk._state.grad_shadow == frozenset(s)
        (blk(coords) * torch.linspace(-1, 1, 36, device=DEV).view(1, 36, 1, 1)).sum().backward()
        res.append((a.grad, b.grad))
    for x, y in zip(res[1], res[0]):
        assert float((x - y).norm() / y.norm()) < 1e-6

