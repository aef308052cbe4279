"""Unit checks of shard.py's per-conv helpers (CPU): the stacked z/r
convolution equals the two separate convolutions and follows in-place
weight updates; the cached interp row mapping equals a fresh one."""
import torch

import pkgload

pkgload.load()
from raft_stereo_amd import shard  # noqa: E402
from raft_stereo_amd.network import ConvGRU  # noqa: E402


def test_stacked_zr_conv_matches_and_tracks_weights():
    torch.manual_seed(0)
    gru = ConvGRU(16, 24).eval()
    x = torch.randn(1, 40, 9, 11)
    w, b, C = shard._zr_conv(gru)
    assert C == 16
    both = torch.nn.functional.conv2d(x, w, b, padding=gru.convz.padding)
    assert torch.allclose(both[:, :C], gru.convz(x), atol=1e-6)
    assert torch.allclose(both[:, C:], gru.convr(x), atol=1e-6)
    with torch.no_grad():                       # in place, as load_state_dict does
        gru.convr.weight.mul_(2.0)
    w2, b2, _ = shard._zr_conv(gru)
    assert torch.equal(w2[C:], gru.convr.weight) and torch.equal(w2[:C], gru.convz.weight)
    assert not torch.equal(w2[C:], w[C:])


def test_stacked_zr_conv_follows_dtype_and_grad_mode():
    """``.double()`` / ``.to()`` keep the Parameter objects, so the
    cache must see the new dtype; an entry built under no_grad must not be
    reused when gradients are recorded (convz/convr would get none)."""
    torch.manual_seed(0)
    gru = ConvGRU(8, 12).eval()
    with torch.no_grad():
        w, _, C = shard._zr_conv(gru)
    assert w.dtype == torch.float32 and not w.requires_grad
    gru.double()
    with torch.no_grad():
        w64, b64, _ = shard._zr_conv(gru)
    assert w64.dtype == torch.float64 and b64.dtype == torch.float64
    x = torch.randn(1, 20, 5, 6, dtype=torch.float64)
    y = torch.nn.functional.conv2d(x, w64, b64, padding=gru.convz.padding)   # no dtype error
    assert torch.allclose(y[:, :C], gru.convz(x), atol=1e-12)
    # grad mode: the stacked weights carry the graph to convz / convr
    wg, bg, _ = shard._zr_conv(gru)
    assert wg.requires_grad
    torch.nn.functional.conv2d(x, wg, bg, padding=gru.convz.padding).sum().backward()
    assert gru.convz.weight.grad is not None and gru.convr.weight.grad is not None
    # and twice (a cached graph could not be back-propagated a second time)
    wg2, bg2, _ = shard._zr_conv(gru)
    torch.nn.functional.conv2d(x, wg2, bg2, padding=gru.convz.padding).sum().backward()


def test_interp_index_cache_is_the_mapping():
    x = torch.randn(1, 3, 7, 5)
    a = shard._interp_rows(x, 10, 40, 21, 33, 80, 10)
    shard._INTERP.clear()
    b = shard._interp_rows(x, 10, 40, 21, 33, 80, 10)
    assert torch.equal(a, b)
    assert len(shard._INTERP) == 1
