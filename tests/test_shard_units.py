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


def test_interp_index_cache_is_the_mapping():
    x = torch.randn(1, 3, 7, 5)
    a = shard._interp_rows(x, 10, 40, 21, 33, 80, 10)
    shard._INTERP.clear()
    b = shard._interp_rows(x, 10, 40, 21, 33, 80, 10)
    assert torch.equal(a, b)
    assert len(shard._INTERP) == 1
