"""Host-side behaviour of the drop-in CorrBlock1D that needs no GPU: the
product path refuses CPU tensors (no silent fallback) and mirrors the
reference's argument errors."""
import pytest
import torch

from raft_stereo_amd import CorrBlock1D, coords_grid


def test_cpu_tensors_fail_loudly():
    f = torch.randn(1, 8, 2, 16)
    with pytest.raises(RuntimeError, match="HIP"):
        CorrBlock1D(f, f, num_levels=2, radius=2)
    with pytest.raises(RuntimeError, match="HIP"):
        CorrBlock1D.corr(f, f)


def test_coords_grid_matches_reference_layout():
    """model.py:329-332: channel 0 is x (w index), channel 1 is y (h index)."""
    g = coords_grid(2, 3, 5)
    assert g.shape == (2, 2, 3, 5) and g.dtype == torch.float32
    assert torch.equal(g[1, 0, 2], torch.arange(5).float())
    assert torch.equal(g[0, 1, :, 4], torch.arange(3).float())


def test_request_validation_before_any_launch():
    """invalid ``grad_shadow`` requests raise at construction (not
    later inside autograd), a ``per_stage=False`` halo below the one-iteration
    cone raises, and the default halo follows the exchange mode."""
    from raft_stereo_amd import corr as rcorr
    from raft_stereo_amd.shard import RowShardedStereo
    with pytest.raises(ValueError):
        rcorr._check_grad_shadow((1,), 4, 4, 240)
    with pytest.raises(ValueError):
        rcorr._check_grad_shadow((0,), 3, 4, 240)        # 3 levels: no pair gradient layout
    with pytest.raises(ValueError):
        rcorr._check_grad_shadow((0, 2), 4, 5, 240)      # radius 5: per-level layout
    rcorr._check_grad_shadow((0, 2), 4, 4, 240)
    rcorr._check_grad_shadow((), 3, 4, 240)
    with pytest.raises(ValueError):
        RowShardedStereo(None, 0, 2, halo=12, per_stage=False)
    assert RowShardedStereo(None, 0, 2).halo == 12
    assert RowShardedStereo(None, 0, 2, per_stage=False).halo == 24
