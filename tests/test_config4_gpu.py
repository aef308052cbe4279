"""BASELINE configs[3] end to end against the reference: one 1x3x1984x2880
pair, 32 iterations, default args, seeded weights -- through the code the
config-4 1/2/4/8-GPU bench times (``shard.RowShardedStereo`` with its product
defaults: per-conv halos, the two-stream pipeline, stacked z/r convs).

Golden: tests/golden/e2e_config4.npz, the patched reference's final disparity
on CPU (make_golden.py, model.py:354-383 + the D8 tail).  Bar: north_star's
0.01 px MAE.  (The plain RAFTStereo at this size is covered by
test_network_gpu.test_seeded_disparity_matches_reference[e2e_config4-*].)"""
import numpy as np
import pytest
import torch

import dist_worker
from golden_util import GOLDEN, load
from test_shard_dist import _spawn

pytestmark = pytest.mark.gpu
MAE_PX = 0.01


def _golden():
    z = load(f"{GOLDEN}/e2e_config4.npz")
    assert int(z["iters"]) == 32
    return z["disparity"]


def test_config4_row_sharded_world1_matches_reference():
    from raft_stereo_amd.shard import RowShardedStereo
    want = _golden()
    net = dist_worker.gpu_model()
    img1, img2, case = dist_worker.seeded_images("e2e_config4")
    with torch.no_grad():
        rs = RowShardedStereo(net, 0, 1)
        assert rs.per_conv and rs.side_stream and rs.fuse_zr
        preds = rs.forward(img1.cuda(), img2.cuda(), iters=case["iters"])
        disp = rs.gather_rows(preds[-1])[:, 0].cpu().numpy()
    assert disp.shape == want.shape == (1, 496, 720)
    err = np.abs(disp - want)
    print(f"config4 RowShardedStereo world 1: MAE {err.mean():.2e} px, max {err.max():.2e}")
    assert err.mean() <= MAE_PX, err.mean()


def test_config4_row_sharded_world2_shared_gpu_matches_reference():
    """Two ranks on cuda:0 over gloo: the same halo exchanges (host-staged)
    the RCCL ranks of an 8-GPU node post, at config 4's real row geometry."""
    want = _golden()
    res = _spawn(dist_worker.run_gpu_config4, 2)
    disp = res[0][0].numpy()
    assert disp.shape == want.shape
    err = np.abs(disp - want)
    print(f"config4 RowShardedStereo world 2 (gloo, shared GPU): MAE {err.mean():.2e} px, "
          f"max {err.max():.2e}")
    assert err.mean() <= MAE_PX, err.mean()
