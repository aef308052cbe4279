"""The oracle is pinned against goldens generated from the reference itself
(tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest
import torch

from golden_util import files, load, manifest, norm_err, rel_l2, same
from oracle import coracle, torch_ref

VOL = files("volume")
LUT = files("lookup")


def test_manifest_covers_cases():
    m = manifest()
    assert len(m["reference_sha256"]) == 64
    assert len(VOL) >= 5 and len(LUT) >= 7
    assert m["cases"]["l_special"]["nan_out"] > 0


@pytest.mark.parametrize("path", VOL, ids=lambda p: p.split("/")[-1])
def test_c_oracle_volume(path):
    z = load(path)
    L = int(z["num_levels"])
    pyr = coracle.corr_pyramid(z["fmap1"], z["fmap2"], L)
    assert norm_err(pyr[0], z["level0"]) <= 1e-6
    assert rel_l2(pyr[0], z["level0"]) <= 1e-6
    for i in range(L):
        # pooling is bit-exact given identical input (model.py:294)
        assert same(coracle.corr_pool(z[f"level{i}"]), z[f"level{i + 1}"])
        assert pyr[i + 1].shape == z[f"level{i + 1}"].shape


@pytest.mark.parametrize("path", LUT, ids=lambda p: p.split("/")[-1])
def test_c_oracle_lookup_bitexact(path):
    z = load(path)
    L, r = int(z["num_levels"]), int(z["radius"])
    out = coracle.corr_lookup([z[f"level{i}"] for i in range(L)], z["coords"], L, r)
    assert out.shape == z["out"].shape
    assert same(out, z["out"])


@pytest.mark.parametrize("path", VOL[:2] + LUT, ids=lambda p: p.split("/")[-1])
def test_torch_ref_matches_golden(path):
    z = load(path)
    L = int(z["num_levels"])
    r = int(z["radius"]) if "radius" in z else 4
    blk = torch_ref.TorchCorrBlock1D(torch.from_numpy(z["fmap1"]), torch.from_numpy(z["fmap2"]), L, r)
    for i in range(L):
        got = blk.corr_pyramid[i].reshape(z[f"level{i}"].shape).numpy()
        assert same(got, z[f"level{i}"])
    if "coords" in z:
        assert same(blk(torch.from_numpy(z["coords"])).numpy(), z["out"])


def test_reference_error_narrow_w2():
    """The reference raises when W2 < 2**num_levels (avg_pool2d, model.py:294)."""
    f = torch.randn(1, 4, 1, 3)
    g = torch.randn(1, 4, 1, 9)
    with pytest.raises(RuntimeError):
        torch_ref.TorchCorrBlock1D(f, g, 4, 2)
