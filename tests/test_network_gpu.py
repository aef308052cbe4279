"""End-to-end parity on the GPU: the host network with the HIP correlation
path vs the reference's per-iteration disparity (goldens from the patched
reference on CPU).  north_star bar: final disparity MAE <= 0.01 px; we check
every iteration against it."""
import numpy as np
import pytest
import torch

from golden_util import GOLDEN, load, manifest
from raft_stereo_amd import CorrBlock1D
from raft_stereo_amd.network import RAFTStereo, StereoArgs

pytestmark = pytest.mark.gpu
CASES = {k: v for k, v in manifest()["cases"].items() if v["kind"] == "e2e"}
MAE_PX = 0.01


@pytest.mark.parametrize("name", sorted(CASES))
def test_disparity_matches_reference(name):
    case = CASES[name]
    z = load(f"{GOLDEN}/e2e_{name.split('_', 1)[1]}.npz")
    torch.manual_seed(0)
    model = RAFTStereo(StereoArgs(**case["args"])).eval()
    assert model.corr_block is CorrBlock1D
    model = model.cuda()
    with torch.no_grad():
        flows = model(torch.from_numpy(z["image1"]).cuda(), torch.from_numpy(z["image2"]).cuda(),
                      iters=int(z["iters"]))
    disp = np.stack([f[:, 0].cpu().numpy() for f in flows], 0)
    mae = np.abs(disp - z["disparity"]).mean(axis=(1, 2, 3))
    assert (mae <= MAE_PX).all(), f"per-iteration MAE {mae}"
    print(f"{name}: final MAE {mae[-1]:.2e} px, max |d| {np.abs(disp - z['disparity']).max():.2e}")


def test_bf16_corr_path_disparity_bound():
    """The bf16 corr path alone (fmaps rounded to bf16, bf16 MFMA volume, bf16
    pyramid; the rest of the network fp32) against the reference's fp32
    golden: final-disparity MAE within north_star's 0.01 px bar at every
    iteration (SURVEY §8d probe: 4.5e-4 px after 32 iterations)."""
    import functools
    case = CASES["e2e_default"]
    z = load(f"{GOLDEN}/e2e_default.npz")
    torch.manual_seed(0)
    model = RAFTStereo(StereoArgs(**case["args"]),
                       corr_block=functools.partial(CorrBlock1D, pyramid_dtype=torch.bfloat16))
    model = model.eval().cuda()
    with torch.no_grad():
        flows = model(torch.from_numpy(z["image1"]).cuda(), torch.from_numpy(z["image2"]).cuda(),
                      iters=int(z["iters"]))
    disp = np.stack([f[:, 0].cpu().numpy() for f in flows], 0)
    mae = np.abs(disp - z["disparity"]).mean(axis=(1, 2, 3))
    assert (mae <= MAE_PX).all(), f"per-iteration MAE {mae}"
    print(f"bf16 corr path: final MAE {mae[-1]:.2e} px")


def test_bf16_autocast_runs():
    """Whole-network mixed precision (every conv in bf16 too, not just the
    corr path): the reference crashes here; we accept the
    half-precision fmaps and stay within a loose bound of the fp32 result --
    the convolutions' bf16 rounding, not the corr path, sets this error (the
    corr path's own bf16 bound is test_bf16_corr_path_disparity_bound)."""
    case = CASES["e2e_default"]
    z = load(f"{GOLDEN}/e2e_default.npz")
    torch.manual_seed(0)
    args = StereoArgs(**case["args"])
    args.mixed_precision = True
    args.autocast_dtype = torch.bfloat16
    model = RAFTStereo(args).eval().cuda()
    with torch.no_grad():
        flows = model(torch.from_numpy(z["image1"]).cuda(), torch.from_numpy(z["image2"]).cuda(),
                      iters=int(z["iters"]))
    disp = flows[-1][:, 0].float().cpu().numpy()
    assert np.isfinite(disp).all()
    assert np.abs(disp - z["disparity"][-1]).mean() < 0.5


@pytest.mark.parametrize("name", sorted(CASES))
def test_disparity_with_fused_convc1(name):
    """The network with the lookup+convc1 fusion stays
    within the north_star bar of the reference."""
    case = CASES[name]
    z = load(f"{GOLDEN}/e2e_{name.split('_', 1)[1]}.npz")
    torch.manual_seed(0)
    model = RAFTStereo(StereoArgs(**case["args"]), fuse_convc1=True).eval().cuda()
    with torch.no_grad():
        flows = model(torch.from_numpy(z["image1"]).cuda(), torch.from_numpy(z["image2"]).cuda(),
                      iters=int(z["iters"]))
    disp = np.stack([f[:, 0].cpu().numpy() for f in flows], 0)
    mae = np.abs(disp - z["disparity"]).mean(axis=(1, 2, 3))
    assert (mae <= MAE_PX).all(), f"per-iteration MAE {mae}"


@pytest.mark.parametrize("name", sorted(CASES))
def test_disparity_with_fused_step(name):
    """The network with the coords update + flow fused into the lookup launch
     vs the unfused network.  The fused ops are bitwise
    identical (test_lookup_step_matches_unfused); the encoders/GRU convs
    (MIOpen) need not be run-to-run deterministic, so the whole-network
    comparison allows the spread of two unfused runs (and at least 1e-4 px)."""
    case = CASES[name]
    z = load(f"{GOLDEN}/e2e_{name.split('_', 1)[1]}.npz")
    img1, img2 = torch.from_numpy(z["image1"]).cuda(), torch.from_numpy(z["image2"]).cuda()
    outs = []
    for fuse in (False, False, True):
        torch.manual_seed(0)
        model = RAFTStereo(StereoArgs(**case["args"]), fuse_step=fuse).eval().cuda()
        with torch.no_grad():
            outs.append(torch.stack([f.cpu() for f in model(img1, img2, iters=int(z["iters"]))]))
    assert outs[0].shape == outs[2].shape and outs[0].shape[0] == int(z["iters"])
    noise = (outs[0] - outs[1]).abs().max().item()
    diff = (outs[2] - outs[0]).abs().max().item()
    assert diff <= max(1e-4, 10 * noise), (diff, noise)
    disp = outs[2][:, :, 0].numpy()
    mae = np.abs(disp - z["disparity"]).mean(axis=(1, 2, 3))
    assert (mae <= MAE_PX).all(), f"per-iteration MAE {mae}"


SEEDED = {k: v for k, v in manifest()["cases"].items() if v["kind"] == "e2e_seeded"}


@pytest.mark.parametrize("fuse", ["none", "step", "convc1"])
@pytest.mark.parametrize("name", sorted(SEEDED))
def test_seeded_disparity_matches_reference(name, fuse):
    """The BASELINE image sizes, one pair each, default args, seeded weights
    (hash checked): configs[0] (320x720, 12 iterations), configs[1]
    (540x960, 32), configs[2]'s image (375x1242, 32) and configs[3]
    (1984x2880, 32) -- the HIP corr path inside the network vs the
    reference's final disparity (model.py:354-383 + the D8 tail), MAE bar
    0.01 px.  Images are regenerated from the seed and their sha256 checked."""
    from golden_util import image_digest, stereo_pair
    case = SEEDED[name]
    z = load(f"{GOLDEN}/e2e_{name.split('_', 1)[1]}.npz")
    img1, img2 = stereo_pair(1, case["H"], case["W"], case["seed"])
    assert image_digest(img1, img2) == case["image_sha256"]
    torch.manual_seed(0)
    model = RAFTStereo(StereoArgs(**case["args"]), fuse_step=fuse == "step",
                       fuse_convc1=fuse == "convc1").eval()
    assert model.corr_block is CorrBlock1D
    model = model.cuda()
    with torch.no_grad():
        flows = model(img1.cuda(), img2.cuda(), iters=case["iters"])
    disp = flows[-1][:, 0].cpu().numpy()
    assert disp.shape == z["disparity"].shape
    mae = float(np.abs(disp - z["disparity"]).mean())
    print(f"{name} [{fuse}]: final MAE {mae:.2e} px, max {np.abs(disp - z['disparity']).max():.2e}")
    assert mae <= MAE_PX, mae


@pytest.mark.parametrize("name", [n for n in sorted(SEEDED) if SEEDED[n]["W"] == 720])
def test_config1_disparity_layout_network(name):
    """CorrBlock1D(layout="disparity") as the network's corr block (the
    RC_LAYOUT_DISPARITY option), on BASELINE configs[0]: at
    every iteration its lookup equals the row layout's bit for bit on the
    network's own coordinates (both blocks built from the same fmaps), its
    corr_pyramid equals the row layout's, and the final disparity meets the
    reference golden's 0.01 px bar.  (Two separate network runs are not
    compared bitwise: MIOpen may pick different convolution algorithms.)"""
    from golden_util import image_digest, stereo_pair
    case = SEEDED[name]
    z = load(f"{GOLDEN}/e2e_{name.split('_', 1)[1]}.npz")
    img1, img2 = stereo_pair(1, case["H"], case["W"], case["seed"])
    assert image_digest(img1, img2) == case["image_sha256"]
    calls = []

    class Checked:
        def __init__(self, f1, f2, radius, num_levels):
            self.d = CorrBlock1D(f1, f2, radius=radius, num_levels=num_levels, layout="disparity")
            self.r = CorrBlock1D(f1, f2, radius=radius, num_levels=num_levels)
            assert self.d.layout == "disparity"
            for a, b in zip(self.d.corr_pyramid, self.r.corr_pyramid):
                assert torch.equal(a.contiguous().view(torch.int32), b.contiguous().view(torch.int32))

        def __call__(self, coords):
            out = self.d(coords)
            assert torch.equal(out.view(torch.int32), self.r(coords).view(torch.int32))
            calls.append(1)
            return out

    torch.manual_seed(0)
    model = RAFTStereo(StereoArgs(**case["args"]), corr_block=Checked).eval().cuda()
    with torch.no_grad():
        flows = model(img1.cuda(), img2.cuda(), iters=case["iters"])
    assert len(calls) == case["iters"]
    disp = flows[-1][:, 0].cpu().numpy()
    mae = float(np.abs(disp - z["disparity"]).mean())
    assert mae <= MAE_PX, mae


@pytest.mark.parametrize("name", [n for n in sorted(SEEDED) if SEEDED[n]["W"] == 1242])
def test_config3_bf16_corr_path_disparity(name):
    """BASELINE configs[2]'s image size (one 1x3x375x1242 pair, 32 iterations,
    default args, seeded weights): the network with the bf16 corr path
    (fmaps rounded to bf16, bf16 MFMA volume, bf16 pyramid -- what config 3
    runs) against the fp32 reference's final disparity, north_star's 0.01 px
    MAE bar (model.py:354-383 + the D8 tail; VERDICT r2 missing item 4)."""
    import functools
    from golden_util import image_digest, stereo_pair
    case = SEEDED[name]
    z = load(f"{GOLDEN}/e2e_{name.split('_', 1)[1]}.npz")
    img1, img2 = stereo_pair(1, case["H"], case["W"], case["seed"])
    assert image_digest(img1, img2) == case["image_sha256"]
    torch.manual_seed(0)
    model = RAFTStereo(StereoArgs(**case["args"]),
                       corr_block=functools.partial(CorrBlock1D, pyramid_dtype=torch.bfloat16))
    model = model.eval().cuda()
    with torch.no_grad():
        flows = model(img1.cuda(), img2.cuda(), iters=case["iters"])
    disp = flows[-1][:, 0].cpu().numpy()
    mae = float(np.abs(disp - z["disparity"]).mean())
    print(f"{name} bf16 corr path: final MAE {mae:.2e} px, max {np.abs(disp - z['disparity']).max():.2e}")
    assert mae <= MAE_PX, mae
