"""RC_OUT_CHANNELS_LAST (ABI v5): the pair kernel can write the lookup output
in NHWC memory order (torch.channels_last).  Same shape, same values bit for
bit; only the strides differ (CorrBlock1D(channels_last=True))."""
import pytest
import torch

from raft_stereo_amd import CorrBlock1D

from test_corr_gpu import CHAIN_SHAPES, BF16_PAIR_SHAPES, special_coords

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def cases():
    f32 = [(s, torch.float32) for s in CHAIN_SHAPES]
    b16 = [(s, torch.bfloat16) for s in BF16_PAIR_SHAPES]
    return f32 + b16


def ids(p):
    s, dt = p
    return "x".join(map(str, s)) + ("-bf16" if dt == torch.bfloat16 else "-f32")


@pytest.mark.parametrize("case", cases(), ids=ids)
def test_channels_last_bit_identical(case):
    """NaN/inf/subnormal coords, tails (P % 64 != 0), C = 18 (not a multiple
    of 4), 3-level blocks (not the pair kernel: converted after the lookup)."""
    (B, D, H, W1, W2, L, r), dt = case
    g = torch.Generator().manual_seed(1700 + B * H + W1 + W2)
    f1 = torch.randn(B, D, H, W1, generator=g).to(DEV)
    f2 = torch.randn(B, D, H, W2, generator=g).to(DEV)
    coords = special_coords(B, H, W1, W2, g).to(DEV)
    with torch.no_grad():
        ref = CorrBlock1D(f1, f2, num_levels=L, radius=r, pyramid_dtype=dt)
        cl = CorrBlock1D(f1, f2, num_levels=L, radius=r, pyramid_dtype=dt, channels_last=True)
        a, b = cl(coords), ref(coords)
        assert a.shape == b.shape and a.is_contiguous(memory_format=torch.channels_last)
        assert torch.equal(a.view(torch.int32), b.view(torch.int32))
        d = torch.randn(coords.shape, generator=g).to(DEV)
        x, y = cl.lookup_step(coords.clone(), d), ref.lookup_step(coords.clone(), d)
        assert x[0].is_contiguous(memory_format=torch.channels_last)
        for u, v in zip(x, y):
            assert torch.equal(u.view(torch.int32), v.view(torch.int32))


def test_channels_last_fullsize_and_network():
    """Config-3 shape at B=8 (bf16): every pixel; and the network with a
    channels-last corr block gives the same disparities bit for bit."""
    B, D, H, W = 8, 256, 94, 311
    g = torch.Generator().manual_seed(9)
    f1 = torch.randn(B, D, H, W, generator=g).to(DEV, torch.bfloat16)
    f2 = torch.randn(B, D, H, W, generator=g).to(DEV, torch.bfloat16)
    x = torch.arange(W).float().view(1, 1, 1, W) - torch.rand(B, 1, H, W, generator=g) * 64
    coords = torch.cat([x, torch.zeros_like(x)], 1).to(DEV)
    with torch.no_grad():
        a = CorrBlock1D(f1, f2, channels_last=True)(coords)
        b = CorrBlock1D(f1, f2)(coords)
    assert torch.equal(a.view(torch.int32), b.view(torch.int32))


def test_network_with_channels_last_corr():
    """RAFTStereo with a channels-last corr block (convc1 consumes either
    layout) still matches the reference's golden disparity (MAE <= 0.01 px)."""
    import functools

    import numpy as np
    from golden_util import GOLDEN, load, manifest
    from raft_stereo_amd.network import RAFTStereo, StereoArgs
    case = manifest()["cases"]["e2e_default"]
    z = load(f"{GOLDEN}/e2e_default.npz")
    torch.manual_seed(0)
    model = RAFTStereo(StereoArgs(**case["args"]),
                       corr_block=functools.partial(CorrBlock1D, channels_last=True)).eval().cuda()
    with torch.no_grad():
        flows = model(torch.from_numpy(z["image1"]).cuda(), torch.from_numpy(z["image2"]).cuda(),
                      iters=int(z["iters"]))
    disp = np.stack([f[:, 0].cpu().numpy() for f in flows], 0)
    mae = np.abs(disp - z["disparity"]).mean(axis=(1, 2, 3))
    assert (mae <= 0.01).all(), f"per-iteration MAE {mae}"
