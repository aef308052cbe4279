"""Convex upsampler.

The reference builds the upsampling mask (model.py:238-241, :264) but its
truncated forward never applies it, so there is no reference output to pin:
the oracle is oracle/torch_ref.convex_upsample (RAFT-Stereo's F.unfold +
softmax formulation), itself checked here against an explicit per-pixel loop
of the formula ("parity unpinned" by the reference).
Tolerance for the HIP kernel: max|d|/max|ref| <= 1e-5 (expf and summation
order differ from torch's softmax)."""
import numpy as np
import pytest
import torch

from golden_util import norm_err
from oracle import torch_ref


def loop_upsample(flow, mask, f):
    N, C, H, W = flow.shape
    out = np.zeros((N, C, f * H, f * W), np.float64)
    fl = np.pad(flow.astype(np.float64), ((0, 0), (0, 0), (1, 1), (1, 1)))
    m = mask.astype(np.float64).reshape(N, 9, f, f, H, W)
    for n in range(N):
        for h in range(H):
            for w in range(W):
                for i in range(f):
                    for j in range(f):
                        e = np.exp(m[n, :, i, j, h, w] - m[n, :, i, j, h, w].max())
                        wgt = e / e.sum()
                        for c in range(C):
                            nb = fl[n, c, h:h + 3, w:w + 3].reshape(9)
                            out[n, c, f * h + i, f * w + j] = (wgt * f * nb).sum()
    return out


@pytest.mark.parametrize("shape", [(1, 2, 3, 4, 2), (2, 1, 4, 3, 4)], ids=str)
def test_restatement_matches_formula(shape):
    N, C, H, W, f = shape
    g = torch.Generator().manual_seed(sum(shape))
    flow = torch.randn(N, C, H, W, generator=g) * 3
    mask = torch.randn(N, 9 * f * f, H, W, generator=g) * 2
    got = torch_ref.convex_upsample(flow, mask, f).double().numpy()
    assert norm_err(got, loop_upsample(flow.numpy(), mask.numpy(), f)) <= 1e-6


SHAPES = [(2, 2, 7, 9, 4), (1, 1, 16, 20, 2), (1, 2, 5, 5, 8), (3, 1, 10, 13, 1),
          (8, 1, 135, 240, 4)]


@pytest.mark.gpu
@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_hip_vs_restatement(shape):
    from raft_stereo_amd.upsample import convex_upsample
    N, C, H, W, f = shape
    g = torch.Generator().manual_seed(3 + sum(shape))
    flow = torch.randn(N, C, H, W, generator=g) * 5
    mask = torch.randn(N, 9 * f * f, H, W, generator=g) * 2
    got = convex_upsample(flow.cuda(), mask.cuda(), f).cpu()
    ref = torch_ref.convex_upsample(flow, mask, f)
    assert got.shape == ref.shape
    assert norm_err(got.numpy(), ref.numpy()) <= 1e-5


@pytest.mark.gpu
def test_network_full_resolution_output():
    """RAFTStereo(..., upsample=True): every prediction is the full-resolution
    x-flow, a convex combination of f x the low-resolution flow around it."""
    from raft_stereo_amd.network import RAFTStereo, StereoArgs
    torch.manual_seed(0)
    model = RAFTStereo(StereoArgs()).eval().cuda()
    g = torch.Generator().manual_seed(8)
    img1 = (torch.rand(1, 3, 64, 96, generator=g) * 255).cuda()
    img2 = torch.roll(img1, -4, dims=-1)
    with torch.no_grad():
        low = model(img1, img2, iters=3)
        up = model(img1, img2, iters=3, upsample=True)
    assert len(up) == 3 and up[-1].shape == (1, 1, 64, 96)
    assert torch.isfinite(up[-1]).all()
    f = 4
    lo = low[-1][:, :1]
    pad = torch.nn.functional.pad(lo, (1, 1, 1, 1))
    nb = torch.nn.functional.unfold(pad, 3).view(1, 9, 16, 24) * f
    hi_max = nb.max(1).values.repeat_interleave(f, 1).repeat_interleave(f, 2)
    hi_min = nb.min(1).values.repeat_interleave(f, 1).repeat_interleave(f, 2)
    # allow the MIOpen run-to-run spread between the two forward passes
    assert (up[-1][0, 0] <= hi_max[0] + 1e-3).all() and (up[-1][0, 0] >= hi_min[0] - 1e-3).all()
