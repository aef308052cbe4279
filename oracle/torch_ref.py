"""The reference's ATen op sequence, restated on CPU (TEST INFRASTRUCTURE ONLY).

This is the CPU baseline that bench.py times on the GPU box's host
(``cpu_baseline.kind == "port"``): the reference source cannot travel there,
so this module restates /root/reference/model.py:267-326 op for op, with the
SURVEY.md Appendix-A fixes D2/D3 (``.contiguous()``, ``.float()``).  It keeps
the reference's costs, including the per-level ``torch.unique`` assert
(model.py:272).  tests/test_oracle_golden.py pins it to the goldens.
"""
import torch
import torch.nn.functional as F


def sample_1d(img, coords):
    """model.py:267-281 (mask=False branch): grid_sample with pixel coords."""
    H, W = img.shape[-2:]
    xgrid, ygrid = coords.split([1, 1], dim=-1)
    xgrid = 2 * xgrid / (W - 1) - 1
    assert torch.unique(ygrid).numel() == 1 and H == 1
    grid = torch.cat([xgrid, ygrid], dim=-1)
    return F.grid_sample(img, grid, align_corners=True)


def volume(fmap1, fmap2):
    """model.py:318-326: per-row all-pairs correlation / sqrt(D)."""
    B, D, H, W1 = fmap1.shape
    W2 = fmap2.shape[3]
    c = torch.einsum('aijk,aijh->ajkh', fmap1.view(B, D, H, W1), fmap2.view(B, D, H, W2))
    c = c.reshape(B, H, W1, 1, W2).contiguous()
    return c / torch.sqrt(torch.tensor(D).float())


class TorchCorrBlock1D:
    """model.py:283-316, restated."""

    def __init__(self, fmap1, fmap2, num_levels=4, radius=4):
        self.num_levels = num_levels
        self.radius = radius
        c = volume(fmap1, fmap2)
        b, h1, w1, dim, w2 = c.shape
        c = c.reshape(b * h1 * w1, dim, 1, w2)
        self.corr_pyramid = [c]
        for _ in range(num_levels):
            c = F.avg_pool2d(c, [1, 2], stride=[1, 2])
            self.corr_pyramid.append(c)

    def __call__(self, coords):
        r = self.radius
        coords = coords[:, :1].permute(0, 2, 3, 1)
        b, h1, w1, _ = coords.shape
        outs = []
        for i in range(self.num_levels):
            dx = torch.linspace(-r, r, 2 * r + 1).view(1, 1, 2 * r + 1, 1).to(coords.device)
            x0 = dx + coords.reshape(b * h1 * w1, 1, 1, 1) / 2 ** i
            grid = torch.cat([x0, torch.zeros_like(x0)], dim=-1)
            outs.append(sample_1d(self.corr_pyramid[i], grid).view(b, h1, w1, -1))
        return torch.cat(outs, dim=-1).permute(0, 3, 1, 2).contiguous().float()


def convex_upsample(flow, mask, factor):
    """RAFT-Stereo's convex upsampler for the mask of model.py:238-241/:264
    (absent from the reference's forward): softmax over the 9 neighbours,
    weighted sum of factor * flow over the 3x3 neighbourhood (F.unfold order).
    Parity of this restatement is unpinned by the reference (no upsampler
    there); tests/test_upsample.py checks it against an explicit loop."""
    N, C, H, W = flow.shape
    m = torch.softmax(mask.view(N, 1, 9, factor, factor, H, W), dim=2)
    up = F.unfold(factor * flow, [3, 3], padding=1).view(N, C, 9, 1, 1, H, W)
    up = torch.sum(m * up, dim=2)                       # N, C, f, f, H, W
    return up.permute(0, 1, 4, 2, 5, 3).reshape(N, C, factor * H, factor * W)
