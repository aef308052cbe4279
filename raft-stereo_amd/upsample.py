"""Convex upsampler on the gfx950 kernel.

The reference's update block produces the mask (model.py:238-241, 0.25-scaled
at :264; f = 2**n_downsample at :236) but its truncated forward never uses it
(SURVEY Appendix A D8).  ``convex_upsample`` applies it the way RAFT-Stereo
does: softmax over the 9 neighbours for every sub-pixel, weighted sum of
f * flow over the low-resolution 3x3 neighbourhood (rc_convex_upsample,
include/raftcorr.h).  No CPU fallback: HIP tensors only.
"""
import torch

from . import _lib
from .corr import _require_hip, _stream


def convex_upsample(flow, mask, factor):
    """flow (N, C, H, W), mask (N, 9*factor**2, H, W) -> (N, C, factor*H, factor*W)
    fp32.  Inputs of other float dtypes are computed in fp32."""
    _require_hip(flow, "flow")
    _require_hip(mask, "mask")
    if torch.is_grad_enabled() and (flow.requires_grad or mask.requires_grad):
        raise RuntimeError("convex_upsample is inference-only (rc_convex_upsample has no "
                           "backward); call it under torch.no_grad()")
    if flow.device != mask.device:
        raise RuntimeError("convex_upsample: flow and mask on different devices")
    if flow.dim() != 4 or mask.dim() != 4:
        raise RuntimeError("convex_upsample: flow and mask must be 4-D")
    N, C, H, W = flow.shape
    if tuple(mask.shape) != (N, 9 * factor * factor, H, W):
        raise RuntimeError(f"convex_upsample: mask {tuple(mask.shape)} != "
                           f"{(N, 9 * factor * factor, H, W)}")
    f = flow.detach().float().contiguous()
    m = mask.detach().float().contiguous()
    out = torch.empty((N, C, factor * H, factor * W), dtype=torch.float32, device=f.device)
    if N * H * W == 0:
        return out
    with torch.cuda.device(f.device):
        rc = _lib.lib().rc_convex_upsample(f.data_ptr(), m.data_ptr(), N, C, H, W, factor,
                                           out.data_ptr(), _stream(f.device))
    _lib.check(rc, "rc_convex_upsample")
    return out
