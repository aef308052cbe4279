"""Drop-in ``CorrBlock1D`` over the gfx950 kernels in ``csrc/``.

Mirrors the reference's correlation class (/root/reference/model.py:283-326)
so that ``RAFTStereo.forward`` can bind it where the reference does
(model.py:366-367 construct, :376 call):

  * ``CorrBlock1D(fmap1, fmap2, num_levels=4, radius=4)``  (model.py:284)
      builds the all-pairs per-row volume / sqrt(D) and its avg-pooled
      pyramid in ONE kernel launch (rc_corr_build).  ``corr_pyramid`` holds
      num_levels+1 tensors of shape (B*H*W1, 1, 1, W2 >> l) like the reference
      (:290-295; the last one is never read, as in the reference).  Rows whose
      width is not a 16-byte multiple are views into row-padded buffers
      (same shape and values, a larger row stride).
  * ``__call__(coords)``  (model.py:297-316)  one rc_corr_lookup launch:
      (B,2,H,W1) fp32 coords -> (B, num_levels*(2r+1), H, W1) fp32.
  * ``CorrBlock1D.corr(fmap1, fmap2)``  (model.py:318-326) -> (B,H,W1,1,W2).

Error behaviour follows the reference where it has one: W2 < 2**num_levels
raises RuntimeError (avg_pool2d, model.py:294); mismatched fmap shapes raise
RuntimeError (einsum, :324); coords that do not match the volume's
(B, H, W1) raise RuntimeError (view, :312); non-fp32 coords raise
RuntimeError (grid_sample dtype check, :275).

Differences, all loud: tensors must live on a HIP device (no CPU fallback);
the path is inference-only (asking for gradients raises); bf16/fp16 fmaps are
accepted (the reference crashes on them): they, or
an explicit ``pyramid_dtype=torch.bfloat16``, select the bf16 MFMA kernel and
a bf16 pyramid (bf16-level tolerance).
"""
import torch

from . import _lib


def _stream(device):
    return ctypes_void(torch.cuda.current_stream(device).cuda_stream)


def ctypes_void(v):
    return v if v else None


def _require_hip(t, what):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{what} must be a torch.Tensor")
    if t.device.type != "cuda":
        raise RuntimeError(
            f"raft_stereo_amd.CorrBlock1D: {what} is on {t.device}; the MI355X path "
            "runs on HIP devices only (no CPU fallback)")


def _dtype_code(dt):
    if dt == torch.float32:
        return _lib.RC_F32
    if dt == torch.bfloat16:
        return _lib.RC_BF16
    raise TypeError(f"raft_stereo_amd: unsupported dtype {dt} (float32 or bfloat16)")


def _check_fmaps(fmap1, fmap2):
    _require_hip(fmap1, "fmap1")
    _require_hip(fmap2, "fmap2")
    if fmap1.dim() != 4 or fmap2.dim() != 4:
        raise RuntimeError("CorrBlock1D: fmaps must be 4-D (B, D, H, W)")
    B, D, H, W1 = fmap1.shape
    B2, D2, H2, W2 = fmap2.shape
    if (B, D, H) != (B2, D2, H2):
        raise RuntimeError(
            f"CorrBlock1D: fmap1 {tuple(fmap1.shape)} and fmap2 {tuple(fmap2.shape)} "
            "disagree on (B, D, H) (einsum 'aijk,aijh->ajkh', model.py:324)")
    if fmap1.device != fmap2.device:
        raise RuntimeError("CorrBlock1D: fmaps on different devices")
    if torch.is_grad_enabled() and (fmap1.requires_grad or fmap2.requires_grad):
        raise RuntimeError(
            "raft_stereo_amd.CorrBlock1D is inference-only (backward is not "
            "implemented); call it under torch.no_grad() or detach the fmaps")
    return B, D, H, W1, W2


def _prep_fmap(f):
    # fp32 and bf16 go to the kernels as they are; fp16 (default autocast)
    # is widened to fp32 and then rounded to bf16 on load by the bf16 kernel.
    if f.dtype == torch.float16:
        f = f.float()
    elif f.dtype not in (torch.float32, torch.bfloat16):
        raise TypeError(f"raft_stereo_amd: unsupported fmap dtype {f.dtype}")
    return f.contiguous()


def _level_buffer(P, W, dtype, device, pad):
    """(P, 1, 1, W) tensor whose rows start 16-byte aligned: a view of a
    (P, ld) buffer with ld = W rounded up to 16 bytes when ``pad`` (the
    kernels then store whole aligned vectors; the padding is never read)."""
    per16 = 16 // torch.tensor([], dtype=dtype).element_size()
    ld = -(-W // per16) * per16 if pad else W
    buf = torch.empty((P, ld), dtype=dtype, device=device)
    if ld == W:
        return buf.view(P, 1, 1, W)
    return buf[:, :W].unsqueeze(1).unsqueeze(1)


def _row_stride(t):
    """Row stride (elements) of a (P, 1, 1, W) level; rows must be unit-stride."""
    if t.stride(-1) != 1:
        raise RuntimeError("raft_stereo_amd: pyramid rows must be contiguous")
    return t.stride(0) if t.shape[0] > 1 else t.shape[-1]


def build_pyramid(fmap1, fmap2, nbuf, pyramid_dtype=torch.float32, pad=True):
    """Run rc_corr_build: returns ``nbuf`` tensors (B*H*W1, 1, 1, W2 >> l)
    (row-padded views when ``pad``; values identical either way)."""
    B, D, H, W1, W2 = _check_fmaps(fmap1, fmap2)
    if (W2 >> (nbuf - 1)) < 1:
        raise RuntimeError(
            f"CorrBlock1D: W2={W2} is too narrow for {nbuf - 1} pooling steps: "
            "avg_pool2d output size is too small (model.py:294)")
    if nbuf > _lib.RC_MAX_LEVELS:
        raise RuntimeError(f"CorrBlock1D: at most {_lib.RC_MAX_LEVELS - 1} levels supported")
    f1, f2 = _prep_fmap(fmap1), _prep_fmap(fmap2)
    if f1.dtype != f2.dtype:
        f1, f2 = f1.float(), f2.float()
    P = B * H * W1
    pyr = [_level_buffer(P, W2 >> l, pyramid_dtype, f1.device, pad) for l in range(nbuf)]
    if P == 0:
        return pyr
    with torch.cuda.device(f1.device):
        rc = _lib.lib().rc_corr_build(
            f1.data_ptr(), f2.data_ptr(), _dtype_code(f1.dtype), B, D, H, W1, W2,
            _lib.ptr_array([t.data_ptr() for t in pyr]),
            _lib.long_array([_row_stride(t) for t in pyr]), nbuf,
            _dtype_code(pyramid_dtype), _stream(f1.device))
    _lib.check(rc, "rc_corr_build")
    return pyr


def _check_coords(pyramid, coords):
    _require_hip(coords, "coords")
    if coords.dim() != 4 or coords.shape[1] < 1:
        raise RuntimeError("CorrBlock1D: coords must be (B, 2, H, W1)")
    if coords.dtype != torch.float32:
        raise RuntimeError(
            f"CorrBlock1D: coords dtype {coords.dtype} != float32 (grid_sample "
            "requires the grid dtype to match the volume, model.py:275)")
    B, _, H, W1 = coords.shape
    if B * H * W1 != pyramid[0].shape[0]:
        raise RuntimeError(
            f"CorrBlock1D: coords {tuple(coords.shape)} do not match the volume's "
            f"{pyramid[0].shape[0]} rows (view at model.py:312)")
    if coords.device != pyramid[0].device:
        raise RuntimeError("CorrBlock1D: coords and pyramid on different devices")
    x = coords[:, 0]
    if x.stride(2) != 1 or x.stride(1) != W1:
        x = x.contiguous()
    cbs = x.stride(0) if B > 1 else H * W1
    return x, cbs


def _level_args(pyramid, num_levels):
    levels = [pyramid[i] for i in range(num_levels)]
    levels = [t if t.stride(-1) == 1 and t.data_ptr() % 16 == 0 else t.contiguous() for t in levels]
    return (levels, _lib.ptr_array([t.data_ptr() for t in levels]),
            _lib.int_array([t.shape[-1] for t in levels]),
            _lib.long_array([_row_stride(t) for t in levels]), _dtype_code(levels[0].dtype))


def lookup_convc1(pyramid, coords, num_levels, radius, weight, bias=None, relu=True):
    """Lookup fused with a 1x1 conv (+ReLU): relu(conv1x1(lookup(coords))),
    i.e. BasicMotionEncoder's ``F.relu(self.convc1(corr))`` (model.py:199, :206)."""
    x, cbs = _check_coords(pyramid, coords)
    B, _, H, W1 = coords.shape
    cin = num_levels * (2 * radius + 1)
    w = weight.detach().reshape(weight.shape[0], -1).float().contiguous()
    if w.shape[1] != cin:
        raise RuntimeError(f"lookup_convc1: weight has {w.shape[1]} input channels, lookup gives {cin}")
    b = bias.detach().float().contiguous() if bias is not None else None
    cout = w.shape[0]
    out = torch.empty((B, cout, H, W1), dtype=torch.float32, device=coords.device)
    if B * H * W1 == 0:
        return out
    keep, ptrs, widths, lds, dt = _level_args(pyramid, num_levels)
    with torch.cuda.device(coords.device):
        rc = _lib.lib().rc_corr_lookup_conv(
            ptrs, widths, lds, dt, num_levels, radius, x.data_ptr(), cbs, B, H, W1,
            w.data_ptr(), b.data_ptr() if b is not None else None, cout, int(relu),
            out.data_ptr(), _stream(coords.device))
    _lib.check(rc, "rc_corr_lookup_conv")
    return out


def lookup(pyramid, coords, num_levels, radius):
    """Run rc_corr_lookup on levels [0, num_levels) of ``pyramid``."""
    _require_hip(coords, "coords")
    if coords.dim() != 4 or coords.shape[1] < 1:
        raise RuntimeError("CorrBlock1D: coords must be (B, 2, H, W1)")
    if coords.dtype != torch.float32:
        raise RuntimeError(
            f"CorrBlock1D: coords dtype {coords.dtype} != float32 (grid_sample "
            "requires the grid dtype to match the volume, model.py:275)")
    B, _, H, W1 = coords.shape
    P = pyramid[0].shape[0]
    if B * H * W1 != P:
        raise RuntimeError(
            f"CorrBlock1D: coords {tuple(coords.shape)} do not match the volume's "
            f"{P} rows (view at model.py:312)")
    if coords.device != pyramid[0].device:
        raise RuntimeError("CorrBlock1D: coords and pyramid on different devices")
    x = coords[:, 0]
    if x.stride(2) != 1 or x.stride(1) != W1:
        x = x.contiguous()
    cbs = x.stride(0) if B > 1 else H * W1
    C = num_levels * (2 * radius + 1)
    out = torch.empty((B, C, H, W1), dtype=torch.float32, device=coords.device)
    if P == 0:
        return out
    levels = [pyramid[i] for i in range(num_levels)]
    levels = [t if t.stride(-1) == 1 and t.data_ptr() % 16 == 0 else t.contiguous() for t in levels]
    dt = levels[0].dtype
    with torch.cuda.device(coords.device):
        rc = _lib.lib().rc_corr_lookup(
            _lib.ptr_array([t.data_ptr() for t in levels]),
            _lib.int_array([t.shape[-1] for t in levels]),
            _lib.long_array([_row_stride(t) for t in levels]),
            _dtype_code(dt), num_levels, radius, x.data_ptr(), cbs, B, H, W1,
            out.data_ptr(), _stream(coords.device))
    _lib.check(rc, "rc_corr_lookup")
    return out


class CorrBlock1D:
    """model.py:283-326, on the gfx950 kernels (see module docstring)."""

    def __init__(self, fmap1, fmap2, num_levels=4, radius=4, *, pyramid_dtype=None):
        self.num_levels = num_levels
        self.radius = radius
        if pyramid_dtype is None:
            low = fmap1.dtype in (torch.bfloat16, torch.float16)
            pyramid_dtype = torch.bfloat16 if low else torch.float32
        self.pyramid_dtype = pyramid_dtype
        self.corr_pyramid = build_pyramid(fmap1, fmap2, num_levels + 1, pyramid_dtype)

    def __call__(self, coords):
        return lookup(self.corr_pyramid, coords, self.num_levels, self.radius)

    def lookup_convc1(self, coords, weight, bias=None, relu=True):
        """``relu(convc1(self(coords)))`` in one launch:
        the motion encoder's first layer (model.py:199, :206) fused into the
        lookup, so the (B, L(2r+1), H, W1) correlation never reaches HBM."""
        return lookup_convc1(self.corr_pyramid, coords, self.num_levels, self.radius, weight,
                             bias, relu)

    @staticmethod
    def corr(fmap1, fmap2):
        B, D, H, W1, W2 = _check_fmaps(fmap1, fmap2)
        lvl0 = build_pyramid(fmap1, fmap2, 1, pad=False)[0]
        return lvl0.view(B, H, W1, 1, W2)


def coords_grid(batch, ht, wd, device=None):
    """model.py:329-332: (batch, 2, ht, wd) fp32, channel 0 = x, channel 1 = y."""
    ys, xs = torch.meshgrid(torch.arange(ht, device=device), torch.arange(wd, device=device),
                            indexing="ij")
    return torch.stack((xs, ys), dim=0).float()[None].repeat(batch, 1, 1, 1)
