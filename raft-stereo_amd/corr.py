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
  * ``__call__(coords)``  (model.py:297-316)  one lookup launch:
      (B,2,H,W1) fp32 coords -> (B, num_levels*(2r+1), H, W1) fp32.  For an
      fp32 pyramid with 2-4 levels it is rc_corr_lookup_chain, which reads two
      stored levels (0 and 2, or 0 and 1 for 3 levels) and recomputes the
      others (bit-identical to rc_corr_lookup, fewer HBM lines per pixel);
      otherwise rc_corr_lookup.
  * ``CorrBlock1D.corr(fmap1, fmap2)``  (model.py:318-326) -> (B,H,W1,1,W2).
  * Autograd: when an fmap requires grad, the lookups
      and the build are autograd nodes.  Each lookup's backward adds its
      grid_sample input gradient into level-gradient buffers shared by the
      block (rc_corr_lookup_backward, no atomics); the build's backward,
      which autograd runs after all of them, folds those through the pooling
      backward and produces d fmap1 / d fmap2 with two fp32 MFMA GEMMs
      (rc_corr_build_backward).  ``corr_pyramid`` itself carries no grad_fn.

Error behaviour follows the reference where it has one: W2 < 2**num_levels
raises RuntimeError (avg_pool2d, model.py:294); mismatched fmap shapes raise
RuntimeError (einsum, :324); coords that do not match the volume's
(B, H, W1) raise RuntimeError (view, :312); non-fp32 coords raise
RuntimeError (grid_sample dtype check, :275).

Differences, all loud: tensors must live on a HIP device (no CPU fallback);
the fused ``lookup_convc1`` is inference-only (asking for gradients raises);
bf16/fp16 fmaps are accepted (the reference crashes on them, SURVEY.md
Appendix A D9; their gradients are computed in fp32): they, or
an explicit ``pyramid_dtype=torch.bfloat16``, select the bf16 MFMA kernel and
a bf16 pyramid (bf16-level tolerance).
"""
import warnings

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
    return B, D, H, W1, W2


def _prep_fmap(f):
    # fp32 and bf16 go to the kernels as they are; fp16 (default autocast)
    # is widened to fp32 and then rounded to bf16 on load by the bf16 kernel.
    if f.dtype == torch.float16:
        f = f.float()
    elif f.dtype not in (torch.float32, torch.bfloat16):
        raise TypeError(f"raft_stereo_amd: unsupported fmap dtype {f.dtype}")
    return f.contiguous()


# Row stride granule of the stored levels (bytes): 16 keeps every store a
# whole aligned vector.
_ROW_ALIGN_BYTES = 16


def _level_buffer(P, W, dtype, device, pad, shadow=False):
    """(P, 1, 1, W) tensor whose rows start 16-byte aligned: a view of a
    (P, ld) buffer with ld = W rounded up to 16 bytes when ``pad`` (the
    kernels then store whole aligned vectors; the padding is never read).
    ``shadow``: the allocation also holds the level's RC_SHADOW copy at
    ``_lib.shadow_offset`` bytes (include/raftcorr.h); the view is the primary."""
    es = torch.tensor([], dtype=dtype).element_size()
    per16 = _ROW_ALIGN_BYTES // es
    ld = -(-W // per16) * per16 if pad else W
    if shadow:
        total = _lib.shadow_offset(P, ld, es) + P * ld * es
        buf = torch.empty(-(-total // es), dtype=dtype, device=device)[:P * ld].view(P, ld)
    else:
        buf = torch.empty((P, ld), dtype=dtype, device=device)
    if ld == W:
        return buf.view(P, 1, 1, W)
    return buf[:, :W].unsqueeze(1).unsqueeze(1)


def _shadow_levels(shadow, n):
    """bool (every level) or an iterable of level indices -> frozenset."""
    if shadow is True:
        return frozenset(range(n))
    if not shadow:
        return frozenset()
    return frozenset(int(l) for l in shadow if 0 <= int(l) < n)


def _shadow_flags(levels, pyr):
    """RC_SHADOW_LEVEL bits for the stored levels of ``pyr`` in ``levels``."""
    return sum(_lib.shadow_level(l) for l in levels if l < len(pyr) and pyr[l] is not None)


def shadow_fits(P, W, dtype):
    """True when a level of width W and its RC_SHADOW copy fit the 4 GiB the
    pair kernel addresses with 32-bit buffer offsets."""
    es = torch.tensor([], dtype=dtype).element_size()
    ld = -(-W // (_ROW_ALIGN_BYTES // es)) * (_ROW_ALIGN_BYTES // es)
    return _lib.shadow_offset(P, ld, es) + P * ld * es <= 0xFFFFFF00


def _row_stride(t):
    """Row stride (elements) of a (P, 1, 1, W) level; rows must be unit-stride."""
    if t.stride(-1) != 1:
        raise RuntimeError("raft_stereo_amd: pyramid rows must be contiguous")
    return t.stride(0) if t.shape[0] > 1 else t.shape[-1]


def build_pyramid(fmap1, fmap2, nbuf, pyramid_dtype=torch.float32, pad=True, skip=(), shadow=False,
                  exact_f32=False):
    """Run rc_corr_build: returns ``nbuf`` tensors (B*H*W1, 1, 1, W2 >> l)
    (row-padded views when ``pad``; values identical either way).  Levels in
    ``skip`` (>= 1) are computed by the fused epilogue but not stored: their
    entries are None.  ``shadow``: every stored level also gets its RC_SHADOW
    copy (same values, half a 128-B line later; read by the pair lookup).
    ``exact_f32``: fp32 fmaps and pyramid run the exact fp32 MFMA kernel
    (RC_BUILD_EXACT_F32) instead of the split-bf16 one (fp32 accuracy,
    DESIGN.md §3.1c)."""
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
    shadow = _shadow_levels(shadow, nbuf) if pad else frozenset()
    pyr = [None if l in skip else _level_buffer(P, W2 >> l, pyramid_dtype, f1.device, pad, l in shadow)
           for l in range(nbuf)]
    if P == 0:
        return pyr
    with torch.cuda.device(f1.device):
        rc = _lib.lib().rc_corr_build(
            f1.data_ptr(), f2.data_ptr(), _dtype_code(f1.dtype), B, D, H, W1, W2,
            _lib.ptr_array([None if t is None else t.data_ptr() for t in pyr]),
            _lib.long_array([W2 >> l if t is None else _row_stride(t) for l, t in enumerate(pyr)]),
            nbuf, _dtype_code(pyramid_dtype) | _shadow_flags(shadow, pyr) |
            (_lib.RC_BUILD_EXACT_F32 if exact_f32 else 0), _stream(f1.device))
    _lib.check(rc, "rc_corr_build")
    return pyr


def pool_level(src):
    """One pyramid step (model.py:294) with rc_corr_pool: (P,1,1,W) -> (P,1,1,W//2)
    in a row-padded buffer, the same fp32 (or bf16) ops as the build epilogue."""
    P, W = src.shape[0], src.shape[-1]
    out = _level_buffer(P, W // 2, src.dtype, src.device, True)
    if P == 0:
        return out
    with torch.cuda.device(src.device):
        rc = _lib.lib().rc_corr_pool(src.data_ptr(), _row_stride(src), out.data_ptr(),
                                     _row_stride(out), P, W, _dtype_code(src.dtype),
                                     _stream(src.device))
    _lib.check(rc, "rc_corr_pool")
    return out


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
    _require_hip(weight, "weight")
    if weight.device != coords.device:
        raise RuntimeError("lookup_convc1: weight and coords on different devices")
    w = weight.detach().reshape(weight.shape[0], -1).float().contiguous()
    if w.shape[1] != cin:
        raise RuntimeError(f"lookup_convc1: weight has {w.shape[1]} input channels, lookup gives {cin}")
    cout = w.shape[0]
    b = None
    if bias is not None:
        _require_hip(bias, "bias")
        if bias.device != coords.device:
            raise RuntimeError("lookup_convc1: bias and coords on different devices")
        if bias.numel() != cout:
            raise RuntimeError(f"lookup_convc1: bias has {bias.numel()} elements, weight has {cout} "
                               "output channels")
        b = bias.detach().float().contiguous()
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
    x, cbs = _check_coords(pyramid, coords)
    B, _, H, W1 = coords.shape
    C = num_levels * (2 * radius + 1)
    out = torch.empty((B, C, H, W1), dtype=torch.float32, device=coords.device)
    if B * H * W1 == 0:
        return out
    keep, ptrs, widths, lds, dt = _level_args(pyramid, num_levels)
    with torch.cuda.device(coords.device):
        rc = _lib.lib().rc_corr_lookup(ptrs, widths, lds, dt, num_levels, radius, x.data_ptr(), cbs,
                                       B, H, W1, out.data_ptr(), _stream(coords.device))
    _lib.check(rc, "rc_corr_lookup")
    return out


def _chain_args(pyramid, num_levels, shadow=False):
    """Pointer / width / stride arrays for the pool-chain kernels: the levels
    present in ``pyramid`` (None = recomputed by the kernel, passed as NULL).
    ``shadow``: levels built with their RC_SHADOW copy (build_pyramid's
    ``shadow``); their flags are passed unless a level had to be copied."""
    src = list(pyramid[:num_levels]) + [None] * (num_levels - len(pyramid))
    lv = [None if t is None else
          (t if t.stride(-1) == 1 and t.data_ptr() % 16 == 0 else t.contiguous())
          for t in src]
    shadow = _shadow_levels(shadow, num_levels) if all(a is b for a, b in zip(lv, src)) else ()
    dt = lv[0].dtype
    if any(t is not None and t.dtype != dt for t in lv):
        raise TypeError("lookup_chain: pyramid levels of one dtype required")
    W0 = lv[0].shape[-1]
    ptrs = _lib.ptr_array([None if t is None else t.data_ptr() for t in lv])
    widths = _lib.int_array([W0 >> i for i in range(num_levels)])
    lds = _lib.long_array([W0 >> i if t is None else _row_stride(t) for i, t in enumerate(lv)])
    return lv, ptrs, widths, lds, _dtype_code(dt) | _shadow_flags(shadow, lv)


def _lookup_out(B, C, H, W1, device, channels_last):
    """(B, C, H, W1) fp32 lookup output; channels_last: NHWC memory order
    (the C-ABI's RC_OUT_CHANNELS_LAST), same shape and values."""
    if channels_last:
        return torch.empty((B, H, W1, C), dtype=torch.float32, device=device).permute(0, 3, 1, 2)
    return torch.empty((B, C, H, W1), dtype=torch.float32, device=device)


def _pair_layout(pyramid, num_levels):
    """The pair kernel serves this request (include/raftcorr.h, chain_kind)."""
    return num_levels == 2 or (num_levels == 4 and len(pyramid) > 2 and pyramid[2] is not None)


def lookup_chain(pyramid, coords, num_levels, radius, shadow=False, channels_last=False):
    """rc_corr_lookup_chain: same result as :func:`lookup` for a pyramid whose
    levels are the avg-pool chain of level 0 (what :func:`build_pyramid`
    writes).  Entries may be None: with 2 levels, or 4 levels and level 2
    present, the kernel reads levels 0 and 2 and derives 1 and 3; otherwise it
    reads levels 0 and 1 and derives the rest (include/raftcorr.h)."""
    x, cbs = _check_coords(pyramid, coords)
    B, _, H, W1 = coords.shape
    cl = channels_last and _pair_layout(pyramid, num_levels)
    out = _lookup_out(B, num_levels * (2 * radius + 1), H, W1, coords.device, cl)
    if B * H * W1 == 0:
        return out
    keep, ptrs, widths, lds, dt = _chain_args(pyramid, num_levels, shadow)
    if cl:
        dt |= _lib.RC_OUT_CHANNELS_LAST
    with torch.cuda.device(coords.device):
        rc = _lib.lib().rc_corr_lookup_chain(
            ptrs, widths, lds, dt, num_levels, radius, x.data_ptr(), cbs, B, H, W1,
            out.data_ptr(), _stream(coords.device))
    _lib.check(rc, "rc_corr_lookup_chain")
    if channels_last and not cl:
        out = out.contiguous(memory_format=torch.channels_last)
    return out


# ------------------------------------------------- disparity-major layout
# RC_LAYOUT_DISPARITY (ABI v9): the pair layout's stored
# levels (0, and 2 of 4) as S_l[b,h][k][w1], k = (w1 >> l) - j + (W2 >> l) - 1.

def _shear_ld(W1):
    return -(-W1 // 4) * 4


def shear_supported(fmap1, fmap2, num_levels, radius, pyramid_dtype):
    """Why CorrBlock1D(layout="disparity") cannot serve these inputs, or None."""
    if pyramid_dtype != torch.float32 or fmap1.dtype != torch.float32 or fmap2.dtype != torch.float32:
        return "fp32 fmaps and an fp32 pyramid only"
    if num_levels not in (2, 4) or not 1 <= radius <= 4:
        return "the pair layout: 2 or 4 levels, radius 1..4"
    B, D, H, W1, W2 = _check_fmaps(fmap1, fmap2)
    if W1 % 4 or W2 % 4:
        return "W1 and W2 multiples of 4 (the split-bf16 build)"
    if W2 > 65536:
        return "level-0 width <= 65536"
    ld = _shear_ld(W1)
    for l in ((0, 2) if num_levels == 4 else (0,)):
        if B * H * _lib.shear_rows(W2, W1, l) * ld * 4 >= 0xFFFFFF00:
            return f"disparity-major level {l} under 4 GiB"
    return None


def build_sheared(fmap1, fmap2, num_levels, exact_f32=False):
    """rc_corr_build with RC_LAYOUT_DISPARITY: {0: S_0, 2: S_2 (4 levels)},
    each a flat fp32 tensor of B*H*RC_SHEAR_ROWS rows of _shear_ld(W1)."""
    if exact_f32:
        raise ValueError("CorrBlock1D(layout='disparity') is built by the split-bf16 kernel only")
    B, D, H, W1, W2 = _check_fmaps(fmap1, fmap2)
    f1, f2 = _prep_fmap(fmap1), _prep_fmap(fmap2)
    ld = _shear_ld(W1)
    keep = (0, 2) if num_levels == 4 else (0,)
    sh = {l: torch.empty(B * H * _lib.shear_rows(W2, W1, l) * ld, dtype=torch.float32, device=f1.device)
          for l in keep}
    if B * H * W1 == 0:
        return sh
    nbuf = 3 if num_levels == 4 else 1
    ptrs = [sh[0].data_ptr(), None, sh[2].data_ptr()] if nbuf == 3 else [sh[0].data_ptr()]
    lds = [ld, W2 >> 1, ld][:nbuf]
    with torch.cuda.device(f1.device):
        rc = _lib.lib().rc_corr_build(
            f1.data_ptr(), f2.data_ptr(), _lib.RC_F32, B, D, H, W1, W2, _lib.ptr_array(ptrs),
            _lib.long_array(lds), nbuf, _lib.RC_F32 | _lib.RC_LAYOUT_DISPARITY, _stream(f1.device))
    _lib.check(rc, "rc_corr_build")
    return sh


def unshear_level(S, l, B, H, W1, W2):
    """A disparity-major level as the reference's (B*H*W1, 1, 1, W2 >> l)
    rows (row-padded buffer): the same values, gathered."""
    W = W2 >> l
    K = _lib.shear_rows(W2, W1, l)
    ld = _shear_ld(W1)
    w1 = torch.arange(W1, device=S.device)
    kk = (w1 >> l)[:, None] - torch.arange(W, device=S.device)[None, :] + W - 1
    rows = S.view(B * H, K, ld)[:, kk, w1[:, None].expand(W1, W)]
    out = _level_buffer(B * H * W1, W, torch.float32, S.device, True)
    out.copy_(rows.reshape(B * H * W1, 1, 1, W))
    return out


def lookup_sheared(sheared, coords, num_levels, radius, W2):
    """rc_corr_lookup_chain with RC_LAYOUT_DISPARITY: the pair kernel's
    results (bit for bit) from the disparity-major levels."""
    _require_hip(coords, "coords")
    if coords.dim() != 4 or coords.shape[1] < 1:
        raise RuntimeError("CorrBlock1D: coords must be (B, 2, H, W1)")
    if coords.dtype != torch.float32:
        raise RuntimeError(f"CorrBlock1D: coords dtype {coords.dtype} != float32 (model.py:275)")
    B, _, H, W1 = coords.shape
    ld = _shear_ld(W1)
    if B * H * _lib.shear_rows(W2, W1, 0) * ld != sheared[0].numel():
        raise RuntimeError(f"CorrBlock1D: coords {tuple(coords.shape)} do not match the volume "
                           "(view at model.py:312)")
    if coords.device != sheared[0].device:
        raise RuntimeError("CorrBlock1D: coords and pyramid on different devices")
    x = coords[:, 0]
    if x.stride(2) != 1 or x.stride(1) != W1:
        x = x.contiguous()
    cbs = x.stride(0) if B > 1 else H * W1
    out = torch.empty((B, num_levels * (2 * radius + 1), H, W1), dtype=torch.float32, device=coords.device)
    if B * H * W1 == 0:
        return out
    ptrs = [sheared.get(l) if l in (0, 2) else None for l in range(num_levels)]
    ptrs = _lib.ptr_array([None if t is None else t.data_ptr() for t in ptrs])
    widths = _lib.int_array([W2 >> l for l in range(num_levels)])
    lds = _lib.long_array([ld if l in (0, 2) else W2 >> l for l in range(num_levels)])
    with torch.cuda.device(coords.device):
        rc = _lib.lib().rc_corr_lookup_chain(
            ptrs, widths, lds, _lib.RC_F32 | _lib.RC_LAYOUT_DISPARITY, num_levels, radius, x.data_ptr(),
            cbs, B, H, W1, out.data_ptr(), _stream(coords.device))
    _lib.check(rc, "rc_corr_lookup_chain")
    return out


# ------------------------------------------------------------ record layout
# RC_LAYOUT_RECORDS (ABI v10): the 4-level bf16 pair layout's
# stored levels 0 and 2 as rec_count(W2) 128-B records per pixel row; record r
# holds level-2 elements 4r-14 .. 4r+11 (slots 0..25) and level-0 elements
# 16r-26 .. 16r+11 (slots 26..63), so a pixel's lookup reads one line.

_REC_L2_SLOTS = 26


def records_supported(fmap1, fmap2, num_levels, radius, pyramid_dtype):
    """Why CorrBlock1D(layout="records") cannot serve these inputs, or None."""
    if pyramid_dtype != torch.bfloat16:
        return "a bf16 pyramid only (bf16 fmaps, or pyramid_dtype=torch.bfloat16)"
    if num_levels != 4 or not 1 <= radius <= 4:
        return "4 levels, radius 1..4"
    B, D, H, W1, W2 = _check_fmaps(fmap1, fmap2)
    if not 64 < W2 <= 320:
        return "64 < W2 <= 320 (one workgroup tile spans the row)"
    if D <= 224:
        return "D > 224 (at least 8 K stages per tile)"
    if D * H * max(W1, W2) * 2 >= 1 << 30:
        return "fmap images under 1 GiB"
    return None


def auto_layout(fmap1, fmap2, num_levels, radius, pyramid_dtype=None, lazy_levels=None, shadow=None,
                low_latency=False, grad_shadow=None, exact_f32=False):
    """CorrBlock1D(layout="auto"): "records" for a bf16 pyramid the record
    build serves (with the default options) whose level 0 exceeds the
    256 MiB Infinity Cache, else "rows" (DESIGN.md §3.2i)."""
    if pyramid_dtype is None:
        pyramid_dtype = torch.bfloat16 if fmap1.dtype in (torch.bfloat16, torch.float16) else torch.float32
    if (low_latency or shadow or grad_shadow or exact_f32 or lazy_levels is False
            or records_supported(fmap1, fmap2, num_levels, radius, pyramid_dtype) is not None):
        return "rows"
    B, D, H, W1, W2 = _check_fmaps(fmap1, fmap2)
    return "records" if B * H * W1 * W2 * 2 > (256 << 20) else "rows"


def build_records(fmap1, fmap2):
    """rc_corr_build with RC_LAYOUT_RECORDS: a (B*H*W1, rec_count(W2), 64)
    bf16 tensor.  fp32/fp16 fmaps are rounded to bf16 first (round to nearest
    even, as the bf16 kernels do on load)."""
    B, D, H, W1, W2 = _check_fmaps(fmap1, fmap2)
    f1 = fmap1.to(torch.bfloat16).contiguous()
    f2 = fmap2.to(torch.bfloat16).contiguous()
    NR = _lib.rec_count(W2)
    rec = torch.empty((B * H * W1, NR, _lib.RC_REC_SLOTS), dtype=torch.bfloat16, device=f1.device)
    if B * H * W1 == 0:
        return rec
    with torch.cuda.device(f1.device):
        rc = _lib.lib().rc_corr_build(
            f1.data_ptr(), f2.data_ptr(), _lib.RC_BF16, B, D, H, W1, W2,
            _lib.ptr_array([rec.data_ptr(), None, None]), _lib.long_array([W2, W2 >> 1, W2 >> 2]), 3,
            _lib.RC_BF16 | _lib.RC_LAYOUT_RECORDS, _stream(f1.device))
    _lib.check(rc, "rc_corr_build")
    return rec


def records_level(rec, l, W2):
    """Level l (0 or 2) of a record-layout pyramid as the reference's
    (B*H*W1, 1, 1, W2 >> l) rows (row-padded buffer): the same values,
    gathered from the records that hold them."""
    P, NR, S = rec.shape
    W = W2 >> l
    e = torch.arange(W, device=rec.device)
    if l == 0:
        r = ((e + 26) >> 4).clamp(max=NR - 1)
        slot = _REC_L2_SLOTS + e - (16 * r - 26)
    elif l == 2:
        r = ((e + 14) >> 2).clamp(max=NR - 1)
        slot = e - (4 * r - 14)
    else:
        raise ValueError("records hold levels 0 and 2")
    out = _level_buffer(P, W, torch.bfloat16, rec.device, True)
    if P:
        out.copy_(rec.view(P, NR * S)[:, r * S + slot].view(P, 1, 1, W))
    return out


def _records_args(rec, W2):
    ptrs = _lib.ptr_array([rec.data_ptr(), None, None, None])
    widths = _lib.int_array([W2 >> l for l in range(4)])
    lds = _lib.long_array([W2 >> l for l in range(4)])
    return ptrs, widths, lds


def _check_records_coords(rec, coords):
    _require_hip(coords, "coords")
    if coords.dim() != 4 or coords.shape[1] < 1:
        raise RuntimeError("CorrBlock1D: coords must be (B, 2, H, W1)")
    if coords.dtype != torch.float32:
        raise RuntimeError(f"CorrBlock1D: coords dtype {coords.dtype} != float32 (model.py:275)")
    B, _, H, W1 = coords.shape
    if B * H * W1 != rec.shape[0]:
        raise RuntimeError(f"CorrBlock1D: coords {tuple(coords.shape)} do not match the volume's "
                           f"{rec.shape[0]} rows (view at model.py:312)")
    if coords.device != rec.device:
        raise RuntimeError("CorrBlock1D: coords and pyramid on different devices")


def lookup_records(rec, coords, radius, W2, channels_last=False):
    """rc_corr_lookup_chain with RC_LAYOUT_RECORDS: the pair kernel's
    results (bit for bit) from the records, one 128-B line per pixel."""
    _check_records_coords(rec, coords)
    B, _, H, W1 = coords.shape
    x = coords[:, 0]
    if x.stride(2) != 1 or x.stride(1) != W1:
        x = x.contiguous()
    cbs = x.stride(0) if B > 1 else H * W1
    out = _lookup_out(B, 4 * (2 * radius + 1), H, W1, coords.device, channels_last)
    if B * H * W1 == 0:
        return out
    ptrs, widths, lds = _records_args(rec, W2)
    dt = _lib.RC_BF16 | _lib.RC_LAYOUT_RECORDS | (_lib.RC_OUT_CHANNELS_LAST if channels_last else 0)
    with torch.cuda.device(coords.device):
        rc = _lib.lib().rc_corr_lookup_chain(ptrs, widths, lds, dt, 4, radius, x.data_ptr(), cbs, B, H, W1,
                                             out.data_ptr(), _stream(coords.device))
    _lib.check(rc, "rc_corr_lookup_chain")
    return out


# ----------------------------------------------------------------- backward

class _GradLevels(list):
    """The level-gradient list, with the levels that carry an RC_SHADOW copy."""
    shadow = frozenset()


def grad_buffers(P, widths, device, pair=False, shadow=(), zero=True):
    """Zeroed fp32 level-gradient buffers (P, W_l) with rows padded to 16 bytes
    (the padding stays zero: rc_corr_lookup_backward never touches it).
    ``zero=False``: uninitialised, for :func:`lookup_backward_calls` with
    ``overwrite=True`` (which writes every row, padding included).
    ``pair``: the pair layout -- levels 1 and 3 are None, their gradients are
    folded into levels 0 and 2 by the pair backward kernel.  ``shadow``:
    levels (0 and/or 2 of the 4-level pair layout) whose allocation also holds
    a zeroed RC_SHADOW copy at ``_lib.shadow_offset``; the lookup backward adds
    each span into the copy where it touches fewer 128-B lines and the build
    backward sums the two."""
    shadow = frozenset(shadow)
    if shadow and not (pair and len(widths) == 4 and shadow <= {0, 2}):
        raise ValueError("gradient shadow copies: levels 0 and 2 of the 4-level pair layout")
    bufs = _GradLevels()
    for l, W in enumerate(widths):
        if pair and l % 2 == 1:
            bufs.append(None)
            continue
        ld = -(-W // 4) * 4
        if l in shadow:
            total = _lib.shadow_offset(P, ld, 4) + P * ld * 4
            buf = torch.zeros(total // 4, dtype=torch.float32, device=device)[:P * ld].view(P, ld)
        elif zero:
            buf = torch.zeros((P, ld), dtype=torch.float32, device=device)
        else:
            buf = torch.empty((P, ld), dtype=torch.float32, device=device)
        bufs.append(buf[:, :W])
    bufs.shadow = shadow
    return bufs


def _grad_shadow_flags(grads):
    return sum(_lib.shadow_level(l) for l in getattr(grads, "shadow", ()))


def _pair_grads_ok(num_levels, radius, W0):
    return num_levels in (2, 4) and 1 <= radius <= 4 and W0 <= 65536


def lookup_backward(grads, coords, grad_out, num_levels, radius):
    """rc_corr_lookup_backward: accumulate d(lookup)/d(level i) . grad_out into
    ``grads`` (from :func:`grad_buffers`) -- grid_sample's input gradient
    (model.py:275) for every level and tap of the lookup at ``coords``."""
    x, cbs = _check_coords(grads, coords)
    B, _, H, W1 = coords.shape
    if B * H * W1 == 0:
        return
    go = grad_out.detach().float().contiguous()
    if go.shape != (B, num_levels * (2 * radius + 1), H, W1):
        raise RuntimeError(f"lookup_backward: grad_out shape {tuple(go.shape)}")
    W0 = grads[0].shape[-1]
    g = [grads[i] for i in range(num_levels)]
    with torch.cuda.device(coords.device):
        rc = _lib.lib().rc_corr_lookup_backward(
            _lib.ptr_array([None if t is None else t.data_ptr() for t in g]),
            _lib.int_array([W0 >> i for i in range(num_levels)]),
            _lib.long_array([W0 >> i if t is None else t.stride(0) for i, t in enumerate(g)]),
            num_levels | _grad_shadow_flags(grads), radius, x.data_ptr(), cbs, B, H, W1, go.data_ptr(),
            _stream(coords.device))
    _lib.check(rc, "rc_corr_lookup_backward")


def lookup_backward_calls(grads, coords_list, grad_out_list, num_levels, radius, overwrite=False):
    """rc_corr_lookup_backward_calls: the gradients of several lookup calls
    (``coords_list[c]``, ``grad_out_list[c]``) summed into ``grads`` in one
    pass -- equal to calling :func:`lookup_backward` once per call up to the
    association of the fp32 sums.  ``overwrite``: ``grads`` receive the sum
    instead of having it added (RC_GRAD_OVERWRITE; they need not be zeroed,
    see ``grad_buffers(zero=False)``).  With the pair layout the pixel's
    gradient rows stay on chip across the calls."""
    if len(coords_list) != len(grad_out_list):
        raise ValueError("lookup_backward_calls: one grad_out per coords")
    if getattr(grads, "shadow", ()):
        raise ValueError("lookup_backward_calls: gradient shadow copies are not supported")
    if not coords_list:
        if overwrite:
            for g in grads:
                if g is not None:
                    g.zero_()
        return
    xs, cbss, gos = [], [], []
    for coords, grad_out in zip(coords_list, grad_out_list):
        x, cbs = _check_coords(grads, coords)
        B, _, H, W1 = coords.shape
        go = grad_out.detach().float().contiguous()
        if go.shape != (B, num_levels * (2 * radius + 1), H, W1):
            raise RuntimeError(f"lookup_backward_calls: grad_out shape {tuple(go.shape)}")
        xs.append(x)
        cbss.append(cbs)
        gos.append(go)
    B, _, H, W1 = coords_list[0].shape
    if any(tuple(c.shape) != tuple(coords_list[0].shape) for c in coords_list):
        raise RuntimeError("lookup_backward_calls: every call needs the same coords shape")
    if B * H * W1 == 0:
        return
    W0 = grads[0].shape[-1]
    g = [grads[i] for i in range(num_levels)]
    flags = num_levels | (_lib.RC_GRAD_OVERWRITE if overwrite else 0)
    with torch.cuda.device(coords_list[0].device):
        rc = _lib.lib().rc_corr_lookup_backward_calls(
            _lib.ptr_array([None if t is None else t.data_ptr() for t in g]),
            _lib.int_array([W0 >> i for i in range(num_levels)]),
            _lib.long_array([W0 >> i if t is None else t.stride(0) for i, t in enumerate(g)]),
            flags, radius, len(xs), _lib.ptr_array([x.data_ptr() for x in xs]),
            _lib.long_array(cbss), B, H, W1, _lib.ptr_array([go.data_ptr() for go in gos]),
            _stream(coords_list[0].device))
    _lib.check(rc, "rc_corr_lookup_backward_calls")


def build_backward(fmap1, fmap2, grads, exact_f32=False):
    """rc_corr_build_backward: level gradients -> (d fmap1, d fmap2), fp32.
    The pooling backward (model.py:294), the 1/sqrt(D) (:326) and the two
    einsum operand gradients (:324) in one launch -- on split-bf16 MFMA
    (fp32 accuracy) by default, on exact fp32 MFMA with ``exact_f32``."""
    f1 = fmap1.detach().float().contiguous()
    f2 = fmap2.detach().float().contiguous()
    B, D, H, W1 = f1.shape
    W2 = f2.shape[3]
    if B * H * W1 == 0:
        return torch.zeros_like(f1), torch.zeros_like(f2)
    df1, df2 = torch.empty_like(f1), torch.empty_like(f2)
    # pair layout [g0, None, g2, None] -> levels 0-2 with level 1 NULL; [g0, None] -> level 0
    flags = _grad_shadow_flags(grads)
    if len(grads) > 1 and grads[1] is None:
        grads = [grads[0], None, grads[2]] if len(grads) > 2 else [grads[0]]
    with torch.cuda.device(f1.device):
        rc = _lib.lib().rc_corr_build_backward(
            f1.data_ptr(), f2.data_ptr(), _lib.RC_F32 | (_lib.RC_BUILD_EXACT_F32 if exact_f32 else 0),
            B, D, H, W1, W2,
            _lib.ptr_array([None if g is None else g.data_ptr() for g in grads]),
            _lib.long_array([W2 >> l if g is None else g.stride(0) for l, g in enumerate(grads)]),
            len(grads) | flags, df1.data_ptr(), df2.data_ptr(), _stream(f1.device))
    _lib.check(rc, "rc_corr_build_backward")
    return df1, df2


def default_shadow_levels(P, W2, num_levels, pyramid_dtype):
    """Stored levels that get an RC_SHADOW copy by default (measured per
    config with the corr step = build + 32 lookups, tools/shadow_probe.py,
    profiles/r03/shadow_*.log): level 2 of a 4-level pair
    layout always; level 0 only for a bf16 pyramid larger than the 256 MiB
    Infinity Cache.  A bf16 span (40 B) then always fits one 128-B line, which
    pays for the copy's writes (config 3, B=64: 6227 us per step with levels
    0 + 2, 6288 with level 2 only); an fp32 level 0 saves too little per
    lookup for its copy (config 4, 1.03 GB: 2376 us with levels 0 + 2, 2281
    with level 2 only; config 2: 1072 vs 1056).  Each copy must fit the
    kernel's 4 GiB window."""
    es = torch.tensor([], dtype=pyramid_dtype).element_size()
    lv = [2] if num_levels == 4 else []
    if pyramid_dtype == torch.bfloat16 and P * W2 * es > (256 << 20):
        lv.insert(0, 0)
    return tuple(l for l in lv if shadow_fits(P, W2 >> l, pyramid_dtype))


def default_grad_shadow_levels(P, widths, num_levels, pair):
    """Gradient levels that get an RC_SHADOW copy by default."""
    return ()


def _check_grad_shadow(grad_shadow, num_levels, radius, W0):
    """Validate a ``grad_shadow`` request at construction: levels
    0 and 2 only, and only with the 4-level pair gradient layout."""
    req = frozenset(int(l) for l in grad_shadow)
    if not req:
        return
    if not req <= {0, 2}:
        raise ValueError(f"grad_shadow={sorted(req)}: gradient shadow copies are levels 0 and 2")
    if not (num_levels == 4 and _pair_grads_ok(num_levels, radius, W0)):
        raise ValueError("grad_shadow needs the 4-level pair gradient layout (num_levels=4, "
                         f"radius <= 4, W2 <= 65536); got num_levels={num_levels}, radius={radius}")


class _GradState:
    """Level gradients shared by one CorrBlock1D's lookup nodes and its build
    node.  Holds no pyramid and no graph node, so no reference cycle keeps the
    pyramid alive.

    With the pair layout and no gradient shadow copies, the lookup nodes only
    record their (coords, grad_out); the build node sums all of them in one
    rc_corr_lookup_backward_calls pass (``deferred``) into
    buffers it never zeroes.  Otherwise each lookup node adds its call into
    zeroed buffers right away (rc_corr_lookup_backward).

    Retention: a recorded grad_out is converted to contiguous
    fp32 when it is recorded (one copy alive, not a second one per call at the
    end), and once ``max_pending_calls`` calls (one kernel launch's worth) or
    ``max_pending_bytes`` of them are pending they are summed right away -- the
    first partial pass overwrites the buffers, later ones add -- so at most
    that much is held however many iterations run.  Config 2 holds 32 x 37 MB
    (= 1.19 GB) until the build node, DESIGN.md §3.4c."""

    max_pending_calls = 32             # kMaxBwdCalls: the calls of one kernel launch
    max_pending_bytes = 2 << 30

    def __init__(self, P, widths, device, num_levels, radius, grad_shadow=None, deferred=None,
                 exact_f32=False):
        self.P, self.widths, self.device = P, widths, device
        self.exact_f32 = bool(exact_f32)
        self.num_levels, self.radius = num_levels, radius
        self.pair = _pair_grads_ok(num_levels, radius, widths[0])
        if grad_shadow is None:
            grad_shadow = default_grad_shadow_levels(P, widths, num_levels, self.pair)
        self.grad_shadow = frozenset(grad_shadow) if self.pair and num_levels == 4 else frozenset()
        if deferred is None:
            deferred = self.pair and not self.grad_shadow
        self.deferred = bool(deferred) and self.pair and not self.grad_shadow
        self.grads = None
        self.pending = []
        self.pending_bytes = 0
        self.token_sent = False

    def token_grad(self, device):
        if self.token_sent:
            return None
        self.token_sent = True
        return torch.zeros((), dtype=torch.float32, device=device)

    def accumulate(self, coords, grad_out):
        if self.deferred:
            go = grad_out.detach().float().contiguous()
            self.pending.append((coords, go))
            self.pending_bytes += go.numel() * go.element_size()
            if (len(self.pending) >= self.max_pending_calls
                    or self.pending_bytes >= self.max_pending_bytes):
                self._flush()
            return
        if self.grads is None:
            self.grads = grad_buffers(self.P, self.widths, self.device, pair=self.pair,
                                      shadow=self.grad_shadow)
        lookup_backward(self.grads, coords, grad_out, self.num_levels, self.radius)

    def _flush(self):
        """Sum the pending calls: into fresh (unzeroed) buffers the first time
        (RC_GRAD_OVERWRITE), added to them afterwards."""
        calls, self.pending, self.pending_bytes = self.pending, [], 0
        first = self.grads is None
        if first:
            self.grads = grad_buffers(self.P, self.widths, self.device, pair=True, zero=False)
        lookup_backward_calls(self.grads, [c for c, _ in calls], [g for _, g in calls],
                              self.num_levels, self.radius, overwrite=first)

    def take(self):
        if self.pending:
            self._flush()
        g, self.grads = self.grads, None
        return g


class _BuildFn(torch.autograd.Function):
    """Autograd node of the build.  Its output is a 0-d token every lookup
    consumes, so autograd runs this backward after all of theirs; by then the
    lookups have summed their level gradients into the shared state."""

    @staticmethod
    def forward(ctx, fmap1, fmap2, state):
        ctx.state = state
        ctx.save_for_backward(fmap1, fmap2)
        return torch.zeros((), dtype=torch.float32, device=fmap1.device)

    @staticmethod
    def backward(ctx, _token_grad):
        f1, f2 = ctx.saved_tensors
        ctx.state.token_sent = False          # a later backward through a new graph
        grads = ctx.state.take()
        if grads is None:          # no lookup output reached the loss
            return None, None, None
        df1, df2 = build_backward(f1, f2, grads, exact_f32=ctx.state.exact_f32)
        return df1.to(f1.dtype), df2.to(f2.dtype), None


class _LookupFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, token, coords, state, fn):
        ctx.state = state
        ctx.save_for_backward(coords)
        return fn(coords)

    @staticmethod
    def backward(ctx, grad_out):
        (coords,) = ctx.saved_tensors
        ctx.state.accumulate(coords, grad_out)
        # the build node only needs SOME defined gradient on its token: the
        # first lookup node to run hands over one zero, the others None (no
        # fill and no add kernel per call)
        return ctx.state.token_grad(coords.device), None, None, None


class CorrBlock1D:
    """model.py:283-326, on the gfx950 kernels (see module docstring)."""

    def __init__(self, fmap1, fmap2, num_levels=4, radius=4, *, pyramid_dtype=None,
                 lazy_levels=None, shadow=None, channels_last=False, low_latency=False,
                 grad_shadow=None, exact_f32=False, grad_deferred=None, layout="rows",
                 check_finite=False):
        self.num_levels = num_levels
        self.radius = radius
        # check_finite (opt-in): the split-bf16 default gives NaN
        # where the reference's fp32 einsum gives +-inf for inf fmap entries
        # (pinned by tests/test_split_gpu.py); with
        # check_finite=True one isfinite reduction over both fmaps (a host
        # sync) sends non-finite inputs to the exact fp32 kernel, with a
        # warning, so the volume keeps the reference's +-inf entries
        if (check_finite and not exact_f32 and fmap1.dtype == torch.float32 and
                fmap2.dtype == torch.float32 and pyramid_dtype in (None, torch.float32)):
            if not (bool(torch.isfinite(fmap1).all()) and bool(torch.isfinite(fmap2).all())):
                warnings.warn("CorrBlock1D: non-finite fmap values -- building on the exact fp32 "
                              "kernel (exact_f32=True) so that +-inf volume entries stay +-inf",
                              RuntimeWarning, stacklevel=2)
                exact_f32 = True
                layout = "rows"      # the disparity-major build is split-bf16 only
        # layout="disparity" (opt-in, RC_LAYOUT_DISPARITY): the
        # stored levels 0 and 2 disparity-major, so a wave's pixels that look
        # at the same disparity read contiguous memory; the same values and
        # lookups bit for bit, faster on the network's coherent coordinates,
        # slower on independent random ones.  corr_pyramid is gathered into
        # the reference's rows when read.
        # layout="records" (opt-in, RC_LAYOUT_RECORDS): the
        # bf16 pair layout's levels 0 and 2 as 128-B records, one line per
        # pixel per lookup instead of two; the same values and lookups bit for
        # bit; the build writes 1.8x the bytes of the shadowed rows.
        # layout="auto": the records where they pay -- a bf16 pyramid the
        # record build serves whose level 0 no longer fits the 256 MiB
        # Infinity Cache (config 3: step 5.31 vs 6.00 ms at B = 64, 1.50 vs
        # 1.64 at B = 16; at B = 8, 145 MB, the rows win: 0.835 vs 0.898,
        # profiles/r06/z, za) -- else the rows.
        if layout == "auto":
            layout = auto_layout(fmap1, fmap2, num_levels, radius, pyramid_dtype, lazy_levels, shadow,
                                 low_latency, grad_shadow, exact_f32)
        if layout not in ("rows", "disparity", "records"):
            raise ValueError(f"CorrBlock1D: layout={layout!r}: 'rows', 'disparity', 'records' or 'auto'")
        self.layout = layout
        self._sheared = None
        self._records = None
        if layout == "disparity":
            self._init_sheared(fmap1, fmap2, num_levels, radius, pyramid_dtype, lazy_levels, shadow,
                               channels_last, low_latency, grad_shadow, exact_f32, grad_deferred)
            return
        if layout == "records":
            self._init_records(fmap1, fmap2, num_levels, radius, pyramid_dtype, lazy_levels, shadow,
                               channels_last, low_latency, grad_shadow, exact_f32, grad_deferred)
            return
        # lookup outputs in NHWC memory order (torch.channels_last): same
        # shape and values; written by the pair kernel as contiguous per-wave
        # runs instead of one 256-B piece per channel plane
        self.channels_last = bool(channels_last)
        if pyramid_dtype is None:
            low = fmap1.dtype in (torch.bfloat16, torch.float16)
            pyramid_dtype = torch.bfloat16 if low else torch.float32
        self.pyramid_dtype = pyramid_dtype
        grad = torch.is_grad_enabled() and (fmap1.requires_grad or fmap2.requires_grad)
        B, D, H, W1, W2 = _check_fmaps(fmap1, fmap2)
        if num_levels < 1 or (W2 >> num_levels) < 1:
            raise RuntimeError(
                f"CorrBlock1D: W2={W2} is too narrow for {num_levels} pooling steps: "
                "avg_pool2d output size is too small (model.py:294)")
        if grad_shadow is not None:      # refused before the build is paid for
            _check_grad_shadow(grad_shadow, num_levels, radius, W2)
        # fp32 pyramids with 2-4 levels use a pool-chain lookup that reads two
        # stored levels and recomputes the others bit for bit (DESIGN.md §3.2c,
        # §3.2d): 2 or 4 levels -> levels 0 and 2 stored (the pair kernel), 3
        # levels -> levels 0 and 1 (the level-1 chain kernel).  The other
        # levels are built only when ``corr_pyramid`` is read (``lazy_levels``,
        # default on in that case): same values, same shapes, pooled by the
        # same fp32 ops.
        # (bf16 pyramids: the pair layout only -- 2 or 4 levels)
        self._chain = (1 <= radius <= 4 and fmap2.shape[-1] <= 65536 and
                       (num_levels in (2, 3, 4) if pyramid_dtype == torch.float32 else
                        num_levels in (2, 4) if pyramid_dtype == torch.bfloat16 else False))
        # low_latency (small inputs, e.g. the realtime config): store the
        # levels a lookup reads and use the per-level lookup, whose launcher gives each level
        # its own wave below 64K pixels (lookup_levelpar_kernel, DESIGN.md
        # §3.2g): a shorter dependent chain per launch, bit-identical values
        # grad_shadow: levels (0, 2 of the 4-level pair layout) whose gradient
        # buffers get an RC_SHADOW copy; None = the default
        # grad_deferred: the lookup nodes record their inputs and the build
        # node sums every call in one pass; None = on
        # wherever the pair gradient layout applies (no gradient shadow copies)
        if low_latency:
            self._chain = False
        lazy = self._chain if lazy_levels is None else (bool(lazy_levels) and self._chain)
        with torch.no_grad():
            if lazy and num_levels == 3:
                nbuf, skip = 2, ()
            elif lazy:
                nbuf, skip = (1, ()) if num_levels == 2 else (3, (1,))
            elif lazy_levels is None or lazy_levels:
                # per-level lookup (low_latency, or no pool chain): levels
                # 0 .. L-1 are read (model.py:303-304); level L, which no
                # lookup reads, is pooled when corr_pyramid is read
                nbuf, skip = num_levels, ()
            else:
                nbuf, skip = num_levels + 1, ()
            # RC_SHADOW: stored levels of the pair layout may
            # get a half-line-shifted copy; the pair lookup reads each span
            # from the copy where it touches fewer 128-B lines (same values).
            # ``shadow``: None = the default levels, True/False, or indices.
            pair = self._chain and num_levels in (2, 4) and lazy
            if shadow is None:
                shadow = default_shadow_levels(B * H * W1, W2, num_levels, pyramid_dtype)
            self._shadow = (frozenset(l for l in _shadow_levels(shadow, nbuf) if l not in skip)
                            if pair else frozenset())
            # an explicit request is held to the same 4 GiB window as the
            # default: a copy the pair kernel cannot address would cost its
            # build writes and make every lookup fail
            too_big = sorted(l for l in self._shadow
                             if not shadow_fits(B * H * W1, W2 >> l, pyramid_dtype))
            if too_big:
                warnings.warn(f"CorrBlock1D: shadow copies of levels {too_big} dropped: a level "
                              "plus its copy exceeds the pair kernel's 4 GiB window", stacklevel=2)
                self._shadow = self._shadow - frozenset(too_big)
            # exact_f32: the exact fp32 MFMA volume kernel instead of the
            # split-bf16 default (both fp32-accurate)
            self._levels = build_pyramid(fmap1, fmap2, nbuf, pyramid_dtype, skip=skip,
                                         shadow=self._shadow, exact_f32=exact_f32)
            self._levels += [None] * (num_levels + 1 - nbuf)
        self._state = self._token = None
        if grad:
            self._state = _GradState(B * H * W1, [W2 >> i for i in range(num_levels)],
                                     fmap1.device, num_levels, radius, grad_shadow,
                                     deferred=grad_deferred, exact_f32=exact_f32)
            self._token = _BuildFn.apply(fmap1, fmap2, self._state)

    def _init_sheared(self, fmap1, fmap2, num_levels, radius, pyramid_dtype, lazy_levels, shadow,
                      channels_last, low_latency, grad_shadow, exact_f32, grad_deferred):
        if pyramid_dtype is None:
            pyramid_dtype = torch.float32
        why = shear_supported(fmap1, fmap2, num_levels, radius, pyramid_dtype)
        if why is None and (channels_last or low_latency or shadow or grad_shadow or exact_f32
                            or lazy_levels is False):
            why = ("the default options only (NCHW output, no low_latency, shadow, grad_shadow, "
                   "exact_f32 or eager levels)")
        if why is not None:
            raise ValueError(f"CorrBlock1D(layout='disparity'): {why}")
        self.pyramid_dtype = pyramid_dtype
        self.channels_last = False
        B, D, H, W1, W2 = _check_fmaps(fmap1, fmap2)
        self._shape = (B, H, W1, W2)
        self._chain, self._shadow = True, frozenset()
        grad = torch.is_grad_enabled() and (fmap1.requires_grad or fmap2.requires_grad)
        with torch.no_grad():
            self._sheared = build_sheared(fmap1, fmap2, num_levels)
        self._levels = [None] * (num_levels + 1)
        self._state = self._token = None
        if grad:
            self._state = _GradState(B * H * W1, [W2 >> i for i in range(num_levels)], fmap1.device,
                                     num_levels, radius, None, deferred=grad_deferred)
            self._token = _BuildFn.apply(fmap1, fmap2, self._state)

    def _init_records(self, fmap1, fmap2, num_levels, radius, pyramid_dtype, lazy_levels, shadow,
                      channels_last, low_latency, grad_shadow, exact_f32, grad_deferred):
        if pyramid_dtype is None:
            pyramid_dtype = torch.bfloat16
        why = records_supported(fmap1, fmap2, num_levels, radius, pyramid_dtype)
        if why is None and (low_latency or shadow or grad_shadow or exact_f32 or lazy_levels is False):
            why = ("no low_latency, shadow, grad_shadow, exact_f32 or eager levels (the records replace "
                   "the stored rows and their shadow copies)")
        if why is not None:
            raise ValueError(f"CorrBlock1D(layout='records'): {why}")
        self.pyramid_dtype = pyramid_dtype
        self.channels_last = bool(channels_last)
        B, D, H, W1, W2 = _check_fmaps(fmap1, fmap2)
        self._shape = (B, H, W1, W2)
        self._chain, self._shadow = True, frozenset()
        grad = torch.is_grad_enabled() and (fmap1.requires_grad or fmap2.requires_grad)
        with torch.no_grad():
            self._records = build_records(fmap1, fmap2)
        self._levels = [None] * (num_levels + 1)
        self._state = self._token = None
        if grad:
            self._state = _GradState(B * H * W1, [W2 >> i for i in range(num_levels)], fmap1.device,
                                     num_levels, radius, None, deferred=grad_deferred)
            self._token = _BuildFn.apply(fmap1, fmap2, self._state)

    @property
    def corr_pyramid(self):
        """num_levels+1 tensors (B*H*W1, 1, 1, W2 >> l) as model.py:287-295;
        lazily pooled levels are built on first access (layout="disparity" /
        "records": the stored levels gathered into rows, the others pooled
        from them)."""
        if any(t is None for t in self._levels):
            with torch.no_grad():
                if self._records is not None:
                    W2 = self._shape[3]
                    for l in (0, 2):
                        if self._levels[l] is None:
                            self._levels[l] = records_level(self._records, l, W2)
                if self._sheared is not None:
                    B, H, W1, W2 = self._shape
                    for l, S in self._sheared.items():
                        if self._levels[l] is None:
                            self._levels[l] = unshear_level(S, l, B, H, W1, W2)
                for l in range(1, len(self._levels)):
                    if self._levels[l] is None:
                        self._levels[l] = pool_level(self._levels[l - 1])
        return self._levels

    @property
    def levels_stored(self):
        """Indices of the pyramid levels currently held in memory (either
        layout)."""
        held = set(self._sheared or ()) | ({0, 2} if self._records is not None else set())
        return sorted(held | {l for l, t in enumerate(self._levels) if t is not None})

    @corr_pyramid.setter
    def corr_pyramid(self, levels):
        # a replaced pyramid need not be a pool chain: use the per-level lookup
        self._levels = list(levels)
        self._chain = False
        self._shadow = frozenset()
        self._sheared = None
        self._records = None
        self.layout = "rows"

    def _read_levels(self):
        """Levels 0 .. num_levels-1 for the per-level kernels (the ones a
        lookup reads), without materialising a lazily pooled top level."""
        L = self.num_levels
        if all(t is not None for t in self._levels[:L]):
            return self._levels[:L]
        return self.corr_pyramid[:L]

    def _lookup(self, coords):
        if self._records is not None:
            return lookup_records(self._records, coords, self.radius, self._shape[3], self.channels_last)
        if self._sheared is not None:
            return lookup_sheared(self._sheared, coords, self.num_levels, self.radius, self._shape[3])
        if self._chain:
            return lookup_chain(self._levels, coords, self.num_levels, self.radius, self._shadow,
                                self.channels_last)
        out = lookup(self._read_levels(), coords, self.num_levels, self.radius)
        return out.contiguous(memory_format=torch.channels_last) if self.channels_last else out

    def __call__(self, coords):
        if self._token is not None and torch.is_grad_enabled():
            return _LookupFn.apply(self._token, coords.detach(), self._state, self._lookup)
        return self._lookup(coords)

    def lookup_step(self, coords1, delta=None, out=None):
        """One iteration's corr step in ONE launch:
        ``coords1 <- coords1 + delta`` with delta's y ignored (the loop tail
        zeroes it), ``flow = coords1 - coords_grid``
        (model.py:377) and the lookup at the new coords1 (:376).  Returns
        ``(corr, coords1_new, flow)``, each bit-identical to the unfused ops.
        ``delta=None`` skips the update (first iteration); ``out=coords1``
        updates in place.  Inference only."""
        if self._token is not None and torch.is_grad_enabled():
            raise RuntimeError("CorrBlock1D.lookup_step is inference-only")
        if self._sheared is not None:
            raise RuntimeError("CorrBlock1D.lookup_step: not available with layout='disparity'")
        if self._records is not None:
            _check_records_coords(self._records, coords1)
        else:
            _check_coords(self._levels, coords1)
        B, C2, H, W1 = coords1.shape
        if C2 != 2:
            raise RuntimeError("lookup_step: coords1 must be (B, 2, H, W1)")
        c1 = coords1.detach().contiguous()
        d = None
        if delta is not None:
            _require_hip(delta, "delta")
            if delta.device != c1.device:
                raise RuntimeError("lookup_step: delta and coords1 on different devices")
            d = delta.detach().float().contiguous()
            if d.shape != c1.shape:
                raise RuntimeError(f"lookup_step: delta {tuple(d.shape)} != coords {tuple(c1.shape)}")
        if out is not None:
            _require_hip(out, "out")
            if out.device != c1.device:
                raise RuntimeError("lookup_step: out and coords1 on different devices")
        new = torch.empty_like(c1) if out is None else out
        if new.shape != c1.shape or not new.is_contiguous() or new.dtype != torch.float32:
            raise RuntimeError("lookup_step: out must be a contiguous fp32 (B, 2, H, W1) tensor")
        flow = torch.empty_like(c1)
        L, r = self.num_levels, self.radius
        cl = self.channels_last and self._chain and (self._records is not None or _pair_layout(self._levels, L))
        corr = _lookup_out(B, L * (2 * r + 1), H, W1, c1.device, cl)
        if B * H * W1 == 0:
            return corr, new, flow
        if self._records is not None:
            ptrs, widths, lds = _records_args(self._records, self._shape[3])
            dt = _lib.RC_BF16 | _lib.RC_LAYOUT_RECORDS
        elif self._chain:
            keep, ptrs, widths, lds, dt = _chain_args(self._levels, L, self._shadow)
        else:
            keep, ptrs, widths, lds, dt = _level_args(self._read_levels(), L)
        if cl:
            dt |= _lib.RC_OUT_CHANNELS_LAST
        with torch.cuda.device(c1.device):
            rc = _lib.lib().rc_corr_lookup_step(
                ptrs, widths, lds, dt, L, r, int(self._chain), c1.data_ptr(),
                d.data_ptr() if d is not None else None, new.data_ptr(), flow.data_ptr(),
                B, H, W1, corr.data_ptr(), _stream(c1.device))
        _lib.check(rc, "rc_corr_lookup_step")
        if self.channels_last and not cl:
            corr = corr.contiguous(memory_format=torch.channels_last)
        return corr, new, flow

    def lookup_convc1(self, coords, weight, bias=None, relu=True):
        """``relu(convc1(self(coords)))`` in one launch:
        the motion encoder's first layer (model.py:199, :206) fused into the
        lookup, so the (B, L(2r+1), H, W1) correlation never reaches HBM.
        Inference only."""
        if torch.is_grad_enabled() and (self._token is not None or weight.requires_grad):
            raise RuntimeError("CorrBlock1D.lookup_convc1 is inference-only; use "
                               "convc1(block(coords)) when gradients are needed")
        if self._sheared is not None or self._records is not None:
            raise RuntimeError(f"CorrBlock1D.lookup_convc1: not available with layout={self.layout!r}")
        return lookup_convc1(self._read_levels(), coords, self.num_levels, self.radius, weight,
                             bias, relu)

    @staticmethod
    def corr(fmap1, fmap2, exact_f32=False):
        B, D, H, W1, W2 = _check_fmaps(fmap1, fmap2)
        lvl0 = build_pyramid(fmap1, fmap2, 1, pad=False, exact_f32=exact_f32)[0]
        return lvl0.view(B, H, W1, 1, W2)


def coords_grid(batch, ht, wd, device=None):
    """model.py:329-332: (batch, 2, ht, wd) fp32, channel 0 = x, channel 1 = y."""
    ys, xs = torch.meshgrid(torch.arange(ht, device=device), torch.arange(wd, device=device),
                            indexing="ij")
    return torch.stack((xs, ys), dim=0).float()[None].repeat(batch, 1, 1, 1)
