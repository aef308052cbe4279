"""Work partitioning for the correlation path across GPUs (one process per GPU).

Batch sharding (BASELINE configs 2-3): stereo pairs are independent in eval
mode (BatchNorm uses running stats, InstanceNorm and the corr path are
per-sample), so each rank runs its contiguous slice of the
batch with no data-path collective; ``gather_batch`` is the single final
all_gather (RCCL over xGMI on the GPU box, gloo in the CPU tests).

Row sharding (config 4): the correlation volume, pyramid and lookup are
strictly row-local -- row h of fmap1 only meets row h of fmap2
(model.py:324) and the lookup ignores y (model.py:299, :308) -- so
``RowShardedCorr`` builds and looks up only its own block of feature rows,
again with no exchange.  ``RowShardedStereo`` runs the whole network that
way, exchanging only the GRU state halos each iteration.
"""
import contextlib
import time
import weakref

import torch
import torch.distributed as dist
import torch.nn.functional as F

from .corr import CorrBlock1D, coords_grid


def _host_staged(t, group=None):
    """gloo moves host memory only: CUDA tensors go through host copies when
    the group is gloo (the CPU tests, and several ranks sharing one GPU in the
    single-GPU tests).  RCCL ("nccl") takes device tensors directly."""
    return t.is_cuda and dist.get_backend(group) == "gloo"


def split_range(n, rank, world):
    """Contiguous [start, stop) of ``n`` items for ``rank``; the first n % world
    ranks take one extra item."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (rank < extra)


def local_batch(t, rank, world):
    s, e = split_range(t.shape[0], rank, world)
    return t[s:e]


def gather_batch(local, world, group=None):
    """all_gather of per-rank batch slices (sizes may differ by one) -> full batch."""
    if world == 1:
        return local
    dev = local.device
    if _host_staged(local, group):
        local = local.cpu()
    n = torch.tensor([local.shape[0]], device=local.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    cap = max(sizes)
    pad = local
    if local.shape[0] < cap:
        pad = torch.cat([local, local.new_zeros((cap - local.shape[0],) + tuple(local.shape[1:]))])
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad.contiguous(), group=group)
    return torch.cat([b[:s] for b, s in zip(bufs, sizes)], dim=0).to(dev)


class RowShardedCorr:
    """CorrBlock1D over feature rows [r0, r1) of (B, D, H, W) fmaps.

    ``__call__`` takes the FULL-height coords (B, 2, H, W1) and returns the
    lookup for this rank's rows, (B, L(2r+1), r1-r0, W1); concatenating the
    ranks' outputs along H equals the unsharded lookup bit for bit.
    """

    def __init__(self, fmap1, fmap2, rank, world, num_levels=4, radius=4, corr_block=CorrBlock1D,
                 **kw):
        self.r0, self.r1 = split_range(fmap1.shape[2], rank, world)
        f1 = fmap1[:, :, self.r0:self.r1].contiguous()
        f2 = fmap2[:, :, self.r0:self.r1].contiguous()
        self.block = corr_block(f1, f2, num_levels=num_levels, radius=radius, **kw)

    def __call__(self, coords):
        return self.block(coords[:, :, self.r0:self.r1].contiguous())


# ---------------------------------------------------------------------------
# Row-sharded network forward (BASELINE config 4: full-resolution, bs=1)
# ---------------------------------------------------------------------------

_INTERP = {}   # row geometry -> (l0, l1, lam): the same every iteration


def _interp_index(src_lo, src_glob, dst_lo, dst_hi, dst_glob, hs, device):
    """The global row mapping of _interp_rows (source rows l0, l1 inside the
    slab and the weight lam of each destination row), computed once per
    geometry and device: the GRU loop asks for the same few every iteration,
    and each recomputation is a dozen tiny kernels.  The key
    holds the current HIP stream: an entry is built and read on one stream
    only, so no reader can see it before its kernels finish and clear()
    frees nothing another stream still has queued."""
    sid = torch.cuda.current_stream(device).stream_id if device.type == "cuda" else 0
    key = (src_lo, src_glob, dst_lo, dst_hi, dst_glob, hs, str(device), sid)
    hit = _INTERP.get(key)
    if hit is None:
        if len(_INTERP) > 256:
            _INTERP.clear()
        scale = (src_glob - 1) / (dst_glob - 1) if dst_glob > 1 else 0.0
        i = torch.arange(dst_lo, dst_hi, device=device, dtype=torch.float32)
        pos = (i * scale).clamp(max=src_glob - 1)
        h0 = pos.floor()
        lam = (pos - h0).view(1, 1, -1, 1)
        h0 = h0.long()
        h1 = torch.clamp(h0 + 1, max=src_glob - 1)
        l0 = (h0 - src_lo).clamp(0, hs - 1)
        l1 = (h1 - src_lo).clamp(0, hs - 1)
        hit = _INTERP[key] = (l0, l1, lam, 1 - lam)
    return hit


def _interp_rows(x, src_lo, src_glob, dst_lo, dst_hi, dst_glob, dst_w):
    """bilinear, align_corners=True resize of a row SLAB (model.py:184-186)
    with the GLOBAL row mapping: destination rows [dst_lo, dst_hi) of a level
    of height dst_glob, from source rows [src_lo, src_lo + x.shape[2]) of a
    level of height src_glob.  Source rows outside the slab are clamped (only
    halo rows can need them; the halo absorbs the error)."""
    l0, l1, lam, one_m_lam = _interp_index(src_lo, src_glob, dst_lo, dst_hi, dst_glob, x.shape[2], x.device)
    rows = x[:, :, l0] * one_m_lam + x[:, :, l1] * lam      # fp32 weights, promoted as before
    return torch.nn.functional.interpolate(rows, (dst_hi - dst_lo, dst_w), mode="bilinear",
                                           align_corners=True)


class _Rows:
    """Rows [g0, g0 + t.shape[2]) of a feature level of global height H
    (held rows outside [0, H), if any, are zeros)."""
    __slots__ = ("t", "g0", "H")

    def __init__(self, t, g0, H):
        self.t, self.g0, self.H = t, g0, H

    @property
    def g1(self):
        return self.g0 + self.t.shape[2]

    def clip(self, lo, hi):
        """[lo, hi) cut to the image; raises if a row inside it is not held
        (a halo too small for the op that asked)."""
        s0, s1 = max(lo, 0), min(hi, self.H)
        if s0 < max(self.g0, 0) or s1 > min(self.g1, self.H):
            raise RuntimeError(f"rows [{lo}, {hi}) of a level of {self.H} rows requested from "
                               f"the held rows [{self.g0}, {self.g1})")
        return s0, s1

    def rows(self, lo, hi):
        """Global rows [lo, hi); rows outside [0, H) are zeros -- the zero
        padding the full-image op applies there (a view when held)."""
        if self.g0 <= lo and hi <= self.g1:
            return self.t[:, :, lo - self.g0:hi - self.g0]
        s0, s1 = self.clip(lo, hi)
        return F.pad(self.t[:, :, s0 - self.g0:s1 - self.g0], (0, 0, s0 - lo, hi - s1))


class _Conv:
    """weight / bias with another conv's geometry (padding, stride, dilation,
    groups), for _conv_rows."""
    __slots__ = ("weight", "bias", "padding", "stride", "dilation", "groups")

    def __init__(self, weight, bias, like):
        self.weight, self.bias = weight, bias
        self.padding, self.stride, self.dilation, self.groups = like.padding, like.stride, like.dilation, like.groups


def _conv_rows(conv, x, lo, hi):
    """``conv`` (stride 1, zero 'same' padding) evaluated on output rows
    [lo, hi) only, clipped to the level: the full-image op's values on those
    rows.  It reads the held input rows [lo - p, hi + p) with no row padding;
    where that range leaves the image, the conv's own zero padding supplies
    the missing rows (the extra output rows of an asymmetric edge are cut)."""
    lo, hi = max(lo, 0), min(hi, x.H)
    p, pw = conv.padding
    if x.g0 <= lo - p and hi + p <= x.g1:
        y = F.conv2d(x.rows(lo - p, hi + p), conv.weight, conv.bias, conv.stride, (0, pw),
                     conv.dilation, conv.groups)
    else:
        s0, s1 = x.clip(lo - p, hi + p)
        m = max(s0 - (lo - p), (hi + p) - s1)          # zero rows the image edge supplies
        y = F.conv2d(x.t[:, :, s0 - x.g0:s1 - x.g0], conv.weight, conv.bias, conv.stride, (m, pw),
                     conv.dilation, conv.groups)
        k0 = lo - s0 + m - p
        if k0 or y.shape[2] != hi - lo:
            y = y[:, :, k0:k0 + hi - lo]
    return _Rows(y, lo, x.H)


def _pool_rows(x, lo, hi, H):
    """pool2x (model.py:182-183: 3x3, stride 2, zero padding counted) of the
    level held by ``x`` on output rows [lo, hi) of the pooled level (height
    ``H``): input rows [2lo-1, 2hi), the image's zero rows supplied by the
    pool's own padding where the stride grid allows, else explicitly -- every
    window is 3 full rows, as in the full op."""
    lo, hi = max(lo, 0), min(hi, H)
    a, b = 2 * lo - 1, 2 * hi
    if x.g0 <= a and b <= x.g1:
        y = F.avg_pool2d(x.rows(a, b), 3, stride=2, padding=(0, 1))
    else:
        s0, s1 = x.clip(a, b)
        if s0 - a == 1:            # the top image edge: the pool's padding row, grid aligned
            y = F.avg_pool2d(x.t[:, :, s0 - x.g0:s1 - x.g0], 3, stride=2, padding=1)
            if y.shape[2] != hi - lo:
                y = y[:, :, :hi - lo]
        else:
            y = F.avg_pool2d(x.rows(a, b), 3, stride=2, padding=(0, 1))
    return _Rows(y, lo, H)


def _interp_rows_held(x, lo, hi, H, W):
    """interp (model.py:184-186: bilinear, align_corners=True) of the level
    held by ``x`` to a level of H x W, on destination rows [lo, hi) only; the
    source rows the global row mapping reads must be held."""
    lo, hi = max(lo, 0), min(hi, H)
    scale = (x.H - 1) / (H - 1) if H > 1 else 0.0
    # the source rows _interp_rows reads, in its own fp32 arithmetic
    ends = (torch.tensor([lo, hi - 1], dtype=torch.float32) * scale).clamp(max=x.H - 1).floor()
    need0, need1 = int(ends[0]), min(int(ends[1]) + 2, x.H)
    if need0 < x.g0 or need1 > x.g1:
        raise RuntimeError(f"interp rows [{lo}, {hi}) need source rows [{need0}, {need1}) of "
                           f"the held [{x.g0}, {x.g1})")
    return _Rows(_interp_rows(x.t, x.g0, x.H, lo, hi, H, W), lo, H)


def _relu(x):
    return _Rows(F.relu(x.t), x.g0, x.H)


def _cat_rows(parts, lo, hi):
    """Channel concatenation of several _Rows on rows [lo, hi) cut to the
    image (one copy, as the full op's torch.cat)."""
    s0, s1 = parts[0].clip(lo, hi)
    return _Rows(torch.cat([p.rows(s0, s1) for p in parts], 1), s0, parts[0].H)


_ZR = weakref.WeakKeyDictionary()   # ConvGRU -> (weight, bias, C, tag): convz and convr stacked


def _zr_conv(gru):
    """convz and convr as ONE conv (weights stacked along the output channels):
    the same per-channel sums, one launch instead of two and no sliced input
    for convz -- at 60-row slabs each launch's fixed cost matters (DESIGN.md
    §5).  Cached per module only while no gradient is recorded (a cached
    autograd node could not be back-propagated twice); the cache entry is
    keyed on each weight's storage, in-place version, dtype and device, so
    ``.to()`` / ``.double()`` / ``load_state_dict`` (which keep the Parameter
    object) rebuild it."""
    wz, wr = gru.convz.weight, gru.convr.weight
    bz, br = gru.convz.bias, gru.convr.bias
    ws = [t for t in (wz, wr, bz, br) if t is not None]
    if torch.is_grad_enabled() and any(t.requires_grad for t in ws):
        w = torch.cat([wz, wr], 0)
        return w, (None if bz is None else torch.cat([bz, br], 0)), wz.shape[0]
    tag = tuple((t.data_ptr(), t._version, t.dtype, t.device) for t in ws)
    hit = _ZR.get(gru)
    if hit is None or hit[3] != tag:
        w = torch.cat([wz, wr], 0)
        b = None if bz is None else torch.cat([bz, br], 0)
        hit = _ZR[gru] = (w, b, wz.shape[0], tag)
    return hit[0], hit[1], hit[2]


def _gru_rows(gru, h, cz, cr, cq, xs, lo, hi, fuse_zr=True):
    """ConvGRU.forward (model.py:164-179) on output rows [lo, hi): z on
    [lo, hi), r on the rows convq reads, both from [h, x] on one more cone
    of rows; r*h and x zero outside the image as the full op pads them.
    ``h``, ``cz``, ``cr``, ``cq`` and each of ``xs`` are _Rows holding
    enough rows.  ``fuse_zr``: convz and convr as one stacked conv over r's
    rows (z's rows cut from it).  Returns the new hidden state's rows [lo, hi)."""
    H = h.H
    p, pq = gru.convz.padding[0], gru.convq.padding[0]
    ra, rb = max(lo - pq, 0), min(hi + pq, H)                 # rows of r (convq's input)
    hx = _cat_rows([h] + list(xs), ra - p, rb + p)
    if fuse_zr and gru.convz.padding == gru.convr.padding and gru.convz.kernel_size == gru.convr.kernel_size:
        w, b, C = _zr_conv(gru)
        zr = _conv_rows(_Conv(w, b, gru.convz), hx, ra, rb).t
        z = torch.sigmoid(zr[:, :C, lo - ra:hi - ra] + cz.rows(lo, hi))
        r = torch.sigmoid(zr[:, C:] + cr.rows(ra, rb))
    else:
        z = torch.sigmoid(_conv_rows(gru.convz, hx, lo, hi).t + cz.rows(lo, hi))
        r = torch.sigmoid(_conv_rows(gru.convr, hx, ra, rb).t + cr.rows(ra, rb))
    rx = _cat_rows([_Rows(r * h.rows(ra, rb), ra, H)] + list(xs), ra, rb)
    q = torch.tanh(_conv_rows(gru.convq, rx, lo, hi).t + cq.rows(lo, hi))
    return (1 - z) * h.rows(lo, hi) + z * q


def _motion_rows(enc, corr, flow, lo, hi):
    """BasicMotionEncoder.forward (model.py:192-213) on output rows [lo, hi)
    from ``corr`` and ``flow`` _Rows holding the rows its cone reads."""
    k = enc.conv.padding[0]
    c = _relu(_conv_rows(enc.convc1, corr, lo - k - enc.convc2.padding[0],
                         hi + k + enc.convc2.padding[0]))
    c = _relu(_conv_rows(enc.convc2, c, lo - k, hi + k))
    f = _relu(_conv_rows(enc.convf1, flow, lo - k - enc.convf2.padding[0],
                         hi + k + enc.convf2.padding[0]))
    f = _relu(_conv_rows(enc.convf2, f, lo - k, hi + k))
    out = _relu(_conv_rows(enc.conv, _cat_rows([c, f], lo - k, hi + k), lo, hi))
    return _cat_rows([out, flow], out.g0, out.g1)


def _all_reduce_sum(t, group=None):
    """In-place SUM all-reduce (host-staged for gloo on CUDA tensors)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return t
    if _host_staged(t, group):
        h = t.cpu()
        dist.all_reduce(h, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, group=group)
    return t


def _instance_norm_rows(y, lo, hi, group, eps):
    """nn.InstanceNorm2d (affine=False, model.py:35-39 'instance') of a row
    SLAB with the statistics of the WHOLE image: every rank sums x and x^2
    over its owned rows [lo, hi) (the owned rows of all ranks partition the
    image), one all-reduce of 2*N*C+1 doubles, then the biased mean/var of
    the image normalise every slab row (halo rows included)."""
    yo = y[:, :, lo:hi].double()
    N, C = y.shape[:2]
    st = torch.cat([yo.sum((2, 3)).reshape(-1), (yo * yo).sum((2, 3)).reshape(-1),
                    torch.tensor([float((hi - lo) * y.shape[3])], dtype=torch.float64, device=y.device)])
    _all_reduce_sum(st, group)
    n = st[-1]
    mean = st[:N * C] / n
    var = (st[N * C:2 * N * C] / n - mean * mean).clamp_min(0)
    inv = torch.rsqrt(var + eps)
    # fp32 out, as InstanceNorm under autocast (fp64 stays fp64)
    dt = torch.promote_types(y.dtype, torch.float32)
    return (y.to(dt) - mean.view(N, C, 1, 1).to(dt)) * inv.view(N, C, 1, 1).to(dt)


class RowShardedStereo:
    """Row-sharded RAFT-Stereo forward over ``world`` ranks (one per GPU).

    * Encoders (``shard_encoders=True``, default):
      each rank runs cnet, conv2 and the context convs on its own band of
      image rows -- its GRU slab (below) plus ``enc_margin`` rows at 1/f res
      on either side, which cover the encoders' receptive field (the
      1/16-res heads and context convs reach past 128 full-res rows at
      f = 4: 32 rows left the slab's edge row at 1/16 res off by 4e-4, 48
      make every slab row equal to the full-image features), so the slab's
      features equal the full-image ones.  cnet's BatchNorms run on running stats in
      eval mode (per pixel); conv2's two InstanceNorms (model.py:35-39, :345)
      take image-wide statistics through one all-reduce each
      (``_instance_norm_rows``).  ``shard_encoders=False`` -- and any model
      in train mode, whose BatchNorms need batch statistics of the whole
      image -- runs the encoders replicated on the full image (no exchange;
      redundant encoder FLOPs).
    * Rank k owns 1/4-res feature rows [r0, r1) (multiples of 4) and keeps GRU
      state for the extended slab [r0 - halo, r1 + halo) (1/8 and 1/16 res:
      halo/2, halo/4).  The correlation pyramid is built for the slab's rows
      only -- the corr path is row-local (model.py:324, :299/:308).
    * Halo exchange (default ``per_stage=True``): the owned
      boundary rows of net[2] go to the two neighbours right after gru32, of
      net[1] after gru16, and of net[0] and coords1 at the end of the
      iteration (point-to-point send/recv: RCCL over xGMI on the GPU box), so
      the halo only has to cover one stage's dependency cone: 12 rows at 1/4
      res are exact to rounding (gloo, 3 ranks: 1.9e-6 px max; 8 rows
      5.7e-6; 4 rows 8.8e-3).  ``per_stage=False`` exchanges every level once
      per iteration and needs a halo covering the whole iteration's cone
      (<= 20 rows): ``halo`` defaults to 12 / 24 rows by mode, and a halo
      below 20 rows with ``per_stage=False`` raises ValueError.
    * ``forward`` returns the per-iteration flow of the OWNED rows;
      ``gather_rows`` assembles full-height tensors.
    """

    def __init__(self, model, rank, world, halo=None, group=None, shard_encoders=True, enc_margin=48,
                 per_stage=True, encoder_halos=True, overlap=True, per_conv=None, side_stream=True,
                 fuse_zr=True):
        # per_conv (the default unless a slab ``halo`` or per_stage=False is
        # asked for): GRU state on own rows, each conv evaluated on the rows its
        # readers need, halos exchanged per update (_forward_perconv)
        if per_conv is None:
            per_conv = halo is None and per_stage
        self.per_conv = bool(per_conv)
        # one stage's cone needs 12 rows; a whole iteration's up to 20
        if halo is None:
            halo = 12 if per_stage else 24
        if not per_stage and halo < 20:
            raise ValueError(f"halo={halo} < 20 rows: with per_stage=False the halo must cover "
                             "one whole iteration's dependency cone (SURVEY.md §8e)")
        if halo % 4:
            raise ValueError("halo must be a multiple of 4")
        if enc_margin % 4:
            raise ValueError("enc_margin must be a multiple of 4")
        self.model, self.rank, self.world, self.halo, self.group = model, rank, world, halo, group
        self.shard_encoders, self.enc_margin = shard_encoders, enc_margin
        self.per_stage = per_stage
        # encoder_halos (default): each encoder module runs on this rank's own
        # rows plus a halo refreshed from the neighbours right before it
        # (_features_halo); False: a band of enc_margin extra rows recomputed
        # locally (_features_rows)
        self.encoder_halos = encoder_halos
        # overlap (default, per_stage only): every halo exchange is posted as
        # soon as its rows are final and waited for only right before the first
        # op that reads the halo; the independent work in between (the next
        # GRU stage's inputs, the corr lookup, the motion encoder; the 1/8-res
        # heads and conv2 during layer4's exchanges) runs while it is in flight
        # (RCCL: on the comm stream).  Same ops on the same values: the result
        # equals the blocking order bit for bit.
        self.overlap = overlap
        # side_stream (per-conv mode, HIP tensors): each iteration's corr
        # lookup + motion encoder run on a second stream while the coarser
        # GRUs run on the current one -- two independent chains of small
        # kernels whose fixed per-launch cost dominates at 60-row slabs
        # (DESIGN.md §5); the same ops on the same values, so the result
        # agrees with the one-stream order within MIOpen's run-to-run noise
        # (measured 2-4e-6 px; tests/test_shard_gpu.py holds it to 1e-4 px)
        self.side_stream = side_stream
        # fuse_zr (per-conv mode): each ConvGRU's convz and convr as one conv
        # with stacked weights (_zr_conv): one launch instead of two
        self.fuse_zr = fuse_zr
        self._fake_xchg = False     # tools/shard_probe.py: time one rank's compute alone
        self.xchg_wait_s = 0.0      # host time spent blocked in exchange waits
        self.xchg_count = 0
        self.xchg_posts = 0         # halo exchanges posted (_halo_start)
        self.xchg_bytes = 0         # bytes received by them
        self.xchg_link_bytes = 0    # the larger neighbour's share of each

    # row geometry -----------------------------------------------------------
    def _ranges(self, H1):
        nblk = (H1 + 3) // 4
        b0, b1 = split_range(nblk, self.rank, self.world)
        r0, r1 = 4 * b0, min(4 * b1, H1)
        if self.world > 1 and (r1 - r0) < self.halo and self.rank < self.world - 1:
            raise ValueError(f"owned rows {r1 - r0} < halo {self.halo}: use fewer ranks or a smaller halo")
        e0, e1 = max(0, r0 - self.halo), min(H1, r1 + self.halo)
        return r0, r1, e0, e1

    @staticmethod
    def _lvl(lo, hi, l):
        d = 1 << l
        return lo // d, -(-hi // d)

    def _exchange(self, t, l, own, ext, glob):
        """Refresh the halo rows of a level-l slab from the two neighbours.
        Level-l rows: owned [r0, r1), slab [e0, e1), level height ``glob``,
        halo h = halo >> l.  I send prev my rows [r0, min(glob, r0+h, r1)) (its
        bottom halo) and next my rows [max(r0, r1-h), r1) (its top halo); I
        receive [e0, r0) and [r1, e1).  Sizes agree because every rank but
        the last owns >= halo rows."""
        return self._exchange_finish(self._exchange_start(t, l, own, ext, glob))

    def _exchange_start(self, t, l, own, ext, glob):
        """Post _exchange's sends and receives and return a handle for
        _exchange_finish; ``t`` is only read (the sends are copies)."""
        if self.world == 1:
            return (t, None, [], False, t.device, [])
        (r0, r1), (e0, e1) = own, ext
        h = self.halo >> l
        dev = t.device
        staged = _host_staged(t, self.group)
        if staged:
            t = t.cpu()
        ops, recv, sends = [], [], []
        prev, nxt = self.rank - 1, self.rank + 1
        if prev >= 0:
            buf = torch.empty_like(t[:, :, 0:r0 - e0]).contiguous()
            ops.append(dist.P2POp(dist.irecv, buf, prev, group=self.group))
            recv.append((buf, 0))
            hi = min(glob, r0 + h, r1)
            sends.append(t[:, :, r0 - e0:hi - e0].clone(memory_format=torch.contiguous_format))
            ops.append(dist.P2POp(dist.isend, sends[-1], prev, group=self.group))
        if nxt < self.world:
            buf = torch.empty_like(t[:, :, r1 - e0:e1 - e0]).contiguous()
            ops.append(dist.P2POp(dist.irecv, buf, nxt, group=self.group))
            recv.append((buf, r1 - e0))
            lo = max(r0, r1 - h)
            sends.append(t[:, :, lo - e0:r1 - e0].clone(memory_format=torch.contiguous_format))
            ops.append(dist.P2POp(dist.isend, sends[-1], nxt, group=self.group))
        reqs = dist.batch_isend_irecv(ops) if ops else []
        return (t, reqs, recv, staged, dev, sends)

    def _exchange_finish(self, hd):
        """Wait for a posted exchange; the slab with its halo rows refreshed."""
        t, reqs, recv, staged, dev, _sends = hd
        if reqs is None:
            return t
        t0 = time.perf_counter()
        for req in reqs:
            req.wait()
        self.xchg_wait_s += time.perf_counter() - t0
        self.xchg_count += 1
        if recv:
            t = t.clone()
            for buf, at in recv:
                t[:, :, at:at + buf.shape[2]] = buf
        return t.to(dev) if staged else t

    # encoders ---------------------------------------------------------------
    @staticmethod
    def _heights(H, n_down, nl):
        """Global row counts of the 1/f, 1/2f, 1/4f feature levels for an image
        of H rows (each stride-2 3x3 conv with padding 1 maps h -> ceil(h/2))."""
        h = H
        for _ in range(n_down):
            h = (h + 1) // 2
        glob = [h]
        for _ in range(1, nl):
            glob.append((glob[-1] + 1) // 2)
        return glob

    def _features_rows(self, image1, image2, e0, e1, r0, r1):
        """RAFTStereo.features (model.py:339-364) on a band of image rows.
        Returns the slab [e0, e1) of fmap1/fmap2 (1/f res) and of every GRU
        level's net / inp tensors -- equal to slicing the full-image features."""
        m, a = self.model, self.model.args
        if m.training:
            raise RuntimeError("RowShardedStereo: encoder row sharding needs eval mode "
                               "(BatchNorm running statistics)")
        f = 2 ** a.n_downsample
        H = image1.shape[2]
        mg = self.enc_margin
        # band of 1/f rows [b0, b1): start a multiple of 4 (the 1/4f heads'
        # stride), so every strided conv of the band samples the global grid
        b0 = max(0, e0 - mg)
        b1 = min(-(-H // f), e1 + mg)
        s0, s1 = f * b0, min(H, f * b1)
        i1 = (2 * (image1[:, :, s0:s1] / 255.0) - 1.0).contiguous()
        i2 = (2 * (image2[:, :, s0:s1] / 255.0) - 1.0).contiguous()
        n = a.n_gru_layers
        with m._autocast():
            *cnet_list, x = m.cnet(torch.cat((i1, i2), dim=0), dual_inp=True, num_layers=n)
            blk, conv = m.conv2[0], m.conv2[1]
            lo, hi = r0 - b0, r1 - b0                      # owned rows, band-local
            eps = blk.norm1.eps
            y = blk.relu(_instance_norm_rows(blk.conv1(x), lo, hi, self.group, eps))
            y = blk.relu(_instance_norm_rows(blk.conv2(y), lo, hi, self.group, eps))
            fm = conv(x + y)
            fmap1, fmap2 = fm.split(dim=0, split_size=x.shape[0] // 2)
            net_list = [torch.tanh(pair[0]) for pair in cnet_list]
            inp_list = [torch.relu(pair[1]) for pair in cnet_list]
            inp_list = [list(c(i).split(dim=1, split_size=c.out_channels // 3))
                        for i, c in zip(inp_list, m.context_zqr_convs)]
        sl = slice(e0 - b0, e1 - b0)
        ext = [self._lvl(e0, e1, l) for l in range(n)]
        bl = [b0 >> l for l in range(n)]
        net = [net_list[l][:, :, ext[l][0] - bl[l]:ext[l][1] - bl[l]] for l in range(n)]
        inp = [[c[:, :, ext[l][0] - bl[l]:ext[l][1] - bl[l]] for c in inp_list[l]] for l in range(n)]
        return fmap1[:, :, sl], fmap2[:, :, sl], net, inp

    # encoders with per-module halo exchange --------------------------------
    def _halo(self, t, lo, hi, Hg, h):
        """Slab of global rows [max(0, lo-h), min(Hg, hi+h)) from ``t`` (this
        rank's own rows [lo, hi) of a level of height Hg): the h rows on
        either side come from the neighbours' own boundary rows (every rank
        owns >= h rows of every level).  Returns (slab, first global row)."""
        return self._halo_finish(self._halo_start(t, lo, hi, Hg, h))

    def _halo_start(self, t, lo, hi, Hg, h):
        """Post _halo's exchange; a handle for _halo_finish."""
        g0, g1 = max(0, lo - h), min(Hg, hi + h)
        if self.world == 1 or h == 0:
            return ("done", t, lo)
        # message accounting (tools/shard_probe.py): rows received from each
        # neighbour; the two links run concurrently, so the larger side is the
        # exchange's per-link transfer
        row = t[:, :, :1].numel() * t.element_size()
        self.xchg_posts += 1
        self.xchg_bytes += (lo - g0 + g1 - hi) * row
        self.xchg_link_bytes += max(lo - g0, g1 - hi) * row
        if self._fake_xchg:          # timing probe: same shapes, no communication
            top = t.new_zeros(t.shape[:2] + (lo - g0,) + t.shape[3:])
            bot = t.new_zeros(t.shape[:2] + (g1 - hi,) + t.shape[3:])
            return ("done", torch.cat([top, t, bot], 2), g0)
        staged = _host_staged(t, self.group)
        src = t.cpu() if staged else t
        ops, top, bot, sends = [], None, None, []
        if lo > 0:
            top = torch.empty_like(src[:, :, :lo - g0]).contiguous()
            sends.append(src[:, :, :min(h, hi - lo)].clone(memory_format=torch.contiguous_format))
            ops += [dist.P2POp(dist.irecv, top, self.rank - 1, group=self.group),
                    dist.P2POp(dist.isend, sends[-1], self.rank - 1, group=self.group)]
        if hi < Hg:
            bot = torch.empty_like(src[:, :, :g1 - hi]).contiguous()
            sends.append(src[:, :, max(0, hi - lo - h):].clone(memory_format=torch.contiguous_format))
            ops += [dist.P2POp(dist.irecv, bot, self.rank + 1, group=self.group),
                    dist.P2POp(dist.isend, sends[-1], self.rank + 1, group=self.group)]
        return ("posted", t, g0, dist.batch_isend_irecv(ops), top, bot, staged, sends)

    def _halo_finish(self, hd):
        if hd[0] == "done":
            return hd[1], hd[2]
        _, t, g0, reqs, top, bot, staged, _sends = hd
        dev = t.device
        t0 = time.perf_counter()
        for req in reqs:
            req.wait()
        self.xchg_wait_s += time.perf_counter() - t0
        self.xchg_count += 1
        seq = ([top.to(dev) if staged else top] if top is not None else []) + [t]
        seq += [bot.to(dev) if staged else bot] if bot is not None else []
        return torch.cat(seq, 2), g0

    @staticmethod
    def _crop(y, lo, hi, g0, stride):
        """Own rows of a module output computed on a slab starting at global
        row g0 (even when stride == 2): returns (rows, lo', hi')."""
        if stride == 1:
            return y[:, :, lo - g0:hi - g0], lo, hi
        lo2, hi2 = lo // 2, (hi + 1) // 2
        return y[:, :, lo2 - g0 // 2:hi2 - g0 // 2], lo2, hi2

    def _run(self, mod, t, lo, hi, Hg, need, stride=1, slab=None):
        """Apply ``mod`` (receptive field +-need rows at its input, ``stride``
        1 or 2, padding preserving the grid) to own rows [lo, hi) of a level of
        height Hg; ``slab`` = an already exchanged (tensor, g0).  Returns the
        output's own rows and (lo, hi, Hg) at its level."""
        if stride == 2 and need % 2:
            need += 1                # the slab must start on an even row
        x, g0 = slab if slab is not None else self._halo(t, lo, hi, Hg, need)
        y, lo2, hi2 = self._crop(mod(x), lo, hi, g0, stride)
        return y, lo2, hi2, (Hg if stride == 1 else (Hg + 1) // 2)

    def _features_halo(self, image1, image2, r0, r1):
        """RAFTStereo.features (model.py:339-364) on this rank's OWN rows:
        every encoder module (stem, each ResidualBlock of layer1-5, each head,
        conv2, the context convs) runs on its own rows plus the halo its
        receptive field needs at that resolution (3x3 convs: 1 row each; a
        residual block 2; a stride-2 block 4 at its input), refreshed from the
        two neighbours right before it (_halo, point-to-point) -- SURVEY.md §8e
        item 2, without recomputing a margin.  The image itself is replicated,
        so the stem reads its rows directly.  conv2's InstanceNorms use
        image-wide statistics (one all-reduce each, _instance_norm_rows).
        Returns own rows of fmap1, fmap2 (1/f res) and of every level's net /
        inp tensors, with (lo, hi, H) per level."""
        m, a = self.model, self.model.args
        if m.training:
            raise RuntimeError("RowShardedStereo: encoder row sharding needs eval mode "
                               "(BatchNorm running statistics)")
        cn = m.cnet
        f = 2 ** a.n_downsample
        H = image1.shape[2]
        lo, hi = min(H, r0 * f), min(H, r1 * f)
        img = torch.cat(((2 * (image1 / 255.0) - 1.0), (2 * (image2 / 255.0) - 1.0)), 0)
        n = a.n_gru_layers
        B = image1.shape[0]
        with m._autocast():
            # stem: conv1 7x7 (+ BatchNorm, ReLU); the image is on every rank
            s0 = cn.conv1.stride[0]
            need = 4 if s0 == 2 else 3
            g0 = max(0, lo - need)
            stem = lambda z: cn.relu1(cn.norm1(cn.conv1(z)))  # noqa: E731
            x, lo, hi, Hg = self._run(stem, None, lo, hi, H, need, s0,
                                      slab=(img[:, :, g0:min(H, hi + need)].contiguous(), g0))
            for layer in (cn.layer1, cn.layer2, cn.layer3):
                for blk in layer:
                    st = blk.conv1.stride[0]
                    x, lo, hi, Hg = self._run(blk, x, lo, hi, Hg, 4 if st == 2 else 2, st)
            assert (lo, hi) == (r0, r1), (lo, hi, r0, r1)
            H1, levels = Hg, [(lo, hi, Hg)]
            xs = self._halo(x, lo, hi, Hg, 4)              # heads08, conv2 and layer4[0] read x

            def level0_heads():
                """heads08 and conv2 (ResidualBlock with InstanceNorm + 3x3
                conv, both images) on the exchanged slab xs."""
                o08 = [self._run(hd, None, lo, hi, Hg, 3, 1, slab=(xs[0][:B], xs[1]))[0]
                       for hd in cn.outputs08]
                blk2, conv = m.conv2[0], m.conv2[1]
                xx, gx = xs
                ol, oh = lo - gx, hi - gx                  # own rows, slab-local
                eps = blk2.norm1.eps
                y2 = blk2.relu(_instance_norm_rows(blk2.conv1(xx), ol, oh, self.group, eps))
                y2 = blk2.relu(_instance_norm_rows(blk2.conv2(y2), ol, oh, self.group, eps))
                fm = conv(xx + y2)[:, :, ol:oh]
                return o08, fm[:B], fm[B:]

            def chain(blocks, y, lo, hi, Hg, slab0, side):
                """Run residual blocks in turn, each on its input's halo slab;
                the first block's exchange of an output is posted before
                ``side()`` runs (overlap) and waited for after it."""
                done = side is None or not self.overlap
                ran, res = False, None
                for i, blk in enumerate(blocks):
                    st = blk.conv1.stride[0]
                    need = 4 if st == 2 else 2
                    if i == 0 and slab0 is not None:
                        y, lo, hi, Hg = self._run(blk, None, lo, hi, Hg, need, st, slab=slab0)
                        continue
                    if not done:
                        h = self._halo_start(y, lo, hi, Hg, need)
                        res, ran, done = side(), True, True
                        y, lo, hi, Hg = self._run(blk, None, lo, hi, Hg, need, st, slab=self._halo_finish(h))
                    else:
                        y, lo, hi, Hg = self._run(blk, y, lo, hi, Hg, need, st)
                if side is not None and not ran:
                    res = side()
                return y, lo, hi, Hg, res

            if n >= 2:
                # layer4[0] (stride 2, 4 rows of halo) reads the same slab xs;
                # the exchange of its output runs under heads08 + conv2
                y, lo, hi, Hg, (o08, fmap1, fmap2) = chain(
                    cn.layer4, None, lo, hi, Hg, (xs[0][:B], xs[1]), level0_heads)
                outs = [o08]
                levels.append((lo, hi, Hg))
                ys = self._halo(y, lo, hi, Hg, 4)          # heads16 and layer5[0] read it
                o16 = lambda: [self._run(hd, None, lo, hi, Hg, 3, 1, slab=ys)[0]  # noqa: E731
                               for hd in cn.outputs16]
                if n >= 3:
                    y, lo3, hi3, Hg3, o16v = chain(cn.layer5, None, lo, hi, Hg, ys, o16)
                    outs.append(o16v)
                    lo, hi, Hg = lo3, hi3, Hg3
                    levels.append((lo, hi, Hg))
                    zs = self._halo(y, lo, hi, Hg, 2)
                    outs.append([self._run(hd, None, lo, hi, Hg, 1, 1, slab=zs)[0] for hd in cn.outputs32])
                else:
                    outs.append(o16())
            else:
                o08, fmap1, fmap2 = level0_heads()
                outs = [o08]
            net = [torch.tanh(o[0]) for o in outs]
            # context convs: every level's exchange posted first, then each
            # level waited for and convolved in turn
            rel = [torch.relu(o[1]) for o in outs]
            hs = [self._halo_start(rel[l], *levels[l], 1) for l in range(len(outs))]
            inp = []
            for l, c in enumerate(m.context_zqr_convs[:len(outs)]):
                ql, qh, qH = levels[l]
                z = self._run(c, None, ql, qh, qH, 1, 1, slab=self._halo_finish(hs[l]))[0]
                inp.append(list(z.split(dim=1, split_size=c.out_channels // 3)))
        return fmap1, fmap2, net, inp, levels, H1

    def _gru_slabs(self, fmap1, fmap2, net, inp, levels):
        """Own rows -> the GRU slabs [e0, e1) (halo >> l at level l), one
        exchange per level (all of that level's tensors side by side)."""
        out_f, out_n, out_i = None, [], []
        for l, (lo, hi, Hg) in enumerate(levels):
            parts = ([fmap1, fmap2] if l == 0 else []) + [net[l]] + inp[l]
            sizes = [p.shape[1] for p in parts]
            dt = parts[0].dtype
            for p in parts[1:]:
                dt = torch.promote_types(dt, p.dtype)
            cat = torch.cat([p.to(dt) for p in parts], 1)
            slab, _ = self._halo(cat, lo, hi, Hg, self.halo >> l)
            pieces = list(slab.split(sizes, 1))
            pieces = [pc.to(p.dtype) for pc, p in zip(pieces, parts)]
            if l == 0:
                out_f = (pieces[0].contiguous(), pieces[1].contiguous())
                pieces = pieces[2:]
            out_n.append(pieces[0])
            out_i.append(pieces[1:])
        return out_f[0], out_f[1], out_n, out_i

    # per-conv halos (default) ---------------------------------------------
    def perconv_halos(self):
        """Rows of halo each GRU-loop tensor needs at its own level, from the
        receptive fields of the ops that read it (model.py:164-265):
          gp  = one ConvGRU's cone (convz/convr, then convq on r*h): 2 rows;
          net[l]: its own GRU (gp), the next coarser GRU's pool2x input
                  (2*gp + 1 = 5), the finer GRU's interp (<= gp), level 0
                  also the flow head (conv1 + conv2: 2);
          inp (context biases): convr's rows of r (1);
          fmaps: gru08's cone + the motion encoder's corr branch (1x1, 3x3,
                 3x3): 4 -- the corr block is built on own rows +- 4;
          coords1: gru08's cone + the flow branch (7x7, 3x3, 3x3): 7."""
        blk, n = self.model.update_block, self.model.args.n_gru_layers
        grus = [blk.gru08, blk.gru16, blk.gru32][:n]
        gp = [g.convz.padding[0] + g.convq.padding[0] for g in grus]
        enc, fh = blk.encoder, blk.flow_head
        k = enc.conv.padding[0]
        net = []
        for l in range(n):
            need = gp[l]
            if l == 0:
                need = max(need, fh.conv1.padding[0] + fh.conv2.padding[0])
            if l + 1 < n:
                need = max(need, 2 * gp[l + 1] + 1)
            if l > 0:
                need = max(need, gp[l - 1])
            net.append(need)
        return {"net": net, "inp": max(g.convq.padding[0] for g in grus),
                "fmap": gp[0] + k + enc.convc2.padding[0] + enc.convc1.padding[0],
                "coords": gp[0] + k + enc.convf2.padding[0] + enc.convf1.padding[0],
                "gp": gp}

    def _own_rows(self, glob, hz):
        """This rank's 1/4-res rows [r0, r1) (multiples of 4); every rank but
        the last must own at least the halo rows each level exchanges (a halo
        comes from the direct neighbour only)."""
        H1 = glob[0]
        nblk = (H1 + 3) // 4
        need = [max([hz["net"][l], hz["inp"]] + ([hz["coords"], hz["fmap"]] if l == 0 else []))
                for l in range(len(glob))]
        for k in range(self.world - 1):
            b0, b1 = split_range(nblk, k, self.world)
            for l, h in enumerate(need):
                lo, hi = self._lvl(4 * b0, min(4 * b1, H1), l)
                if hi - lo < h:
                    raise ValueError(f"rank {k} owns {hi - lo} rows at level {l} < the {h}-row "
                                     "halo: use fewer ranks")
        b0, b1 = split_range(nblk, self.rank, self.world)
        return 4 * b0, min(4 * b1, H1)

    def _perconv_state(self, image1, image2, r0, r1, glob, hz):
        """Encoders -> _Rows of fmap1, fmap2 (own rows +- the fmap halo),
        every level's net (own rows + its halo) and context biases (+- 1)."""
        m, n = self.model, self.model.args.n_gru_layers
        if self.shard_encoders and not m.training and self.encoder_halos:
            f1, f2, net, inp, levels, _ = self._features_halo(image1, image2, r0, r1)
            fS, netS, inpS = None, [], []
            for l, (lo, hi, Hg) in enumerate(levels):
                parts = ([f1, f2] if l == 0 else []) + [net[l]] + inp[l]
                h = max([hz["net"][l], hz["inp"]] + ([hz["fmap"]] if l == 0 else []))
                dt = parts[0].dtype
                for p in parts[1:]:
                    dt = torch.promote_types(dt, p.dtype)
                slab, g0 = self._halo(torch.cat([p.to(dt) for p in parts], 1), lo, hi, Hg, h)
                pieces = [pc.to(p.dtype) for pc, p in
                          zip(slab.split([p.shape[1] for p in parts], 1), parts)]
                if l == 0:
                    fS = (_Rows(pieces[0], g0, Hg), _Rows(pieces[1], g0, Hg))
                    pieces = pieces[2:]
                netS.append(_Rows(pieces[0], g0, Hg))
                inpS.append([_Rows(c, g0, Hg) for c in pieces[1:]])
            return fS, netS, inpS
        if self.shard_encoders and not m.training:
            # round 2's band encoders: a slab of own rows +- 12 (covers every
            # halo above at every level) with enc_margin recomputed rows
            H1 = glob[0]
            e0, e1 = max(0, r0 - 12), min(H1, r1 + 12)
            f1, f2, net, inp = self._features_rows(image1, image2, e0, e1, r0, r1)
            g = [self._lvl(e0, e1, l)[0] for l in range(n)]
            return ((_Rows(f1, e0, H1), _Rows(f2, e0, H1)),
                    [_Rows(net[l], g[l], glob[l]) for l in range(n)],
                    [[_Rows(c, g[l], glob[l]) for c in inp[l]] for l in range(n)])
        # replicated encoders (or train mode): the full image's features
        f1, f2, net, inp = m.features(image1, image2)
        return ((_Rows(f1, 0, glob[0]), _Rows(f2, 0, glob[0])),
                [_Rows(net[l], 0, glob[l]) for l in range(n)],
                [[_Rows(c, 0, glob[l]) for c in inp[l]] for l in range(n)])

    def _forward_perconv(self, image1, image2, iters):
        """The GRU loop with per-conv halos: every tensor lives on the rank's
        OWN rows; each op is evaluated on exactly the rows its consumers read
        (_conv_rows, _pool_rows, _interp_rows_held: the full-image op's values
        there, zero padding at the image edges), and after each update the
        new rows' halo (perconv_halos) is posted to the two neighbours and
        waited for at its first reader:
          gru32 -> post net[2] | wait coords1 (previous iteration); corr
                               | lookup on own rows +- 4; flow; motion encoder
          wait net[2] -> gru16 -> post net[1]
          wait net[1] -> gru08 -> post net[0] -> wait -> flow head on own rows
          coords1 update -> post coords1 | next iteration's gru32
        Nothing is recomputed beyond the halo rows a conv's own receptive field
        needs, so per-rank work is own rows + O(1) rows per conv (the slab of
        the per-stage mode carried 12 extra rows on either side)."""
        m, a = self.model, self.model.args
        blk, n = m.update_block, a.n_gru_layers
        glob = self._heights(image1.shape[2], a.n_downsample, n)
        H1 = glob[0]
        hz = self.perconv_halos()
        r0, r1 = self._own_rows(glob, hz)
        own = [self._lvl(r0, r1, l) for l in range(n)]
        fS, netS, inpS = self._perconv_state(image1, image2, r0, r1, glob, hz)
        c0, c1 = max(0, r0 - hz["fmap"]), min(H1, r1 + hz["fmap"])
        corr_fn = m.corr_block(fS[0].rows(c0, c1).contiguous(), fS[1].rows(c0, c1).contiguous(),
                               radius=a.corr_radius, num_levels=a.corr_levels)
        del fS
        B, W1 = netS[0].t.shape[0], netS[0].t.shape[3]
        widths = [netS[l].t.shape[3] for l in range(n)]
        grid = coords_grid(B, H1, W1).to(netS[0].t.device)
        hc = hz["coords"]
        k0, k1 = max(0, r0 - hc), min(H1, r1 + hc)
        coords0 = grid[:, :, k0:k1]
        state = {"net0": netS[0], "coords": _Rows(coords0.clone(), k0, H1)}
        if n > 1:
            state["net1"] = netS[1]
        if n > 2:
            state["net2"] = netS[2]
        gp = hz["gp"]

        def post(key, t, l, h):
            hd = self._halo_start(t, own[l][0], own[l][1], glob[l], h)
            state[key] = ("pending", hd, glob[l])
            if not self.overlap:
                get(key)

        def get(key):
            v = state[key]
            if isinstance(v, tuple):
                t, g0 = self._halo_finish(v[1])
                v = state[key] = _Rows(t, g0, v[2])
            return v

        def gru(l, xs):
            g = (blk.gru08, blk.gru16, blk.gru32)[l]
            lo, hi = own[l]
            h = _gru_rows(g, get(f"net{l}"), *inpS[l], xs, lo, hi, fuse_zr=self.fuse_zr)
            post(f"net{l}", h, l, hz["net"][l])

        def gru32():
            lo, hi = own[2]
            gru(2, [_pool_rows(get("net1"), lo - gp[2], hi + gp[2], glob[2])])

        def gru16():
            lo, hi = own[1]
            xs = [_pool_rows(get("net0"), lo - gp[1], hi + gp[1], glob[1])]
            if n == 3:
                xs.append(_interp_rows_held(get("net2"), lo - gp[1], hi + gp[1], glob[1], widths[1]))
            gru(1, xs)

        preds = []
        lo0, hi0 = own[0]
        fh = blk.flow_head
        p2 = fh.conv2.padding[0]
        dev = netS[0].t.device
        side = None
        if self.side_stream and dev.type == "cuda":      # one side stream per instance and device
            if getattr(self, "_side", None) is None or self._side.device != dev:
                self._side = torch.cuda.Stream(dev)
            side = self._side

        def motion_chain():
            """corr lookup + motion encoder of this iteration (current stream)."""
            cS = get("coords")
            corr = _Rows(corr_fn(cS.rows(c0, c1).contiguous()), c0, H1)
            flow = _Rows(cS.t - coords0, k0, H1)
            with m._autocast():
                motion = _motion_rows(blk.encoder, corr, flow, lo0 - gp[0], hi0 + gp[0])
            return cS, motion

        def gru08(motion):
            with m._autocast():
                xs = [motion]
                if n > 1:
                    xs.append(_interp_rows_held(get("net1"), lo0 - gp[0], hi0 + gp[0], glob[0],
                                                widths[0]))
                gru(0, xs)

        def flow_head(cS):
            """flow head, coords update and its exchange (current stream)."""
            with m._autocast():
                hid = _relu(_conv_rows(fh.conv1, get("net0"), lo0 - p2, hi0 + p2))
                delta = _conv_rows(fh.conv2, hid, lo0, hi0).t
            delta = delta.float()
            delta[:, 1] = 0.0
            c_own = cS.rows(lo0, hi0) + delta
            preds.append(c_own - grid[:, :, lo0:hi0])
            post("coords", c_own, 0, hc)

        if side is not None and n == 3 and not a.slow_fast_gru:
            # the default schedule as a two-stream pipeline: this stream runs
            # gru16 and gru08; the side stream runs the corr lookup + motion
            # encoder, the next iteration's gru32 (inputs: this iteration's
            # net1 and net2) and the flow head + coords update (input: gru08's
            # net0), each behind the event of what it reads.  Every exchange
            # a stream reads is completed (get) on this stream before the side
            # stream is ordered after it; tensors made on the side stream and
            # read here are record_stream-ed.
            main = torch.cuda.current_stream(dev)
            with m._autocast():
                gru32()
            get("coords")
            side.wait_stream(main)
            with torch.cuda.stream(side):
                cS, motion = motion_chain()
            e32 = None
            for it in range(iters):
                if e32 is not None:
                    main.wait_event(e32)
                with m._autocast():
                    gru16()
                main.wait_stream(side)
                motion.t.record_stream(main)
                last = it + 1 == iters
                if not last:
                    get("net1")
                    side.wait_stream(main)
                    with torch.cuda.stream(side):
                        with m._autocast():
                            gru32()
                        e32 = side.record_event()
                gru08(motion)
                get("net0")
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    flow_head(cS)
                    if not last:
                        cS, motion = motion_chain()
            main.wait_stream(side)
            for p_ in preds:
                p_.record_stream(main)
        else:
            for _ in range(iters):
                with m._autocast():
                    if n == 3 and a.slow_fast_gru:
                        gru32()
                    if n >= 2 and a.slow_fast_gru:
                        if n == 3:
                            gru32()
                        gru16()
                    if n == 3:
                        gru32()
                if side is not None:      # the motion chain on the side stream, gru16 on this one
                    main = torch.cuda.current_stream(dev)
                    get("coords")
                    side.wait_stream(main)
                    with torch.cuda.stream(side):
                        cS, motion = motion_chain()
                    with m._autocast():
                        if n >= 2:
                            gru16()
                    main.wait_stream(side)
                    motion.t.record_stream(main)
                else:
                    cS, motion = motion_chain()
                    with m._autocast():
                        if n >= 2:
                            gru16()
                gru08(motion)
                flow_head(cS)
        for key in list(state):         # drain the last iteration's exchanges
            get(key)
        return preds

    # forward ----------------------------------------------------------------
    def forward(self, image1, image2, iters=12):
        m, a = self.model, self.model.args
        nl = a.n_gru_layers
        if self.per_conv:
            return self._forward_perconv(image1, image2, iters)
        # train-mode BatchNorm needs the whole image's batch statistics: the
        # replicated encoders give exactly the unsharded network's features
        if self.shard_encoders and not m.training:
            glob = self._heights(image1.shape[2], a.n_downsample, nl)
            H1 = glob[0]
            r0, r1, e0, e1 = self._ranges(H1)
            if self.encoder_halos:
                f1o, f2o, no, io, lv, _ = self._features_halo(image1, image2, r0, r1)
                assert [h for _, _, h in lv] == glob, (lv, glob)
                fmap1, fmap2, net, inp = self._gru_slabs(f1o, f2o, no, io, lv)
            else:
                fmap1, fmap2, net, inp = self._features_rows(image1, image2, e0, e1, r0, r1)
        else:
            fmap1, fmap2, net_full, inp_full = m.features(image1, image2)
            H1 = fmap1.shape[2]
            r0, r1, e0, e1 = self._ranges(H1)
            glob = [t.shape[2] for t in net_full]
            ext0 = [self._lvl(e0, e1, l) for l in range(nl)]
            net = [net_full[l][:, :, ext0[l][0]:ext0[l][1]] for l in range(nl)]
            inp = [[c[:, :, ext0[l][0]:ext0[l][1]] for c in inp_full[l]] for l in range(nl)]
            fmap1, fmap2 = fmap1[:, :, e0:e1], fmap2[:, :, e0:e1]
        own = [self._lvl(r0, r1, l) for l in range(nl)]
        ext = [self._lvl(e0, e1, l) for l in range(nl)]
        corr_fn = m.corr_block(fmap1.contiguous(), fmap2.contiguous(),
                               radius=a.corr_radius, num_levels=a.corr_levels)
        B, _, _, W1 = fmap1.shape
        coords0 = coords_grid(B, H1, W1).to(fmap1.device)[:, :, e0:e1]
        coords1 = coords0.clone()
        blk = m.update_block
        n = a.n_gru_layers

        def interp(x, ls, ld):
            return _interp_rows(x, ext[ls][0], glob[ls], ext[ld][0], ext[ld][1], glob[ld],
                                net[ld].shape[3])

        # per_stage: refresh net[2] after gru32 and net[1] after gru16 as well
        # (the exchange per stage), so the halo only has to cover
        # one stage's cone instead of a whole iteration's
        xch = ((lambda t, l: self._exchange(t, l, own[l], ext[l], glob[l])) if self.per_stage
               else None)
        preds = []
        if self.per_stage and self.overlap:
            return self._forward_overlap(corr_fn, coords0, coords1, net, inp, interp, iters, own, ext,
                                         glob, r0 - e0, r1 - e0)
        for _ in range(iters):
            corr = corr_fn(coords1)
            flow = coords1 - coords0
            with m._autocast():
                if n == 3 and a.slow_fast_gru:
                    self._gru(blk, net, inp, None, None, interp, True, False, False, xch)
                if n >= 2 and a.slow_fast_gru:
                    self._gru(blk, net, inp, None, None, interp, n == 3, True, False, xch)
                delta = self._gru(blk, net, inp, corr, flow, interp, n == 3, n >= 2, True, xch)
            delta[:, 1] = 0.0
            coords1 = coords1 + delta.float()
            preds.append((coords1 - coords0)[:, :, r0 - e0:r1 - e0])
            for l in range(1 if self.per_stage else nl):
                net[l] = self._exchange(net[l], l, own[l], ext[l], glob[l])
            coords1 = self._exchange(coords1, 0, own[0], ext[0], glob[0])
        return preds

    def _forward_overlap(self, corr_fn, coords0, coords1, net, inp, interp, iters, own, ext, glob,
                         o0, o1):
        """The per-stage loop of ``forward`` with every exchange posted when
        its rows are final and waited for right before its first reader
        (model.py:374-383 order per tensor, so the values are those of the
        blocking loop bit for bit):
          gru32 -> post net[2]  | corr lookup + flow (after coords1 / net[0] of
                                |   the previous iteration arrive)
          wait net[2] -> gru16 -> post net[1] | motion encoder (flow, corr)
          wait net[1] -> gru08 -> flow head -> coords1 update
          post net[0] and coords1 | next iteration's gru32 (reads net[1],
                                  |   net[2] only)."""
        from .network import pool2x
        m, a = self.model, self.model.args
        blk = m.update_block
        n = a.n_gru_layers
        X = lambda t, l: self._exchange_start(t, l, own[l], ext[l], glob[l])  # noqa: E731
        W = self._exchange_finish
        preds, pend = [], None          # pend: (net[0], coords1) exchanges in flight

        def settle():
            nonlocal pend, coords1
            if pend is not None:
                net[0], coords1 = W(pend[0]), W(pend[1])
                pend = None

        for _ in range(iters):
            with m._autocast():
                if n == 3 and a.slow_fast_gru:       # gru32 only: needs net[1], net[2]
                    net[2] = W(X(blk.gru32(net[2], *inp[2], pool2x(net[1])), 2))
                if n >= 2 and a.slow_fast_gru:
                    if n == 3:
                        net[2] = W(X(blk.gru32(net[2], *inp[2], pool2x(net[1])), 2))
                    settle()                         # gru16 pools net[0]
                    extra = (interp(net[2], 2, 1),) if n > 2 else ()
                    net[1] = W(X(blk.gru16(net[1], *inp[1], pool2x(net[0]), *extra), 1))
                h2 = X(blk.gru32(net[2], *inp[2], pool2x(net[1])), 2) if n == 3 else None
            settle()
            corr = corr_fn(coords1)
            flow = coords1 - coords0
            with m._autocast():
                if n >= 2:
                    if h2 is not None:
                        net[2] = W(h2)
                    extra = (interp(net[2], 2, 1),) if n > 2 else ()
                    h1 = X(blk.gru16(net[1], *inp[1], pool2x(net[0]), *extra), 1)
                    motion = blk.encoder(flow, corr)
                    net[1] = W(h1)
                else:
                    motion = blk.encoder(flow, corr)
                extra = (interp(net[1], 1, 0),) if n > 1 else ()
                net[0] = blk.gru08(net[0], *inp[0], motion, *extra)
                delta = blk.flow_head(net[0])
            delta[:, 1] = 0.0
            coords1 = coords1 + delta.float()
            preds.append((coords1 - coords0)[:, :, o0:o1])
            pend = (X(net[0], 0), X(coords1, 0))
        settle()
        return preds

    @staticmethod
    def _gru(blk, net, inp, corr, flow, interp, iter32, iter16, iter08, xch=None):
        """BasicMultiUpdateBlock.forward (model.py:242-265) on a slab, with the
        global-row interp; returns delta_flow when iter08.  ``xch(t, level)``
        (per-stage mode) refreshes a level's halo rows after its update."""
        from .network import pool2x
        n = blk.args.n_gru_layers
        if iter32:
            net[2] = blk.gru32(net[2], *inp[2], pool2x(net[1]))
            if xch is not None:
                net[2] = xch(net[2], 2)
        if iter16:
            extra = (interp(net[2], 2, 1),) if n > 2 else ()
            net[1] = blk.gru16(net[1], *inp[1], pool2x(net[0]), *extra)
            if xch is not None:
                net[1] = xch(net[1], 1)
        if iter08:
            motion = blk.encoder(flow, corr)
            extra = (interp(net[1], 1, 0),) if n > 1 else ()
            net[0] = blk.gru08(net[0], *inp[0], motion, *extra)
            return blk.flow_head(net[0])
        return None

    def gather_rows(self, local):
        """all_gather of per-rank owned-row slabs -> full-height tensor."""
        if self.world == 1:
            return local
        dev = local.device
        if _host_staged(local, self.group):
            local = local.cpu()
        n = torch.tensor([local.shape[2]], device=local.device)
        sizes = [torch.zeros_like(n) for _ in range(self.world)]
        dist.all_gather(sizes, n, group=self.group)
        sizes = [int(s.item()) for s in sizes]
        cap = max(sizes)
        pad = torch.zeros(local.shape[:2] + (cap,) + local.shape[3:], dtype=local.dtype,
                          device=local.device)
        pad[:, :, :local.shape[2]] = local
        bufs = [torch.empty_like(pad) for _ in range(self.world)]
        dist.all_gather(bufs, pad, group=self.group)
        return torch.cat([b[:, :, :s] for b, s in zip(bufs, sizes)], dim=2).to(dev)
