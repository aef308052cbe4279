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
again with no exchange.  (The GRU's halo exchange for a fully row-sharded
network is outside the corr path; see DESIGN.md.)
"""
import torch
import torch.distributed as dist

from .corr import CorrBlock1D


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
    return torch.cat([b[:s] for b, s in zip(bufs, sizes)], dim=0)


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
