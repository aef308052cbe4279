"""Multi-process (gloo, world_size 2, CPU) tests of the partitioning logic.
The correlation block is the oracle's ATen restatement here (the HIP path
needs a GPU); the partitioning code under test is the same."""
import queue
import socket
import time

import pytest
import torch
import torch.multiprocessing as mp

import dist_worker
from oracle import torch_ref
from raft_stereo_amd.shard import split_range


def test_split_range_covers_exactly():
    for n in (0, 1, 7, 8, 135, 496):
        for world in (1, 2, 3, 4, 8):
            got = [split_range(n, r, world) for r in range(world)]
            assert got[0][0] == 0 and got[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(got, got[1:]))
            assert max(e - s for s, e in got) - min(e - s for s, e in got) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(target, world, *args):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    return _collect(procs, q, world)


def _collect(procs, q, world):
    res, deadline = {}, time.time() + 300
    try:
        while len(res) < world:
            try:
                rank, full, rows = q.get(timeout=5)
                res[rank] = (full, rows)
            except queue.Empty:
                dead = [p for p in procs if p.exitcode not in (None, 0)]
                assert not dead, f"worker died: {[p.exitcode for p in dead]}"
                assert time.time() < deadline, "timeout waiting for workers"
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert not isinstance(res[r][0], str), res[r][0]
    return res


def test_gloo_world2_batch_and_row_sharding():
    world = 2
    res = _spawn(dist_worker.run, world)
    img1, img2 = dist_worker.pairs()
    with torch.no_grad():
        ref = dist_worker.model()(img1, img2, iters=3)[-1]
    for r in range(world):
        assert res[r][0].shape == ref.shape
        assert torch.allclose(res[r][0], ref, atol=1e-4, rtol=0)
    f1, f2, coords = dist_worker.row_case()
    assert torch.equal(res[0][1], torch_ref.TorchCorrBlock1D(f1, f2, 3, 3)(coords))


@pytest.mark.parametrize("world,halo,H,W,shard_enc,per_stage", [
    (2, 32, 320, 96, False, False), (3, 24, 320, 96, True, False),
    (3, 12, 320, 96, True, True), (2, 12, 800, 64, True, True)])
def test_gloo_row_sharded_network(world, halo, H, W, shard_enc, per_stage):
    """Full network row-sharded over ``world`` ranks (GRU halo exchange by
    point-to-point send/recv each iteration) == unsharded forward.  H=320 ->
    80 feature rows: 40/40 rows with a 32-row halo, 28/28/24 with 24.  A halo
    that covers the one-iteration cone (<= 20 rows) is exact to
    rounding (measured 3.8e-6 px max); 8 rows gives 1.3e-4, 4 rows 6e-3.
    ``shard_enc``: the encoders run on each rank's band of image rows with
    all-reduced InstanceNorm statistics (H=800: the bands do not cover the
    image) instead of replicated on the full image.  ``per_stage``: halos
    refreshed after each GRU stage, so 12 rows suffice (the default)."""
    iters = 4
    res = _spawn(dist_worker.run_rows, world, halo, H, W, iters, shard_enc, per_stage)
    g = torch.Generator().manual_seed(3)
    img1 = torch.rand(1, 3, H, W, generator=g) * 255
    img2 = torch.roll(img1, -4, dims=-1)
    with torch.no_grad():
        ref = torch.stack(dist_worker.model()(img1, img2, iters=iters))
    for r in range(world):
        got = res[r][0]
        assert got.shape == ref.shape
        assert (got - ref).abs().max() < 5e-5, (got - ref).abs().max()
        assert (got - ref).abs().mean() < 1e-6


@pytest.mark.parametrize("world,slow_fast", [(3, False), (2, True)])
def test_gloo_overlapped_exchanges_equal_blocking(world, slow_fast):
    """with ``overlap`` (the default) every halo exchange
    -- the encoders' per-module halos and the GRU's per-stage ones -- is
    posted when its rows are final and waited for right before its first
    reader, with independent work in between (model.py:374-383 per tensor);
    the per-iteration flows equal the blocking order's bit for bit, with and
    without the slow-fast GRU schedule."""
    H, W, iters = 800, 64, 3
    got = {}
    for overlap in (True, False):
        res = _spawn(dist_worker.run_rows, world, 12, H, W, iters, True, True, overlap, slow_fast)
        got[overlap] = res[0][0]
        for r in range(world):
            assert torch.equal(res[r][0], got[overlap])
    assert torch.equal(got[True], got[False])


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_row_sharded_encoders_match_full(world):
    """each rank's encoder band (its GRU slab + 48
    rows of 1/f margin) with conv2's InstanceNorm statistics all-reduced
    gives the full-image features on the slab, to fp32 rounding of the
    statistics (sums in fp64 vs PyTorch's fp32 reduction)."""
    res = _spawn(dist_worker.run_features, world, 24, 800, 64)
    H1 = res[0][1][0]
    for r in range(world):
        assert res[r][0] < 2e-5, (r, res[r][0])
    # the bands are proper sub-ranges: encoders really ran on part of the image
    assert any(b != (0, H1) for _, (_, b) in ((r, res[r][1]) for r in range(world)))


@pytest.mark.parametrize("world,H,layers,down,f64", [(2, 800, 3, 2, True), (3, 375, 3, 2, True),
                                                     (2, 640, 2, 3, True), (3, 800, 3, 2, False)])
def test_gloo_encoder_halo_exchange_matches_full(world, H, layers, down, f64):
    """the encoders run on each rank's OWN rows, every
    module's halo (1-4 rows at its own resolution) refreshed from the two
    neighbours right before it (point-to-point, no recomputed margin), and the
    GRU slabs then assembled by one more exchange per level: equal to the
    full-image features on the rank's slab (model.py:136-161, :345).  In
    float64 to 1e-12 (the only differences are the summation order of
    conv2's InstanceNorm statistics); in fp32 to 5e-5 absolute (measured
    2.3e-5 on the 1/16-res heads: CPU convolutions pick other algorithms for
    other input heights, 1e-6 relative to values up to 20)."""
    res = _spawn(dist_worker.run_features_halo, world, 12, H, 64, layers, down, f64)
    for r in range(world):
        assert res[r][0] < (1e-12 if f64 else 5e-5), (r, res[r][0])
    # own rows really partition the 1/f grid (no rank computed the whole image)
    owns = sorted(res[r][1][1] for r in range(world))
    H1 = res[0][1][0]
    assert owns[0][0] == 0 and owns[-1][1] == H1
    assert all(a[1] == b[0] for a, b in zip(owns, owns[1:]))


@pytest.mark.parametrize("world,H,W,shard_enc,enc_halos,slow_fast,layers", [
    (2, 320, 96, True, True, False, 3), (3, 320, 96, True, True, False, 3),
    (3, 320, 96, False, True, False, 3), (2, 320, 96, True, False, True, 3),
    (3, 320, 96, True, True, True, 2), (2, 320, 64, True, True, False, 1)])
def test_gloo_perconv_row_sharded_network(world, H, W, shard_enc, enc_halos, slow_fast, layers):
    """the default row-sharded GRU loop keeps every tensor
    on the rank's OWN rows and evaluates each conv / pool / interp on exactly
    the rows its readers need, with the halos (2-7 rows per tensor at its own
    level, RowShardedStereo.perconv_halos) exchanged after each update
    (model.py:164-265) -- equal to the unsharded network to fp32 rounding
    (CPU convolutions of other input heights pick other summation orders),
    for the three encoder modes, the slow-fast schedule and 1-3 GRU levels."""
    iters = 4
    res = _spawn(dist_worker.run_rows, world, None, H, W, iters, shard_enc, True, True,
                 slow_fast, True, enc_halos, layers)
    g = torch.Generator().manual_seed(3)
    img1 = torch.rand(1, 3, H, W, generator=g) * 255
    img2 = torch.roll(img1, -4, dims=-1)
    with torch.no_grad():
        ref = torch.stack(dist_worker.model(slow_fast, layers)(img1, img2, iters=iters))
    for r in range(world):
        got = res[r][0]
        assert got.shape == ref.shape
        assert (got - ref).abs().max() < 5e-5, (got - ref).abs().max()
        assert (got - ref).abs().mean() < 1e-6


@pytest.mark.parametrize("world", [4, 8])
def test_gloo_perconv_row_sharded_config4_geometry(world):
    """config 4's ROW geometry (1984 image rows -> 496 /
    248 / 124 feature rows) at world 4 and 8, narrow (64 columns) so the CPU
    can run it.  At world 8 each rank owns 60-64 rows at 1/4 res and 15-16 at
    1/16 res against net halos of [5, 5, 2] rows, so every GRU level's halo
    reaches across a whole neighbour-adjacent band -- the edge-to-edge
    bookkeeping the 8-GPU run relies on.  Per-conv default (own rows,
    encoders with per-module halos, overlapped exchanges) == the unsharded
    network at the fp32 bars of test_gloo_perconv_row_sharded_network."""
    H, W, iters = 1984, 64, 2
    res = _spawn(dist_worker.run_rows, world, None, H, W, iters, True, True, True, False, True,
                 True, None)
    g = torch.Generator().manual_seed(3)
    img1 = torch.rand(1, 3, H, W, generator=g) * 255
    img2 = torch.roll(img1, -4, dims=-1)
    with torch.no_grad():
        ref = torch.stack(dist_worker.model()(img1, img2, iters=iters))
    for r in range(world):
        got = res[r][0]
        assert got.shape == ref.shape
        assert (got - ref).abs().max() < 5e-5, (r, (got - ref).abs().max())
        assert (got - ref).abs().mean() < 1e-6
    from raft_stereo_amd.shard import RowShardedStereo
    hz = RowShardedStereo(dist_worker.model(), 0, 1).perconv_halos()
    glob = RowShardedStereo._heights(H, 2, 3)
    owns = [RowShardedStereo(dist_worker.model(), k, world)._own_rows(glob, hz) for k in range(world)]
    assert owns[0][0] == 0 and owns[-1][1] == glob[0]
    # the geometry the docstring describes: 1/16-res bands of 15-16 rows at
    # world 8 (31-32 at world 4), i.e. about three net halos (5 rows) tall
    band16 = sorted((b - a) >> 2 for a, b in owns)
    assert band16[0] >= max(hz["net"]) and band16[-1] <= 496 // (4 * world) + 1, band16


def test_gloo_perconv_overlap_equals_blocking():
    """Per-conv mode: exchanges posted at the update and waited for at the
    first reader give the same flows, bit for bit, as waiting right away."""
    got = {}
    for overlap in (True, False):
        res = _spawn(dist_worker.run_rows, 3, None, 320, 96, 3, True, True, overlap, False, True)
        got[overlap] = res[0][0]
        for r in range(3):
            assert torch.equal(res[r][0], got[overlap])
    assert torch.equal(got[True], got[False])


def test_perconv_halos_and_rank_limit():
    """The halo table follows the modules' receptive fields, and a world so
    large that a rank owns fewer rows than a halo is refused up front."""
    from raft_stereo_amd.shard import RowShardedStereo
    rs = RowShardedStereo(dist_worker.model(), 0, 1)
    assert rs.per_conv
    hz = rs.perconv_halos()
    assert hz["net"] == [5, 5, 2] and hz["inp"] == 1 and hz["fmap"] == 4 and hz["coords"] == 7
    glob = RowShardedStereo._heights(1984, 2, 3)
    assert glob == [496, 248, 124]
    for world in (1, 2, 4, 8):
        r0, r1 = RowShardedStereo(dist_worker.model(), world - 1, world)._own_rows(glob, hz)
        assert r1 == 496 and r0 % 4 == 0
    with pytest.raises(ValueError, match="halo"):
        RowShardedStereo(dist_worker.model(), 0, 62)._own_rows(glob, hz)
