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


def test_gloo_world2_batch_and_row_sharding():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=dist_worker.run, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
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
    img1, img2 = dist_worker.pairs()
    with torch.no_grad():
        ref = dist_worker.model()(img1, img2, iters=3)[-1]
    for r in range(world):
        assert res[r][0].shape == ref.shape
        assert torch.allclose(res[r][0], ref, atol=1e-4, rtol=0)
    f1, f2, coords = dist_worker.row_case()
    assert torch.equal(res[0][1], torch_ref.TorchCorrBlock1D(f1, f2, 3, 3)(coords))
