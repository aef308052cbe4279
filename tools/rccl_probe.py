"""Does RCCL run two ranks on ONE GPU?  (Probe for rehearsing the N>1 RCCL
path on the one-GPU box; RCCL may refuse duplicate devices.)

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29533 tools/rccl_probe.py

Each rank: init_process_group("nccl", device_id=cuda:0), an all_reduce of a
device tensor, a batch_isend_irecv exchange with the other rank, a barrier.
Prints one line per rank with the results or the error text.
"""
import os
import sys
import time

import torch
import torch.distributed as dist


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    t0 = time.time()
    try:
        dist.init_process_group("nccl", device_id=dev)
        x = torch.full((1024,), float(rank + 1), device=dev)
        dist.all_reduce(x)
        peer = (rank + 1) % world
        src = (rank - 1) % world
        s = torch.full((4096,), float(rank), device=dev)
        r = torch.empty(4096, device=dev)
        reqs = dist.batch_isend_irecv([dist.P2POp(dist.isend, s, peer), dist.P2POp(dist.irecv, r, src)])
        for q in reqs:
            q.wait()
        torch.cuda.synchronize()
        dist.barrier()
        print(f"rank {rank}: ok all_reduce={x[0].item()} (want {world * (world + 1) / 2}) "
              f"recv={r[0].item()} (want {src}) {time.time() - t0:.1f}s", flush=True)
        dist.destroy_process_group()
    except Exception as e:   # noqa: BLE001 -- report whatever RCCL says
        print(f"rank {rank}: FAILED {type(e).__name__}: {str(e)[:400]}", flush=True)
        sys.exit(3)


if __name__ == "__main__":
    main()
