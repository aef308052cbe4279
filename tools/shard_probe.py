"""Config 4 (Middlebury 1984x2880, bs=1, 32 iters) on ONE GPU: the pieces of
the row-sharded forward, timed separately, and the scaling cap they imply.

    python tools/shard_probe.py [--iters 32] [--halo 12]

shard.RowShardedStereo shards the per-iteration work (corr lookup + GRU
update, model.py:374-383) by rows of the 1/4-resolution grid, each rank
keeping a +-halo slab, and either runs the encoders (cnet + conv2 + context
convs, model.py:359-365) replicated on the full image or (default) on a band
of image rows around its slab (``shard_encoders``).  Timed here:
  E    = RAFTStereo.features on the full image (the replicated encoders);
  Es(N)= the encoders of a middle rank with per-module halo exchange
         (RowShardedStereo._features_halo + _gru_slabs, the default): its own
         rows plus 1-4 halo rows per module; timed in one process with the
         exchanges replaced by zero rows of the same shapes (_fake_xchg), so
         the messages themselves (tens of KB to a few MB per module, one xGMI
         hop) and the two InstanceNorm all-reduces are not included;
  Eb(N)= the same rank's encoders on a band of +-enc_margin recomputed rows
         (RowShardedStereo._features_rows, encoder_halos=False);
  C(n) = the corr build of an n-row slab;
  U(n) = one iteration on an n-row slab: lookup + update block (with the
         slab-local interp of RowShardedStereo._gru), n = H1/N + 2*halo;
then T(N) = E + C(n_N) + iters * U(n_N) (halo exchange not included: a few
MB per neighbour per iteration over xGMI, tens of us) and the speedup
T(1) / T(N).  The replicated encoder bounds it: T(N) >= E; with sharded
encoders Ts(N) = Es(N) + C(n_N) + iters * U(n_N).

    python tools/shard_probe.py --xchg [--world 3]

Exposed exchange time instead: ``world`` CPU processes
over gloo run RowShardedStereo.forward on a small image with the exchanges
overlapped (the default) and blocking, and report per rank the forward time,
the host time blocked in exchange waits (``xchg_wait_s``) and the number of
waits.  A CPU/gloo rehearsal of the schedule, not an xGMI measurement.

    python tools/shard_probe.py --perconv [--link-gbs 153 --msg-us 15]

The default per-conv mode end to end: for N = 1, 2, 4, 8
a middle rank's WHOLE RowShardedStereo.forward (encoders with per-module
halos, corr build on own rows +- 4, 32 GRU iterations with per-conv halos)
on one GPU, exchanges replaced by zero rows of the same shapes
(``_fake_xchg``), plus the message bytes that rank would receive.  The
projection adds the transfers as if none overlapped compute: per exchange
the larger neighbour's bytes / link GB/s + a per-message latency (the two
links run concurrently); "speedup_overlapped" leaves them out.  Not an RCCL
measurement.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pkgload  # noqa: E402

pkgload.load()
from raft_stereo_amd.network import RAFTStereo, StereoArgs  # noqa: E402
from raft_stereo_amd.shard import RowShardedStereo  # noqa: E402


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2]


def _xchg_rank(rank, world, port, q, H, W, iters, threads):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(threads)
    try:
        from oracle import torch_ref   # CPU processes: the ATen corr block
        torch.manual_seed(0)
        model = RAFTStereo(StereoArgs(), corr_block=torch_ref.TorchCorrBlock1D).eval()
        g = torch.Generator().manual_seed(1234)
        img1 = torch.rand(1, 3, H, W, generator=g) * 255
        img2 = torch.roll(img1, -8, dims=-1)
        out = {}
        with torch.no_grad():
            for overlap in (True, False, True, False):
                rs = RowShardedStereo(model, rank, world, overlap=overlap)
                dist.barrier()
                t0 = time.perf_counter()
                rs.forward(img1, img2, iters=iters)
                t = time.perf_counter() - t0
                out["overlap" if overlap else "blocking"] = {
                    "forward_s": round(t, 3), "xchg_wait_s": round(rs.xchg_wait_s, 3),
                    "waits": rs.xchg_count, "exposed_frac": round(rs.xchg_wait_s / t, 3)}
        q.put((rank, out))
    except Exception:
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def xchg_main(world, H, W, iters):
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    threads = max(1, (os.cpu_count() or 2) // world)
    ps = [ctx.Process(target=_xchg_rank, args=(r, world, port, q, H, W, iters, threads))
          for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=1800) for _ in ps)
    for p in ps:
        p.join()
    print(json.dumps({"rehearsal": "CPU processes over gloo (not xGMI)", "world": world,
                      "image": [H, W], "iters": iters, "threads_per_rank": threads,
                      "per_rank": {r: res[r] for r in sorted(res)}}, indent=1))


def perconv_main(a):
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = RAFTStereo(StereoArgs()).eval().to(dev)
    g = torch.Generator().manual_seed(1234)
    img1 = (torch.rand(1, 3, a.H, a.W, generator=g) * 255).to(dev)
    img2 = torch.roll(img1, -8, dims=-1)
    res = {"image": [a.H, a.W], "iters": a.iters, "mode": "per-conv halos (default)",
           "link_gbs": a.link_gbs, "msg_us": a.msg_us, "per_N": {}}
    glob = RowShardedStereo._heights(a.H, model.args.n_downsample, model.args.n_gru_layers)
    reps = 3
    with torch.no_grad():
        for N in (1, 2, 4, 8):
            rs = RowShardedStereo(model, N // 2, N)
            rs._fake_xchg = True
            r0, r1 = rs._own_rows(glob, rs.perconv_halos())
            rs.xchg_posts = rs.xchg_bytes = rs.xchg_link_bytes = 0
            T = timed(lambda: rs.forward(img1, img2, iters=a.iters), reps)
            runs = reps + 1
            posts, link = rs.xchg_posts / runs, rs.xchg_link_bytes / runs
            xfer = link / (a.link_gbs * 1e9) + posts * a.msg_us * 1e-6
            res["per_N"][N] = {"rank": N // 2, "own_rows": [r0, r1], "T_compute_ms": T * 1e3,
                               "exchanges": posts, "recv_bytes": rs.xchg_bytes / runs,
                               "link_bytes": link, "transfer_ms_if_exposed": xfer * 1e3}
            print(f"N={N}: {json.dumps(res['per_N'][N])}", flush=True)
    T1 = res["per_N"][1]["T_compute_ms"]
    for N, o in res["per_N"].items():
        o["speedup_overlapped"] = T1 / o["T_compute_ms"]
        o["speedup_exposed"] = T1 / (o["T_compute_ms"] + o["transfer_ms_if_exposed"])
    print(json.dumps(res, indent=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=32)
    ap.add_argument("--halo", type=int, default=12,
                    help="1/4-res halo rows (12: per-stage exchange, the default; 32: once per iteration)")
    ap.add_argument("--H", type=int, default=1984)
    ap.add_argument("--W", type=int, default=2880)
    ap.add_argument("--xchg", action="store_true", help="exposed-exchange rehearsal (gloo, CPU)")
    ap.add_argument("--world", type=int, default=3)
    ap.add_argument("--perconv", action="store_true",
                    help="the per-conv default, whole forward per rank + transfer estimate")
    ap.add_argument("--link-gbs", type=float, default=153.0, help="xGMI GB/s per link")
    ap.add_argument("--msg-us", type=float, default=15.0, help="latency per exchange (us)")
    a = ap.parse_args()
    if a.perconv:
        return perconv_main(a)
    if a.xchg:
        return xchg_main(a.world, 768 if a.H == 1984 else a.H, 256 if a.W == 2880 else a.W,
                         8 if a.iters == 32 else a.iters)
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = RAFTStereo(StereoArgs()).eval().to(dev)
    g = torch.Generator().manual_seed(1234)
    img1 = (torch.rand(1, 3, a.H, a.W, generator=g) * 255).to(dev)
    img2 = torch.roll(img1, -8, dims=-1)
    res = {"image": [a.H, a.W], "iters": a.iters, "halo": a.halo}
    with torch.no_grad():
        E = timed(lambda: model.features(img1, img2))
        fmap1, fmap2, net, inp = model.features(img1, img2)
        H1 = fmap1.shape[2]
        res["E_encoders_ms"] = E * 1e3
        print(f"E = {E * 1e3:.1f} ms", flush=True)
        blk = model.update_block
        out = {}
        for N in (1, 2, 4, 8):
            rs = RowShardedStereo(model, 0, N, halo=a.halo)
            r0, r1, e0, e1 = rs._ranges(H1)
            # rank 0 holds [0, r1 + halo): the largest slab is a middle rank's
            n = min(H1, (r1 - r0) + (2 * a.halo if N > 2 else a.halo if N == 2 else 0))
            sl = lambda t, l: t[:, :, : max(1, -(-n // (1 << l)))].contiguous()
            f1, f2 = fmap1[:, :, :n].contiguous(), fmap2[:, :, :n].contiguous()
            C = timed(lambda: model.corr_block(f1, f2, radius=4, num_levels=4))
            corr_fn = model.corr_block(f1, f2, radius=4, num_levels=4)
            c1 = model.initialize_flow(sl(net[0], 0))[1]
            nets = [sl(t, l) for l, t in enumerate(net)]
            inps = [[sl(c, l) for c in cl] for l, cl in enumerate(inp)]

            def one_iter():
                corr = corr_fn(c1)
                flow = c1 - c1
                RowShardedStereo._gru(blk, list(nets), inps, corr, flow,
                                      lambda x, ls, ld: torch.nn.functional.interpolate(
                                          x, nets[ld].shape[2:], mode="bilinear",
                                          align_corners=True), True, True, True)
            U = timed(one_iter)
            T = E + C + a.iters * U
            if N > 1:   # a middle rank (single process: no messages, no all-reduce)
                rm = RowShardedStereo(model, N // 2, N, halo=a.halo)
                rm._fake_xchg = True
                q0, q1, x0, x1 = rm._ranges(H1)

                def halo_features():
                    o = rm._features_halo(img1, img2, q0, q1)
                    return rm._gru_slabs(o[0], o[1], o[2], o[3], o[4])
                Es = timed(halo_features)
                Eb = timed(lambda: rm._features_rows(img1, img2, x0, x1, q0, q1))
                band = min(H1, x1 + rm.enc_margin) - max(0, x0 - rm.enc_margin)
                own = q1 - q0
            else:
                Es, Eb, band, own = E, E, H1, H1
            out[N] = {"slab_rows": n, "own_rows": own, "C_build_ms": C * 1e3, "U_iter_ms": U * 1e3,
                      "T_ms": T * 1e3, "Es_halo_ms": Es * 1e3, "Eb_band_ms": Eb * 1e3,
                      "band_rows": band, "Ts_sharded_ms": (Es + C + a.iters * U) * 1e3,
                      "Tb_band_ms": (Eb + C + a.iters * U) * 1e3}
            print(f"N={N}: {json.dumps(out[N])}", flush=True)   # progress (long run)
        T1 = out[1]["T_ms"]
        for N in out:
            out[N]["speedup"] = T1 / out[N]["T_ms"]
            out[N]["encoder_share"] = res["E_encoders_ms"] / out[N]["T_ms"]
            out[N]["speedup_sharded"] = T1 / out[N]["Ts_sharded_ms"]
            out[N]["speedup_band"] = T1 / out[N]["Tb_band_ms"]
        res["per_N"] = out
        res["amdahl_cap"] = T1 / res["E_encoders_ms"]
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
