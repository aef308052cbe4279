"""Benchmark of the RAFT-Stereo correlation path on MI355X.

Contract (see task spec): ``python bench.py --gpus N --steps K --warmup W``;
one rank per GPU.  Under a launcher (``torch.distributed.run``, WORLD_SIZE
set) WORLD_SIZE must equal N; without one, ``--gpus N > 1`` starts the N
ranks itself (a ``torch.distributed.run`` child, before this process touches
the GPU).  Rank 0 prints ONE JSON line.

Workload (BASELINE.json configs[1], the metric's config): SceneFlow-size
540x960 stereo pairs, batch 8 per GPU, 32 GRU iterations, fp32 corr.  One
"step" = one pass of the hot path over one batch: CorrBlock1D construction
(volume + fused pyramid, one launch, model.py:366-367) followed by 32 lookups
(model.py:376), each with its own coordinates, all inputs resident in HBM
before timing.  Feature maps are synthetic (B, 256, 135, 240) randn (the
conv2 output shape at 540x960, n_downsample=2); coordinates are
coords_grid - U[0, 64) per pixel, a fresh draw per iteration.

value = stereo pairs/s through the corr path, all ranks (weak scaling: every
rank processes its own batch of 8; the path shards by pair with no collective).
The end-to-end model (encoders/GRU on PyTorch ops) is not in this number; it
is reported beside it (``e2e``), and so is the row-sharded full network of
BASELINE configs[3] (``config4_network``: 1984x2880, 32 iterations, GRU halo
exchange over RCCL in the timed region).  ``--config middlebury --network``
makes that network rate the line's ``value``.
"""
import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import pkgload  # noqa: E402

pkgload.load()
from raft_stereo_amd import CorrBlock1D, _lib, coords_grid  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
HBM_ACHIEVABLE_GBS = 6290.0    # the same guide's measured float4 copy (report both)
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: f32-input MFMA peak
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA peak (no sparsity)
SPLIT_PRODUCTS = 6             # bf16 MFMAs per fp32 product in rc::build_split_kernel

CONFIGS = {
    # name: (B per GPU, D, H1, W1, W2, levels, radius, iters, description)
    "sceneflow": (8, 256, 135, 240, 240, 4, 4, 32,
                  "corr path: CorrBlock1D build + 32 lookups, 540x960 -> 135x240 fmaps, "
                  "batch 8/GPU, fp32, 4 levels, radius 4"),
    "kitti": (64, 256, 94, 311, 311, 4, 4, 32,
              "corr path: build + 32 lookups, 375x1242 -> 94x311 fmaps, global batch 64 "
              "split over the GPUs, bf16 fmaps, bf16 MFMA volume + bf16 pyramid"),
    "realtime": (1, 256, 120, 160, 160, 3, 4, 7,
                 "corr path: build + 7 lookups, 480x640 -> 120x160, batch 1, 3 levels"),
    "middlebury": (1, 256, 496, 720, 720, 4, 4, 32,
                   "corr path: build + 32 lookups, 1984x2880 -> 496x720, batch 1, fp32"),
}


def lookup_bytes(P, L, r, s_pyr=4):
    """Algorithmic bytes of one lookup: coords x (4 B) + per level 2r+2 pyramid
    elements + (2r+1) fp32 outputs, per pixel."""
    return P * (4 + L * (2 * r + 2) * s_pyr + L * (2 * r + 1) * 4)


def volume_flops(B, D, H, W1, W2):
    return 2.0 * B * H * W1 * W2 * D


def volume_bytes(B, D, H, W1, W2, levels, s_in=4, s_pyr=4):
    """fmaps read + the pyramid levels the build writes (all L+1, or e.g.
    levels 0 and 2 when the chain lookup recomputes the rest)."""
    P = B * H * W1
    return 2 * B * D * H * W1 * s_in + sum(P * (W2 >> l) * s_pyr for l in levels)


BF16_CONFIGS = {"kitti"}
ROW_SHARD_CONFIGS = {"middlebury"}
# BASELINE configs[2]: "batch 64 ... batch-sharded across 2/4/8 GPUs" -- the
# config's B is the GLOBAL batch, split over the ranks (strong scaling)
GLOBAL_BATCH_CONFIGS = {"kitti"}
# small latency-bound config: every level stored, one wave per level per
# 64 pixels in the lookup (CorrBlock1D(low_latency=True))
LOW_LATENCY_CONFIGS = {"realtime"}


FIELDS = ("random", "smooth", "slant")


def make_inputs(cfg, device, seed, dtype=torch.float32, field="random"):
    """randn fmaps and one coords tensor per iteration.  ``field``: the
    disparity d of x = w1 - d -- "random" U[0, 64) per pixel, a fresh draw per
    iteration (the headline); "smooth" a bilinear field from a
    9x16 grid of U[0, 64) with +-0.25 px of noise; "slant" planes with
    |slope| <= 0.25 px/px -- the coherent fields a network's coords resemble."""
    B, D, H, W1, W2, L, r, iters, _ = cfg
    g = torch.Generator().manual_seed(seed)
    f1 = torch.randn(B, D, H, W1, generator=g).to(device, dtype)
    f2 = torch.randn(B, D, H, W2, generator=g).to(device, dtype)
    grid = coords_grid(B, H, W1)
    coords = []
    for it in range(iters):
        gi = torch.Generator().manual_seed(seed * 1000 + it + 1)
        c = grid.clone()
        if field == "random":
            d = torch.rand(B, H, W1, generator=gi) * 64.0
        elif field == "smooth":
            k = torch.rand(B, 1, 9, 16, generator=gi) * 64.0
            d = torch.nn.functional.interpolate(k, size=(H, W1), mode="bilinear", align_corners=True)[:, 0]
            d = d + (torch.rand(B, H, W1, generator=gi) - 0.5) * 0.5
        elif field == "slant":
            a0 = torch.rand(B, 1, 1, generator=gi) * 32 + 16
            bw = (torch.rand(B, 1, 1, generator=gi) - 0.5) * 0.5
            ch = (torch.rand(B, 1, 1, generator=gi) - 0.5) * 0.5
            w = torch.arange(W1).view(1, 1, W1) - W1 / 2
            h = torch.arange(H).view(1, H, 1) - H / 2
            d = (a0 + bw * w + ch * h).clamp(0, 63.9) + torch.rand(B, H, W1, generator=gi) * 0.25
        else:
            raise ValueError(f"unknown coords field {field!r}")
        c[:, 0] -= d
        coords.append(c.to(device))
    return f1, f2, coords


def host_cores():
    """CPUs this process may use: the affinity mask, capped by a cgroup CPU
    quota when one is set (the GPU box shows the whole machine in the mask
    but gives one GPU's share of it)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
            if q != "max":
                quota = max(1, math.ceil(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    return (min(aff, quota) if quota else aff), aff, quota


def _median_time(fn, reps, budget_s):
    """Median wall time of ``fn`` over up to ``reps`` runs after one warm-up
    (fewer when the budget runs out; always at least one timed run)."""
    fn()
    times, t_end = [], time.perf_counter() + budget_s
    while not times or (len(times) < reps and time.perf_counter() < t_end):
        t0 = time.perf_counter()
        fn()
        times.append(time.perf_counter() - t0)
    times.sort()
    return times[len(times) // 2], len(times)


def cpu_baseline(cfg, seconds_target=15.0, full=True):
    """BASELINE.md §3 on this host's cores, through the oracle's restatement
    of the reference (oracle/torch_ref.py: model.py:267-326 op for op,
    including the torch.unique assert at :272; pinned bit-exact to goldens
    from the reference itself):
      value     corr path pairs/s: one pair (B=1) of the bench workload,
                build + ``iters`` lookups;
      e2e_config1  BASELINE configs[0]: the whole network (network.RAFTStereo
                with the oracle corr block, pinned to the reference's config-1
                golden by tests/test_network_cpu.py) on one 1x3x320x720 pair,
                12 iterations;
      build / lookup  the corr build alone (GFLOP/s) and one lookup alone
                (algorithmic GB/s) at the full config-2 shape (B=8).
    Each is the median of up to 5 runs after one warm-up."""
    from oracle import torch_ref
    B, D, H, W1, W2, L, r, iters, _ = cfg
    cores, aff, quota = host_cores()
    torch.set_num_threads(cores)
    budget = seconds_target / 4
    f1, f2, coords = make_inputs((1,) + cfg[1:], "cpu", seed=7)

    def corr_pair():
        blk = torch_ref.TorchCorrBlock1D(f1, f2, L, r)
        for it in range(iters):
            blk(coords[it])
    t_pair, n_pair = _median_time(corr_pair, 5, budget)
    cpu_name = ""
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    cpu_name = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    out = {"value": 1.0 / t_pair, "unit": "pairs/s", "cores": cores, "kind": "port",
           "sample": f"corr path, 1 pair (B=1) of the bench workload: build + {iters} lookups "
                     f"via oracle/torch_ref.py (the reference's ATen op sequence incl. the "
                     f"torch.unique assert), median of {n_pair} after 1 warm-up; {cpu_name}",
           "sec_per_pair": t_pair, "affinity_cpus": aff, "cgroup_cpu_quota": quota}
    if not full:
        return out

    # BASELINE configs[0]: one 1x3x320x720 pair, 12 iterations, fp32 CPU
    from raft_stereo_amd.network import RAFTStereo, StereoArgs
    torch.manual_seed(0)
    model = RAFTStereo(StereoArgs(), corr_block=torch_ref.TorchCorrBlock1D).eval()
    g = torch.Generator().manual_seed(1234)
    img1 = torch.rand(1, 3, 320, 720, generator=g) * 255
    img2 = torch.roll(img1, shifts=-8, dims=-1)
    with torch.no_grad():
        t_e2e, n_e2e = _median_time(lambda: model(img1, img2, iters=12), 5, seconds_target)

    # build and one lookup alone at the full config shape (B as configured)
    F1, F2, C = make_inputs(cfg, "cpu", seed=8)
    t_build, n_build = _median_time(lambda: torch_ref.TorchCorrBlock1D(F1, F2, L, r), 5, budget)
    blk = torch_ref.TorchCorrBlock1D(F1, F2, L, r)
    t_look, n_look = _median_time(lambda: blk(C[0]), 5, budget)
    P = B * H * W1
    return {**out,
            "e2e_config1": {"sec_per_pair": t_e2e, "pairs_per_s": 1.0 / t_e2e, "runs": n_e2e,
                            "workload": "BASELINE configs[0]: network.RAFTStereo (default args, "
                                        "seeded weights) + oracle corr block, 1x3x320x720, "
                                        "12 iters, fp32"},
            "build": {"ms": t_build * 1e3, "runs": n_build,
                      "gflops": volume_flops(B, D, H, W1, W2) / t_build / 1e9,
                      "shape": [B, D, H, W1, W2], "levels": L + 1},
            "lookup": {"ms": t_look * 1e3, "runs": n_look,
                       "gbs": lookup_bytes(P, L, r) / t_look / 1e9,
                       "algorithmic_bytes": lookup_bytes(P, L, r)}}


def e2e_pairs_per_s(cfg, device, steps, warmup, image_hw=(540, 960), mixed=False,
                    fuse_step=False, world=1):
    """Whole network (encoders/GRU on PyTorch ops + the HIP corr path) on
    synthetic pairs at the config's image size.  Every rank runs its own batch;
    the timed region is bracketed by barriers and the MAX over ranks is the
    job's time, so ``pairs_per_s_all_ranks`` = B * world / max time."""
    from raft_stereo_amd.network import RAFTStereo, StereoArgs
    B, D, H1, W1, W2, L, r, iters, _ = cfg
    torch.manual_seed(0)
    args = StereoArgs(corr_levels=L, corr_radius=r, mixed_precision=mixed)
    if mixed:
        args.autocast_dtype = torch.bfloat16
    model = RAFTStereo(args, fuse_step=fuse_step).eval().to(device)
    g = torch.Generator().manual_seed(1234)
    H, W = image_hw
    img1 = (torch.rand(B, 3, H, W, generator=g) * 255).to(device)
    img2 = torch.roll(img1, shifts=-8, dims=-1)
    with torch.no_grad():
        for _ in range(warmup):
            model(img1, img2, iters=iters)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            model(img1, img2, iters=iters)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt = torch.tensor([(time.perf_counter() - t0) / steps], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    dt = float(dt.item())
    return {"pairs_per_s": B / dt, "pairs_per_s_all_ranks": B * world / dt,
            "ms_per_batch": dt * 1e3, "batch": B, "world": world, "image": [H, W],
            "iters": iters, "mixed_precision": mixed, "fuse_step": fuse_step,
            "note": "full network; encoders/GRU/heads on PyTorch (MIOpen) ops per north_star; "
                    "max over ranks"}


def backward_timing(cfg, f1, f2, coords, reps=3):
    """Corr-path backward on the bench workload:
    * the product lookup backward -- ONE rc_corr_lookup_backward_calls launch
      summing all `iters` calls (what CorrBlock1D's autograd runs, DESIGN.md
      §3.4c), event-timed;
    * the per-call kernel (rc_corr_lookup_backward, one launch per call) and
      its zeroed buffers, for comparison;
    * rc_corr_build_backward;
    * a whole autograd step (build + lookups + backward through CorrBlock1D)
      with random output gradients."""
    from raft_stereo_amd import corr as rcorr
    B, D, H, W1, W2, L, r, iters, _ = cfg
    P = B * H * W1
    dev = f1.device
    widths = [W2 >> i for i in range(L)]
    g = torch.Generator().manual_seed(99)
    # one output gradient per call, as in training (two alternating tensors
    # would leave the calls' reads partly in the Infinity Cache)
    gl = [torch.randn(B, L * (2 * r + 1), H, W1, generator=g).to(dev) for _ in range(iters)]
    gouts = gl
    pair = rcorr._pair_grads_ok(L, r, W2)      # the layout CorrBlock1D's autograd uses
    grads = rcorr.grad_buffers(P, widths, dev, pair=pair)
    cgrads = rcorr.grad_buffers(P, widths, dev, pair=pair, zero=False)

    def lbwd(c, go):
        rcorr.lookup_backward(grads, c, go, L, r)

    def lcalls():
        rcorr.lookup_backward_calls(cgrads, coords[:iters], gl, L, r, overwrite=True)

    for _ in range(2):   # warm-up
        lbwd(coords[0], gouts[0])
        lcalls()
        rcorr.build_backward(f1, f2, grads)
    lb, vb, lc = [], [], []
    for _ in range(reps):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(iters + 4)]
        ev[0].record()
        for it in range(iters):
            lbwd(coords[it], gl[it])
            ev[it + 1].record()
        rcorr.build_backward(f1, f2, grads)
        ev[iters + 1].record()
        lcalls()
        ev[iters + 2].record()
        torch.cuda.synchronize()
        lb += [ev[k].elapsed_time(ev[k + 1]) for k in range(iters)]
        vb.append(ev[iters].elapsed_time(ev[iters + 1]))
        lc.append(ev[iters + 1].elapsed_time(ev[iters + 2]))
    lb_ms = sorted(lb)[len(lb) // 2]
    vb_ms = sorted(vb)[len(vb) // 2]
    lc_ms = sorted(lc)[len(lc) // 2]
    # whole autograd step through the drop-in class
    a = f1.detach().clone().requires_grad_(True)
    b = f2.detach().clone().requires_grad_(True)

    def train_step(deferred=None):
        blk = CorrBlock1D(a, b, num_levels=L, radius=r, grad_deferred=deferred)
        outs = [blk(coords[it]) for it in range(iters)]
        torch.autograd.backward(outs, gl)

    def timed(fn):
        # median over synchronised single steps of the GPU time between two
        # events around the step (host-side jitter of one step, e.g. an
        # allocator call, stays out of the median)
        fn()
        torch.cuda.synchronize()
        steps = []
        for _ in range(max(reps, 9)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            steps.append(e0.elapsed_time(e1))
        return sorted(steps)[len(steps) // 2]
    step_ms = timed(train_step)
    step_per_call_ms = timed(lambda: train_step(False))
    vflops = 2 * volume_flops(B, D, H, W1, W2)        # two GEMMs
    # per-call kernel: x, grad_out, per-level window RMW (the layout-independent
    # definition of round 1; the pair layout's RMW touches 2 spans of 2(2r+4))
    lbytes = P * (4 + L * (2 * r + 1) * 4 + 2 * L * (2 * r + 2) * 4)
    # all calls in one pass: every call's x and grad_out read once, the pair
    # rows (16-B padded) written once
    rows = sum(-(-(W2 >> l) // 4) * 4 for l in range(0, L, 2)) if pair else 0
    cbytes = iters * P * (4 + L * (2 * r + 1) * 4) + P * rows * 4
    out = {"lookup_bwd_calls_us": lc_ms * 1e3, "lookup_bwd_us": lb_ms * 1e3,
           "volume_bwd_us": vb_ms * 1e3,
           "train_step_ms": step_ms, "train_pairs_per_s": B / (step_ms * 1e-3),
           "train_step_per_call_bwd_ms": step_per_call_ms,
           # split-bf16 GEMMs (the default since ABI v8): 6 bf16 MFMA products per
           # fp32 product; priced as fp32-equivalent FLOP/s against the fp32
           # MFMA peak (as roofline_volume) and as executed bf16 FLOP/s
           "roofline_volume_bwd": {"bound": "mfma", "achieved": vflops / (vb_ms * 1e-3) / 1e12,
                                   "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                                   "frac": vflops / (vb_ms * 1e-3) / 1e12 / FP32_MFMA_PEAK_TFLOPS,
                                   "mfma_bf16_executed_tflops": 6 * vflops / (vb_ms * 1e-3) / 1e12,
                                   "mfma_bf16_frac": 6 * vflops / (vb_ms * 1e-3) / 1e12 / BF16_MFMA_PEAK_TFLOPS,
                                   "kernel": ("rc::volume_bwd_split_kernel<true,kPairFold>" if pair
                                              else "rc::volume_bwd_split_kernel<true,1>" if L == 2
                                              else f"rc::volume_bwd_kernel<true,{L}>")},
           "roofline_lookup_bwd_per_call": {
               "bound": "hbm", "achieved": lbytes / (lb_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
               "unit": "GB/s", "frac": lbytes / (lb_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
               "algorithmic_bytes": lbytes,
               "kernel": (f"rc::lookup_bwd_pair_kernel<{r},{L}>" if pair else
                          f"rc::lookup_bwd_pre_kernel<{r},{L}>" if r <= 4 and L <= 4
                          else f"rc::lookup_bwd_kernel<{r}>")},
           "note": "step = CorrBlock1D build + lookups + autograd backward to both fmaps "
                   "(random output gradients; the lookup backward of all calls in one "
                   "rc_corr_lookup_backward_calls pass, train_step_per_call_bwd_ms: one "
                   "rc_corr_lookup_backward per call into zeroed buffers); kernel times are "
                   "medians of event-timed launches"}
    if pair:
        out["roofline_lookup_bwd"] = {
            "bound": "hbm", "achieved": cbytes / (lc_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": cbytes / (lc_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "algorithmic_bytes": cbytes, "calls_per_launch": iters,
            "kernel": f"rc::lookup_bwd_calls_compact_kernel<{r},{L}>"}
    return out


def upsample_timing(cfg, device, reps=20):
    """Convex upsampler on the config's low-resolution
    x-flow and a synthetic (B, 9*16, H, W) mask: event-timed launches and the
    HBM roofline (mask + flow read, full-resolution flow written)."""
    from raft_stereo_amd.upsample import convex_upsample
    B, D, H, W1, W2, L, r, iters, _ = cfg
    f = 4
    g = torch.Generator().manual_seed(5)
    flow = (torch.randn(B, 1, H, W1, generator=g) * 8).to(device)
    mask = torch.randn(B, 9 * f * f, H, W1, generator=g).to(device)
    for _ in range(3):
        convex_upsample(flow, mask, f)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    ev[0].record()
    for k in range(reps):
        convex_upsample(flow, mask, f)
        ev[k + 1].record()
    torch.cuda.synchronize()
    ts = sorted(ev[k].elapsed_time(ev[k + 1]) for k in range(reps))
    ms = ts[len(ts) // 2]
    nbytes = 4 * B * H * W1 * (9 * f * f + 1 + f * f)
    return {"us": ms * 1e3, "bytes": nbytes,
            "roofline": {"bound": "hbm", "achieved": nbytes / (ms * 1e-3) / 1e9,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "kernel": "rc::convex_upsample_kernel<4>"},
            "shape": {"flow": [B, 1, H, W1], "mask": [B, 9 * f * f, H, W1], "factor": f}}


def load_pmc(path, config):
    """profiles/pmc.json (tools/pmc_collect.py): per-kernel counters measured by
    running THIS script for ``config`` under rocprofv3 --pmc; {} if absent."""
    try:
        with open(path) as fh:
            return json.load(fh).get(config, {})
    except (OSError, ValueError):
        return {}


def pmc_entry(pmc, family):
    """The one kernel of ``family`` (e.g. 'rc::lookup_pair_kernel') that the
    PMC run of this config recorded: (exact name, entry), or (None, {}) when
    there is none or more than one instance (then no counter is reported)."""
    hits = [(k, v) for k, v in pmc.get("kernels", {}).items()
            if k == family or k.startswith(family + "<")]
    return hits[0] if len(hits) == 1 else (None, {})


def launch_plan(gpus, env):
    """How this invocation runs: ("run", world) -- this process is one rank
    of ``world`` (WORLD_SIZE from a launcher, or 1) -- or ("spawn", gpus):
    start ``gpus`` ranks under torch.distributed.run first.  A launcher whose
    WORLD_SIZE disagrees with ``--gpus`` is an error (ValueError): the line
    would otherwise report a world the caller did not ask for."""
    if gpus < 1:
        raise ValueError(f"--gpus must be >= 1, got {gpus}")
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            raise ValueError(f"WORLD_SIZE={ws} from the launcher but --gpus {gpus}")
        return "run", int(ws)
    return ("spawn", gpus) if gpus > 1 else ("run", 1)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launcher_cmd(gpus, argv, port):
    """torch.distributed.run command for ``gpus`` ranks of this script on one
    node (the driver's own form: 127.0.0.1 rendezvous, one rank per GPU)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={gpus}", "--master-addr", "127.0.0.1", "--master-port", str(port),
            os.path.abspath(__file__)] + list(argv)


def leg_watchdog(result, rank, limit):
    """Timer for the default line's config-4 side leg: if it fires, rank 0
    prints the line as measured so far with ``config4_network`` marked timed
    out, and every rank exits 0 (the corr-path measurement stands)."""
    import threading

    def fire():
        if rank == 0:
            line = dict(result)
            line["config4_network"] = {"error": f"not finished after {limit:.0f} s (hung exchange?)"}
            line["status"] = "config4_leg_timeout"
            print(json.dumps(line), flush=True)
        sys.stdout.flush()
        os._exit(0)
    t = threading.Timer(limit, fire)
    t.daemon = True
    t.start()
    return t


def row_sharded_network(device, rank, world, steps, warmup, iters=32, image_hw=(1984, 2880)):
    """BASELINE configs[3] end to end: ONE synthetic full-resolution pair,
    RAFTStereo (seeded random-init weights, fp32, eval) row-sharded over the
    ``world`` ranks by ``shard.RowShardedStereo`` -- encoders on each rank's
    own rows with per-module halos and all-reduced InstanceNorm statistics,
    the corr path on its rows, the GRU loop with its per-conv halo exchanges
    (point-to-point; RCCL over xGMI when the group is nccl) -- 32 iterations.
    Every exchange is inside the timed region.  Timed as the MAX over ranks
    of the barrier-bracketed wall time (strong scaling: one pair per step)."""
    from raft_stereo_amd.network import RAFTStereo, StereoArgs
    from raft_stereo_amd.shard import RowShardedStereo
    torch.manual_seed(0)
    model = RAFTStereo(StereoArgs()).eval().to(device)
    g = torch.Generator().manual_seed(1234)
    H, W = image_hw
    img1 = (torch.rand(1, 3, H, W, generator=g) * 255).to(device)
    img2 = torch.roll(img1, shifts=-8, dims=-1)
    rs = RowShardedStereo(model, rank, world)
    with torch.no_grad():
        for _ in range(warmup):
            rs.forward(img1, img2, iters=iters)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        rs.xchg_wait_s, rs.xchg_count, rs.xchg_bytes, rs.xchg_posts = 0.0, 0, 0, 0
        t0 = time.perf_counter()
        for _ in range(steps):
            preds = rs.forward(img1, img2, iters=iters)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        own = time.perf_counter() - t0
    dt = torch.tensor([own / steps], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    sec = float(dt.item())
    hz = rs.perconv_halos()
    r0, r1 = rs._own_rows(RowShardedStereo._heights(H, model.args.n_downsample,
                                                    model.args.n_gru_layers), hz)
    flow_rows = int(preds[-1].shape[2])
    unsharded = None
    if world == 1:
        # the plain RAFTStereo on the same pair: the N=1 baseline every
        # N-rank speedup is computed against is the faster of the two
        # 
        del preds
        with torch.no_grad():
            model(img1, img2, iters=iters)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                model(img1, img2, iters=iters)
            torch.cuda.synchronize()
        unsharded = (time.perf_counter() - t0) / steps * 1e3
    return {"pairs_per_s": 1.0 / sec, "ms_per_pair": sec * 1e3, "world": world,
            "unsharded_ms_per_pair": unsharded,
            "n1_baseline_ms_per_pair": None if unsharded is None else min(unsharded, sec * 1e3),
            "image": [H, W], "iters": iters, "steps": steps, "warmup": warmup,
            "rank0_own_rows": [r0, r1], "halos": {k: hz[k] for k in ("net", "inp", "fmap", "coords")},
            "rank0_exchanges_per_pair": rs.xchg_count / steps,
            "rank0_recv_mb_per_pair": rs.xchg_bytes / steps / 1e6,
            "rank0_wait_ms_per_pair": rs.xchg_wait_s / steps * 1e3,
            "rank0_own_time_ms": own / steps * 1e3,
            "flow_rows": flow_rows,
            "backend": dist.get_backend() if world > 1 else None,
            "note": "full network (encoders/GRU/heads on PyTorch ops, corr path on the HIP "
                    "kernels), one 1984x2880 pair row-sharded over the ranks; halo exchanges "
                    "and InstanceNorm all-reduces inside the timed region; max over ranks"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="sceneflow", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--graph", action="store_true",
                    help="capture one step (build + lookups) in a HIP graph and replay it")
    ap.add_argument("--e2e-steps", type=int, default=2,
                    help="also time the whole network this many steps (0 = skip)")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc.json"),
                    help="per-kernel PMC counters of this script's own kernels, per config "
                         "(tools/pmc_collect.py)")
    ap.add_argument("--pmc-calibrate", action="store_true",
                    help="copy 1 GiB first (the FETCH_SIZE/WRITE_SIZE calibration dispatch of a "
                         "rocprofv3 --pmc run, tools/pmc_collect.py)")
    ap.add_argument("--exact-f32", action="store_true",
                    help="fp32 builds on the exact fp32 MFMA kernel (RC_BUILD_EXACT_F32) instead of "
                         "the split-bf16 default")
    ap.add_argument("--channels-last", action="store_true", default=None,
                    help="lookup output in NHWC memory order (CorrBlock1D(channels_last=True): "
                         "same shape and values); default for the bf16 config (kitti), whose "
                         "output does not fit the Infinity Cache (DESIGN.md §3.2f)")
    ap.add_argument("--nchw", dest="channels_last", action="store_false",
                    help="force the reference's NCHW-contiguous lookup output")
    ap.add_argument("--no-backward", action="store_true",
                    help="skip the corr-path backward timing (sceneflow only)")
    ap.add_argument("--per-rank-of", type=int, default=0,
                    help="single-GPU projection input: run rank 0's share of an N-GPU job "
                         "(kitti: batch 64/N; middlebury: H/N feature rows); value stays the "
                         "measured work's rate, the N-rank rate goes to 'projection' (DESIGN.md §5)")
    ap.add_argument("--shadow", default="default",
                    help="pyramid levels with an RC_SHADOW copy: 'default' (per-shape rule, "
                         "corr.default_shadow_levels), 'none', or a comma list such as 0,2")
    ap.add_argument("--layout", default=None, choices=("rows", "disparity", "records", "auto"),
                    help="CorrBlock1D pyramid layout: the reference's rows (default for the fp32 "
                         "configs), the opt-in disparity-major levels (RC_LAYOUT_DISPARITY, DESIGN.md "
                         "§3.2h), the bf16 record layout (RC_LAYOUT_RECORDS, §3.2i) or auto (default "
                         "for kitti: records once the bf16 level 0 exceeds the 256 MiB Infinity Cache, "
                         "i.e. per-GPU batch >= 16; 10 %% shorter steps at batch 64)")
    ap.add_argument("--field", default="random", choices=FIELDS,
                    help="coords field: random (SURVEY §8d, the headline), smooth or slant (coherent)")
    ap.add_argument("--network", action="store_true",
                    help="--config middlebury: the line's value is the row-sharded FULL network "
                         "(BASELINE configs[3]: 1984x2880, 32 iterations, GRU halo exchange) "
                         "instead of the corr path alone")
    ap.add_argument("--config4-timeout", type=float, default=300.0,
                    help="seconds the default line waits for its config-4 side leg")
    ap.add_argument("--config4-steps", type=int, default=1,
                    help="default (sceneflow) run: also time the row-sharded config-4 network "
                         "this many steps, after one warm-up (0 = skip)")
    args = ap.parse_args()
    if args.channels_last is None:   # NHWC output where it goes to HBM (the bf16 config)
        args.channels_last = args.config in BF16_CONFIGS
    if args.layout is None:          # the record layout where it pays (bf16, level 0 past the MALL)
        args.layout = "auto" if args.config in BF16_CONFIGS else "rows"
    if args.network and args.config != "middlebury":
        ap.error("--network applies to --config middlebury")
    shadow = (None if args.shadow == "default" else () if args.shadow == "none"
              else tuple(int(v) for v in args.shadow.split(",")))

    # one rank per GPU: decided before anything touches the GPU, so that the
    # self-launch below starts its ranks from a process with no HIP context
    try:
        plan, world = launch_plan(args.gpus, os.environ)
    except ValueError as e:
        print(f"bench.py: {e}", file=sys.stderr)
        sys.exit(2)
    if plan == "spawn":
        cmd = launcher_cmd(world, sys.argv[1:], _free_port())
        sys.exit(subprocess.run(cmd).returncode)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # RAFTCORR_BENCH_BACKEND=gloo: rehearsal of the N>1 path with several
    # ranks sharing the GPUs there are (collectives host-side); default RCCL
    backend = os.environ.get("RAFTCORR_BENCH_BACKEND", "nccl")
    ndev = max(1, torch.cuda.device_count())
    local_dev = local % ndev if backend != "nccl" else local
    if world > 1:
        torch.cuda.set_device(local_dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_dev))
        else:
            dist.init_process_group(backend)
    device = torch.device("cuda", local_dev)
    torch.cuda.set_device(device)
    if args.pmc_calibrate:
        big = torch.empty(1 << 28, device=device).fill_(1.0)
        big.clone()
        del big
        torch.cuda.synchronize()

    cfg = CONFIGS[args.config]
    global_batch = args.config in GLOBAL_BATCH_CONFIGS
    proj = args.per_rank_of if world == 1 and args.per_rank_of > 1 else 0
    split_world = proj or world                    # ranks the job's work is cut into
    if global_batch:
        from raft_stereo_amd.shard import split_range
        b0, b1 = split_range(cfg[0], rank, split_world)
        cfg = (b1 - b0,) + cfg[1:]
    B, D, H, W1, W2, L, r, iters, desc = cfg
    bf16 = args.config in BF16_CONFIGS
    row_shard = args.config in ROW_SHARD_CONFIGS and split_world > 1
    if row_shard:
        # config 4: ONE full-resolution pair, image rows sharded over ranks
        # (strong scaling); the corr path is row-local, so no exchange.
        from raft_stereo_amd.shard import split_range
        r0, r1 = split_range(H, rank, split_world)
        f1, f2, coords = make_inputs(cfg, device, seed=1, field=args.field)
        f1 = f1[:, :, r0:r1].contiguous()
        f2 = f2[:, :, r0:r1].contiguous()
        coords = [c[:, :, r0:r1].contiguous() for c in coords]
        H = r1 - r0
    else:
        f1, f2, coords = make_inputs(cfg, device, seed=1 + rank,
                                     dtype=torch.bfloat16 if bf16 else torch.float32, field=args.field)
    P = B * H * W1

    def step(ev=None):
        if ev is not None:
            ev[0].record()
        blk = CorrBlock1D(f1, f2, num_levels=L, radius=r, channels_last=args.channels_last,
                          low_latency=args.config in LOW_LATENCY_CONFIGS, exact_f32=args.exact_f32,
                          shadow=shadow, layout=args.layout)
        if ev is not None:
            ev[1].record()
        for it in range(iters):
            out = blk(coords[it])
        if ev is not None:
            ev[2].record()
        return out

    run = step
    if args.graph:
        # The whole step -- pyramid allocation (graph memory pool) and every
        # libraftcorr launch on the capturing stream -- becomes one replay.
        with torch.no_grad():
            for _ in range(2):
                step()
            torch.cuda.synchronize()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                step()
        torch.cuda.synchronize()

        def run(ev=None):
            if ev is not None:
                ev[0].record()
                ev[1].record()
            graph.replay()
            if ev is not None:
                ev[2].record()

    with torch.no_grad():
        for _ in range(args.warmup):
            run()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        # the timed region: K bare steps (no events inside: three event
        # records per step cost ~16 us of a 67 us realtime graph step,
        # tools/graph_floor.py)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(args.steps):
            run()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t1 = time.perf_counter()
        # kernel-level split of a step (build / lookups) from a second,
        # instrumented pass: events on the launch stream (torch's current
        # stream, which CorrBlock1D launches on)
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
        for k in range(args.steps):
            run(evs[k])
        torch.cuda.synchronize()
        build_in_loop_ms = sum(e[0].elapsed_time(e[1]) for e in evs) / args.steps
        lookup_ms = sum(e[1].elapsed_time(e[2]) for e in evs) / args.steps / iters

        # Build duration without host time: a device-side sleep first, so the
        # host has queued the whole CorrBlock1D construction (allocations,
        # validation, the build launch) before the GPU reaches the first event
        # -- at small sizes (realtime) the event pair otherwise spans the host
        # gap in front of the launch.  Median of 7.
        bl = []
        for _ in range(7):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(5_000_000)
            e0.record()
            CorrBlock1D(f1, f2, num_levels=L, radius=r, channels_last=args.channels_last,
                        low_latency=args.config in LOW_LATENCY_CONFIGS, exact_f32=args.exact_f32,
                        shadow=shadow, layout=args.layout)
            e1.record()
            torch.cuda.synchronize()
            bl.append(e0.elapsed_time(e1))
        bl.sort()
        build_ms = bl[len(bl) // 2]
        # per-launch lookup duration without the host gaps between launches:
        # events around each launch of one extra pass
        # A device-side sleep first lets the host queue every launch before the
        # GPU reaches them, so no event pair spans a host gap; median over 3
        # passes of all launches.
        blk = CorrBlock1D(f1, f2, num_levels=L, radius=r, channels_last=args.channels_last,
                          low_latency=args.config in LOW_LATENCY_CONFIGS, exact_f32=args.exact_f32,
                          shadow=shadow, layout=args.layout)
        per_launch = []
        for _ in range(3):
            le = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(iters)]
            torch.cuda._sleep(5_000_000)
            for it in range(iters):
                le[it][0].record()
                blk(coords[it])
                le[it][1].record()
            torch.cuda.synchronize()
            per_launch += [a.elapsed_time(b) for a, b in le]
        per_launch.sort()
        lookup_launch_ms = per_launch[len(per_launch) // 2]

    # per-step latency distribution (p50) for the latency-bound realtime config
    lat = []
    with torch.no_grad():
        for _ in range(min(args.steps, 50)):
            torch.cuda.synchronize()
            a0 = time.perf_counter()
            run()
            torch.cuda.synchronize()
            lat.append((time.perf_counter() - a0) * 1e3)
    lat.sort()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    sec = float(elapsed.item())
    ms_per_step = 1e3 * sec / args.steps
    # pairs the whole job processed per step: one row-sharded pair, the global
    # batch, or B per rank (weak scaling)
    job_pairs = 1 if row_shard else (CONFIGS[args.config][0] if global_batch else world * B)
    if proj:
        # one GPU ran only rank 0's share: value counts the work that ran (B
        # pairs, or the row share of one pair); the N-rank rate is reported
        # under "projection" only
        run_pairs = (r1 - r0) / CONFIGS[args.config][2] if row_shard else B
    else:
        run_pairs = job_pairs
    value = run_pairs * args.steps / sec

    vflops = volume_flops(B, D, H, W1, W2)
    s_el = 2 if bf16 else 4
    lbytes = lookup_bytes(P, L, r, s_pyr=s_el)
    written = blk.levels_stored                      # levels the build wrote
    vbytes = volume_bytes(B, D, H, W1, W2, written, s_in=s_el, s_pyr=s_el)
    pmc = load_pmc(args.pmc, args.config)
    split = not bf16 and not args.exact_f32 and W1 % 4 == 0 and W2 % 4 == 0
    vfamily = ("rc::build_bf16_ring_kernel" if bf16 and W2 > 64 else "rc::build_bf16_kernel" if bf16
               else "rc::build_split_kernel" if split else "rc::build_f32_ring_kernel")
    vname, vpmc = pmc_entry(pmc, vfamily)
    vgbs = vbytes / (build_ms * 1e-3) / 1e9
    roof_volume = {"bound": "hbm", "achieved": vgbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                   "frac": vgbs / HBM_PEAK_GBS, "traffic": vpmc.get("hbm_bytes"),
                   "algorithmic_bytes": vbytes, "flops": vflops, "kernel": vname or vfamily,
                   "avg_launch_us": build_ms * 1e3, "levels_written": written,
                   "shadow_levels": sorted(blk._shadow)}
    if bf16:
        pass   # HBM-bound in bf16: priced in bytes
    elif split:
        # fp32 volume on bf16 MFMA (three-way split, six products per fp32
        # product, csrc/volume_split.hip): its own roofline is HBM (8 TB/s for
        # the bytes vs 2.5 PF for the executed bf16 FLOPs); also reported: the
        # executed bf16 MFMA rate and the fp32-equivalent rate vs the fp32 peak
        ex = SPLIT_PRODUCTS * vflops / (build_ms * 1e-3) / 1e12
        roof_volume.update({
            "mfma_bf16_executed_tflops": ex, "mfma_bf16_frac": ex / BF16_MFMA_PEAK_TFLOPS,
            "fp32_equivalent_tflops": vflops / (build_ms * 1e-3) / 1e12,
            "fp32_equivalent_frac_of_fp32_mfma_peak": vflops / (build_ms * 1e-3) / 1e12 / FP32_MFMA_PEAK_TFLOPS,
            "arithmetic": "fp32 operands split exactly into 3 bf16 pieces; 6 bf16 MFMA products "
                          "(v_mfma_f32_16x16x32_bf16, fp32 accumulate) per fp32 product"})
    else:
        roof_volume = {"bound": "mfma", "achieved": vflops / (build_ms * 1e-3) / 1e12,
                       "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                       "frac": vflops / (build_ms * 1e-3) / 1e12 / FP32_MFMA_PEAK_TFLOPS,
                       "traffic": vpmc.get("hbm_bytes"), "algorithmic_bytes": vbytes,
                       "kernel": vname or vfamily, "avg_launch_us": build_ms * 1e3,
                       "levels_written": written, "shadow_levels": sorted(blk._shadow)}
    if "mfma_util" in vpmc:
        roof_volume["mfma_util_pmc"] = vpmc["mfma_util"]
    lgbs = lbytes / (lookup_launch_ms * 1e-3) / 1e9
    pair = blk._chain and (L == 2 or (L == 4 and 2 in written))
    lfamily = ("rc::lookup_sheared_pair_kernel" if blk.layout == "disparity"
               else "rc::lookup_records_kernel" if blk.layout == "records"
               else "rc::lookup_pair_kernel" if pair else "rc::lookup_chain_kernel" if blk._chain
               else "rc::lookup_levelpar_kernel" if P < 65536 and L <= 4 else "rc::lookup_kernel")
    lname, lpmc = pmc_entry(pmc, lfamily)
    ltraffic = lpmc.get("hbm_bytes")
    # FETCH_SIZE's scale depends on the access shape (profiles/r03/n/
    # calib_scattered.txt): a wide stream reads 0.5x its bytes (hence the 2x
    # of hbm_bytes), isolated 64-B / 128-B rows 2.0x / 1.0x their bytes, i.e.
    # whole 128-B lines at 1x.  The lookup's reads are isolated lines, so the
    # uncalibrated sum is the other end of the range its real traffic lies in.
    ltraffic_raw = (lpmc["fetch_bytes_raw"] + lpmc["write_bytes_raw"]
                    if "fetch_bytes_raw" in lpmc and "write_bytes_raw" in lpmc else None)
    roof_lookup = {"bound": "hbm", "achieved": lgbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                   "frac": lgbs / HBM_PEAK_GBS, "frac_of_achievable": lgbs / HBM_ACHIEVABLE_GBS,
                   "traffic": ltraffic,
                   "algorithmic_bytes": lbytes, "kernel": lname or lfamily,
                   "avg_launch_us": lookup_launch_ms * 1e3}
    if ltraffic:   # the HBM bytes the kernel really moves (PMC), per second
        roof_lookup["traffic_gbs"] = ltraffic / (lookup_launch_ms * 1e-3) / 1e9
        roof_lookup["traffic_frac"] = roof_lookup["traffic_gbs"] / HBM_PEAK_GBS
        roof_lookup["traffic_over_algorithmic"] = ltraffic / lbytes
    if ltraffic_raw:
        roof_lookup["traffic_uncalibrated"] = ltraffic_raw
        roof_lookup["traffic_uncalibrated_over_algorithmic"] = ltraffic_raw / lbytes
    if pmc:
        roof_lookup["pmc_source"] = f"{os.path.relpath(args.pmc, ROOT)} [{args.config}] {pmc.get('tag', '')}"
    dominant = roof_lookup if lookup_ms * iters >= build_ms else roof_volume

    result = {
        "metric": "stereo pairs/s at 540x960, 32 iters, 1-8 GPUs; corr-lookup HBM GB/s",
        "value": value,
        "unit": "pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong" if ((row_shard or global_batch) and not proj) else "weak",
        "vs_baseline": None,
        "dtype": "bf16" if bf16 else "f32",
        "data": ("synthetic (randn fmaps, coords_grid - U[0,64) per iteration)" if args.field == "random"
                 else f"synthetic (randn fmaps, coords_grid - a {args.field} disparity field in [0,64))"),
        "config": {"workload": desc + (" (HIP graph replay)" if args.graph else "")
                   + (f" (rows sharded over {world} ranks)" if row_shard else ""),
                   "config": args.config, "global_batch": run_pairs,
                   "fmap": [B, D, H, W1], "W2": W2, "levels": L, "radius": r, "iters": iters,
                   "parallelism": (f"row-shard x{world}" if row_shard else f"batch-shard x{world}"),
                   "corr_out_layout": "channels_last" if args.channels_last else "nchw",
                   "pyramid_layout": blk.layout, "coords_field": args.field},
        "roofline": dominant,
        "roofline_volume": roof_volume,
        "roofline_lookup": roof_lookup,
        "lookup_gbs": lgbs,
        "latency_ms": {"p50": lat[len(lat) // 2], "min": lat[0], "max": lat[-1]},
        "kernel_ms": {"build": build_ms, "build_in_loop": None if args.graph else build_in_loop_ms,
                      "lookup_in_loop": lookup_ms,
                      "lookup_per_launch": lookup_launch_ms},
        "cpu_baseline": None,
        "notes": (f"disparity-major block (layout='disparity', RC_LAYOUT_DISPARITY): the build writes "
                  f"levels {written} as S[b,h][k][w1], k = (w1 >> l) - j + W_l - 1 (the same values and "
                  "bytes as the rows), the lookup reads them with the disparity-major pair kernel; "
                  "corr_pyramid is gathered into rows only when read" if blk.layout == "disparity" else
                  f"record block (layout='records', RC_LAYOUT_RECORDS): the build writes levels {written} "
                  f"as {_lib.rec_count(W2)} 128-B records per pixel row (the rows' values, 1.8x the "
                  "shadowed rows' bytes; the extra writes are in the build's time, not in its "
                  "algorithmic bytes), each lookup reads one line per pixel; corr_pyramid is "
                  "gathered into rows only when read" if blk.layout == "records" else
                  f"pool-chain block: the build writes pyramid levels {written} (levels "
                  f"{sorted(blk._shadow)} also as a half-line-shifted RC_SHADOW copy: those "
                  "writes are in the build's time, not in its algorithmic bytes); every lookup "
                  "recomputes the others from them bit-exactly (rc_corr_lookup_chain); the rest "
                  "are materialised only when corr_pyramid is read" if blk._chain else
                  f"per-level lookup: the build writes the levels a lookup reads, {written}; "
                  "level num_levels is pooled only when corr_pyramid is read"),
    }
    if not args.no_backward and args.config == "sceneflow":
        result["backward"] = backward_timing(cfg, f1, f2, coords)
        bw = result["backward"]
        for key, us in (("roofline_lookup_bwd", "lookup_bwd_calls_us"),
                        ("roofline_lookup_bwd_per_call", "lookup_bwd_us")):
            rl = bw.get(key)
            if rl is None:
                continue
            bname, bpmc = pmc_entry(pmc, rl["kernel"].split("<")[0])
            if bpmc.get("hbm_bytes"):   # PMC bytes the kernel really moves, per launch
                rl["kernel"] = bname
                rl["traffic"] = bpmc["hbm_bytes"]
                rl["traffic_gbs"] = rl["traffic"] / (bw[us] * 1e-6) / 1e9
                rl["traffic_frac"] = rl["traffic_gbs"] / HBM_PEAK_GBS
                rl["traffic_over_algorithmic"] = rl["traffic"] / rl["algorithmic_bytes"]
        rv = result["backward"]["roofline_volume_bwd"]
        vbname, vbpmc = pmc_entry(pmc, rv["kernel"].split("<")[0])
        if "mfma_util" in vbpmc:    # the exact instance the backward ran (one per config)
            rv["kernel"] = vbname
            rv["mfma_util_pmc"] = vbpmc["mfma_util"]
        result["upsample"] = upsample_timing(cfg, device)
    if args.e2e_steps > 0 and args.config == "sceneflow":
        result["e2e"] = e2e_pairs_per_s(cfg, device, args.e2e_steps, 1, world=world)
        result["e2e"]["corr_path_share"] = (ms_per_step / result["e2e"]["ms_per_batch"])
    if args.e2e_steps > 0 and args.config == "realtime":
        # C5 is latency-bound: whole network per pair, with and without the
        # loop's coords update + flow fused into the lookup
        result["e2e"] = {
            "unfused": e2e_pairs_per_s(cfg, device, max(args.e2e_steps, 10), 3, (480, 640)),
            "fused_step": e2e_pairs_per_s(cfg, device, max(args.e2e_steps, 10), 3, (480, 640),
                                          fuse_step=True)}
    if proj:
        # one GPU ran rank 0's share of a proj-GPU job: the rate proj such
        # ranks reach when nothing is exchanged (batch shards; the corr path of
        # row shards).  A projection from measured per-rank work, not a
        # multi-GPU measurement.
        result["projection"] = {
            "per_rank_of": proj, "rank_share": ({"rows": [r0, r1]} if row_shard else {"batch": B}),
            "projected_ms_per_step": ms_per_step,
            "projected_value": job_pairs / (ms_per_step * 1e-3),
            "projected_global_batch": job_pairs,
            "note": "single GPU timing rank 0's share; no collective in the timed path; "
                    "projected_value assumes every rank takes as long -- not a measurement "
                    "of N GPUs (the line's value is the work that ran, per second)"}
        result["config"]["parallelism"] = f"rank 0 of {proj} (single-GPU projection input)"
    # BASELINE configs[3] end to end: in the default run as a side leg (so an
    # N-GPU run of the default command measures config 4's scaling too), or as
    # the line's value with --config middlebury --network
    net_steps = (max(args.steps, 1) if args.network else
                 args.config4_steps if args.config == "sceneflow" and not proj else 0)
    if net_steps > 0 and not args.network:
        # the side leg must not take the corr-path line down with it: an error
        # (e.g. from RCCL, which raises on every rank alike) is recorded in
        # the line instead, and a leg that has not finished after
        # --config4-timeout seconds (a hung exchange) prints the line without
        # it and ends every rank with status 0
        dog = leg_watchdog(result, rank, args.config4_timeout)
        try:
            result["config4_network"] = row_sharded_network(device, rank, world, net_steps, 1)
        except Exception as e:  # noqa: BLE001
            result["config4_network"] = {"error": f"{type(e).__name__}: {e}"[:600]}
        dog.cancel()
    elif net_steps > 0:
        leg = row_sharded_network(device, rank, world, net_steps, max(args.warmup, 1))
        result["corr_path"] = {k: result[k] for k in ("value", "ms_per_step", "config")}
        result.update({
            "value": leg["pairs_per_s"], "ms_per_step": leg["ms_per_pair"],
            "steps": net_steps, "warmup": leg["warmup"], "scaling": "strong",
            "network": leg,
            "config": {"workload": "BASELINE configs[3]: full RAFTStereo network, one "
                                   "1984x2880 pair, 32 iterations, fp32, image rows sharded "
                                   f"over {world} rank(s) (encoders with per-module halos, "
                                   "corr path on own rows, GRU per-conv halo exchange)",
                       "config": "middlebury", "global_batch": 1, "image": [1984, 2880],
                       "iters": 32, "parallelism": f"row-shard x{world}"}})
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(cfg, args.cpu_seconds,
                                              full=args.config == "sceneflow")
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
