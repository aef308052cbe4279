"""Worker for tests/test_shard_dist.py, spawned per rank (gloo on CPU).
Kept import-clean: paths are set up before the package is imported."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, HERE):
    if p not in sys.path:
        sys.path.insert(0, p)


def pairs():
    import torch
    from golden_util import GOLDEN, load
    z = load(f"{GOLDEN}/e2e_default.npz")
    img1 = torch.from_numpy(z["image1"]).repeat(3, 1, 1, 1)
    img2 = torch.from_numpy(z["image2"]).repeat(3, 1, 1, 1)
    img2[1] = torch.flip(img2[1], dims=[-1])          # make the pairs differ
    return img1, img2


def row_case():
    import torch
    g = torch.Generator().manual_seed(5)
    f1 = torch.randn(2, 16, 7, 24, generator=g)
    f2 = torch.randn(2, 16, 7, 40, generator=g)
    x = torch.arange(24).float().view(1, 1, 1, 24).expand(2, 1, 7, 24) - 10 * torch.rand(2, 1, 7, 24, generator=g)
    return f1, f2, torch.cat([x, torch.zeros(2, 1, 7, 24)], 1)


def model(slow_fast=False, n_gru_layers=None):
    import torch
    import pkgload
    pkgload.load()
    from golden_util import manifest
    from oracle import torch_ref
    from raft_stereo_amd.network import RAFTStereo, StereoArgs
    torch.manual_seed(0)
    case = manifest()["cases"]["e2e_default"]
    args = dict(case["args"])
    if slow_fast:
        args["slow_fast_gru"] = True
    if n_gru_layers is not None:
        args["n_gru_layers"] = n_gru_layers
    return RAFTStereo(StereoArgs(**args), corr_block=torch_ref.TorchCorrBlock1D).eval()


def run(rank, world, port, q):
    import torch
    import torch.distributed as dist
    import pkgload
    pkgload.load()
    from oracle import torch_ref
    from raft_stereo_amd.shard import RowShardedCorr, gather_batch, local_batch

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    try:
        img1, img2 = pairs()
        net = model()
        with torch.no_grad():
            flows = net(local_batch(img1, rank, world), local_batch(img2, rank, world), iters=3)
        full = gather_batch(flows[-1], world)
        f1, f2, coords = row_case()
        part = RowShardedCorr(f1, f2, rank, world, num_levels=3, radius=3,
                              corr_block=torch_ref.TorchCorrBlock1D)(coords)
        parts = [None] * world
        dist.all_gather_object(parts, part)
        q.put((rank, full, torch.cat(parts, dim=2) if rank == 0 else None))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, repr(e), None))
    finally:
        dist.destroy_process_group()


def run_rows(rank, world, port, q, halo=32, H=144, W=96, iters=4, shard_encoders=True,
             per_stage=False, overlap=True, slow_fast=False, per_conv=None, encoder_halos=True,
             n_gru_layers=None):
    """Row-sharded network forward vs the unsharded one (oracle corr block);
    ``halo=None`` with per_stage: the per-conv default."""
    import torch
    import torch.distributed as dist
    import pkgload
    pkgload.load()
    from raft_stereo_amd.shard import RowShardedStereo

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    try:
        g = torch.Generator().manual_seed(3)
        img1 = torch.rand(1, 3, H, W, generator=g) * 255
        img2 = torch.roll(img1, -4, dims=-1)
        net = model(slow_fast=slow_fast, n_gru_layers=n_gru_layers)
        rs = RowShardedStereo(net, rank, world, halo=halo, shard_encoders=shard_encoders,
                              per_stage=per_stage, overlap=overlap, per_conv=per_conv,
                              encoder_halos=encoder_halos)
        with torch.no_grad():
            preds = rs.forward(img1, img2, iters=iters)
            full = [rs.gather_rows(p) for p in preds]
        q.put((rank, torch.stack(full), None))
    except Exception as e:
        import traceback
        q.put((rank, traceback.format_exc(), None))
    finally:
        dist.destroy_process_group()


def run_features(rank, world, port, q, halo=24, H=800, W=64):
    """Row-sharded encoders (band of image rows + InstanceNorm all-reduce)
    vs the full-image encoders sliced to this rank's GRU slab: max |diff|
    over fmap1, fmap2 and every level's net / inp tensors, and the band's
    1/f row range (to show the band did not cover the whole image)."""
    import torch
    import torch.distributed as dist
    import pkgload
    pkgload.load()
    from raft_stereo_amd.shard import RowShardedStereo

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    try:
        g = torch.Generator().manual_seed(11)
        img1 = torch.rand(1, 3, H, W, generator=g) * 255
        img2 = torch.roll(img1, -3, dims=-1)
        net = model()
        rs = RowShardedStereo(net, rank, world, halo=halo)
        with torch.no_grad():
            f1, f2, nf, inf = net.features(img1, img2)
            H1 = f1.shape[2]
            r0, r1, e0, e1 = rs._ranges(H1)
            s1, s2, ns, ins = rs._features_rows(img1, img2, e0, e1, r0, r1)
            d = max((s1 - f1[:, :, e0:e1]).abs().max().item(), (s2 - f2[:, :, e0:e1]).abs().max().item())
            for l in range(len(nf)):
                lo, hi = rs._lvl(e0, e1, l)
                d = max(d, (ns[l] - nf[l][:, :, lo:hi]).abs().max().item())
                for a, b in zip(ins[l], inf[l]):
                    d = max(d, (a - b[:, :, lo:hi]).abs().max().item())
        band = (max(0, e0 - rs.enc_margin), min(H1, e1 + rs.enc_margin))
        q.put((rank, d, (H1, band)))
    except Exception:
        import traceback
        q.put((rank, traceback.format_exc(), None))
    finally:
        dist.destroy_process_group()


def run_features_halo(rank, world, port, q, halo=12, H=800, W=64, n_gru_layers=3, n_downsample=2,
                      f64=False):
    """Encoders on this rank's OWN rows with per-module halo exchange
    (RowShardedStereo._features_halo + _gru_slabs) vs the full-image encoders
    sliced to the rank's GRU slab [e0, e1): max |diff| over fmap1, fmap2 and
    every level's net / inp tensors, and the own 1/f row range."""
    import torch
    import torch.distributed as dist
    import pkgload
    pkgload.load()
    from raft_stereo_amd.network import RAFTStereo, StereoArgs
    from raft_stereo_amd.shard import RowShardedStereo

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    try:
        g = torch.Generator().manual_seed(11)
        img1 = torch.rand(1, 3, H, W, generator=g) * 255
        img2 = torch.roll(img1, -3, dims=-1)
        torch.manual_seed(0)
        net = RAFTStereo(StereoArgs(n_gru_layers=n_gru_layers, n_downsample=n_downsample)).eval()
        if f64:       # exactness of the halo bookkeeping, free of fp32 conv-algorithm rounding
            net, img1, img2 = net.double(), img1.double(), img2.double()
        rs = RowShardedStereo(net, rank, world, halo=halo)
        with torch.no_grad():
            f1, f2, nf, inf = net.features(img1, img2)
            H1 = f1.shape[2]
            r0, r1, e0, e1 = rs._ranges(H1)
            o1, o2, no, io, lv, _ = rs._features_halo(img1, img2, r0, r1)
            s1, s2, ns, ins = rs._gru_slabs(o1, o2, no, io, lv)
            d = max((s1 - f1[:, :, e0:e1]).abs().max().item(), (s2 - f2[:, :, e0:e1]).abs().max().item())
            for l in range(len(nf)):
                lo, hi = rs._lvl(e0, e1, l)
                assert ns[l].shape[2] == hi - lo, (l, ns[l].shape, lo, hi)
                d = max(d, (ns[l] - nf[l][:, :, lo:hi]).abs().max().item())
                for a, b in zip(ins[l], inf[l]):
                    d = max(d, (a - b[:, :, lo:hi]).abs().max().item())
        q.put((rank, d, (H1, (r0, r1))))
    except Exception:
        import traceback
        q.put((rank, traceback.format_exc(), None))
    finally:
        dist.destroy_process_group()


def gpu_model():
    """The default network with the HIP corr block, on cuda:0, seeded weights."""
    import torch
    import pkgload
    pkgload.load()
    from golden_util import manifest
    from raft_stereo_amd.network import RAFTStereo, StereoArgs
    torch.manual_seed(0)
    case = manifest()["cases"]["e2e_default"]
    return RAFTStereo(StereoArgs(**case["args"])).eval().to("cuda:0")


def rows_images(H=320, W=96):
    import torch
    g = torch.Generator().manual_seed(3)
    img1 = torch.rand(1, 3, H, W, generator=g) * 255
    return img1, torch.roll(img1, -4, dims=-1)


def run_gpu(rank, world, port, q, halo=32, iters=4):
    """GPU ranks sharing cuda:0 over gloo (host-staged collectives): the
    batch-sharded network + gather_batch and the row-sharded network + GRU
    halo exchange, both with the HIP CorrBlock1D (not the oracle)."""
    import torch
    import torch.distributed as dist
    import pkgload
    pkgload.load()
    from raft_stereo_amd import CorrBlock1D
    from raft_stereo_amd.shard import RowShardedStereo, gather_batch, local_batch

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        net = gpu_model()
        assert net.corr_block is CorrBlock1D
        img1, img2 = pairs()
        with torch.no_grad():
            flows = net(local_batch(img1, rank, world).cuda(), local_batch(img2, rank, world).cuda(),
                        iters=3)
            full = gather_batch(flows[-1], world)
            r1, r2 = rows_images()
            rs = RowShardedStereo(net, rank, world, halo=halo)
            preds = rs.forward(r1.cuda(), r2.cuda(), iters=iters)
            rows = torch.stack([rs.gather_rows(p) for p in preds])
        q.put((rank, full.cpu(), rows.cpu()))
    except Exception:
        import traceback
        q.put((rank, traceback.format_exc(), None))
    finally:
        dist.destroy_process_group()


def seeded_images(name):
    """The images of a seeded BASELINE-size golden (make_golden.e2e_seeded_case),
    regenerated from its seed, with the manifest's sha256 checked."""
    from golden_util import image_digest, manifest, stereo_pair
    case = manifest()["cases"][name]
    img1, img2 = stereo_pair(1, case["H"], case["W"], case["seed"])
    assert image_digest(img1, img2) == case["image_sha256"], name
    return img1, img2, case


def run_gpu_config4(rank, world, port, q, iters=32):
    """BASELINE configs[3] row-sharded over ``world`` ranks sharing cuda:0
    (gloo, host-staged exchanges): the product RowShardedStereo defaults
    (per-conv halos, side stream, stacked z/r convs) on the 1984x2880 golden
    pair; rank 0 returns the gathered final disparity."""
    import torch
    import torch.distributed as dist
    import pkgload
    pkgload.load()
    from raft_stereo_amd.shard import RowShardedStereo

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        net = gpu_model()
        img1, img2, _ = seeded_images("e2e_config4")
        with torch.no_grad():
            rs = RowShardedStereo(net, rank, world)
            assert rs.per_conv and rs.side_stream and rs.fuse_zr
            preds = rs.forward(img1.cuda(), img2.cuda(), iters=iters)
            disp = rs.gather_rows(preds[-1])[:, 0].cpu()
        q.put((rank, disp if rank == 0 else torch.zeros(0), None))
    except Exception:
        import traceback
        q.put((rank, traceback.format_exc(), None))
    finally:
        dist.destroy_process_group()
