"""Backward of the correlation path.

The reference path is differentiable to the feature maps (model.py:375
detaches only the coordinates).  Goldens (tests/golden/backward_*.npz, made
by make_golden.py with the reference's own autograd) hold the fmap gradients
and every read level's total gradient for several lookup calls per block.

Tolerances (fp32, the SURVEY §8d contract): max|d|/max|ref| <= 1e-4 and
rel-L2 <= 1e-5 for the fmap gradients; level gradients <= 1e-5 normalised
(the only difference is the summation order of tap / call contributions).
"""
import contextlib

import numpy as np
import pytest
import torch

from golden_util import files, load, norm_err, rel_l2
from oracle import coracle

BWD = files("backward")
TOL, L2 = 1e-4, 1e-5


def oracle_grads(z):
    """Oracle backward for a golden case: per-level grads, folded totals,
    fmap grads."""
    L, r = int(z["num_levels"]), int(z["radius"])
    W2 = z["fmap2"].shape[3]
    widths = [W2 >> i for i in range(L)]
    g = None
    for k in range(z["coords"].shape[0]):
        g = coracle.corr_lookup_backward(widths, z["coords"][k], z["grad_out"][k], L, r, g)
    df1, df2 = coracle.corr_build_backward(z["fmap1"], z["fmap2"], g)
    return g, coracle.fold_grads(g), df1, df2


def test_backward_goldens_present():
    assert len(BWD) >= 4


@pytest.mark.parametrize("path", BWD, ids=lambda p: p.split("/")[-1])
def test_oracle_backward_vs_reference(path):
    """The C oracle restates the reference's autograd (CPU only)."""
    z = load(path)
    L = int(z["num_levels"])
    _, tot, df1, df2 = oracle_grads(z)
    for i in range(L):
        assert norm_err(tot[i], z[f"grad_level{i}"]) <= 1e-5, f"level {i}"
    assert norm_err(df1, z["grad_fmap1"]) <= 1e-5 and rel_l2(df1, z["grad_fmap1"]) <= 1e-6
    assert norm_err(df2, z["grad_fmap2"]) <= 1e-5 and rel_l2(df2, z["grad_fmap2"]) <= 1e-6


# ------------------------------------------------------------------ GPU

DEV = "cuda:0"


def cu(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def run_autograd(f1, f2, coords_list, gout_list, L, r, pyramid_dtype=None):
    """Our CorrBlock1D under autograd: returns (d fmap1, d fmap2)."""
    from raft_stereo_amd import CorrBlock1D
    a = f1.detach().clone().requires_grad_(True)
    b = f2.detach().clone().requires_grad_(True)
    blk = CorrBlock1D(a, b, num_levels=L, radius=r, pyramid_dtype=pyramid_dtype)
    loss = sum((blk(c) * g).sum() for c, g in zip(coords_list, gout_list))
    loss.backward()
    return a.grad, b.grad


@pytest.mark.gpu
@pytest.mark.parametrize("path", BWD, ids=lambda p: p.split("/")[-1])
def test_backward_vs_golden(path):
    z = load(path)
    L, r = int(z["num_levels"]), int(z["radius"])
    n = z["coords"].shape[0]
    d1, d2 = run_autograd(cu(z["fmap1"]), cu(z["fmap2"]), [cu(z["coords"][k]) for k in range(n)],
                          [cu(z["grad_out"][k]) for k in range(n)], L, r)
    d1, d2 = d1.cpu().numpy(), d2.cpu().numpy()
    assert norm_err(d1, z["grad_fmap1"]) <= TOL and rel_l2(d1, z["grad_fmap1"]) <= L2
    assert norm_err(d2, z["grad_fmap2"]) <= TOL and rel_l2(d2, z["grad_fmap2"]) <= L2


@pytest.mark.gpu
@pytest.mark.parametrize("path", BWD, ids=lambda p: p.split("/")[-1])
def test_lookup_backward_levels_vs_oracle(path):
    """rc_corr_lookup_backward alone: per-level gradients vs the oracle."""
    from raft_stereo_amd import corr as rcorr
    z = load(path)
    L, r = int(z["num_levels"]), int(z["radius"])
    g_ref, _, _, _ = oracle_grads(z)
    B, _, H, W1 = z["coords"][0].shape
    W2 = z["fmap2"].shape[3]
    grads = rcorr.grad_buffers(B * H * W1, [W2 >> i for i in range(L)], torch.device(DEV))
    for k in range(z["coords"].shape[0]):
        rcorr.lookup_backward(grads, cu(z["coords"][k]), cu(z["grad_out"][k]), L, r)
    for i in range(L):
        got = grads[i].cpu().numpy()
        assert norm_err(got, g_ref[i]) <= 1e-6, f"level {i}"
        # the row padding is never written
        full = torch.as_strided(grads[i], (grads[i].shape[0], grads[i].stride(0)),
                                (grads[i].stride(0), 1))
        assert torch.count_nonzero(full[:, grads[i].shape[1]:]) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("L,r,W2", [(4, 4, 240), (3, 4, 311), (4, 3, 70), (2, 2, 33), (1, 1, 16),
                                    (4, 1, 37)])
def test_lookup_backward_prefetch_kernel_bit_identical(L, r, W2, monkeypatch):
    """lookup_bwd_pre_kernel (all loads up front) vs lookup_bwd_kernel (per-level
    waits, RAFTCORR_LOOKUP_BWD_VARIANT=1): same accumulation, bit for bit,
    including NaN / inf / far out-of-range coordinates."""
    from raft_stereo_amd import corr as rcorr
    g = torch.Generator().manual_seed(L * 100 + r * 10 + W2)
    B, H, W1 = 2, 3, 57
    widths = [W2 >> i for i in range(L)]
    cs, gs = [], []
    for _ in range(3):
        x = torch.arange(W1).float().view(1, 1, 1, W1) - torch.rand(B, 1, H, W1, generator=g) * 48
        x[..., ::5] = torch.randint(-20, W2 + 20, x[..., ::5].shape, generator=g).float()
        x[0, 0, 0, :6] = torch.tensor([float("nan"), float("inf"), -float("inf"), 1e30, -1e30, 1e-40])
        cs.append(torch.cat([x, torch.randn(B, 1, H, W1, generator=g)], 1).to(DEV))
        gs.append(torch.randn(B, L * (2 * r + 1), H, W1, generator=g).to(DEV))
    from raft_stereo_amd import _lib
    out = {}
    for v in ("1", "0"):
        # "1": the dev library's knob; "0": the product library
        monkeypatch.setenv("RAFTCORR_LOOKUP_BWD_VARIANT", v)
        with (_lib.dev_library() if v == "1" else contextlib.nullcontext()):
            grads = rcorr.grad_buffers(B * H * W1, widths, torch.device(DEV))
            for c, go in zip(cs, gs):
                rcorr.lookup_backward(grads, c, go, L, r)
            torch.cuda.synchronize()
        out[v] = grads
    for i in range(L):
        a0 = torch.as_strided(out["0"][i], (out["0"][i].shape[0], out["0"][i].stride(0)),
                              (out["0"][i].stride(0), 1))
        a1 = torch.as_strided(out["1"][i], (out["1"][i].shape[0], out["1"][i].stride(0)),
                              (out["1"][i].stride(0), 1))
        assert torch.equal(a0, a1), f"level {i}"


SHAPES = [
    # B, D, H, W1, W2, L, r, calls
    (2, 256, 3, 240, 240, 4, 4, 3),     # config-2 row width
    (1, 64, 2, 311, 311, 4, 4, 2),      # W % 4 != 0 (scalar paths)
    (1, 37, 2, 33, 70, 3, 3, 2),        # D % 4 != 0, W1 != W2
    (1, 200, 1, 130, 129, 5, 2, 2),     # D, W not multiples of 128; 5 levels
    (3, 16, 1, 8, 16, 1, 1, 4),         # tiny, one level
]


@pytest.mark.gpu
@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_backward_random_vs_oracle(shape):
    B, D, H, W1, W2, L, r, calls = shape
    g = torch.Generator().manual_seed(sum(shape))
    f1 = torch.randn(B, D, H, W1, generator=g)
    f2 = torch.randn(B, D, H, W2, generator=g)
    cs, gs = [], []
    for _ in range(calls):
        x = torch.arange(W1).float().view(1, 1, 1, W1) - torch.rand(B, 1, H, W1, generator=g) * 48
        x[..., ::5] = torch.randint(-12, W2 + 12, x[..., ::5].shape, generator=g).float()
        cs.append(torch.cat([x, torch.randn(B, 1, H, W1, generator=g)], 1))
        gs.append(torch.randn(B, L * (2 * r + 1), H, W1, generator=g))
    d1, d2 = run_autograd(f1.to(DEV), f2.to(DEV), [c.to(DEV) for c in cs], [x.to(DEV) for x in gs],
                          L, r)
    widths = [W2 >> i for i in range(L)]
    gr = None
    for c, x in zip(cs, gs):
        gr = coracle.corr_lookup_backward(widths, c.numpy(), x.numpy(), L, r, gr)
    r1, r2 = coracle.corr_build_backward(f1.numpy(), f2.numpy(), gr)
    d1, d2 = d1.cpu().numpy(), d2.cpu().numpy()
    assert norm_err(d1, r1) <= TOL and rel_l2(d1, r1) <= L2
    assert norm_err(d2, r2) <= TOL and rel_l2(d2, r2) <= L2


@pytest.mark.gpu
def test_backward_matches_torch_autograd_of_restatement():
    """Same inputs through the reference's ATen sequence (oracle/torch_ref.py,
    autograd on the GPU) and through our kernels."""
    from oracle import torch_ref
    g = torch.Generator().manual_seed(77)
    B, D, H, W1, W2, L, r = 2, 64, 4, 96, 96, 4, 4
    f1 = torch.randn(B, D, H, W1, generator=g).to(DEV)
    f2 = torch.randn(B, D, H, W2, generator=g).to(DEV)
    x = torch.arange(W1).float().view(1, 1, 1, W1) - torch.rand(B, 1, H, W1, generator=g) * 40
    c = torch.cat([x, torch.zeros_like(x)], 1).to(DEV)
    go = torch.randn(B, L * (2 * r + 1), H, W1, generator=g).to(DEV)
    d1, d2 = run_autograd(f1, f2, [c], [go], L, r)
    a = f1.clone().requires_grad_(True)
    b = f2.clone().requires_grad_(True)
    (torch_ref.TorchCorrBlock1D(a, b, L, r)(c) * go).sum().backward()
    assert norm_err(d1.cpu().numpy(), a.grad.cpu().numpy()) <= TOL
    assert norm_err(d2.cpu().numpy(), b.grad.cpu().numpy()) <= TOL


@pytest.mark.gpu
def test_backward_bf16_fmaps_and_unused_lookup():
    """bf16 fmaps get bf16 gradients (computed in fp32); a block whose lookups
    never reach the loss gives no gradient; inference is unaffected."""
    from raft_stereo_amd import CorrBlock1D
    g = torch.Generator().manual_seed(5)
    f1 = torch.randn(1, 32, 2, 64, generator=g).to(DEV, torch.bfloat16).requires_grad_(True)
    f2 = torch.randn(1, 32, 2, 64, generator=g).to(DEV, torch.bfloat16).requires_grad_(True)
    c = (torch.arange(64).float().view(1, 1, 1, 64) - 10).expand(1, 2, 2, 64).contiguous().to(DEV)
    blk = CorrBlock1D(f1, f2, num_levels=4, radius=4)
    blk(c).sum().backward()
    assert f1.grad.dtype == torch.bfloat16 and torch.isfinite(f1.grad.float()).all()
    assert f2.grad.abs().sum() > 0
    h1 = f1.detach().float().requires_grad_(True)
    blk2 = CorrBlock1D(h1, h1.detach(), num_levels=2, radius=2)
    blk2(c)                                     # output unused
    (h1 * 0).sum().backward()
    assert torch.count_nonzero(h1.grad) == 0
    with torch.no_grad():
        out = CorrBlock1D(h1, h1, num_levels=2, radius=2)(c)
    assert out.grad_fn is None


PAIR_SHAPES = [
    # B, D, H, W1, W2, L, r, calls
    (2, 32, 3, 57, 240, 4, 4, 3),
    (1, 16, 2, 40, 311, 4, 3, 2),      # odd widths 311/155/77/38
    (1, 8, 2, 33, 64, 2, 2, 3),        # 2 levels: level 1 folded into level 0
    (1, 8, 2, 20, 16, 4, 1, 2),        # level 3 of width 2
]


@pytest.mark.gpu
@pytest.mark.parametrize("shape", PAIR_SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_pair_layout_backward(shape):
    """The pair layout (levels 1, 3 folded into 0, 2 by lookup_bwd_pair_kernel,
    then rc_corr_build_backward's pair fold) vs the oracle's per-level
    gradients folded the same way (<= 1e-6 normalised: only the order of
    additions differs), and its fmap gradients vs the per-level layout's
    (fp32 contract), NaN / inf / far out-of-range coords included."""
    from raft_stereo_amd import corr as rcorr
    B, D, H, W1, W2, L, r, calls = shape
    g = torch.Generator().manual_seed(sum(shape) * 7)
    f1 = torch.randn(B, D, H, W1, generator=g)
    f2 = torch.randn(B, D, H, W2, generator=g)
    widths = [W2 >> i for i in range(L)]
    cs, gs = [], []
    for _ in range(calls):
        x = torch.arange(W1).float().view(1, 1, 1, W1) - torch.rand(B, 1, H, W1, generator=g) * 48
        x[..., ::5] = torch.randint(-20, W2 + 20, x[..., ::5].shape, generator=g).float()
        x[0, 0, 0, :6] = torch.tensor([float("nan"), float("inf"), -float("inf"), 1e30, -1e30, 0.5])
        cs.append(torch.cat([x, torch.randn(B, 1, H, W1, generator=g)], 1))
        gs.append(torch.randn(B, L * (2 * r + 1), H, W1, generator=g))
    P = B * H * W1
    pair = rcorr.grad_buffers(P, widths, torch.device(DEV), pair=True)
    full = rcorr.grad_buffers(P, widths, torch.device(DEV))
    for c, go in zip(cs, gs):
        rcorr.lookup_backward(pair, c.to(DEV), go.to(DEV), L, r)
        rcorr.lookup_backward(full, c.to(DEV), go.to(DEV), L, r)
    ref = None
    for c, go in zip(cs, gs):
        ref = coracle.corr_lookup_backward(widths, c.numpy(), go.numpy(), L, r, ref)
    for e in range(0, L, 2):                 # ref_e = g_e + avg_pool2d backward of g_{e+1}
        want = np.array(ref[e], dtype=np.float64)
        half = np.repeat(np.asarray(ref[e + 1], np.float64) * 0.5, 2, axis=1)
        want[:, :half.shape[1]] += half
        got = pair[e].cpu().numpy()
        assert norm_err(got, want) <= 1e-6, f"level {e}"
    a1, a2 = rcorr.build_backward(f1.to(DEV), f2.to(DEV), pair)
    b1, b2 = rcorr.build_backward(f1.to(DEV), f2.to(DEV), full)
    for a_, b_ in ((a1, b1), (a2, b2)):
        a_, b_ = a_.cpu().numpy(), b_.cpu().numpy()
        assert norm_err(a_, b_) <= 1e-5 and rel_l2(a_, b_) <= 1e-6
