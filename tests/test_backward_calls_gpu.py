"""rc_corr_lookup_backward_calls (ABI v7): the gradients of
all lookup calls of a block summed in one pass, the pixel's pair-layout rows
held on chip.

Reference: grid_sample's input gradient (model.py:275) for every call of the
lookup (:376) added into the levels, then avg_pool2d's backward (:294).
Parity: against the C oracle's per-level gradients folded into the pair
layout (<= 1e-6 normalised: only the association of the fp32 sums differs)
and against the per-call kernel (the same bound), NaN / inf / subnormal /
far out-of-range x included; overwrite mode must write every row of a
NaN-filled buffer (padding columns as zeros), accumulate mode must add to
what is there; more than 32 calls run as two launches; rows too wide for
LDS and the per-level layout fall back to per-call launches with the same
results.
"""
import numpy as np
import pytest
import torch

from golden_util import norm_err, rel_l2
from oracle import coracle
from raft_stereo_amd import CorrBlock1D
from raft_stereo_amd import corr as rcorr

from test_corr_gpu import special_coords

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

SHAPES = [
    # B, H, W1, W2, L, r, calls
    (2, 3, 57, 240, 4, 4, 32),
    (1, 4, 96, 240, 4, 4, 37),      # two launches (32 + 5)
    (1, 2, 40, 311, 4, 3, 5),       # odd widths 311/155/77/38
    (1, 3, 33, 64, 2, 2, 3),        # one level pair
    (1, 2, 20, 16, 4, 1, 4),        # level 3 of width 2
    (1, 2, 64, 125, 2, 4, 1),       # odd level 0, one call
    (3, 1, 70, 720, 4, 4, 6),       # config-4 width (32-pixel workgroups would exceed 64 KB)
]


def make_calls(B, H, W1, W2, L, r, calls, seed):
    g = torch.Generator().manual_seed(seed)
    cs, gs = [], []
    for k in range(calls):
        c = special_coords(B, H, W1, W2, g)
        if k % 3 == 1:                       # integer x (the ne corner weight is 0)
            c[:, 0] = torch.round(c[:, 0])
        cs.append(c)
        gs.append(torch.randn(B, L * (2 * r + 1), H, W1, generator=g))
    return cs, gs


def oracle_pair(widths, cs, gs, L, r):
    ref = None
    for c, go in zip(cs, gs):
        ref = coracle.corr_lookup_backward(widths, c.numpy(), go.numpy(), L, r, ref)
    out = []
    for e in range(0, L, 2):                 # g_e + avg_pool2d backward of g_{e+1}
        want = np.array(ref[e], dtype=np.float64)
        half = np.repeat(np.asarray(ref[e + 1], np.float64) * 0.5, 2, axis=1)
        want[:, :half.shape[1]] += half
        out.append(want)
    return out


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_calls_vs_oracle_and_per_call(shape):
    B, H, W1, W2, L, r, calls = shape
    widths = [W2 >> i for i in range(L)]
    P = B * H * W1
    cs, gs = make_calls(B, H, W1, W2, L, r, calls, seed=sum(shape) * 11)
    cd = [c.to(DEV) for c in cs]
    gd = [x.to(DEV) for x in gs]
    dev = torch.device(DEV)
    # overwrite into NaN-filled buffers: every row and its padding is written
    calls_buf = rcorr.grad_buffers(P, widths, dev, pair=True, zero=False)
    for t in calls_buf:
        if t is not None:
            (t._base if t._base is not None else t).fill_(float("nan"))
    rcorr.lookup_backward_calls(calls_buf, cd, gd, L, r, overwrite=True)
    per_call = rcorr.grad_buffers(P, widths, dev, pair=True)
    for c, go in zip(cd, gd):
        rcorr.lookup_backward(per_call, c, go, L, r)
    torch.cuda.synchronize()
    want = oracle_pair(widths, cs, gs, L, r)
    for k, e in enumerate(range(0, L, 2)):
        got = calls_buf[e].cpu().numpy()
        assert np.isfinite(got).all(), f"level {e}: unwritten rows"
        assert norm_err(got, want[k]) <= 1e-6 and rel_l2(got, want[k]) <= 1e-6, f"level {e} vs oracle"
        pc = per_call[e].cpu().numpy()
        assert norm_err(got, pc) <= 1e-6, f"level {e} vs per-call kernel"
        full = calls_buf[e]._base if calls_buf[e]._base is not None else calls_buf[e]
        pad = full.view(P, -1)[:, widths[e]:].cpu().numpy()
        assert (pad == 0).all(), f"level {e}: padding not zeroed"


def test_calls_accumulate_adds_to_buffers():
    B, H, W1, W2, L, r, calls = 1, 3, 48, 120, 4, 4, 7
    widths = [W2 >> i for i in range(L)]
    P = B * H * W1
    cs, gs = make_calls(B, H, W1, W2, L, r, calls, seed=4321)
    dev = torch.device(DEV)
    buf = rcorr.grad_buffers(P, widths, dev, pair=True)
    g = torch.Generator().manual_seed(5)
    init = []
    for t in buf:
        if t is not None:
            v = torch.randn(t.shape, generator=g)
            t.copy_(v)
            init.append(v.double().numpy())
    rcorr.lookup_backward_calls(buf, [c.to(DEV) for c in cs], [x.to(DEV) for x in gs], L, r)
    want = oracle_pair(widths, cs, gs, L, r)
    for k, e in enumerate(range(0, L, 2)):
        got = buf[e].cpu().numpy()
        assert norm_err(got, want[k] + init[k]) <= 1e-6, f"level {e}"


@pytest.mark.parametrize("case", ["wide", "per_level"])
def test_calls_fallbacks_match_per_call(case):
    """Rows too wide for the whole-row kernel (W2 = 2600: the compact kernel
    keeps only each lane's touched range, so it serves them; same sums up to
    association), and the per-level layout (3 levels: per-call launches,
    zeroed first in overwrite mode -- the per-call sums bit for bit)."""
    if case == "wide":
        B, H, W1, W2, L, r, calls, pair = 1, 2, 16, 2600, 4, 4, 3, True
    else:
        B, H, W1, W2, L, r, calls, pair = 1, 3, 40, 96, 3, 4, 4, False
    widths = [W2 >> i for i in range(L)]
    P = B * H * W1
    cs, gs = make_calls(B, H, W1, W2, L, r, calls, seed=77 + L)
    cd = [c.to(DEV) for c in cs]
    gd = [x.to(DEV) for x in gs]
    dev = torch.device(DEV)
    a = rcorr.grad_buffers(P, widths, dev, pair=pair, zero=False)
    for t in a:
        if t is not None:
            t.fill_(float("nan"))
    rcorr.lookup_backward_calls(a, cd, gd, L, r, overwrite=True)
    b = rcorr.grad_buffers(P, widths, dev, pair=pair)
    for c, go in zip(cd, gd):
        rcorr.lookup_backward(b, c, go, L, r)
    for ta, tb in zip(a, b):
        if ta is not None:
            if case == "per_level":
                assert torch.equal(ta, tb)
            else:
                assert norm_err(ta.cpu().numpy(), tb.cpu().numpy()) <= 1e-6


@pytest.mark.parametrize("L", [2, 4])
def test_autograd_deferred_equals_per_call(L):
    """CorrBlock1D's autograd with the deferred sum (the default for the pair
    layout) vs grad_deferred=False: fmap gradients within the fp32 contract."""
    B, D, H, W1, W2, r, calls = 2, 32, 3, 50, 96, 4, 6
    g = torch.Generator().manual_seed(60 + L)
    f1 = torch.randn(B, D, H, W1, generator=g)
    f2 = torch.randn(B, D, H, W2, generator=g)
    cs, gs = make_calls(B, H, W1, W2, L, r, calls, seed=61 + L)
    grads = {}
    for deferred in (True, False):
        a = f1.to(DEV).requires_grad_(True)
        b = f2.to(DEV).requires_grad_(True)
        blk = CorrBlock1D(a, b, num_levels=L, radius=r, grad_deferred=deferred)
        assert blk._state.deferred == deferred
        outs = [blk(c.to(DEV)) for c in cs]
        torch.autograd.backward(outs, [x.to(DEV) for x in gs])
        grads[deferred] = (a.grad.cpu().numpy(), b.grad.cpu().numpy())
    for x, y in zip(grads[True], grads[False]):
        assert norm_err(x, y) <= 1e-5 and rel_l2(x, y) <= 1e-6


def test_autograd_deferred_bounded_retention():
    """the deferred state holds at most max_pending_calls recorded
    calls (here 3 of 7: partial passes of 3, 3, then 1 at the build node, the
    first overwriting, the rest adding) and stores every grad_out as contiguous
    fp32 when it is recorded (channels_last gradients here); the fmap
    gradients equal the one-pass deferred sum within the fp32 contract."""
    B, D, H, W1, W2, L, r, calls = 2, 32, 3, 50, 96, 4, 4, 7
    g = torch.Generator().manual_seed(71)
    f1 = torch.randn(B, D, H, W1, generator=g)
    f2 = torch.randn(B, D, H, W2, generator=g)
    cs, gs = make_calls(B, H, W1, W2, L, r, calls, seed=72)
    grads, seen = {}, []
    for cap in (32, 3):
        a = f1.to(DEV).requires_grad_(True)
        b = f2.to(DEV).requires_grad_(True)
        blk = CorrBlock1D(a, b, num_levels=L, radius=r)
        st = blk._state
        st.max_pending_calls = cap
        flush = st._flush

        def spy(flush=flush, st=st):
            seen.append((cap, len(st.pending)))
            assert all(go.dtype == torch.float32 and go.is_contiguous() for _, go in st.pending)
            flush()
        st._flush = spy
        outs = [blk(c.to(DEV)) for c in cs]
        gos = [x.to(DEV).contiguous(memory_format=torch.channels_last) for x in gs]
        torch.autograd.backward(outs, gos)
        assert not st.pending and st.pending_bytes == 0
        grads[cap] = (a.grad.cpu().numpy(), b.grad.cpu().numpy())
    assert [n for c, n in seen if c == 3] == [3, 3, 1] and [n for c, n in seen if c == 32] == [7]
    for x, y in zip(grads[3], grads[32]):
        assert norm_err(x, y) <= 1e-5 and rel_l2(x, y) <= 1e-6


@pytest.mark.parametrize("spread", ["bench", "whole_row"])
def test_compact_equals_whole_row_kernel(spread):
    """The compact-row kernel (RAFTCORR_BWDC_VARIANT=3; the launcher's choice
    for wide rows) against the whole-row kernel (=1), bit for bit: at the bench's
    coordinates (one pass) and with x spread over the whole row (every lane
    needs its full row: several passes per block)."""
    import os
    from raft_stereo_amd import _lib
    B, H, W1, W2, L, r, calls = 2, 3, 60, 240, 4, 4, 12
    g = torch.Generator().manual_seed(11 if spread == "bench" else 12)
    cs, gs = make_calls(B, H, W1, W2, L, r, calls, seed=21 if spread == "bench" else 22)
    if spread == "whole_row":
        for c in cs:
            c[:, 0] = torch.rand(B, H, W1, generator=g) * (W2 + 20) - 10
    cd = [c.to(DEV) for c in cs]
    gd = [x.to(DEV) for x in gs]
    P = B * H * W1
    widths = [W2 >> i for i in range(L)]
    out = {}
    with _lib.dev_library():
        for v in ("3", "1"):
            os.environ["RAFTCORR_BWDC_VARIANT"] = v
            buf = rcorr.grad_buffers(P, widths, torch.device(DEV), pair=True, zero=False)
            for t in buf:
                if t is not None:
                    (t._base if t._base is not None else t).fill_(float("nan"))
            rcorr.lookup_backward_calls(buf, cd, gd, L, r, overwrite=True)
            out[v] = buf
        os.environ["RAFTCORR_BWDC_VARIANT"] = "0"
    for ta, tb in zip(out["3"], out["1"]):
        if ta is not None:
            assert torch.equal(ta, tb)
