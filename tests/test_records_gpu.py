"""RC_LAYOUT_RECORDS (ABI v10): the 4-level bf16 pair
layout's stored levels 0 and 2 rewritten by the build as 128-B records, one
line per pixel per lookup.  The record values are the row layout's, so every
lookup must equal the row-layout block's bit for bit -- and through it the C
oracle and the reference goldens that pin the bf16 pair kernel
(test_corr_gpu.py::test_bf16_pair_lookup_bitexact, test_shadow_gpu.py).
Reference: model.py:284-316."""
import pytest
import torch

from raft_stereo_amd import CorrBlock1D, _lib
from raft_stereo_amd import corr as rcorr

from test_corr_gpu import special_coords

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

# (B, D, H, W1, W2, radius): W2 over 2..5 waves per tile row, W1 over 1..3
# tiles, W1 != W2 both ways, D with 8 and 10 K stages, radius 1..4
SHAPES = [
    (1, 256, 3, 100, 100, 4),
    (2, 256, 4, 130, 130, 4),
    (1, 256, 5, 200, 200, 4),
    (2, 256, 3, 311, 311, 4),
    (1, 256, 2, 320, 320, 4),
    (1, 256, 3, 96, 311, 4),
    (1, 256, 3, 311, 68, 4),
    (1, 320, 3, 130, 130, 4),
    (1, 256, 3, 150, 150, 3),
    (1, 256, 3, 150, 150, 2),
    (1, 256, 3, 150, 150, 1),
    (2, 256, 1, 40, 130, 4),        # W1 < 64: the second wave row of every tile idle
]


def sid(s):
    return "x".join(map(str, s))


def fmaps(B, D, H, W1, W2, seed):
    g = torch.Generator().manual_seed(seed)
    f1 = torch.randn(B, D, H, W1, generator=g).to(DEV, torch.bfloat16)
    f2 = torch.randn(B, D, H, W2, generator=g).to(DEV, torch.bfloat16)
    return f1, f2, g


def edge_coords(B, H, W1, W2, g):
    """special_coords (NaN, +-inf, +-1e30, +-0, subnormals, tails) plus a
    sweep across both row edges and beyond the last record's centres."""
    c = special_coords(B, H, W1, W2, g)
    x = c[:, 0].reshape(-1)
    n = min(x.numel() - 40, 400)
    x[40:40 + n] = torch.linspace(-90.0, W2 + 90.0, n)
    return c


def bits(t):
    return t.contiguous().view(torch.int32)


@pytest.mark.parametrize("cl", [False, True], ids=["nchw", "nhwc"])
@pytest.mark.parametrize("shape", SHAPES, ids=sid)
def test_records_lookup_bit_identical(shape, cl):
    B, D, H, W1, W2, r = shape
    f1, f2, g = fmaps(B, D, H, W1, W2, 4100 + sum(shape))
    with torch.no_grad():
        rows = CorrBlock1D(f1, f2, num_levels=4, radius=r, channels_last=cl)
        rec = CorrBlock1D(f1, f2, num_levels=4, radius=r, channels_last=cl, layout="records")
        assert rec.layout == "records" and rec._records.shape == (B * H * W1, _lib.rec_count(W2), 64)
        assert rec.levels_stored == [0, 2]
        for c in (edge_coords(B, H, W1, W2, g),
                  torch.cat([torch.arange(W1).float().view(1, 1, 1, W1) - torch.rand(B, 1, H, W1, generator=g) * 64,
                             torch.zeros(B, 1, H, W1)], 1)):
            c = c.to(DEV)
            a, b = rows(c), rec(c)
            assert b.is_contiguous(memory_format=torch.channels_last) == cl
            assert torch.equal(bits(a), bits(b))
        # the fused loop step (coords update + flow + lookup)
        c1 = edge_coords(B, H, W1, W2, g).to(DEV)
        d = torch.randn(c1.shape, generator=g).to(DEV)
        for x, y in zip(rows.lookup_step(c1, d), rec.lookup_step(c1, d)):
            assert torch.equal(bits(x), bits(y))


@pytest.mark.parametrize("shape", [(1, 256, 3, 311, 311, 4), (2, 256, 3, 200, 130, 4)], ids=sid)
def test_records_corr_pyramid(shape):
    """corr_pyramid gathered from the records == the row layout's, every
    level bit for bit (levels 1, 3 and 4 pooled from them on read)."""
    B, D, H, W1, W2, r = shape
    f1, f2, _ = fmaps(B, D, H, W1, W2, 4300 + sum(shape))
    with torch.no_grad():
        rows = CorrBlock1D(f1, f2, num_levels=4, radius=r)
        rec = CorrBlock1D(f1, f2, num_levels=4, radius=r, layout="records")
        pa, pb = rows.corr_pyramid, rec.corr_pyramid
        assert len(pa) == len(pb) == 5
        for l, (x, y) in enumerate(zip(pa, pb)):
            assert x.shape == y.shape == (B * H * W1, 1, 1, W2 >> l)
            assert torch.equal(x.contiguous().view(torch.int16), y.contiguous().view(torch.int16)), l


def test_records_many_tiles_per_workgroup():
    """More tiles than workgroups (the persistent walk): every tile but each
    workgroup's last emits its records inside the next tile's K loop.  Config
    3's per-GPU rows (94 x 311) at B = 4: 1,128 tiles on 256 workgroups."""
    B, D, H, W1, W2, r = 4, 256, 94, 311, 311, 4
    f1, f2, g = fmaps(B, D, H, W1, W2, 4500)
    with torch.no_grad():
        rows = CorrBlock1D(f1, f2, num_levels=4, radius=r, channels_last=True)
        rec = CorrBlock1D(f1, f2, num_levels=4, radius=r, channels_last=True, layout="records")
        lv0 = rcorr.records_level(rec._records, 0, W2)
        lv2 = rcorr.records_level(rec._records, 2, W2)
        assert torch.equal(lv0.contiguous().view(torch.int16), rows._levels[0].contiguous().view(torch.int16))
        assert torch.equal(lv2.contiguous().view(torch.int16), rows._levels[2].contiguous().view(torch.int16))
        # zero padding: level-2 slots past the row and level-0 slots before it
        recs = rec._records.view(-1, _lib.rec_count(W2), 64)
        assert int(recs[:, 0, :14].view(torch.int16).abs().sum()) == 0          # level-2 elements -14..-1
        assert int(recs[:, 0, 26:52].view(torch.int16).abs().sum()) == 0        # level-0 elements -26..-1
        for _ in range(3):
            c = edge_coords(B, H, W1, W2, g).to(DEV)
            assert torch.equal(bits(rows(c)), bits(rec(c)))


def test_records_gradients_equal_rows():
    """The backward does not read the pyramid: the record block's fmap
    gradients are the row block's (same kernels, same inputs)."""
    B, D, H, W1, W2, r = 1, 256, 3, 130, 130, 4
    f1, f2, g = fmaps(B, D, H, W1, W2, 4700)
    c = edge_coords(B, H, W1, W2, g).to(DEV)
    c[:, 0] = torch.nan_to_num(c[:, 0], nan=3.0, posinf=5.0, neginf=-5.0).clamp(-100, 400)
    grads = []
    for layout in ("rows", "records"):
        a, b = f1.clone().requires_grad_(), f2.clone().requires_grad_()
        blk = CorrBlock1D(a, b, num_levels=4, radius=r, layout=layout)
        (blk(c) * torch.linspace(-1, 1, 36, device=DEV).view(1, 36, 1, 1)).sum().backward()
        grads.append((a.grad, b.grad))
    for x, y in zip(*grads):
        assert torch.equal(x.float(), y.float())


def test_records_refusals():
    f1, f2, _ = fmaps(1, 256, 2, 130, 130, 4900)
    for kw in (dict(pyramid_dtype=torch.float32), dict(num_levels=2), dict(radius=5), dict(shadow=True),
               dict(low_latency=True), dict(exact_f32=True)):
        args = dict(num_levels=4, radius=4, layout="records")
        args.update(kw)
        with pytest.raises(ValueError):
            CorrBlock1D(f1, f2, **args)
    g1, g2, _ = fmaps(1, 256, 2, 64, 64, 4901)            # W2 <= 64
    with pytest.raises(ValueError):
        CorrBlock1D(g1, g2, num_levels=4, radius=4, layout="records")
    h1, h2, _ = fmaps(1, 128, 2, 130, 130, 4902)          # D <= 224
    with pytest.raises(ValueError):
        CorrBlock1D(h1, h2, num_levels=4, radius=4, layout="records")
    blk = CorrBlock1D(f1, f2, num_levels=4, radius=4, layout="records")
    with torch.no_grad(), pytest.raises(RuntimeError):
        blk.lookup_convc1(torch.zeros(1, 2, 2, 130, device=DEV), torch.zeros(64, 36, 1, 1, device=DEV))
    # the C-ABI: the per-level lookup refuses the flag; the chain lookup
    # refuses it with fp32 or a shadow flag
    c = torch.zeros(1, 2, 130, device=DEV)
    out = torch.empty(1, 36, 2, 130, device=DEV)
    ptrs, widths, lds = rcorr._records_args(blk._records, 130)
    lib = _lib.lib()
    rc = lib.rc_corr_lookup(ptrs, widths, lds, _lib.RC_BF16 | _lib.RC_LAYOUT_RECORDS, 4, 4, c.data_ptr(),
                            2 * 130, 1, 2, 130, out.data_ptr(), None)
    assert rc == _lib.RC_EUNSUPPORTED
    for dt in (_lib.RC_F32 | _lib.RC_LAYOUT_RECORDS, _lib.RC_BF16 | _lib.RC_LAYOUT_RECORDS | _lib.shadow_level(0),
               _lib.RC_BF16 | _lib.RC_LAYOUT_RECORDS | _lib.RC_LAYOUT_DISPARITY):
        rc = lib.rc_corr_lookup_chain(ptrs, widths, lds, dt, 4, 4, c.data_ptr(), 2 * 130, 1, 2, 130,
                                      out.data_ptr(), None)
        assert rc in (_lib.RC_EUNSUPPORTED, _lib.RC_EINVAL), dt


def test_records_config3_fullsize_bit_identical():
    """BASELINE config 3 at its per-GPU size (B = 64, 94 x 311 fmaps): the
    records (5.27 GB, past 4 GiB: the build stores through 64-bit addresses,
    the lookup addresses each block's records from its own base) against the
    shadowed rows, on the bench field and the special coordinates."""
    B, D, H, W1, W2, r = 64, 256, 94, 311, 311, 4
    f1, f2, g = fmaps(B, D, H, W1, W2, 5100)
    with torch.no_grad():
        rows = CorrBlock1D(f1, f2, num_levels=4, radius=r, channels_last=True)
        rec = CorrBlock1D(f1, f2, num_levels=4, radius=r, channels_last=True, layout="records")
        assert rec._records.numel() * 2 > 4 << 30
        bench_field = torch.cat([torch.arange(W1).float().view(1, 1, 1, W1) - torch.rand(B, 1, H, W1, generator=g) * 64,
                                 torch.zeros(B, 1, H, W1)], 1)
        for c in (bench_field, edge_coords(B, H, W1, W2, g)):
            c = c.to(DEV)
            assert torch.equal(bits(rows(c)), bits(rec(c)))


def test_auto_layout_rule():
    """layout="auto": the records for a bf16 pyramid the record build serves
    once its level 0 exceeds the 256 MiB Infinity Cache (config 3 per-GPU
    batch >= 16), the rows otherwise (profiles/r06/z, za)."""
    def z(B, D, H, W, dt=torch.bfloat16):
        return torch.zeros(B, D, H, W, dtype=dt, device=DEV)
    assert rcorr.auto_layout(z(16, 256, 94, 311), z(16, 256, 94, 311), 4, 4) == "records"
    assert rcorr.auto_layout(z(8, 256, 94, 311), z(8, 256, 94, 311), 4, 4) == "rows"       # 145 MB
    assert rcorr.auto_layout(z(16, 256, 94, 311, torch.float32), z(16, 256, 94, 311, torch.float32), 4, 4) == "rows"
    assert rcorr.auto_layout(z(16, 256, 94, 311), z(16, 256, 94, 311), 4, 4, shadow=True) == "rows"
    assert rcorr.auto_layout(z(4, 256, 94, 400), z(4, 256, 94, 400), 4, 4) == "rows"       # W2 > 320
    with torch.no_grad():
        f = z(16, 256, 94, 311)
        assert CorrBlock1D(f, f, num_levels=4, radius=4, layout="auto").layout == "records"
        g = z(2, 256, 8, 311)
        assert CorrBlock1D(g, g, num_levels=4, radius=4, layout="auto").layout == "rows"
