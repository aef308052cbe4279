// Persistent split-bf16 volume kernel with a deferred epilogue.
//
// DEV LIBRARY ONLY (RAFTCORR_SPLIT_KERNEL=4): measured and not kept --
// bit-identical, but config 2 287.2 vs 250.2 us and Middlebury 1240 vs 1032
// for build_split_kernel (profiles/r04/q): holding two
// fragment columns costs 249 VGPRs and 211 SGPR spills, and every K step's
// vmcnt(0) now also waits for the previous step's piece stores.
//
// Same arithmetic, tiles, ring and per-wave blocks as build_split_kernel
// (volume_split.hip) -- bit-identical output -- but each
// workgroup walks a run of tiles, and a finished tile's epilogue is not run
// between tiles: its scaled level-0 values stay in registers (64 VGPRs) and
// are stored in eight half-pieces (8 w1 rows of one fragment column, every
// level) during the NEXT tile's K steps, one per step, through a 2 KB
// per-wave LDS image beside the ring.  The ring runs on across tiles (the
// last K step of a tile issues the next tile's first), so neither the
// epilogue nor a new tile's first DMA round trip stalls the MFMAs.  Why
// (profiles/r04/lmno): the epilogue's own instructions -- staging, reads,
// waits -- not its HBM bytes, cost ~15-20 % of the per-tile kernel
// (L2-resident stores 271 vs 274 us; no stores 216).
//
// The piece stores are issued before the next K step's DMA and covered by
// the same vmcnt(0) at the following step: they get one K step to drain.

#include "split_ring.h"

#ifdef RAFTCORR_DEV
namespace rc {

constexpr int kPStb = 8 * (64 + 4) * 4;                   // per-wave half-piece image (2,176 B)
constexpr int kPLds = kSpSL * kSpSlot + 4 * kPStb;        // 75,264 B
static_assert(2 * kPLds <= 160 * 1024, "two workgroups per CU");

// One tile of the walk as one wave sees it (the wave's block inside it).
struct PTile {
    __amdgpu_buffer_rsrc_t r1, r2;
    int row, h, M0, N0, o1, o2, fa, fb;
};

__device__ __forceinline__ PTile p_tile(const BuildArgs &a, int id, int tf1, int tf2, int tiles1, int tiles2,
                                        int wave) {
    PTile t;
    const int T = tiles1 * tiles2;
    t.row = id / T;
    const int tile = id - t.row * T, tm = tile / tiles2, tn = tile - tm * tiles2;
    const int b = t.row / a.H;
    t.h = t.row - b * a.H;
    t.M0 = tm * 16 * tf1;
    t.N0 = tn * 16 * tf2;
    const int wm = wave & 1, wn = wave >> 1;
    const int h1 = (tf1 + 1) >> 1, h2 = (tf2 + 1) >> 1;
    t.o1 = 16 * h1 * wm;
    t.o2 = 16 * h2 * wn;
    const long long img1 = (long long)a.D * a.H * a.W1, img2 = (long long)a.D * a.H * a.W2;
    t.r1 = make_rsrc(reinterpret_cast<const float *>(a.f1) + b * img1, clamp_bytes(img1 * 4));
    t.r2 = make_rsrc(reinterpret_cast<const float *>(a.f2) + b * img2, clamp_bytes(img2 * 4));
    const int n1 = wm ? tf1 - h1 : h1, n2 = wn ? tf2 - h2 : h2;
    const int cw1 = a.W1 - (t.M0 + t.o1), cw2 = a.W2 - (t.N0 + t.o2);
    const int v1 = cw1 <= 0 ? 0 : min(n1, (cw1 + 15) >> 4), v2 = cw2 <= 0 ? 0 : min(n2, (cw2 + 15) >> 4);
    t.fa = v1 == 0 ? 0 : v2;
    t.fb = v1;
    return t;
}

// This wave's DMA share of d-stage dst of tile t into ring slot `slot`
// (sp_issue's mapping: rows 4w..4w+3 of both operand tiles).
__device__ __forceinline__ void p_issue(const PTile &t, const BuildArgs &a, char *smem, int slot, int dst,
                                        int tw1, int tw2, int wave, int lane) {
    typedef __attribute__((address_space(3))) void lds_void;
    char *sA = smem + slot * kSpSlot, *sB = sA + kSpOp;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int r0 = 4 * wave + 2 * i;
        const int d = dst * kSpBK + r0 + (lane >> 5);
        const int w = 4 * (lane & 31);
        const long long base = (long long)(d < a.D ? d : 0) * a.H + t.h;
        const uint32_t offA = d < a.D && w < tw1 ? (uint32_t)((base * a.W1 + t.M0 + w) * 4) : 0xFFFFFF00u;
        const uint32_t offB = d < a.D && w < tw2 ? (uint32_t)((base * a.W2 + t.N0 + w) * 4) : 0xFFFFFF00u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(t.r1, (lds_void *)(sA + (r0 >> 1) * kSpBlk), 16, (int)offA, 0, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(t.r2, (lds_void *)(sB + (r0 >> 1) * kSpBlk), 16, (int)offB, 0, 0, 0);
    }
}

// The held tile: scaled level-0 values [ma][nb] (lane (i, g): w1 = m0 + 16nb
// + i, w2 = n0 + 16ma + 4g + r) and where they go.
constexpr int kHold = 2;        // held fragment columns (nb = 4 - kHold .. 3); the rest stored at tile end
struct PHold {
    f32x4 v[4][kHold];
};
struct PMeta {
    int row, m0, n0, fa, w1e;
};

// Rows [0, 8) of a wave's staged image of level L (CW columns, pitch CW + 4)
// -> memory; columns at or past cend (the wave's block end) or the level's
// width are not stored.  All reads before one wait, as flush_rows16_fast.
template <int CW, int L>
__device__ __forceinline__ void p_flush8(uint32_t st, const BuildArgs &a, long long rowbase, int w1_0, int n0,
                                         int cend, int w1e, int lane) {
    constexpr int LP = CW / 4, RPI = 64 / LP, NI = (8 + RPI - 1) / RPI;
    static_assert(NI == 1 || NI == 2, "flush instruction count");
    const int Rl = lane / LP, j = (lane - Rl * LP) * 4;
    const int col = (n0 >> L) + j;
    const bool lok = Rl < RPI && col < (a.W2 >> L) && col < (cend >> L);
    f32x4 x[NI];
#pragma unroll
    for (int k = 0; k < NI; ++k) {
        const int R = k * RPI + Rl;
        const uint32_t src = st + 4 * ((R < 8 ? R : 7) * (CW + 4) + j);
        asm volatile("ds_read_b128 %0, %1" : "=v"(x[k]) : "v"(src));
    }
    if constexpr (NI == 1) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(x[0])::"memory");
    else asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(x[0]), "+v"(x[1])::"memory");
#pragma unroll
    for (int k = 0; k < NI; ++k) {
        const int R = k * RPI + Rl, w1 = w1_0 + R;
        if (lok && R < 8 && w1 < w1e) {
            const float v[4] = {x[k][0], x[k][1], x[k][2], x[k][3]};
            store_vec<4>(a.lvl[L], false, (rowbase + w1) * a.ld[L] + col, v, a.shadow[L]);
        }
    }
}

// Half-piece (nb, half) of the held tile, nb = the held column in hd.v[.][0]
// (the hold rotates one column down after both halves): levels 0..nl-1
// (nl <= 3) of rows m0 + 16nb + 8half .. +7, pooled as epilogue_swapped does
// (levels 1-2 are lane-local), staged in this wave's image and stored.
__device__ __forceinline__ void p_piece(const BuildArgs &a, const f32x4 (&c)[4], const PMeta &m, int nb, int half,
                                        int nl, int lane, uint32_t st) {
    const int g = lane >> 4, i = lane & 15, r = i & 7;
    const bool mine = (i >> 3) == half;
    const int w1_0 = m.m0 + 16 * nb + 8 * half;
    const long long rowbase = (long long)m.row * a.W1;
    const int cend = m.n0 + 16 * m.fa;
    if (a.lvl[0]) {
        if (mine) {
#pragma unroll
            for (int ma = 0; ma < 4; ++ma)
                if (ma < m.fa) lds_st4(st + 4 * (r * 68 + 16 * ma + 4 * g), c[ma]);
        }
        p_flush8<64, 0>(st, a, rowbase, w1_0, m.n0, cend, m.w1e, lane);
    }
    if (nl < 2) return;
    float u[4][2];
#pragma unroll
    for (int ma = 0; ma < 4; ++ma) {
        u[ma][0] = pool2(c[ma][0], c[ma][1], false);
        u[ma][1] = pool2(c[ma][2], c[ma][3], false);
    }
    if (a.lvl[1]) {
        if (mine) {
#pragma unroll
            for (int ma = 0; ma < 4; ++ma)
                if (ma < m.fa) lds_st2(st + 4 * (r * 36 + 8 * ma + 2 * g), f32x2{u[ma][0], u[ma][1]});
        }
        p_flush8<32, 1>(st, a, rowbase, w1_0, m.n0, cend, m.w1e, lane);
    }
    if (nl < 3) return;
    if (a.lvl[2]) {
        if (mine) {
#pragma unroll
            for (int ma = 0; ma < 4; ++ma)
                if (ma < m.fa) lds_st1(st + 4 * (r * 20 + 4 * ma + g), pool2(u[ma][0], u[ma][1], false));
        }
        p_flush8<16, 2>(st, a, rowbase, w1_0, m.n0, cend, m.w1e, lane);
    }
}

// Held half-piece q (0 .. 2 kHold - 1): column 4 - kHold + q / 2, which is
// hd.v[.][0] (the hold rotates one column down after both halves).
__device__ __forceinline__ void p_piece_q(const BuildArgs &a, PHold &hd, const PMeta &m, int q, int nl, int lane,
                                          uint32_t st) {
    const f32x4 c[4] = {hd.v[0][0], hd.v[1][0], hd.v[2][0], hd.v[3][0]};
    p_piece(a, c, m, 4 - kHold + (q >> 1), q & 1, nl, lane, st);
    if (q & 1) {
#pragma unroll
        for (int ma = 0; ma < 4; ++ma)
#pragma unroll
            for (int k = 0; k + 1 < kHold; ++k) hd.v[ma][k] = hd.v[ma][k + 1];
    }
}

// Walk state shared by the tile bodies.
struct PWalk {
    int G0, nks, totalK, nl, tw1, tw2, wave, lane;
    uint32_t stg;
};

// One tile: nks K steps (global steps G0 ..), storing the held tile's
// half-pieces as it goes, then this tile's values into the hold.
template <int FA, int FB, int MODE>
__device__ __forceinline__ void p_body(const BuildArgs &a, char *smem, const PTile &ct, const PTile &cn,
                                       const PWalk &w, PHold &hd, PMeta &hm, bool &held) {
    const int lane = w.lane, i = lane & 15, g = lane >> 4;
    const int lrow = (g & 1) * 4 * kSpBlk;
    f32x4 acc[FA > 0 ? FA : 1][4];
#pragma unroll
    for (int x0 = 0; x0 < (FA > 0 ? FA : 1); ++x0)
#pragma unroll
        for (int y0 = 0; y0 < 4; ++y0) acc[x0][y0] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int per = (2 * kHold + w.nks - 1) / w.nks;          // held half-pieces per K step
    for (int ks = 0; ks < w.nks; ++ks) {
        const int G = w.G0 + ks;
        // RAW: my DMA of K step G landed (at G = 0 the prologue's K step 1
        // may still fly); it also covers the previous step's piece stores.
        // WAR: my LDS reads of K step G - 1 are done.  Barrier.
        if (G == 0 && w.totalK > 1) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (held) {
            for (int q0 = 0; q0 < per; ++q0) {
                const int q = ks * per + q0;
                if (q < 2 * kHold) p_piece_q(a, hd, hm, q, w.nl, lane, w.stg);
            }
        }
        __builtin_amdgcn_sched_barrier(0);   // keep the piece code out of the MFMA schedule
        if (G >= 1 && G + 1 < w.totalK) {                      // K step G + 1 into the slots of G - 1
            const bool nx = ks + 1 == w.nks;                   // ... the next tile's first
            const PTile &it = nx ? cn : ct;
            const int lks = nx ? 0 : ks + 1;
            p_issue(it, a, smem, (2 * G + 2) & 3, 2 * lks, w.tw1, w.tw2, w.wave, lane);
            p_issue(it, a, smem, (2 * G + 3) & 3, 2 * lks + 1, w.tw1, w.tw2, w.wave, lane);
        }
        if constexpr (FA > 0) {
            const char *st = smem + ((2 * G + (g >> 1)) & 3) * kSpSlot + lrow;
            const char *pb = st + 4 * (ct.o1 + i);
            const char *pa = st + kSpOp + 4 * (ct.o2 + i);
            SplitFrag fb[FB];
#pragma unroll
            for (int n = 0; n < FB; ++n) fb[n] = sp_read<MODE>(pb + 64 * n);
#pragma unroll
            for (int m = 0; m < FA; ++m) {
                const SplitFrag fa = sp_read<MODE>(pa + 64 * m);
#pragma unroll
                for (int n = 0; n < FB; ++n) sp_mma6(acc[m][n], fa, fb[n]);
            }
        }
    }
    if constexpr (FA > 0) {
        hm.row = ct.row;
        hm.m0 = ct.M0 + ct.o1;
        hm.n0 = ct.N0 + ct.o2;
        hm.fa = FA;
        hm.w1e = min(a.W1, hm.m0 + 16 * FB);
        auto scaled = [&](int ma, int nb) {
            f32x4 x = acc[ma < FA ? ma : 0][nb];
#pragma unroll
            for (int r = 0; r < 4; ++r) x[r] = a.pow2 ? x[r] * a.scale : x[r] / a.sq;
            return x;
        };
        // columns 0 .. 3 - kHold now (the held tile's pieces are all stored by now)
#pragma unroll
        for (int nb = 0; nb < 4 - kHold; ++nb) {
            f32x4 c[4];
#pragma unroll
            for (int ma = 0; ma < 4; ++ma) c[ma] = ma < FA ? scaled(ma, nb) : f32x4{0.f, 0.f, 0.f, 0.f};
            p_piece(a, c, hm, nb, 0, w.nl, lane, w.stg);
            p_piece(a, c, hm, nb, 1, w.nl, lane, w.stg);
        }
#pragma unroll
        for (int ma = 0; ma < 4; ++ma)
#pragma unroll
            for (int k = 0; k < kHold; ++k)
                if (ma < FA) hd.v[ma][k] = scaled(ma, 4 - kHold + k);
        held = true;
    } else {
        held = false;
    }
}

template <int FA, int MODE>
__device__ __forceinline__ void p_fb(int fb, const BuildArgs &a, char *smem, const PTile &ct, const PTile &cn,
                                     const PWalk &w, PHold &hd, PMeta &hm, bool &held) {
    if (fb >= 4) p_body<FA, 4, MODE>(a, smem, ct, cn, w, hd, hm, held);
    else if (fb == 3) p_body<FA, 3, MODE>(a, smem, ct, cn, w, hd, hm, held);
    else if (fb == 2) p_body<FA, 2, MODE>(a, smem, ct, cn, w, hd, hm, held);
    else p_body<FA, 1, MODE>(a, smem, ct, cn, w, hd, hm, held);
}

template <int MODE>
__global__ __launch_bounds__(256, 2) void build_split_persist_kernel(BuildArgs a, int ntiles, int tf1, int tf2,
                                                                     int tiles1, int tiles2) {
    __shared__ __attribute__((aligned(16))) char smem[kPLds];
    PWalk w;
    w.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    w.lane = threadIdx.x & 63;
    // XCD-contiguous runs: workgroup v runs on XCD v % 8; the tiles are cut
    // into 8 runs, one per XCD, in proportion to its workgroups, which take
    // them round-robin -- a row's tiles run at the same time on one XCD
    const int nwg = gridDim.x, v = blockIdx.x, xcd = v & 7, lw = v >> 3;
    const int gx = (nwg - xcd + 7) >> 3;
    const int before = xcd * (nwg >> 3) + min(xcd, nwg & 7);
    const int t0 = (int)((long long)ntiles * before / nwg);
    const int t1 = (int)((long long)ntiles * (before + gx) / nwg);
    const int nmine = t0 + lw < t1 ? (t1 - t0 - lw + gx - 1) / gx : 0;
    if (nmine == 0) return;                                     // workgroup-uniform
    w.nks = (a.D + 2 * kSpBK - 1) / (2 * kSpBK);
    w.totalK = nmine * w.nks;
    w.nl = a.nfused < 3 ? a.nfused : 3;
    w.tw1 = 16 * tf1;
    w.tw2 = 16 * tf2;
    w.stg = lds_u32(smem + kSpSL * kSpSlot + w.wave * kPStb);
    PTile ct = p_tile(a, t0 + lw, tf1, tf2, tiles1, tiles2, w.wave);
    PTile cn = nmine > 1 ? p_tile(a, t0 + lw + gx, tf1, tf2, tiles1, tiles2, w.wave) : ct;
    // prologue: global K steps 0 and 1
    p_issue(ct, a, smem, 0, 0, w.tw1, w.tw2, w.wave, w.lane);
    p_issue(ct, a, smem, 1, 1, w.tw1, w.tw2, w.wave, w.lane);
    if (w.totalK > 1) {
        const bool nx = w.nks == 1;
        p_issue(nx ? cn : ct, a, smem, 2, nx ? 0 : 2, w.tw1, w.tw2, w.wave, w.lane);
        p_issue(nx ? cn : ct, a, smem, 3, nx ? 1 : 3, w.tw1, w.tw2, w.wave, w.lane);
    }
    PHold hd;
    PMeta hm = {0, 0, 0, 0, 0};
    bool held = false;
    w.G0 = 0;
    for (int k = 0; k < nmine; ++k) {
        const int fa = ct.fa, fb = ct.fb;
        if (fa == 4) p_fb<4, MODE>(fb, a, smem, ct, cn, w, hd, hm, held);
        else if (fa == 3) p_fb<3, MODE>(fb, a, smem, ct, cn, w, hd, hm, held);
        else if (fa == 2) p_fb<2, MODE>(fb, a, smem, ct, cn, w, hd, hm, held);
        else if (fa == 1) p_fb<1, MODE>(fb, a, smem, ct, cn, w, hd, hm, held);
        else p_body<0, 1, MODE>(a, smem, ct, cn, w, hd, hm, held);
        w.G0 += w.nks;
        ct = cn;
        if (k + 2 < nmine) cn = p_tile(a, t0 + lw + (k + 2) * gx, tf1, tf2, tiles1, tiles2, w.wave);
    }
    // the last tile's pieces (no DMA is pending: the last K step issued none)
    if (held) {
        for (int q = 0; q < 2 * kHold; ++q) p_piece_q(a, hd, hm, q, w.nl, w.lane, w.stg);
    }
}

}  // namespace rc

static int device_cus_persist() {
    static int n = 0;
    if (!n) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
    }
    return n;
}

// The persistent kernel when it applies: fp32 levels 0-2 only (a.nfused <= 3)
// with 16-B-aligned rows, and enough tiles for two per workgroup slot;
// hipErrorNotSupported otherwise (the caller launches build_split_kernel).
// tf1/tf2/tiles are the caller's balanced tiling.
hipError_t rc_launch_build_split_persist(const rc::BuildArgs &a, long long ntiles, int tf1, int tf2, int tiles1,
                                         int tiles2, hipStream_t s) {
    if (a.nfused > 3 || a.pyr_bf16) return hipErrorNotSupported;
    for (int l = 0; l < 3 && l < a.nfused; ++l)
        if (a.lvl[l] && a.ld[l] % 4) return hipErrorNotSupported;
    const long long slots = 2LL * device_cus_persist();
    if (ntiles < 2 * slots || ntiles > 0x7FFFFFFF) return hipErrorNotSupported;
    hipLaunchKernelGGL((rc::build_split_persist_kernel<0>), dim3((unsigned)slots), dim3(256), 0, s, a, (int)ntiles,
                       tf1, tf2, tiles1, tiles2);
    return hipGetLastError();
}
#else
hipError_t rc_launch_build_split_persist(const rc::BuildArgs &, long long, int, int, int, int, hipStream_t) {
    return hipErrorNotSupported;
}
#endif  // RAFTCORR_DEV
