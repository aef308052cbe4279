// Correlation volume + fused pyramid epilogue, fp32 MFMA (gfx950).
//
// Replaces CorrBlock1D.corr (/root/reference/model.py:318-326) and the
// avg_pool2d loop of CorrBlock1D.__init__ (:284-295).
//
// Per (b,h) image row the volume is a GEMM  C[w1][w2] = sum_d F1[d][w1] F2[d][w2]
// with K = D.  F1/F2 are NCHW, so for a fixed row both operands are "K-major":
// row d of an operand is W contiguous floats.  v_mfma_f32_16x16x4_f32 takes one
// f32 per lane for A and for B: lane l supplies A[i=l&15][k=l>>4] and
// B[k=l>>4][j=l&15].  A lane loads FM (A) or 4 (B) consecutive floats along w
// (16 lanes cover one contiguous d-row segment, the wave 4 d-rows); component
// c of that vector is the operand of the c-th of FM (or 4) 16-wide fragments
// whose rows are w = w0 + FM*i + c.  The output is therefore interleaved:
// fragment (ma,nb) register r of lane l holds
//     C[m0 + FM*((l>>4)*4 + r) + ma][n0 + 4*(l&15) + nb].
// Each lane thus owns 4 consecutive w2 of a row, which makes the first two
// pooling steps lane-local and the next ones xor-shuffles (l^1, l^2, ...).
//
// Workgroup: 256 threads = 4 waves in a 2x2 arrangement of 64x64 wave tiles
// (a 128x128 tile of one row's volume).  A wave whose tile has fewer than 64
// valid w1 rows uses FM = ceil(rows/16) fragments (e.g. 3 for the 48-row tail
// of W1 = 240), so padding costs at most 15 rows of MFMA work.  Workgroups are
// remapped so all tiles of one (b,h) row run on one XCD (blocks b, b+8, ...
// share an XCD) and share that XCD's L2 copy of the row's feature maps.
//
// K loop: two named register sets (no copies, static indexing) each holding U
// k-steps; one set is loading while the other feeds the MFMAs.  K steps past D
// load zeros (buffer offset pushed out of range), so there are no per-step
// guards.
#include "common.h"
#include "epilogue.h"

namespace rc {


// First-round stagger: workgroup slot k of a CU (blockIdx / nCU) waits k
// units before starting, so the co-resident workgroups of a CU sit in
// different phases (load / MFMA / store) instead of in lockstep; later
// workgroups inherit the offset when they take a finished slot.
__device__ __forceinline__ void stagger_start(int bid, int ncu, int unit_sleeps) {
    const int slot = bid / ncu;
    if (slot >= 1 && slot <= 2) {
        const int n = slot * unit_sleeps;
        for (int i = 0; i < n; ++i) __builtin_amdgcn_s_sleep(127);  // ~8k cycles each
    }
}

constexpr int kStageFloats = 64 * 32;  // per-wave LDS staging: one 64x32 fp32 level-1 tile


// Store level l of a wave tile from its LDS staging image [FM*16 rows][cw =
// 64>>l] as whole-row vector stores of VW elements per lane, 64/(cw/VW) rows
// per wave instruction.  VW divides the row stride ld and the tile column
// offset, so every vector is aligned; a vector that starts inside the row
// (col < Wl) is written whole -- its tail lands in the row's padding
// (ld >= round_up(Wl, VW) by construction).
template <int FM, int VW>
__device__ __forceinline__ void store_staged(const float *st, int l, void *lvl, long long ld,
                                             bool bf16, long long rowbase, int m0, int n0, int W1,
                                             int Wl, int lane, long long sh) {
    const int cw = 64 >> l;
    constexpr int lvw = VW == 8 ? 3 : (VW == 4 ? 2 : (VW == 2 ? 1 : 0));
    const int llpr = 6 - l - lvw;     // log2(lanes per row)
    const int rpi = 64 >> llpr;       // rows per instruction
    const int Rl = lane >> llpr, j = (lane & ((1 << llpr) - 1)) * VW;
    const int col = (n0 >> l) + j;
    for (int r0 = 0; r0 < FM * 16; r0 += rpi) {
        const int R = r0 + Rl;
        const int w1 = m0 + R;
        if (R < FM * 16 && w1 < W1 && col < Wl) {
            float v[VW];
#pragma unroll
            for (int c = 0; c < VW; ++c) v[c] = st[R * cw + j + c];
            store_vec<VW>(lvl, bf16, (rowbase + w1) * ld + col, v, sh);
        }
    }
}

template <int FM>
__device__ __forceinline__ void store_staged_any(const float *st, int l, void *lvl, long long ld,
                                                 bool bf16, long long rowbase, int m0, int n0,
                                                 int W1, int Wl, int lane, long long sh) {
    const int cw = 64 >> l;
    if (bf16 && ld % 8 == 0 && cw >= 8)
        store_staged<FM, 8>(st, l, lvl, ld, bf16, rowbase, m0, n0, W1, Wl, lane, sh);
    else if (ld % 4 == 0 && cw >= 4)
        store_staged<FM, 4>(st, l, lvl, ld, bf16, rowbase, m0, n0, W1, Wl, lane, sh);
    else if (ld % 2 == 0 && cw >= 2)
        store_staged<FM, 2>(st, l, lvl, ld, bf16, rowbase, m0, n0, W1, Wl, lane, sh);
    else
        store_staged<FM, 1>(st, l, lvl, ld, bf16, rowbase, m0, n0, W1, Wl, lane, sh);
}

template <int N>
struct FragVec;
template <>
struct FragVec<4> { typedef f32x4 T; };
template <>
struct FragVec<3> { typedef float T __attribute__((ext_vector_type(3))); };
template <>
struct FragVec<2> { typedef f32x2 T; };
template <>
struct FragVec<1> { typedef float T __attribute__((ext_vector_type(1))); };

// Load N consecutive floats along w at (d, w) of one image, zeros when d >= D.
template <int N, bool VEC>
__device__ __forceinline__ typename FragVec<N>::T load_frag(__amdgpu_buffer_rsrc_t r, int d, int D,
                                                            int H, int h, int W, int w) {
    typedef typename FragVec<N>::T V;
    uint32_t off = (uint32_t)(((long long)(d * H + h) * W + w) * 4);
    if (d >= D) off = 0xFFFFFF00u;
    V v;
    if constexpr (VEC && N == 4) {
        v = ld4(r, off);
    } else if constexpr (VEC && N == 3) {
        v = __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b96(r, (int)off, 0, 0));
    } else if constexpr (VEC && N == 2) {
        v = __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0));
    } else {
#pragma unroll
        for (int c = 0; c < N; ++c) v[c] = ld1(r, off + 4 * c);
    }
    return v;
}

template <int FM, int U>
struct Stage {
    typename FragVec<FM>::T a[U];
    f32x4 b[U];
};

template <int FM, int U, bool VEC, int MODE>
__device__ __forceinline__ void load_stage(Stage<FM, U> &s, int k0, int kd,
                                           __amdgpu_buffer_rsrc_t r1, __amdgpu_buffer_rsrc_t r2,
                                           int D, int H, int h, int W1, int W2, int wa, int wb) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
        if constexpr (MODE & kModeNoLoads) {
#pragma unroll
            for (int c = 0; c < FM; ++c) s.a[u][c] = (float)(wa + c + u) * 1e-3f;
            s.b[u] = f32x4{(float)wb, (float)(wb + 1), (float)(k0 + u), 1.0f} * 1e-3f;
        } else {
            s.a[u] = load_frag<FM, VEC>(r1, k0 + 4 * u + kd, D, H, h, W1, wa);
            s.b[u] = load_frag<4, VEC>(r2, k0 + 4 * u + kd, D, H, h, W2, wb);
        }
    }
}

template <int FM, int U>
__device__ __forceinline__ void mma_stage(const Stage<FM, U> &s, f32x4 (&acc)[FM][4]) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
        for (int ma = 0; ma < FM; ++ma)
#pragma unroll
            for (int nb = 0; nb < 4; ++nb)
                acc[ma][nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(s.a[u][ma], s.b[u][nb],
                                                                   acc[ma][nb], 0, 0, 0);
}

// Epilogue shared by the fp32 and bf16 kernels: scale, level 0 from
// registers, pooled levels through the wave's LDS staging image.
// acc[ma][nb] register r of lane l holds C[m0 + R][n0 + 4*(l&15) + nb] with
// R = FM*((l>>4)*4 + r) + ma (interleaved rows, fp32 kernel) or
// R = 16*ma + (l>>4)*4 + r (blocked rows, bf16 kernel).
template <int FM, int MODE, bool BLOCKED>
__device__ __forceinline__ void epilogue(const f32x4 (&acc)[FM][4], const BuildArgs &a, int row,
                                         int m0, int n0, int lane, float *stA, float *stB) {
    const int W1 = a.W1, W2 = a.W2;
    const int wb = n0 + 4 * (lane & 15);            // this lane's w2 quad
    const long long rowbase = (long long)row * W1;  // pyramid row of w1 = 0
    const int col = lane & 15;
    const bool bf = a.pyr_bf16 != 0;
    const long long ld0 = a.ld[0];
    const bool vec0 = (ld0 & 3) == 0;               // quad stores stay aligned
#pragma unroll
    for (int ma = 0; ma < FM; ++ma) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int R = BLOCKED ? 16 * ma + (lane >> 4) * 4 + r
                                  : FM * ((lane >> 4) * 4 + r) + ma;  // tile row (w1 - m0)
            const int w1 = m0 + R;
            const long long p = rowbase + w1;
            float c[4];
#pragma unroll
            for (int nb = 0; nb < 4; ++nb) c[nb] = acc[ma][nb][r];
            apply_scale(c, a);
            // a bf16 pyramid pools each level from the level below AS
            // STORED (bf16), like avg_pool2d on a bf16 tensor and like
            // rc_corr_pool: the pool-chain lookups can then derive a level
            // from a stored one bit for bit
#pragma unroll
            for (int nb = 0; nb < 4; ++nb)
                if (bf) c[nb] = round_bf16(c[nb]);
            if constexpr (MODE & kModeNoStores) {
                float keep = c[0] + c[1] + c[2] + c[3];
                asm volatile("" ::"v"(keep));
                continue;
            }
            // level 0: 4 consecutive w2 per lane, 16 lanes = one 64-wide row segment
            if (w1 < W1 && wb < W2) {
                if (vec0) {
                    store_vec<4>(a.lvl[0], bf, p * ld0 + wb, c, a.shadow[0]);
                } else {
#pragma unroll
                    for (int nb = 0; nb < 4; ++nb)
                        if (wb + nb < W2) store_vec<1>(a.lvl[0], bf, p * ld0 + wb + nb, &c[nb], a.shadow[0]);
                }
            }
            if (a.nfused < 2) continue;
            // level 1 (lane-local pairs), staged in this wave's LDS image [R][32]
            f32x2 l1 = {(c[0] + c[1]) * 0.5f, (c[2] + c[3]) * 0.5f};
            if (bf) l1 = f32x2{round_bf16(l1[0]), round_bf16(l1[1])};
            *reinterpret_cast<f32x2 *>(stA + R * 32 + 2 * col) = l1;
        }
    }
    if constexpr (!(MODE & kModeNoStores)) {
        if (a.nfused < 2) return;
        // Levels >= 1 from the wave-private LDS images (in-order LDS within a
        // wave: no barrier needed).  Level l+1 = pairwise mean of level l,
        // read back from LDS in fp32: the same ops as avg_pool2d (:294)
        // (bf16 pyramid: of level l rounded to bf16, as stored).
        // a NULL level is computed (the next one needs it) but not stored
        if (a.lvl[1]) store_staged_any<FM>(stA, 1, a.lvl[1], a.ld[1], bf, rowbase, m0, n0, W1, W2 >> 1, lane, a.shadow[1]);
        float *src = stA, *dst = stB;
        for (int l = 2; l < a.nfused; ++l) {
            const int cw = 64 >> l, cwp = 2 * cw;
            const int lcw = 6 - l;
            for (int idx = lane; idx < FM * 16 * cw; idx += 64) {
                const int R = idx >> lcw, j = idx & (cw - 1);
                const f32x2 pr = *reinterpret_cast<const f32x2 *>(src + R * cwp + 2 * j);
                const float pm = (pr[0] + pr[1]) * 0.5f;
                dst[R * cw + j] = bf ? round_bf16(pm) : pm;
            }
            if (a.lvl[l]) store_staged_any<FM>(dst, l, a.lvl[l], a.ld[l], bf, rowbase, m0, n0, W1, W2 >> l, lane, a.shadow[l]);
            float *t = src;
            src = dst;
            dst = t;
        }
    }
}

template <int FM, int U, bool VEC, int MODE>
__device__ __forceinline__ void wave_tile(const BuildArgs &a, int row, int b, int h, int m0,
                                          int n0, int lane, float *stA, float *stB) {
    const int D = a.D, H = a.H, W1 = a.W1, W2 = a.W2;
    const long long img1 = (long long)D * H * W1, img2 = (long long)D * H * W2;
    const auto r1 = make_rsrc(reinterpret_cast<const float *>(a.f1) + b * img1, clamp_bytes(img1 * 4));
    const auto r2 = make_rsrc(reinterpret_cast<const float *>(a.f2) + b * img2, clamp_bytes(img2 * 4));
    const int kd = lane >> 4;             // d offset inside a k-step
    const int wa = m0 + FM * (lane & 15); // this lane's w1 group
    const int wb = n0 + 4 * (lane & 15);  // this lane's w2 quad

    f32x4 acc[FM][4];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    constexpr int KS = 4 * U;                      // d per stage
    const int nst = (D + KS - 1) / KS;             // stages (tail stages read zeros)
    Stage<FM, U> s0, s1;
    load_stage<FM, U, VEC, MODE>(s0, 0, kd, r1, r2, D, H, h, W1, W2, wa, wb);
    load_stage<FM, U, VEC, MODE>(s1, KS, kd, r1, r2, D, H, h, W1, W2, wa, wb);
    for (int st = 0; st < nst; st += 2) {
        mma_stage<FM, U>(s0, acc);
        if (st + 2 < nst) load_stage<FM, U, VEC, MODE>(s0, (st + 2) * KS, kd, r1, r2, D, H, h, W1, W2, wa, wb);
        if (st + 1 < nst) {
            mma_stage<FM, U>(s1, acc);
            if (st + 3 < nst) load_stage<FM, U, VEC, MODE>(s1, (st + 3) * KS, kd, r1, r2, D, H, h, W1, W2, wa, wb);
        }
    }

    epilogue<FM, MODE, false>(acc, a, row, m0, n0, lane, stA, stB);
}

template <bool VEC, int U, int MODE>
__global__ __launch_bounds__(256) void build_f32_kernel(BuildArgs a, int nwg_total) {
    if constexpr ((MODE & kModeStagger) != 0) stagger_start(blockIdx.x, 256, a.stagger);
    // one LDS array (guide §5 trap 4a): per wave an 8 KB + 4 KB ping-pong
    // staging image for the pooled levels
    __shared__ __attribute__((aligned(16))) float smem[4][kStageFloats + kStageFloats / 2];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float *stA = smem[wave], *stB = smem[wave] + kStageFloats;
    const int T = a.tiles_m * a.tiles_n;
    auto tile_body = [&](int v) {
        // XCD-aware bijective remap (cdna_hip_programming.md §5, "XCD swizzle").
        const int xcd = v & 7, q = nwg_total >> 3, rr = nwg_total & 7;
        const int wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (v >> 3);
        const int row = wgid / T, tile = wgid - row * T;
        const int tm = tile / a.tiles_n, tn = tile - tm * a.tiles_n;
        const int b = row / a.H, h = row - b * a.H;
        const int m0 = tm * 128 + (wave >> 1) * 64;
        const int n0 = tn * 128 + (wave & 1) * 64;
        if (m0 >= a.W1 || n0 >= a.W2) return;   // wave-uniform; no barriers in this kernel
        const int rows = a.W1 - m0;             // valid w1 rows of this wave tile
        if (rows > 48)
            wave_tile<4, U, VEC, MODE>(a, row, b, h, m0, n0, lane, stA, stB);
        else if (rows > 32)
            wave_tile<3, U, VEC, MODE>(a, row, b, h, m0, n0, lane, stA, stB);
        else if (rows > 16)
            wave_tile<2, U, VEC, MODE>(a, row, b, h, m0, n0, lane, stA, stB);
        else
            wave_tile<1, U, VEC, MODE>(a, row, b, h, m0, n0, lane, stA, stB);
    };
    tile_body(blockIdx.x);
}

// ===================== bf16 MFMA path (HBM-bound) =====================
//
// v_mfma_f32_16x16x32_bf16: lane l supplies A[i=l&15][k=8(l>>4)+j] and
// B[k=8(l>>4)+j][j'=l&15], j = 0..7 -- eight consecutive k (= d) per lane,
// while the NCHW fmaps are contiguous along w.  Each wave therefore stages
// its [32 d][64 w] operand tiles in a private LDS image (rows padded to
// 160 B: conflict-free for both the row writes and the transposed reads) and
// reads fragments with ds_read_b64_tr_b16, which hands lane i column i of a
// 4-row block.  A's image is in natural w order (fragment ma = 16 consecutive
// w1); B's columns are permuted, column 16*nb + i <- w2 = n0 + 4i + nb, so the
// accumulator layout is the fp32 kernel's (4 consecutive w2 per lane) and the
// same epilogue applies with blocked rows.  The LDS image is private to the
// wave: LDS executes a wave's instructions in order, so no barriers.
// Rows whose start is not 16-B aligned (e.g. W = 311) load two aligned chunks
// and shift in registers.

typedef short s16x4 __attribute__((ext_vector_type(4)));
constexpr int kImgRow = 160;              // bytes per LDS image row (64 bf16 + pad)
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

// One 16x16x32 operand fragment: two transposed 4-row reads (d = 8g+q and
// 8g+4+q rows of the image, this lane's 4 columns), i.e. k = 8g .. 8g+7.
__device__ __forceinline__ bf16x8 read_frag(const char *p) {
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(p));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(p + 4 * kImgRow));
    const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
}
constexpr int kImgBytes = 32 * kImgRow;   // one operand image


// 8 consecutive elements (as 4 dwords of bf16 pairs) starting at element
// index e of one image; zeros when off-range (d >= D pushes e out of range).
template <bool IN_BF16, bool ALIGNED>
__device__ __forceinline__ u32x4 load_chunk8(__amdgpu_buffer_rsrc_t r, long long e, bool valid) {
    if constexpr (IN_BF16) {
        if constexpr (ALIGNED) {
            const uint32_t off = valid ? (uint32_t)(e * 2) : 0xFFFFFF00u;
            return __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
        } else {
            const long long ea = e & ~7LL;
            const int sft = (int)(e - ea);                 // 0..7 elements
            const uint32_t off = valid ? (uint32_t)(ea * 2) : 0xFFFFFF00u;
            const u32x4 lo = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
            const u32x4 hi = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(off + 16u), 0, 0);
            const unsigned x[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            const int dsh = sft >> 1;
            u32x4 out;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                unsigned a0 = x[k], a1 = x[k + 1];
#pragma unroll
                for (int t = 1; t < 4; ++t) {
                    a0 = (dsh == t) ? x[k + t] : a0;
                    a1 = (dsh == t) ? x[k + t + 1] : a1;
                }
                out[k] = (sft & 1) ? __builtin_amdgcn_alignbyte(a1, a0, 2) : a0;
            }
            return out;
        }
    } else {
        float v[8];
        if constexpr (ALIGNED) {
            const uint32_t off = valid ? (uint32_t)(e * 4) : 0xFFFFFF00u;
            const f32x4 p0 = ld4(r, off), p1 = ld4(r, off + 16u);
#pragma unroll
            for (int c = 0; c < 4; ++c) { v[c] = p0[c]; v[4 + c] = p1[c]; }
        } else {
            const long long ea = e & ~3LL;
            const int sft = (int)(e - ea);                 // 0..3 elements
            const uint32_t off = valid ? (uint32_t)(ea * 4) : 0xFFFFFF00u;
            float x[12];
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                const f32x4 p = ld4(r, off + 16u * q);
#pragma unroll
                for (int c = 0; c < 4; ++c) x[4 * q + c] = p[c];
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                float t = x[k];
#pragma unroll
                for (int u = 1; u < 4; ++u) t = (sft == u) ? x[k + u] : t;
                v[k] = t;
            }
        }
        u32x4 out;
#pragma unroll
        for (int k = 0; k < 4; ++k) out[k] = pack_bf16x2(v[2 * k], v[2 * k + 1]);
        return out;
    }
}

template <bool IN_BF16, bool ALIGNED, int MODE>
__device__ __forceinline__ void wave_tile_bf16(const BuildArgs &a, int row, int b, int h, int m0,
                                               int n0, int lane, char *img, float *stA, float *stB) {
    const int D = a.D, H = a.H, W1 = a.W1, W2 = a.W2;
    constexpr int ES = IN_BF16 ? 2 : 4;
    const long long img1 = (long long)D * H * W1, img2 = (long long)D * H * W2;
    const auto r1 = make_rsrc(reinterpret_cast<const char *>(a.f1) + b * img1 * ES, clamp_bytes(img1 * ES));
    const auto r2 = make_rsrc(reinterpret_cast<const char *>(a.f2) + b * img2 * ES, clamp_bytes(img2 * ES));
    char *imgA = img, *imgB = img + kImgBytes;

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // staging assignment: chunk c = lane + 64t (t = 0..3) -> d-row c>>3, w chunk c&7
    u32x4 ra[4], rb[4];
    auto load_step = [&](int k0) {
        if constexpr ((MODE & kModeNoLoads) != 0) {
#pragma unroll
            for (int t = 0; t < 4; ++t) { ra[t] = u32x4{(unsigned)k0, 1u, 2u, (unsigned)lane}; rb[t] = ra[t]; }
            return;
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int c = lane + 64 * t, d = k0 + (c >> 3), m = c & 7;
            const bool ok = d < D;
            const long long base = (long long)(ok ? d : 0) * H + h;
            ra[t] = load_chunk8<IN_BF16, ALIGNED>(r1, base * W1 + m0 + 8 * m, ok);
            rb[t] = load_chunk8<IN_BF16, ALIGNED>(r2, base * W2 + n0 + 8 * m, ok);
        }
    };
    auto write_step = [&]() {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int c = lane + 64 * t, dr = c >> 3, m = c & 7;
            *reinterpret_cast<u32x4 *>(imgA + dr * kImgRow + 16 * m) = ra[t];
            // B: element e of the chunk (w2 = n0 + 8m + e) goes to column
            // 16*(e&3) + 2m + (e>>2); elements e and e+4 share one dword.
            const u32x4 u = rb[t];
            const unsigned pk[4] = {(u[0] & 0xFFFFu) | (u[2] << 16), (u[0] >> 16) | (u[2] & 0xFFFF0000u),
                                    (u[1] & 0xFFFFu) | (u[3] << 16), (u[1] >> 16) | (u[3] & 0xFFFF0000u)};
#pragma unroll
            for (int k = 0; k < 4; ++k)
                *reinterpret_cast<unsigned *>(imgB + dr * kImgRow + 32 * k + 4 * m) = pk[k];
        }
    };
    // transposed-read address of this lane inside a 4-row x 16-col block
    const int g = (lane >> 4) & 3, q = (lane >> 2) & 3, p4 = lane & 3;

    const int nk = (D + 31) >> 5;
    load_step(0);
    for (int ks = 0; ks < nk; ++ks) {
        write_step();
        if (ks + 1 < nk) load_step((ks + 1) * 32);
        bf16x8 fa[4], fb[4];
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            const int colb = (16 * f + 4 * p4) * 2;
            fa[f] = read_frag(imgA + (8 * g + q) * kImgRow + colb);
            fb[f] = read_frag(imgB + (8 * g + q) * kImgRow + colb);
        }
#pragma unroll
        for (int ma = 0; ma < 4; ++ma)
#pragma unroll
            for (int nb = 0; nb < 4; ++nb)
                acc[ma][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[ma], fb[nb], acc[ma][nb], 0, 0, 0);
    }
    epilogue<4, MODE, true>(acc, a, row, m0, n0, lane, stA, stB);
}

template <bool IN_BF16, bool ALIGNED, int MODE>
__global__ __launch_bounds__(256) void build_bf16_kernel(BuildArgs a, int nwg_total) {
    // per wave: 2 operand images (10 KB) during the K loop, then the 12 KB
    // epilogue staging area (aliases them: the loop is over by then)
    __shared__ __attribute__((aligned(16))) float smem[4][kStageFloats + kStageFloats / 2];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float *stA = smem[wave], *stB = smem[wave] + kStageFloats;
    char *img = reinterpret_cast<char *>(smem[wave]);
    const int T = a.tiles_m * a.tiles_n;
    const int v = blockIdx.x;
    const int xcd = v & 7, q = nwg_total >> 3, rr = nwg_total & 7;
    const int wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (v >> 3);
    const int row = wgid / T, tile = wgid - row * T;
    const int tm = tile / a.tiles_n, tn = tile - tm * a.tiles_n;
    const int b = row / a.H, h = row - b * a.H;
    const int m0 = tm * 128 + (wave >> 1) * 64;
    const int n0 = tn * 128 + (wave & 1) * 64;
    if (m0 >= a.W1 || n0 >= a.W2) return;   // wave-uniform; no barriers in this kernel
    wave_tile_bf16<IN_BF16, ALIGNED, MODE>(a, row, b, h, m0, n0, lane, img, stA, stB);
}

// ====== bf16 fmaps: persistent workgroups, shared LDS-DMA ring ======
//
// The per-wave staging above loads every operand tile twice per workgroup
// (two waves share each A and each B tile) and re-reads each fmap row once
// per 128-wide tile on the other side: at W = 311 that is ~7x the unique
// fmap bytes through L1 per row, plus two loads and a shift per unaligned
// chunk (1.80 ms at config 3, B = 64).  This kernel instead:
//   * covers up to 320 w2 in one tile (2 x NWN compute waves, wave tile 64
//     w1 x 16*FMA w2, FMA = 4 or 5 fragments), so per image row F2 is read
//     ceil(W1/128) times and F1 once;
//   * stages [32 d][cols] bf16 tiles of F1 and F2, shared by all waves, in an
//     SL-slot ring filled by buffer->LDS DMA from two loader waves (no VGPR
//     staging).  Each lane's 16-B source is 8 consecutive w of one d-row at
//     any 2-B alignment, so rows that do not start on a 16-B boundary
//     (W = 311) need no shifting;
//   * is persistent: one workgroup per CU walks its tiles and the ring runs on
//     across tile boundaries;
//   * swaps the MFMA operands (A = F2: M = w2, B = F1: N = w1) so each lane's
//     accumulator registers hold 4 CONSECUTIVE w2 of one w1: pyramid levels
//     1-2 are lane-local poolings, 3-4 xor-16 / xor-32 lane exchanges -- all
//     in registers, in the order avg_pool2d uses (model.py:294);
//   * for the bf16 pair layout (levels 0 and 2 stored) defers the epilogue:
//     a finished tile's level 0 is held in registers as packed bf16 and
//     stored 16 rows at a time during the next tile's K loop, overlapping
//     the ring's loads; other layouts write every level (at most 5 fused;
//     more are pooled by rc_launch_pool) in 16-row pieces through a
//     wave-private fp32 image right after the tile.
// LDS image rows are 256-B multiples, with 16-B chunk j of row r stored at
// chunk j ^ 2*sigma(r), sigma(r) = (r & 3) | ((r >> 3) & 1) << 2: the eight
// rows one half-wave's ds_read_b64_tr_b16 touches land on eight different
// 32-B bank groups (conflict-free).  The DMA writes LDS lane-linearly, so
// the swizzle is applied to each lane's SOURCE chunk; pad chunks get an
// out-of-range (no-op) offset.
constexpr int kB16BK = 32;                  // d rows per stage
constexpr int kB16P1 = 256;                 // F1 image pitch: 128 w1
constexpr int kB16MaxFused = 5;             // levels the ring epilogue writes
constexpr int kB16DeferStage = 16 * 144;    // deferred epilogue: per-wave bf16 image of 16 rows
// RC_LAYOUT_RECORDS: 16 rows of one wave row's levels 0 and 2 (every w2 of
// the tile, which spans the whole row) staged in a workgroup-shared bf16
// image -- element e of row i at byte 2 (pad + e) of the row's level-0 /
// level-2 part, zeros outside [0, W) -- as two halves of 8 rows, one being
// written while the wave row gathers the other's records.  Sized for
// W2 <= 320 (RC_REC_COUNT(W2) <= 22: level-0 elements up to 347, level-2 up
// to 95).
constexpr int kRecL0Pad = 28, kRecL2Pad = 14;                 // element -pad at byte 0
constexpr int kRecL0P = 752, kRecL2P = 224;                   // bytes per image row
constexpr int kRecImg = 16 * (kRecL0P + kRecL2P);             // one wave row's piece image
constexpr int kRecMaxW2 = 320;
static_assert(2 * (kRecL0Pad + rec_e0(21) + kRecSlots - kRecL2Slots) <= kRecL0P &&
                  2 * (kRecL2Pad + rec_e2(21) + kRecL2Slots) <= kRecL2P && kRecL0Pad >= -rec_e0(0) + 2 &&
                  kRecL2Pad == -rec_e2(0),
              "records image geometry");

// RC_LAYOUT_RECORDS: the records of unit u (the 8 pixel rows em0 + 8u ..,
// image half u & 1 of a wave row's piece image `img`) of the tile held at
// image row erow, gathered and stored by NL lanes (ll: this lane among them;
// NL a multiple of 8).  Chunk c = ll & 7 of each record holds slots 8c..8c+7:
// level 2 (slots < 26) for c < 3, level 0 for c > 3, and for c = 3 slots
// 24-25 of level 2 then 26-31 of level 0.  Each lane reads dword 0 at A and
// dwords 1-3 at B, B + 4 (8-B aligned): A, B one part's consecutive bytes
// for c != 3, the two parts for c = 3 -- three LDS reads per chunk, the same
// for every lane.  The unit's records are one contiguous run of 8 * rec_nr
// lines (16 B per lane, 128 B per 8 lanes, written whole).
typedef unsigned rec_u32x4 __attribute__((ext_vector_type(4)));

template <int MODE, int NL>
__device__ __forceinline__ void rec_emit_unit(const BuildArgs &a, const char *img, int u, int erow, int em0, int ll) {
    const int c = ll & 7;
    const int NR = a.rec_nr, W1 = a.W1;
    const int w1u = em0 + 8 * u;                                  // the unit's first pixel row
    const int J = min(8, W1 - w1u) * NR;                          // records of the unit
    // kModeL2Stores (dev timing only, wrong output): 8 L2-resident rows
    const long long rrow = (MODE & kModeL2Stores) ? (erow & 7) : erow;
    char *base = static_cast<char *>(a.rec) + (rrow * W1 + w1u) * NR * 128 + 16 * c;
    const int hb = 8 * (u & 1);                                   // the unit's first image row
    const int a2 = 16 * kRecL0P + hb * kRecL2P + 2 * (kRecL2Pad + rec_e2(0));         // level-2 slot 0
    const int a0 = hb * kRecL0P + 2 * (kRecL0Pad + rec_e0(0) - kRecL2Slots);          // level-0 "slot 0"
    const bool cl2 = c < 3, cmix = c == 3;
    const int A0 = (cl2 || cmix ? a2 : a0) + 16 * c, PA = cl2 || cmix ? kRecL2P : kRecL0P;
    const int mA = cl2 || cmix ? 8 : 32;
    const int B0 = (cl2 ? a2 : a0) + 16 * c + 4, PB = cl2 ? kRecL2P : kRecL0P, mB = cl2 ? 8 : 32;
    // record t = (row, r): t advances by S = NL / 8 per step, (row, r) by
    // (drow, dr) with a carry -- no division in the loop
    constexpr int S = NL >> 3;
    const int drow = S / NR, dr = S - drow * NR;
    int t = ll >> 3;
    int row = t / NR, r = t - row * NR;
    constexpr int BT = 2;                                         // records' reads in flight per wait (3: VGPR spills)
    for (; t < J; t += BT * S) {
        uint32_t v[BT][4];
#pragma unroll
        for (int b = 0; b < BT; ++b) {
            if (t + b * S < J) {
                const char *pa = img + A0 + row * PA + r * mA;
                const char *pb = img + B0 + row * PB + r * mB;
                v[b][0] = *reinterpret_cast<const uint32_t *>(pa);
                v[b][1] = *reinterpret_cast<const uint32_t *>(pb);
                const uint2 w = *reinterpret_cast<const uint2 *>(pb + 4);
                v[b][2] = w.x;
                v[b][3] = w.y;
            }
            r += dr;
            row += drow;
            if (r >= NR) { r -= NR; ++row; }
        }
#pragma unroll
        for (int b = 0; b < BT; ++b) {
            if (t + b * S < J) {
                if constexpr ((MODE & kModeRecNoStore) != 0)       // dev timing: gathered, not stored
                    asm volatile("" ::"v"(v[b][0]), "v"(v[b][1]), "v"(v[b][2]), "v"(v[b][3]));
                else if constexpr ((MODE & kModeRecNT) != 0)       // dev A/B: streaming (non-temporal) stores
                    __builtin_nontemporal_store(rec_u32x4{v[b][0], v[b][1], v[b][2], v[b][3]},
                                                reinterpret_cast<rec_u32x4 *>(base + (long long)(t + b * S) * 128));
                else
                    *reinterpret_cast<uint4 *>(base + (long long)(t + b * S) * 128) =
                        uint4{v[b][0], v[b][1], v[b][2], v[b][3]};
            }
        }
    }
}

template <int NWN, int FMA>
struct B16Geom {
    static constexpr int NW = 2 * NWN;                              // waves
    static constexpr int WT = 16 * FMA;                             // wave tile w2 width
    static constexpr int TW = WT * NWN;                             // workgroup tile w2 width
    static constexpr int P2 = (2 * TW + 255) / 256 * 256;           // F2 image pitch (B)
    static constexpr int C2 = P2 / 16, C1 = kB16P1 / 16;            // 16-B chunks per row
    static constexpr int SLOT = kB16BK * (P2 + kB16P1);             // bytes per ring slot
    static constexpr int NINS2 = kB16BK * C2 / 64;                  // F2 DMA instructions per stage
    static constexpr int NINS = NINS2 + kB16BK * C1 / 64;           // all
    static constexpr int IPW = (NINS + NW - 1) / NW;                // per wave (max)
    static constexpr int STP = WT + 4;                              // level-0 staging pitch (floats)
    static constexpr int STB = 16 * STP * 4;                        // staging bytes per wave
    static_assert((kB16BK * C2) % 64 == 0 && (kB16BK * C1) % 64 == 0, "whole DMA pieces");
    static_assert(C2 % 16 == 0, "swizzle groups");
};

__device__ __forceinline__ int b16_swz(int r) { return 2 * ((r & 3) | (((r >> 3) & 1) << 2)); }

// ds_read_b64_tr_b16 as inline asm.  The compiler puts an s_waitcnt
// vmcnt(0) (every LDS DMA in flight, the ring's prefetch included) in front
// of any LDS access it sees while LDS DMA is pending; these reads are
// ordered by the ring's own waits and barriers instead, and their results by
// an lgkmcnt wait that names them.
template <int OFF>
__device__ __forceinline__ s16x4 tr_read_asm(uint32_t lds_addr) {
    s16x4 v;
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(lds_addr), "i"(OFF));
    return v;
}

// Pitch-parametrised fragment read (see read_frag): rows 8g+q and 8g+4+q.
__device__ __forceinline__ bf16x8 read_frag_p(const char *p, int pitch) {
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(p));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(p + 4 * pitch));
    const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
}


// s_waitcnt vmcnt(m) lgkmcnt(0) with m = n rounded down to a multiple of 4,
// capped at 60 (waiting for more than asked is always safe); the immediate
// is chosen by a 4-deep branch tree on the wave-uniform n.
template <int LO, int HI>
__device__ __forceinline__ void wait_vm_tree(int m) {
    if constexpr (LO == HI) {
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"(LO) : "memory");
    } else {
        constexpr int MID = (LO + HI) / 8 * 4;   // last multiple of 4 in the lower half
        if (m <= MID) wait_vm_tree<LO, MID>(m);
        else wait_vm_tree<MID + 4, HI>(m);
    }
}
__device__ __forceinline__ void wait_vm_lgkm0(int n) {
    const int m = n >= 60 ? 60 : (n < 0 ? 0 : n & ~3);
    wait_vm_tree<0, 60>(m);
}



// One tile of the persistent walk: its image row and workgroup origin.
struct B16Tile {
    int row, b, h, M0, N0;
};

// 2*NWN compute waves + 2 loader waves.  Only the loader waves issue the
// ring's DMA, and only the compute waves store: vmcnt on gfx950 counts
// loads and stores together, and a load may complete after a later store,
// so a wave that had stored could wait for its DMA only by waiting for its
// stores too.  Each stage: loaders wait for their DMA of stage gs ->
// barrier -> loaders refill the slot stage gs-1 used; compute waves read
// stage gs's fragments and run its MFMAs (and a tile's epilogue after its
// last stage) -- their lgkmcnt(0) before the next barrier releases the slot.
template <int NWN, int FMA, int SL, int MODE, int NLM, bool DEFER>
__global__ __launch_bounds__(128 * NWN + 128) void build_bf16_ring_kernel(BuildArgs a, int ntiles, int tiles_m,
                                                                           int tiles_n) {
    typedef B16Geom<NWN, FMA> G;
    constexpr int NC = G::NW;                                     // compute waves
    constexpr int LIPW = G::NINS / 2;                             // DMA instructions per loader wave per stage
    static_assert(G::NINS % 2 == 0 && LIPW * (SL - 1) + 2 <= 60, "loader vmcnt budget");
    static_assert(!DEFER || FMA == 4, "deferred epilogue: 4 fragments per wave");
    constexpr bool REC = (MODE & kModeRecords) != 0;              // RC_LAYOUT_RECORDS
    static_assert(!REC || DEFER, "records: the deferred epilogue");
    constexpr bool LEMIT = REC && (MODE & kModeRecLoaderEmit) != 0;   // dev: the loader waves emit
    __shared__ __attribute__((aligned(16)))
    char smem[SL * G::SLOT + (REC ? 2 * kRecImg : NC * (DEFER ? kB16DeferStage : G::STB))];
    typedef __attribute__((address_space(3))) void lds_void;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int D = a.D, H = a.H, W1 = a.W1, W2 = a.W2;
    const int T = tiles_m * tiles_n;

    // Persistent walk, XCD-aware: workgroup v runs on XCD v % 8; the tiles
    // are cut into 8 contiguous runs, one per XCD, in proportion to its
    // workgroups, which take them round-robin -- so the tiles of one image
    // row run at the same time on one XCD and share its L2 copy of the row.
    const int nwg = gridDim.x, v = blockIdx.x;
    const int xcd = v & 7, lw = v >> 3;
    const int gx = (nwg - xcd + 7) >> 3;                          // workgroups on this XCD
    const int before = xcd * (nwg >> 3) + min(xcd, nwg & 7);      // workgroups on lower XCDs
    const int t0 = (int)((long long)ntiles * before / nwg);
    const int t1 = (int)((long long)ntiles * (before + gx) / nwg);
    auto tile_at = [&](int k) {                                   // k-th tile of this workgroup
        B16Tile t;
        const int id = t0 + lw + k * gx;
        t.row = id / T;
        const int tl = id - t.row * T, tm = tl / tiles_n, tn = tl - tm * tiles_n;
        t.b = t.row / H;
        t.h = t.row - t.b * H;
        t.M0 = tm * 128;
        t.N0 = tn * G::TW;
        return t;
    };
    const int ntile_mine = t0 + lw < t1 ? (t1 - t0 - lw + gx - 1) / gx : 0;
    if (ntile_mine == 0) return;                                  // workgroup-uniform
    const long long img1 = (long long)D * H * W1, img2 = (long long)D * H * W2;
    const int nst = (D + kB16BK - 1) / kB16BK;                    // >= 2 (launcher)
    const int total = ntile_mine * nst;

    if (wave >= NC) {
        // ------------------------------ loader ------------------------------
        const int lid = wave - NC;                                // its instructions: ins = lid + 2k
        const uint32_t sstep2 = (uint32_t)((long long)kB16BK * H * W2 * 2);
        const uint32_t sstep1 = (uint32_t)((long long)kB16BK * H * W1 * 2);
        // per lane and instruction: d row, logical (unswizzled) source chunk,
        // tile-independent source offset
        int dr[LIPW], dj[LIPW];
        uint32_t dbase[LIPW];
#pragma unroll
        for (int k = 0; k < LIPW; ++k) {
            const int ins = lid + 2 * k;
            const bool f2 = ins < G::NINS2;
            const int c = f2 ? 64 * ins + lane : 64 * (ins - G::NINS2) + lane;
            const int rd = f2 ? c / G::C2 : c / G::C1;
            const int j = (c - rd * (f2 ? G::C2 : G::C1)) ^ b16_swz(rd);
            dr[k] = rd;
            dj[k] = f2 && 8 * j >= G::TW ? 1 << 20 : j;           // F2 pad chunks never load
            dbase[k] = (uint32_t)((rd * H * (f2 ? W2 : W1) + 8 * j) * 2);
        }
        __amdgpu_buffer_rsrc_t ir1 = make_rsrc(a.f1, 0), ir2 = make_rsrc(a.f2, 0);
        // stage-0 source offsets; kOOB (past any image: num_records < 2^31,
        // and adding the stage steps keeps it there) = nothing to load
        constexpr uint32_t kOOB = 0x80000000u;
        uint32_t tb[LIPW];
        B16Tile it;
        auto set_issue_tile = [&](const B16Tile &t) {
            it = t;
            ir1 = make_rsrc(reinterpret_cast<const char *>(a.f1) + t.b * img1 * 2, clamp_bytes(img1 * 2));
            ir2 = make_rsrc(reinterpret_cast<const char *>(a.f2) + t.b * img2 * 2, clamp_bytes(img2 * 2));
            const uint32_t o2 = (uint32_t)((t.h * W2 + t.N0) * 2), o1 = (uint32_t)((t.h * W1 + t.M0) * 2);
#pragma unroll
            for (int k = 0; k < LIPW; ++k) {
                constexpr int K2 = G::NINS2 / 2;                    // k < K2: an F2 instruction (NINS2 even)
                const bool ok = k < K2 ? t.N0 + 8 * dj[k] < W2 : t.M0 + 8 * dj[k] < W1;
                tb[k] = ok ? dbase[k] + (k < K2 ? o2 : o1) : kOOB;
            }
        };
        // A 16-B DMA source that is only 2-B aligned is range-checked per 4-B
        // piece counted from its start, so the piece holding the LAST element
        // of an image (d = D-1, h = H-1, w = W-1) and the element after it
        // reads as zero.  The lane that DMAs that chunk loads the element (in
        // range) just before the stage's DMA and writes it into LDS once the
        // stage has landed: (LDS offset << 16 | value), ~0 = none.
        uint32_t pp[2] = {0xFFFFFFFFu, 0xFFFFFFFFu};
        int pp_gs = -1;
        int vmq = 0, q[SL], nq = 0;                                // loads issued; vmq after each pending stage
        auto issue = [&](int gs, int st) {
            char *slot = smem + (gs % SL) * G::SLOT;
            if (st == nst - 1 && it.h == H - 1) {
                const int rd = (D - 1) % kB16BK;
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    const bool f2 = t == 0;
                    const int Wt = f2 ? W2 : W1, org = f2 ? it.N0 : it.M0, span = f2 ? G::TW : 128;
                    if (Wt - 1 < org || Wt - 1 >= org + span) continue;
                    const int j = (Wt - 1 - org) >> 3, p = j ^ b16_swz(rd);
                    const int c = f2 ? rd * G::C2 + p : G::NINS2 * 64 + rd * G::C1 + p;
                    if ((c >> 6) % 2 != lid) continue;              // wave-uniform
                    if ((c & 63) == lane) {
                        const unsigned short val = __builtin_amdgcn_raw_buffer_load_b16(
                            f2 ? ir2 : ir1, (int)((((long long)(D - 1) * H + it.h) * Wt + Wt - 1) * 2), 0, 0);
                        pp[t] = ((uint32_t)(16 * c + 2 * ((Wt - 1 - org) & 7)) << 16) | val;
                    }
                    ++vmq;
                    pp_gs = gs;
                }
            }
            const int dlim = D - kB16BK * st;                      // rows d >= D read zeros
            const uint32_t s2 = (uint32_t)st * sstep2, s1 = (uint32_t)st * sstep1;
#pragma unroll
            for (int k = 0; k < LIPW; ++k) {
                constexpr int K2 = G::NINS2 / 2;
                uint32_t o = tb[k] + (k < K2 ? s2 : s1);
                if (dlim < kB16BK && dr[k] >= dlim) o = kOOB;      // only a last stage with D % 32 != 0
                if constexpr ((MODE & kModeAlignedSrc) != 0) o &= ~15u;   // dev timing only: wrong data
                if constexpr ((MODE & kModeNoLoads) == 0)
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(k < K2 ? ir2 : ir1,
                                                             (lds_void *)(slot + 1024 * (lid + 2 * k)), 16, (int)o,
                                                             0, 0, 0);
            }
            if constexpr ((MODE & kModeNoLoads) == 0) vmq += LIPW;
#pragma unroll
            for (int x = 0; x < SL; ++x)
                if (x == nq) q[x] = vmq;
            ++nq;
        };
        int issued = 0, it_k = 0, it_st = 0;
        auto issue_next = [&]() {
            if (issued >= total) return;
            issue(issued, it_st);
            ++issued;
            if (++it_st == nst) {
                it_st = 0;
                if (++it_k < ntile_mine) set_issue_tile(tile_at(it_k));
            }
        };
        set_issue_tile(tile_at(0));
#pragma unroll
        for (int s = 0; s < SL - 1; ++s) issue_next();
        for (int gs = 0; gs < total; ++gs) {
            // stage gs landed: every load issued up to its DMA is done
            // (loads complete in order)
            wait_vm_lgkm0(vmq - q[0]);
#pragma unroll
            for (int x = 0; x + 1 < SL; ++x) q[x] = q[x + 1];
            --nq;
            if (gs == pp_gs) {
                char *slotp = smem + (gs % SL) * G::SLOT;
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    if (pp[t] != 0xFFFFFFFFu)
                        *reinterpret_cast<unsigned short *>(slotp + (pp[t] >> 16)) = (unsigned short)pp[t];
                    pp[t] = 0xFFFFFFFFu;
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            }
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            issue_next();
            if constexpr (LEMIT) {
                // dev: this loader wave emits its wave row's units -- unit
                // st - 1 of the tile before (stage st = 1..8), or unit 7 of
                // the tile two back at stage 0 of 8-stage tiles
                const int k = gs / nst, st = gs - k * nst;
                int ek = -1, eu = 0;
                if (st >= 1 && st <= 8 && k >= 1) { ek = k - 1; eu = st - 1; }
                else if (st == 0 && nst == 8 && k >= 2) { ek = k - 2; eu = 7; }
                if (ek >= 0) {
                    const B16Tile et = tile_at(ek);
                    if (et.M0 + 64 * lid < W1)
                        rec_emit_unit<MODE, 64>(a, smem + SL * G::SLOT + lid * kRecImg, eu, et.row,
                                                et.M0 + 64 * lid, lane);
                }
            }
        }
        if constexpr (REC) {   // the compute waves' last-tile records (rec_write / rec_emit)
#pragma unroll
            for (int u = 0; u <= 8; ++u) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                asm volatile("" ::: "memory");
                if constexpr (LEMIT) {
                    int ek = -1, eu = 0;
                    if (u == 0 && nst == 8 && ntile_mine >= 2) { ek = ntile_mine - 2; eu = 7; }
                    else if (u >= 1) { ek = ntile_mine - 1; eu = u - 1; }
                    if (ek >= 0) {
                        const B16Tile et = tile_at(ek);
                        if (et.M0 + 64 * lid < W1)
                            rec_emit_unit<MODE, 64>(a, smem + SL * G::SLOT + lid * kRecImg, eu, et.row,
                                                    et.M0 + 64 * lid, lane);
                    }
                }
            }
        }
        return;
    }

    // ------------------------------ compute ------------------------------
    // transposed-read addresses of this lane inside a slot (row 8g+q, 4 cols
    // of fragment f, swizzled); the k = 8g+4.. rows are +4 rows (same swizzle)
    const int gq = (lane >> 4) & 3, qq = (lane >> 2) & 3, p4 = lane & 3;
    const int rr = 8 * gq + qq, sw = b16_swz(rr);
    const int wm = wave & 1, wn = wave >> 1;
    const uint32_t a_row = rr * G::P2 + 8 * (p4 & 1), b_row = kB16BK * G::P2 + rr * kB16P1 + 8 * (p4 & 1);
    const int a_ch = (G::WT / 8) * wn + (p4 >> 1), b_ch = 8 * wm + (p4 >> 1);
    const uint32_t stg = lds_u32(smem + SL * G::SLOT + wave * G::STB);
    f32x4 acc[FMA][4];
    // DEFER (bf16 pair layout: levels 0 and 2): a finished tile's levels are
    // held in registers as packed bf16 and stored one piece (16 rows) every
    // nst/4 stages during the next tile's K loop, so the stores overlap the
    // ring's loads instead of stalling the workgroup between tiles.  Level 2
    // is stored when the tile ends, after a lane transpose that gives lane
    // (g, i) the 4 level-2 values of fragment ma = g.
    uint32_t h0[FMA][4][2];
    uint32_t h2[REC ? 4 : 1][2];                                  // REC: level 2 (bf16 pairs of ma)
    int hrow = 0, hm0 = 0, hn0 = 0;
    // per-lane row offsets of the deferred stores (elements): level-0 piece
    // rows (lane >> 3) and 8 + (lane >> 3), level-2 row (lane & 15)
    const int loff0 = (lane >> 3) * (int)a.ld[0], loff1 = loff0 + 8 * (int)a.ld[0];
    const int l2off = (lane & 15) * (int)a.ld[2];
    bool hact = false, held = false;
    const int g = lane >> 4, i16 = lane & 15;
    auto hold = [&](int row, int m0h, int n0h, bool act) {
        hrow = row; hm0 = m0h; hn0 = n0h; hact = act; held = true;
        if (!act) return;
        float s2[FMA][4];
        // the scale as one wave-uniform branch around the whole block (a
        // select per element would run the division sequence every time);
        // each pair is rounded once: the packed bf16 is the level-0 value and
        // its halves, widened, the pooling inputs (RNE is idempotent, so this
        // equals rounding, widening and packing again)
        auto level0 = [&](auto scale_fn) {
#pragma unroll
            for (int ma = 0; ma < FMA; ++ma)
#pragma unroll
                for (int nb = 0; nb < 4; ++nb) {
                    const f32x4 x = acc[ma][nb];
                    const uint32_t p0 = pack_bf16x2(scale_fn(x[0]), scale_fn(x[1]));
                    const uint32_t p1 = pack_bf16x2(scale_fn(x[2]), scale_fn(x[3]));
                    h0[ma][nb][0] = p0;
                    h0[ma][nb][1] = p1;
                    if constexpr ((MODE & kModeNoStores) != 0)   // dev timing: keep the MFMAs alive
                        asm volatile("" ::"v"(p0), "v"(p1));
                    const float v0 = __builtin_bit_cast(float, p0 << 16), v1 = __builtin_bit_cast(float, p0 & 0xFFFF0000u);
                    const float v2 = __builtin_bit_cast(float, p1 << 16), v3 = __builtin_bit_cast(float, p1 & 0xFFFF0000u);
                    s2[ma][nb] = pool2(pool2(v0, v1, true), pool2(v2, v3, true), true);
                }
        };
        if (a.pow2) {
            const float sc = a.scale;
            level0([sc](float x) { return x * sc; });
        } else {
            const float sq = a.sq;
            level0([sq](float x) { return x / sq; });
        }
        if constexpr (REC) {
            // level 2 stays in registers too, transposed like the row
            // layout's stores below: lane (g, i) holds columns n0/4 + 4g ..
            // + 3 of row 16 nb + i (one 8-B image write per unit), zero past
            // the level's width (the records' padding)
#pragma unroll
            for (int nb = 0; nb < 4; ++nb) {
                uint32_t R0 = __builtin_bit_cast(uint32_t, s2[0][nb]), R1 = __builtin_bit_cast(uint32_t, s2[1][nb]);
                uint32_t R2 = __builtin_bit_cast(uint32_t, s2[2][nb]), R3 = __builtin_bit_cast(uint32_t, s2[3][nb]);
                auto t02 = __builtin_amdgcn_permlane32_swap(R0, R2, false, false);
                auto t13 = __builtin_amdgcn_permlane32_swap(R1, R3, false, false);
                auto t01 = __builtin_amdgcn_permlane16_swap(t02[0], t13[0], false, false);
                auto t23 = __builtin_amdgcn_permlane16_swap(t02[1], t13[1], false, false);
                const uint32_t qu[4] = {(uint32_t)t01[0], (uint32_t)t01[1], (uint32_t)t23[0], (uint32_t)t23[1]};
                float q[4];
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    q[j] = (n0h >> 2) + 4 * g + j < (W2 >> 2) ? __builtin_bit_cast(float, qu[j]) : 0.0f;
                h2[nb][0] = pack_bf16x2(q[0], q[1]);
                h2[nb][1] = pack_bf16x2(q[2], q[3]);
            }
            return;
        }
        // (hold runs for DEFER kernels only, which have FMA == 4)
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) {
            // lane group g gets fragment g's level-2 value of every group j
            // (a 4 x 4 transpose of 16-lane rows x fragments): two 32-lane
            // swaps, then two 16-lane swaps -- afterwards register j of
            // group g holds what group j had in register g
            uint32_t R0 = __builtin_bit_cast(uint32_t, s2[0][nb]), R1 = __builtin_bit_cast(uint32_t, s2[1][nb]);
            uint32_t R2 = __builtin_bit_cast(uint32_t, s2[2][nb]), R3 = __builtin_bit_cast(uint32_t, s2[3][nb]);
            auto t02 = __builtin_amdgcn_permlane32_swap(R0, R2, false, false);
            auto t13 = __builtin_amdgcn_permlane32_swap(R1, R3, false, false);
            auto t01 = __builtin_amdgcn_permlane16_swap(t02[0], t13[0], false, false);
            auto t23 = __builtin_amdgcn_permlane16_swap(t02[1], t13[1], false, false);
            const float qv[4] = {__builtin_bit_cast(float, (uint32_t)t01[0]), __builtin_bit_cast(float, (uint32_t)t01[1]),
                                 __builtin_bit_cast(float, (uint32_t)t23[0]), __builtin_bit_cast(float, (uint32_t)t23[1])};
            // level 2 is small (8 B per lane and column): stored right away
            const int w1 = m0h + 16 * nb + i16, col = (n0h >> 2) + 4 * g;
            if (!(MODE & kModeNoStores) && w1 < W1 && col < (W2 >> 2)) {
                const long long r2 = (long long)((MODE & kModeL2Stores) ? (row & 7) : row) * W1 + m0h + 16 * nb;
                uint16_t *d = reinterpret_cast<uint16_t *>(a.lvl[2]) + r2 * a.ld[2] + l2off + col;
                const uint2 x = uint2{pack_bf16x2(qv[0], qv[1]), pack_bf16x2(qv[2], qv[3])};
                *reinterpret_cast<uint2 *>(d) = x;
                if (a.shadow[2]) *reinterpret_cast<uint2 *>(reinterpret_cast<char *>(d) + a.shadow[2]) = x;
            }
        }
    };
    // piece nb = level-0 rows 16nb..16nb+15 of the held tile: staged as bf16
    // in this wave's LDS image (16 rows x 128 B, pitch 144 B) and stored as
    // whole 128-B row segments, 16 B per lane -- 8-B stores straight from
    // the registers would write each line in four pieces at different times
    // (measured 1.5x the HBM write bytes)
    // halves [h0b, h1b) of piece nb: half 0 also stages the piece in LDS
    auto store_piece = [&](int nb, int h0b = 0, int h1b = 2) {
        if (!hact) return;
        // opaque per piece, so that the addresses of all pieces are not
        // precomputed per tile and kept live through the K loop
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const int g = ln >> 4, i16 = ln & 15;
        char *img = smem + SL * G::SLOT + wave * kB16DeferStage;
        if (h0b == 0) {
#pragma unroll
            for (int ma = 0; ma < FMA; ++ma)
                *reinterpret_cast<uint2 *>(img + i16 * 144 + (16 * ma + 4 * g) * 2) =
                    uint2{h0[ma][nb][0], h0[ma][nb][1]};
        }
        uint16_t *l0 = reinterpret_cast<uint16_t *>(a.lvl[0]);
        // kModeL2Stores (dev timing only, wrong output): 8 L2-resident rows
        const long long rowbase = (long long)((MODE & kModeL2Stores) ? (hrow & 7) : hrow) * W1;
        // the piece's first row (wave-uniform, scalar math) + this lane's
        // row offset (precomputed): no vector multiplies per store
        uint16_t *t0 = l0 + (rowbase + hm0 + 16 * nb) * a.ld[0] + hn0;
        for (int half = h0b; half < h1b; ++half) {
            const int R = 8 * half + (ln >> 3), c = ln & 7;
            const uint4 x = *reinterpret_cast<const uint4 *>(img + R * 144 + 16 * c);
            const int w1 = hm0 + 16 * nb + R, col = hn0 + 8 * c;
            if (w1 < W1 && col < W2) {
                uint16_t *d = t0 + (half ? loff1 : loff0) + 8 * c;
                *reinterpret_cast<uint4 *>(d) = x;
                if (a.shadow[0]) *reinterpret_cast<uint4 *>(reinterpret_cast<char *>(d) + a.shadow[0]) = x;
            }
        }
    };
    // REC: the held tile's rows go out in 8 units of 8 rows (unit u = rows
    // 8u..8u+7 of this wave row, in half u & 1 of the wave row's shared
    // 16-row image), one unit per stage of the next tile's K loop, each in two
    // steps a barrier apart:
    // rec_write(u) -- at stage u each wave puts its 64 level-0 and 16 level-2
    //   columns of the unit's rows in;
    // rec_emit(u) -- at stage u + 1 the wave row's NWN waves gather the rows'
    //   records from it, one 16-B chunk per lane, 128 B per 8 lanes: the
    //   unit's records are one contiguous run of 8 * rec_nr lines, written
    //   whole.
    // Stage s then emits unit s - 1 from one half while unit s goes into the
    // other, so every stage carries half a piece of stores (the same stores
    // in bursts of a whole piece every other stage: +0.35 ms at config 3).
    // Unit 7 is emitted at stage 8, or at the next tile's stage 0 (pending)
    // when the tile has exactly 8 stages.
    char *const rimg = smem + SL * G::SLOT + wm * kRecImg;
    auto rec_write = [&](int u) {
        if (!hact) return;
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const int g = ln >> 4, i16 = ln & 15;
        if ((i16 >> 3) != (u & 1)) return;                        // this lane's row is in the other half
        const int p = u >> 1;
        char *r0 = rimg + i16 * kRecL0P, *r2 = rimg + 16 * kRecL0P + i16 * kRecL2P;
#pragma unroll
        for (int ma = 0; ma < FMA; ++ma) {
            const int wb = hn0 + 16 * ma + 4 * g;                 // tiles_n == 1: hn0 is the w2 column
            uint32_t p0 = h0[ma][p][0], p1 = h0[ma][p][1];
            const int nv = W2 - wb;                               // valid columns of the four
            if (nv < 4) {
                p1 = nv <= 2 ? 0u : (p1 & 0xFFFFu);
                p0 = nv <= 0 ? 0u : (nv == 1 ? (p0 & 0xFFFFu) : p0);
            }
            *reinterpret_cast<uint2 *>(r0 + 2 * (kRecL0Pad + wb)) = uint2{p0, p1};
        }
        // level-2 columns n0/4 + 4g .. + 3 (4-B aligned: two dwords)
        uint32_t *d2 = reinterpret_cast<uint32_t *>(r2 + 2 * (kRecL2Pad + (hn0 >> 2) + 4 * g));
        d2[0] = h2[p][0];
        d2[1] = h2[p][1];
    };
    // unit u of the tile held at (erow, em0): its image half -> its records
    auto rec_emit = [&](int u, int erow, int em0, bool eact) {
        if (!eact) return;
        int ll = wn * 64 + lane;
        asm volatile("" : "+v"(ll));                              // recomputed per unit (see store_piece)
        rec_emit_unit<MODE, 64 * NWN>(a, rimg, u, erow, em0, ll);
    };
    // the unit 7 that waits for the next tile's stage 0 (8-stage tiles)
    bool pend = false;
    int prow = 0, pm0 = 0;
    if constexpr (REC) {
        // zeros around the rows (element -pad.. and past W): never overwritten
        for (int o = 16 * (int)(threadIdx.x); o < 2 * kRecImg; o += 16 * 64 * NC)
            *reinterpret_cast<uint4 *>(smem + SL * G::SLOT + o) = uint4{0u, 0u, 0u, 0u};
    }
    auto zero_acc = [&]() {
#pragma unroll
        for (int x = 0; x < FMA; ++x)
#pragma unroll
            for (int y = 0; y < 4; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};
    };
    int k = 0, st = 0;
    B16Tile cur = tile_at(0);
    int m0 = cur.M0 + 64 * wm, n0 = cur.N0 + G::WT * wn;         // this wave's w1 / w2 origin
    bool active = m0 < W1 && n0 < W2;                             // wave-uniform
    zero_acc();
    for (int gs = 0; gs < total; ++gs) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (active && !(MODE & kModeNoMath)) {
            // compiler-visible LDS reads are fine here: no LDS DMA is ever
            // pending on the compute waves' path, so no vmcnt wait is added,
            // and the compiler pairs each fragment's two reads in one tuple
            const char *slot = smem + (gs % SL) * G::SLOT;
            bf16x8 fa[FMA], fb[4];
            if constexpr ((MODE & kModeNoFragReads) != 0) {    // dev timing only: MFMAs on stale registers
#pragma unroll
                for (int f = 0; f < FMA; ++f) { fa[f] = bf16x8{}; asm volatile("" : "+v"(fa[f])); }
#pragma unroll
                for (int f = 0; f < 4; ++f) { fb[f] = bf16x8{}; asm volatile("" : "+v"(fb[f])); }
            } else {
#pragma unroll
                for (int f = 0; f < FMA; ++f) fa[f] = read_frag_p(slot + a_row + 16 * ((a_ch + 2 * f) ^ sw), G::P2);
#pragma unroll
                for (int f = 0; f < 4; ++f) fb[f] = read_frag_p(slot + b_row + 16 * ((b_ch + 2 * f) ^ sw), kB16P1);
            }
#pragma unroll
            for (int ma = 0; ma < FMA; ++ma)
#pragma unroll
                for (int nb = 0; nb < 4; ++nb)
                    acc[ma][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[ma], fb[nb], acc[ma][nb], 0, 0, 0);
        }
        if constexpr (REC && !(MODE & (kModeNoStores | kModeRecNoEmit | kModeRecLoaderEmit))) {
            if (pend && st == 0) {   // unit 7 of the tile held before the current one
                rec_emit(7, prow, pm0, true);
                pend = false;
            }
        }
        if constexpr (DEFER && !(MODE & kModeNoStores)) {
            if (held) {
                if constexpr (REC) {   // unit u: image at stage u, records at u + 1 (nst >= 8: launcher)
#pragma unroll
                    for (int u = 0; u <= 8; ++u) {
                        if (st == u) {
                            if constexpr (!(MODE & (kModeRecNoEmit | kModeRecLoaderEmit))) {
                                if (u >= 1) rec_emit(u - 1, hrow, hm0, hact);
                            }
                            if (u < 8) rec_write(u);
                        }
                    }
                } else if constexpr ((MODE & kModeSpread) != 0) {   // 8 half-pieces, one per stage at nst = 8
#pragma unroll
                    for (int p = 0; p < 8; ++p)
                        if (((p * nst) >> 3) == st) store_piece(p >> 1, p & 1, (p & 1) + 1);
                } else if constexpr ((MODE & kModeStagger) != 0) {   // odd waves one stage later
                    const int off = nst >= 8 ? (wave & 1) : 0;
#pragma unroll
                    for (int nb = 0; nb < 4; ++nb)
                        if (((nb * nst) >> 2) + off == st) store_piece(nb);
                } else {
#pragma unroll
                    for (int nb = 0; nb < 4; ++nb)
                        if (((nb * nst) >> 2) == st) store_piece(nb);
                }
            }
        }
        if (++st == nst) {
            if constexpr (REC) {   // 8-stage tiles: the held tile's unit 7 goes out at the next stage 0
                if (held && nst == 8 && hact) {
                    pend = true;
                    prow = hrow;
                    pm0 = hm0;
                }
            }
            if constexpr (DEFER) hold(cur.row, m0, n0, active);
            else if (active) epilogue_swapped<FMA, MODE, NLM>(acc, a, cur.row, m0, n0, lane, stg);
            st = 0;
            if (++k < ntile_mine) {
                cur = tile_at(k);
                m0 = cur.M0 + 64 * wm;
                n0 = cur.N0 + G::WT * wn;
                active = m0 < W1 && n0 < W2;
                zero_acc();
            }
        }
    }
    if constexpr (REC) {
        // the last tile (held: ntile_mine >= 1): 9 barriers, matched by the
        // loader waves' 9 before they end.  Barrier u orders stage u - 1's
        // image writes before unit u - 1's gather and unit u - 2's gather
        // before unit u's writes into the same half.
#pragma unroll
        for (int u = 0; u <= 8; ++u) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            if constexpr (!(MODE & (kModeRecNoEmit | kModeNoStores | kModeRecLoaderEmit))) {
                if (u == 0 && pend) rec_emit(7, prow, pm0, true);
                if (u >= 1) rec_emit(u - 1, hrow, hm0, hact);
            }
            if constexpr (!(MODE & kModeNoStores)) {
                if (u < 8) rec_write(u);
            }
        }
    } else if constexpr (DEFER && !(MODE & kModeNoStores)) {
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) store_piece(nb);
    }
}

// (waves along w2, fragments per wave, deferred epilogue) for the ring
// kernel: the fewest padded w2 columns per row, ties to the wider tile;
// nwn = 0: use the per-wave kernel.  The deferred (register-held) epilogue
// serves the bf16 pair layout (levels 0 and 2 stored, level 1 not) with
// 8-B-aligned rows; it uses 64-wide wave tiles, up to 5 along w2.
struct B16Shape { int nwn, fma; bool defer; };
static B16Shape bf16_ring_shape(const BuildArgs &a) {
    if (a.W2 <= 64 || (a.D + kB16BK - 1) / kB16BK < 2) return {0, 0, false};
    // 32-bit source offsets with an out-of-range marker at 2^31
    if ((long long)a.D * a.H * (a.W1 > a.W2 ? a.W1 : a.W2) * 2 >= (1LL << 30)) return {0, 0, false};
    if (a.nfused > kB16MaxFused)              // levels past the ring's are pooled from memory
        for (int l = kB16MaxFused - 1; l < a.nfused; ++l)
            if (!a.lvl[l]) return {0, 0, false};
    const bool defer = a.pyr_bf16 && a.nfused == 3 && a.lvl[0] && !a.lvl[1] && a.lvl[2] && a.ld[0] % 8 == 0 &&
                       a.ld[2] % 4 == 0;
    static const B16Shape cand[] = {{4, 5, false}, {4, 4, false}, {3, 5, false}, {3, 4, false}, {2, 5, false},
                                    {2, 4, false}};
    static const B16Shape cand_defer[] = {{5, 4, true}, {4, 4, true}, {3, 4, true}, {2, 4, true}};
    B16Shape best = {0, 0, false};
    long long bestpad = 0;
    auto consider = [&](const B16Shape &c) {
        const long long w = 16LL * c.fma * c.nwn, pad = (a.W2 + w - 1) / w * w;
        if (!best.nwn || pad < bestpad) { best = c; bestpad = pad; }
    };
    if (defer)
        for (const B16Shape &c : cand_defer) consider(c);
    else
        for (const B16Shape &c : cand) consider(c);
    return best;
}

static int device_cus() {
    static int n = 0;
    if (!n) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
    }
    return n;
}

template <int NWN, int FMA, int SL, int MODE, bool DEFER>
static void launch_bf16_ring_n(const BuildArgs &a, hipStream_t s, int per_cu = 1) {
    constexpr int TW = B16Geom<NWN, FMA>::TW;
    const int tiles_m = (a.W1 + 127) / 128, tiles_n = (a.W2 + TW - 1) / TW;
    const long long ntiles = (long long)a.B * a.H * tiles_m * tiles_n;
    if (ntiles <= 0 || ntiles > 0x7FFFFFFF) return;
    const long long cap = (long long)device_cus() * per_cu;                 // resident workgroups (LDS-bound)
    const long long nwg = ntiles < cap ? ntiles : cap;
    // up to 3 fused levels (the default pair layout) keeps the epilogue's
    // level pointers out of the scalar registers the K loop needs
    if (DEFER || a.nfused <= 3)
        hipLaunchKernelGGL((build_bf16_ring_kernel<NWN, FMA, SL, MODE, 3, DEFER>), dim3((unsigned)nwg),
                           dim3(128 * NWN + 128), 0, s, a, (int)ntiles, tiles_m, tiles_n);
    else
        hipLaunchKernelGGL((build_bf16_ring_kernel<NWN, FMA, SL, MODE, kB16MaxFused, DEFER>), dim3((unsigned)nwg),
                           dim3(128 * NWN + 128), 0, s, a, (int)ntiles, tiles_m, tiles_n);
}


// the deferred-epilogue kernel has no staging area: 4 ring slots
template <int MODE>
static void launch_bf16_ring(const BuildArgs &a, B16Shape sh, hipStream_t s) {
    if (sh.defer) {
        if (sh.nwn == 5) launch_bf16_ring_n<5, 4, 4, MODE, true>(a, s);
        else if (sh.nwn == 4) launch_bf16_ring_n<4, 4, 4, MODE, true>(a, s);
        else if (sh.nwn == 3) launch_bf16_ring_n<3, 4, 4, MODE, true>(a, s);
        else launch_bf16_ring_n<2, 4, 4, MODE, true>(a, s);
    } else if (sh.nwn == 4 && sh.fma == 5) launch_bf16_ring_n<4, 5, 3, MODE, false>(a, s);
    else if (sh.nwn == 4) launch_bf16_ring_n<4, 4, 3, MODE, false>(a, s);
    else if (sh.nwn == 3 && sh.fma == 5) launch_bf16_ring_n<3, 5, 3, MODE, false>(a, s);
    else if (sh.nwn == 3) launch_bf16_ring_n<3, 4, 3, MODE, false>(a, s);
    else if (sh.fma == 5) launch_bf16_ring_n<2, 5, 3, MODE, false>(a, s);
    else launch_bf16_ring_n<2, 4, 3, MODE, false>(a, s);
}

// ============ fp32 MFMA with a workgroup LDS-DMA ring (default) ============
//
// Operand tiles are shared by the workgroup's four waves through a 3-slot LDS
// ring filled by buffer->LDS DMA (buffer_load_dwordx4 ... lds): slot = a
// [16 d][128 w] tile of F1 and of F2 (16 KB), two stages in flight ahead of
// the one being multiplied, no VGPR staging.  Stage s+2 is issued into the
// slot stage s-1 used, after the barrier that follows every wave's counted
// vmcnt for stage s (RAW) and its lgkmcnt(0) for the reads of stage s-1
// (WAR) -- cdna_hip_programming.md §5 "Pipelining across barriers".
// Fragments are read with ds_read_b128 (conflict-free: the 16-lane groups of
// a b128 read cover all 64 banks of two 512-B rows).  Waves with no valid
// rows still issue their share of the DMA and join every barrier.
constexpr int kRingSlots = 3;
constexpr int kBK = 16;                       // d rows per ring stage
constexpr int kSlotFloats = 2 * kBK * 128;    // A + B tiles of one stage
static_assert(kRingSlots * kSlotFloats >= 4 * (kStageFloats + kStageFloats / 2),
              "epilogue staging must fit in the ring");

template <int FM, int FN>
__device__ __forceinline__ void ring_stage(const float *sA, const float *sB, int am, int bn,
                                           int lane, f32x4 (&acc)[FM][4]) {
#pragma unroll
    for (int kk = 0; kk < kBK / 4; ++kk) {
        const int dr = 4 * kk + (lane >> 4);
        const float *pa = sA + dr * 128 + am + FM * (lane & 15);
        float av[4], bv[4];
        if constexpr (FM == 4) {
            const f32x4 v = *reinterpret_cast<const f32x4 *>(pa);
            av[0] = v[0]; av[1] = v[1]; av[2] = v[2]; av[3] = v[3];
        } else if constexpr (FM == 2) {
            const f32x2 v = *reinterpret_cast<const f32x2 *>(pa);
            av[0] = v[0]; av[1] = v[1];
        } else {
#pragma unroll
            for (int c = 0; c < FM; ++c) av[c] = pa[c];
        }
        const float *pb = sB + dr * 128 + bn + FN * (lane & 15);
        if constexpr (FN == 4) {
            const f32x4 v = *reinterpret_cast<const f32x4 *>(pb);
            bv[0] = v[0]; bv[1] = v[1]; bv[2] = v[2]; bv[3] = v[3];
        } else {
#pragma unroll
            for (int c = 0; c < FN; ++c) bv[c] = pb[c];
        }
#pragma unroll
        for (int ma = 0; ma < FM; ++ma)
#pragma unroll
            for (int nb = 0; nb < FN; ++nb)
                acc[ma][nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[ma], bv[nb], acc[ma][nb], 0, 0, 0);
    }
}

struct RingCtx {
    __amdgpu_buffer_rsrc_t r1, r2;
    int D, H, h, W1, W2, M0, N0, wave, lane, nst;
};

// DMA share of this wave per stage: rows 4w..4w+3 of both tiles, 2 rows
// (1 KB = 64 lanes x 16 B) per instruction -> 4 instructions per stage.
template <int SL>
__device__ __forceinline__ void ring_issue(const RingCtx &c, float *smem, int st) {
    typedef __attribute__((address_space(3))) void lds_void;
    float *sA = smem + (st % SL) * kSlotFloats, *sB = sA + kBK * 128;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int r0 = 4 * c.wave + 2 * i;
        const int d = st * kBK + r0 + (c.lane >> 5);
        const int w = 4 * (c.lane & 31);
        const long long base = (long long)(d < c.D ? d : 0) * c.H + c.h;
        const uint32_t offA = d < c.D ? (uint32_t)((base * c.W1 + c.M0 + w) * 4) : 0xFFFFFF00u;
        const uint32_t offB = d < c.D ? (uint32_t)((base * c.W2 + c.N0 + w) * 4) : 0xFFFFFF00u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(c.r1, (lds_void *)(sA + r0 * 128), 16, (int)offA, 0, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(c.r2, (lds_void *)(sB + r0 * 128), 16, (int)offB, 0, 0, 0);
    }
}

// The whole K loop + epilogue for one wave with FM A-fragments and FN
// B-fragments (FM = 0: a wave with no valid rows -- it still issues its DMA
// share and joins every barrier, so all four waves execute the same barrier
// sequence).
template <int FM, int FN, int MODE, int SL>
__device__ __forceinline__ void ring_body(const RingCtx &c, const BuildArgs &a, float *smem, int row,
                                          int am, int bn) {
    f32x4 acc[FM > 0 ? FM : 1][4];
#pragma unroll
    for (int i = 0; i < (FM > 0 ? FM : 1); ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < SL - 1; ++s)
        if (s < c.nst) ring_issue<SL>(c, smem, s);
    for (int st = 0; st < c.nst; ++st) {
        // RAW: my DMA for stage st landed (the later stages' 4 instructions
        // each may stay in flight); WAR: my LDS reads of stage st-1 are done.
        // Then the barrier.
        const int later = min(SL - 2, c.nst - 1 - st);
        if (later >= 3) asm volatile("s_waitcnt vmcnt(12) lgkmcnt(0)" ::: "memory");
        else if (later == 2) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
        else if (later == 1) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (st + SL - 1 < c.nst) ring_issue<SL>(c, smem, st + SL - 1);
        if constexpr (FM > 0) {
            const float *sA = smem + (st % SL) * kSlotFloats, *sB = sA + kBK * 128;
            ring_stage<FM, FN>(sA, sB, am, bn, c.lane, acc);
        }
    }
    // everyone is done with the ring before it becomes epilogue staging
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if constexpr (FM > 0) {
        float *stA = smem + c.wave * (kStageFloats + kStageFloats / 2), *stB = stA + kStageFloats;
        epilogue<FM, MODE, false>(acc, a, row, c.M0 + am, c.N0 + bn, c.lane, stA, stB);
    }
}

// FN = 4 B-fragments: 64-wide wave tiles, WG 128x128.  (48-wide tiles with
// FN = 3, which avoid padding at W = 240/720, measured slower: 414 vs 372 us
// at config 2 -- more workgroups re-read A and the B DMA/FLOP grows.)
template <int FN, int MODE, int SL = kRingSlots>
__global__ __launch_bounds__(256) void build_f32_ring_kernel(BuildArgs a, int nwg_total) {
    static_assert(SL >= 3 && SL <= 5, "ring depth");
    __shared__ __attribute__((aligned(16))) float smem[SL * kSlotFloats];
    RingCtx c;
    c.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    c.lane = threadIdx.x & 63;
    const int T = a.tiles_m * a.tiles_n;
    const int v = blockIdx.x;
    const int xcd = v & 7, q = nwg_total >> 3, rr = nwg_total & 7;
    const int wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (v >> 3);
    const int row = wgid / T, tile = wgid - row * T;
    const int tm = tile / a.tiles_n, tn = tile - tm * a.tiles_n;
    const int b = row / a.H;
    c.h = row - b * a.H;
    c.D = a.D; c.H = a.H; c.W1 = a.W1; c.W2 = a.W2;
    c.M0 = tm * 128; c.N0 = tn * 32 * FN;
    c.nst = (a.D + kBK - 1) / kBK;
    const long long img1 = (long long)a.D * a.H * a.W1, img2 = (long long)a.D * a.H * a.W2;
    c.r1 = make_rsrc(reinterpret_cast<const float *>(a.f1) + b * img1, clamp_bytes(img1 * 4));
    c.r2 = make_rsrc(reinterpret_cast<const float *>(a.f2) + b * img2, clamp_bytes(img2 * 4));
    const int am = (c.wave >> 1) * 64, bn = (c.wave & 1) * 16 * FN;   // wave tile in the WG tile
    const int m0 = c.M0 + am, n0 = c.N0 + bn;
    const int rows = a.W1 - m0;
    const bool active = rows > 0 && n0 < a.W2;                         // wave-uniform
    if (!active) ring_body<0, FN, MODE, SL>(c, a, smem, row, am, bn);
    else if (rows > 48) ring_body<4, FN, MODE, SL>(c, a, smem, row, am, bn);
    else if (rows > 32) ring_body<3, FN, MODE, SL>(c, a, smem, row, am, bn);
    else if (rows > 16) ring_body<2, FN, MODE, SL>(c, a, smem, row, am, bn);
    else ring_body<1, FN, MODE, SL>(c, a, smem, row, am, bn);
}

template <bool VEC, int U, int MODE>
static void launch(const BuildArgs &a, unsigned nwg, hipStream_t s) {
    hipLaunchKernelGGL((build_f32_kernel<VEC, U, MODE>), dim3(nwg), dim3(256), 0, s, a, (int)nwg);
}

template <int MODE, int SL = kRingSlots>
static void launch_ring(const BuildArgs &a, hipStream_t s) {
    const long long nwg = (long long)a.B * a.H * a.tiles_m * a.tiles_n;
    if (nwg <= 0 || nwg > 0x7FFFFFFF) return;
    hipLaunchKernelGGL((build_f32_ring_kernel<4, MODE, SL>), dim3((unsigned)nwg), dim3(256), 0, s, a, (int)nwg);
}

#ifdef RAFTCORR_DEV
#include "dev/volume_dev.inc"   // ablation modes and measured variants: libraftcorr_dev.so only
#endif

template <bool IN_BF16, bool ALIGNED>
static void launch_bf16(const BuildArgs &a, unsigned nwg, hipStream_t s) {
#ifdef RAFTCORR_DEV
    if (dev_launch_bf16_pw<IN_BF16, ALIGNED>(a, nwg, s)) return;
#endif
    hipLaunchKernelGGL((build_bf16_kernel<IN_BF16, ALIGNED, 0>), dim3(nwg), dim3(256), 0, s, a, (int)nwg);
}

}  // namespace rc

// bf16 MFMA build.  The ring kernel fuses at most kB16MaxFused levels:
// a.nfused is lowered to what was written, and the caller pools the rest.
hipError_t rc_launch_build_bf16mma(rc::BuildArgs &a, int in_bf16, hipStream_t s) {
    const long long nwg = (long long)a.B * a.H * a.tiles_m * a.tiles_n;
    if (nwg <= 0) return hipSuccess;
    if (nwg > 0x7FFFFFFF) return hipErrorInvalidValue;
    const unsigned n = (unsigned)nwg;
    if (a.rec) {
        // RC_LAYOUT_RECORDS: the deferred ring kernel with one tile across
        // the whole row (NWN = ceil(W2 / 64) waves along w2) and at least
        // 8 stages per tile (its four pieces take two stages each)
        const int nwn = (a.W2 + 63) / 64;
        if (!in_bf16 || !a.pyr_bf16 || nwn < 2 || a.W2 > rc::kRecMaxW2 || (a.D + rc::kB16BK - 1) / rc::kB16BK < 8 ||
            (long long)a.D * a.H * (a.W1 > a.W2 ? a.W1 : a.W2) * 2 >= (1LL << 30))
            return hipErrorNotSupported;
        constexpr int RM = rc::kModeRecords;
#ifdef RAFTCORR_DEV
        if (const hipError_t e = rc::dev_launch_records(a, nwn, s); e != hipErrorNotSupported) return e;
#endif
        if (nwn == 5) rc::launch_bf16_ring_n<5, 4, 4, RM, true>(a, s);
        else if (nwn == 4) rc::launch_bf16_ring_n<4, 4, 4, RM, true>(a, s);
        else if (nwn == 3) rc::launch_bf16_ring_n<3, 4, 4, RM, true>(a, s);
        else rc::launch_bf16_ring_n<2, 4, 4, RM, true>(a, s);
        return hipGetLastError();
    }
    rc::B16Shape sh = in_bf16 ? rc::bf16_ring_shape(a) : rc::B16Shape{0, 0, false};
#ifdef RAFTCORR_DEV
    if (const hipError_t e = rc::dev_launch_bf16mma(a, sh, s); e != hipErrorNotSupported) return e;
#endif
    if (sh.nwn) {
        if (a.nfused > rc::kB16MaxFused) a.nfused = rc::kB16MaxFused;
        rc::launch_bf16_ring<0>(a, sh, s);
        return hipGetLastError();
    }
    if (in_bf16) {
        if (a.W1 % 8 == 0 && a.W2 % 8 == 0) rc::launch_bf16<true, true>(a, n, s);
        else rc::launch_bf16<true, false>(a, n, s);
    } else {
        if (a.W1 % 4 == 0 && a.W2 % 4 == 0) rc::launch_bf16<false, true>(a, n, s);
        else rc::launch_bf16<false, false>(a, n, s);
    }
    return hipGetLastError();
}

// The exact fp32 MFMA build (LDS-DMA ring kernel, 3 slots).
hipError_t rc_launch_build_f32(const rc::BuildArgs &a, hipStream_t s) {
    const long long nwg = (long long)a.B * a.H * a.tiles_m * a.tiles_n;
    if (nwg <= 0) return hipSuccess;
    if (nwg > 0x7FFFFFFF) return hipErrorInvalidValue;
    const bool vec = (a.W1 % 4 == 0) && (a.W2 % 4 == 0);
    const unsigned n = (unsigned)nwg;
    if (!vec) {
        rc::launch<false, 2, 0>(a, n, s);
        return hipGetLastError();
    }
#ifdef RAFTCORR_DEV
    if (const hipError_t e = rc::dev_launch_f32(a, n, s); e != hipErrorNotSupported) return e;
#endif
    rc::launch_ring<0>(a, s);
    return hipGetLastError();
}
