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

namespace rc {

// Dev-only ablation flags (RAFTCORR_BUILD_MODE): 1 = no operand loads,
// 2 = no epilogue stores.  Product launches use 0.
enum { kModeNoLoads = 1, kModeNoStores = 2, kModeStagger = 64 };

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

// VW consecutive level values -> memory (fp32, or bf16 rounded to nearest even).
template <int VW>
__device__ __forceinline__ void store_vec(void *lvl, bool bf16, long long g, const float *v) {
    if (bf16) {
        uint16_t *d = reinterpret_cast<uint16_t *>(lvl) + g;
        if constexpr (VW == 1) {
            d[0] = f32_to_bf16(v[0]);
        } else {
            unsigned w[VW / 2];
#pragma unroll
            for (int k = 0; k < VW / 2; ++k)
                w[k] = (unsigned)f32_to_bf16(v[2 * k]) | ((unsigned)f32_to_bf16(v[2 * k + 1]) << 16);
            if constexpr (VW == 8) *reinterpret_cast<uint4 *>(d) = uint4{w[0], w[1], w[2], w[3]};
            else if constexpr (VW == 4) *reinterpret_cast<uint2 *>(d) = uint2{w[0], w[1]};
            else *reinterpret_cast<unsigned *>(d) = w[0];
        }
    } else {
        float *d = reinterpret_cast<float *>(lvl) + g;
        if constexpr (VW >= 4) {
#pragma unroll
            for (int k = 0; k < VW; k += 4)
                *reinterpret_cast<f32x4 *>(d + k) = f32x4{v[k], v[k + 1], v[k + 2], v[k + 3]};
        } else if constexpr (VW == 2) {
            *reinterpret_cast<f32x2 *>(d) = f32x2{v[0], v[1]};
        } else {
            d[0] = v[0];
        }
    }
}

// Store level l of a wave tile from its LDS staging image [FM*16 rows][cw =
// 64>>l] as whole-row vector stores of VW elements per lane, 64/(cw/VW) rows
// per wave instruction.  VW divides the row stride ld and the tile column
// offset, so every vector is aligned; a vector that starts inside the row
// (col < Wl) is written whole -- its tail lands in the row's padding
// (ld >= round_up(Wl, VW) by construction).
template <int FM, int VW>
__device__ __forceinline__ void store_staged(const float *st, int l, void *lvl, long long ld,
                                             bool bf16, long long rowbase, int m0, int n0, int W1,
                                             int Wl, int lane) {
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
            store_vec<VW>(lvl, bf16, (rowbase + w1) * ld + col, v);
        }
    }
}

template <int FM>
__device__ __forceinline__ void store_staged_any(const float *st, int l, void *lvl, long long ld,
                                                 bool bf16, long long rowbase, int m0, int n0,
                                                 int W1, int Wl, int lane) {
    const int cw = 64 >> l;
    if (bf16 && ld % 8 == 0 && cw >= 8)
        store_staged<FM, 8>(st, l, lvl, ld, bf16, rowbase, m0, n0, W1, Wl, lane);
    else if (ld % 4 == 0 && cw >= 4)
        store_staged<FM, 4>(st, l, lvl, ld, bf16, rowbase, m0, n0, W1, Wl, lane);
    else if (ld % 2 == 0 && cw >= 2)
        store_staged<FM, 2>(st, l, lvl, ld, bf16, rowbase, m0, n0, W1, Wl, lane);
    else
        store_staged<FM, 1>(st, l, lvl, ld, bf16, rowbase, m0, n0, W1, Wl, lane);
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
            for (int nb = 0; nb < 4; ++nb) {
                const float v = acc[ma][nb][r];
                c[nb] = a.pow2 ? v * a.scale : v / a.sq;
                // a bf16 pyramid pools each level from the level below AS
                // STORED (bf16), like avg_pool2d on a bf16 tensor and like
                // rc_corr_pool: the pool-chain lookups can then derive a
                // level from a stored one bit for bit
                if (bf) c[nb] = round_bf16(c[nb]);
            }
            if constexpr (MODE & kModeNoStores) {
                float keep = c[0] + c[1] + c[2] + c[3];
                asm volatile("" ::"v"(keep));
                continue;
            }
            // level 0: 4 consecutive w2 per lane, 16 lanes = one 64-wide row segment
            if (w1 < W1 && wb < W2) {
                if (vec0) {
                    store_vec<4>(a.lvl[0], bf, p * ld0 + wb, c);
                } else {
#pragma unroll
                    for (int nb = 0; nb < 4; ++nb)
                        if (wb + nb < W2) store_vec<1>(a.lvl[0], bf, p * ld0 + wb + nb, &c[nb]);
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
        if (a.lvl[1]) store_staged_any<FM>(stA, 1, a.lvl[1], a.ld[1], bf, rowbase, m0, n0, W1, W2 >> 1, lane);
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
            if (a.lvl[l]) store_staged_any<FM>(dst, l, a.lvl[l], a.ld[l], bf, rowbase, m0, n0, W1, W2 >> l, lane);
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
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
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

__device__ __forceinline__ unsigned pack_bf16x2(float lo, float hi) {
    return (unsigned)f32_to_bf16(lo) | ((unsigned)f32_to_bf16(hi) << 16);
}

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

template <bool IN_BF16, bool ALIGNED>
static void launch_bf16(const BuildArgs &a, unsigned nwg, hipStream_t s) {
#ifdef RAFTCORR_DEV
    switch (dev_knob("RAFTCORR_BUILD_MODE")) {   // dev-only ablation (see rc_launch_build_f32)
        case 1: hipLaunchKernelGGL((build_bf16_kernel<IN_BF16, ALIGNED, 1>), dim3(nwg), dim3(256), 0, s, a, (int)nwg); return;
        case 2: hipLaunchKernelGGL((build_bf16_kernel<IN_BF16, ALIGNED, 2>), dim3(nwg), dim3(256), 0, s, a, (int)nwg); return;
        case 3: hipLaunchKernelGGL((build_bf16_kernel<IN_BF16, ALIGNED, 3>), dim3(nwg), dim3(256), 0, s, a, (int)nwg); return;
        default: break;
    }
#endif
    hipLaunchKernelGGL((build_bf16_kernel<IN_BF16, ALIGNED, 0>), dim3(nwg), dim3(256), 0, s, a, (int)nwg);
}

}  // namespace rc

hipError_t rc_launch_build_bf16mma(const rc::BuildArgs &a, int in_bf16, hipStream_t s) {
    const long long nwg = (long long)a.B * a.H * a.tiles_m * a.tiles_n;
    if (nwg <= 0) return hipSuccess;
    if (nwg > 0x7FFFFFFF) return hipErrorInvalidValue;
    const unsigned n = (unsigned)nwg;
    if (in_bf16) {
        if (a.W1 % 8 == 0 && a.W2 % 8 == 0) rc::launch_bf16<true, true>(a, n, s);
        else rc::launch_bf16<true, false>(a, n, s);
    } else {
        if (a.W1 % 4 == 0 && a.W2 % 4 == 0) rc::launch_bf16<false, true>(a, n, s);
        else rc::launch_bf16<false, false>(a, n, s);
    }
    return hipGetLastError();
}

// RAFTCORR_BUILD_MODE (dev library only, read per call): 0 = product (LDS-DMA
// ring kernel, 3 slots), 2 = ring without epilogue stores, 4 / 5 = 4- / 5-slot
// ring; 128+flags = the direct-load
// kernel (flags 1 no operand loads, 2 no stores, 64 stagger).
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
    switch (rc::dev_knob("RAFTCORR_BUILD_MODE")) {
        case 2: rc::launch_ring<2>(a, s); return hipGetLastError();
        case 4: rc::launch_ring<0, 4>(a, s); return hipGetLastError();         // 4-slot ring
        case 5: rc::launch_ring<0, 5>(a, s); return hipGetLastError();         // 5-slot ring
        case 128: rc::launch<true, 2, 0>(a, n, s); return hipGetLastError();   // direct-load kernel
        case 130: rc::launch<true, 2, 2>(a, n, s); return hipGetLastError();
        case 131: rc::launch<true, 2, 3>(a, n, s); return hipGetLastError();
        case 129: rc::launch<true, 2, 1>(a, n, s); return hipGetLastError();
        case 192: rc::launch<true, 2, 64>(a, n, s); return hipGetLastError();
        default: break;
    }
#endif
    rc::launch_ring<0>(a, s);
    return hipGetLastError();
}
