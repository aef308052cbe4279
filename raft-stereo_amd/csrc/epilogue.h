// Epilogue helpers shared by the volume kernels (volume.hip,
// volume_split.hip): scaled level values -> pyramid memory, including the
// swapped-operand epilogue that pools levels 1-2 lane-locally and stages
// each level through a wave-private LDS image for whole-row stores.
#pragma once
#include "common.h"

namespace rc {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// Dev-only ablation flags (RAFTCORR_BUILD_MODE): 1 = no operand loads,
// 2 = no epilogue stores.  Product launches use 0.
enum { kModeNoLoads = 1, kModeNoStores = 2, kModeNoMath = 4, kModeAlignedSrc = 8, kModeNoFragReads = 16,
       kModeStagger = 64, kModeNoMfma = 512, kModeNoSplit = 1024, kModeSpread = 2048, kModeSheared = 4096,
       kModePackedSub = 8192,
       kModeL2Stores = 65536, kModeDirect = 131072, kModeFastEpi = 262144, kModeGenericEpi = 524288,
       kModePairEpi = 1048576, kModeRecords = 1 << 23, kModeRecNoStore = 1 << 24, kModeRecNoEmit = 1 << 25,
       kModeRecLoaderEmit = 1 << 26, kModeRecNT = 1 << 27,
       kModePhasePrio = 1 << 28, kModeMfmaPrio = 1 << 29 };

// VW consecutive level values -> memory (fp32, or bf16 rounded to nearest even).
template <int VW>
__device__ __forceinline__ void store_vec1(void *lvl, bool bf16, long long g, const float *v) {
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

// ... and to the level's line-phase shadow copy at +sh bytes when sh != 0
// (RC_SHADOW: the same values, every store duplicated; sh is wave-uniform).
template <int VW>
__device__ __forceinline__ void store_vec(void *lvl, bool bf16, long long g, const float *v, long long sh) {
    store_vec1<VW>(lvl, bf16, g, v);
    if (sh) store_vec1<VW>(static_cast<char *>(lvl) + sh, bf16, g, v);
}

__device__ __forceinline__ unsigned pack_bf16x2(float lo, float hi) {
    return (unsigned)f32_to_bf16(lo) | ((unsigned)f32_to_bf16(hi) << 16);
}

__device__ __forceinline__ uint32_t lds_u32(const void *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char *)(p);
}

// The epilogue's wave-private staging accesses are inline asm too (see
// tr_read_asm): in-order LDS execution within a wave orders them, and a
// read's result is used only after the lgkmcnt(0) wait inside its asm.
__device__ __forceinline__ void lds_st4(uint32_t a, f32x4 v) {
    asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(v));
}
__device__ __forceinline__ void lds_st2(uint32_t a, f32x2 v) {
    asm volatile("ds_write_b64 %0, %1" ::"v"(a), "v"(v));
}
__device__ __forceinline__ void lds_st1(uint32_t a, float v) {
    asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(v));
}

// Rows [0, 16) of a wave's staged level image (fp32 at LDS address st,
// pitch p floats, cw columns) -> level memory, VW elements per lane, cw / VW
// lanes per row.
template <int VW>
__device__ __forceinline__ void store_rows16(uint32_t st, int p, int cw, void *lvl, long long ld,
                                             bool bf16, long long rowbase, int w1_0, int col0, int W1,
                                             int Wl, int lane, long long sh) {
    const int lpr = cw / VW;                 // lanes per row
    const int rpi = 64 / lpr;                // rows per instruction
    const int Rl = lane / lpr, j = (lane - Rl * lpr) * VW;
    const int col = col0 + j;
    for (int r0 = 0; r0 < 16; r0 += rpi) {
        const int R = r0 + Rl, w1 = w1_0 + R;
        const uint32_t src = st + 4 * (R * p + j);
        float v[VW];
        if constexpr (VW == 8) {
            f32x4 x0, x1;
            asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:16\n\ts_waitcnt lgkmcnt(0)"
                         : "=&v"(x0), "=&v"(x1) : "v"(src));
#pragma unroll
            for (int c = 0; c < 4; ++c) { v[c] = x0[c]; v[4 + c] = x1[c]; }
        } else if constexpr (VW == 4) {
            f32x4 x0;
            asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(x0) : "v"(src));
#pragma unroll
            for (int c = 0; c < 4; ++c) v[c] = x0[c];
        } else if constexpr (VW == 2) {
            f32x2 x0;
            asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(x0) : "v"(src));
            v[0] = x0[0]; v[1] = x0[1];
        } else {
            float x0;
            asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(x0) : "v"(src));
            v[0] = x0;
        }
        const bool ok = Rl < rpi && R < 16 && w1 < W1 && col < Wl;
        if (ok) store_vec<VW>(lvl, bf16, (rowbase + w1) * ld + col, v, sh);
    }
}

__device__ __forceinline__ void store_rows16_any(uint32_t st, int p, int cw, void *lvl, long long ld,
                                                 bool bf16, long long rowbase, int w1_0, int col0,
                                                 int W1, int Wl, int lane, long long sh) {
    // widest vector dividing the image width, the first column (so every
    // vector is naturally aligned) and the row stride
    if (bf16 && ld % 8 == 0 && cw % 8 == 0 && col0 % 8 == 0)
        store_rows16<8>(st, p, cw, lvl, ld, bf16, rowbase, w1_0, col0, W1, Wl, lane, sh);
    else if (ld % 4 == 0 && cw % 4 == 0 && col0 % 4 == 0)
        store_rows16<4>(st, p, cw, lvl, ld, bf16, rowbase, w1_0, col0, W1, Wl, lane, sh);
    else if (ld % 2 == 0 && cw % 2 == 0 && col0 % 2 == 0)
        store_rows16<2>(st, p, cw, lvl, ld, bf16, rowbase, w1_0, col0, W1, Wl, lane, sh);
    else
        store_rows16<1>(st, p, cw, lvl, ld, bf16, rowbase, w1_0, col0, W1, Wl, lane, sh);
}

__device__ __forceinline__ float pool2(float x, float y, bool bf) {
    const float m = (x + y) * 0.5f;
    return bf ? round_bf16(m) : m;
}

// Rows [0, 16) of a wave's staged fp32 image of level L (CW columns, a
// multiple of VW, pitch CW + 4 floats) -> level memory as VW-float vectors,
// with the geometry known at compile time: every LDS read of the flush
// issued before one wait, then the stores (store_rows16's loop waits once per
// row group and divides by runtime widths).
template <int VW> struct FlushVec;
template <> struct FlushVec<4> { typedef f32x4 T; };
template <> struct FlushVec<2> { typedef f32x2 T; };
template <> struct FlushVec<1> { typedef float T; };

template <int CW, int L, int VW>
__device__ __forceinline__ void flush_rows16_fast(uint32_t st, const BuildArgs &a, long long rowbase, int w1_0,
                                                  int n0, int w1e, int lane) {
    static_assert(CW % VW == 0, "whole vectors per row");
    typedef typename FlushVec<VW>::T V;
    constexpr int LP = CW / VW;                // lanes per row
    constexpr int RPI = 64 / LP;               // rows per instruction
    constexpr int NI = (16 + RPI - 1) / RPI;   // instructions
    const int Rl = lane / LP, j = (lane - Rl * LP) * VW;
    const int col = (n0 >> L) + j;
    const bool lok = Rl < RPI && col < (a.W2 >> L);
    V x[NI];
#pragma unroll
    for (int k = 0; k < NI; ++k) {
        const int R = k * RPI + Rl;
        const uint32_t src = st + 4 * ((R < 16 ? R : 15) * (CW + 4) + j);
        if constexpr (VW == 4) asm volatile("ds_read_b128 %0, %1" : "=v"(x[k]) : "v"(src));
        else if constexpr (VW == 2) asm volatile("ds_read_b64 %0, %1" : "=v"(x[k]) : "v"(src));
        else asm volatile("ds_read_b32 %0, %1" : "=v"(x[k]) : "v"(src));
    }
    // one wait, then the read registers pass through an asm each that
    // follows it (volatile asms keep their order), so no use of them moves
    // above the wait
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < NI; ++k) asm volatile("" : "+v"(x[k]));
#pragma unroll
    for (int k = 0; k < NI; ++k) {
        const int R = k * RPI + Rl, w1 = w1_0 + R;
        if (lok && R < 16 && w1 < w1e) {
            float v[VW];
            if constexpr (VW == 1) v[0] = x[k];
            else {
#pragma unroll
                for (int c = 0; c < VW; ++c) v[c] = x[k][c];
            }
            store_vec<VW>(a.lvl[L], false, (rowbase + w1) * a.ld[L] + col, v, a.shadow[L]);
        }
    }
}

// The same flush split in two, so that several images' reads share one
// wait: flush_issue (LDS reads of rows [0, 16) of a staged image) and
// flush_store (their stores), with flush_settle between them.
template <int CW, int L>
struct FlushRegs {
    static constexpr int LP = CW / 4, RPI = 64 / LP, NI = (16 + RPI - 1) / RPI;
    f32x4 x[NI];
};
template <int CW, int L>
__device__ __forceinline__ void flush_issue(FlushRegs<CW, L> &f, uint32_t st, int lane) {
    typedef FlushRegs<CW, L> F;
    const int Rl = lane / F::LP, j = (lane - Rl * F::LP) * 4;
#pragma unroll
    for (int k = 0; k < F::NI; ++k) {
        const int R = k * F::RPI + Rl;
        const uint32_t src = st + 4 * ((R < 16 ? R : 15) * (CW + 4) + j);
        asm volatile("ds_read_b128 %0, %1" : "=v"(f.x[k]) : "v"(src));
    }
}
// after the shared wait: the registers pass through an asm that follows it,
// so no use of them moves above the wait
template <int CW, int L>
__device__ __forceinline__ void flush_settle(FlushRegs<CW, L> &f) {
#pragma unroll
    for (int k = 0; k < FlushRegs<CW, L>::NI; ++k) asm volatile("" : "+v"(f.x[k]));
}
template <int CW, int L>
__device__ __forceinline__ void flush_store(const FlushRegs<CW, L> &f, const BuildArgs &a, long long rowbase,
                                            int w1_0, int n0, int w1e, int lane) {
    typedef FlushRegs<CW, L> F;
    const int Rl = lane / F::LP, j = (lane - Rl * F::LP) * 4;
    const int col = (n0 >> L) + j;
    const bool lok = Rl < F::RPI && col < (a.W2 >> L);
#pragma unroll
    for (int k = 0; k < F::NI; ++k) {
        const int R = k * F::RPI + Rl, w1 = w1_0 + R;
        if (lok && R < 16 && w1 < w1e) {
            const float v[4] = {f.x[k][0], f.x[k][1], f.x[k][2], f.x[k][3]};
            store_vec<4>(a.lvl[L], false, (rowbase + w1) * a.ld[L] + col, v, a.shadow[L]);
        }
    }
}

// Disparity-major stores (RC_LAYOUT_DISPARITY, ABI v9) of the pair layout's
// levels 0 and 2: level i of row block `row` is S_i[k][w1] with
// k = (w1 >> i) - j + (W2 >> i) - 1, row stride a.ld[i], a.shk[i] rows per
// block, so the pixels of one image row that look at the same disparity read
// one contiguous run of a row of S_i.  The values and their pooling order are
// epilogue_swapped's (the same bits, elsewhere); level 1 is pooled but not
// stored.  Per fragment column nb the wave stages its 16 x WT level-0 values
// (pitch WT + 4) and 16 x WT/4 level-2 values (pitch WT/4 + 4) in LDS and
// writes them along diagonals, one lane per 4 consecutive w1 of a diagonal:
// a 16-B store when all four lie in the wave's block (w1 < w1e, j inside
// [n0, n0 + WT) and < W2 >> i), else one dword per element that does.  A
// diagonal's 64-B piece of an nb joins the piece of the next nb in L2.
template <int STRIDE>     // four floats STRIDE floats apart, one wait
__device__ __forceinline__ void sheared_rd4(uint32_t a0, float (&x)[4]) {
    asm volatile("ds_read_b32 %0, %4\n\tds_read_b32 %1, %4 offset:%5\n\t"
                 "ds_read_b32 %2, %4 offset:%6\n\tds_read_b32 %3, %4 offset:%7\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(x[0]), "=&v"(x[1]), "=&v"(x[2]), "=&v"(x[3])
                 : "v"(a0), "i"(4 * STRIDE), "i"(8 * STRIDE), "i"(12 * STRIDE));
}

template <int FMA>
__device__ __forceinline__ void epilogue_sheared(f32x4 (&acc)[FMA][4], const BuildArgs &a, int row, int m0,
                                                 int n0, int lane, uint32_t st0, int w1e) {
    constexpr int WT = 16 * FMA, P0 = WT + 4, P2 = WT / 4 + 4;
    constexpr int ND = WT + 15;                     // level-0 diagonals of a 16 x WT block
    constexpr int NS0 = 4 * ND;                     // (w1 group, diagonal) slots
    constexpr uint32_t S2OFF = 16 * P0 * 4;         // level-2 image after the level-0 one
    const int g = lane >> 4, i = lane & 15;
    const int W0 = a.W2, Wq = a.W2 >> 2;
    const bool lv2 = a.nfused >= 3 && a.lvl[2] != nullptr;
    float *S0 = static_cast<float *>(a.lvl[0]) + (long long)row * a.shk[0] * a.ld[0];
    float *S2 = lv2 ? static_cast<float *>(a.lvl[2]) + (long long)row * a.shk[2] * a.ld[2] : nullptr;
    // one loop body for the four columns (code size): column nb is always
    // acc[.][0], the others move down one per pass (no dynamic register index)
#pragma unroll 1
    for (int nb = 0; nb < 4; ++nb) {
        const int w1_0 = m0 + 16 * nb;
        float v[FMA][4];
#pragma unroll
        for (int ma = 0; ma < FMA; ++ma) {
#pragma unroll
            for (int r = 0; r < 4; ++r) v[ma][r] = acc[ma][0][r];
            apply_scale(v[ma], a);
            acc[ma][0] = acc[ma][1];
            acc[ma][1] = acc[ma][2];
            acc[ma][2] = acc[ma][3];
        }
#pragma unroll
        for (int ma = 0; ma < FMA; ++ma)
            lds_st4(st0 + 4 * (i * P0 + 16 * ma + 4 * g), f32x4{v[ma][0], v[ma][1], v[ma][2], v[ma][3]});
        if (lv2) {
#pragma unroll
            for (int ma = 0; ma < FMA; ++ma) {
                const float s2 = pool2(pool2(v[ma][0], v[ma][1], false), pool2(v[ma][2], v[ma][3], false), false);
                lds_st1(st0 + S2OFF + 4 * (i * P2 + 4 * ma + g), s2);
            }
        }
        // level 0: slot s = q + 4 dd, rows w1l = 4q + r, diagonal d = w1l - jl
#pragma unroll
        for (int s0 = 0; s0 < NS0; s0 += 64) {
            const int s = s0 + lane;
            const int q = s & 3, d = (s >> 2) - (WT - 1);
            bool ok[4], all = s < NS0;
            int jl0 = 4 * q - d;                            // jl of r = 0
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int jl = jl0 + r;
                ok[r] = s < NS0 && jl >= 0 && jl < WT && n0 + jl < W0 && w1_0 + 4 * q + r < w1e;
                all = all && ok[r];
            }
            const int jc = jl0 < 0 ? 0 : (jl0 > WT - 4 ? WT - 4 : jl0);   // an address inside the image
            float x[4];
            sheared_rd4<P0 + 1>(st0 + 4 * ((4 * q) * P0 + jc), x);
            const long long k = (long long)(w1_0 - n0 + d + W0 - 1);
            float *dst = S0 + k * a.ld[0] + (w1_0 + 4 * q);
            if (all) {
                *reinterpret_cast<f32x4 *>(dst) = f32x4{x[0], x[1], x[2], x[3]};
            } else if (s < NS0 && (ok[0] || ok[1] || ok[2] || ok[3])) {
                // the clamped address read other elements: re-read the exact ones
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    if (!ok[r]) continue;
                    float y;
                    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)"
                                 : "=v"(y) : "v"(st0 + 4 * ((4 * q + r) * P0 + jl0 + r)));
                    dst[r] = y;
                }
            }
        }
        if (lv2) {
            // level 2: slot = q + 4 j2l; rows 4q..4q+3 share the column
#pragma unroll
            for (int s0 = 0; s0 < WT; s0 += 64) {
                const int s = s0 + lane;
                const int q = s & 3, j2l = s >> 2;
                bool ok[4], all = s < WT && (n0 >> 2) + j2l < Wq;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    ok[r] = all && w1_0 + 4 * q + r < w1e;
                }
                const bool any = ok[0];
                all = ok[0] && ok[1] && ok[2] && ok[3];
                float x[4];
                sheared_rd4<P2>(st0 + S2OFF + 4 * ((4 * q) * P2 + (j2l < WT / 4 ? j2l : 0)), x);
                const long long k = (long long)(((w1_0 >> 2) + q) - ((n0 >> 2) + j2l) + Wq - 1);
                float *dst = S2 + k * a.ld[2] + (w1_0 + 4 * q);
                if (all) {
                    *reinterpret_cast<f32x4 *>(dst) = f32x4{x[0], x[1], x[2], x[3]};
                } else if (any) {
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (ok[r]) dst[r] = x[r];
                }
            }
        }
    }
}

// Epilogue of the swapped-operand tile: acc[ma][nb] register r of lane l =
// C[w1 = m0 + 16nb + (l&15)][w2 = n0 + 16ma + 4(l>>4) + r].  One fragment
// column nb (16 w1 rows) at a time, every level: level l's image has rows
// w1 - m0 - 16nb, columns (w2 - n0) >> l, pitch (WT >> l) + 4 floats.
// w1_end: rows (w1) at or past it are not stored -- the image edge, or the
// end of this wave's block when it covers fewer than 4 fragments of w1 inside
// a tile (split kernel, volume_split.hip); -1 = a.W1.
template <int FMA, int MODE, int NLM>
__device__ __forceinline__ void epilogue_swapped(f32x4 (&acc)[FMA][4], const BuildArgs &a, int row,
                                                 int m0, int n0, int lane0, uint32_t st0, int w1_end = -1) {
    const int w1e = w1_end < 0 || w1_end > a.W1 ? a.W1 : w1_end;
    constexpr int WT = 16 * FMA;
    const bool bf = a.pyr_bf16 != 0;
    // kModeL2Stores (dev timing only, wrong output): every row stores into
    // one of 8 rows, so the same instructions write L2-resident lines
    const long long rowbase = (long long)((MODE & kModeL2Stores) ? (row & 7) : row) * a.W1;
    const int nl = a.nfused < NLM ? a.nfused : NLM;
    if constexpr ((MODE & kModeFastEpi) != 0 && (MODE & (kModeNoStores | kModeL2Stores | kModeDirect)) == 0) {
        // fp32 levels 0-2, power-of-two scale, 16-B aligned rows: the
        // geometry of every flush is compile-time (flush_rows16_fast)
        const bool fast = !bf && a.pow2 && (!a.lvl[0] || a.ld[0] % 4 == 0) &&
                          (nl < 2 || !a.lvl[1] || a.ld[1] % 4 == 0) && (nl < 3 || !a.lvl[2] || a.ld[2] % 4 == 0) &&
                          (nl < 4 || !a.lvl[3] || a.ld[3] % 2 == 0);
        if constexpr (NLM <= 3 && (MODE & kModePairEpi) != 0) {
            if (fast) {
                // two fragment columns at a time: every level image of both
                // staged in its own region of the wave's 16 KB of the ring,
                // all their reads, ONE wait, then all their stores
                const int g = lane0 >> 4, i = lane0 & 15;
                constexpr int S0 = 16 * (WT + 4) * 4, S1 = 16 * (WT / 2 + 4) * 4, S2 = 16 * (WT / 4 + 4) * 4;
                constexpr int SNB = S0 + S1 + S2;
#pragma unroll
                for (int p = 0; p < 2; ++p) {
                    FlushRegs<WT, 0> r0[2];
                    FlushRegs<WT / 2, 1> r1[2];
                    FlushRegs<WT / 4, 2> r2[2];
#pragma unroll
                    for (int k = 0; k < 2; ++k) {
                        const int nb = 2 * p + k;
                        const uint32_t b = st0 + k * SNB;
                        float v[FMA][4];
#pragma unroll
                        for (int ma = 0; ma < FMA; ++ma)
#pragma unroll
                            for (int r = 0; r < 4; ++r) v[ma][r] = acc[ma][nb][r] * a.scale;
                        if (a.lvl[0]) {
#pragma unroll
                            for (int ma = 0; ma < FMA; ++ma)
                                lds_st4(b + 4 * (i * (WT + 4) + 16 * ma + 4 * g), f32x4{v[ma][0], v[ma][1], v[ma][2], v[ma][3]});
                            flush_issue(r0[k], b, lane0);
                        }
                        if (nl < 2) continue;
                        float u[FMA][2];
#pragma unroll
                        for (int ma = 0; ma < FMA; ++ma) {
                            u[ma][0] = pool2(v[ma][0], v[ma][1], false);
                            u[ma][1] = pool2(v[ma][2], v[ma][3], false);
                        }
                        if (a.lvl[1]) {
#pragma unroll
                            for (int ma = 0; ma < FMA; ++ma)
                                lds_st2(b + S0 + 4 * (i * (WT / 2 + 4) + 8 * ma + 2 * g), f32x2{u[ma][0], u[ma][1]});
                            flush_issue(r1[k], b + S0, lane0);
                        }
                        if (nl < 3) continue;
                        if (a.lvl[2]) {
#pragma unroll
                            for (int ma = 0; ma < FMA; ++ma)
                                lds_st1(b + S0 + S1 + 4 * (i * (WT / 4 + 4) + 4 * ma + g), pool2(u[ma][0], u[ma][1], false));
                            flush_issue(r2[k], b + S0 + S1, lane0);
                        }
                    }
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
                    for (int k = 0; k < 2; ++k) {
                        flush_settle(r0[k]);
                        flush_settle(r1[k]);
                        flush_settle(r2[k]);
                    }
#pragma unroll
                    for (int k = 0; k < 2; ++k) {
                        const int w1_0 = m0 + 16 * (2 * p + k);
                        if (a.lvl[0]) flush_store(r0[k], a, rowbase, w1_0, n0, w1e, lane0);
                        if (nl >= 2 && a.lvl[1]) flush_store(r1[k], a, rowbase, w1_0, n0, w1e, lane0);
                        if (nl >= 3 && a.lvl[2]) flush_store(r2[k], a, rowbase, w1_0, n0, w1e, lane0);
                    }
                }
                return;
            }
        }
        if (fast) {
            const int g = lane0 >> 4, i = lane0 & 15;
#pragma unroll
            for (int nb = 0; nb < 4; ++nb) {
                float v[FMA][4];
#pragma unroll
                for (int ma = 0; ma < FMA; ++ma)
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[ma][r] = acc[ma][nb][r] * a.scale;
                const int w1_0 = m0 + 16 * nb;
                if (a.lvl[0]) {
#pragma unroll
                    for (int ma = 0; ma < FMA; ++ma)
                        lds_st4(st0 + 4 * (i * (WT + 4) + 16 * ma + 4 * g), f32x4{v[ma][0], v[ma][1], v[ma][2], v[ma][3]});
                    flush_rows16_fast<WT, 0, 4>(st0, a, rowbase, w1_0, n0, w1e, lane0);
                }
                if (nl < 2) continue;
                float u[FMA][2];
#pragma unroll
                for (int ma = 0; ma < FMA; ++ma) {
                    u[ma][0] = pool2(v[ma][0], v[ma][1], false);
                    u[ma][1] = pool2(v[ma][2], v[ma][3], false);
                }
                if (a.lvl[1]) {
#pragma unroll
                    for (int ma = 0; ma < FMA; ++ma)
                        lds_st2(st0 + 4 * (i * (WT / 2 + 4) + 8 * ma + 2 * g), f32x2{u[ma][0], u[ma][1]});
                    flush_rows16_fast<WT / 2, 1, 4>(st0, a, rowbase, w1_0, n0, w1e, lane0);
                }
                if (nl < 3) continue;
                float s2[FMA];
#pragma unroll
                for (int ma = 0; ma < FMA; ++ma) s2[ma] = pool2(u[ma][0], u[ma][1], false);
                if (a.lvl[2]) {
#pragma unroll
                    for (int ma = 0; ma < FMA; ++ma) lds_st1(st0 + 4 * (i * (WT / 4 + 4) + 4 * ma + g), s2[ma]);
                    flush_rows16_fast<WT / 4, 2, 4>(st0, a, rowbase, w1_0, n0, w1e, lane0);
                }
                if constexpr (NLM >= 4) {
                    if (nl < 4) continue;
                    // level 3: lanes l, l^16; level 4: lanes l, l^32 (as below)
                    float s3[FMA];
#pragma unroll
                    for (int ma = 0; ma < FMA; ++ma) {
                        const float o = __shfl_xor(s2[ma], 16);
                        s3[ma] = (g & 1) ? pool2(o, s2[ma], false) : pool2(s2[ma], o, false);
                    }
                    if (a.lvl[3]) {
                        if (!(g & 1)) {
#pragma unroll
                            for (int ma = 0; ma < FMA; ++ma)
                                lds_st1(st0 + 4 * (i * (WT / 8 + 4) + 2 * ma + (g >> 1)), s3[ma]);
                        }
                        flush_rows16_fast<WT / 8, 3, 2>(st0, a, rowbase, w1_0, n0, w1e, lane0);
                    }
                    if constexpr (NLM >= 5) {
                        if (nl < 5) continue;
                        float s4[FMA];
#pragma unroll
                        for (int ma = 0; ma < FMA; ++ma) {
                            const float o = __shfl_xor(s3[ma], 32);
                            s4[ma] = (g & 2) ? pool2(o, s3[ma], false) : pool2(s3[ma], o, false);
                        }
                        if (a.lvl[4]) {
                            if (g == 0) {
#pragma unroll
                                for (int ma = 0; ma < FMA; ++ma) lds_st1(st0 + 4 * (i * (WT / 16 + 4) + ma), s4[ma]);
                            }
                            flush_rows16_fast<WT / 16, 4, 1>(st0, a, rowbase, w1_0, n0, w1e, lane0);
                        }
                    }
                }
            }
            return;
        }
    }
    if constexpr ((MODE & kModeDirect) != 0) {
        // each lane stores its own values straight from the registers (no
        // LDS image): level l of lane (i, g) for fragment (ma, nb) is row
        // w1 = m0 + 16nb + i, columns ((n0 + 16ma + 4g) >> l) .. +(4 >> l)
        const int g = lane0 >> 4, i = lane0 & 15;
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) {
            const int w1 = m0 + 16 * nb + i;
            const bool rok = w1 < w1e;
            const long long rb = rowbase + w1;
            float v[FMA][4];
#pragma unroll
            for (int ma = 0; ma < FMA; ++ma)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float x = acc[ma][nb][r];
                    const float c = a.pow2 ? x * a.scale : x / a.sq;
                    v[ma][r] = bf ? round_bf16(c) : c;
                }
            auto put = [&](int l, int col, const float *x, int n) {   // n consecutive values of level l
                if (!a.lvl[l] || !rok || col >= (a.W2 >> l)) return;
                const long long e = rb * a.ld[l] + col;
                if (n == 4 && a.ld[l] % 4 == 0) store_vec<4>(a.lvl[l], bf, e, x, a.shadow[l]);
                else if (n >= 2 && a.ld[l] % 2 == 0) {
                    store_vec<2>(a.lvl[l], bf, e, x, a.shadow[l]);
                    if (n == 4) store_vec<2>(a.lvl[l], bf, e + 2, x + 2, a.shadow[l]);
                } else {
                    for (int k = 0; k < n; ++k) store_vec<1>(a.lvl[l], bf, e + k, x + k, a.shadow[l]);
                }
            };
#pragma unroll
            for (int ma = 0; ma < FMA; ++ma) {
                put(0, n0 + 16 * ma + 4 * g, v[ma], 4);
                if (nl < 2) continue;
                const float u[2] = {pool2(v[ma][0], v[ma][1], bf), pool2(v[ma][2], v[ma][3], bf)};
                put(1, (n0 >> 1) + 8 * ma + 2 * g, u, 2);
                if (nl < 3) continue;
                const float s2 = pool2(u[0], u[1], bf);
                put(2, (n0 >> 2) + 4 * ma + g, &s2, 1);
                if (nl < 4) continue;
                const float o3 = __shfl_xor(s2, 16);
                const float s3 = (g & 1) ? pool2(o3, s2, bf) : pool2(s2, o3, bf);
                if (!(g & 1)) put(3, (n0 >> 3) + 2 * ma + (g >> 1), &s3, 1);
                if (nl < 5) continue;
                const float o4 = __shfl_xor(s3, 32);
                const float s4 = (g & 2) ? pool2(o4, s3, bf) : pool2(s3, o4, bf);
                if (g == 0) put(4, (n0 >> 4) + ma, &s4, 1);
            }
        }
        return;
    }
    // one loop body for the four columns (code size, registers): column nb
    // is always acc[.][0], the others move down one per pass
#pragma unroll 1
    for (int nb = 0; nb < 4; ++nb) {
        // opaque per pass: otherwise the compiler hoists the per-lane staging
        // and store addresses of every level and vector width out of the
        // loops and keeps ~100 of them in VGPRs
        int lane = lane0;
        uint32_t st = st0;
        asm volatile("" : "+v"(lane), "+v"(st));
        const int g = lane >> 4, i = lane & 15;
        auto flush = [&](int l) {
            const int cw = WT >> l;
            store_rows16_any(st, cw + 4, cw, a.lvl[l], a.ld[l], bf, rowbase, m0 + 16 * nb, n0 >> l, w1e,
                             a.W2 >> l, lane, a.shadow[l]);
        };
        float v[FMA][4];
#pragma unroll
        for (int ma = 0; ma < FMA; ++ma) {
#pragma unroll
            for (int r = 0; r < 4; ++r) v[ma][r] = acc[ma][0][r];
            apply_scale(v[ma], a);
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (bf) v[ma][r] = round_bf16(v[ma][r]);
            acc[ma][0] = acc[ma][1];
            acc[ma][1] = acc[ma][2];
            acc[ma][2] = acc[ma][3];
        }
        if constexpr (MODE & kModeNoStores) {
            float keep = 0.f;
#pragma unroll
            for (int ma = 0; ma < FMA; ++ma) keep += v[ma][0] + v[ma][3];
            asm volatile("" ::"v"(keep));
            continue;
        }
        if (a.lvl[0]) {
#pragma unroll
            for (int ma = 0; ma < FMA; ++ma)
                lds_st4(st + 4 * (i * (WT + 4) + 16 * ma + 4 * g), f32x4{v[ma][0], v[ma][1], v[ma][2], v[ma][3]});
            flush(0);
        }
        if (nl < 2) continue;
        // level 1: lane-local pairs of w2
        float u[FMA][2];
#pragma unroll
        for (int ma = 0; ma < FMA; ++ma) {
            u[ma][0] = pool2(v[ma][0], v[ma][1], bf);
            u[ma][1] = pool2(v[ma][2], v[ma][3], bf);
        }
        if (a.lvl[1]) {
#pragma unroll
            for (int ma = 0; ma < FMA; ++ma)
                lds_st2(st + 4 * (i * (WT / 2 + 4) + 8 * ma + 2 * g), f32x2{u[ma][0], u[ma][1]});
            flush(1);
        }
        if (nl < 3) continue;
        // level 2: lane-local
        float s2[FMA];
#pragma unroll
        for (int ma = 0; ma < FMA; ++ma) s2[ma] = pool2(u[ma][0], u[ma][1], bf);
        if (a.lvl[2]) {
#pragma unroll
            for (int ma = 0; ma < FMA; ++ma) lds_st1(st + 4 * (i * (WT / 4 + 4) + 4 * ma + g), s2[ma]);
            flush(2);
        }
        if (nl < 4) continue;
        // level 3: lanes l, l^16 (w2 groups g, g^1); the even-g lane stores it
        float s3[FMA];
#pragma unroll
        for (int ma = 0; ma < FMA; ++ma) {
            const float o = __shfl_xor(s2[ma], 16);
            s3[ma] = (g & 1) ? pool2(o, s2[ma], bf) : pool2(s2[ma], o, bf);
        }
        if (a.lvl[3]) {
            if (!(g & 1)) {
#pragma unroll
                for (int ma = 0; ma < FMA; ++ma) lds_st1(st + 4 * (i * (WT / 8 + 4) + 2 * ma + (g >> 1)), s3[ma]);
            }
            flush(3);
        }
        if (nl < 5) continue;
        // level 4: lanes l, l^32 (g = 0 with g = 2)
        float s4[FMA];
#pragma unroll
        for (int ma = 0; ma < FMA; ++ma) {
            const float o = __shfl_xor(s3[ma], 32);
            s4[ma] = (g & 2) ? pool2(o, s3[ma], bf) : pool2(s3[ma], o, bf);
        }
        if (a.lvl[4]) {
            if (g == 0) {
#pragma unroll
                for (int ma = 0; ma < FMA; ++ma) lds_st1(st + 4 * (i * (WT / 16 + 4) + ma), s4[ma]);
            }
            flush(4);
        }
    }
}

}  // namespace rc
