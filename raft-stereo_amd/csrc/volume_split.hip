// fp32 correlation volume on bf16 MFMA by a three-way split of every operand
// (gfx950) -- the default fp32 build since ABI v6.
//
// Replaces CorrBlock1D.corr (/root/reference/model.py:318-326) and the
// avg_pool2d loop of CorrBlock1D.__init__ (:284-295), like the exact fp32
// MFMA kernel of volume.hip, at fp32 accuracy for a third of its MFMA time.
//
// Each fp32 operand x is cut into three bf16 pieces, x = h + m + l EXACTLY
// (h = RN_bf16(x), m = RN_bf16(x - h), l = RN_bf16(x - h - m); every
// subtraction is exact, and 3 x 8 significant bits plus the two sign bits the
// round-to-nearest steps gain cover fp32's 24).  Per 32-deep K step the
// product of two operands is the sum of six bf16 MFMAs,
//     mm + hl + lh + hm + mh + hh   (v_mfma_f32_16x16x32_bf16, fp32 accumulate)
// which drops only ml, lm, ll: below 2^-27 of |a||b| per product, under the
// fp32 rounding of the accumulation itself.  Measured against the fp64 oracle
// it is as accurate as the fp32 MFMA chain (tests/test_split_gpu.py).  bf16
// MFMA runs 16x the fp32 MFMA rate, so six of them cost 3/8 of the fp32 MFMA
// time; the build becomes bound by HBM (fmaps in, pyramid out) instead of by
// the fp32 matrix rate.
//
// Non-finite fmap values: an inf operand splits into inf and NaN pieces, so
// an inf in a row gives NaN where an fp32 GEMM gives +-inf (a NaN stays NaN);
// |x| > 3.39e38 rounds its bf16 head to inf.  RC_BUILD_EXACT_F32 selects the
// exact fp32 MFMA kernel for such inputs.
//
// Workgroup: 256 threads = 4 waves as 2 x 2 wave tiles of 64 (w2) x 64 (w1)
// (swapped operands: A = F2 rows -> M = w2, B = F1 rows -> N = w1, so every
// lane's accumulators hold 4 consecutive w2 of one w1 row and pyramid levels
// 1-2 pool lane-locally -- the epilogue of the bf16 ring kernel,
// epilogue_swapped).  Operand staging is the fp32 kernel's LDS-DMA ring
// (volume.hip): 16-d stages of [16 d][128 w] fp32 for F1 and for F2, filled
// by buffer_load ... lds with no VGPR staging, SL slots, one K step (32 d =
// two stages) multiplied while the next is in flight.  Each DMA instruction
// lands two 512-B rows; the blocks are 1040 B apart (16 B of padding) so the
// two 16-lane halves of a fragment read (rows 8 apart) fall on different
// banks.  Fragments are read in fp32 (lane (i, g): 8 consecutive d at one w,
// eight ds_read_b32 with immediate offsets) and split in registers right
// before their MFMAs.  Fragments (16 w) that lie wholly beyond W1 / W2 are
// skipped (template FA / FB), so W = 240 wastes no MFMA work.
#include "common.h"
#include "epilogue.h"
#include "split.h"

namespace rc {

}  // namespace rc
#include "split_ring.h"
namespace rc {

struct SpCtx {
    __amdgpu_buffer_rsrc_t r1, r2;
    int D, H, h, W1, W2, M0, N0, wave, lane, nst;
    int tw1, tw2;      // tile extent (w) along w1 / w2: 16 x fragments, <= 128
    int o1, o2;        // this wave's first column (w) inside the tile, w1 / w2
    // DMA source offsets of this lane's two rows at stage 0 (F1, F2) and the
    // per-stage step (kSpBK rows of d): a stage's offsets are one add away,
    // no per-stage 32-bit multiplies (8 % of the K loop's VALU issue)
    uint32_t oA[2], oB[2], sA, sB;
    int dr0;           // this lane's d row inside a stage, first instruction
    bool wA, wB;       // the lane's 4 columns inside the tile extent
};

// DMA share of this wave per stage: rows 4w..4w+3 of both tiles, 2 rows
// (1 KB = 64 lanes x 16 B) per instruction -> 4 instructions per stage.
template <int MODE>
__device__ __forceinline__ void sp_issue(const SpCtx &c, char *smem, int st) {
    typedef __attribute__((address_space(3))) void lds_void;
    char *sA = smem + (st % kSpSL) * kSpSlot, *sB = sA + kSpOp;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int r0 = 4 * c.wave + 2 * i;
        const int d = st * kSpBK + c.dr0 + 2 * i;
        // rows d >= D and columns past the tile extent are not fetched
        // (out-of-range offset)
        uint32_t offA = d < c.D && c.wA ? c.oA[i] + (uint32_t)st * c.sA : 0xFFFFFF00u;
        uint32_t offB = d < c.D && c.wB ? c.oB[i] + (uint32_t)st * c.sB : 0xFFFFFF00u;
        if constexpr ((MODE & kModeOldAddr) != 0) {   // dev A/B: the per-stage multiplies of round 3
            const int w = 4 * (c.lane & 31);
            const long long base = (long long)(d < c.D ? d : 0) * c.H + c.h;
            offA = d < c.D && w < c.tw1 ? (uint32_t)((base * c.W1 + c.M0 + w) * 4) : 0xFFFFFF00u;
            offB = d < c.D && w < c.tw2 ? (uint32_t)((base * c.W2 + c.N0 + w) * 4) : 0xFFFFFF00u;
        }
        if constexpr (!(MODE & kModeNoLoads)) {
            __builtin_amdgcn_raw_ptr_buffer_load_lds(c.r1, (lds_void *)(sA + (r0 >> 1) * kSpBlk), 16, (int)offA, 0, 0, 0);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(c.r2, (lds_void *)(sB + (r0 >> 1) * kSpBlk), 16, (int)offB, 0, 0, 0);
        }
    }
}

// K loop + epilogue of one wave with FA valid A fragments (w2) and FB valid B
// fragments (w1); FA = 0: no valid columns -- the wave still issues its DMA
// share and joins every barrier.
template <int FA, int FB, int MODE, int NLM>
__device__ __forceinline__ void split_body(const SpCtx &c, const BuildArgs &a, char *smem, int row) {
    const int lane = c.lane, i = lane & 15, g = lane >> 4;
    // lane (i, g) reads d rows 8(g & 1) .. +7 of stage (g >> 1) of the K step
    const int lrow = (g & 1) * 4 * kSpBlk;               // rows 8(g&1): 4 blocks in
    f32x4 acc[FA > 0 ? FA : 1][4];
#pragma unroll
    for (int x0 = 0; x0 < (FA > 0 ? FA : 1); ++x0)
#pragma unroll
        for (int y0 = 0; y0 < 4; ++y0) acc[x0][y0] = f32x4{0.f, 0.f, 0.f, 0.f};
    // kMode32: 32-wide fragments (ceil of the 16-wide counts)
    constexpr int FA2 = (FA + 1) / 2 > 0 ? (FA + 1) / 2 : 1, FB2 = (FB + 1) / 2;
    f32x16 acc32[(MODE & kMode32) ? FA2 : 1][(MODE & kMode32) ? FB2 : 1];
    if constexpr ((MODE & kMode32) != 0) {
#pragma unroll
        for (int x0 = 0; x0 < FA2; ++x0)
#pragma unroll
            for (int y0 = 0; y0 < FB2; ++y0)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc32[x0][y0][r] = 0.f;
    }
    const int nks = (c.nst + 1) >> 1;                     // K steps (the launcher pads nst to even)
    // stages of K steps 0 and 1 in flight
#pragma unroll
    for (int st = 0; st < 4; ++st)
        if (st < c.nst) sp_issue<MODE>(c, smem, st);
    for (int ks = 0; ks < nks; ++ks) {
        // RAW: my 8 DMA instructions of K step ks landed (K step 1, issued
        // with K step 0 before the loop, may still fly at ks = 0; later K
        // steps are issued after this wait); WAR: my LDS reads of K step
        // ks - 1 are done.  Barrier.
        if (ks == 0 && nks > 1) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (ks >= 1 && 2 * ks + 2 < c.nst) {             // K step ks + 1 into the slots of K step ks - 1
            sp_issue<MODE>(c, smem, 2 * ks + 2);
            sp_issue<MODE>(c, smem, 2 * ks + 3);
        }
        if constexpr (FA > 0 && !(MODE & kModeNoMath) && (MODE & kMode32)) {
            // 32x32x16 form: each 16-d stage is one MFMA k-step; lane
            // (r = l & 31, h = l >> 5) reads rows 8h..8h+7 at column r of
            // its 32-wide fragments (dev A/B, kMode32)
#pragma unroll
            for (int sub = 0; sub < 2; ++sub) {
                const char *st = smem + ((2 * ks + sub) % kSpSL) * kSpSlot + (lane >> 5) * 4 * kSpBlk;
                const char *pb = st + 4 * (c.o1 + (lane & 31));
                const char *pa = st + kSpOp + 4 * (c.o2 + (lane & 31));
                SplitFrag fb2[FB2];
#pragma unroll
                for (int n = 0; n < FB2; ++n) fb2[n] = sp_read<MODE>(pb + 128 * n);
#pragma unroll
                for (int m = 0; m < FA2; ++m) {
                    const SplitFrag fa = sp_read<MODE>(pa + 128 * m);
#pragma unroll
                    for (int n = 0; n < FB2; ++n) sp_mma6_32(acc32[m][n], fa, fb2[n]);
                }
            }
        } else if constexpr (FA > 0 && !(MODE & kModeNoMath)) {
            const char *st = smem + ((2 * ks + (g >> 1)) % kSpSL) * kSpSlot + lrow;
            const char *pb = st + 4 * (c.o1 + i);                        // F1 (B): this wave's w1
            const char *pa = st + kSpOp + 4 * (c.o2 + i);                // F2 (A): this wave's w2
            auto mma6 = [&](f32x4 &c, const SplitFrag &x, const SplitFrag &y) {
                if constexpr (MODE & kModeNoMfma) {   // dev timing probe: keep the split live
                    const u32x4s a = __builtin_bit_cast(u32x4s, x.h) ^ __builtin_bit_cast(u32x4s, x.m) ^
                                     __builtin_bit_cast(u32x4s, x.l) ^ __builtin_bit_cast(u32x4s, y.h) ^
                                     __builtin_bit_cast(u32x4s, y.m) ^ __builtin_bit_cast(u32x4s, y.l);
                    c[0] += __builtin_bit_cast(float, a[0] | a[1] | a[2] | a[3]);
                    return;
                }
                sp_mma6(c, x, y);
            };
            SplitFrag fb[FB];
            if constexpr (MODE & kModePhase) {
                // phased order (dev A/B): every fragment of the K step read and
                // split first, then all the MFMAs -- a wave alternates a VALU
                // phase and an MFMA phase, and its SIMD partner (the other
                // workgroup's wave) can fill one with the other.  Same products,
                // same order per accumulator: bit-identical.
                SplitFrag fas[FA];
#pragma unroll
                for (int n = 0; n < FB; ++n) fb[n] = sp_read<MODE>(pb + 64 * n);
#pragma unroll
                for (int m = 0; m < FA; ++m) fas[m] = sp_read<MODE>(pa + 64 * m);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int m = 0; m < FA; ++m)
#pragma unroll
                    for (int n = 0; n < FB; ++n) mma6(acc[m][n], fas[m], fb[n]);
            } else if constexpr (MODE & (kModeSched | kModeReorder)) {
                // pipelined order (dev A/B): only A0 and B0 are split before
                // the first MFMA; B1.. are split while the MFMAs of A0 run,
                // A(m+1) while those of A(m) run.  Same products, same
                // order per accumulator: bit-identical.
                SplitFrag fa = sp_read<MODE>(pa);
                fb[0] = sp_read<MODE>(pb);
#pragma unroll
                for (int n = 0; n < FB; ++n) {
                    if (n + 1 < FB) fb[n + 1] = sp_read<MODE>(pb + 64 * (n + 1));
                    mma6(acc[0][n], fa, fb[n]);
                }
#pragma unroll
                for (int m = 1; m < FA; ++m) {
                    fa = sp_read<MODE>(pa + 64 * m);
#pragma unroll
                    for (int n = 0; n < FB; ++n) mma6(acc[m][n], fa, fb[n]);
                }
                if constexpr (MODE & kModeSched) {
                    // the schedule: A0 + B0 up front (8 LDS reads, their split),
                    // then one MFMA per ~3 VALU with an LDS read every 4th
                    constexpr int NM = 6 * FA * FB, NV = 36 * (FA + FB - 2) + 8;
                    constexpr int VPM = (NV + NM - 1) / NM;
                    __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, 72, 0);
#pragma unroll
                    for (int k = 0; k < NM; ++k) {
                        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                        __builtin_amdgcn_sched_group_barrier(0x002, VPM, 0);
                        if (k % 4 == 0) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    }
                }
            } else {
#pragma unroll
                for (int n = 0; n < FB; ++n) fb[n] = sp_read<MODE>(pb + 64 * n);
#pragma unroll
                for (int m = 0; m < FA; ++m) {
                    const SplitFrag fa = sp_read<MODE>(pa + 64 * m);
#pragma unroll
                    for (int n = 0; n < FB; ++n) mma6(acc[m][n], fa, fb[n]);
                }
            }
        }
    }
    if constexpr (FA > 0 && (MODE & kMode32) != 0) {
        // 32x32 layout (lane l: w1 = 32n + (l & 31), w2 = 32m + (R & 3) +
        // 8(R >> 2) + 4(l >> 5)) -> the 16x16 layout epilogue_swapped takes
        // (lane 16g + i: w1 = 16nb + i, w2 = 16ma + 4g + r): lane 16g + i reads
        // lane 32(g & 1) + 16(nb & 1) + i, register 4(2(ma & 1) + (g >> 1)) + r
#pragma unroll
        for (int ma = 0; ma < FA; ++ma)
#pragma unroll
            for (int nb = 0; nb < 4; ++nb) {
                if (nb >= 2 * FB2) {
                    acc[ma][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
                    continue;
                }
                const int src = 32 * (g & 1) + 16 * (nb & 1) + i;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float v0 = acc32[ma >> 1][nb >> 1][8 * (ma & 1) + r];
                    const float v1 = acc32[ma >> 1][nb >> 1][8 * (ma & 1) + 4 + r];
                    const float a0 = __shfl(v0, src, 64), a1 = __shfl(v1, src, 64);
                    acc[ma][nb][r] = (g >> 1) ? a1 : a0;
                }
            }
    }
    // the ring becomes the waves' epilogue staging images
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if constexpr (FA > 0)
        // the compile-time-geometry flushes (fp32 levels 0-2) unless the dev
        // A/B asks for the generic epilogue: config 2 262.5 vs 281.2 us
        // (profiles/r04/o/build_ablate.log, bit-identical)
        epilogue_swapped<FA, (MODE & kModeGenericEpi) ? MODE : (MODE | kModeFastEpi), NLM>(
            acc, a, row, c.M0 + c.o1, c.N0 + c.o2, lane,
            lds_u32(smem + c.wave * (kSpSL * kSpSlot / 4)), c.M0 + c.o1 + 16 * FB);
}

template <int FA, int MODE, int NLM>
__device__ __forceinline__ void split_fb(int fb, const SpCtx &c, const BuildArgs &a, char *smem, int row) {
    if (fb >= 4) split_body<FA, 4, MODE, NLM>(c, a, smem, row);
    else if (fb == 3) split_body<FA, 3, MODE, NLM>(c, a, smem, row);
    else if (fb == 2) split_body<FA, 2, MODE, NLM>(c, a, smem, row);
    else split_body<FA, 1, MODE, NLM>(c, a, smem, row);
}

template <int MODE, int NLM>
__global__ __launch_bounds__(256, 2) void build_split_kernel(BuildArgs a, int nwg_total, int tf1, int tf2,
                                                             int tiles1, int tiles2) {
    __shared__ __attribute__((aligned(16))) char smem[kSpSL * kSpSlot];
    SpCtx c;
    c.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    c.lane = threadIdx.x & 63;
    // tiles of tf1 x tf2 16-wide fragments (launcher: balanced over the row,
    // at most 8 = 128 w); the four waves split them 2 x 2, ceil / floor
    const int T = tiles1 * tiles2;
    const int wgid = xcd_remap(blockIdx.x, nwg_total);   // a row's tiles share an XCD (and its L2)
    const int row = wgid / T, tile = wgid - row * T;
    const int tm = tile / tiles2, tn = tile - tm * tiles2;
    const int b = row / a.H;
    c.h = row - b * a.H;
    c.D = a.D; c.H = a.H; c.W1 = a.W1; c.W2 = a.W2;
    c.M0 = tm * 16 * tf1; c.N0 = tn * 16 * tf2;
    c.tw1 = 16 * tf1; c.tw2 = 16 * tf2;
    const int wm = c.wave & 1, wn = c.wave >> 1;
    const int h1 = (tf1 + 1) >> 1, h2 = (tf2 + 1) >> 1;  // fragments of the first wave half
    c.o1 = 16 * h1 * wm; c.o2 = 16 * h2 * wn;
    c.nst = 2 * ((a.D + 2 * kSpBK - 1) / (2 * kSpBK));   // whole K steps (d >= D reads zeros)
    {
        const int w = 4 * (c.lane & 31);
        c.dr0 = 4 * c.wave + (c.lane >> 5);
        c.wA = w < c.tw1;
        c.wB = w < c.tw2;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const long long base = (long long)(c.dr0 + 2 * i) * a.H + c.h;
            c.oA[i] = (uint32_t)((base * a.W1 + c.M0 + w) * 4);
            c.oB[i] = (uint32_t)((base * a.W2 + c.N0 + w) * 4);
        }
        c.sA = (uint32_t)kSpBK * (uint32_t)a.H * (uint32_t)a.W1 * 4u;
        c.sB = (uint32_t)kSpBK * (uint32_t)a.H * (uint32_t)a.W2 * 4u;
    }
    const long long img1 = (long long)a.D * a.H * a.W1, img2 = (long long)a.D * a.H * a.W2;
    c.r1 = make_rsrc(reinterpret_cast<const float *>(a.f1) + b * img1, clamp_bytes(img1 * 4));
    c.r2 = make_rsrc(reinterpret_cast<const float *>(a.f2) + b * img2, clamp_bytes(img2 * 4));
    // valid 16-wide fragments of this wave's block (wave-uniform): its share
    // of the tile, cut at the image edge
    const int n1 = wm ? tf1 - h1 : h1, n2 = wn ? tf2 - h2 : h2;
    const int cw1 = a.W1 - (c.M0 + c.o1), cw2 = a.W2 - (c.N0 + c.o2);
    const int v1 = cw1 <= 0 ? 0 : min(n1, (cw1 + 15) >> 4), v2 = cw2 <= 0 ? 0 : min(n2, (cw2 + 15) >> 4);
    const int fa = v1 == 0 ? 0 : v2, fb = v1;
    if (fa == 4) split_fb<4, MODE, NLM>(fb, c, a, smem, row);
    else if (fa == 3) split_fb<3, MODE, NLM>(fb, c, a, smem, row);
    else if (fa == 2) split_fb<2, MODE, NLM>(fb, c, a, smem, row);
    else if (fa == 1) split_fb<1, MODE, NLM>(fb, c, a, smem, row);
    else split_body<0, 1, MODE, NLM>(c, a, smem, row);
}

#ifdef RAFTCORR_DEV
// ====== warp-specialised persistent split kernel: every element split once ======
// DEV LIBRARY ONLY (RAFTCORR_SPLIT_KERNEL=3): measured and not kept --
// config 2: 383 us against 283 for build_split_kernel.
//
// The kernel above splits every fragment in the registers of each wave that
// reads it, i.e. twice (each operand tile is shared by two of the four
// waves), and its VALU -- not the matrix pipe -- sets its pace (DESIGN.md
// §3.1c).  Here a workgroup of 8 waves owns a CU: waves 0-3 compute (the same
// 2 x 2 wave tiles, swapped operands, epilogue_swapped), waves 4-7 load:
//   raw ring   2 slots x [2 operands][32 d][128 w] fp32 (64 KB), filled by
//              LDS-DMA (buffer_load_dwordx4 ... lds, 1 KB per instruction);
//   plane ring 2 slots x [2 operands][3 pieces][128 rows][32 d] bf16 (96 KB),
//              written by the loaders: each splits its 4 (operand, w, 8-d)
//              items of a K step once (raw via ds_read2_b32, planes via
//              ds_write_b128 at the conflict-free chunk swizzle of v1);
// 160 KB in all.  One s_barrier per K step g: after it the compute waves
// multiply planes(g) while the loaders issue the DMA of raw(g+2) into the raw
// slot of raw(g), split raw(g+1) into the other plane slot and wait for
// raw(g+2).  Loaders never store and compute waves never load from global
// memory, so neither role's vmcnt mixes loads with stores.  At a tile's last
// K step a second barrier lets the compute waves stage the epilogue in the
// plane slot they just finished; they arrive at the next K step's barrier
// after it, so the loaders cannot overwrite the staging.  Persistent walk
// over the tiles in XCD-contiguous runs (as build_bf16_ring_kernel).
constexpr int kWsRaw = 32 * 128 * 4;                 // one operand of a raw K step
constexpr int kWsRawSlot = 2 * kWsRaw;               // 32 KB
constexpr int kWsPlane = 128 * 64;                   // [128 rows][32 d] bf16
constexpr int kWsPlaneSlot = 6 * kWsPlane;           // 48 KB
constexpr int kWsLds = 2 * kWsRawSlot + 2 * kWsPlaneSlot;
static_assert(kWsLds <= 163840, "LDS");
static_assert(4 * kSpStb <= kWsPlaneSlot, "epilogue staging fits a plane slot");

__device__ __forceinline__ uint32_t ws_swz(int r, int c) { return (uint32_t)(r * 64 + 16 * (c ^ (-(r >> 2) & 3))); }

struct WsTile {
    int row, b, h, M0, N0;
};

__device__ __forceinline__ void ws_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// One K step of one compute wave: FA x FB fragments of plane slot ps.
template <int FA, int FB, int MODE>
__device__ __forceinline__ void ws_mma(f32x4 (&acc)[FA > 0 ? FA : 1][4], const char *ps, int o1, int o2,
                                       uint32_t loff) {
    if constexpr (FA > 0 && !(MODE & kModeNoMath)) {
        const char *pb = ps + o1 * 64 + loff;                   // F1 planes (B): this wave's w1
        const char *pa = ps + 3 * kWsPlane + o2 * 64 + loff;    // F2 planes (A): this wave's w2
        bf16x8 bh[FB], bm[FB], bl[FB], ah[FA], am[FA], al[FA];
#pragma unroll
        for (int n = 0; n < FB; ++n) {
            bh[n] = *reinterpret_cast<const bf16x8 *>(pb + 1024 * n);
            bm[n] = *reinterpret_cast<const bf16x8 *>(pb + kWsPlane + 1024 * n);
            bl[n] = *reinterpret_cast<const bf16x8 *>(pb + 2 * kWsPlane + 1024 * n);
        }
#pragma unroll
        for (int m = 0; m < FA; ++m) {
            ah[m] = *reinterpret_cast<const bf16x8 *>(pa + 1024 * m);
            am[m] = *reinterpret_cast<const bf16x8 *>(pa + kWsPlane + 1024 * m);
            al[m] = *reinterpret_cast<const bf16x8 *>(pa + 2 * kWsPlane + 1024 * m);
        }
#pragma unroll
        for (int m = 0; m < FA; ++m)
#pragma unroll
            for (int n = 0; n < FB; ++n) {
                acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[m], bm[n], acc[m][n], 0, 0, 0);
                acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[m], bl[n], acc[m][n], 0, 0, 0);
                acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[m], bh[n], acc[m][n], 0, 0, 0);
                acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[m], bm[n], acc[m][n], 0, 0, 0);
                acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[m], bh[n], acc[m][n], 0, 0, 0);
                acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[m], bh[n], acc[m][n], 0, 0, 0);
            }
    }
}

// A compute wave's whole tile: nks K steps (one barrier each, global step g0
// onwards), then the tile-end barrier and the epilogue.
template <int FA, int FB, int MODE, int NLM>
__device__ __forceinline__ void ws_tile(const BuildArgs &a, char *smem, const WsTile &t, int g0, int nks, int o1,
                                        int o2, int lane) {
    f32x4 acc[FA > 0 ? FA : 1][4];
#pragma unroll
    for (int x0 = 0; x0 < (FA > 0 ? FA : 1); ++x0)
#pragma unroll
        for (int y0 = 0; y0 < 4; ++y0) acc[x0][y0] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int i = lane & 15, g = lane >> 4;
    const uint32_t loff = (uint32_t)(i * 64 + 16 * (g ^ (-(i >> 2) & 3)));
    for (int k = 0; k < nks; ++k) {
        ws_barrier();                                             // B(g): planes(g) written
        ws_mma<FA, FB, MODE>(acc, smem + 2 * kWsRawSlot + ((g0 + k) & 1) * kWsPlaneSlot, o1, o2, loff);
    }
    ws_barrier();                                                 // E: every wave done with planes(g)
    if constexpr (FA > 0) {
        const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        char *st = smem + 2 * kWsRawSlot + ((g0 + nks - 1) & 1) * kWsPlaneSlot + wave * kSpStb;
        epilogue_swapped<FA, MODE, NLM>(acc, a, t.row, t.M0 + o1, t.N0 + o2, lane, lds_u32(st),
                                        t.M0 + o1 + 16 * FB);
    }
}

template <int FA, int MODE, int NLM>
__device__ __forceinline__ void ws_tile_fb(int fb, const BuildArgs &a, char *smem, const WsTile &t, int g0,
                                           int nks, int o1, int o2, int lane) {
    if (fb >= 4) ws_tile<FA, 4, MODE, NLM>(a, smem, t, g0, nks, o1, o2, lane);
    else if (fb == 3) ws_tile<FA, 3, MODE, NLM>(a, smem, t, g0, nks, o1, o2, lane);
    else if (fb == 2) ws_tile<FA, 2, MODE, NLM>(a, smem, t, g0, nks, o1, o2, lane);
    else ws_tile<FA, 1, MODE, NLM>(a, smem, t, g0, nks, o1, o2, lane);
}

template <int MODE, int NLM>
__global__ __launch_bounds__(512, 1) void build_split_ws_kernel(BuildArgs a, int ntiles, int tf1, int tf2,
                                                                  int tiles1, int tiles2) {
    __shared__ __attribute__((aligned(16))) char smem[kWsLds];
    typedef __attribute__((address_space(3))) void lds_void;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int D = a.D, H = a.H, W1 = a.W1, W2 = a.W2;
    const int T = tiles1 * tiles2;
    // persistent walk: the tiles are cut into 8 contiguous runs, one per XCD
    // (workgroup v runs on XCD v % 8), taken round-robin by its workgroups
    const int nwg = gridDim.x, v = blockIdx.x;
    const int xcd = v & 7, lw = v >> 3;
    const int gx = (nwg - xcd + 7) >> 3;
    const int before = xcd * (nwg >> 3) + min(xcd, nwg & 7);
    const int t0 = (int)((long long)ntiles * before / nwg);
    const int t1 = (int)((long long)ntiles * (before + gx) / nwg);
    auto tile_at = [&](int k) {
        WsTile t;
        const int id = t0 + lw + k * gx;
        t.row = id / T;
        const int tl = id - t.row * T, tm = tl / tiles2, tn = tl - tm * tiles2;
        t.b = t.row / H;
        t.h = t.row - t.b * H;
        t.M0 = tm * 16 * tf1;
        t.N0 = tn * 16 * tf2;
        return t;
    };
    const int nmine = t0 + lw < t1 ? (t1 - t0 - lw + gx - 1) / gx : 0;
    if (nmine == 0) return;                                       // workgroup-uniform
    const int nks = (D + 31) / 32;
    const int total = nmine * nks;
    const int tw1 = 16 * tf1, tw2 = 16 * tf2;

    if (wave >= 4) {
        // ------------------------------ loaders ------------------------------
        const int lt = threadIdx.x - 256, lw4 = wave - 4;
        const int r = lt & 127, cb = lt >> 7;
        const long long img1 = (long long)D * H * W1, img2 = (long long)D * H * W2;
        // DMA of global K step gs (tile gs / nks, step gs % nks) into raw slot gs & 1
        auto dma = [&](int gs) {
            const WsTile t = tile_at(gs / nks);
            const int s = gs - (gs / nks) * nks;
            const auto r1 = make_rsrc(reinterpret_cast<const float *>(a.f1) + t.b * img1, clamp_bytes(img1 * 4));
            const auto r2 = make_rsrc(reinterpret_cast<const float *>(a.f2) + t.b * img2, clamp_bytes(img2 * 4));
            char *slot = smem + (gs & 1) * kWsRawSlot;
            const int w = 4 * (lane & 31);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int ins = 8 * lw4 + k;                      // 0..15 F1 rows, 16..31 F2 rows
                const int o = ins >> 4, rp = ins & 15;            // operand, row pair
                const int d = 32 * s + 2 * rp + (lane >> 5);
                const int Wo = o ? W2 : W1, org = o ? t.N0 : t.M0, tw = o ? tw2 : tw1;
                const bool ok = d < D && w < tw && org + w < Wo;
                const uint32_t off = ok ? (uint32_t)((((long long)d * H + t.h) * Wo + org + w) * 4) : 0xFFFFFF00u;
                if constexpr (!(MODE & kModeNoLoads))
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(o ? r2 : r1, (lds_void *)(slot + o * kWsRaw + rp * 1024),
                                                             16, (int)off, 0, 0, 0);
            }
        };
        // L2 touch of K step gs: one dword per 128-B line of its 32 KB (one
        // load per loader lane), so the DMA two steps later hits L2; the value
        // is never used and the load stays outside every vmcnt wait but the
        // last (it is issued after the DMA, and loads complete in order)
        auto touch = [&](int gs) {
            if constexpr (!(MODE & kModeNoLoads) && !(MODE & 64)) {
                const WsTile t = tile_at(gs / nks);
                const int s = gs - (gs / nks) * nks;
                const int o = lt >> 7, q = lt & 127;              // 128 lines per operand
                const int d = 32 * s + (q >> 2), w = 32 * (q & 3);
                const int Wo = o ? W2 : W1, org = o ? t.N0 : t.M0, tw = o ? tw2 : tw1;
                const long long img = o ? img2 : img1;
                const auto rr = make_rsrc(reinterpret_cast<const float *>(o ? a.f2 : a.f1) + t.b * img,
                                          clamp_bytes(img * 4));
                const bool ok = d < D && w < tw && org + w < Wo;
                const uint32_t off = ok ? (uint32_t)((((long long)d * H + t.h) * Wo + org + w) * 4) : 0xFFFFFF00u;
                const float v = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rr, (int)off, 0, 0));
                asm volatile("" ::"v"(v));
            }
        };
        // split raw K step gs into plane slot gs & 1
        auto split = [&](int gs) {
            const char *raw = smem + (gs & 1) * kWsRawSlot;
            char *pl = smem + 2 * kWsRawSlot + (gs & 1) * kWsPlaneSlot;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int o = j >> 1, c = cb + 2 * (j & 1);
                float x[8];
#pragma unroll
                for (int q = 0; q < 8; ++q)
                    x[q] = *reinterpret_cast<const float *>(raw + o * kWsRaw + (8 * c + q) * 512 + 4 * r);
                const SplitFrag f = sp_split(x);
                char *dst = pl + o * 3 * kWsPlane + ws_swz(r, c);
                *reinterpret_cast<bf16x8 *>(dst) = f.h;
                *reinterpret_cast<bf16x8 *>(dst + kWsPlane) = f.m;
                *reinterpret_cast<bf16x8 *>(dst + 2 * kWsPlane) = f.l;
            }
        };
        dma(0);
        if (total > 1) dma(1);
        if (total > 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        ws_barrier();                                             // P: raw(0) landed everywhere
        split(0);
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        if (total > 2) touch(2);
        if (total > 3) touch(3);
        for (int gs = 0; gs < total; ++gs) {
            ws_barrier();                                         // B(gs)
            if (gs + 2 < total) dma(gs + 2);                      // into the raw slot of raw(gs)
            if (gs + 4 < total) touch(gs + 4);
            if (gs + 1 < total) split(gs + 1);                    // raw(gs + 1) landed before B(gs)
            // raw(gs + 2) landed; the newest touch may still fly
            if (gs + 4 < total) asm volatile("s_waitcnt vmcnt(1) lgkmcnt(0)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            if ((gs + 1) % nks == 0) ws_barrier();                // E of the compute waves' tile end
        }
        return;
    }
    // ------------------------------ compute ------------------------------
    ws_barrier();                                                 // P
    const int wm = wave & 1, wn = wave >> 1;
    const int h1 = (tf1 + 1) >> 1, h2 = (tf2 + 1) >> 1;
    const int o1 = 16 * h1 * wm, o2 = 16 * h2 * wn;
    const int n1 = wm ? tf1 - h1 : h1, n2 = wn ? tf2 - h2 : h2;
    for (int k = 0; k < nmine; ++k) {
        const WsTile t = tile_at(k);
        const int cw1 = W1 - (t.M0 + o1), cw2 = W2 - (t.N0 + o2);
        const int v1 = cw1 <= 0 ? 0 : min(n1, (cw1 + 15) >> 4), v2 = cw2 <= 0 ? 0 : min(n2, (cw2 + 15) >> 4);
        const int fa = v1 == 0 ? 0 : v2, fb = v1;
        const int g0 = k * nks;
        if (fa == 4) ws_tile_fb<4, MODE, NLM>(fb, a, smem, t, g0, nks, o1, o2, lane);
        else if (fa == 3) ws_tile_fb<3, MODE, NLM>(fb, a, smem, t, g0, nks, o1, o2, lane);
        else if (fa == 2) ws_tile_fb<2, MODE, NLM>(fb, a, smem, t, g0, nks, o1, o2, lane);
        else if (fa == 1) ws_tile_fb<1, MODE, NLM>(fb, a, smem, t, g0, nks, o1, o2, lane);
        else ws_tile<0, 1, MODE, NLM>(a, smem, t, g0, nks, o1, o2, lane);
    }
}
#endif  // RAFTCORR_DEV

}  // namespace rc

#ifdef RAFTCORR_DEV
static int device_cus_split() {
    static int n = 0;
    if (!n) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
    }
    return n;
}
#endif

// Split-bf16 build for fp32 fmaps and an fp32 pyramid.  Returns
// hipErrorNotSupported (nothing launched) when the shape is outside what the
// kernel addresses; the caller then runs the exact fp32 MFMA kernel.  Fuses
// at most kSpMaxFused levels: a.nfused is lowered to what was written
// and the caller pools the rest.
hipError_t rc_launch_build_split(rc::BuildArgs &a, hipStream_t s) {
    // per-image byte offsets are 32-bit (0xFFFFFF00 = the out-of-range marker),
    // and rows are DMA'd in 16-B pieces (W1, W2 multiples of 4)
    const long long img = (long long)a.D * a.H * (a.W1 > a.W2 ? a.W1 : a.W2) * 4;
    if (img >= 0xFFFFFF00LL || a.pyr_bf16 || a.W1 % 4 || a.W2 % 4) return hipErrorNotSupported;
    if (a.nfused > rc::kSpMaxFused) {
        // levels past the fused ones are pooled from memory: they must exist
        for (int l = rc::kSpMaxFused - 1; l < a.nfused; ++l)
            if (!a.lvl[l]) return hipErrorNotSupported;
        a.nfused = rc::kSpMaxFused;
    }
    // balanced tiles: a row of nf fragments in ceil(nf / 8) tiles of equal
    // size (W = 160: two of 5 fragments instead of 8 + 2; W = 240: 8 + 7)
    auto tile_frags = [](int W) {
        const int nf = (W + 15) / 16, nt = (nf + 7) / 8;
        return (nf + nt - 1) / nt;
    };
    const int tf1 = tile_frags(a.W1), tf2 = tile_frags(a.W2);
    const int tiles1 = ((a.W1 + 15) / 16 + tf1 - 1) / tf1, tiles2 = ((a.W2 + 15) / 16 + tf2 - 1) / tf2;
    const long long nwg = (long long)a.B * a.H * tiles1 * tiles2;
    if (nwg <= 0) return hipSuccess;
    if (nwg > 0x7FFFFFFF) return hipErrorInvalidValue;
#ifdef RAFTCORR_DEV
    // dev-only: RAFTCORR_SPLIT_KERNEL=3 runs the warp-specialised persistent
    // kernel (measured and not kept) with the same
    // RAFTCORR_SPLIT_MODE ablation flags
    if (rc::dev_knob("RAFTCORR_SPLIT_KERNEL") == 3) {
        const unsigned cus = (unsigned)device_cus_split();
        const long long ntiles = nwg;
        const unsigned nws = (unsigned)(ntiles < cus ? ntiles : cus);   // persistent: one workgroup per CU
        switch (rc::dev_knob("RAFTCORR_SPLIT_MODE")) {
            case 1: hipLaunchKernelGGL((rc::build_split_ws_kernel<1, 3>), dim3(nws), dim3(512), 0, s, a, (int)ntiles, tf1, tf2, tiles1, tiles2); break;
            case 2: hipLaunchKernelGGL((rc::build_split_ws_kernel<2, 3>), dim3(nws), dim3(512), 0, s, a, (int)ntiles, tf1, tf2, tiles1, tiles2); break;
            case 4: hipLaunchKernelGGL((rc::build_split_ws_kernel<4, 3>), dim3(nws), dim3(512), 0, s, a, (int)ntiles, tf1, tf2, tiles1, tiles2); break;
            case 3: hipLaunchKernelGGL((rc::build_split_ws_kernel<3, 3>), dim3(nws), dim3(512), 0, s, a, (int)ntiles, tf1, tf2, tiles1, tiles2); break;
            case 64: hipLaunchKernelGGL((rc::build_split_ws_kernel<64, 3>), dim3(nws), dim3(512), 0, s, a, (int)ntiles, tf1, tf2, tiles1, tiles2); break;
            default:
                if (a.nfused <= 3) hipLaunchKernelGGL((rc::build_split_ws_kernel<0, 3>), dim3(nws), dim3(512), 0, s, a, (int)ntiles, tf1, tf2, tiles1, tiles2);
                else hipLaunchKernelGGL((rc::build_split_ws_kernel<0, rc::kSpMaxFused>), dim3(nws), dim3(512), 0, s, a, (int)ntiles, tf1, tf2, tiles1, tiles2);
        }
        return hipGetLastError();
    }
#endif
    // the 8-wave kernel (volume_split8.hip) when it applies
    {
        const hipError_t e8 = rc_launch_build_split8(a, s);
        if (e8 != hipErrorNotSupported) return e8;
    }
#ifdef RAFTCORR_DEV
    // dev-only: RAFTCORR_SPLIT_KERNEL=4 runs the persistent deferred-epilogue
    // kernel (volume_split_p.hip) where it applies
    if (rc::dev_knob("RAFTCORR_SPLIT_KERNEL") == 4) {
        const hipError_t ep = rc_launch_build_split_persist(a, nwg, tf1, tf2, tiles1, tiles2, s);
        if (ep != hipErrorNotSupported) return ep;
    }
#endif
#ifdef RAFTCORR_DEV
    // dev-only ablations (timing only): RAFTCORR_SPLIT_MODE = kMode* flags
    // (1 no operand loads, 2 no epilogue stores, 4 no MFMAs; sums combine)
    switch (rc::dev_knob("RAFTCORR_SPLIT_MODE")) {
        case 1: hipLaunchKernelGGL((rc::build_split_kernel<1, 3>), dim3((unsigned)nwg), dim3(256), 0, s, a, (int)nwg, tf1, tf2, tiles1, tiles2); return hipGetLastError();
        case 2: hipLaunchKernelGGL((rc::build_split_kernel<2, 3>), dim3((unsigned)nwg), dim3(256), 0, s, a, (int)nwg, tf1, tf2, tiles1, tiles2); return hipGetLastError();
        case 3: hipLaunchKernelGGL((rc::build_split_kernel<3, 3>), dim3((unsigned)nwg), dim3(256), 0, s, a, (int)nwg, tf1, tf2, tiles1, tiles2); return hipGetLastError();
        case 4: hipLaunchKernelGGL((rc::build_split_kernel<4, 3>), dim3((unsigned)nwg), dim3(256), 0, s, a, (int)nwg, tf1, tf2, tiles1, tiles2); return hipGetLastError();
        case 5: hipLaunchKernelGGL((rc::build_split_kernel<5, 3>), dim3((unsigned)nwg), dim3(256), 0, s, a, (int)nwg, tf1, tf2, tiles1, tiles2); return hipGetLastError();
        case 65541: hipLaunchKernelGGL((rc::build_split_kernel<65541, 3>), dim3((unsigned)nwg), dim3(256), 0, s, a, (int)nwg, tf1, tf2, tiles1, tiles2); return hipGetLastError();
        case 6: hipLaunchKernelGGL((rc::build_split_kernel<6, 3>), dim3((unsigned)nwg), dim3(256), 0, s, a, (int)nwg, tf1, tf2, tiles1, tiles2); return hipGetLastError();
        case 7: hipLaunchKernelGGL((rc::build_split_kernel<7, 3>), dim3((unsigned)nwg), dim3(256), 0, s, a, (int)nwg, tf1, tf2, tiles1, tiles2); return hipGetLastError();
        case 128: hipLaunchKernelGGL((rc::build_split_kernel<128, 3>), dim3((unsigned)nwg), dim3(256), 0, s, a, (int)nwg, tf1, tf2, tiles1, tiles2); return hipGetLastError();
        case 512: hipLaunchKernelGGL((rc::build_split_kernel<512, 3>), dim3((unsigned)nwg), dim3(256), 0, s, a, (int)nwg, tf1, tf2, tiles1, tiles2); return hipGetLastError();
        case 1024: hipLaunchKernelGGL((rc::build_split_kernel<1024, 3>), dim3((unsigned)nwg), dim3(256), 0, s, a, (int)nwg, tf1, tf2, tiles1, tiles2); return hipGetLastError();
        case 1027: hipLaunchKernelGGL((rc::build_split_kernel<1027, 3>), dim3((unsigned)nwg), dim3(256), 0, s, a, (int)nwg, tf1, tf2, tiles1, tiles2); return hipGetLastError();
        case 515: hipLaunchKernelGGL((rc::build_split_kernel<515, 3>), dim3((unsigned)nwg), dim3(256), 0, s, a, (int)nwg, tf1, tf2, tiles1, tiles2); return hipGetLastError();
        case 256: hipLaunchKernelGGL((rc::build_split_kernel<256, 3>), dim3((unsigned)nwg), dim3(256), 0, s, a, (int)nwg, tf1, tf2, tiles1, tiles2); return hipGetLastError();
        case 8192: hipLaunchKernelGGL((rc::build_split_kernel<8192, 3>), dim3((unsigned)nwg), dim3(256), 0, s, a, (int)nwg, tf1, tf2, tiles1, tiles2); return hipGetLastError();
        case 16384: hipLaunchKernelGGL((rc::build_split_kernel<16384, 3>), dim3((unsigned)nwg), dim3(256), 0, s, a, (int)nwg, tf1, tf2, tiles1, tiles2); return hipGetLastError();
        case 24576: hipLaunchKernelGGL((rc::build_split_kernel<24576, 3>), dim3((unsigned)nwg), dim3(256), 0, s, a, (int)nwg, tf1, tf2, tiles1, tiles2); return hipGetLastError();
        case 32768: hipLaunchKernelGGL((rc::build_split_kernel<32768, 3>), dim3((unsigned)nwg), dim3(256), 0, s, a, (int)nwg, tf1, tf2, tiles1, tiles2); return hipGetLastError();
        case 2097152: hipLaunchKernelGGL((rc::build_split_kernel<2097152, 3>), dim3((unsigned)nwg), dim3(256), 0, s, a, (int)nwg, tf1, tf2, tiles1, tiles2); return hipGetLastError();
        case 1048576: hipLaunchKernelGGL((rc::build_split_kernel<1048576, 3>), dim3((unsigned)nwg), dim3(256), 0, s, a, (int)nwg, tf1, tf2, tiles1, tiles2); return hipGetLastError();
        case 524288: hipLaunchKernelGGL((rc::build_split_kernel<524288, 3>), dim3((unsigned)nwg), dim3(256), 0, s, a, (int)nwg, tf1, tf2, tiles1, tiles2); return hipGetLastError();
        case 524293: hipLaunchKernelGGL((rc::build_split_kernel<524288, rc::kSpMaxFused>), dim3((unsigned)nwg), dim3(256), 0, s, a, (int)nwg, tf1, tf2, tiles1, tiles2); return hipGetLastError();
        case 262144: hipLaunchKernelGGL((rc::build_split_kernel<262144, 3>), dim3((unsigned)nwg), dim3(256), 0, s, a, (int)nwg, tf1, tf2, tiles1, tiles2); return hipGetLastError();
        case 262149: hipLaunchKernelGGL((rc::build_split_kernel<262149, 3>), dim3((unsigned)nwg), dim3(256), 0, s, a, (int)nwg, tf1, tf2, tiles1, tiles2); return hipGetLastError();
        case 131072: hipLaunchKernelGGL((rc::build_split_kernel<131072, 3>), dim3((unsigned)nwg), dim3(256), 0, s, a, (int)nwg, tf1, tf2, tiles1, tiles2); return hipGetLastError();
        case 131077: hipLaunchKernelGGL((rc::build_split_kernel<131072, rc::kSpMaxFused>), dim3((unsigned)nwg), dim3(256), 0, s, a, (int)nwg, tf1, tf2, tiles1, tiles2); return hipGetLastError();
        case 65536: hipLaunchKernelGGL((rc::build_split_kernel<65536, 3>), dim3((unsigned)nwg), dim3(256), 0, s, a, (int)nwg, tf1, tf2, tiles1, tiles2); return hipGetLastError();
        case 32771: hipLaunchKernelGGL((rc::build_split_kernel<32771, 3>), dim3((unsigned)nwg), dim3(256), 0, s, a, (int)nwg, tf1, tf2, tiles1, tiles2); return hipGetLastError();
        default: break;
    }
#endif
    // up to 3 fused levels (the pair layout: 0 and 2 stored) keeps the
    // epilogue's level pointers out of the scalar registers
    if (a.nfused <= 3)
        hipLaunchKernelGGL((rc::build_split_kernel<0, 3>), dim3((unsigned)nwg), dim3(256), 0, s, a, (int)nwg, tf1, tf2, tiles1, tiles2);
    else
        hipLaunchKernelGGL((rc::build_split_kernel<0, rc::kSpMaxFused>), dim3((unsigned)nwg), dim3(256), 0, s, a,
                           (int)nwg, tf1, tf2, tiles1, tiles2);
    return hipGetLastError();
}
