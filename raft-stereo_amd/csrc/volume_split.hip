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
// (TW / 2 lanes x 16 B: all 64 at TW = 128) per instruction -> 4 instructions
// per stage.
template <int MODE, int TW, int SL>
__device__ __forceinline__ void sp_issue(const SpCtx &c, char *smem, int st) {
    typedef __attribute__((address_space(3))) void lds_void;
    using G = SpRing<TW, SL>;
    char *sA = smem + (st % SL) * G::Slot, *sB = sA + G::Op;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int r0 = 4 * c.wave + 2 * i;
        const int d = st * kSpBK + c.dr0 + 2 * i;
        // rows d >= D and columns past the tile extent are not fetched
        // (out-of-range offset)
        uint32_t offA = d < c.D && c.wA ? c.oA[i] + (uint32_t)st * c.sA : 0xFFFFFF00u;
        uint32_t offB = d < c.D && c.wB ? c.oB[i] + (uint32_t)st * c.sB : 0xFFFFFF00u;
        // lanes past the block's 2 TW floats write nothing (EXEC), so the
        // next block is not overwritten
        if constexpr (!(MODE & kModeNoLoads)) {
            if (TW == 128 || c.lane < TW / 2) {
                __builtin_amdgcn_raw_ptr_buffer_load_lds(c.r1, (lds_void *)(sA + (r0 >> 1) * G::Blk), 16, (int)offA, 0, 0, 0);
                __builtin_amdgcn_raw_ptr_buffer_load_lds(c.r2, (lds_void *)(sB + (r0 >> 1) * G::Blk), 16, (int)offB, 0, 0, 0);
            }
        }
    }
}

// K loop + epilogue of one wave with FA valid A fragments (w2) and FB valid B
// fragments (w1); FA = 0: no valid columns -- the wave still issues its DMA
// share and joins every barrier.
template <int FA, int FB, int MODE, int NLM, int TW, int SL>
__device__ __forceinline__ void split_body(const SpCtx &c, const BuildArgs &a, char *smem, int row) {
    using G = SpRing<TW, SL>;
    const int lane = c.lane, i = lane & 15, g = lane >> 4;
    // lane (i, g) reads d rows 8(g & 1) .. +7 of stage (g >> 1) of the K step
    const int lrow = (g & 1) * 4 * G::Blk;               // rows 8(g&1): 4 blocks in
    f32x4 acc[FA > 0 ? FA : 1][4];
#pragma unroll
    for (int x0 = 0; x0 < (FA > 0 ? FA : 1); ++x0)
#pragma unroll
        for (int y0 = 0; y0 < 4; ++y0) acc[x0][y0] = f32x4{0.f, 0.f, 0.f, 0.f};
    constexpr int KA = G::KA;
    const int nks = (c.nst + 1) >> 1;                     // K steps (the launcher pads nst to even)
    // stages of K steps 0 .. KA - 1 in flight
#pragma unroll
    for (int st = 0; st < 2 * KA; ++st)
        if (st < c.nst) sp_issue<MODE, TW, SL>(c, smem, st);
    for (int ks = 0; ks < nks; ++ks) {
        // RAW: my 8 DMA instructions of K step ks landed (the K steps issued
        // after it may still fly: KA - 1 of them at ks = 0, from the
        // prologue, KA - 2 later, since K step ks + KA - 1 is issued after
        // this wait); WAR: my LDS reads of K step ks - 1 are done.  Barrier.
        const int later = min(ks == 0 ? KA - 1 : KA - 2, nks - 1 - ks);
        if (KA >= 3 && later >= 2) asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)" ::: "memory");
        else if (later >= 1) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (ks >= 1 && 2 * (ks + KA - 1) < c.nst) {      // K step ks + KA - 1 into the slots of K step ks - 1
            sp_issue<MODE, TW, SL>(c, smem, 2 * (ks + KA - 1));
            sp_issue<MODE, TW, SL>(c, smem, 2 * (ks + KA - 1) + 1);
        }
        if constexpr (FA > 0 && !(MODE & kModeNoMath)) {
            const char *st = smem + ((2 * ks + (g >> 1)) % SL) * G::Slot + lrow;
            const char *pb = st + 4 * (c.o1 + i);                        // F1 (B): this wave's w1
            const char *pa = st + G::Op + 4 * (c.o2 + i);                // F2 (A): this wave's w2
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
#pragma unroll
            for (int n = 0; n < FB; ++n) fb[n] = sp_read<MODE, TW>(pb + 64 * n);
            if constexpr ((MODE & kModePhasePrio) != 0) {
                // dev A/B: every fragment read and split first, then all the
                // MFMAs at raised wave priority, so that the SIMD's other wave
                // fills the issue slots with its split while these run
                SplitFrag fa[FA];
#pragma unroll
                for (int m = 0; m < FA; ++m) fa[m] = sp_read<MODE, TW>(pa + 64 * m);
                __builtin_amdgcn_sched_barrier(0);
                __builtin_amdgcn_s_setprio(3);
#pragma unroll
                for (int m = 0; m < FA; ++m)
#pragma unroll
                    for (int n = 0; n < FB; ++n) mma6(acc[m][n], fa[m], fb[n]);
                __builtin_amdgcn_sched_barrier(0);
                __builtin_amdgcn_s_setprio(0);
            } else {
#pragma unroll
                for (int m = 0; m < FA; ++m) {
                    const SplitFrag fa = sp_read<MODE, TW>(pa + 64 * m);
                    if constexpr ((MODE & kModeMfmaPrio) != 0) {   // dev A/B: each fragment's MFMAs at raised priority
                        __builtin_amdgcn_sched_barrier(0);
                        __builtin_amdgcn_s_setprio(3);
                    }
#pragma unroll
                    for (int n = 0; n < FB; ++n) mma6(acc[m][n], fa, fb[n]);
                    if constexpr ((MODE & kModeMfmaPrio) != 0) {
                        __builtin_amdgcn_sched_barrier(0);
                        __builtin_amdgcn_s_setprio(0);
                    }
                }
            }
        }
    }
    // the ring becomes the waves' epilogue staging images
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if constexpr (FA > 0 && (MODE & kModeSheared) != 0) {
        // RC_LAYOUT_DISPARITY: levels 0 and 2 written disparity-major
        const int w1e = c.M0 + c.o1 + 16 * FB;
        epilogue_sheared<FA>(acc, a, row, c.M0 + c.o1, c.N0 + c.o2, lane,
                             lds_u32(smem + c.wave * G::Wave), w1e < a.W1 ? w1e : a.W1);
    } else if constexpr (FA > 0) {
        // the compile-time-geometry flushes (fp32 levels 0-2) unless the dev
        // A/B asks for the generic epilogue: config 2 262.5 vs 281.2 us
        // (profiles/r04/o/build_ablate.log, bit-identical)
        epilogue_swapped<FA, (MODE & kModeGenericEpi) ? MODE : (MODE | kModeFastEpi), NLM>(
            acc, a, row, c.M0 + c.o1, c.N0 + c.o2, lane,
            lds_u32(smem + c.wave * G::Wave), c.M0 + c.o1 + 16 * FB);
    }
}

template <int FA, int MODE, int NLM, int TW, int SL>
__device__ __forceinline__ void split_fb(int fb, const SpCtx &c, const BuildArgs &a, char *smem, int row) {
    if constexpr ((TW / 16 + 1) / 2 >= 4) {            // a wave's share: ceil(TW / 32) fragments
        if (fb >= 4) {
            split_body<FA, 4, MODE, NLM, TW, SL>(c, a, smem, row);
            return;
        }
    }
    if (fb == 3) split_body<FA, 3, MODE, NLM, TW, SL>(c, a, smem, row);
    else if (fb == 2) split_body<FA, 2, MODE, NLM, TW, SL>(c, a, smem, row);
    else split_body<FA, 1, MODE, NLM, TW, SL>(c, a, smem, row);
}

// TW, SL: the ring geometry (SpRing); tiles at most TW wide (the launcher)
template <int MODE, int NLM, int TW = 128, int SL = 4>
__global__ __launch_bounds__(256, 2) void build_split_kernel(BuildArgs a, int nwg_total, int tf1, int tf2,
                                                             int tiles1, int tiles2) {
    __shared__ __attribute__((aligned(16))) char smem[SpRing<TW, SL>::Bytes];
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
        // lane -> (row of its 2-row block, 4 columns); lanes >= TW / 2 idle
        const int w = 4 * (c.lane % (TW / 4));
        c.dr0 = 4 * c.wave + (c.lane >= TW / 4 ? 1 : 0);
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
    constexpr int FMAX = (TW / 16 + 1) / 2;                // fragments per wave at most (4 or 3)
    static_assert(FMAX == 3 || FMAX == 4, "split tile width");
    if (FMAX == 4 && fa >= 4) split_fb<FMAX, MODE, NLM, TW, SL>(fb, c, a, smem, row);
    else if (fa == 3) split_fb<3, MODE, NLM, TW, SL>(fb, c, a, smem, row);
    else if (fa == 2) split_fb<2, MODE, NLM, TW, SL>(fb, c, a, smem, row);
    else if (fa == 1) split_fb<1, MODE, NLM, TW, SL>(fb, c, a, smem, row);
    else split_body<0, 1, MODE, NLM, TW, SL>(c, a, smem, row);
}

#ifdef RAFTCORR_DEV
#include "dev/volume_split_dev.inc"   // ablation modes: libraftcorr_dev.so only
#endif

}  // namespace rc

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
    if (const hipError_t e = rc::dev_launch_build_split(a, nwg, tf1, tf2, tiles1, tiles2, s); e != hipErrorNotSupported)
        return e;
#endif
    if (a.shk[0]) {   // disparity-major levels 0 and 2 (the caller checked the pair layout)
        hipLaunchKernelGGL((rc::build_split_kernel<rc::kModeSheared, 3>), dim3((unsigned)nwg), dim3(256), 0, s, a,
                           (int)nwg, tf1, tf2, tiles1, tiles2);
        return hipGetLastError();
    }
    // up to 3 fused levels (the pair layout: 0 and 2 stored) keeps the
    // epilogue's level pointers out of the scalar registers
    if (a.nfused <= 3)
        hipLaunchKernelGGL((rc::build_split_kernel<0, 3>), dim3((unsigned)nwg), dim3(256), 0, s, a, (int)nwg, tf1, tf2, tiles1, tiles2);
    else
        hipLaunchKernelGGL((rc::build_split_kernel<0, rc::kSpMaxFused>), dim3((unsigned)nwg), dim3(256), 0, s, a,
                           (int)nwg, tf1, tf2, tiles1, tiles2);
    return hipGetLastError();
}
