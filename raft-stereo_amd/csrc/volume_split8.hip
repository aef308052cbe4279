// fp32 correlation volume on bf16 MFMA, 8-wave variant (gfx950): the
// arithmetic of volume_split.hip (three exact bf16 pieces per fp32 operand,
// six v_mfma_f32_16x16x32_bf16 products per fp32 product) with 64 x 128
// wave tiles.  Replaces CorrBlock1D.corr (/root/reference/model.py:318-326)
// and the avg_pool2d loop of CorrBlock1D.__init__ (:284-295).
#include "split_ring.h"

// DEV LIBRARY ONLY (RAFTCORR_SPLIT_KERNEL=8): measured and not kept -- config 2
// 309 vs 277 us for build_split_kernel, compute alone 193 vs 189 us
// (profiles/r04/f/build_ablate.log); Middlebury 1061 vs 1128.
#ifdef RAFTCORR_DEV
namespace rc {

// ====== 8-wave variant: 64 x 128 wave tiles, one workgroup per 256 x 256 tile ======
// The split's VALU, not the matrix pipe, paces build_split_kernel: a wave
// splits FA + FB = 8 fragments per K step for 16 fragment products (96
// MFMAs), ~3.8 VALU instructions per MFMA, while a 16x16x32 MFMA leaves its
// SIMD's vector issue free for about two (MI355X_MICROARCH.md, constants
// table).  Here a wave owns 4 (w1) x 8 (w2) fragments: 12 splits for 32
// products (192 MFMAs), 2.75 VALU per MFMA, and every F1 fragment is split
// by ONE wave per K step.  Workgroup: 8 waves (2 per SIMD, 128 accumulator
// registers each) as 4 along w1 x 2 along w2 over a tile of up to 16 x 16
// fragments -- a whole 240-wide row -- staged as four [16 d][128 w] images
// per ring stage (F1 and F2, two halves each: the halves hold tile fragments
// [0, h) and [h, tf), h = ceil(tf / 2)), 4 stages of 33 KB = 133 KB of LDS,
// one workgroup per CU.  Each wave issues 4 of the 32 DMA instructions of a
// stage, like build_split_kernel's 4 waves.
constexpr int kS8Img = 8 * kSpBlk;          // one [16 d][128 w] half image
constexpr int kS8Slot = 4 * kS8Img;         // F1 halves 0, 1; F2 halves 0, 1
constexpr int kS8Stb = 16 * (128 + 4) * 4;  // per-wave epilogue staging (WT 128)
static_assert(8 * kS8Stb <= kSpSL * kS8Slot, "epilogue staging aliases the ring");

struct Sp8Ctx {
    __amdgpu_buffer_rsrc_t rd;   // this wave's DMA source image (F1 for waves 0-3, F2 for 4-7)
    int D, H, h, M0, N0, wave, lane, nst;
    int dW, dorg, dhw;    // its DMA: image width, first tile column of its half, columns
    int ho1, ho2;         // tile column where half 1 starts (16 * h)
    int img1, img2;       // this wave's half image of F1 / F2 (0 or 1) for the MFMAs
    int o1, o2;           // this wave's first column inside its half image
};

// DMA share of wave w per stage: half image w >> 1 (F1 half 0, F1 half 1,
// F2 half 0, F2 half 1), blocks 4(w & 1) .. +3 (rows 8(w & 1) .. +7).
template <int MODE>
__device__ __forceinline__ void s8_issue(const Sp8Ctx &c, char *smem, int st) {
    typedef __attribute__((address_space(3))) void lds_void;
    char *dst = smem + (st % kSpSL) * kS8Slot + (c.wave >> 1) * kS8Img;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int blk = 4 * (c.wave & 1) + k;         // rows 2 blk, 2 blk + 1
        const int d = st * kSpBK + 2 * blk + (c.lane >> 5);
        const int w = 4 * (c.lane & 31);
        const long long base = (long long)(d < c.D ? d : 0) * c.H + c.h;
        const uint32_t off = d < c.D && w < c.dhw ? (uint32_t)((base * c.dW + c.dorg + w) * 4) : 0xFFFFFF00u;
        if constexpr (!(MODE & kModeNoLoads))
            __builtin_amdgcn_raw_ptr_buffer_load_lds(c.rd, (lds_void *)(dst + blk * kSpBlk), 16, (int)off, 0, 0, 0);
    }
}

template <int FA, int FB, int MODE, int NLM>
__device__ __forceinline__ void split8_body(const Sp8Ctx &c, const BuildArgs &a, char *smem, int row) {
    const int lane = c.lane, i = lane & 15, g = lane >> 4;
    const int lrow = (g & 1) * 4 * kSpBlk;             // rows 8(g&1): 4 blocks in
    f32x4 acc[FA > 0 ? FA : 1][4];
#pragma unroll
    for (int x0 = 0; x0 < (FA > 0 ? FA : 1); ++x0)
#pragma unroll
        for (int y0 = 0; y0 < 4; ++y0) acc[x0][y0] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nks = (c.nst + 1) >> 1;
#pragma unroll
    for (int st = 0; st < 4; ++st)
        if (st < c.nst) s8_issue<MODE>(c, smem, st);
    for (int ks = 0; ks < nks; ++ks) {
        // as split_body: my 4 DMA instructions per stage of K step ks landed
        // (8 of K step 1 may still fly at ks = 0); my reads of ks - 1 done
        if (ks == 0 && nks > 1) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (ks >= 1 && 2 * ks + 2 < c.nst) {
            s8_issue<MODE>(c, smem, 2 * ks + 2);
            s8_issue<MODE>(c, smem, 2 * ks + 3);
        }
        if constexpr (FA > 0 && !(MODE & kModeNoMath)) {
            const char *st = smem + ((2 * ks + (g >> 1)) % kSpSL) * kS8Slot + lrow;
            const char *pb = st + c.img1 * kS8Img + 4 * (c.o1 + i);              // F1 (B)
            const char *pa = st + (2 + c.img2) * kS8Img + 4 * (c.o2 + i);        // F2 (A)
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
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if constexpr (FA > 0) {
        const int m0 = c.M0 + c.img1 * c.ho1 + c.o1, n0 = c.N0 + c.img2 * c.ho2 + c.o2;
        epilogue_swapped<FA, (MODE & kModeGenericEpi) ? MODE : (MODE | kModeFastEpi), NLM>(
            acc, a, row, m0, n0, lane, lds_u32(smem + c.wave * kS8Stb), m0 + 16 * FB);
    }
}

// The launcher takes this kernel only for tiles of >= 9 fragments along both
// w1 and w2 (W >= 129), where every wave holds 4..8 F2 and 2..4 F1
// fragments; the rest (and a wave past the image edge) runs the empty body.
template <int FA, int MODE, int NLM>
__device__ __forceinline__ void split8_fb(int fb, const Sp8Ctx &c, const BuildArgs &a, char *smem, int row) {
    if (fb == 4) split8_body<FA, 4, MODE, NLM>(c, a, smem, row);
    else if (fb == 3) split8_body<FA, 3, MODE, NLM>(c, a, smem, row);
    else if (fb == 2) split8_body<FA, 2, MODE, NLM>(c, a, smem, row);
    else split8_body<0, 1, MODE, NLM>(c, a, smem, row);
}

template <int MODE, int NLM>
__global__ __launch_bounds__(512, 1) void build_split8_kernel(BuildArgs a, int nwg_total, int tf1, int tf2,
                                                               int tiles1, int tiles2) {
    __shared__ __attribute__((aligned(16))) char smem[kSpSL * kS8Slot];
    Sp8Ctx c;
    c.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    c.lane = threadIdx.x & 63;
    const int T = tiles1 * tiles2;
    const int wgid = xcd_remap(blockIdx.x, nwg_total);
    const int row = wgid / T, tile = wgid - row * T;
    const int tm = tile / tiles2, tn = tile - tm * tiles2;
    const int b = row / a.H;
    c.h = row - b * a.H;
    c.D = a.D; c.H = a.H;
    c.M0 = tm * 16 * tf1; c.N0 = tn * 16 * tf2;
    const int h1 = (tf1 + 1) >> 1, h2 = (tf2 + 1) >> 1;   // fragments of half 0
    c.ho1 = 16 * h1; c.ho2 = 16 * h2;
    {
        const bool f2 = c.wave >= 4;                      // wave-uniform
        const int half = (c.wave >> 1) & 1, hf = f2 ? h2 : h1, tf = f2 ? tf2 : tf1;
        c.dW = f2 ? a.W2 : a.W1;
        c.dorg = (f2 ? c.N0 : c.M0) + 16 * hf * half;
        c.dhw = 16 * (half ? tf - hf : hf);
    }
    // wave w: F1 quarter q = w & 3 (half q >> 1, ceil / floor split of that
    // half between its two waves), F2 half w >> 2 (all of it)
    const int q = c.wave & 3;
    c.img1 = q >> 1;
    c.img2 = c.wave >> 2;
    const int hf1 = c.img1 ? tf1 - h1 : h1;               // fragments of this F1 half
    const int qa = (hf1 + 1) >> 1;
    c.o1 = (q & 1) ? 16 * qa : 0;
    const int n1 = (q & 1) ? hf1 - qa : qa;
    const int n2 = c.img2 ? tf2 - h2 : h2;
    c.o2 = 0;
    c.nst = 2 * ((a.D + 2 * kSpBK - 1) / (2 * kSpBK));
    {
        const long long imgsz = (long long)a.D * a.H * c.dW;
        const float *src = reinterpret_cast<const float *>(c.wave >= 4 ? a.f2 : a.f1) + b * imgsz;
        c.rd = make_rsrc(src, clamp_bytes(imgsz * 4));
    }
    const int cw1 = a.W1 - (c.M0 + c.img1 * c.ho1 + c.o1), cw2 = a.W2 - (c.N0 + c.img2 * c.ho2);
    const int v1 = cw1 <= 0 ? 0 : min(n1, (cw1 + 15) >> 4), v2 = cw2 <= 0 ? 0 : min(n2, (cw2 + 15) >> 4);
    const int fa = v1 == 0 ? 0 : v2, fb = v1;
    switch (fa) {
        case 8: split8_fb<8, MODE, NLM>(fb, c, a, smem, row); break;
        case 7: split8_fb<7, MODE, NLM>(fb, c, a, smem, row); break;
        case 6: split8_fb<6, MODE, NLM>(fb, c, a, smem, row); break;
        case 5: split8_fb<5, MODE, NLM>(fb, c, a, smem, row); break;
        case 4: split8_fb<4, MODE, NLM>(fb, c, a, smem, row); break;
        default: split8_body<0, 1, MODE, NLM>(c, a, smem, row);
    }
}

}  // namespace rc
#endif  // RAFTCORR_DEV

// Launches the 8-wave kernel when it applies (tiles of >= 9 fragments along
// both widths, i.e. W1, W2 >= 129, and the launcher's choice); otherwise
// returns hipErrorNotSupported and launches nothing.
hipError_t rc_launch_build_split8(const rc::BuildArgs &a, hipStream_t s) {
#ifndef RAFTCORR_DEV
    (void)a;
    (void)s;
    return hipErrorNotSupported;
#else
    // 8-wave kernel: tiles of up to 16 x 16 fragments, balanced like the
    // 4-wave kernel's (W = 240: one 15-fragment tile; W = 720: three)
    auto tile16 = [](int W) {
        const int nf = (W + 15) / 16, nt = (nf + 15) / 16;
        return (nf + nt - 1) / nt;
    };
    const int tg1 = tile16(a.W1), tg2 = tile16(a.W2);
    const int tl1 = ((a.W1 + 15) / 16 + tg1 - 1) / tg1, tl2 = ((a.W2 + 15) / 16 + tg2 - 1) / tg2;
    const long long nwg8 = (long long)a.B * a.H * tl1 * tl2;
    const bool fits8 = tg1 >= 9 && tg2 >= 9 && nwg8 <= 0x7FFFFFFF;
    bool use8 = false;
#ifdef RAFTCORR_DEV
    {
        const int kk = rc::dev_knob("RAFTCORR_SPLIT_KERNEL");
        if (kk == 8) use8 = fits8;
        if (kk == 4) use8 = false;
    }
#endif
    if (use8) {
        const int m = 0
#ifdef RAFTCORR_DEV
            + rc::dev_knob("RAFTCORR_SPLIT_MODE")
#endif
            ;
#define RC_S8(MM) hipLaunchKernelGGL((rc::build_split8_kernel<MM, 3>), dim3((unsigned)nwg8), dim3(512), 0, s, a, (int)nwg8, tg1, tg2, tl1, tl2)
        switch (m) {
#ifdef RAFTCORR_DEV
            case 3: RC_S8(3); break;
            case 6: RC_S8(6); break;
            case 8192: RC_S8(8192); break;
#endif
            default:
                if (a.nfused <= 3) RC_S8(0);
                else hipLaunchKernelGGL((rc::build_split8_kernel<0, rc::kSpMaxFused>), dim3((unsigned)nwg8), dim3(512), 0, s,
                                        a, (int)nwg8, tg1, tg2, tl1, tl2);
        }
#undef RC_S8
        return hipGetLastError();
    }
    return hipErrorNotSupported;
#endif
}
