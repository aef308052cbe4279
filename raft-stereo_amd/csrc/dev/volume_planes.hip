// DEV ONLY (libraftcorr_dev.so, RAFTCORR_SPLIT_RING=100): measured and not
// kept -- config 2 340.7 vs 263.5 us with one K step prefetched, 450.7 us
// with two (256 VGPRs, 35 spilled); DESIGN.md §3.1c.
// fp32 correlation volume on bf16 MFMA, split ONCE per workgroup (gfx950):
// the "planes" variant of build_split_kernel (volume_split.hip).
//
// Replaces CorrBlock1D.corr (/root/reference/model.py:318-326) and the
// avg_pool2d loop of CorrBlock1D.__init__ (:284-295) with the same tiles,
// waves, fragments, three-way split and MFMA order as build_split_kernel, so
// the same bits (tests/test_split_gpu.py).  What differs is where the split
// runs: there, every wave splits the fp32 fragments it reads, so each operand
// element is split by the two waves that share it, on the MFMAs' critical
// path; here each element is split once, by one thread, into bf16 planes in
// LDS that the waves then read straight into the MFMAs.
#include "../common.h"
#include "../epilogue.h"
#include "../split.h"
#include "../split_ring.h"

namespace rc {

struct PlCtx {
    int H, h, W1, W2, M0, N0, wave, lane;
    int tw1, tw2;      // tile extent (w) along w1 / w2: 16 x fragments, <= 128
    int o1, o2;        // this wave's first column (w) inside the tile, w1 / w2
};

// ---------------------------------------------------------------------------
// Split once per workgroup: the "planes" kernel.  The same tiles, waves,
// fragments, split and MFMA order as build_split_kernel (so the same bits),
// but every fp32 operand element is split ONCE per workgroup instead of once
// per wave that reads it (twice): thread t loads column t & 127 of operand
// t >> 7 (F1, F2) for the 32 d of a K step into VGPRs (coalesced 256-B rows,
// prefetched one K step ahead), splits it and writes its h / m / l bf16
// pieces into three LDS planes per operand, [w][32 d] rows of 64 B whose four
// 16-B chunks are XOR-swizzled by (w >> 1) & 3 -- conflict-free for both the
// 8-lane ds_write_b128 groups (consecutive w) and the fragment ds_read_b128
// groups (lane (i, g): chunk g of row w0 + i).  Waves then feed the MFMAs
// straight from the planes: no split on the MFMA critical path.
constexpr int kPlRow = 64;                       // bytes per plane row: 32 d bf16
constexpr int kPlPlane = 128 * kPlRow;           // one piece of one operand: 128 w
constexpr int kPlBytes = 6 * kPlPlane;           // 2 operands x 3 pieces = 48 KB
static_assert(4 * kSpStb <= kPlBytes, "epilogue staging aliases the planes");

__device__ __forceinline__ int pl_chunk(int w, int k) { return (k ^ ((w >> 1) & 3)) * 16; }

// raw barrier: waits for this wave's LDS traffic only, so the operand loads
// prefetched into VGPRs stay in flight across it (__syncthreads() would add
// a vmcnt(0) and drain them -- cdna_hip_programming.md "Pipelining across
// barriers"; round 6's first measurement of this kernel used it)
__device__ __forceinline__ void pl_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

template <int FA, int FB, int MODE, int NLM, int DEPTH>
__device__ __forceinline__ void planes_body(const PlCtx &c, const BuildArgs &a, char *smem, int row,
                                            __amdgpu_buffer_rsrc_t rs, uint32_t off0, uint32_t rstep, int nks) {
    const int t = threadIdx.x, lane = c.lane, i = lane & 15, g = lane >> 4;
    const int op = t >> 7, wcol = t & 127;
    f32x4 acc[FA > 0 ? FA : 1][4];
#pragma unroll
    for (int x0 = 0; x0 < (FA > 0 ? FA : 1); ++x0)
#pragma unroll
        for (int y0 = 0; y0 < 4; ++y0) acc[x0][y0] = f32x4{0.f, 0.f, 0.f, 0.f};
    // this thread's plane rows (one per piece) and the fragment read offsets
    char *prow = smem + op * 3 * kPlPlane + wcol * kPlRow;
    const int rchunk = pl_chunk(i, g);             // w0 + i with 16 | w0: the swizzle of i
    const char *pb = smem + (c.o1 + i) * kPlRow + rchunk;                  // F1 (B), piece h
    const char *pa = smem + 3 * kPlPlane + (c.o2 + i) * kPlRow + rchunk;   // F2 (A), piece h
    // DEPTH K steps of operand columns in flight (32 VGPRs each): a K step's
    // loads are issued DEPTH MFMA phases before its split reads them
    float xa[32], xb[DEPTH > 1 ? 32 : 1];
    auto load = [&](float (&x)[32], int ks) {
        uint32_t o = off0 + (uint32_t)(32 * ks) * rstep;
#pragma unroll
        for (int j = 0; j < 32; ++j, o += rstep) x[j] = ld1(rs, o);
    };
    auto kstep = [&](float (&x)[32], int ks) {
        // split the landed K step into the planes (the previous K step's
        // fragment reads finished at the barrier that ended it)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = x[8 * k + j];
            const SplitFrag s = sp_split(v);
            const int ch = pl_chunk(wcol, k);
            *reinterpret_cast<bf16x8 *>(prow + ch) = s.h;
            *reinterpret_cast<bf16x8 *>(prow + kPlPlane + ch) = s.m;
            *reinterpret_cast<bf16x8 *>(prow + 2 * kPlPlane + ch) = s.l;
        }
        if (ks + DEPTH < nks) load(x, ks + DEPTH);
        pl_barrier();
        if constexpr (FA > 0 && !(MODE & kModeNoMath)) {
            SplitFrag fb[FB];
#pragma unroll
            for (int n = 0; n < FB; ++n) {
                const char *p = pb + n * 16 * kPlRow;
                fb[n] = SplitFrag{*reinterpret_cast<const bf16x8 *>(p),
                                  *reinterpret_cast<const bf16x8 *>(p + kPlPlane),
                                  *reinterpret_cast<const bf16x8 *>(p + 2 * kPlPlane)};
            }
#pragma unroll
            for (int m = 0; m < FA; ++m) {
                const char *p = pa + m * 16 * kPlRow;
                const SplitFrag fa{*reinterpret_cast<const bf16x8 *>(p),
                                   *reinterpret_cast<const bf16x8 *>(p + kPlPlane),
                                   *reinterpret_cast<const bf16x8 *>(p + 2 * kPlPlane)};
#pragma unroll
                for (int n = 0; n < FB; ++n) sp_mma6(acc[m][n], fa, fb[n]);
            }
        }
        pl_barrier();
    };
    load(xa, 0);
    if constexpr (DEPTH > 1) {
        if (nks > 1) load(xb, 1);
        for (int ks = 0; ks < nks; ks += 2) {
            kstep(xa, ks);
            if (ks + 1 < nks) kstep(xb, ks + 1);
        }
    } else {
        for (int ks = 0; ks < nks; ++ks) kstep(xa, ks);
    }
    if constexpr (FA > 0) {
        epilogue_swapped<FA, (MODE & kModeGenericEpi) ? MODE : (MODE | kModeFastEpi), NLM>(
            acc, a, row, c.M0 + c.o1, c.N0 + c.o2, lane, lds_u32(smem + c.wave * (kPlBytes / 4)),
            c.M0 + c.o1 + 16 * FB);
    }
}

template <int FA, int MODE, int NLM, int DEPTH>
__device__ __forceinline__ void planes_fb(int fb, const PlCtx &c, const BuildArgs &a, char *smem, int row,
                                          __amdgpu_buffer_rsrc_t rs, uint32_t off0, uint32_t rstep, int nks) {
    if (fb >= 4) planes_body<FA, 4, MODE, NLM, DEPTH>(c, a, smem, row, rs, off0, rstep, nks);
    else if (fb == 3) planes_body<FA, 3, MODE, NLM, DEPTH>(c, a, smem, row, rs, off0, rstep, nks);
    else if (fb == 2) planes_body<FA, 2, MODE, NLM, DEPTH>(c, a, smem, row, rs, off0, rstep, nks);
    else planes_body<FA, 1, MODE, NLM, DEPTH>(c, a, smem, row, rs, off0, rstep, nks);
}

template <int MODE, int NLM, int DEPTH>
__global__ __launch_bounds__(256, 2) void build_split_planes_kernel(BuildArgs a, int nwg_total, int tf1, int tf2,
                                                                    int tiles1, int tiles2) {
    __shared__ __attribute__((aligned(16))) char smem[kPlBytes];
    PlCtx c;
    c.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    c.lane = threadIdx.x & 63;
    const int T = tiles1 * tiles2;
    const int wgid = xcd_remap(blockIdx.x, nwg_total);
    const int row = wgid / T, tile = wgid - row * T;
    const int tm = tile / tiles2, tn = tile - tm * tiles2;
    const int b = row / a.H;
    c.h = row - b * a.H;
    c.H = a.H; c.W1 = a.W1; c.W2 = a.W2;
    c.M0 = tm * 16 * tf1; c.N0 = tn * 16 * tf2;
    c.tw1 = 16 * tf1; c.tw2 = 16 * tf2;
    const int wm = c.wave & 1, wn = c.wave >> 1;
    const int h1 = (tf1 + 1) >> 1, h2 = (tf2 + 1) >> 1;
    c.o1 = 16 * h1 * wm; c.o2 = 16 * h2 * wn;
    const int nks = (a.D + 31) >> 5;
    // this thread's operand column: F1 for threads 0-127, F2 for 128-255;
    // columns past the tile read zeros (out-of-range offset), d >= D reads
    // zeros (past the image)
    const int op = threadIdx.x >> 7, wcol = threadIdx.x & 127;
    const int W = op ? a.W2 : a.W1, X0 = op ? c.N0 : c.M0, tw = op ? c.tw2 : c.tw1;
    const long long img = (long long)a.D * a.H * W;
    const __amdgpu_buffer_rsrc_t rs =
        make_rsrc(reinterpret_cast<const float *>(op ? a.f2 : a.f1) + b * img, clamp_bytes(img * 4));
    const uint32_t off0 = wcol < tw ? (uint32_t)(((long long)c.h * W + X0 + wcol) * 4) : 0xFFFFFF00u;
    const uint32_t rstep = wcol < tw ? (uint32_t)a.H * (uint32_t)W * 4u : 0u;
    const int n1 = wm ? tf1 - h1 : h1, n2 = wn ? tf2 - h2 : h2;
    const int cw1 = a.W1 - (c.M0 + c.o1), cw2 = a.W2 - (c.N0 + c.o2);
    const int v1 = cw1 <= 0 ? 0 : min(n1, (cw1 + 15) >> 4), v2 = cw2 <= 0 ? 0 : min(n2, (cw2 + 15) >> 4);
    const int fa = v1 == 0 ? 0 : v2, fb = v1;
    if (fa >= 4) planes_fb<4, MODE, NLM, DEPTH>(fb, c, a, smem, row, rs, off0, rstep, nks);
    else if (fa == 3) planes_fb<3, MODE, NLM, DEPTH>(fb, c, a, smem, row, rs, off0, rstep, nks);
    else if (fa == 2) planes_fb<2, MODE, NLM, DEPTH>(fb, c, a, smem, row, rs, off0, rstep, nks);
    else if (fa == 1) planes_fb<1, MODE, NLM, DEPTH>(fb, c, a, smem, row, rs, off0, rstep, nks);
    else planes_body<0, 1, MODE, NLM, DEPTH>(c, a, smem, row, rs, off0, rstep, nks);
}



// ---------------------------------------------------------------------------
// planes8 (RAFTCORR_SPLIT_RING=102): the same split-once planes, double
// buffered (2 x 48 KB: one workgroup of 8 waves per CU, two waves per SIMD)
// so that each wave's split of K step ks + 1 runs between its MFMAs of K step
// ks -- one barrier per K step, the split VALU in the MFMAs' issue gaps.
// Tiles stay 128 (w1) x 128 (w2); the 8 waves are 4 (w1, 32 each) x 2 (w2,
// 64 each), so a wave holds FA <= 4 A (w2) and FB <= 2 B (w1) fragments and
// the epilogue is epilogue_swapped's (4 consecutive w2 per lane).  Thread t
// splits column t & 255 (F1: 0-127, F2: 128-255) for d half t >> 8 of each K
// step: 16 elements, two 16-B chunks per piece.
constexpr int kP8Bytes = 2 * kPlBytes;           // 96 KB

template <int FA, int FB, int MODE, int NLM>
__device__ __forceinline__ void planes8_body(const PlCtx &c, const BuildArgs &a, char *smem, int row,
                                             __amdgpu_buffer_rsrc_t rs, uint32_t off0, uint32_t rstep, int nks) {
    const int t = threadIdx.x, lane = c.lane, i = lane & 15, g = lane >> 4;
    const int col = t & 255, op = col >> 7, wcol = col & 127, dh = t >> 8;
    f32x4 acc[FA > 0 ? FA : 1][4];
#pragma unroll
    for (int x0 = 0; x0 < (FA > 0 ? FA : 1); ++x0)
#pragma unroll
        for (int y0 = 0; y0 < 4; ++y0) acc[x0][y0] = f32x4{0.f, 0.f, 0.f, 0.f};
    char *prow = smem + op * 3 * kPlPlane + wcol * kPlRow;
    const int rchunk = pl_chunk(i, g);
    const char *pb = smem + (c.o1 + i) * kPlRow + rchunk;                  // F1 (B)
    const char *pa = smem + 3 * kPlPlane + (c.o2 + i) * kPlRow + rchunk;   // F2 (A)
    // row j of a 16-d half: the scalar offset j * rstep (no per-load VALU);
    // the vector offset steps by 32 rows per K step.  K steps past D read
    // past the image: zeros, no memory traffic, and never multiplied
    const uint32_t ovec = off0 + 16u * (uint32_t)dh * rstep;
    const uint32_t kstep = 32u * rstep;
    float xa[16], xb[16];
    auto load = [&](float (&x)[16], int ks) {
        const uint32_t o = ovec + (uint32_t)ks * kstep;
#pragma unroll
        for (int j = 0; j < 16; ++j)
            x[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, (int)o, (int)(j * rstep), 0));
    };
    auto split = [&](const float (&x)[16], int buf) {
        char *p = prow + buf * kPlBytes;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = x[8 * k + j];
            const SplitFrag sf = sp_split(v);
            const int ch = pl_chunk(wcol, 2 * dh + k);
            *reinterpret_cast<bf16x8 *>(p + ch) = sf.h;
            *reinterpret_cast<bf16x8 *>(p + kPlPlane + ch) = sf.m;
            *reinterpret_cast<bf16x8 *>(p + 2 * kPlPlane + ch) = sf.l;
        }
    };
    auto mma = [&](int buf) {
        if constexpr (FA > 0 && !(MODE & kModeNoMath)) {
            const char *qb = pb + buf * kPlBytes, *qa = pa + buf * kPlBytes;
            SplitFrag fb[FB], fa[FA];
#pragma unroll
            for (int n = 0; n < FB; ++n) {
                const char *p = qb + n * 16 * kPlRow;
                fb[n] = SplitFrag{*reinterpret_cast<const bf16x8 *>(p),
                                  *reinterpret_cast<const bf16x8 *>(p + kPlPlane),
                                  *reinterpret_cast<const bf16x8 *>(p + 2 * kPlPlane)};
            }
#pragma unroll
            for (int m = 0; m < FA; ++m) {
                const char *p = qa + m * 16 * kPlRow;
                fa[m] = SplitFrag{*reinterpret_cast<const bf16x8 *>(p),
                                  *reinterpret_cast<const bf16x8 *>(p + kPlPlane),
                                  *reinterpret_cast<const bf16x8 *>(p + 2 * kPlPlane)};
            }
#pragma unroll
            for (int m = 0; m < FA; ++m)
#pragma unroll
                for (int n = 0; n < FB; ++n) sp_mma6(acc[m][n], fa[m], fb[n]);
        }
    };
    // one K step: its MFMAs from planes buffer B while this thread splits the
    // next K step's columns (registers x) into the other buffer and reloads x
    // with the K step after that -- one scheduling region, the split's VALU
    // placed two per MFMA (sched_group_barrier): fragment reads, then
    // (1 MFMA, 2 VALU) x n, then the plane writes and the loads
    auto step = [&](int B, float (&x)[16], int ks) {
        mma(B);
        split(x, B ^ 1);
        load(x, ks + 3);
        if constexpr (FA > 0 && !(MODE & kModeNoMath)) {
            constexpr int NM = 6 * FA * FB;
            __builtin_amdgcn_sched_group_barrier(0x100, 3 * (FA + FB), 0);   // DS reads
#pragma unroll
            for (int q = 0; q < NM; ++q) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);           // MFMA
                __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);           // VALU
            }
            __builtin_amdgcn_sched_group_barrier(0x200, 6, 0);               // DS writes
            __builtin_amdgcn_sched_group_barrier(0x020, 16, 0);              // VMEM reads
        }
    };
    // K step s: registers xa (s even) / xb (s odd), planes buffer s & 1;
    // loaded right after the split of K step s - 2 freed the registers
    load(xa, 0);
    load(xb, 1);
    split(xa, 0);
    load(xa, 2);
    pl_barrier();
    // nks is even (the kernel pads it: an odd count's last K step reads zeros)
    for (int ks = 0; ks < nks; ks += 2) {
        step(0, xb, ks);              // MFMAs of ks (buffer 0), split ks + 1, load ks + 3
        pl_barrier();
        step(1, xa, ks + 1);          // MFMAs of ks + 1 (buffer 1), split ks + 2, load ks + 4
        pl_barrier();
    }
    if constexpr (FA > 0) {
        epilogue_swapped<FA, (MODE & kModeGenericEpi) ? MODE : (MODE | kModeFastEpi), NLM>(
            acc, a, row, c.M0 + c.o1, c.N0 + c.o2, lane, lds_u32(smem + c.wave * (kP8Bytes / 8)),
            c.M0 + c.o1 + 16 * FB);
    }
}

template <int FA, int MODE, int NLM>
__device__ __forceinline__ void planes8_fb(int fb, const PlCtx &c, const BuildArgs &a, char *smem, int row,
                                           __amdgpu_buffer_rsrc_t rs, uint32_t off0, uint32_t rstep, int nks) {
    if (fb >= 2) planes8_body<FA, 2, MODE, NLM>(c, a, smem, row, rs, off0, rstep, nks);
    else planes8_body<FA, 1, MODE, NLM>(c, a, smem, row, rs, off0, rstep, nks);
}

template <int MODE, int NLM>
__global__ __launch_bounds__(512, 1) void build_split_planes8_kernel(BuildArgs a, int nwg_total, int tf1, int tf2,
                                                                     int tiles1, int tiles2) {
    __shared__ __attribute__((aligned(16))) char smem[kP8Bytes];
    PlCtx c;
    c.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    c.lane = threadIdx.x & 63;
    const int T = tiles1 * tiles2;
    const int wgid = xcd_remap(blockIdx.x, nwg_total);
    const int row = wgid / T, tile = wgid - row * T;
    const int tm = tile / tiles2, tn = tile - tm * tiles2;
    const int b = row / a.H;
    c.h = row - b * a.H;
    c.H = a.H; c.W1 = a.W1; c.W2 = a.W2;
    c.M0 = tm * 16 * tf1; c.N0 = tn * 16 * tf2;
    c.tw1 = 16 * tf1; c.tw2 = 16 * tf2;
    const int wm = c.wave & 3, wn = c.wave >> 2;           // 4 along w1 (32 each), 2 along w2 (64 each)
    c.o1 = 32 * wm; c.o2 = 64 * wn;
    const int nks = ((a.D + 63) >> 6) << 1;                  // K steps, padded to even
    const int col = threadIdx.x & 255, op = col >> 7, wcol = col & 127;
    const int W = op ? a.W2 : a.W1, X0 = op ? c.N0 : c.M0, tw = op ? c.tw2 : c.tw1;
    const long long img = (long long)a.D * a.H * W;
    const __amdgpu_buffer_rsrc_t rs =
        make_rsrc(reinterpret_cast<const float *>(op ? a.f2 : a.f1) + b * img, clamp_bytes(img * 4));
    const uint32_t off0 = wcol < tw ? (uint32_t)(((long long)c.h * W + X0 + wcol) * 4) : 0xFFFFFF00u;
    const uint32_t rstep = wcol < tw ? (uint32_t)a.H * (uint32_t)W * 4u : 0u;
    // valid fragments of this wave's block, cut at the tile and the image edge
    const int cw1 = min(c.tw1, a.W1 - c.M0) - c.o1, cw2 = min(c.tw2, a.W2 - c.N0) - c.o2;
    const int v1 = cw1 <= 0 ? 0 : min(2, (cw1 + 15) >> 4), v2 = cw2 <= 0 ? 0 : min(4, (cw2 + 15) >> 4);
    const int fa = v1 == 0 ? 0 : v2, fb = v1;
    if (fa >= 4) planes8_fb<4, MODE, NLM>(fb, c, a, smem, row, rs, off0, rstep, nks);
    else if (fa == 3) planes8_fb<3, MODE, NLM>(fb, c, a, smem, row, rs, off0, rstep, nks);
    else if (fa == 2) planes8_fb<2, MODE, NLM>(fb, c, a, smem, row, rs, off0, rstep, nks);
    else if (fa == 1) planes8_fb<1, MODE, NLM>(fb, c, a, smem, row, rs, off0, rstep, nks);
    else planes8_body<0, 1, MODE, NLM>(c, a, smem, row, rs, off0, rstep, nks);
}
}  // namespace rc

// Planes build for fp32 fmaps and an fp32 pyramid in the row layout, at most
// 3 fused levels; hipErrorNotSupported (nothing launched) otherwise.
hipError_t rc_launch_build_planes(rc::BuildArgs &a, hipStream_t s) {
    const long long img = (long long)(a.D + 31) * a.H * (a.W1 > a.W2 ? a.W1 : a.W2) * 4;
    if (img >= 0xFFFFFF00LL || a.pyr_bf16 || a.W1 % 4 || a.W2 % 4 || a.shk[0] || a.nfused > 3)
        return hipErrorNotSupported;
    auto tile_frags = [](int W) {
        const int nf = (W + 15) / 16, nt = (nf + 7) / 8;
        return (nf + nt - 1) / nt;
    };
    const int tf1 = tile_frags(a.W1), tf2 = tile_frags(a.W2);
    const int tiles1 = ((a.W1 + 15) / 16 + tf1 - 1) / tf1, tiles2 = ((a.W2 + 15) / 16 + tf2 - 1) / tf2;
    const long long nwg = (long long)a.B * a.H * tiles1 * tiles2;
    if (nwg <= 0) return hipSuccess;
    if (nwg > 0x7FFFFFFF) return hipErrorInvalidValue;
    const int ring = rc::dev_knob("RAFTCORR_SPLIT_RING");
    if (ring == 102) {   // planes8: double-buffered planes, 8 waves
        switch (rc::dev_knob("RAFTCORR_PLANES_MODE")) {
#define P8_CASE(M)                                                                                                \
    case M:                                                                                                       \
        hipLaunchKernelGGL((rc::build_split_planes8_kernel<M, 3>), dim3((unsigned)nwg), dim3(512), 0, s, a,       \
                           (int)nwg, tf1, tf2, tiles1, tiles2);                                                   \
        return hipGetLastError();
        P8_CASE(0) P8_CASE(2) P8_CASE(4) P8_CASE(6)
#undef P8_CASE
        default: return hipErrorNotSupported;
        }
    }
    const bool deep = ring == 101;   // two K steps prefetched
    switch (rc::dev_knob("RAFTCORR_PLANES_MODE") + (deep ? 1000 : 0)) {   // ablation flags (epilogue.h kMode*)
#define PL_CASE(M, DP)                                                                                           \
    case M + (DP > 1 ? 1000 : 0):                                                                                \
        hipLaunchKernelGGL((rc::build_split_planes_kernel<M, 3, DP>), dim3((unsigned)nwg), dim3(256), 0, s, a,   \
                           (int)nwg, tf1, tf2, tiles1, tiles2);                                                  \
        return hipGetLastError();
    PL_CASE(0, 1) PL_CASE(2, 1) PL_CASE(4, 1) PL_CASE(6, 1)
    PL_CASE(0, 2) PL_CASE(2, 2) PL_CASE(4, 2) PL_CASE(6, 2)
#undef PL_CASE
    default: return hipErrorNotSupported;
    }
}
