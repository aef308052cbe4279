// Internal helpers shared by the gfx950 kernels and the C-ABI layer.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifdef RAFTCORR_DEV
#include <stdlib.h>
#endif

namespace rc {

// Dev-only A/B knobs (environment variables read per launch).  They exist
// only in libraftcorr_dev.so (built with -DRAFTCORR_DEV, tools/ablate.py);
// the product library has no knobs, no getenv and no ablation kernels.
#ifdef RAFTCORR_DEV
inline int dev_knob(const char *name) {
    const char *e = getenv(name);
    return e ? atoi(e) : 0;
}
#endif

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int kMaxLevels = 8;

// Correctly rounded a / b for the sampler's normalisation xn = 2x/(W-1) - 1
// (model.py:271), with b = W - 1 a positive integer.  rb = RN(1/b) is computed
// once per level; per tap Markstein's correction q0 = RN(a*rb) (within 1 ulp
// of a/b), r = a - q0*b (exact with fma), q = RN(q0 + r*rb) = RN(a/b)
// (Markstein, IBM J. R&D 34(1), 1990; Muller et al., Handbook of
// Floating-Point Arithmetic, ch. 4) costs 3 VALU ops instead of the ~10-op
// IEEE division sequence with its quarter-rate v_rcp.  tests/test_div_rn.py
// checks it bit for bit against IEEE division on gfx950 for EVERY b in
// [1, 8192] and every fp32 a with 2^-30 <= |a| < 2^15, and for sampled wider
// b.  Outside that a-range a difference could not reach the sampler's output:
// |a| < 2^-30 gives |q| < 2^-25, so xn = q - 1 rounds to -1 either way, and
// |a| > 2(W + R + 2) puts every tap outside the row (zeros).  A NaN/inf
// numerator gives NaN where division gives +-inf; the sampler turns both into
// the same NaN output (W = 1, b = 0, likewise: (xn + 1) * 0 is NaN both ways).
struct DivRN {
    float b, rb;
};
__device__ __forceinline__ DivRN div_prep(float b) { return DivRN{b, 1.0f / b}; }
__device__ __forceinline__ float div_rn(float a, const DivRN &d) {
    const float q0 = a * d.rb;
    const float r = __builtin_fmaf(-q0, d.b, a);
    return __builtin_fmaf(r, d.rb, q0);
}

// XCD-aware bijective block remap: hardware workgroup v runs on XCD v % 8, so
// give XCD x the contiguous logical range [x*q + min(x, n%8), ...) of the n
// blocks: neighbouring logical blocks then share an XCD (and its L2).
__device__ __forceinline__ int xcd_remap(int v, int n) {
    const int xcd = v & 7, q = n >> 3, rr = n & 7;
    return (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (v >> 3);
}

// Raw buffer resource over [base, base + bytes): loads past the end (or at a
// "negative" offset, which wraps to a huge unsigned one) return 0 and never
// fault.  Build it from wave-uniform values only (cdna_hip_programming.md T20).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, (int)bytes,
                                             0x00020000);
}

__device__ __forceinline__ f32x4 ld4(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)byte_off, 0, 0));
}

__device__ __forceinline__ float ld1(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)byte_off, 0, 0));
}

__device__ __forceinline__ uint32_t clamp_bytes(long long n) {
    return n <= 0 ? 0u : (n > 0xFFFFFF00LL ? 0xFFFFFF00u : (uint32_t)n);
}

// bf16 helpers (round-to-nearest-even; NaN stays NaN via the hardware cvt).
__device__ __forceinline__ float bf16_to_f32(uint16_t v) {
    return __builtin_bit_cast(float, (uint32_t)v << 16);
}
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
    __bf16 b = (__bf16)f;
    return __builtin_bit_cast(uint16_t, b);
}
// fp32 value rounded to bf16 precision (RNE), kept in fp32.
__device__ __forceinline__ float round_bf16(float f) { return bf16_to_f32(f32_to_bf16(f)); }

// v / sqrt(D) as the reference's division (model.py:326): a multiply by the
// exact 1/sqrt(D) when D is a power of four (a.pow2), the correctly rounded
// division otherwise.  One wave-uniform branch around the whole group: the
// empty volatile asm keeps the division path a real branch, so the
// power-of-two path never evaluates it (a select per element would).
template <int N, class Args>
__device__ __forceinline__ void apply_scale(float (&v)[N], const Args &a) {
    if (a.pow2) {
#pragma unroll
        for (int k = 0; k < N; ++k) v[k] *= a.scale;
    } else {
        asm volatile("");
#pragma unroll
        for (int k = 0; k < N; ++k) v[k] = v[k] / a.sq;
    }
}

// Kernel parameter blocks (passed by value).
struct BuildArgs {
    const void *f1, *f2;      // [B][D][H][W1], [B][D][H][W2]
    void *lvl[kMaxLevels];    // pyramid outputs
    long long ld[kMaxLevels]; // their row strides (elements, >= W2 >> l)
    int B, D, H, W1, W2;
    int nfused;               // levels written by the epilogue (1..7)
    int tiles_m, tiles_n;     // 128x128 workgroup tiles per (b,h) row
    float scale;              // exact reciprocal of sqrt(D) when pow2 != 0
    float sq;                 // sqrtf(D)
    int pow2;                 // sqrt(D) is a power of two -> multiply is exact
    int pyr_bf16;             // store pyramid as bf16
    int stagger;              // dev-only: first-round stagger unit (s_sleep(127) count)
    // line-phase shadow copies (ABI v5, RC_SHADOW): a stored level l is also
    // written at (char*)lvl[l] + shadow[l] bytes (0 = no copy)
    long long shadow[kMaxLevels];
    // RC_LAYOUT_DISPARITY (ABI v9): levels 0 and 2 disparity-major, shk[l]
    // rows (diagonals) of ld[l] elements per row block; 0 = row layout
    long long shk[kMaxLevels];
    // RC_LAYOUT_RECORDS (ABI v10): levels 0 and 2 as rec_nr 128-B records
    // per pixel row at rec (the bf16 ring build's deferred epilogue)
    void *rec;
    int rec_nr;
};

// RC_LAYOUT_RECORDS geometry (include/raftcorr.h): record r of a pixel row
// holds level-2 elements 4r - 14 .. 4r + 11 in slots 0..25 and level-0
// elements 16r - 26 .. 16r + 11 in slots 26..63 (bf16), so a pixel whose
// level-1 centre floor(x/2) lies in [8r - 8, 8r) finds the spans of all four
// levels (radius <= 4) in that one line.
constexpr int kRecSlots = 64, kRecL2Slots = 26;
constexpr int kRecM0 = -8;                       // level-1 centre of record 0's first pixel
__host__ __device__ constexpr int rec_e0(int r) { return 16 * r + 2 * kRecM0 - 10; }   // first level-0 element
__host__ __device__ constexpr int rec_e2(int r) { return 4 * r + kRecM0 / 2 - 10; }    // first level-2 element

struct LookupArgs {
    const void *lvl[kMaxLevels];
    int W[kMaxLevels];
    long long ld[kMaxLevels]; // row strides (elements, >= W)
    const float *coords;
    long long cbs;            // coords batch stride (elements)
    float *out;
    long long P;              // B*H*W1
    int HW;                   // H*W1
    int levels;
    // rc_corr_lookup_step only (step != 0): coords is the whole (B,2,H,W1)
    // coords1; x = coords1.x + delta.x (delta may be null), and the advanced
    // coords and flow = coords - coords_grid are written before the lookup
    int step;
    int W1;
    const float *delta;
    float *coords_out;
    float *flow_out;
    // line-phase shadow copy of level i at (char*)lvl[i] + shadow[i] bytes
    // (0 = none); read by the pair kernel (RC_SHADOW, ABI v5)
    long long shadow[kMaxLevels];
    int out_cl;               // channels-last output out[p*C + ch] (pair kernel; ABI v5)
    // RC_LAYOUT_DISPARITY (ABI v9): levels 0 and 2 disparity-major, shk[l]
    // rows (diagonals) of ld[l] elements per row block; 0 = row layout
    long long shk[kMaxLevels];
    // RC_LAYOUT_RECORDS (ABI v10): lvl[0] = the records, rec_nr per pixel row
    int rec_nr;
};

// Backward of the lookup: level gradients (fp32, row stride ld[i] % 4 == 0).
struct LookupBwdArgs {
    float *g[kMaxLevels];
    int W[kMaxLevels];
    long long ld[kMaxLevels];
    const float *coords;
    long long cbs;
    const float *grad_out;    // [B][levels*(2r+1)][H][W1]
    long long P;
    int HW;
    int levels;
    long long shadow[kMaxLevels];   // bytes from g[l] to its RC_SHADOW copy (pair layout), 0 = none
};

// Deferred lookup backward (backward_calls.hip): the gradients of up to
// kMaxBwdCalls lookup calls summed into pair-layout buffers in one pass.
constexpr int kMaxBwdCalls = 32;
struct LookupBwdCallsArgs {
    float *g[2];              // level 0 and level 2 gradient rows (pair layout)
    long long ld[2];          // their row strides (floats, % 4 == 0)
    int W[4];                 // level widths W0 >> l
    int wout[2];              // columns written back per row (round4(W), <= ld)
    int rowbase[2];           // LDS float offset of row 0, element 0, of pair k
    int S[2];                 // LDS row stride (floats) of pair k
    int lds_floats;           // LDS floats zeroed per workgroup (% 4 == 0)
    int pix;                  // pixels per workgroup
    int ncalls;               // 1..kMaxBwdCalls
    int accumulate;           // 0: overwrite the rows; 1: add to them
    int budget;               // compact kernel: LDS floats per block (one wave)
    long long P;
    int HW;
    const float *coords[kMaxBwdCalls];
    long long cbs[kMaxBwdCalls];
    const float *grad_out[kMaxBwdCalls];   // [B][levels*(2r+1)][H][W1]
};

// Backward of the build: level gradients -> feature-map gradients (fp32).
struct BuildBwdArgs {
    const float *f1, *f2;     // [B][D][H][W1], [B][D][H][W2]
    const float *g[kMaxLevels];
    long long ld[kMaxLevels]; // level-gradient row strides (ld[0] % 4 == 0)
    int Wl[kMaxLevels];       // level widths W2 >> l
    int nlev;
    float *df1, *df2;         // outputs, layouts of f1 / f2
    int B, D, H, W1, W2;
    int tm, tn1, tn2;         // 128-row d tiles; 128-col tiles over W1 (dF1) / W2 (dF2)
    float scale, sq;
    int pow2;
    long long shadow[kMaxLevels];   // floats from g[l] to its RC_SHADOW copy (kPairFold), 0 = none
    int exact;                      // 1: exact fp32 MFMA kernel (RC_BUILD_EXACT_F32); 0: split-bf16
    int dev_only;                   // dev library timing probe: 1 = dF1 tiles only, 2 = dF2 only
};

}  // namespace rc

// Host-side launchers (defined in the .hip files, called by capi.cpp).
hipError_t rc_launch_build_f32(const rc::BuildArgs &a, hipStream_t s);
hipError_t rc_launch_build_split(rc::BuildArgs &a, hipStream_t s);     // may lower a.nfused
hipError_t rc_launch_build_planes(rc::BuildArgs &a, hipStream_t s);   // dev library only
hipError_t rc_launch_build_bf16mma(rc::BuildArgs &a, int in_bf16, hipStream_t s);   // may lower a.nfused
hipError_t rc_launch_pool(const void *in, long long ld_in, void *out, long long ld_out, long rows,
                          int W_in, int bf16, hipStream_t s);
hipError_t rc_launch_lookup(const rc::LookupArgs &a, int radius, int pyr_bf16, hipStream_t s);
hipError_t rc_launch_lookup_conv(const rc::LookupArgs &a, int radius, int pyr_bf16, const float *w,
                                 const float *b, int cout, int relu, float *out, hipStream_t s);
hipError_t rc_launch_lookup_chain(const rc::LookupArgs &a, int radius, hipStream_t s);
hipError_t rc_launch_lookup_pair(const rc::LookupArgs &a, int radius, int pyr_bf16, hipStream_t s);
hipError_t rc_launch_lookup_bwd(const rc::LookupBwdArgs &a, int radius, hipStream_t s);
// fills a.pix / rowbase / S / lds_floats from W, radius, levels
hipError_t rc_launch_lookup_bwd_calls(rc::LookupBwdCallsArgs &a, int radius, int levels, hipStream_t s);
bool rc_lookup_bwd_calls_fits(const rc::LookupBwdCallsArgs &a, int radius, int levels, const long *cbs,
                              int n_calls);
hipError_t rc_launch_volume_bwd(const rc::BuildBwdArgs &a, hipStream_t s);
hipError_t rc_launch_convex_upsample(const float *flow, const float *mask, int N, int C, int H,
                                     int W, int factor, float *out, hipStream_t s);
