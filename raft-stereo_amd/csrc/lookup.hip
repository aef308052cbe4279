// Radius-r lookup over the correlation pyramid (gfx950).
//
// Replaces CorrBlock1D.__call__ (/root/reference/model.py:297-316) and the
// grid_sample-based bilinear_sampler it calls (:267-281).  For pixel p =
// (b,h,w1), level i and tap t in -r..r the reference samples row p of level i at
//     x_t = t + x/2^i                                          (:305-307)
//     xn  = 2*x_t/(W_i-1) - 1                                  (:271)
//     x'  = (xn + 1) * ((W_i-1)/2)      grid_sample, align_corners=True (:275)
//     x0 = floor(x'), w1 = x' - x0, w0 = 1 - w1
//     out = fma(w1, v(x0+1), w0*v(x0)),  v(k) = 0 outside [0, W_i)   (zeros pad)
// and writes channel i*(2r+1)+t+r of a (B, L(2r+1), H, W1) fp32 tensor
// (:315-316).  The normalise/unnormalise round trip is kept bit-for-bit: it
// moves x' by up to ~1e-4 px at W=720.  The file is built with
// -ffp-contract=off so the only fused op is the explicit fmaf.
//
// Memory: one lane per pixel.  The taps of one level touch at most 2r+4
// consecutive elements [n-r-1, n+r+2] (n = floor(x/2^i)) because the round trip
// moves floor(x') by at most one.  The lane fetches that window with
// ceil((2r+4+3)/4) aligned 16-byte buffer loads (out-of-range -> 0, never a
// fault), shifts it by the 0..3 misalignment with selects, and picks each
// tap's pair with a 3-way select.  A tap whose floor is off by more than one
// (impossible for |x| < 2^22 by the error bound; kept for safety) takes a
// guarded scalar path.  Output stores are coalesced along w1.
#include "common.h"

namespace rc {

template <int R, bool BF16>
__global__ __launch_bounds__(256) void lookup_kernel(LookupArgs a) {
    constexpr int T = 2 * R + 1;
    constexpr int NW = 2 * R + 4;                 // window elements needed
    constexpr int EPV = BF16 ? 8 : 4;             // elements per 16-B load
    constexpr int NV = (NW + EPV - 1 + EPV - 1) / EPV;  // loads incl. misalignment
    constexpr int NE = NV * EPV;

    const long long pblk = (long long)blockIdx.x * 256;
    const long long p = pblk + threadIdx.x;
    const bool active = p < a.P;
    const long long pp = active ? p : a.P - 1;
    const long long bimg = pp / a.HW, rem = pp - bimg * a.HW;
    const float x = a.coords[bimg * a.cbs + rem];
    const int C = a.levels * T;
    float *outp = a.out + bimg * (long long)C * a.HW + rem;
    const long long lrow = pp - pblk;             // row index relative to block base

    for (int i = 0; i < a.levels; ++i) {
        const int W = a.W[i];
        const float Wm1 = (float)(W - 1);
        const float half = Wm1 / 2.0f;
        const float xl = x / (float)(1 << i);
        constexpr int ES = BF16 ? 2 : 4;
        const char *base = reinterpret_cast<const char *>(a.lvl[i]) + pblk * W * ES;
        const auto rs = make_rsrc(base, clamp_bytes((a.P - pblk) * (long long)W * ES));

        // Window start (in elements, relative to the block base).
        const bool inwin = (xl > -(float)(R + 4)) && (xl < (float)(W + R + 4));  // false for NaN
        const float n = inwin ? floorf(xl) : 0.0f;
        const long long e = lrow * W + (long long)n - (R + 1);
        const long long ea = e & ~(long long)(EPV - 1);
        const int sh = (int)(e - ea);

        float v[NE];
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            const uint32_t off = (uint32_t)((ea + (long long)k * EPV) * ES);
            if constexpr (BF16) {
                const auto q = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 0);
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const uint32_t u = q[c];
                    v[k * 8 + 2 * c] = __builtin_bit_cast(float, u << 16);
                    v[k * 8 + 2 * c + 1] = __builtin_bit_cast(float, u & 0xFFFF0000u);
                }
            } else {
                const f32x4 q = ld4(rs, off);
#pragma unroll
                for (int c = 0; c < 4; ++c) v[k * 4 + c] = q[c];
            }
        }
        // s[j] = element (e + j) = v[j + sh]
        float s[NW];
#pragma unroll
        for (int j = 0; j < NW; ++j) {
            float r = v[j];
#pragma unroll
            for (int k = 1; k < EPV; ++k)
                r = (sh == k) ? v[j + k] : r;
            s[j] = r;
        }

#pragma unroll
        for (int t = 0; t < T; ++t) {
            const float xt = (float)(t - R) + xl;
            const float xn = (2.0f * xt) / Wm1 - 1.0f;
            const float xp = (xn + 1.0f) * half;
            const float x0 = floorf(xp);
            const float w1 = xp - x0, w0 = 1.0f - w1;
            const float nt = n + (float)(t - R);
            const bool lo = x0 < nt, hi = x0 > nt;
            float a0 = lo ? s[t] : (hi ? s[t + 2] : s[t + 1]);
            float a1 = lo ? s[t + 1] : (hi ? s[t + 3] : s[t + 2]);
            const bool ok0 = (x0 >= 0.0f) && (x0 <= Wm1);
            const bool ok1 = (x0 + 1.0f >= 0.0f) && (x0 + 1.0f <= Wm1);
            if (__builtin_expect(inwin && (x0 < nt - 1.0f || x0 > nt + 1.0f), 0)) {
                // Guarded scalar fallback (never taken within the error bound).
                const long long k0 = lrow * W + (long long)x0;
                if constexpr (BF16) {
                    const uint16_t *rowp = reinterpret_cast<const uint16_t *>(base);
                    a0 = ok0 ? bf16_to_f32(rowp[k0]) : 0.0f;
                    a1 = ok1 ? bf16_to_f32(rowp[k0 + 1]) : 0.0f;
                } else {
                    const float *rowp = reinterpret_cast<const float *>(base);
                    a0 = ok0 ? rowp[k0] : 0.0f;
                    a1 = ok1 ? rowp[k0 + 1] : 0.0f;
                }
            }
            const float v0 = ok0 ? a0 : 0.0f;
            const float v1 = ok1 ? a1 : 0.0f;
            const float res = fmaf(w1, v1, w0 * v0);
            if (active) outp[(long long)(i * T + t) * a.HW] = res;
        }
    }
}

template <int R>
static hipError_t launch_r(const LookupArgs &a, int bf16, hipStream_t s) {
    const unsigned nblk = (unsigned)((a.P + 255) / 256);
    if (bf16)
        hipLaunchKernelGGL((lookup_kernel<R, true>), dim3(nblk), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL((lookup_kernel<R, false>), dim3(nblk), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace rc

hipError_t rc_launch_lookup(const rc::LookupArgs &a, int radius, int pyr_bf16, hipStream_t s) {
    if (a.P <= 0) return hipSuccess;
    switch (radius) {
        case 1: return rc::launch_r<1>(a, pyr_bf16, s);
        case 2: return rc::launch_r<2>(a, pyr_bf16, s);
        case 3: return rc::launch_r<3>(a, pyr_bf16, s);
        case 4: return rc::launch_r<4>(a, pyr_bf16, s);
        case 5: return rc::launch_r<5>(a, pyr_bf16, s);
        case 6: return rc::launch_r<6>(a, pyr_bf16, s);
        case 7: return rc::launch_r<7>(a, pyr_bf16, s);
        case 8: return rc::launch_r<8>(a, pyr_bf16, s);
        default: return hipErrorInvalidValue;
    }
}
