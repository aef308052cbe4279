// Lookup over a disparity-major ("sheared") pyramid (gfx950) -- prototype.
//
// Same arithmetic as lookup.hip (CorrBlock1D.__call__, model.py:297-316 and
// bilinear_sampler :267-281); only the storage order of the pyramid differs.
// Level i of row block (b,h) is a [K_i][ldw] array
//     S_i[k][w1] = C_i[(b,h,w1)][j],   k = (w1 >> i) - j + (W_i - 1),
//     K_i = W_i + ((W1 - 1) >> i),
// so pixels of one image row that look at the same disparity read one
// contiguous run of S_i: a wave of 64 consecutive w1 fetches 256 B per element
// of its window instead of 64 separate 40-byte windows.  Entries with j outside
// [0, W_i) are never read (the loads are predicated on the reference's zero
// padding), so they need not be written.
#include <stdlib.h>

#include "../common.h"

namespace rc {

struct ShearArgs {
    const float *lvl[kMaxLevels];
    int W[kMaxLevels];
    long long K[kMaxLevels];  // rows per (b,h) block
    long long ldw;            // row stride (elements, >= W1)
    const float *coords;
    long long cbs;
    float *out;
    long long P;
    long long BH;             // B*H row blocks
    int HW, W1, H;
    int levels;
};

template <int R>
struct ShearWindow {
    static constexpr int T = 2 * R + 1, NW = 2 * R + 4;
    float s[NW];
    float xp[T];
    float n;
    bool inwin;
};

template <int R>
__device__ __forceinline__ void shear_issue(ShearWindow<R> &sw, const ShearArgs &a, int i, float x,
                                            long long bh0, int rel, int w1) {
    constexpr int T = ShearWindow<R>::T, NW = ShearWindow<R>::NW;
    const int W = a.W[i];
    const float Wm1 = (float)(W - 1);
    const DivRN dv = div_prep(Wm1);
    const float half = Wm1 / 2.0f;
    const float xl = x / (float)(1 << i);
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const float xt = (float)(t - R) + xl;
        const float xn = div_rn(2.0f * xt, dv) - 1.0f;
        sw.xp[t] = (xn + 1.0f) * half;
    }
    sw.inwin = (xl > -(float)(R + 4)) && (xl < (float)(W + R + 4));
    sw.n = sw.inwin ? floorf(xl) : 0.0f;
    const int ni = (int)sw.n;
    const int first = sw.inwin ? (int)floorf(sw.xp[0]) : 0;
    const int last = sw.inwin ? (int)floorf(sw.xp[T - 1]) + 1 : -1;
    // wave-uniform descriptor at the block's first (b,h) row block; the lane's
    // row block is an offset (a divergent base would waterfall every load)
    const float *blk0 = a.lvl[i] + bh0 * a.K[i] * a.ldw;
    const auto rs = make_rsrc(blk0, clamp_bytes((a.BH - bh0) * a.K[i] * a.ldw * 4));
    const int kc = rel * (int)a.K[i] + (w1 >> i) + W - 1;  // row (within blk0) of element 0
#pragma unroll
    for (int jj = 0; jj < NW; ++jj) {
        const int e = ni - R - 1 + jj;
        const bool ok = sw.inwin && e >= first && e <= last && e >= 0 && e < W;
        const uint32_t off = ok ? (uint32_t)(((long long)(kc - e) * a.ldw + w1) * 4) : 0xFFFFFF00u;
        sw.s[jj] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, (int)off, 0, 0));
    }
}

template <int R, class Sink>
__device__ __forceinline__ void shear_finish(const ShearWindow<R> &sw, const ShearArgs &a, int i,
                                             long long bh, int w1, Sink &&sink) {
    constexpr int T = ShearWindow<R>::T;
    const int W = a.W[i];
    const float Wm1 = (float)(W - 1);
    const int kc = (w1 >> i) + W - 1;
    float s[ShearWindow<R>::NW];
#pragma unroll
    for (int j = 0; j < ShearWindow<R>::NW; ++j) s[j] = sw.s[j];
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const float xq = sw.xp[t];
        const float x0 = floorf(xq);
        const float wt1 = xq - x0, wt0 = 1.0f - wt1;
        const float nt = sw.n + (float)(t - R);
        const bool lo = x0 < nt, hi = x0 > nt;
        float a0 = lo ? s[t] : (hi ? s[t + 2] : s[t + 1]);
        float a1 = lo ? s[t + 1] : (hi ? s[t + 3] : s[t + 2]);
        const bool ok0 = (x0 >= 0.0f) && (x0 <= Wm1);
        const bool ok1 = (x0 + 1.0f >= 0.0f) && (x0 + 1.0f <= Wm1);
        if (__builtin_expect(sw.inwin && (x0 < nt - 1.0f || x0 > nt + 1.0f), 0)) {
            const float *blk = a.lvl[i] + bh * a.K[i] * a.ldw;
            const long long e0 = (long long)x0;
            a0 = ok0 ? blk[(kc - e0) * a.ldw + w1] : 0.0f;
            a1 = ok1 ? blk[(kc - e0 - 1) * a.ldw + w1] : 0.0f;
        }
        const float v0 = ok0 ? a0 : 0.0f;
        const float v1 = ok1 ? a1 : 0.0f;
        sink(t, fmaf(wt1, v1, wt0 * v0));
    }
}

// NL > 0: levels unrolled, every level's loads issued before any tap math
// (one memory round trip per wave); capped at 128 VGPRs so 4 waves/SIMD fit.
template <int R, int NL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4)))
void lookup_sheared_kernel(ShearArgs a) {
    constexpr int T = 2 * R + 1;
    const long long p = (long long)blockIdx.x * 256 + threadIdx.x;
    const bool active = p < a.P;
    const long long pp = active ? p : a.P - 1;
    const long long bimg = pp / a.HW, rem = pp - bimg * a.HW;
    const int h = (int)(rem / a.W1), w1 = (int)(rem - (long long)h * a.W1);
    const float x = a.coords[bimg * a.cbs + rem];
    float *outp = a.out + bimg * (long long)(a.levels * T) * a.HW + rem;
    const long long bh = bimg * a.H + h;
    const long long p0 = (long long)blockIdx.x * 256;
    const long long bh0 = p0 / a.W1;  // uniform
    const int rel = (int)(bh - bh0);
    const long long HW = a.HW;
    if constexpr (NL > 0) {
        ShearWindow<R> sw[NL];
#pragma unroll
        for (int i = 0; i < NL; ++i) shear_issue<R>(sw[i], a, i, x, bh0, rel, w1);
#pragma unroll
        for (int i = 0; i < NL; ++i)
            shear_finish<R>(sw[i], a, i, bh, w1, [&](int t, float v) {
                if (active) outp[(long long)(i * T + t) * HW] = v;
            });
    } else {
        for (int i = 0; i < a.levels; ++i) {
            ShearWindow<R> sw;
            shear_issue<R>(sw, a, i, x, bh0, rel, w1);
            shear_finish<R>(sw, a, i, bh, w1, [&](int t, float v) {
                if (active) outp[(long long)(i * T + t) * HW] = v;
            });
        }
    }
}

}  // namespace rc

// Dev-only entry (prototype A/B; not part of include/raftcorr.h yet).
extern "C" int rc_dev_lookup_sheared(const void *const *lvl, const int *widths, const long *kdim,
                                     long ldw, int levels, int radius, const float *coords_x,
                                     long cbs, int B, int H, int W1, float *out, void *stream) {
    rc::ShearArgs a;
    for (int i = 0; i < levels; ++i) {
        a.lvl[i] = static_cast<const float *>(lvl[i]);
        a.W[i] = widths[i];
        a.K[i] = kdim[i];
    }
    a.ldw = ldw;
    a.coords = coords_x;
    a.cbs = cbs;
    a.out = out;
    a.P = (long long)B * H * W1;
    a.HW = H * W1;
    a.W1 = W1;
    a.H = H;
    a.BH = (long long)B * H;
    a.levels = levels;
    if (a.P <= 0) return 0;
    const unsigned nblk = (unsigned)((a.P + 255) / 256);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    int variant = 0;
    if (const char *e = getenv("RAFTCORR_LOOKUP_VARIANT")) variant = atoi(e);
    if (radius != 4) return 2;
    if (variant == 3 && levels == 4)
        hipLaunchKernelGGL((rc::lookup_sheared_kernel<4, 4>), dim3(nblk), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL((rc::lookup_sheared_kernel<4, 0>), dim3(nblk), dim3(256), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}
