// Backward of the correlation path (gfx950), SURVEY.md §8f rank 2.
//
// The reference path is differentiable to the feature maps (model.py:375
// detaches only the coordinates), so autograd runs, per lookup call, the input
// gradient of grid_sample (:275), then avg_pool2d's backward for every pyramid
// step (:294), the division by sqrt(D) (:326) and the einsum's two operand
// gradients (:324).  Two kernels replace that:
//
// (1) lookup_bwd_kernel -- one lane per pixel p.  For level i and tap t the
//     forward read row p of level i at x0 = floor(x') and x0+1 with weights
//     (x0+1-x') and (x'-x0) (grid_sample's nw/ne corners; the other two
//     corners have weight 0 or lie outside the H = 1 image).  The backward
//     adds weight*grad to the same elements of the level-i gradient row.  Row
//     p belongs to lane p alone, so there are no atomics: the lane sums its
//     2r+4-element window in registers (taps in ascending order, like the
//     reference's loop) and read-modify-writes the 16-byte chunks that overlap
//     the elements it touched.  Calls accumulate, one per lookup call.
//
// (2) volume_bwd_kernel -- per (b,h) image row, with the level gradients
//     g_0..g_{L-1} folded through the pooling backward on load,
//         Dl_{L-1} = g_{L-1},   Dl_i[k] = g_i[k] + Dl_{i+1}[k>>1] / 2
//     (the coarser term only where k>>1 < W_{i+1}: floor widths), and
//     G = Dl_0 / sqrt(D) (:326):
//         dF1[d][w1] = sum_w2 F2[d][w2] G[w1][w2]      (K = W2)
//         dF2[d][w2] = sum_w1 F1[d][w1] G[w1][w2]      (K = W1)
//     Both are "out[d][n] = sum_k X[d][k] Y[n][k]" with X a feature map
//     (k contiguous) and Y = G or G^T; one launch holds the tiles of both.
//     v_mfma_f32_16x16x4_f32 on 128x128 workgroup tiles (4 waves of 64x64);
//     K is staged 16 at a time through a double-buffered LDS image of
//     [128 rows][24 floats] per operand (96-byte rows: every 16-lane group of
//     a ds_read_b128 hits distinct banks, MI355X_MICROARCH.md §LDS).  Lane
//     group g supplies k = 4g+kk in MFMA step kk, so a lane's four k values
//     come from one b128 read.  The MFMA computes out^T (A = Y rows, B = X
//     rows), so each lane ends with 4 consecutive n of one d row: 16-byte
//     output stores.  The workgroups of one (b,h) row are remapped onto one
//     XCD, which then reads that row's operands from HBM once.
#include <type_traits>

#include "common.h"

namespace rc {

// ---------------------------------------------------------------- lookup bwd

template <int R>
__global__ __launch_bounds__(256) void lookup_bwd_kernel(LookupBwdArgs a) {
    constexpr int T = 2 * R + 1, NW = 2 * R + 4, NV = (NW + 6) / 4;
    const long long p = (long long)blockIdx.x * 256 + threadIdx.x;
    if (p >= a.P) return;   // no barriers in this kernel
    const long long bimg = p / a.HW, rem = p - bimg * a.HW;
    const float x = a.coords[bimg * a.cbs + rem];
    const float *go = a.grad_out + bimg * (long long)(a.levels * T) * a.HW + rem;
    for (int i = 0; i < a.levels; ++i) {
        const int W = a.W[i];
        const float Wm1 = (float)(W - 1);
        const float half = Wm1 / 2.0f;
        const float xl = x / (float)(1 << i);
        const bool inwin = (xl > -(float)(R + 4)) && (xl < (float)(W + R + 4));  // false for NaN
        const float n = inwin ? floorf(xl) : 0.0f;
        float *row = a.g[i] + p * a.ld[i];
        float acc[NW];
#pragma unroll
        for (int j = 0; j < NW; ++j) acc[j] = 0.0f;
        int first = 0x7FFFFFFF, last = -1;   // span of touched elements
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const float xt = (float)(t - R) + xl;
            const float xn = (2.0f * xt) / Wm1 - 1.0f;       // model.py:271
            const float xp = (xn + 1.0f) * half;              // :275 unnormalise
            const float x0 = floorf(xp);
            const float w1 = xp - x0, w0 = (x0 + 1.0f) - xp;  // ne / nw corner weights
            const float gv = go[(long long)(i * T + t) * a.HW];
            const bool ok0 = (x0 >= 0.0f) && (x0 <= Wm1);
            const bool ok1 = (x0 + 1.0f >= 0.0f) && (x0 + 1.0f <= Wm1);
            const float c0 = w0 * gv, c1 = w1 * gv;
            const float nt = n + (float)(t - R);
            if (__builtin_expect(!inwin || x0 < nt - 1.0f || x0 > nt + 1.0f, 0)) {
                // outside the register window: direct update (unreachable
                // within the round trip's error bound; !inwin => !ok0 && !ok1)
                if (ok0) row[(long long)x0] += c0;
                if (ok1) row[(long long)x0 + 1] += c1;
                continue;
            }
            // x0 = nt + delta, delta in {-1,0,1}: window index of x0 is t+1+delta
            const int j0 = t + (x0 < nt ? 0 : (x0 > nt ? 2 : 1));
            const int e = (int)x0;
            if (ok0) { first = min(first, e); last = max(last, e); }
            if (ok1) { first = min(first, e + 1); last = max(last, e + 1); }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int j = t + q;
                if (j < NW) {
                    float add = acc[j];
                    if (ok0 && j0 == j) add += c0;
                    if (ok1 && j0 + 1 == j) add += c1;
                    acc[j] = add;
                }
            }
        }
        if (last < first) continue;
        // window element j <-> row element e0 + j; 16-byte chunks from ea
        const int e0 = (int)n - R - 1;
        const int ea = e0 & ~3;   // round down to a multiple of 4 (also below 0)
        const int sh = e0 - ea;
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            const int cs = ea + 4 * k;
            // every touched element lies in [0, W) of the lane's own row and
            // the row stride is a multiple of 4, so such a chunk is in the row
            if (cs > last || cs + 3 < first) continue;
            f32x4 v = *reinterpret_cast<const f32x4 *>(row + cs);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                float add = 0.0f;   // acc[4k + c - sh]
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    const int j = 4 * k + c - s;
                    if (j >= 0 && j < NW) add = (sh == s) ? acc[j] : add;
                }
                v[c] += add;
            }
            *reinterpret_cast<f32x4 *>(row + cs) = v;
        }
    }
}

// ------------------------------------------------ lookup bwd, pool chain
// The build's backward folds the level gradients through avg_pool2d's
// backward (Dl_i[k] = g_i[k] + Dl_{i+1}[k>>1] / 2), which is linear: a
// gradient c on level-i element j reaches each of level-1 elements
// [2^(i-1) j, 2^(i-1) (j+1)) as c / 2^(i-1).  This kernel adds levels >= 2
// there directly, so -- like the forward chain lookup (lookup.hip) -- it
// touches one level-0 window and one level-1 span per pixel instead of one
// window per level, and the build backward folds two buffers.  All loads
// (grad_out, both read-modify-write ranges) are issued before any math: one
// memory round trip per wave.  Taps that fall outside the register windows
// (unreachable within the round trip's error bound, or a subnormal x) are
// applied after the chunk stores with direct read-modify-writes.

// Direct read-modify-write of the taps in `mask` of level i (the chain
// backward's rare off-window path).  Out of line: inlined, its recomputed
// tap coordinates would be merged with the main path's and kept live.
__device__ __attribute__((noinline)) void bwd_chain_fallback(const LookupBwdArgs &a, int i, int R,
                                                            float x, float *row, const float *go,
                                                            unsigned mask) {
    const int T = 2 * R + 1, SI = i == 0 ? 1 : 1 << (i - 1);
    const float scale = 1.0f / (float)SI;
    const float Wm1 = (float)(a.W[i] - 1), half = Wm1 / 2.0f;
    const float xl = x / (float)(1 << i);
    for (int t = 0; t < T; ++t) {
        if (!((mask >> t) & 1u)) continue;
        const float xt = (float)(t - R) + xl;
        const float xn = (2.0f * xt) / Wm1 - 1.0f;
        const float xp = (xn + 1.0f) * half;
        const float x0 = floorf(xp);
        const float w1 = xp - x0, w0 = (x0 + 1.0f) - xp;
        const float g = go[(long long)(i * T + t) * a.HW];
        if (x0 >= 0.0f && x0 <= Wm1)
            for (int c = 0; c < SI; ++c) row[SI * (long long)x0 + c] += w0 * g * scale;
        if (x0 + 1.0f >= 0.0f && x0 + 1.0f <= Wm1)
            for (int c = 0; c < SI; ++c) row[SI * ((long long)x0 + 1) + c] += w1 * g * scale;
    }
}

template <int R, int NL>
__global__ __launch_bounds__(256) void lookup_bwd_chain_kernel(LookupBwdArgs a) {
    static_assert(NL >= 3 && NL <= 4, "chain backward: 3 or 4 levels");
    constexpr int T = 2 * R + 1, NW = 2 * R + 4, NV0 = (NW + 6) / 4;
    constexpr int TOP = NL - 1, S = 1 << (TOP - 1);
    constexpr int NE1 = S * NW, SHM = (S % 4 == 0) ? 0 : 4 - S, NC1 = (NE1 + SHM + 3) / 4;
    // the level-1 span accumulator, one private column per lane ([k][lane]:
    // lane-consecutive addresses, conflict-free for any per-lane k)
    __shared__ float span[NE1][256];
    const int lane = threadIdx.x;
    const long long p = (long long)blockIdx.x * 256 + lane;
    if (p >= a.P) return;   // no barriers in this kernel
    const long long bimg = p / a.HW, rem = p - bimg * a.HW;
    const float x = a.coords[bimg * a.cbs + rem];
    const float *go = a.grad_out + bimg * (long long)(NL * T) * a.HW + rem;

    // level 0: window [e00, e00 + NW), touched span [f0, l0]
    float *row0 = a.g[0] + p * a.ld[0];
    const int W0 = a.W[0];
    const float Wm10 = (float)(W0 - 1), half0 = Wm10 / 2.0f;
    const bool inwin0 = (x > -(float)(R + 4)) && (x < (float)(W0 + R + 4));
    const float n0 = inwin0 ? floorf(x) : 0.0f;
    int f0 = 1, l0 = 0;
    if (inwin0) {
        const float pa = ((2.0f * ((float)(-R) + x)) / Wm10 - 1.0f + 1.0f) * half0;
        const float pb = ((2.0f * ((float)R + x)) / Wm10 - 1.0f + 1.0f) * half0;
        f0 = max((int)floorf(pa), 0);
        l0 = min((int)floorf(pb) + 1, W0 - 1);
    }
    const int e00 = (int)n0 - R - 1, ea0 = e00 & ~3, sh0 = e00 - ea0;
    f32x4 v0[NV0];
#pragma unroll
    for (int k = 0; k < NV0; ++k) {
        const int cs = ea0 + 4 * k;
        v0[k] = (f0 <= l0 && cs <= l0 && cs + 3 >= f0) ? *reinterpret_cast<const f32x4 *>(row0 + cs)
                                                       : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    // levels 1..TOP: one level-1 span [e1, e1 + NE1), e1 = S (n_top - R - 1);
    // union of the touched elements [lo, hi] (level-1 coordinates)
    float *row1 = a.g[1] + p * a.ld[1];
    const float xtop = x / (float)(1 << TOP);
    const bool inwin = (xtop > -(float)(R + 4)) && (xtop < (float)(a.W[TOP] + R + 4));
    const float ntop = inwin ? floorf(xtop) : 0.0f;
    const int e1 = S * ((int)ntop - R - 1), ea1 = e1 & ~3, sh1 = e1 - ea1;
    int lo = 0x7FFFFFFF, hi = -1;
    if (inwin) {
#pragma unroll
        for (int i = 1; i <= TOP; ++i) {
            const float Wm1 = (float)(a.W[i] - 1), half = Wm1 / 2.0f;
            const float xl = x / (float)(1 << i);
            const float pa = ((2.0f * ((float)(-R) + xl)) / Wm1 - 1.0f + 1.0f) * half;
            const float pb = ((2.0f * ((float)R + xl)) / Wm1 - 1.0f + 1.0f) * half;
            const int f = max((int)floorf(pa), 0), l = min((int)floorf(pb) + 1, a.W[i] - 1);
            if (f <= l) {
                lo = min(lo, f << (i - 1));
                hi = max(hi, ((l + 1) << (i - 1)) - 1);
            }
        }
    }
    f32x4 v1[NC1];
#pragma unroll
    for (int k = 0; k < NC1; ++k) {
        const int cs = ea1 + 4 * k;
        v1[k] = (cs <= hi && cs + 3 >= lo) ? *reinterpret_cast<const f32x4 *>(row1 + cs)
                                           : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int k = 0; k < NE1; ++k) span[k][lane] = 0.0f;

    unsigned fallback[NL];   // per level: taps left for the direct path (bit t)
    {   // level 0 -> register window -> its chunks
        float acc[NW];
#pragma unroll
        for (int j = 0; j < NW; ++j) acc[j] = 0.0f;
        fallback[0] = 0u;
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const float xt = (float)(t - R) + x;
            const float xn = (2.0f * xt) / Wm10 - 1.0f;       // model.py:271
            const float xp = (xn + 1.0f) * half0;              // :275
            const float x0 = floorf(xp);
            const float w1 = xp - x0, w0 = (x0 + 1.0f) - xp;
            const bool ok0 = (x0 >= 0.0f) && (x0 <= Wm10);
            const bool ok1 = (x0 + 1.0f >= 0.0f) && (x0 + 1.0f <= Wm10);
            if (!(ok0 || ok1)) continue;
            const float nt = n0 + (float)(t - R);
            if (!inwin0 || x0 < nt - 1.0f || x0 > nt + 1.0f) {
                fallback[0] |= 1u << t;
                continue;
            }
            const float g = go[(long long)t * a.HW];
            const float c0 = w0 * g, c1 = w1 * g;
            const int j0 = t + (x0 < nt ? 0 : (x0 > nt ? 2 : 1));
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int j = t + q;
                if (j < NW) {
                    float add = acc[j];
                    if (ok0 && j0 == j) add += c0;
                    if (ok1 && j0 + 1 == j) add += c1;
                    acc[j] = add;
                }
            }
        }
#pragma unroll
        for (int k = 0; k < NV0; ++k)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                float add = 0.0f;   // acc[4k + c - sh0]
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    const int j = 4 * k + c - s;
                    if (j >= 0 && j < NW) add = (sh0 == s) ? acc[j] : add;
                }
                v0[k][c] += add;
            }
    }
    // levels 1..TOP -> the span: a gradient c on level-i element e lands on
    // level-1 elements [SI e, SI e + SI) as c / SI (SI = 2^(i-1))
#pragma unroll
    for (int i = 1; i <= TOP; ++i) {
        const int SI = 1 << (i - 1);
        const float scale = 1.0f / (float)SI;
        const float Wm1 = (float)(a.W[i] - 1), half = Wm1 / 2.0f;
        const float xl = x / (float)(1 << i);
        fallback[i] = 0u;
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const float xt = (float)(t - R) + xl;
            const float xn = (2.0f * xt) / Wm1 - 1.0f;
            const float xp = (xn + 1.0f) * half;
            const float x0 = floorf(xp);
            const float w1 = xp - x0, w0 = (x0 + 1.0f) - xp;
            const bool ok0 = (x0 >= 0.0f) && (x0 <= Wm1);
            const bool ok1 = (x0 + 1.0f >= 0.0f) && (x0 + 1.0f <= Wm1);
            if (!(ok0 || ok1)) continue;
            // level-1 offset of element x0 inside the span (x0 in [-1, W_i])
            const int off = inwin ? SI * (int)x0 - e1 : -1;
            if (off < 0 || off + 2 * SI > NE1) {
                fallback[i] |= 1u << t;
                continue;
            }
            const float g = go[(long long)(i * T + t) * a.HW];
            const float c0 = w0 * g * scale, c1 = w1 * g * scale;
            for (int c = 0; c < SI; ++c) {
                if (ok0) span[off + c][lane] += c0;
                if (ok1) span[off + SI + c][lane] += c1;
            }
        }
    }
    // span element k sits at register element k + sh1 of the loaded chunks
#pragma unroll
    for (int k = 0; k < NE1; ++k) {
        const float add = span[k][lane];
        if constexpr (SHM == 0) {
            v1[k >> 2][k & 3] += add;
        } else {
#pragma unroll
            for (int s = 0; s <= SHM; ++s)
                if (k + s < 4 * NC1) v1[(k + s) >> 2][(k + s) & 3] += (sh1 == s) ? add : 0.0f;
        }
    }

    // write back the chunks that were read (each inside the lane's own row)
#pragma unroll
    for (int k = 0; k < NV0; ++k) {
        const int cs = ea0 + 4 * k;
        if (f0 <= l0 && cs <= l0 && cs + 3 >= f0) *reinterpret_cast<f32x4 *>(row0 + cs) = v0[k];
    }
#pragma unroll
    for (int k = 0; k < NC1; ++k) {
        const int cs = ea1 + 4 * k;
        if (cs <= hi && cs + 3 >= lo) *reinterpret_cast<f32x4 *>(row1 + cs) = v1[k];
    }

    // off-window taps: direct read-modify-writes (after the chunk stores)
#pragma unroll
    for (int i = 0; i < NL; ++i)
        if (__builtin_expect(fallback[i] != 0u, 0))
            bwd_chain_fallback(a, i, R, x, i == 0 ? row0 : row1, go, fallback[i]);
}

// ---------------------------------------------------------------- volume bwd

constexpr int kBwdRow = 24;                      // floats per LDS image row (16 used)
constexpr int kBwdImg = 128 * kBwdRow;           // one operand image (floats)

// Raw level-gradient values behind G[w1][w2 .. w2+3] (w2 % 4 == 0): loaded
// in one stage, folded in the next (so the loads overlap the MFMAs).
struct FoldRaw {
    f32x4 g0;
    float l1[2];                   // level 1 at w2/2, w2/2 + 1
    float lc[kMaxLevels - 2];      // level i >= 2 at w2 >> i (one value per quad)
};

__device__ __forceinline__ void fold_load(const BuildBwdArgs &a, long long prow, int w2, bool ok,
                                          FoldRaw &r) {
    r.g0 = f32x4{0.f, 0.f, 0.f, 0.f};
    r.l1[0] = r.l1[1] = 0.0f;
#pragma unroll
    for (int i = 0; i < kMaxLevels - 2; ++i) r.lc[i] = 0.0f;
    if (!ok || w2 >= a.W2) return;
    // rows of level 0 are padded to a multiple of 4, so the quad is in the row
    r.g0 = *reinterpret_cast<const f32x4 *>(a.g[0] + prow * a.ld[0] + w2);
    if (a.nlev > 1) {
        const int k = w2 >> 1;
        const float *g1 = a.g[1] + prow * a.ld[1];
        if (k < a.Wl[1]) r.l1[0] = g1[k];
        if (k + 1 < a.Wl[1]) r.l1[1] = g1[k + 1];
    }
#pragma unroll
    for (int i = 2; i < kMaxLevels; ++i) {
        const int k = w2 >> i;
        if (i < a.nlev && k < a.Wl[i]) r.lc[i - 2] = a.g[i][prow * a.ld[i] + k];
    }
}

__device__ __forceinline__ f32x4 fold_math(const BuildBwdArgs &a, int w2, const FoldRaw &r) {
    f32x4 out;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        float t = 0.0f;   // Dl_i, i from nlev-1 down to 1
#pragma unroll
        for (int i = kMaxLevels - 1; i >= 2; --i)
            if (i < a.nlev) t = (((w2 + c) >> i) < a.Wl[i]) ? r.lc[i - 2] + t * 0.5f : 0.0f;
        if (a.nlev > 1) t = (((w2 + c) >> 1) < a.Wl[1]) ? r.l1[c >> 1] + t * 0.5f : 0.0f;
        float d0 = r.g0[c] + t * 0.5f;
        d0 = (w2 + c < a.W2) ? d0 : 0.0f;   // the row padding may hold anything
        out[c] = a.pow2 ? d0 * a.scale : d0 / a.sq;
    }
    return out;
}

template <bool VEC>
__device__ __forceinline__ f32x4 load_x_quad(const float *rowp, int k, int K, bool ok) {
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (!ok) return v;
    if constexpr (VEC) {
        if (k < K) v = *reinterpret_cast<const f32x4 *>(rowp + k);
    } else {
#pragma unroll
        for (int c = 0; c < 4; ++c)
            if (k + c < K) v[c] = rowp[k + c];
    }
    return v;
}

template <bool VEC>
__global__ __launch_bounds__(256) void volume_bwd_kernel(BuildBwdArgs a, int nwg_total) {
    __shared__ __attribute__((aligned(16))) float smem[2][2][kBwdImg];   // [buf][X | Y]
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    // XCD-aware bijective remap: consecutive wgid (one (b,h) row) on one XCD
    const int v = blockIdx.x;
    const int xcd = v & 7, q = nwg_total >> 3, rr = nwg_total & 7;
    const int wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (v >> 3);
    const int T1 = a.tm * a.tn1, T = T1 + a.tm * a.tn2;
    const int row = wgid / T;
    int tile = wgid - row * T;
    const bool kind2 = tile >= T1;              // false: a dF1 tile, true: a dF2 tile
    if (kind2) tile -= T1;
    const int tn = kind2 ? a.tn2 : a.tn1;
    const int tmi = tile / tn, tni = tile - tmi * tn;
    const int b = row / a.H, h = row - b * a.H;
    const int D = a.D, H = a.H, W1 = a.W1;
    const int K = kind2 ? W1 : a.W2;            // reduction length
    const int N = kind2 ? a.W2 : W1;            // output row length
    const int m0 = tmi * 128, n0 = tni * 128;
    const long long prow0 = (long long)row * W1;   // pyramid row of w1 = 0
    // X = the other image's feature map [d][k]: row d at ((b*D + d)*H + h)*K
    const float *X = kind2 ? a.f1 : a.f2;
    float *out = kind2 ? a.df2 : a.df1;

    // Staging, 2 quads per thread per operand and stage (c = tid + 256u):
    //   X, and Y of dF1 (G rows, k = w2 contiguous): row c>>2, k 4(c&3)
    //   Y of dF2 (G^T: n = w2 contiguous in G):     k c&15, n 4(c>>4)
    f32x4 rx[2];
    FoldRaw ry[2];
    auto load_stage = [&](int kb) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int c = tid + 256 * u;
            const int r = c >> 2, kq = 4 * (c & 3);
            const int d = m0 + r;
            const float *xrow = X + ((long long)(b * D + (d < D ? d : 0)) * H + h) * K;
            rx[u] = load_x_quad<VEC>(xrow, kb + kq, K, d < D);
            if (!kind2) {
                const int w1 = n0 + r;
                fold_load(a, prow0 + w1, kb + kq, w1 < W1, ry[u]);
            } else {
                const int w1 = kb + (c & 15);
                fold_load(a, prow0 + w1, n0 + 4 * (c >> 4), w1 < W1, ry[u]);
            }
        }
    };
    auto write_stage = [&](int buf, int kb) {
        float *sx = smem[buf][0], *sy = smem[buf][1];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int c = tid + 256 * u;
            const int r = c >> 2, kq = 4 * (c & 3);
            *reinterpret_cast<f32x4 *>(sx + r * kBwdRow + kq) = rx[u];
            if (!kind2) {
                *reinterpret_cast<f32x4 *>(sy + r * kBwdRow + kq) = fold_math(a, kb + kq, ry[u]);
            } else {
                const int k = c & 15, nq = 4 * (c >> 4);
                const f32x4 gq = fold_math(a, n0 + nq, ry[u]);
#pragma unroll
                for (int e = 0; e < 4; ++e) sy[(nq + e) * kBwdRow + k] = gq[e];
            }
        }
    };

    // wave tile: 64 d (X rows) x 64 n (Y rows); acc[nb][ma] = out^T fragment
    const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
    const int g = lane >> 4, i16 = lane & 15;
    f32x4 acc[4][4];
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nst = (K + 15) / 16;
    load_stage(0);
    write_stage(0, 0);
    __syncthreads();
    for (int st = 0; st < nst; ++st) {
        const int buf = st & 1;
        if (st + 1 < nst) load_stage((st + 1) * 16);
        const float *sx = smem[buf][0], *sy = smem[buf][1];
        f32x4 av[4], bv[4];
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            av[f] = *reinterpret_cast<const f32x4 *>(sy + (wn + 16 * f + i16) * kBwdRow + 4 * g);
            bv[f] = *reinterpret_cast<const f32x4 *>(sx + (wm + 16 * f + i16) * kBwdRow + 4 * g);
        }
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
#pragma unroll
            for (int nb = 0; nb < 4; ++nb)
#pragma unroll
                for (int ma = 0; ma < 4; ++ma)
                    acc[nb][ma] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[nb][kk], bv[ma][kk],
                                                                      acc[nb][ma], 0, 0, 0);
        if (st + 1 < nst) write_stage(buf ^ 1, (st + 1) * 16);
        __syncthreads();
    }

    // lane holds out^T[n = 4g + r][d = i16] of fragment (nb, ma): 4 consecutive n
#pragma unroll
    for (int ma = 0; ma < 4; ++ma) {
        const int d = m0 + wm + 16 * ma + i16;
        if (d >= D) continue;
        float *orow = out + ((long long)(b * D + d) * H + h) * N;
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) {
            const int n = n0 + wn + 16 * nb + 4 * g;
            if (VEC && n + 3 < N) {
                *reinterpret_cast<f32x4 *>(orow + n) = acc[nb][ma];
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (n + r < N) orow[n + r] = acc[nb][ma][r];
            }
        }
    }
}

}  // namespace rc

hipError_t rc_launch_lookup_bwd(const rc::LookupBwdArgs &a, int radius, hipStream_t s) {
    if (a.P <= 0) return hipSuccess;
    const unsigned nblk = (unsigned)((a.P + 255) / 256);
    switch (radius) {
        case 1: hipLaunchKernelGGL(rc::lookup_bwd_kernel<1>, dim3(nblk), dim3(256), 0, s, a); break;
        case 2: hipLaunchKernelGGL(rc::lookup_bwd_kernel<2>, dim3(nblk), dim3(256), 0, s, a); break;
        case 3: hipLaunchKernelGGL(rc::lookup_bwd_kernel<3>, dim3(nblk), dim3(256), 0, s, a); break;
        case 4: hipLaunchKernelGGL(rc::lookup_bwd_kernel<4>, dim3(nblk), dim3(256), 0, s, a); break;
        case 5: hipLaunchKernelGGL(rc::lookup_bwd_kernel<5>, dim3(nblk), dim3(256), 0, s, a); break;
        case 6: hipLaunchKernelGGL(rc::lookup_bwd_kernel<6>, dim3(nblk), dim3(256), 0, s, a); break;
        case 7: hipLaunchKernelGGL(rc::lookup_bwd_kernel<7>, dim3(nblk), dim3(256), 0, s, a); break;
        case 8: hipLaunchKernelGGL(rc::lookup_bwd_kernel<8>, dim3(nblk), dim3(256), 0, s, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t rc_launch_lookup_bwd_chain(const rc::LookupBwdArgs &a, int radius, hipStream_t s) {
    if (a.P <= 0) return hipSuccess;
    const unsigned nblk = (unsigned)((a.P + 255) / 256);
#define RC_BWD_CHAIN(R)                                                                          \
    if (a.levels == 4) hipLaunchKernelGGL((rc::lookup_bwd_chain_kernel<R, 4>), dim3(nblk), dim3(256), 0, s, a); \
    else hipLaunchKernelGGL((rc::lookup_bwd_chain_kernel<R, 3>), dim3(nblk), dim3(256), 0, s, a);
    if (a.levels != 3 && a.levels != 4) return hipErrorInvalidValue;
    switch (radius) {
        case 1: RC_BWD_CHAIN(1) break;
        case 2: RC_BWD_CHAIN(2) break;
        case 3: RC_BWD_CHAIN(3) break;
        case 4: RC_BWD_CHAIN(4) break;
        default: return hipErrorInvalidValue;
    }
#undef RC_BWD_CHAIN
    return hipGetLastError();
}

hipError_t rc_launch_volume_bwd(const rc::BuildBwdArgs &a, hipStream_t s) {
    const long long nwg = (long long)a.B * a.H * a.tm * (a.tn1 + a.tn2);
    if (nwg <= 0) return hipSuccess;
    if (nwg > 0x7FFFFFFF) return hipErrorInvalidValue;
    const bool vec = (a.W1 % 4 == 0) && (a.W2 % 4 == 0);
    if (vec)
        hipLaunchKernelGGL(rc::volume_bwd_kernel<true>, dim3((unsigned)nwg), dim3(256), 0, s, a, (int)nwg);
    else
        hipLaunchKernelGGL(rc::volume_bwd_kernel<false>, dim3((unsigned)nwg), dim3(256), 0, s, a, (int)nwg);
    return hipGetLastError();
}
