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
#include "common.h"
#include "split.h"

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
        const DivRN dv = div_prep(Wm1);
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
            const float xn = div_rn(2.0f * xt, dv) - 1.0f;       // model.py:271
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

// lookup_bwd_pre_kernel -- the same arithmetic as lookup_bwd_kernel, with the
// level count fixed at compile time so that every load of the launch issues
// before any tap math: all NL*(2r+1) output-gradient values, then, per level,
// the 16-byte chunks of the gradient row that intersect the lane's register
// window [n-R-1, n+R+2] clipped to [0, W).  (lookup_bwd_kernel waits on each
// level's read-modify-write chunks in turn, so the wave pays the load latency
// NL times.)  Every element a tap touches lies in that window (x0 is within
// one of the tap's nominal index nt), so a touched chunk is always loaded; only
// touched chunks are stored.  A lane with an out-of-window tap (unreachable
// within the division's error bound, kept for exactness) applies those direct
// updates first and reloads its chunks, in lookup_bwd_kernel's order, so the
// results are bit-identical to it.
template <int R, int NL, int WPE = 1, int PF = 8, bool GVL = false, bool NTG = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void lookup_bwd_pre_kernel(LookupBwdArgs a) {
    constexpr int T = 2 * R + 1, NW = 2 * R + 4, NV = (NW + 6) / 4;
    const long long pblk = (long long)blockIdx.x * 256;
    const long long p = pblk + threadIdx.x;
    if (p >= a.P) return;   // no barriers in this kernel
    const long long lrow = p - pblk;
    const long long bimg = p / a.HW, rem = p - bimg * a.HW;
    const float x = a.coords[bimg * a.cbs + rem];
    const float *go = a.grad_out + bimg * (long long)(NL * T) * a.HW + rem;

    float gv[NL][T];
    f32x4 v[NL][NV];
    float nn[NL];
    bool win[NL];
    // issue(i): level i's output-gradient values and gradient-row chunks
    auto issue = [&](int i) {
        if constexpr (!GVL) {
#pragma unroll
            for (int t = 0; t < T; ++t)
                gv[i][t] = NTG ? __builtin_nontemporal_load(go + (long long)(i * T + t) * a.HW)
                               : go[(long long)(i * T + t) * a.HW];
        }
        const int W = a.W[i];
        const float xl = x / (float)(1 << i);
        win[i] = (xl > -(float)(R + 4)) && (xl < (float)(W + R + 4));   // false for NaN
        nn[i] = win[i] ? floorf(xl) : 0.0f;
        const int e0 = (int)nn[i] - R - 1;
        const int ea = e0 & ~3;
        const int wlo = max(e0, 0), whi = min(e0 + NW - 1, W - 1);
        // block-uniform resource over this block's rows; a skipped chunk gets
        // an out-of-range offset (reads 0, no fault)
        const long long ld = a.ld[i];
        const auto rs = make_rsrc(a.g[i] + pblk * ld, clamp_bytes((a.P - pblk) * ld * 4));
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            const int cs = ea + 4 * k;
            // cs >= 0 and cs <= W - 1 < ld: the chunk is inside the lane's row
            const bool ok = win[i] && cs <= whi && cs + 3 >= wlo;
            v[i][k] = ld4(rs, ok ? (uint32_t)((lrow * ld + cs) * 4) : 0xFFFFFF00u);
        }
    };
    // PF levels in flight ahead of the one being computed (PF >= NL: all up front)
#pragma unroll
    for (int i = 0; i < (PF < NL ? PF : NL); ++i) issue(i);

#pragma unroll
    for (int i = 0; i < NL; ++i) {
        if (i + PF < NL) issue(i + PF);
        if constexpr (GVL) {   // output gradients loaded at their level (fewer live registers)
#pragma unroll
            for (int t = 0; t < T; ++t) gv[i][t] = go[(long long)(i * T + t) * a.HW];
        }
        const int W = a.W[i];
        const float Wm1 = (float)(W - 1);
        const DivRN dv = div_prep(Wm1);
        const float half = Wm1 / 2.0f;
        const float xl = x / (float)(1 << i);
        const bool inwin = win[i];
        const float n = nn[i];
        float *row = a.g[i] + p * a.ld[i];
        float acc[NW];
#pragma unroll
        for (int j = 0; j < NW; ++j) acc[j] = 0.0f;
        int first = 0x7FFFFFFF, last = -1;
        bool bad = false;
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const float xt = (float)(t - R) + xl;
            const float xn = div_rn(2.0f * xt, dv) - 1.0f;       // model.py:271
            const float xp = (xn + 1.0f) * half;              // :275 unnormalise
            const float x0 = floorf(xp);
            const float w1 = xp - x0, w0 = (x0 + 1.0f) - xp;
            const bool ok0 = (x0 >= 0.0f) && (x0 <= Wm1);
            const bool ok1 = (x0 + 1.0f >= 0.0f) && (x0 + 1.0f <= Wm1);
            const float c0 = w0 * gv[i][t], c1 = w1 * gv[i][t];
            const float nt = n + (float)(t - R);
            const bool out = !inwin || x0 < nt - 1.0f || x0 > nt + 1.0f;
            bad |= out && (ok0 || ok1);
            const int j0 = t + (x0 < nt ? 0 : (x0 > nt ? 2 : 1));
            const int e = (int)x0;
            const bool u0 = ok0 && !out, u1 = ok1 && !out;
            if (u0) { first = min(first, e); last = max(last, e); }
            if (u1) { first = min(first, e + 1); last = max(last, e + 1); }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int j = t + q;
                if (j < NW) {
                    float add = acc[j];
                    if (u0 && j0 == j) add += c0;
                    if (u1 && j0 + 1 == j) add += c1;
                    acc[j] = add;
                }
            }
        }
        const int e0 = (int)n - R - 1;
        const int ea = e0 & ~3;
        const int sh = e0 - ea;
        if (__builtin_expect(bad, 0)) {
            // lookup_bwd_kernel's order: direct updates first (tap order), then
            // the window's read-modify-write on fresh chunk values
            for (int t = 0; t < T; ++t) {
                const float xt = (float)(t - R) + xl;
                const float xn = div_rn(2.0f * xt, dv) - 1.0f;
                const float xp = (xn + 1.0f) * half;
                const float x0 = floorf(xp);
                const float w1 = xp - x0, w0 = (x0 + 1.0f) - xp;
                const bool ok0 = (x0 >= 0.0f) && (x0 <= Wm1);
                const bool ok1 = (x0 + 1.0f >= 0.0f) && (x0 + 1.0f <= Wm1);
                const float nt = n + (float)(t - R);
                if (!inwin || x0 < nt - 1.0f || x0 > nt + 1.0f) {
                    if (ok0) row[(long long)x0] += w0 * gv[i][t];
                    if (ok1) row[(long long)x0 + 1] += w1 * gv[i][t];
                }
            }
#pragma unroll
            for (int k = 0; k < NV; ++k) {
                const int cs = ea + 4 * k;
                if (!(cs > last || cs + 3 < first)) v[i][k] = *reinterpret_cast<const f32x4 *>(row + cs);
            }
        }
        if (last < first) continue;
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            const int cs = ea + 4 * k;
            if (cs > last || cs + 3 < first) continue;
            f32x4 w = v[i][k];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                float add = 0.0f;   // acc[4k + c - sh]
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    const int j = 4 * k + c - s;
                    if (j >= 0 && j < NW) add = (sh == s) ? acc[j] : add;
                }
                w[c] += add;
            }
            *reinterpret_cast<f32x4 *>(row + cs) = w;
        }
    }
}

// lookup_bwd_pair_kernel -- the lookup backward for pool-chain gradients
// stored as levels 0 and 2 only (the forward's pair kernel in reverse,
// lookup.hip).  A level-(2k+1) tap contribution c to element j equals c/2 to
// level-2k elements 2j and 2j+1 (avg_pool2d's backward, model.py:294, exact
// in fp32), so the lane accumulates both levels of a pair into ONE register
// window over the level-2k span [2(m-R-1), 2(m+R+3)) and read-modify-writes
// the 16-B chunks of that span it touched: two spans per pixel instead of
// four windows (~3.8 instead of ~5.4 64-B requests each way at the bench
// coordinates).  rc_corr_build_backward then folds level 2
// into level 0 (volume_bwd_kernel<.., kPairFold, ..>).  The summation order
// differs from the per-level kernels (tolerance-level parity, not bitwise).
// Taps never leave the window for W <= 2^16 (the argument in lookup.hip,
// window_taps); a lane whose pair breaks n = 2m + dd (only a subnormal x)
// updates memory tap by tap and stores no chunk.
template <int R>
struct PairGradSpan {
    static constexpr int NW = 2 * R + 4, NS = 2 * NW, NC = (NS + 2 + 3) / 4;
    f32x4 q[NC];
    float gv[2][2 * R + 1];        // output gradients of the even / odd level
    float m, n;
    int sh, lo_e, hi_e;            // chunk shift; touched element range
    uint32_t ph;                   // bytes to the copy this span goes to (0 or a.shadow[lo])
    bool inwin, valid;
};

template <int R>
__device__ __forceinline__ void tap_range(float xl, int W, int &f, int &l) {
    const float Wm1 = (float)(W - 1), half = Wm1 / 2.0f;
    const DivRN dv = div_prep(Wm1);
    const float pa = ((div_rn(2.0f * ((float)(-R) + xl), dv) - 1.0f) + 1.0f) * half;
    const float pb = ((div_rn(2.0f * ((float)R + xl), dv) - 1.0f) + 1.0f) * half;
    f = max((int)floorf(pa), 0);
    l = min((int)floorf(pb) + 1, W - 1);
}

template <int R>
__device__ __forceinline__ void issue_pair_grad(PairGradSpan<R> &ps, const LookupBwdArgs &a, int lo,
                                                float x, const float *go, long long pblk,
                                                long long lrow) {
    typedef PairGradSpan<R> PS;
    constexpr int T = 2 * R + 1;
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
        for (int t = 0; t < T; ++t) ps.gv[e][t] = go[(long long)((lo + e) * T + t) * a.HW];
    const int Wlo = a.W[lo], Whi = a.W[lo + 1];
    const float xlo = x / (float)(1 << lo), xhi = x / (float)(2 << lo);
    ps.inwin = (xhi > -(float)(R + 4)) && (xhi < (float)(Whi + R + 4));   // false for NaN
    ps.m = ps.inwin ? floorf(xhi) : 0.0f;
    ps.n = ps.inwin ? floorf(xlo) : 0.0f;
    const int dd = (int)ps.n - 2 * (int)ps.m;
    ps.valid = ps.inwin && (dd == 0 || dd == 1);
    ps.lo_e = 0x7FFFFFFF;
    ps.hi_e = -1;
    if (ps.valid) {
        int f, l;
        tap_range<R>(xlo, Wlo, f, l);
        if (f <= l) { ps.lo_e = f; ps.hi_e = l; }
        tap_range<R>(xhi, Whi, f, l);
        if (f <= l) { ps.lo_e = min(ps.lo_e, 2 * f); ps.hi_e = max(ps.hi_e, 2 * l + 1); }
    }
    const int sa = 2 * ((int)ps.m - R - 1), ea = sa & ~3;
    ps.sh = sa - ea;
    const long long ld = a.ld[lo];
    // RC_SHADOW gradient copy: the span's chunks go to the
    // copy, half a 128-B line away, in which they touch fewer lines; the
    // build backward sums the two copies.  pblk * ld * 4 is a multiple of
    // 4 KB, so the line phase relative to the block base is the absolute one.
    const long long shb = a.shadow[lo];
    ps.ph = 0;
    if (shb && ps.hi_e >= ps.lo_e) {
        const long long b0 = (lrow * ld + (ps.lo_e & ~3)) * 4, b1 = (lrow * ld + (ps.hi_e | 3)) * 4 + 3;
        if (((b1 + shb) >> 7) - ((b0 + shb) >> 7) < (b1 >> 7) - (b0 >> 7)) ps.ph = (uint32_t)shb;
    }
    const auto rs = make_rsrc(a.g[lo] + pblk * ld, clamp_bytes((a.P - pblk) * ld * 4 + shb));
#pragma unroll
    for (int k = 0; k < PS::NC; ++k) {
        const int cs = ea + 4 * k;
        const bool ok = cs <= ps.hi_e && cs + 3 >= ps.lo_e;   // inside the row (lo_e >= 0, hi_e < W)
        ps.q[k] = ld4(rs, ok ? (uint32_t)((lrow * ld + cs) * 4) + ps.ph : 0xFFFFFF00u);
    }
}

// acc[j] += v at the runtime index j = base + STRIDE*off, off in [0, NOFF),
// with static indices only (the window stays in registers).
template <int NS, int NOFF, int STRIDE = 1>
__device__ __forceinline__ void win_add(float (&acc)[NS], int base, int off, float v) {
#pragma unroll
    for (int q = 0; q < NOFF; ++q) {
        const int j = base + STRIDE * q;
        if (j >= 0 && j < NS) acc[j] += (off == q) ? v : 0.0f;
    }
}

template <int R>
__device__ __forceinline__ void finish_pair_grad(PairGradSpan<R> &ps, const LookupBwdArgs &a, int lo,
                                                 float x, long long p) {
    typedef PairGradSpan<R> PS;
    constexpr int T = 2 * R + 1, NS = PS::NS;
    const int Wlo = a.W[lo], Whi = a.W[lo + 1];
    const float xlo = x / (float)(1 << lo), xhi = x / (float)(2 << lo);
    float *row = a.g[lo] + p * a.ld[lo];
    if (__builtin_expect(ps.inwin && !ps.valid, 0)) {   // subnormal x: tap by tap, to memory
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int W = e ? Whi : Wlo;
            const float xl = e ? xhi : xlo, Wm1 = (float)(W - 1), half = Wm1 / 2.0f;
            const DivRN dv = div_prep(Wm1);
            for (int t = 0; t < T; ++t) {
                const float xp = ((div_rn(2.0f * ((float)(t - R) + xl), dv) - 1.0f) + 1.0f) * half;
                const float x0 = floorf(xp);
                const float c1 = (xp - x0) * ps.gv[e][t], c0 = ((x0 + 1.0f) - xp) * ps.gv[e][t];
                for (int s = 0; s < 2; ++s) {
                    const float xe = x0 + (float)s;
                    if (!(xe >= 0.0f && xe <= Wm1)) continue;
                    const float c = s ? c1 : c0;
                    if (e == 0) row[(long long)xe] += c;
                    else { row[2 * (long long)xe] += c * 0.5f; row[2 * (long long)xe + 1] += c * 0.5f; }
                }
            }
        }
        return;
    }
    if (ps.hi_e < ps.lo_e) return;                       // nothing in range (or !inwin)
    // register window over the span: acc[j] <-> element 2(m-R-1) + j
    float acc[NS];
#pragma unroll
    for (int j = 0; j < NS; ++j) acc[j] = 0.0f;
    const int dd = (int)ps.n - 2 * (int)ps.m;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const int W = e ? Whi : Wlo;
        const float xl = e ? xhi : xlo, nwin = e ? ps.m : ps.n;
        const float Wm1 = (float)(W - 1), half = Wm1 / 2.0f;
        const DivRN dv = div_prep(Wm1);
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const float xt = (float)(t - R) + xl;
            const float xn = div_rn(2.0f * xt, dv) - 1.0f;        // model.py:271
            const float xp = (xn + 1.0f) * half;               // :275 unnormalise
            const float x0 = floorf(xp);
            const float w1 = xp - x0, w0 = (x0 + 1.0f) - xp;   // ne / nw corner weights
            const float gv = ps.gv[e][t];
            const float c0 = w0 * gv, c1 = w1 * gv;
            const bool ok0 = (x0 >= 0.0f) && (x0 <= Wm1);
            const bool ok1 = (x0 + 1.0f >= 0.0f) && (x0 + 1.0f <= Wm1);
            const float nt = nwin + (float)(t - R);
            const int d = x0 < nt ? 0 : (x0 > nt ? 2 : 1);     // window index of x0 is t + d
            if (e == 0) {
                // even level: element n-R-1+(t+d) is span index dd+R+1+t+d
                win_add<NS, 4>(acc, R + 1 + t, dd + d, ok0 ? c0 : 0.0f);
                win_add<NS, 4>(acc, R + 2 + t, dd + d, ok1 ? c1 : 0.0f);
            } else {
                // odd level: element m-R-1+(t+d) covers span indices 2(t+d), 2(t+d)+1
                const float h0 = ok0 ? c0 * 0.5f : 0.0f, h1 = ok1 ? c1 * 0.5f : 0.0f;
                win_add<NS, 3, 2>(acc, 2 * t, d, h0);
                win_add<NS, 3, 2>(acc, 2 * t + 1, d, h0);
                win_add<NS, 3, 2>(acc, 2 * t + 2, d, h1);
                win_add<NS, 3, 2>(acc, 2 * t + 3, d, h1);
            }
        }
    }
    // read-modify-write the touched chunks: chunk k = elements ea+4k.., span
    // index 4k+c-sh (sh in {0, 2})
    const int ea = 2 * ((int)ps.m - R - 1) - ps.sh;
    float *wrow = reinterpret_cast<float *>(reinterpret_cast<char *>(row) + ps.ph);
#pragma unroll
    for (int k = 0; k < PS::NC; ++k) {
        const int cs = ea + 4 * k;
        if (cs > ps.hi_e || cs + 3 < ps.lo_e) continue;
        f32x4 w = ps.q[k];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int j0 = 4 * k + c, j2 = 4 * k + c - 2;
            const float a0 = j0 < NS ? acc[j0] : 0.0f;
            const float a2 = (j2 >= 0 && j2 < NS) ? acc[j2] : 0.0f;
            w[c] += ps.sh ? a2 : a0;
        }
        *reinterpret_cast<f32x4 *>(wrow + cs) = w;
    }
}

// NL = 2 (levels 0-1) or 4 (levels 0-3); a.g[1] (and a.g[3]) are not used.
// WPE / SEQ: dev A/B only (an occupancy floor; each pair's loads issued after
// the previous pair's stores instead of all up front).
template <int R, int NL, int WPE = 1, bool SEQ = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void lookup_bwd_pair_kernel(LookupBwdArgs a) {
    static_assert(NL == 2 || NL == 4, "pair backward: 2 or 4 levels");
    constexpr int NP = NL / 2, T = 2 * R + 1;
    // XCD-contiguous block order (as the forward pair kernel): neighbouring
    // blocks' output-gradient segments share lines at the channel planes'
    // seams and meet in one XCD's L2
    const long long pblk = (long long)xcd_remap(blockIdx.x, gridDim.x) * 256;
    const long long p = pblk + threadIdx.x;
    if (p >= a.P) return;   // no barriers in this kernel
    const long long bimg = p / a.HW, rem = p - bimg * a.HW;
    const float x = a.coords[bimg * a.cbs + rem];
    const float *go = a.grad_out + bimg * (long long)(NL * T) * a.HW + rem;
    if constexpr (SEQ) {
#pragma unroll
        for (int k = 0; k < NP; ++k) {
            PairGradSpan<R> sp;
            issue_pair_grad<R>(sp, a, 2 * k, x, go, pblk, p - pblk);
            finish_pair_grad<R>(sp, a, 2 * k, x, p);
        }
        return;
    }
    PairGradSpan<R> sp[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) issue_pair_grad<R>(sp[k], a, 2 * k, x, go, pblk, p - pblk);
#pragma unroll
    for (int k = 0; k < NP; ++k) finish_pair_grad<R>(sp[k], a, 2 * k, x, p);
}

// ---------------------------------------------------------------- volume bwd

// Reduction elements per stage KS = 16 (LDS rows of 24 floats; the product
// choice) or 32 (rows of 40; dev A/B): both strides keep every 16-lane
// group of a ds_read_b128 on distinct banks.  The stage holds KS/8 quads
// per thread and operand.
template <int KS>
struct BwdTile {
    static constexpr int ROW = KS == 32 ? 40 : 24;   // floats per LDS image row
    static constexpr int IMG = 128 * ROW;             // one operand image (floats)
    static constexpr int QPT = KS / 8;                // staged quads per thread
};

// Raw level-gradient values behind G[w1][w2 .. w2+3] (w2 % 4 == 0): loaded
// in one stage, folded in the next (so the loads overlap the MFMAs).
// NLEV = the exact level count (1..4, compile time), 0 (any, up to 8), or
// kPairFold: gradients of levels 0 and 2 only, levels 1 and 3 already folded
// into them by lookup_bwd_pair_kernel (g[1] = g[3] = NULL, nlev = 3):
//   Dl_0[k] = g0[k] + ((g2[k>>2] * 0.5) * 0.5),  k>>2 < W_2
// (the generic fold with a zero level 1, in the same fp32 operations).
constexpr int kPairFold = -1;
template <int NLEV>
struct FoldRaw {
    static constexpr int NC = NLEV == kPairFold ? 1 : NLEV == 0 ? kMaxLevels - 2 : (NLEV > 2 ? NLEV - 2 : 0);
    f32x4 g0;
    float l1[2];                   // level 1 at w2/2, w2/2 + 1
    float lc[NC > 0 ? NC : 1];     // level i >= 2 at w2 >> i (one value per quad)
};

template <int NLEV>
__device__ __forceinline__ void fold_load(const BuildBwdArgs &a, long long prow, int w2, bool ok,
                                          FoldRaw<NLEV> &r) {
    constexpr int NC = FoldRaw<NLEV>::NC;
    r.g0 = f32x4{0.f, 0.f, 0.f, 0.f};
    r.l1[0] = r.l1[1] = 0.0f;
#pragma unroll
    for (int i = 0; i < NC; ++i) r.lc[i] = 0.0f;
    if (!ok || w2 >= a.W2) return;
    // rows of level 0 are padded to a multiple of 4, so the quad is in the row
    r.g0 = *reinterpret_cast<const f32x4 *>(a.g[0] + prow * a.ld[0] + w2);
    if constexpr (NLEV == kPairFold) {      // one level-2 value per quad
        // RC_SHADOW gradient copies: G sums the two copies of each level
        if (a.shadow[0]) r.g0 += *reinterpret_cast<const f32x4 *>(a.g[0] + a.shadow[0] + prow * a.ld[0] + w2);
        const int k = w2 >> 2;
        if (k < a.Wl[2]) {
            const float *g2 = a.g[2] + prow * a.ld[2] + k;
            r.lc[0] = a.shadow[2] ? g2[0] + g2[a.shadow[2]] : g2[0];
        }
        return;
    }
    if (NLEV >= 2 || (NLEV == 0 && a.nlev > 1)) {
        const int k = w2 >> 1;
        const float *g1 = a.g[1] + prow * a.ld[1];
        if (k < a.Wl[1]) r.l1[0] = g1[k];
        if (k + 1 < a.Wl[1]) r.l1[1] = g1[k + 1];
    }
#pragma unroll
    for (int i = 2; i < 2 + NC; ++i) {
        const int k = w2 >> i;
        if ((NLEV > 0 || i < a.nlev) && k < a.Wl[i]) r.lc[i - 2] = a.g[i][prow * a.ld[i] + k];
    }
}

template <int NLEV>
__device__ __forceinline__ f32x4 fold_math(const BuildBwdArgs &a, int w2, const FoldRaw<NLEV> &r) {
    constexpr int NC = FoldRaw<NLEV>::NC;
    float d[4];
    if constexpr (NLEV == kPairFold) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const float t = (((w2 + c) >> 2) < a.Wl[2]) ? (r.lc[0] * 0.5f) * 0.5f : 0.0f;
            float d0 = r.g0[c] + t;
            d[c] = (w2 + c < a.W2) ? d0 : 0.0f;
        }
        apply_scale(d, a);
        return f32x4{d[0], d[1], d[2], d[3]};
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        float t = 0.0f;   // Dl_i, i from nlev-1 down to 1
#pragma unroll
        for (int i = 1 + NC; i >= 2; --i)
            if (NLEV > 0 || i < a.nlev) t = (((w2 + c) >> i) < a.Wl[i]) ? r.lc[i - 2] + t * 0.5f : 0.0f;
        if (NLEV >= 2 || (NLEV == 0 && a.nlev > 1))
            t = (((w2 + c) >> 1) < a.Wl[1]) ? r.l1[c >> 1] + t * 0.5f : 0.0f;
        float d0 = r.g0[c] + t * 0.5f;
        d[c] = (w2 + c < a.W2) ? d0 : 0.0f;   // the row padding may hold anything
    }
    apply_scale(d, a);
    return f32x4{d[0], d[1], d[2], d[3]};
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

template <bool VEC, int NLEV, int KS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NLEV == 0 ? 1 : 2)))
void volume_bwd_kernel(BuildBwdArgs a, int nwg_total) {
    static_assert(NLEV >= kPairFold, "level count");
    typedef BwdTile<KS> TL;
    constexpr int kBwdK = KS, kBwdRow = TL::ROW, QPT = TL::QPT;
    __shared__ __attribute__((aligned(16))) float smem[2][2][TL::IMG];   // [buf][X | Y]
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

    // Staging, QPT quads per thread per operand and stage (c = tid + 256u):
    //   X, and Y of dF1 (G rows, k = w2 contiguous): row c/(KS/4), k 4(c%(KS/4))
    //   Y of dF2 (G^T: n = w2 contiguous in G):     k c%KS, n 4(c/KS)
    constexpr int QR = KS / 4;                  // quads per staged row
    f32x4 rx[QPT];
    FoldRaw<NLEV> ry[QPT];
    auto load_stage = [&](int kb) {
#pragma unroll
        for (int u = 0; u < QPT; ++u) {
            const int c = tid + 256 * u;
            const int r = c / QR, kq = 4 * (c % QR);
            const int d = m0 + r;
            const float *xrow = X + ((long long)(b * D + (d < D ? d : 0)) * H + h) * K;
            rx[u] = load_x_quad<VEC>(xrow, kb + kq, K, d < D);
            if (!kind2) {
                const int w1 = n0 + r;
                fold_load<NLEV>(a, prow0 + w1, kb + kq, w1 < W1, ry[u]);
            } else {
                const int w1 = kb + (c % KS);
                fold_load<NLEV>(a, prow0 + w1, n0 + 4 * (c / KS), w1 < W1, ry[u]);
            }
        }
    };
    auto write_stage = [&](int buf, int kb) {
        float *sx = smem[buf][0], *sy = smem[buf][1];
#pragma unroll
        for (int u = 0; u < QPT; ++u) {
            const int c = tid + 256 * u;
            const int r = c / QR, kq = 4 * (c % QR);
            *reinterpret_cast<f32x4 *>(sx + r * kBwdRow + kq) = rx[u];
            if (!kind2) {
                *reinterpret_cast<f32x4 *>(sy + r * kBwdRow + kq) = fold_math<NLEV>(a, kb + kq, ry[u]);
            } else {
                const int k = c % KS, nq = 4 * (c / KS);
                const f32x4 gq = fold_math<NLEV>(a, n0 + nq, ry[u]);
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

    const int nst = (K + kBwdK - 1) / kBwdK;
    load_stage(0);
    write_stage(0, 0);
    __syncthreads();
    for (int st = 0; st < nst; ++st) {
        const int buf = st & 1;
        if (st + 1 < nst) load_stage((st + 1) * kBwdK);
        const float *sx = smem[buf][0], *sy = smem[buf][1];
#pragma unroll
        for (int kh = 0; kh < kBwdK / 16; ++kh) {
            f32x4 av[4], bv[4];
#pragma unroll
            for (int f = 0; f < 4; ++f) {
                av[f] = *reinterpret_cast<const f32x4 *>(sy + (wn + 16 * f + i16) * kBwdRow + 16 * kh + 4 * g);
                bv[f] = *reinterpret_cast<const f32x4 *>(sx + (wm + 16 * f + i16) * kBwdRow + 16 * kh + 4 * g);
            }
#pragma unroll
            for (int kk = 0; kk < 4; ++kk)
#pragma unroll
                for (int nb = 0; nb < 4; ++nb)
#pragma unroll
                    for (int ma = 0; ma < 4; ++ma)
                        acc[nb][ma] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[nb][kk], bv[ma][kk],
                                                                          acc[nb][ma], 0, 0, 0);
        }
        if (st + 1 < nst) write_stage(buf ^ 1, (st + 1) * kBwdK);
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

// volume_bwd_split_kernel -- the same two GEMMs on bf16 MFMA by the exact
// three-way split of every fp32 operand (split.h; the forward's arithmetic,
// DESIGN.md §3.1c, §3.4): per 32-k step six v_mfma_f32_16x16x32_bf16 per
// 16x16 output fragment pair instead of eight v_mfma_f32_16x16x4f32.
// Staging, fold and output stores are volume_bwd_kernel's with 32-k stages
// (LDS rows of 40 floats, 80 KiB: two workgroups per CU).  A lane (i16, g)
// supplies k = 4g..4g+3 and 16+4g..16+4g+3 of its row to the MFMA's 8-k
// slot g (the sum over k is order-free; both operands use the same
// permutation), i.e. two conflict-free ds_read_b128 at row*40 + 4g and +16.
template <bool VEC, int NLEV, bool KM, bool K2>
__device__ __forceinline__ void volume_bwd_split_tile(const BuildBwdArgs &a, float (*smem)[2][BwdTile<32>::IMG],
                                                      int row, int tile, int T1) {
    constexpr bool kind2 = K2;                  // false: a dF1 tile, true: a dF2 tile
    typedef BwdTile<32> TL;
    constexpr int kBwdK = 32, kBwdRow = TL::ROW, QPT = TL::QPT;
    constexpr int kYP = 132;                    // KM: pitch of the k-major G image (32 x 132 <= 128 x 40)
    static_assert(32 * kYP <= TL::IMG, "k-major image fits the operand slot");
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    if (kind2) tile -= T1;
    const int tn = kind2 ? a.tn2 : a.tn1;
    const int tmi = tile / tn, tni = tile - tmi * tn;
    const int b = row / a.H, h = row - b * a.H;
    const int D = a.D, H = a.H, W1 = a.W1;
    const int K = kind2 ? W1 : a.W2;            // reduction length
    const int N = kind2 ? a.W2 : W1;            // output row length
    const int m0 = tmi * 128, n0 = tni * 128;
    const long long prow0 = (long long)row * W1;
    const float *X = kind2 ? a.f1 : a.f2;
    float *out = kind2 ? a.df2 : a.df1;

    constexpr int QR = kBwdK / 4;
    f32x4 rx[QPT];
    FoldRaw<NLEV> ry[QPT];
    // buffer loads (pair-folded / one-level gradients, the product layouts):
    // wave-uniform resources over the image's feature map and the gradient
    // levels, 32-bit offsets, out-of-range offsets read zeros -- no 64-bit
    // address arithmetic and no branch per load (the launcher keeps every
    // operand below 4 GiB)
    constexpr bool BUF = VEC && (NLEV == kPairFold || NLEV == 1);
    const auto rX = make_rsrc(X + (long long)b * D * H * K, clamp_bytes((long long)D * H * K * 4));
    const long long Prow = (long long)a.B * a.H * W1;
    const auto rG0 = make_rsrc(a.g[0], clamp_bytes((Prow * a.ld[0] + a.shadow[0]) * 4));
    const auto rG2 = make_rsrc(NLEV == kPairFold ? a.g[2] : a.g[0],
                               clamp_bytes(NLEV == kPairFold ? (Prow * a.ld[2] + a.shadow[2]) * 4 : 0));
    auto fold_buf = [&](long long prow, int w2, bool ok, FoldRaw<NLEV> &rr) {
        ok = ok && w2 < a.W2;
        const uint32_t o0 = ok ? (uint32_t)((prow * a.ld[0] + w2) * 4) : 0xFFFFFF00u;
        rr.g0 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rG0, (int)o0, 0, 0));
        rr.l1[0] = rr.l1[1] = 0.0f;
        if (a.shadow[0])         // wave-uniform: RC_SHADOW gradient copies sum
            rr.g0 += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                  rG0, (int)o0, (int)(a.shadow[0] * 4), 0));
        if constexpr (NLEV == kPairFold) {
            const int k2 = w2 >> 2;
            const uint32_t o2 = ok && k2 < a.Wl[2] ? (uint32_t)((prow * a.ld[2] + k2) * 4) : 0xFFFFFF00u;
            float v = ld1(rG2, o2);
            if (a.shadow[2]) v = v + __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                                 rG2, (int)o2, (int)(a.shadow[2] * 4), 0));
            rr.lc[0] = v;
        }
    };
    auto load_stage = [&](int kb) {
#pragma unroll
        for (int u = 0; u < QPT; ++u) {
            const int c = tid + 256 * u;
            const int r = c / QR, kq = 4 * (c % QR);
            const int d = m0 + r;
            if constexpr (BUF) {
                const uint32_t ox = d < D && kb + kq < K ? (uint32_t)((((long long)d * H + h) * K + kb + kq) * 4)
                                                         : 0xFFFFFF00u;
                rx[u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rX, (int)ox, 0, 0));
                if (!kind2) {
                    const int w1 = n0 + r;
                    fold_buf(prow0 + w1, kb + kq, w1 < W1, ry[u]);
                } else if constexpr (KM) {            // G rows, coalesced along w2
                    const int w1 = kb + (c >> 5);
                    fold_buf(prow0 + w1, n0 + 4 * (c & 31), w1 < W1, ry[u]);
                } else {                              // the mapping write_stage's !KM branch reads
                    const int w1 = kb + (c % kBwdK);
                    fold_buf(prow0 + w1, n0 + 4 * (c / kBwdK), w1 < W1, ry[u]);
                }
                continue;
            }
            const float *xrow = X + ((long long)(b * D + (d < D ? d : 0)) * H + h) * K;
            rx[u] = load_x_quad<VEC>(xrow, kb + kq, K, d < D);
            if (!kind2) {
                const int w1 = n0 + r;
                fold_load<NLEV>(a, prow0 + w1, kb + kq, w1 < W1, ry[u]);
            } else if constexpr (KM) {                // G rows, coalesced along w2
                const int w1 = kb + (c >> 5);
                fold_load<NLEV>(a, prow0 + w1, n0 + 4 * (c & 31), w1 < W1, ry[u]);
            } else {
                const int w1 = kb + (c % kBwdK);
                fold_load<NLEV>(a, prow0 + w1, n0 + 4 * (c / kBwdK), w1 < W1, ry[u]);
            }
        }
    };
    auto write_stage = [&](int buf, int kb) {
        float *sx = smem[buf][0], *sy = smem[buf][1];
#pragma unroll
        for (int u = 0; u < QPT; ++u) {
            const int c = tid + 256 * u;
            const int r = c / QR, kq = 4 * (c % QR);
            *reinterpret_cast<f32x4 *>(sx + r * kBwdRow + kq) = rx[u];
            if (!kind2) {
                *reinterpret_cast<f32x4 *>(sy + r * kBwdRow + kq) = fold_math<NLEV>(a, kb + kq, ry[u]);
            } else if constexpr (KM) {                // k-major image [32 w1][kYP]
                *reinterpret_cast<f32x4 *>(sy + (c >> 5) * kYP + 4 * (c & 31)) =
                    fold_math<NLEV>(a, n0 + 4 * (c & 31), ry[u]);
            } else {
                const int k = c % kBwdK, nq = 4 * (c / kBwdK);
                const f32x4 gq = fold_math<NLEV>(a, n0 + nq, ry[u]);
#pragma unroll
                for (int e = 0; e < 4; ++e) sy[(nq + e) * kBwdRow + k] = gq[e];
            }
        }
    };
    // the k-major image's fragment: column n, rows k of slot g (8 dwords;
    // pitch 132 puts the g and g+1 halves of a 32-lane group 16 banks apart)
    auto frag_km = [&](const float *img, int n, int g) {
        float x[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            x[j] = img[(4 * g + j) * kYP + n];
            x[4 + j] = img[(16 + 4 * g + j) * kYP + n];
        }
        return sp_split(x);
    };
    // a lane's fragment of image row `rr`: k = 4g..4g+3 and 16+4g..16+4g+3
    auto frag = [&](const float *img, int rr, int g) {
        const f32x4 lo = *reinterpret_cast<const f32x4 *>(img + rr * kBwdRow + 4 * g);
        const f32x4 hi = *reinterpret_cast<const f32x4 *>(img + rr * kBwdRow + 16 + 4 * g);
        const float x[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        return sp_split(x);
    };

    // wave tile: 64 d (X rows) x 64 n (Y rows); acc[nb][ma] = out^T fragment
    const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
    const int g = lane >> 4, i16 = lane & 15;
    f32x4 acc[4][4];
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nst = (K + kBwdK - 1) / kBwdK;
    load_stage(0);
    write_stage(0, 0);
    __syncthreads();
    for (int st = 0; st < nst; ++st) {
        const int buf = st & 1;
        if (st + 1 < nst) load_stage((st + 1) * kBwdK);
        const float *sx = smem[buf][0], *sy = smem[buf][1];
        SplitFrag bx[4];
#pragma unroll
        for (int ma = 0; ma < 4; ++ma) bx[ma] = frag(sx, wm + 16 * ma + i16, g);
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) {
            const SplitFrag ay = (KM && kind2) ? frag_km(sy, wn + 16 * nb + i16, g) : frag(sy, wn + 16 * nb + i16, g);
#pragma unroll
            for (int ma = 0; ma < 4; ++ma) sp_mma6(acc[nb][ma], ay, bx[ma]);
        }
        if (st + 1 < nst) write_stage(buf ^ 1, (st + 1) * kBwdK);
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


template <bool VEC, int NLEV, bool KM = true>
__global__ __launch_bounds__(256, 2) void volume_bwd_split_kernel(BuildBwdArgs a, int nwg_total) {
    static_assert(NLEV >= kPairFold, "level count");
    __shared__ __attribute__((aligned(16))) float smem[2][2][BwdTile<32>::IMG];   // [buf][X | Y]
    const int wgid = xcd_remap(blockIdx.x, nwg_total);   // one (b,h) row's tiles on one XCD
    const int T1 = a.tm * a.tn1, T = T1 + a.tm * a.tn2;
    const int row = wgid / T;
    const int tile = wgid - row * T;
    const bool kind2 = tile >= T1;              // false: a dF1 tile, true: a dF2 tile
#ifdef RAFTCORR_DEV
    if ((a.dev_only == 1 && kind2) || (a.dev_only == 2 && !kind2)) return;   // timing probe
#endif
    // one instantiation per GEMM, so each is register-allocated on its own
    if (kind2) volume_bwd_split_tile<VEC, NLEV, KM, true>(a, smem, row, tile, T1);
    else volume_bwd_split_tile<VEC, NLEV, KM, false>(a, smem, row, tile, T1);
}

#ifdef RAFTCORR_DEV
#include "dev/backward_dev.inc"   // A/B variants: libraftcorr_dev.so only
#endif

}  // namespace rc

hipError_t rc_launch_lookup_bwd(const rc::LookupBwdArgs &a, int radius, hipStream_t s) {
    if (a.P <= 0) return hipSuccess;
    const unsigned nblk = (unsigned)((a.P + 255) / 256);
#ifdef RAFTCORR_DEV
    if (const hipError_t e = rc::dev_launch_lookup_bwd(a, radius, nblk, s); e != hipErrorNotSupported) return e;
#endif
    if (a.levels >= 2 && a.g[1] == nullptr) {   // pair-folded gradient buffers (levels 0, 2)
#define RC_LBWDP(RR)                                                                                 \
    if (a.levels == 4) hipLaunchKernelGGL((rc::lookup_bwd_pair_kernel<RR, 4>), dim3(nblk), dim3(256), 0, s, a); \
    else hipLaunchKernelGGL((rc::lookup_bwd_pair_kernel<RR, 2>), dim3(nblk), dim3(256), 0, s, a);
        switch (radius) {
            case 1: RC_LBWDP(1) break;
            case 2: RC_LBWDP(2) break;
            case 3: RC_LBWDP(3) break;
            case 4: RC_LBWDP(4) break;
            default: return hipErrorInvalidValue;
        }
#undef RC_LBWDP
        return hipGetLastError();
    }
    if (radius >= 1 && radius <= 4 && a.levels >= 1 && a.levels <= 4) {
#define RC_LBWD(RR)                                                                                      \
    switch (a.levels) {                                                                                  \
        case 1: hipLaunchKernelGGL((rc::lookup_bwd_pre_kernel<RR, 1>), dim3(nblk), dim3(256), 0, s, a); break; \
        case 2: hipLaunchKernelGGL((rc::lookup_bwd_pre_kernel<RR, 2>), dim3(nblk), dim3(256), 0, s, a); break; \
        case 3: hipLaunchKernelGGL((rc::lookup_bwd_pre_kernel<RR, 3>), dim3(nblk), dim3(256), 0, s, a); break; \
        default: hipLaunchKernelGGL((rc::lookup_bwd_pre_kernel<RR, 4>), dim3(nblk), dim3(256), 0, s, a); break; \
    }
        switch (radius) {
            case 1: RC_LBWD(1) break;
            case 2: RC_LBWD(2) break;
            case 3: RC_LBWD(3) break;
            default: RC_LBWD(4) break;
        }
#undef RC_LBWD
        return hipGetLastError();
    }
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

hipError_t rc_launch_volume_bwd(const rc::BuildBwdArgs &a_in, hipStream_t s) {
    rc::BuildBwdArgs a = a_in;
    const long long nwg = (long long)a.B * a.H * a.tm * (a.tn1 + a.tn2);
    if (nwg <= 0) return hipSuccess;
    if (nwg > 0x7FFFFFFF) return hipErrorInvalidValue;
    const bool vec = (a.W1 % 4 == 0) && (a.W2 % 4 == 0);
    const dim3 grid((unsigned)nwg), blk(256);
    // the split-bf16 kernel (fp32 accuracy on bf16 MFMA) unless the exact
    // fp32 MFMA kernel is asked for (RC_BUILD_EXACT_F32, non-finite inputs)
    // (the split kernel is instantiated where it fits 256 VGPRs without
    // spilling: vector rows (widths % 4 == 0) and the pair-folded, 1- and
    // 2-level gradients; 3+ per-level layouts and odd widths keep the exact
    // kernel)
    const bool pairfold = a.nlev == 3 && a.g[1] == nullptr;
    const long long Prow = (long long)a.B * a.H * a.W1;
    const bool fits = (long long)a.D * a.H * (a.W1 > a.W2 ? a.W1 : a.W2) * 4 < 0xFFFFFF00LL &&
                      (Prow * a.ld[0] + a.shadow[0]) * 4 < 0xFFFFFF00LL &&
                      (!pairfold || (Prow * a.ld[2] + a.shadow[2]) * 4 < 0xFFFFFF00LL);
    const bool split = !a.exact && vec && fits && (pairfold || a.nlev == 1 || a.nlev == 2);
#ifdef RAFTCORR_DEV
    if (const hipError_t e = rc::dev_launch_volume_bwd(a, split, vec, pairfold, nwg, s); e != hipErrorNotSupported)
        return e;
#endif
    if (split) {
        if (pairfold) hipLaunchKernelGGL((rc::volume_bwd_split_kernel<true, rc::kPairFold>), grid, blk, 0, s, a, (int)nwg);
        else if (a.nlev == 1) hipLaunchKernelGGL((rc::volume_bwd_split_kernel<true, 1>), grid, blk, 0, s, a, (int)nwg);
        else hipLaunchKernelGGL((rc::volume_bwd_split_kernel<true, 2>), grid, blk, 0, s, a, (int)nwg);
        return hipGetLastError();
    }
    // 16-k stages for every level count: 49 KB of LDS lets three workgroups
    // share a CU (round 1 staged 32 for 1-2 levels: 851 / 976 us vs 718 /
    // 862 us at config 2 with 1 / 2 levels, the same bits)
#define RC_VBWD(NL)                                                                                 \
    if (vec) hipLaunchKernelGGL((rc::volume_bwd_kernel<true, NL, 16>), grid, blk, 0, s, a, (int)nwg); \
    else hipLaunchKernelGGL((rc::volume_bwd_kernel<false, NL, 16>), grid, blk, 0, s, a, (int)nwg);
    // pair-folded gradients (levels 0 and 2): 16-k stages, 49 KB of LDS, so
    // three workgroups share a CU (784 vs 906 us for 32-k stages at config 2,
    // the same bits)
    if (a.nlev == 3 && a.g[1] == nullptr) {
        if (vec) hipLaunchKernelGGL((rc::volume_bwd_kernel<true, rc::kPairFold, 16>), grid, blk, 0, s, a, (int)nwg);
        else hipLaunchKernelGGL((rc::volume_bwd_kernel<false, rc::kPairFold, 16>), grid, blk, 0, s, a, (int)nwg);
        return hipGetLastError();
    }
    switch (a.nlev) {   // the level count fixes the fold's loads at compile time
        case 1: RC_VBWD(1) break;
        case 2: RC_VBWD(2) break;
        case 3: RC_VBWD(3) break;
        case 4: RC_VBWD(4) break;
        default: RC_VBWD(0) break;
    }
#undef RC_VBWD
    return hipGetLastError();
}
