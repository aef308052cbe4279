// Deferred lookup backward (gfx950): the level gradients of ALL lookup calls
// of one CorrBlock1D summed in one pass, SURVEY.md §8f rank 2.
//
// The reference runs grid_sample's input gradient (model.py:275) once per
// lookup call (:376, `iters` calls) and autograd adds the results into the
// pyramid levels' gradients, then through avg_pool2d's backward (:294).
// lookup_bwd_pair_kernel (backward.hip) does that per call: each call
// read-modify-writes two spans of every pixel's gradient rows in HBM (~724 B
// of traffic per pixel and call at config 2, 1.55x its algorithmic bytes,
// because 16-B chunks of per-pixel rows cost whole lines).
//
// This kernel keeps the pixel's whole pair-layout gradient rows -- level 0
// (with level 1 folded in, c/2 to both children) and level 2 (with level 3)
// -- in LDS while it walks the calls, so HBM sees each call's coordinates and
// output gradients once (coalesced, 4 + L(2r+1)*4 B per pixel) and each row
// written once at the end (no zeroing pass, no read-modify-write):
//
//   workgroup = `pix` consecutive pixels x NL/2 level pairs, one lane per
//   (pixel, pair); lane (k, i) owns LDS row i of pair k.  Per call the lane
//   sums its 2(2r+1) taps into two register strips -- s0 over level-2k
//   elements n-r..n+r+1 (n = floor(x/2^2k)), s1 over level-(2k+1) elements
//   m-r..m+r+1 (m = floor(x/2^(2k+1))) -- with static indices, then adds s1
//   to LDS elements 2(m-r)+2j, +1 (8-B aligned ds ops) and s0 to n-r+j.
//   Elements outside [0, W) get exactly +0.0 (masked), so the strips need no
//   per-element guard: rows are separated by margins of 4r+4 floats that
//   receive only +0.0 from the lanes on either side (racing writes of equal
//   values) and that the write-back never copies.
//
// A lane takes that strip path when every tap sits where the exact
// arithmetic puts it (floor of the unnormalised tap = n-r+t at level 2k,
// m-r+t at level 2k+1) and n - 2m is 0 or 1; otherwise (rounding at integer
// x, subnormal x) it adds tap by tap to in-range elements, the per-call
// kernel's order.  Sums differ from the per-call kernel only in association
// (tolerance-level parity, tests/test_backward_calls_gpu.py).
//
// Loads: four calls in flight per lane (19 dwords each) while the current
// one is summed; calls past the last reload the last one (no branch around
// a load, so the wait counts stay static).
//
// Measured and not kept: the row updates as LDS-side adds (ds_add_f32, no
// read on the lane's chain; same order): 2499 vs 669 us per 32-call launch
// at config 2 (r03m).
#include <algorithm>

#include "common.h"

namespace rc {

extern __shared__ float bwd_calls_lds[];

template <int R>
struct BwdCall {
    float x;
    float gv[2][2 * R + 1];   // output gradients of levels 2k and 2k+1
};

// One call's x and output gradients for this lane's (pixel, level pair):
// buffer loads through a per-call resource (wave-uniform base), the lane's
// offset in a VGPR and each channel's plane offset in an SGPR -- no 64-bit
// address arithmetic per load.
template <int R, int NL>
__device__ __forceinline__ void bwd_call_load(BwdCall<R> &c, const LookupBwdCallsArgs &a, int call,
                                              long long bimg, long long rem, long long go_off) {
    constexpr int T = 2 * R + 1;
    const long long nb = a.P / a.HW;
    const auto rx = make_rsrc(a.coords[call], clamp_bytes(((nb - 1) * a.cbs[call] + a.HW) * 4));
    c.x = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                        rx, (int)(uint32_t)((bimg * a.cbs[call] + rem) * 4), 0, 0));
    const auto rg = make_rsrc(a.grad_out[call], clamp_bytes(a.P * (NL * T) * 4));
    const uint32_t vo = (uint32_t)(go_off * 4);
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
        for (int t = 0; t < T; ++t)
            c.gv[e][t] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                      rg, (int)vo, (e * T + t) * a.HW * 4, 0));
}

struct PairGeom {
    int Wlo, Whi;
    float slo, shi;       // 2^-2k, 2^-(2k+1)
    float halflo, halfhi; // (W-1)/2
    DivRN dvlo, dvhi;     // division by W-1
};

// grid_sample's unnormalised tap position (model.py:271-275 with
// align_corners=True), the forward's exact arithmetic.
__device__ __forceinline__ float tap_pos(float xl, int t_minus_r, const DivRN &dv, float half) {
    return ((div_rn(2.0f * ((float)t_minus_r + xl), dv) - 1.0f) + 1.0f) * half;
}

template <int R>
__device__ __forceinline__ void bwd_call_add(const BwdCall<R> &c, float *row, const PairGeom &g) {
    constexpr int T = 2 * R + 1, NJ = 2 * R + 2;
    const float xlo = c.x * g.slo, xhi = c.x * g.shi;
    if (!(xhi > -(float)(R + 4) && xhi < (float)(g.Whi + R + 4))) return;   // also NaN
    const float mf = floorf(xhi), nf = floorf(xlo);
    const int m = (int)mf, n = (int)nf;
    if (m < -R - 2 || m > g.Whi + R) return;   // every tap of both levels outside the row
    const int dd = n - 2 * m;
    bool fast = dd == 0 || dd == 1;
    float s0[NJ], s1[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) s0[j] = s1[j] = 0.0f;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const float xp = e ? tap_pos(xhi, t - R, g.dvhi, g.halfhi) : tap_pos(xlo, t - R, g.dvlo, g.halflo);
            const float x0 = floorf(xp);
            const float gv = c.gv[e][t];
            const float c1 = (xp - x0) * gv, c0 = ((x0 + 1.0f) - xp) * gv;   // ne / nw corners
            fast = fast && (x0 == (e ? mf : nf) + (float)(t - R));
            if (e == 0) {
                s0[t] += c0;
                s0[t + 1] += c1;
            } else {                       // avg_pool2d's backward: c/2 to both children
                s1[t] += c0 * 0.5f;
                s1[t + 1] += c1 * 0.5f;
            }
        }
    }
    if (fast) {
        const int jb = m - R, ib = n - R;
        f32x2 *q = reinterpret_cast<f32x2 *>(row + 2 * jb);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int jj = jb + j;
            const float v = (jj >= 0 && jj < g.Whi) ? s1[j] : 0.0f;
            f32x2 w = q[j];
            w[0] += v;
            w[1] += v;
            q[j] = w;
        }
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int ii = ib + j;
            row[ib + j] += (ii >= 0 && ii < g.Wlo) ? s0[j] : 0.0f;
        }
        return;
    }
    // tap by tap, in-range elements only
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const int W = e ? g.Whi : g.Wlo;
        const float Wm1 = (float)(W - 1);
        for (int t = 0; t < T; ++t) {
            const float xp = e ? tap_pos(xhi, t - R, g.dvhi, g.halfhi) : tap_pos(xlo, t - R, g.dvlo, g.halflo);
            const float x0 = floorf(xp);
            const float gv = c.gv[e][t];
            const float c1 = (xp - x0) * gv, c0 = ((x0 + 1.0f) - xp) * gv;
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const float xe = x0 + (float)s;
                if (!(xe >= 0.0f && xe <= Wm1)) continue;
                const float cc = s ? c1 : c0;
                const int k = (int)xe;
                if (e == 0) {
                    row[k] += cc;
                } else {
                    row[2 * k] += cc * 0.5f;
                    row[2 * k + 1] += cc * 0.5f;
                }
            }
        }
    }
}

// ---- software-pipelined form (the product since r03) ----------------------
// The same sums, bit for bit, with two changes to the lane's chain:
//  * one read-modify-write per call: both strips lie inside the 2NJ-element
//    window [2(m-R), 2(m+R+2)) of level 2k (n = 2m + dd), so the window is
//    read once, gets the level-(2k+1) pair contributions and then the
//    level-2k ones in registers (each element: + pair value, then + own
//    value, as the two separate updates did -- extra +0.0 adds are
//    identities, a row never holds -0.0), and is written once;
//  * the window's reads issue before the NEXT call's tap math, which then
//    hides their latency.
template <int R>
struct CallStrip {
    static constexpr int NJ = 2 * R + 2;
    float s0[NJ], s1[NJ];
    int m, dd;
    bool live, fast;
};

template <int R>
__device__ __forceinline__ void strip_compute(CallStrip<R> &s, const BwdCall<R> &c, const PairGeom &g) {
    constexpr int T = 2 * R + 1, NJ = 2 * R + 2;
    const float xlo = c.x * g.slo, xhi = c.x * g.shi;
    const bool inw = xhi > -(float)(R + 4) && xhi < (float)(g.Whi + R + 4);   // false for NaN
    const float mf = inw ? floorf(xhi) : 0.0f, nf = inw ? floorf(xlo) : 0.0f;
    s.m = (int)mf;
    const int n = (int)nf;
    s.live = inw && s.m >= -R - 2 && s.m <= g.Whi + R;
    s.dd = n - 2 * s.m;
    bool fast = s.dd == 0 || s.dd == 1;
#pragma unroll
    for (int j = 0; j < NJ; ++j) s.s0[j] = s.s1[j] = 0.0f;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const float xp = e ? tap_pos(xhi, t - R, g.dvhi, g.halfhi) : tap_pos(xlo, t - R, g.dvlo, g.halflo);
            const float x0 = floorf(xp);
            const float gv = c.gv[e][t];
            const float c1 = (xp - x0) * gv, c0 = ((x0 + 1.0f) - xp) * gv;
            fast = fast && (x0 == (e ? mf : nf) + (float)(t - R));
            if (e == 0) {
                s.s0[t] += c0;
                s.s0[t + 1] += c1;
            } else {
                s.s1[t] += c0 * 0.5f;
                s.s1[t + 1] += c1 * 0.5f;
            }
        }
    }
    s.fast = fast;
}

// Apply call `cur` (its window read already issued into w) and compute the
// strips of the next call in between.
template <int R>
__device__ __forceinline__ void strip_apply_fast(const CallStrip<R> &s, f32x2 (&w)[2 * R + 2], float *row,
                                                 const PairGeom &g) {
    constexpr int NJ = 2 * R + 2;
    const int jb = s.m - R, ib = 2 * s.m + s.dd - R;
    // in-row masks as one unsigned range test per element: j in [-jb, Whi - jb)
    const unsigned uwhi = (unsigned)g.Whi, uwlo = (unsigned)g.Wlo;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {                  // level 2k+1: c/2 to both children
        const float v = (unsigned)(jb + j) < uwhi ? s.s1[j] : 0.0f;
        w[j][0] += v;
        w[j][1] += v;
    }
    float s0m[NJ];                                  // level-2k strip, zero outside the row
#pragma unroll
    for (int j = 0; j < NJ; ++j) s0m[j] = (unsigned)(ib + j) < uwlo ? s.s0[j] : 0.0f;
#pragma unroll
    for (int k = R; k <= R + NJ; ++k) {             // level 2k: window element k = dd + R + j
        const float v0 = k - R < NJ ? s0m[k - R < NJ ? k - R : 0] : 0.0f;
        const float v1 = k - R - 1 >= 0 ? s0m[k - R - 1 >= 0 ? k - R - 1 : 0] : 0.0f;
        w[k >> 1][k & 1] += s.dd ? v1 : v0;
    }
    f32x2 *q = reinterpret_cast<f32x2 *>(row + 2 * (s.m - R));
#pragma unroll
    for (int j = 0; j < NJ; ++j) q[j] = w[j];
}

template <int R>
__device__ __forceinline__ void strip_apply_slow(const CallStrip<R> &s, const BwdCall<R> &c, float *row,
                                                 const PairGeom &g) {
    constexpr int T = 2 * R + 1;
    const float xlo = c.x * g.slo, xhi = c.x * g.shi;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const int W = e ? g.Whi : g.Wlo;
        const float Wm1 = (float)(W - 1);
        for (int t = 0; t < T; ++t) {
            const float xp = e ? tap_pos(xhi, t - R, g.dvhi, g.halfhi) : tap_pos(xlo, t - R, g.dvlo, g.halflo);
            const float x0 = floorf(xp);
            const float gv = c.gv[e][t];
            const float c1 = (xp - x0) * gv, c0 = ((x0 + 1.0f) - xp) * gv;
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const float xe = x0 + (float)q;
                if (!(xe >= 0.0f && xe <= Wm1)) continue;
                const float cc = q ? c1 : c0;
                const int k = (int)xe;
                if (e == 0) {
                    row[k] += cc;
                } else {
                    row[2 * k] += cc * 0.5f;
                    row[2 * k + 1] += cc * 0.5f;
                }
            }
        }
    }
}

// one pipeline step: apply `cur` (call c, when `valid`), compute `cur` anew
// from `nb` (call c + 1) while its window reads are in flight
template <int R>
__device__ __forceinline__ void strip_step(CallStrip<R> &cur, const BwdCall<R> &cb, const BwdCall<R> &nb,
                                           bool valid, float *row, const PairGeom &g) {
    constexpr int NJ = 2 * R + 2;
    f32x2 w[NJ];
    const bool fast = valid && cur.live && cur.fast;
    if (fast) {
        const f32x2 *q = reinterpret_cast<const f32x2 *>(row + 2 * (cur.m - R));
#pragma unroll
        for (int j = 0; j < NJ; ++j) w[j] = q[j];
    }
    CallStrip<R> nxt;
    strip_compute<R>(nxt, nb, g);
    if (fast) strip_apply_fast<R>(cur, w, row, g);
    if (valid && cur.live && !cur.fast) strip_apply_slow<R>(cur, cb, row, g);
    cur = nxt;
}

// NL = 2 (one level pair) or 4 (two); blockDim = pix * NL / 2.
template <int R, int NL, bool PIPE = true>
__global__ __launch_bounds__(128) void lookup_bwd_calls_kernel(LookupBwdCallsArgs a) {
    constexpr int NP = NL / 2, T = 2 * R + 1;
    float *lds = bwd_calls_lds;
    const int tid = threadIdx.x, nthr = blockDim.x;
    // XCD-contiguous block order: a call's output-gradient planes start at
    // multiples of H*W1*4 B (64 mod 128 at config 2), so a block's channel
    // segments straddle lines its neighbours read too -- on one XCD they meet
    // in its L2 instead of being fetched by two XCDs
    const long long pblk = (long long)xcd_remap(blockIdx.x, gridDim.x) * a.pix;
    const int npix = (int)min((long long)a.pix, a.P - pblk);
    for (int f = 4 * tid; f < a.lds_floats; f += 4 * nthr)
        *reinterpret_cast<f32x4 *>(lds + f) = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    __syncthreads();

    const int k = tid / a.pix, i = tid - k * a.pix;
    if (k < NP && i < npix) {
        const int lo = 2 * k;
        PairGeom g;
        g.Wlo = a.W[lo];
        g.Whi = a.W[lo + 1];
        g.slo = 1.0f / (float)(1 << lo);
        g.shi = 0.5f * g.slo;
        g.halflo = (float)(g.Wlo - 1) / 2.0f;
        g.halfhi = (float)(g.Whi - 1) / 2.0f;
        g.dvlo = div_prep((float)(g.Wlo - 1));
        g.dvhi = div_prep((float)(g.Whi - 1));
        float *row = lds + a.rowbase[k] + i * a.S[k];
        const long long p = pblk + i, bimg = p / a.HW, rem = p - bimg * a.HW;
        const long long go_off = (bimg * (NL * T) + lo * T) * (long long)a.HW + rem;
        const int last = a.ncalls - 1;
        BwdCall<R> b0, b1, b2, b3;
        bwd_call_load<R, NL>(b0, a, 0, bimg, rem, go_off);
        bwd_call_load<R, NL>(b1, a, min(1, last), bimg, rem, go_off);
        bwd_call_load<R, NL>(b2, a, min(2, last), bimg, rem, go_off);
        bwd_call_load<R, NL>(b3, a, min(3, last), bimg, rem, go_off);
        if constexpr (PIPE) {
            CallStrip<R> cur;
            strip_compute<R>(cur, b0, g);
            for (int c = 0; c < a.ncalls; c += 4) {
                strip_step<R>(cur, b0, b1, true, row, g);                 // call c
                bwd_call_load<R, NL>(b0, a, min(c + 4, last), bimg, rem, go_off);
                strip_step<R>(cur, b1, b2, c + 1 < a.ncalls, row, g);
                bwd_call_load<R, NL>(b1, a, min(c + 5, last), bimg, rem, go_off);
                strip_step<R>(cur, b2, b3, c + 2 < a.ncalls, row, g);
                bwd_call_load<R, NL>(b2, a, min(c + 6, last), bimg, rem, go_off);
                strip_step<R>(cur, b3, b0, c + 3 < a.ncalls, row, g);     // b0 holds call c + 4
                bwd_call_load<R, NL>(b3, a, min(c + 7, last), bimg, rem, go_off);
            }
        } else
        for (int c = 0; c < a.ncalls; c += 4) {
            bwd_call_add<R>(b0, row, g);
            bwd_call_load<R, NL>(b0, a, min(c + 4, last), bimg, rem, go_off);
            if (c + 1 < a.ncalls) bwd_call_add<R>(b1, row, g);
            bwd_call_load<R, NL>(b1, a, min(c + 5, last), bimg, rem, go_off);
            if (c + 2 < a.ncalls) bwd_call_add<R>(b2, row, g);
            bwd_call_load<R, NL>(b2, a, min(c + 6, last), bimg, rem, go_off);
            if (c + 3 < a.ncalls) bwd_call_add<R>(b3, row, g);
            bwd_call_load<R, NL>(b3, a, min(c + 7, last), bimg, rem, go_off);
        }
    }
    __syncthreads();

    // write back: one wave per row, 16-B chunks along the row (coalesced)
    // (a block narrower than a wave -- wide rows leave 8-16 pixels per block --
    // strides its lanes by the block width, not by 64)
    const int lane = tid & 63, wave = tid >> 6, nwave = (nthr + 63) >> 6, lstep = nthr < 64 ? nthr : 64;
#pragma unroll
    for (int kk = 0; kk < NP; ++kk) {
        const int n4 = a.wout[kk] >> 2;
        for (int r = wave; r < npix; r += nwave) {
            const f32x4 *src = reinterpret_cast<const f32x4 *>(lds + a.rowbase[kk] + r * a.S[kk]);
            f32x4 *dst = reinterpret_cast<f32x4 *>(a.g[kk] + (pblk + r) * a.ld[kk]);
            for (int c4 = lane; c4 < n4; c4 += lstep) {
                f32x4 v = src[c4];
                if (a.accumulate) v += dst[c4];
                dst[c4] = v;
            }
        }
    }
}

// ---- compact rows (the product since r03y) ----------------------------------
// The kernel above gives every (pixel, level pair) lane its whole gradient
// row in LDS (1.36 KB per pixel at W2 = 240), so a CU holds 3 waves and the
// lanes' serial call chains are not hidden.  A call only touches the window
// [2(m-R), 2(m+R+2)) of its lane's row (plus, on the rare tap-by-tap path,
// in-row elements near it), so each lane first reads its calls' x and keeps
// only the union of its windows, [lo, hi), in LDS: ~70 floats per lane at
// the bench coordinates instead of 170.  A block is ONE wave (64 lanes); the
// lanes' ranges are packed in lane order into `budget` floats, in as many
// passes as they need (one at the bench coordinates; a pass runs its lanes'
// calls and writes their rows while the other lanes wait), so any
// coordinates stay correct.  Rows are written whole (zeros outside [lo, hi)
// in overwrite mode).  The per-call updates are strip_step's in the same
// order: bit-identical to the whole-row kernel.  (With 64-bit address
// arithmetic per load it measured slower than the whole-row kernel at
// W2 = 240, 692-815 vs 633-760 us; with per-call buffer resources the 8
// waves per CU pay: 527 vs 681 us.)
template <int R, int NL>
__global__ __launch_bounds__(64) void lookup_bwd_calls_compact_kernel(LookupBwdCallsArgs a) {
    constexpr int NP = NL / 2, T = 2 * R + 1;
    float *lds = bwd_calls_lds;
    const int lane = threadIdx.x;
    const int pix = 64 / NP;
    const long long pblk = (long long)xcd_remap(blockIdx.x, gridDim.x) * pix;   // see lookup_bwd_calls_kernel
    const int npix = (int)min((long long)pix, a.P - pblk);
    const int k = lane / pix, i = lane - k * pix;
    const bool active = k < NP && i < npix;
    const int lo = 2 * k;
    PairGeom g;
    g.Wlo = a.W[lo];
    g.Whi = a.W[lo + 1];
    g.slo = 1.0f / (float)(1 << lo);
    g.shi = 0.5f * g.slo;
    g.halflo = (float)(g.Wlo - 1) / 2.0f;
    g.halfhi = (float)(g.Whi - 1) / 2.0f;
    g.dvlo = div_prep((float)(g.Wlo - 1));
    g.dvhi = div_prep((float)(g.Whi - 1));
    const long long p = pblk + (active ? i : 0), bimg = p / a.HW, rem = p - bimg * a.HW;

    // 1. the lane's element range: the union over its live calls of
    //    [2m - 2R - 4, 2m + 2R + 8) (the window and the tap-by-tap path's
    //    elements, |n - 2m| <= 2), 16-B aligned
    int rlo = 0x3FFFFFFF, rhi = -0x3FFFFFFF;
    if (active) {
        for (int c = 0; c < a.ncalls; ++c) {
            const float xhi = a.coords[c][bimg * a.cbs[c] + rem] * g.shi;
            if (xhi > -(float)(R + 4) && xhi < (float)(g.Whi + R + 4)) {   // false for NaN
                const int m = (int)floorf(xhi);
                if (m >= -R - 2 && m <= g.Whi + R) {
                    rlo = min(rlo, 2 * m - 2 * R - 4);
                    rhi = max(rhi, 2 * m + 2 * R + 8);
                }
            }
        }
    }
    int S = 0;
    if (rlo <= rhi) {
        rlo = rlo & ~3;                            // floor to a multiple of 4 (two's complement)
        S = (rhi - rlo + 3) & ~3;
    } else {
        rlo = 0;
    }
    // 2. pack the lanes' ranges into passes of `budget` floats, in lane order
    int my_off = 0, my_pass = 0, npass = 1;
    {
        int cur = 0, pass = 0;
        for (int l = 0; l < 64; ++l) {
            const int sl = __shfl(S, l, 64);
            if (cur + sl > a.budget) { ++pass; cur = 0; }
            if (lane == l) { my_off = cur; my_pass = pass; }
            cur += sl;
        }
        npass = pass + 1;
    }
    const long long go_off = (bimg * (NL * T) + lo * T) * (long long)a.HW + rem;
    const int last = a.ncalls - 1;
    for (int ps = 0; ps < npass; ++ps) {
        // zero the budget (one wave: LDS runs its operations in order)
        for (int f = 4 * lane; f < a.budget; f += 256)
            *reinterpret_cast<f32x4 *>(lds + f) = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        if (active && my_pass == ps && S > 0) {
            float *row = lds + my_off - rlo;           // row[e] = element e of the lane's row
            BwdCall<R> b0, b1, b2, b3;
            bwd_call_load<R, NL>(b0, a, 0, bimg, rem, go_off);
            bwd_call_load<R, NL>(b1, a, min(1, last), bimg, rem, go_off);
            bwd_call_load<R, NL>(b2, a, min(2, last), bimg, rem, go_off);
            bwd_call_load<R, NL>(b3, a, min(3, last), bimg, rem, go_off);
            CallStrip<R> cur;
            strip_compute<R>(cur, b0, g);
            for (int c = 0; c < a.ncalls; c += 4) {
                strip_step<R>(cur, b0, b1, true, row, g);
                bwd_call_load<R, NL>(b0, a, min(c + 4, last), bimg, rem, go_off);
                strip_step<R>(cur, b1, b2, c + 1 < a.ncalls, row, g);
                bwd_call_load<R, NL>(b1, a, min(c + 5, last), bimg, rem, go_off);
                strip_step<R>(cur, b2, b3, c + 2 < a.ncalls, row, g);
                bwd_call_load<R, NL>(b2, a, min(c + 6, last), bimg, rem, go_off);
                strip_step<R>(cur, b3, b0, c + 3 < a.ncalls, row, g);
                bwd_call_load<R, NL>(b3, a, min(c + 7, last), bimg, rem, go_off);
            }
        }
        // 3. write back this pass's rows: one row per step, the wave's lanes
        //    along it in 16-B chunks
        for (int l = 0; l < 64; ++l) {
            const int lp = __shfl(my_pass, l, 64), la = __shfl(active ? 1 : 0, l, 64);
            if (!la || lp != ps) continue;             // wave-uniform
            const int kk = l / pix, ii = l - kk * pix;
            const int llo = __shfl(rlo, l, 64), lS = __shfl(S, l, 64), loff = __shfl(my_off, l, 64);
            const int n4 = a.wout[kk] >> 2;
            f32x4 *dst = reinterpret_cast<f32x4 *>(a.g[kk] + (pblk + ii) * a.ld[kk]);
            for (int c4 = lane; c4 < n4; c4 += 64) {
                const int e = 4 * c4 - llo;            // element offset inside the range
                const bool in = e >= 0 && e < lS;
                const f32x4 v = in ? *reinterpret_cast<const f32x4 *>(lds + loff + e) : f32x4{0.f, 0.f, 0.f, 0.f};
                if (a.accumulate) {
                    if (in) dst[c4] = dst[c4] + v;
                } else {
                    dst[c4] = v;
                }
            }
        }
    }
}

#ifdef RAFTCORR_DEV
#include "dev/backward_calls_dev.inc"   // A/B variants: libraftcorr_dev.so only
#endif

}  // namespace rc

// The one geometry decision of the all-calls backward (asked by
// rc_lookup_bwd_calls_fits before any launch and followed by the launcher,
// so the two cannot drift apart): 1 = compact rows (one wave per block,
// ``budget`` floats of LDS: twice the widest lane range W + 8R + 24 and at
// least 20 KB), 2 = whole rows (64 KB of LDS at >= 8 pixels per block), 0 =
// neither fits, or a per-call buffer offset would pass 32 bits.  Compact
// rows are the default (buffer loads per call: 527 vs 681 us for whole rows
// at W2 = 240, 1195 vs 2591 at W2 = 720, r03w/r03y); ``whole`` asks for
// whole rows.
static int bwd_calls_layout(const rc::LookupBwdCallsArgs &a, int radius, int levels, const long long *cbs,
                            int n_calls, bool whole = false) {
    if ((levels != 2 && levels != 4) || radius < 1 || radius > 4) return 0;
    if (a.P * levels * (2 * radius + 1) * 4 >= 0xFFFFFF00LL) return 0;
    for (int c = 0; c < n_calls; ++c)
        if (((a.P / a.HW - 1) * cbs[c] + a.HW) * 4 >= 0xFFFFFF00LL) return 0;
    const int np = levels / 2, M = 4 * radius + 4;
    int maxS = 0, per_pix = 0;
    for (int k = 0; k < np; ++k) {
        maxS = std::max(maxS, ((a.W[2 * k] + 8 * radius + 24) + 3) & ~3);
        per_pix += ((a.W[2 * k] + 3) & ~3) + M;
    }
    if (!whole && (long long)std::max(5120, 2 * maxS) * 4 <= 65536) return 1;
    return (long long)(per_pix * 8 + np * M) * 4 <= 65536 ? 2 : 0;
}

// Whether rc_launch_lookup_bwd_calls can take a request: radius 1-4, 2 or 4
// levels, 32-bit per-call offsets, and a block's rows in 64 KB of LDS.
// rc_corr_lookup_backward_calls asks this once, before any launch, and
// otherwise takes the per-call path for the whole request.
bool rc_lookup_bwd_calls_fits(const rc::LookupBwdCallsArgs &a, int radius, int levels, const long *cbs,
                              int n_calls) {
    long long c64[rc::kMaxBwdCalls];
    for (int c0 = 0; c0 < n_calls; c0 += rc::kMaxBwdCalls) {
        const int n = std::min(rc::kMaxBwdCalls, n_calls - c0);
        for (int c = 0; c < n; ++c) c64[c] = cbs[c0 + c];
        if (!bwd_calls_layout(a, radius, levels, c64, n)) return false;
    }
    return true;
}

hipError_t rc_launch_lookup_bwd_calls(rc::LookupBwdCallsArgs &a, int radius, int levels, hipStream_t s) {
    if (a.P <= 0 || a.ncalls <= 0) return hipSuccess;
    if (a.ncalls > rc::kMaxBwdCalls) return hipErrorInvalidValue;
    bool whole = false;
#ifdef RAFTCORR_DEV
    whole = rc::dev_bwdc_whole_rows(radius, levels);
#endif
    const int layout = bwd_calls_layout(a, radius, levels, a.cbs, a.ncalls, whole);
    if (layout == 0) return hipErrorNotSupported;
    if (layout == 1) {
        const int np = levels / 2;
        int maxS = 0;
        for (int k = 0; k < np; ++k) {
            maxS = std::max(maxS, ((a.W[2 * k] + 8 * radius + 24) + 3) & ~3);
            a.wout[k] = (a.W[2 * k] + 3) & ~3;     // columns written per row (padding as zeros)
        }
        a.budget = std::max(5120, 2 * maxS);
        a.pix = 64 / np;
        const unsigned nblk = (unsigned)((a.P + a.pix - 1) / a.pix);
        const size_t lds = (size_t)a.budget * 4;
#define RC_LBWDCC(RR)                                                                                                 \
    if (levels == 4) hipLaunchKernelGGL((rc::lookup_bwd_calls_compact_kernel<RR, 4>), dim3(nblk), dim3(64), lds, s, a); \
    else hipLaunchKernelGGL((rc::lookup_bwd_calls_compact_kernel<RR, 2>), dim3(nblk), dim3(64), lds, s, a);
        switch (radius) {
            case 1: RC_LBWDCC(1) break;
            case 2: RC_LBWDCC(2) break;
            case 3: RC_LBWDCC(3) break;
            case 4: RC_LBWDCC(4) break;
        }
#undef RC_LBWDCC
        return hipGetLastError();
    }

    const int np = levels / 2, M = 4 * radius + 4;
    int per_pix = 0;
    for (int k = 0; k < np; ++k) {
        const int w4 = (a.W[2 * k] + 3) & ~3;
        a.S[k] = w4 + M;
        a.wout[k] = w4;
        per_pix += a.S[k];
    }
    int pix = 64 / np;
    while (pix > 8 && (long long)(per_pix * pix + np * M) * 4 > 65536) pix >>= 1;
    if ((long long)(per_pix * pix + np * M) * 4 > 65536) return hipErrorNotSupported;
    a.pix = pix;
    int off = 0;
    for (int k = 0; k < np; ++k) {
        a.rowbase[k] = off + M;
        off += M + pix * a.S[k];
    }
    a.lds_floats = (off + 3) & ~3;
    const unsigned nblk = (unsigned)((a.P + pix - 1) / pix);
    const size_t lds = (size_t)a.lds_floats * 4;
    const dim3 blk(pix * np);
#ifdef RAFTCORR_DEV
    if (const hipError_t e = rc::dev_launch_bwdc_whole(a, radius, levels, nblk, blk, lds, s); e != hipErrorNotSupported)
        return e;
#endif
#define RC_LBWDC(RR)                                                                                      \
    if (levels == 4) hipLaunchKernelGGL((rc::lookup_bwd_calls_kernel<RR, 4>), dim3(nblk), blk, lds, s, a); \
    else hipLaunchKernelGGL((rc::lookup_bwd_calls_kernel<RR, 2>), dim3(nblk), blk, lds, s, a);
    switch (radius) {
        case 1: RC_LBWDC(1) break;
        case 2: RC_LBWDC(2) break;
        case 3: RC_LBWDC(3) break;
        case 4: RC_LBWDC(4) break;
    }
#undef RC_LBWDC
    return hipGetLastError();
}
