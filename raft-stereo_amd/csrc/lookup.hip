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
// Memory: one lane per pixel.  The taps of one level touch the elements
// [x0_first, x0_last + 1] (x0 is monotone in t), which lie inside the 2r+4
// element window [n-r-1, n+r+2] (n = floor(x/2^i)) because the round trip
// moves floor(x') by at most one.  The lane fetches that window with 16-byte
// buffer loads aligned to the row start of the level; a load whose 16 bytes
// miss [x0_first, x0_last+1] gets an out-of-range offset instead, so it
// returns zeros and touches no memory (branch-free predication).  The window
// is shifted by its 0..3 (fp32) / 0..7 (bf16) misalignment with selects and
// each tap picks its pair with a 3-way select.  With the level count a
// template parameter, every level's loads issue before any tap math.  A tap
// whose floor is off by more than one (impossible for |x| < 2^22 by the error
// bound; kept for safety) takes a guarded scalar path.  Output stores are
// coalesced along w1.
#include <type_traits>

#include "common.h"

namespace rc {

// x coordinate of pixel (bimg, rem).  For rc_corr_lookup_step the pixel's
// coordinates are first advanced by the previous iteration's update (the
// forward loop's tail, SURVEY Appendix A D8: coords1 + delta_flow with the
// y component zeroed) and the new coords and flow = coords1 - coords0
// (model.py:377, coords0 = coords_grid, :329-332) are written -- the
// loop's per-iteration elementwise ops, fused into the lookup launch.
__device__ __forceinline__ float pixel_x(const LookupArgs &a, long long bimg, long long rem,
                                         bool active) {
    if (!a.step) return a.coords[bimg * a.cbs + rem];
    const long long o = bimg * 2LL * a.HW + rem;   // (B,2,H,W1) contiguous
    float x = a.coords[o];
    float y = a.coords[o + a.HW];
    if (a.delta) {
        x = x + a.delta[o];
        y = y + 0.0f;                               // delta_flow[:,1] = 0
    }
    if (active) {
        const int h = (int)(rem / a.W1), w = (int)(rem - (long long)h * a.W1);
        a.coords_out[o] = x;
        a.coords_out[o + a.HW] = y;
        a.flow_out[o] = x - (float)w;
        a.flow_out[o + a.HW] = y - (float)h;
    }
    return x;
}

template <int R, bool BF16>
struct LevelWindow {
    static constexpr int T = 2 * R + 1;
    static constexpr int NW = 2 * R + 4;              // window elements
    static constexpr int EPV = BF16 ? 8 : 4;          // elements per 16-B load
    static constexpr int NV = (NW + 2 * (EPV - 1)) / EPV;
    static constexpr int ES = BF16 ? 2 : 4;
    uint32_t q[NV][4];                                 // raw loaded dwords
    float xp[T];
    float n;
    int sh;
    bool inwin;
};

template <int R, bool BF16, bool EXACT>
__device__ __forceinline__ void issue_level(LevelWindow<R, BF16> &lw, const LookupArgs &a, int i,
                                            float x, long long pblk, long long lrow) {
    typedef LevelWindow<R, BF16> LW;
    const int W = a.W[i];
    const long long ld = a.ld[i];
    const float Wm1 = (float)(W - 1);
    const DivRN dv = div_prep(Wm1);
    const float half = Wm1 / 2.0f;
    const float xl = x / (float)(1 << i);
#pragma unroll
    for (int t = 0; t < LW::T; ++t) {
        const float xt = (float)(t - R) + xl;
        const float xn = div_rn(2.0f * xt, dv) - 1.0f;
        lw.xp[t] = (xn + 1.0f) * half;
    }
    lw.inwin = (xl > -(float)(R + 4)) && (xl < (float)(W + R + 4));  // false for NaN
    lw.n = lw.inwin ? floorf(xl) : 0.0f;
    const long long e = lrow * ld + (long long)lw.n - (R + 1);
    const long long ea = e & ~(long long)(LW::EPV - 1);
    lw.sh = (int)(e - ea);
    // exact span of elements the taps read, clipped to the row's [0, W): the
    // zero padding masks everything outside (relative to the block base;
    // selects on floats first: a NaN/huge float must never reach an integer cast)
    const float f0 = lw.inwin ? fmaxf(floorf(lw.xp[0]), 0.0f) : 0.0f;
    const float f1 = lw.inwin ? fminf(floorf(lw.xp[LW::T - 1]) + 1.0f, Wm1) : -1.0f;
    const bool any = lw.inwin && f0 <= f1;
    const long long first = lrow * ld + (long long)f0;
    const long long last = lrow * ld + (long long)f1;
    const char *base = reinterpret_cast<const char *>(a.lvl[i]) + pblk * ld * LW::ES;
    const auto rs = make_rsrc(base, clamp_bytes((a.P - pblk) * ld * LW::ES));
#pragma unroll
    for (int k = 0; k < LW::NV; ++k) {
        const long long c0 = ea + (long long)k * LW::EPV;
        uint32_t off = (uint32_t)(c0 * LW::ES);
        if (EXACT && !(any && c0 <= last && c0 + LW::EPV - 1 >= first)) off = 0xFFFFFF00u;
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 0);
#pragma unroll
        for (int c = 0; c < 4; ++c) lw.q[k][c] = v[c];
    }
}

template <int R, bool BF16, class Sink>
__device__ __forceinline__ void finish_level(const LevelWindow<R, BF16> &lw, const LookupArgs &a,
                                             int i, long long pblk, long long lrow, Sink &&sink) {
    typedef LevelWindow<R, BF16> LW;
    constexpr int T = LW::T, NW = LW::NW, EPV = LW::EPV, NE = LW::NV * EPV;
    const int W = a.W[i];
    const float Wm1 = (float)(W - 1);
    float v[NE];
#pragma unroll
    for (int k = 0; k < LW::NV; ++k)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const uint32_t u = lw.q[k][c];
            if constexpr (BF16) {
                v[k * 8 + 2 * c] = __builtin_bit_cast(float, u << 16);
                v[k * 8 + 2 * c + 1] = __builtin_bit_cast(float, u & 0xFFFF0000u);
            } else {
                v[k * 4 + c] = __builtin_bit_cast(float, u);
            }
        }
    // s[j] = element (n - R - 1 + j) = v[j + sh]
    float s[NW];
#pragma unroll
    for (int j = 0; j < NW; ++j) {
        float r = v[j];
#pragma unroll
        for (int k = 1; k < EPV; ++k) r = (lw.sh == k) ? v[j + k] : r;
        s[j] = r;
    }
    // fast path for every tap, then ONE wave-level check for the (unreachable
    // within the error bound) taps whose floor left the window
    float res[T];
    bool bad = false;
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const float xp = lw.xp[t];
        const float x0 = floorf(xp);
        const float w1 = xp - x0, w0 = 1.0f - w1;
        const float nt = lw.n + (float)(t - R);
        const bool lo = x0 < nt, hi = x0 > nt;
        const float a0 = lo ? s[t] : (hi ? s[t + 2] : s[t + 1]);
        const float a1 = lo ? s[t + 1] : (hi ? s[t + 3] : s[t + 2]);
        const bool ok0 = (x0 >= 0.0f) && (x0 <= Wm1);
        const bool ok1 = (x0 + 1.0f >= 0.0f) && (x0 + 1.0f <= Wm1);
        bad |= lw.inwin && (x0 < nt - 1.0f || x0 > nt + 1.0f);
        const float v0 = ok0 ? a0 : 0.0f;
        const float v1 = ok1 ? a1 : 0.0f;
        res[t] = fmaf(w1, v1, w0 * v0);
    }
    if (__builtin_expect(bad, 0)) {
        // Guarded scalar fallback: re-read every tap of this lane from memory.
        const char *base = reinterpret_cast<const char *>(a.lvl[i]) + pblk * a.ld[i] * LW::ES;
        for (int t = 0; t < T; ++t) {
            const float xp = lw.xp[t];
            const float x0 = floorf(xp);
            const float w1 = xp - x0, w0 = 1.0f - w1;
            const bool ok0 = (x0 >= 0.0f) && (x0 <= Wm1);
            const bool ok1 = (x0 + 1.0f >= 0.0f) && (x0 + 1.0f <= Wm1);
            const long long k0 = lrow * a.ld[i] + (long long)x0;
            float v0 = 0.0f, v1 = 0.0f;
            if constexpr (BF16) {
                const uint16_t *rowp = reinterpret_cast<const uint16_t *>(base);
                if (ok0) v0 = bf16_to_f32(rowp[k0]);
                if (ok1) v1 = bf16_to_f32(rowp[k0 + 1]);
            } else {
                const float *rowp = reinterpret_cast<const float *>(base);
                if (ok0) v0 = rowp[k0];
                if (ok1) v1 = rowp[k0 + 1];
            }
            res[t] = fmaf(w1, v1, w0 * v0);
        }
    }
#pragma unroll
    for (int t = 0; t < T; ++t) sink(t, res[t]);
}

// NL > 0: compile-time level count (all loads issue first); NL == 0: runtime.
// BS = threads per block (256 for throughput, 64 to spread small problems).
template <int R, int NL, bool BF16, bool EXACT, int BS = 256, int WPE = 1>
__global__ __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(WPE)))
void lookup_kernel(LookupArgs a) {
    constexpr int T = 2 * R + 1;
    const long long pblk = (long long)blockIdx.x * BS;
    const long long p = pblk + threadIdx.x;
    const bool active = p < a.P;
    const long long pp = active ? p : a.P - 1;
    const long long bimg = pp / a.HW, rem = pp - bimg * a.HW;
    const float x = pixel_x(a, bimg, rem, active);
    const int L = NL > 0 ? NL : a.levels;
    float *outp = a.out + bimg * (long long)(L * T) * a.HW + rem;
    const long long lrow = pp - pblk;
    if constexpr (NL > 0) {
        LevelWindow<R, BF16> lw[NL];
#pragma unroll
        for (int i = 0; i < NL; ++i) issue_level<R, BF16, EXACT>(lw[i], a, i, x, pblk, lrow);
#pragma unroll
        for (int i = 0; i < NL; ++i)
            finish_level<R, BF16>(lw[i], a, i, pblk, lrow, [&](int t, float v) {
                if (active) outp[(long long)(i * T + t) * a.HW] = v;
            });
    } else {
        for (int i = 0; i < L; ++i) {
            LevelWindow<R, BF16> lw;
            issue_level<R, BF16, EXACT>(lw, a, i, x, pblk, lrow);
            finish_level<R, BF16>(lw, a, i, pblk, lrow, [&](int t, float v) {
                if (active) outp[(long long)(i * T + t) * a.HW] = v;
            });
        }
    }
}

// Small problems (the realtime config: 19,200 pixels): a launch then lasts
// about one wave's chain of window loads and tap math, so a block gives each
// LEVEL its own wave -- wave i of block b looks up level i for pixels
// [64b, 64b+64) -- which shortens that chain ~L-fold.  Per level the code is
// lookup_kernel's (issue_level / finish_level): bit-identical results.  In
// the fused loop step every wave reads the pixel's coords before the block
// barrier and only wave 0 writes the advanced coords and flow after it (the
// outputs may alias coords1).
// XA: pixel blocks placed XCD by XCD (xcd_remap), so each XCD looks up one
// contiguous eighth of the rows -- the rows whose pyramid lines the build
// (xcd_remap'd by row) wrote through that XCD's L2.
template <int R, bool BF16, bool XA = true>
__global__ __launch_bounds__(256) void lookup_levelpar_kernel(LookupArgs a) {
    constexpr int T = 2 * R + 1;
    const int i = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));   // this wave's level
    const int blk = XA ? xcd_remap((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;
    const long long pblk = (long long)blk * 64;
    const long long p = pblk + (threadIdx.x & 63);
    const bool active = p < a.P;
    const long long pp = active ? p : a.P - 1;
    const long long bimg = pp / a.HW, rem = pp - bimg * a.HW;
    const float x = pixel_x(a, bimg, rem, false);
    if (a.step) {                                       // block-uniform
        __syncthreads();
        if (i == 0) (void)pixel_x(a, bimg, rem, active);
    }
    float *outp = a.out + bimg * (long long)(a.levels * T) * a.HW + rem;
    LevelWindow<R, BF16> lw;
    issue_level<R, BF16, true>(lw, a, i, x, pblk, pp - pblk);
    finish_level<R, BF16>(lw, a, i, pblk, pp - pblk, [&](int t, float v) {
        if (active) outp[(long long)(i * T + t) * a.HW] = v;
    });
}

// ---- lookup over a pool-chain pyramid: levels >= 2 derived from level 1 ----
// When the levels are the avg_pool chain of level 0 -- the pyramid
// rc_corr_build writes -- element j of level i >= 2 is the pairwise-mean tree
// of level-1 elements [2^(i-1) j, 2^(i-1) (j+1)) evaluated in the same fp32
// order as model.py:294 applied i-1 times, so it is recomputed from level 1
// bit for bit.  The windows of levels 1..L-1 around x all lie inside ONE span
// of level 1: the top level's 2r+4 window scaled by S = 2^(L-2) (48 elements
// at L = 4, r = 4), starting at a multiple of S.  Reading that span once
// (~2.1 128-B lines for its ~160-B exact part) replaces one ~1.3-line window
// per level, so a pixel touches ~3.4 lines instead of ~4.9.
// Level 0 keeps its own window.  fp32 pyramids only (a bf16 pyramid rounds
// every level separately).

template <int S>
__device__ __forceinline__ float pool_tree(const float *v) {
    if constexpr (S == 1) return v[0];
    else return (pool_tree<S / 2>(v) + pool_tree<S / 2>(v + S / 2)) * 0.5f;
}

// level-i element k (S_i = 2^(i-1) level-1 elements) straight from memory
template <int SI>
__device__ __forceinline__ float derived_elem(const float *row1, long long k) {
    float v[SI];
#pragma unroll
    for (int c = 0; c < SI; ++c) v[c] = row1[SI * k + c];
    return pool_tree<SI>(v);
}

// M: dev-only ablation (RAFTCORR_LOOKUP_VARIANT in launch_chain_r): 0 = product,
// 1 = no output stores (kept live by an impossible compare), 2 = no pyramid loads,
// 3 = pyramid loads only (no tap math, no stores), 4 = tap math only,
// 5 = the product with non-temporal output stores.
template <int R, int NL, int M = 0>
__global__ __launch_bounds__(256) void lookup_chain_kernel(LookupArgs a) {
    static_assert(NL >= 3 && NL <= 4, "chain lookup: 3 or 4 levels");
    constexpr int T = 2 * R + 1, NW = 2 * R + 4, TOP = NL - 1, S = 1 << (TOP - 1);
    constexpr int NE1 = S * NW;                        // span elements of level 1
    constexpr int SHM = (S % 4 == 0) ? 0 : 4 - S;      // max misalignment of its start
    constexpr int NC1 = (NE1 + SHM + 3) / 4;           // 16-B chunks
    const long long pblk = (long long)blockIdx.x * 256;
    const long long p = pblk + threadIdx.x;
    const bool active = p < a.P;
    const long long pp = active ? p : a.P - 1;
    const long long bimg = pp / a.HW, rem = pp - bimg * a.HW;
    const float x = pixel_x(a, bimg, rem, active);
    float *outp = a.out + bimg * (long long)(NL * T) * a.HW + rem;
    const long long lrow = pp - pblk;

    // level 0: its own window (lookup_kernel's path)
    LevelWindow<R, false> lw0;
    constexpr bool NOLOAD = M == 2 || M == 4, NOSTORE = M == 1 || M == 4;
    issue_level<R, false, true>(lw0, a, 0, NOLOAD ? NAN : x, pblk, lrow);

    // levels 1..TOP: one span of level 1, starting at e1 = S (n_top - R - 1)
    const float xtop = x / (float)(1 << TOP);
    const bool inwin = (xtop > -(float)(R + 4)) && (xtop < (float)(a.W[TOP] + R + 4));
    const float ntop = inwin ? floorf(xtop) : 0.0f;
    const int e1 = S * ((int)ntop - R - 1);
    const int ea = e1 & ~3;
    const int sh = e1 - ea;                            // 0 when S % 4 == 0
    int lo = 0x7FFFFFFF, hi = -1;                      // union of the exact spans
    if (inwin) {
#pragma unroll
        for (int i = 1; i <= TOP; ++i) {
            const float Wm1 = (float)(a.W[i] - 1), half = Wm1 / 2.0f;
            const DivRN dv = div_prep(Wm1);
            const float xl = x / (float)(1 << i);
            const float xa = (float)(-R) + xl, xb = (float)R + xl;
            const float pa = ((div_rn(2.0f * xa, dv) - 1.0f) + 1.0f) * half;
            const float pb = ((div_rn(2.0f * xb, dv) - 1.0f) + 1.0f) * half;
            const int f = max((int)floorf(pa), 0);
            const int l = min((int)floorf(pb) + 1, a.W[i] - 1);
            if (f <= l) {
                lo = min(lo, f << (i - 1));
                hi = max(hi, ((l + 1) << (i - 1)) - 1);
            }
        }
    }
    const long long ld1 = a.ld[1];
    const float *lvl1 = static_cast<const float *>(a.lvl[1]);
    const auto rs1 = make_rsrc(lvl1 + pblk * ld1, clamp_bytes((a.P - pblk) * ld1 * 4));
    f32x4 q1[NC1];
#pragma unroll
    for (int k = 0; k < NC1; ++k) {
        const int cs = ea + 4 * k;
        const bool ok = !NOLOAD && cs <= hi && cs + 3 >= lo;   // lo >= 0 and hi < W_1: inside the row
        q1[k] = ld4(rs1, ok ? (uint32_t)((lrow * ld1 + cs) * 4) : 0xFFFFFF00u);
    }
    if constexpr (M == 3) {
        uint32_t acc = 0;
#pragma unroll
        for (int k = 0; k < LevelWindow<R, false>::NV; ++k)
#pragma unroll
            for (int c = 0; c < 4; ++c) acc ^= lw0.q[k][c];
#pragma unroll
        for (int k = 0; k < NC1; ++k)
#pragma unroll
            for (int c = 0; c < 4; ++c) acc ^= __builtin_bit_cast(uint32_t, q1[k][c]);
        if (acc == 0x12345678u) outp[0] = 0.0f;
        return;
    }

    // level 0 math + stores while the span is in flight
    finish_level<R, false>(lw0, a, 0, pblk, lrow, [&](int t, float v) {
        if (!active) return;
        if constexpr (M == 5) __builtin_nontemporal_store(v, outp + (long long)t * a.HW);
        else if (!NOSTORE || v == 1234.5f) outp[(long long)t * a.HW] = v;
    });

    // s1[k] = level-1 element e1 + k
    float s1[NE1];
#pragma unroll
    for (int k = 0; k < NE1; ++k) {
        float r = q1[k >> 2][k & 3];
#pragma unroll
        for (int s = 1; s <= SHM; ++s)
            if (k + s < 4 * NC1) r = (sh == s) ? q1[(k + s) >> 2][(k + s) & 3] : r;
        s1[k] = r;
    }
    const float *row1 = lvl1 + pp * ld1;

    auto level = [&](auto ic) {
        constexpr int i = decltype(ic)::value;
        constexpr int SI = 1 << (i - 1), NDD = 1 << (TOP - i);
        const int W = a.W[i];
        const float Wm1 = (float)(W - 1), half = Wm1 / 2.0f;
        const DivRN dv = div_prep(Wm1);
        const float xl = x / (float)(1 << i);
        const float n = inwin ? floorf(xl) : 0.0f;
        // n = NDD * n_top + dd, dd in [0, NDD) (x / 2^i is exact); a subnormal
        // x can break that -- such a lane reads memory instead (valid = false)
        const int dd = inwin ? (int)n - NDD * (int)ntop : 0;
        const bool valid = inwin && dd >= 0 && dd < NDD;
        // window element jj (level-i element n - R - 1 + jj) starts at level-1
        // offset SI*(dd + jj) + (R+1)*(S - SI) of the span
        float w[NW];
#pragma unroll
        for (int jj = 0; jj < NW; ++jj) {
            float val = 0.0f;
#pragma unroll
            for (int d = 0; d < NDD; ++d) {
                constexpr int base = (R + 1) * (S - SI);
                const float v = pool_tree<SI>(s1 + base + SI * (d + jj));
                val = (dd == d) ? v : val;
            }
            w[jj] = val;
        }
        float res[T];
        bool bad = false;
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const float xt = (float)(t - R) + xl;
            const float xn = div_rn(2.0f * xt, dv) - 1.0f;
            const float xp = (xn + 1.0f) * half;
            const float x0 = floorf(xp);
            const float w1 = xp - x0, w0 = 1.0f - w1;
            const float nt = n + (float)(t - R);
            const bool lo_ = x0 < nt, hi_ = x0 > nt;
            const float a0 = lo_ ? w[t] : (hi_ ? w[t + 2] : w[t + 1]);
            const float a1 = lo_ ? w[t + 1] : (hi_ ? w[t + 3] : w[t + 2]);
            const bool ok0 = (x0 >= 0.0f) && (x0 <= Wm1);
            const bool ok1 = (x0 + 1.0f >= 0.0f) && (x0 + 1.0f <= Wm1);
            bad |= inwin && (!valid || x0 < nt - 1.0f || x0 > nt + 1.0f);
            const float v0 = ok0 ? a0 : 0.0f;
            const float v1 = ok1 ? a1 : 0.0f;
            res[t] = fmaf(w1, v1, w0 * v0);
        }
        if (__builtin_expect(bad, 0)) {   // one wave-level check per level
            for (int t = 0; t < T; ++t) {
                const float xt = (float)(t - R) + xl;
                const float xn = div_rn(2.0f * xt, dv) - 1.0f;
                const float xp = (xn + 1.0f) * half;
                const float x0 = floorf(xp);
                const float w1 = xp - x0, w0 = 1.0f - w1;
                const bool ok0 = (x0 >= 0.0f) && (x0 <= Wm1);
                const bool ok1 = (x0 + 1.0f >= 0.0f) && (x0 + 1.0f <= Wm1);
                const float v0 = ok0 ? derived_elem<SI>(row1, (long long)x0) : 0.0f;
                const float v1 = ok1 ? derived_elem<SI>(row1, (long long)x0 + 1) : 0.0f;
                res[t] = fmaf(w1, v1, w0 * v0);
            }
        }
        // inactive lanes (tail block) stand in for pixel P-1 and store nothing:
        // with rc_corr_lookup_step in place (coords_out == coords) they may have
        // read coords the real lane already advanced
        if (active) {
#pragma unroll
            for (int t = 0; t < T; ++t)
                if constexpr (M == 5) __builtin_nontemporal_store(res[t], outp + (long long)(i * T + t) * a.HW);
                else if (!NOSTORE || res[t] == 1234.5f) outp[(long long)(i * T + t) * a.HW] = res[t];
        }
    };
    level(std::integral_constant<int, 1>{});
    level(std::integral_constant<int, 2>{});
    if constexpr (TOP >= 3) level(std::integral_constant<int, 3>{});
}

// ---- lookup over a pool-chain pyramid stored as levels 0 and 2 ("pair") ----
// Level 2k+1 element j is the pairwise mean of level-2k elements 2j, 2j+1
// (model.py:294, the fp32 ops (a + b) * 0.5), so ONE span of level 2k feeds
// the windows of both levels 2k and 2k+1:
//   span  = level-2k elements [2(m-R-1), 2(m+R+3)),  m = floor(x / 2^(2k+1))
//   level 2k+1, window element jj (element m-R-1+jj) = mean(span[2jj], span[2jj+1])
//   level 2k,   window element jj (element n-R-1+jj) = span[dd+R+1+jj],
//               n = floor(x / 2^(2k)) = 2m + dd, dd in {0, 1}
// With 4 levels the build stores levels 0 and 2 only and a pixel reads two
// such spans (2(2r+4) elements each): ~2.8 128-B lines per pixel at the bench
// coordinates against ~3.0 for the level-1 chain (level-0 window + level-1
// span) and ~4.4 for one window per level, in 14 instead of
// 16 16-B loads per lane, and with fewer selects.  Window elements outside
// [0, W_level) are zeroed once per level, which is exactly the reference's
// per-tap zero padding (a tap reads window elements x0 and x0+1 only).
template <int R, bool BF16 = false>
struct PairSpan {
    static constexpr int NW = 2 * R + 4;              // window elements per level
    static constexpr int NS = 2 * NW;                 // span elements
    static constexpr int EPC = BF16 ? 8 : 4;          // elements per 16-B chunk
    static constexpr int ES = BF16 ? 2 : 4;           // element bytes
    // the span starts at an even element: misaligned by 0, 2, .., EPC-2
    static constexpr int NC = (NS + EPC - 2 + EPC - 1) / EPC;
    uint32_t q[NC][4];                                // raw chunks
    float m, n;                                       // window centres of the odd / even level
    int sh;                                           // span start - chunk base (elements)
    bool inwin, valid;
    // element e of the loaded chunks, as fp32
    __device__ __forceinline__ float elem(int e) const {
        if constexpr (BF16) {
            const uint32_t u = q[e >> 3][(e & 7) >> 1];
            return __builtin_bit_cast(float, (e & 1) ? (u & 0xFFFF0000u) : (u << 16));
        } else {
            return __builtin_bit_cast(float, q[e >> 2][e & 3]);
        }
    }
};

// Exact element range [f, l] (clipped to [0, W-1]) the taps of one level read.
template <int R>
__device__ __forceinline__ void tap_span(float xl, int W, int &f, int &l) {
    const float Wm1 = (float)(W - 1), half = Wm1 / 2.0f;
    const DivRN dv = div_prep(Wm1);
    const float pa = ((div_rn(2.0f * ((float)(-R) + xl), dv) - 1.0f) + 1.0f) * half;
    const float pb = ((div_rn(2.0f * ((float)R + xl), dv) - 1.0f) + 1.0f) * half;
    f = max((int)floorf(pa), 0);
    l = min((int)floorf(pb) + 1, W - 1);
}

template <int R, bool BF16 = false>
__device__ __forceinline__ void issue_pair(PairSpan<R, BF16> &ps, const LookupArgs &a, int lo, float x,
                                           long long pblk, long long lrow) {
    typedef PairSpan<R, BF16> PS;
    const int Wlo = a.W[lo], Whi = a.W[lo + 1];
    const float xlo = x / (float)(1 << lo), xhi = x / (float)(2 << lo);
    // false for NaN; outside it every tap of both levels is zero padding
    ps.inwin = (xhi > -(float)(R + 4)) && (xhi < (float)(Whi + R + 4));
    ps.m = ps.inwin ? floorf(xhi) : 0.0f;
    ps.n = ps.inwin ? floorf(xlo) : 0.0f;
    const int dd = (int)ps.n - 2 * (int)ps.m;
    ps.valid = ps.inwin && (dd == 0 || dd == 1);      // a subnormal x can break it
    int lo_e = 0x7FFFFFFF, hi_e = -1;
    if (ps.inwin) {
        int f, l;
        tap_span<R>(xlo, Wlo, f, l);
        if (f <= l) { lo_e = f; hi_e = l; }
        tap_span<R>(xhi, Whi, f, l);
        if (f <= l) { lo_e = min(lo_e, 2 * f); hi_e = max(hi_e, 2 * l + 1); }
    }
    const int sa = 2 * ((int)ps.m - R - 1);
    const int ea = sa & ~(PS::EPC - 1);
    ps.sh = sa - ea;
    const long long ld = a.ld[lo];
    const char *lvl = static_cast<const char *>(a.lvl[lo]);
    // RC_SHADOW: the level also lies at +shb bytes, shifted by half a 128-B
    // line; each lane reads its span from the copy in which it touches fewer
    // lines (same values either way).  The resource then spans both copies.
    const long long shb = a.shadow[lo];
    const auto rs = make_rsrc(lvl + pblk * ld * PS::ES, clamp_bytes((a.P - pblk) * ld * PS::ES + shb));
    uint32_t phase = 0;
    if (shb != 0 && lo_e <= hi_e) {
        const unsigned long long b0 =
            (unsigned long long)(uintptr_t)(lvl + ((pblk + lrow) * ld + (lo_e & ~(PS::EPC - 1))) * PS::ES);
        const unsigned long long b1 = (unsigned long long)(uintptr_t)(lvl + ((pblk + lrow) * ld + hi_e) * PS::ES);
        const unsigned long long sh = (unsigned long long)shb;
        const long long l0 = (long long)(b1 >> 7) - (long long)(b0 >> 7);
        const long long l1 = (long long)((b1 + sh) >> 7) - (long long)((b0 + sh) >> 7);
        phase = l1 < l0 ? (uint32_t)sh : 0u;
    }
#pragma unroll
    for (int k = 0; k < PS::NC; ++k) {
        const int cs = ea + PS::EPC * k;
        // lo_e >= 0 and hi_e < Wlo: a loaded chunk starts inside the row and
        // ends inside its 16-B padded extent (ld % EPC == 0)
        const bool ok = cs <= hi_e && cs + PS::EPC - 1 >= lo_e;
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(
            rs, ok ? (int)((uint32_t)((lrow * ld + cs) * PS::ES) + phase) : (int)0xFFFFFF00u, 0, 0);
#pragma unroll
        for (int c = 0; c < 4; ++c) ps.q[k][c] = v[c];
    }
}

// Taps of one level from its zero-padded window w[NW] (element nwin-R-1+jj),
// the reference's fp32 sequence (see lookup_kernel).  No per-tap check that
// the tap's floor stayed in the window is needed here, because it cannot leave
// it: for a lane in the window's range (|xl| < W + R + 4) and W <= 2^16,
//  (1) xt = fl(xl + k) lies in [m, m + 1] with m = floor(xl) + k = nt
//      (integers are representable and rounding is monotone);
//  (2) the round trip xp = fl(fl(fl(fl(2 xt)/(W-1)) - 1) + 1) * (W-1)/2
//      differs from xt by at most (4|xt| + 1.5(W-1)) 2^-24 < 0.03;
// so x0 = floor(xp) is nt - 1, nt or nt + 1 (nt + 2 would need xt = nt + 1
// and an error >= 1), i.e. taps x0 and x0 + 1 are window elements t..t+3.
// The C-ABI rejects wider levels for this kernel (include/raftcorr.h).
template <int R>
__device__ __forceinline__ void window_taps(const float *w, float xl, float nwin, int W,
                                            float *res) {
    constexpr int T = 2 * R + 1;
    const float Wm1 = (float)(W - 1), half = Wm1 / 2.0f;
    const DivRN dv = div_prep(Wm1);
#pragma unroll
    for (int t = 0; t < T; ++t) {
        const float xt = (float)(t - R) + xl;
        const float xn = div_rn(2.0f * xt, dv) - 1.0f;
        const float xp = (xn + 1.0f) * half;
        const float x0 = floorf(xp);
        const float w1 = xp - x0, w0 = 1.0f - w1;
        const float nt = nwin + (float)(t - R);
        const bool lo_ = x0 < nt, hi_ = x0 > nt;
        // opaque copies: the selects must stay selects of registers (folded
        // into a load from a select of addresses, the window goes to scratch
        // memory: 112 B/lane and 87 instead of 14 vector loads per wave)
        float e0 = w[t], e1 = w[t + 1], e2 = w[t + 2], e3 = w[t + 3];
        asm("" : "+v"(e0), "+v"(e1), "+v"(e2), "+v"(e3));
        const float v0 = lo_ ? e0 : (hi_ ? e2 : e1);
        const float v1 = lo_ ? e1 : (hi_ ? e3 : e2);
        res[t] = fmaf(w1, v1, w0 * v0);
    }
}

// The memory path for a lane whose level pair breaks the span relation
// n = 2m + dd (only a subnormal x can): every tap re-read, level-i element k
// = pool of S consecutive span-level elements.
// level-i element k (S consecutive bf16 span-level elements, each level of
// the chain rounded to bf16 as stored)
template <int S>
__device__ __forceinline__ float derived_elem_bf16(const uint16_t *row, long long k) {
    if constexpr (S == 1) {
        return bf16_to_f32(row[k]);
    } else {
        const float a = derived_elem_bf16<S / 2>(row, 2 * k), b = derived_elem_bf16<S / 2>(row, 2 * k + 1);
        return round_bf16((a + b) * 0.5f);
    }
}

template <int R, int S, bool BF16 = false>
__device__ __forceinline__ void level_taps_mem(const void *rowv, float xl, int W, float *res) {
    constexpr int T = 2 * R + 1;
    const float Wm1 = (float)(W - 1), half = Wm1 / 2.0f;
    const DivRN dv = div_prep(Wm1);
    for (int t = 0; t < T; ++t) {
        const float xt = (float)(t - R) + xl;
        const float xn = div_rn(2.0f * xt, dv) - 1.0f;
        const float xp = (xn + 1.0f) * half;
        const float x0 = floorf(xp);
        const float w1 = xp - x0, w0 = 1.0f - w1;
        const bool ok0 = (x0 >= 0.0f) && (x0 <= Wm1);
        const bool ok1 = (x0 + 1.0f >= 0.0f) && (x0 + 1.0f <= Wm1);
        float v0 = 0.0f, v1 = 0.0f;
        if constexpr (BF16) {
            const uint16_t *row = static_cast<const uint16_t *>(rowv);
            if (ok0) v0 = derived_elem_bf16<S>(row, (long long)x0);
            if (ok1) v1 = derived_elem_bf16<S>(row, (long long)x0 + 1);
        } else {
            const float *row = static_cast<const float *>(rowv);
            if (ok0) v0 = derived_elem<S>(row, (long long)x0);
            if (ok1) v1 = derived_elem<S>(row, (long long)x0 + 1);
        }
        res[t] = fmaf(w1, v1, w0 * v0);
    }
}

template <int R, bool NOFALLBACK = false, bool BF16 = false, class Sink>
__device__ __forceinline__ void finish_pair(const PairSpan<R, BF16> &ps, const LookupArgs &a, int lo,
                                            float x, long long pp, Sink &&sink) {
    typedef PairSpan<R, BF16> PS;
    constexpr int T = 2 * R + 1, NW = PS::NW, NS = PS::NS, EPC = PS::EPC;
    const int Wlo = a.W[lo], Whi = a.W[lo + 1];
    // span element j = chunk element j + sh, sh in {0, 2, .., EPC-2}
    float s[NS];
#pragma unroll
    for (int j = 0; j < NS; ++j) {
        float v = ps.elem(j);
#pragma unroll
        for (int d = 2; d < EPC; d += 2)
            if (j + d < PS::NC * EPC) v = (ps.sh == d) ? ps.elem(j + d) : v;
        s[j] = v;
    }
    const int mi = (int)ps.m - R - 1, ni = (int)ps.n - R - 1;
    const int dd = (int)ps.n - 2 * (int)ps.m;
    float wodd[NW], weven[NW];
#pragma unroll
    for (int jj = 0; jj < NW; ++jj) {
        float pm = (s[2 * jj] + s[2 * jj + 1]) * 0.5f;      // model.py:294 in fp32
        if constexpr (BF16) pm = round_bf16(pm);           // the odd level as stored
        wodd[jj] = (unsigned)(mi + jj) < (unsigned)Whi ? pm : 0.0f;
        const float e = dd == 0 ? s[R + 1 + jj] : s[R + 2 + jj];
        weven[jj] = (unsigned)(ni + jj) < (unsigned)Wlo ? e : 0.0f;
    }
    const float xlo = x / (float)(1 << lo), xhi = x / (float)(2 << lo);
    float r0[T], r1[T];
    window_taps<R>(weven, xlo, ps.n, Wlo, r0);
    window_taps<R>(wodd, xhi, ps.m, Whi, r1);
    if (!NOFALLBACK && __builtin_expect(ps.inwin && !ps.valid, 0)) {   // subnormal x only
        const char *row = static_cast<const char *>(a.lvl[lo]) + pp * a.ld[lo] * PS::ES;
        level_taps_mem<R, 1, BF16>(row, xlo, Wlo, r0);
        level_taps_mem<R, 2, BF16>(row, xhi, Whi, r1);
    }
#pragma unroll
    for (int t = 0; t < T; ++t) sink(lo * T + t, r0[t]);
#pragma unroll
    for (int t = 0; t < T; ++t) sink((lo + 1) * T + t, r1[t]);
}

// One lane's pixel of one group: index, x, output pointer, rsrc base row.
struct PairPixel {
    long long pblk, pp, lrow;
    float *outp;
    float x;
    bool active;
};

template <int R, int NL>
__device__ __forceinline__ PairPixel pair_pixel(const LookupArgs &a, long long pblk) {
    PairPixel q;
    q.pblk = pblk;
    const long long p = pblk + threadIdx.x;
    q.active = p < a.P;
    q.pp = q.active ? p : a.P - 1;
    const long long bimg = q.pp / a.HW, rem = q.pp - bimg * a.HW;
    q.x = pixel_x(a, bimg, rem, q.active);
    q.outp = a.out + bimg * (long long)(NL * (2 * R + 1)) * a.HW + rem;
    q.lrow = q.pp - pblk;
    return q;
}

// NL = 2 (levels 0-1) or 4 (levels 0-3; level 2 stored, levels 1 and 3 derived).
// Both spans' loads issue first; pair 0's math and stores run while pair 2's
// loads are in flight.  Measured and not kept: 16-B output
// stores through a per-wave LDS tile (9 instead of 36 store instructions per
// wave: 26.0 vs 25.8 us), two pixels per lane with both pixels' loads in
// flight (26.6 us, 198 VGPRs).
// M: ablation modes (dev library only, dev/lookup_dev.inc): 1 = no output
// stores, 2 = no fallback path, 5 = hardware block order (no XCD remap; same
// values), 7 = non-temporal output stores, 9 = the channels-last store path
// writing into an NCHW buffer (timing A/B of the two layouts); WPE caps
// registers for 5/6 waves/SIMD.
template <int R, int NL, int M = 0, bool BF16 = false, int WPE = 1, bool CL = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void lookup_pair_kernel(LookupArgs a) {
    static_assert(NL == 2 || NL == 4, "pair lookup: 2 or 4 levels");
    constexpr int NP = NL / 2;                        // spans per pixel
    // XCD-contiguous block order: neighbouring pixel blocks, whose output
    // rows share 128-B lines at every channel plane's seams, run on one XCD
    // (kitti B=64: 172 -> 166 us; config 2 unchanged; dev variant 205 = off)
    const int blk = M == 5 ? (int)blockIdx.x : xcd_remap(blockIdx.x, gridDim.x);
    const PairPixel q = pair_pixel<R, NL>(a, (long long)blk * 256);
    PairSpan<R, BF16> sp[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k)
        issue_pair<R, BF16>(sp[k], a, 2 * k, q.x, q.pblk, q.lrow);
    constexpr int C = NL * (2 * R + 1);
    // CL: channels-last output (RC_OUT_CHANNELS_LAST), out[p*C + ch].  A
    // wave's 64 pixels own one contiguous run of 64*C floats; it is gathered
    // in a per-wave LDS tile and written as 16-B vectors, 1 KB per store
    // instruction (instead of C dword stores, 256 B each, to C channel planes)
    constexpr bool TILE = CL || M == 9;
    __shared__ __attribute__((aligned(16))) float ctile[TILE ? 4 * 64 * C : 1];
    auto sink = [&](int ch, float v) {
        if constexpr (TILE) {
            ctile[(threadIdx.x >> 6) * 64 * C + (threadIdx.x & 63) * C + ch] = v;
        } else if constexpr (M == 7) {        // dev: non-temporal output stores
            if (q.active) __builtin_nontemporal_store(v, q.outp + (long long)ch * a.HW);
        } else {
            if (q.active && (M != 1 || v == 1234.5f)) q.outp[(long long)ch * a.HW] = v;
        }
    };
#pragma unroll
    for (int k = 0; k < NP; ++k) finish_pair<R, M == 2, BF16>(sp[k], a, 2 * k, q.x, q.pp, sink);
    if constexpr (TILE) {
        // the wave's tile is private and LDS runs a wave's operations in
        // order: no barrier.  The run starts 256*C-byte aligned.
        const int lane = threadIdx.x & 63;
        const long long pw = q.pblk + (threadIdx.x & ~63);
        const float *t = ctile + (threadIdx.x >> 6) * 64 * C;
        const long long lim = (a.P - pw < 64 ? a.P - pw : 64) * C;   // valid elements of the run
#pragma unroll
        for (int k = 0; k < (16 * C + 63) / 64; ++k) {
            const int e = (k * 64 + lane) * 4;             // element of the wave's [64][C] run
            if (e >= 64 * C || e >= lim) continue;
            const f32x4 v = *reinterpret_cast<const f32x4 *>(t + e);
            if (e + 4 <= lim) {
                *reinterpret_cast<f32x4 *>(a.out + pw * C + e) = v;
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (e + j < lim) a.out[pw * C + e + j] = v[j];
            }
        }
    }
}

// finish_pair's memory path over the disparity-major layout: every tap of
// level lo (stored) and lo + 1 (its pairwise means) re-read, the fp32 ops of
// level_taps_mem.
template <int R, class Sink>
__device__ __forceinline__ void sheared_taps_mem(const LookupArgs &a, int lo, float x, long long bh, int w1,
                                                 Sink &&sink) {
    constexpr int T = 2 * R + 1;
    const float *S = static_cast<const float *>(a.lvl[lo]) + bh * a.shk[lo] * a.ld[lo];
    const int W0 = a.W[lo];
    const long long base = (long long)((w1 >> lo) + W0 - 1);        // row of element 0 is base - j
    auto elem = [&](long long j) { return S[(base - j) * a.ld[lo] + w1]; };
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        const int W = a.W[lo + half];
        const float Wm1 = (float)(W - 1), hw = Wm1 / 2.0f;
        const DivRN dv = div_prep(Wm1);
        const float xl = x / (float)(1 << (lo + half));
        for (int t = 0; t < T; ++t) {
            const float xt = (float)(t - R) + xl;
            const float xn = div_rn(2.0f * xt, dv) - 1.0f;
            const float xp = (xn + 1.0f) * hw;
            const float x0 = floorf(xp);
            const float wt1 = xp - x0, wt0 = 1.0f - wt1;
            const bool ok0 = (x0 >= 0.0f) && (x0 <= Wm1);
            const bool ok1 = (x0 + 1.0f >= 0.0f) && (x0 + 1.0f <= Wm1);
            const long long e = (long long)x0;
            float v0 = 0.0f, v1 = 0.0f;
            if (half == 0) {
                if (ok0) v0 = elem(e);
                if (ok1) v1 = elem(e + 1);
            } else {
                if (ok0) v0 = (elem(2 * e) + elem(2 * e + 1)) * 0.5f;
                if (ok1) v1 = (elem(2 * e + 2) + elem(2 * e + 3)) * 0.5f;
            }
            sink((lo + half) * T + t, fmaf(wt1, v1, wt0 * v0));
        }
    }
}

// ---- lookup over a disparity-major pair layout (RC_LAYOUT_DISPARITY) ----
// The pair kernel's arithmetic (levels 0 and 2 stored, 1 and 3 their
// pairwise means, finish_pair: bit-identical) over levels stored as
// S_i[b,h][k][w1], k = (w1 >> i) - j + W_i - 1 (rc_corr_build with the
// flag; a.shk[i] rows of a.ld[i] floats per image row): the lanes of a wave
// whose pixels look at the same disparity read one contiguous run of a row
// per span element -- coalesced along w1 -- instead of a 16-B piece of 64
// different pixel rows.  A span is 2(2r+4) dword loads per lane (exact-span
// predicated).  Faster than the row layout where neighbouring pixels' coords
// agree (the network's own fields), slower on independent random ones
// (DESIGN.md §3.2h).
template <int R, int NL>
__global__ __launch_bounds__(256) void lookup_sheared_pair_kernel(LookupArgs a) {
    static_assert(NL == 2 || NL == 4, "pair lookup: 2 or 4 levels");
    constexpr int NP = NL / 2, NS = PairSpan<R>::NS;
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const long long pblk = (long long)blk * 256;
    const long long p = pblk + threadIdx.x;
    const bool active = p < a.P;
    const long long pp = active ? p : a.P - 1;
    const long long bimg = pp / a.HW, rem = pp - bimg * a.HW;
    const float x = pixel_x(a, bimg, rem, active);
    const int H = a.HW / a.W1;
    const int h = (int)(rem / a.W1), w1 = (int)(rem - (long long)h * a.W1);
    const long long bh = bimg * H + h, bh0 = pblk / a.W1;          // bh0: block-uniform
    float *outp = a.out + bimg * (long long)(NL * (2 * R + 1)) * a.HW + rem;
    auto sink = [&](int ch, float v) {
        if (active) outp[(long long)ch * a.HW] = v;
    };
    PairSpan<R> sp[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) {
        const int lo = 2 * k;
        PairSpan<R> &ps = sp[k];
        const int Wlo = a.W[lo], Whi = a.W[lo + 1];
        const float xlo = x / (float)(1 << lo), xhi = x / (float)(2 << lo);
        ps.inwin = (xhi > -(float)(R + 4)) && (xhi < (float)(Whi + R + 4));
        ps.m = ps.inwin ? floorf(xhi) : 0.0f;
        ps.n = ps.inwin ? floorf(xlo) : 0.0f;
        const int dd = (int)ps.n - 2 * (int)ps.m;
        ps.valid = ps.inwin && (dd == 0 || dd == 1);
        int lo_e = 0x7FFFFFFF, hi_e = -1;
        if (ps.inwin) {
            int f, l;
            tap_span<R>(xlo, Wlo, f, l);
            if (f <= l) { lo_e = f; hi_e = l; }
            tap_span<R>(xhi, Whi, f, l);
            if (f <= l) { lo_e = min(lo_e, 2 * f); hi_e = max(hi_e, 2 * l + 1); }
        }
        ps.sh = 0;
        const int sa = 2 * ((int)ps.m - R - 1);
        const long long K = a.shk[lo], ldw = a.ld[lo];
        const float *lv = static_cast<const float *>(a.lvl[lo]);
        const auto rs = make_rsrc(lv + bh0 * K * ldw, clamp_bytes((a.P / a.W1 - bh0) * K * ldw * 4));
        const long long rowk = (bh - bh0) * K + (w1 >> lo) + Wlo - 1;    // row of element 0
#pragma unroll
        for (int c = 0; c < PairSpan<R>::NC * 4; ++c) {
            const int j = sa + c;
            const bool ok = c < NS && j >= lo_e && j <= hi_e;
            const uint32_t off = ok ? (uint32_t)(((rowk - j) * ldw + w1) * 4) : 0xFFFFFF00u;
            ps.q[c >> 2][c & 3] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)off, 0, 0);
        }
    }
    // a subnormal x (the only way to break n = 2m + dd) takes the memory path
    // of finish_pair, which reads the row layout: not available here, so the
    // taps of such a lane come from sheared_taps_mem below instead
#pragma unroll
    for (int k = 0; k < NP; ++k) {
        if (__builtin_expect(sp[k].inwin && !sp[k].valid, 0)) {
            sheared_taps_mem<R>(a, 2 * k, x, bh, w1, sink);
            continue;
        }
        finish_pair<R, true>(sp[k], a, 2 * k, x, pp, sink);
    }
}

// ---- lookup over the record layout (RC_LAYOUT_RECORDS, bf16, 4 levels) ----
// Each pixel row holds a.rec_nr 128-B records (rc_corr_build with the flag;
// geometry in common.h): record r has level-2 elements rec_e2(r) .. +25 in
// slots 0..25 and level-0 elements rec_e0(r) .. +37 in slots 26..63, so a
// pixel whose level-1 centre m1 = floor(x/2) lies in [8r - 8, 8r) finds both
// of its pair spans (level 0's from 2(m1 - R - 1), level 2's from
// 2(floor(m1/4) - R - 1)) in record r: ONE 128-B line per pixel instead of
// two.  A pixel outside the records' m1 range takes the
// nearest record; its exact spans are then empty or lie at the row edge that
// record covers.  The chunks are read with issue_pair's exact-span predicate
// and finish_pair runs unchanged, so the output is the row layout's bit for
// bit.

// issue_pair over a record: level-lo element e sits in slot e - e_first + slot_first.
// plan_record_pair fills the span's window fields and returns the first
// chunk's slot (cb, a multiple of 8) and which of the NC chunks the taps read.
template <int R>
__device__ __forceinline__ int plan_record_pair(PairSpan<R, true> &ps, const LookupArgs &a, int lo, float x,
                                                int e_first, int slot_first, uint32_t &okmask) {
    typedef PairSpan<R, true> PS;
    const int Wlo = a.W[lo], Whi = a.W[lo + 1];
    const float xlo = x / (float)(1 << lo), xhi = x / (float)(2 << lo);
    ps.inwin = (xhi > -(float)(R + 4)) && (xhi < (float)(Whi + R + 4));
    ps.m = ps.inwin ? floorf(xhi) : 0.0f;
    ps.n = ps.inwin ? floorf(xlo) : 0.0f;
    const int dd = (int)ps.n - 2 * (int)ps.m;
    ps.valid = ps.inwin && (dd == 0 || dd == 1);
    int lo_e = 0x7FFFFFFF, hi_e = -1;
    if (ps.inwin) {
        int f, l;
        tap_span<R>(xlo, Wlo, f, l);
        if (f <= l) { lo_e = f; hi_e = l; }
        tap_span<R>(xhi, Whi, f, l);
        if (f <= l) { lo_e = min(lo_e, 2 * f); hi_e = max(hi_e, 2 * l + 1); }
    }
    const int sslot = 2 * ((int)ps.m - R - 1) - e_first + slot_first;   // span start (even)
    const int cb = sslot >= 0 ? sslot & ~7 : -((-sslot + 7) & ~7);      // chunk base (floor to 8)
    ps.sh = sslot - cb;
    const int slo = lo_e - e_first + slot_first, shi = hi_e - e_first + slot_first;
    okmask = 0;
#pragma unroll
    for (int k = 0; k < PS::NC; ++k) {
        const int cs = cb + 8 * k;
        if (lo_e <= hi_e && cs <= shi && cs + 7 >= slo && cs >= 0 && cs + 8 <= kRecSlots) okmask |= 1u << k;
    }
    return cb;
}

template <int R, bool NOLOAD = false>
__device__ __forceinline__ void issue_record_pair(PairSpan<R, true> &ps, const LookupArgs &a, int lo, float x,
                                                  const __amdgpu_buffer_rsrc_t &rs, uint32_t rbyte, int e_first,
                                                  int slot_first) {
    typedef PairSpan<R, true> PS;
    uint32_t okm;
    const int cb = plan_record_pair<R>(ps, a, lo, x, e_first, slot_first, okm);
#pragma unroll
    for (int k = 0; k < PS::NC; ++k) {
        const int cs = cb + 8 * k;
        const bool ok = (okm >> k) & 1u;
        if constexpr (NOLOAD) {   // dev timing: the addresses, not the loads
            uint32_t o = ok ? rbyte + 2u * (uint32_t)cs : 0u;
            asm volatile("" : "+v"(o));
#pragma unroll
            for (int c = 0; c < 4; ++c) ps.q[k][c] = o + c;
        } else {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(
                rs, ok ? (int)(rbyte + 2u * (uint32_t)cs) : (int)0xFFFFFF00u, 0, 0);
#pragma unroll
            for (int c = 0; c < 4; ++c) ps.q[k][c] = v[c];
        }
    }
}

// The same chunks from the pixel's whole record staged in LDS (COOP).
template <int R>
__device__ __forceinline__ void lds_record_pair(PairSpan<R, true> &ps, const LookupArgs &a, int lo, float x,
                                                const char *rec, int e_first, int slot_first) {
    typedef PairSpan<R, true> PS;
    uint32_t okm;
    const int cb = plan_record_pair<R>(ps, a, lo, x, e_first, slot_first, okm);
#pragma unroll
    for (int k = 0; k < PS::NC; ++k) {
        const int cs = cb + 8 * k;
        uint4 v = uint4{0u, 0u, 0u, 0u};
        if ((okm >> k) & 1u) v = *reinterpret_cast<const uint4 *>(rec + 2 * cs);
        ps.q[k][0] = v.x;
        ps.q[k][1] = v.y;
        ps.q[k][2] = v.z;
        ps.q[k][3] = v.w;
    }
}

// finish_pair's memory path over the records (a subnormal x, the only way to
// break n = 2m + dd): level lo (0 or 2) element e from a record that holds
// it, level lo + 1 the bf16-rounded pairwise mean, the ops of level_taps_mem
template <int R, class Sink>
__device__ __forceinline__ void record_taps_mem(const LookupArgs &a, const uint16_t *rec, int lo, float x,
                                                Sink &&sink) {
    constexpr int T = 2 * R + 1;
    const int NR = a.rec_nr;
    auto elem = [&](long long e) {
        int r = lo == 0 ? (int)((e - rec_e0(0)) >> 4) : (int)((e - rec_e2(0)) >> 2);
        r = r < NR ? r : NR - 1;
        const int slot = lo == 0 ? kRecL2Slots + (int)e - rec_e0(r) : (int)e - rec_e2(r);
        return bf16_to_f32(rec[r * kRecSlots + slot]);
    };
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        const int W = a.W[lo + half];
        const float Wm1 = (float)(W - 1), hw = Wm1 / 2.0f;
        const DivRN dv = div_prep(Wm1);
        const float xl = x / (float)(1 << (lo + half));
        for (int t = 0; t < T; ++t) {
            const float xt = (float)(t - R) + xl;
            const float xn = div_rn(2.0f * xt, dv) - 1.0f;
            const float xp = (xn + 1.0f) * hw;
            const float x0 = floorf(xp);
            const float wt1 = xp - x0, wt0 = 1.0f - wt1;
            const bool ok0 = (x0 >= 0.0f) && (x0 <= Wm1);
            const bool ok1 = (x0 + 1.0f >= 0.0f) && (x0 + 1.0f <= Wm1);
            const long long e = (long long)x0;
            float v0 = 0.0f, v1 = 0.0f;
            if (half == 0) {
                if (ok0) v0 = elem(e);
                if (ok1) v1 = elem(e + 1);
            } else {
                if (ok0) v0 = round_bf16((elem(2 * e) + elem(2 * e + 1)) * 0.5f);
                if (ok1) v1 = round_bf16((elem(2 * e + 2) + elem(2 * e + 3)) * 0.5f);
            }
            sink((lo + half) * T + t, fmaf(wt1, v1, wt0 * v0));
        }
    }
}

// CL: channels-last output (RC_OUT_CHANNELS_LAST) through the per-wave LDS
// tile of lookup_pair_kernel; else NCHW dword stores.  COOP (the product)
// see below; without it each lane loads its own chunks (the dev A/B).  M: dev timing modes
// (libraftcorr_dev.so, wrong output): 1 no output stores, 2 no record loads,
// 3 record loads only (no tap math, no stores).
// COOP: each wave's 64 records are fetched whole, eight 128-B lines per
// buffer_load ... lds instruction (lane L: record 8k + L/8, 16-B chunk L % 8)
// into a per-wave LDS image, then each lane reads its chunks from there:
// 8 line requests per instruction instead of 64 partial ones.
template <int R, bool CL, int M = 0, bool COOP = false, int WPE = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void lookup_records_kernel(LookupArgs a) {
    constexpr int NL = 4, C = NL * (2 * R + 1);
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const PairPixel q = pair_pixel<R, NL>(a, (long long)blk * 256);
    const int NR = a.rec_nr;
    // the pixel's record (clamped as floats before the integer cast: NaN -> 0)
    float mf = floorf(q.x / 2.0f);
    mf = fminf(fmaxf(mf, (float)kRecM0), (float)(kRecM0 + 8 * NR - 1));
    const int r = ((int)mf - kRecM0) >> 3;
    const uint16_t *blkrec = static_cast<const uint16_t *>(a.lvl[0]) + q.pblk * (long long)NR * kRecSlots;
    // the block's records (< 4 GiB: 256 rows of <= 22 lines)
    const auto rs = make_rsrc(blkrec, clamp_bytes((a.P - q.pblk) * (long long)NR * kRecSlots * 2));
    const uint32_t rbyte = (uint32_t)((q.lrow * NR + r) * kRecSlots * 2);
    PairSpan<R, true> sp[2];
    // per wave: the staged records (8 KB), then the channels-last tile
    // (64 C floats, 9 KB at R = 4) in the same bytes once they are read
    constexpr int WB = CL ? (COOP && 64 * C * 4 < 8192 ? 8192 : 64 * C * 4) : (COOP ? 8192 : 16);
    __shared__ __attribute__((aligned(16))) char lds[4 * WB];
    char *wlds = lds + (threadIdx.x >> 6) * WB;
    if constexpr (COOP) {
        typedef __attribute__((address_space(3))) void lds_void;
        const int lane = threadIdx.x & 63;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            // record of pixel 8k + lane/8 of this wave, its chunk lane % 8
            const uint32_t rb = (uint32_t)__shfl((int)rbyte, 8 * k + (lane >> 3), 64);
            const int wp = (int)(threadIdx.x & ~63) + 8 * k + (lane >> 3);
            const uint32_t off = q.pblk + wp < a.P ? rb + 16u * (uint32_t)(lane & 7) : 0xFFFFFF00u;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void *)(wlds + 1024 * k), 16, (int)off, 0, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const char *myrec = wlds + 128 * lane;
        lds_record_pair<R>(sp[0], a, 0, q.x, myrec, rec_e0(r), kRecL2Slots);
        lds_record_pair<R>(sp[1], a, 2, q.x, myrec, rec_e2(r), 0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // all reads done before the tile reuses the bytes
    } else {
        issue_record_pair<R, M == 2>(sp[0], a, 0, q.x, rs, rbyte, rec_e0(r), kRecL2Slots);
        issue_record_pair<R, M == 2>(sp[1], a, 2, q.x, rs, rbyte, rec_e2(r), 0);
    }
    if constexpr (M == 3) {   // dev: the loads alone
        uint32_t acc = 0;
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
            for (int j = 0; j < PairSpan<R, true>::NC; ++j) acc ^= sp[k].q[j][0] ^ sp[k].q[j][1] ^ sp[k].q[j][2] ^ sp[k].q[j][3];
        asm volatile("" ::"v"(acc));
        return;
    }
    float *const ctw = reinterpret_cast<float *>(wlds);       // this wave's channels-last tile
    auto sink = [&](int ch, float v) {
        if constexpr (CL) ctw[(threadIdx.x & 63) * C + ch] = v;
        else if (q.active) q.outp[(long long)ch * a.HW] = v;
    };
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        if (__builtin_expect(sp[k].inwin && !sp[k].valid, 0)) {
            record_taps_mem<R>(a, blkrec + q.lrow * (long long)NR * kRecSlots, 2 * k, q.x, sink);
            continue;
        }
        finish_pair<R, true, true>(sp[k], a, 2 * k, q.x, q.pp, sink);
    }
    if constexpr (CL) {
        const int lane = threadIdx.x & 63;
        const long long pw = q.pblk + (threadIdx.x & ~63);
        const float *t = ctw;
        const long long lim = (a.P - pw < 64 ? a.P - pw : 64) * C;
#pragma unroll
        for (int k = 0; k < (16 * C + 63) / 64; ++k) {
            const int e = (k * 64 + lane) * 4;
            if (e >= 64 * C || e >= lim) continue;
            const f32x4 v = *reinterpret_cast<const f32x4 *>(t + e);
            if constexpr (M == 1) {   // dev: no output stores
                asm volatile("" ::"v"(v));
            } else if (e + 4 <= lim) {
                *reinterpret_cast<f32x4 *>(a.out + pw * C + e) = v;
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (e + j < lim) a.out[pw * C + e + j] = v[j];
            }
        }
    }
}

// One 64-pixel group of the record lookup: pixels, records, fetch offset.
struct RecGroup {
    PairPixel q;
    int r;
    const uint16_t *blkrec;
    __amdgpu_buffer_rsrc_t rs;
    uint32_t rbyte;
};

// Two 64-pixel groups per wave (dev A/B, RAFTCORR_REC_LOOKUP=10/11): both
// groups' records are fetched cooperatively up front, so the second group's
// lines are in flight while the first group's taps are computed; block b
// covers pixels [512b, 512b + 512), wave w groups w and w + 4.  LDS per wave:
// 9 KB (group A's records, then each group's channels-last tile) + 8 KB
// (group B's records): two blocks per CU.
template <int R, bool CL>
__global__ __launch_bounds__(256) void lookup_records2_kernel(LookupArgs a) {
    constexpr int NL = 4, C = NL * (2 * R + 1);
    constexpr int TB = CL && 64 * C * 4 > 8192 ? 64 * C * 4 : 8192;
    __shared__ __attribute__((aligned(16))) char lds[4 * (TB + 8192)];
    typedef __attribute__((address_space(3))) void lds_void;
    const int lane = threadIdx.x & 63;
    char *bufA = lds + (threadIdx.x >> 6) * (TB + 8192), *bufB = bufA + TB;
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const int NR = a.rec_nr;
    auto setup = [&](long long pblk) {
        RecGroup g;
        g.q = pair_pixel<R, NL>(a, pblk);
        float mf = floorf(g.q.x / 2.0f);
        mf = fminf(fmaxf(mf, (float)kRecM0), (float)(kRecM0 + 8 * NR - 1));
        g.r = ((int)mf - kRecM0) >> 3;
        g.blkrec = static_cast<const uint16_t *>(a.lvl[0]) + g.q.pblk * (long long)NR * kRecSlots;
        g.rs = make_rsrc(g.blkrec, clamp_bytes((a.P - g.q.pblk) * (long long)NR * kRecSlots * 2));
        g.rbyte = (uint32_t)((g.q.lrow * NR + g.r) * kRecSlots * 2);
        return g;
    };
    auto fetch = [&](const RecGroup &g, char *buf) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t rb = (uint32_t)__shfl((int)g.rbyte, 8 * k + (lane >> 3), 64);
            const int wp = (int)(threadIdx.x & ~63) + 8 * k + (lane >> 3);
            const uint32_t off = g.q.pblk + wp < a.P ? rb + 16u * (uint32_t)(lane & 7) : 0xFFFFFF00u;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(g.rs, (lds_void *)(buf + 1024 * k), 16, (int)off, 0, 0, 0);
        }
    };
    // the group's taps from its staged records; CL: into the tile at bufA
    auto compute = [&](const RecGroup &g, const char *recbuf) {
        PairSpan<R, true> sp[2];
        const char *myrec = recbuf + 128 * lane;
        lds_record_pair<R>(sp[0], a, 0, g.q.x, myrec, rec_e0(g.r), kRecL2Slots);
        lds_record_pair<R>(sp[1], a, 2, g.q.x, myrec, rec_e2(g.r), 0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        float *const ctw = reinterpret_cast<float *>(bufA);
        auto sink = [&](int ch, float v) {
            if constexpr (CL) ctw[lane * C + ch] = v;
            else if (g.q.active) g.q.outp[(long long)ch * a.HW] = v;
        };
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            if (__builtin_expect(sp[k].inwin && !sp[k].valid, 0)) {
                record_taps_mem<R>(a, g.blkrec + g.q.lrow * (long long)NR * kRecSlots, 2 * k, g.q.x, sink);
                continue;
            }
            finish_pair<R, true, true>(sp[k], a, 2 * k, g.q.x, g.q.pp, sink);
        }
    };
    auto store_tile = [&](const RecGroup &g) {
        if constexpr (CL) {
            const long long pw = g.q.pblk + (threadIdx.x & ~63);
            const float *t = reinterpret_cast<const float *>(bufA);
            const long long lim = (a.P - pw < 64 ? a.P - pw : 64) * C;
#pragma unroll
            for (int k = 0; k < (16 * C + 63) / 64; ++k) {
                const int e = (k * 64 + lane) * 4;
                if (e >= 64 * C || e >= lim) continue;
                const f32x4 v = *reinterpret_cast<const f32x4 *>(t + e);
                if (e + 4 <= lim) {
                    *reinterpret_cast<f32x4 *>(a.out + pw * C + e) = v;
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (e + j < lim) a.out[pw * C + e + j] = v[j];
                }
            }
        }
    };
    const RecGroup ga = setup((long long)blk * 512), gb = setup((long long)blk * 512 + 256);
    fetch(ga, bufA);
    fetch(gb, bufB);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");            // group A's 8 DMA landed
    compute(ga, bufA);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");            // group B's (and, NCHW, A's stores)
    store_tile(ga);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");          // tile A read: bufA free again
    compute(gb, bufB);
    store_tile(gb);
}

template <int R, int NL, bool BF16, bool EXACT, int BS = 256, int WPE = 1>
static void launch_k(const LookupArgs &a, hipStream_t s) {
    const unsigned nblk = (unsigned)((a.P + BS - 1) / BS);
    hipLaunchKernelGGL((lookup_kernel<R, NL, BF16, EXACT, BS, WPE>), dim3(nblk), dim3(BS), 0, s, a);
}

// Below this many pixels the launch cannot fill the chip with the 256-thread
// runtime-loop kernel (one dependent memory round trip per level): use
// 64-thread blocks and issue every level's loads up front instead.
constexpr long long kSmallP = 256LL * 256 * 2;
// Below this many pixels one wave per (64 pixels, level) still leaves the
// chip under-filled or about full: lookup_levelpar_kernel.
constexpr long long kLevelParP = 64LL * 1024;

// ---- lookup fused with the motion encoder's convc1 (+ ReLU) ----
// BasicMotionEncoder.convc1 (model.py:199, :206) is a 1x1 conv over the
// lookup's NL*(2r+1) channels: out[c] = relu(bias[c] + sum_k W[c][k] corr[k]).
// The lane keeps its pixel's corr values in registers (levels unrolled, so
// every index is static) and never writes them; the weights are read with
// wave-uniform addresses (scalar loads).  Summation order: bias, then k
// ascending, one fmaf each.
// PRE (default): every level's loads issue before any tap math (NL windows
// live at once) instead of one level's round trip at a time: 52.9 vs 57.5 us
// at config 2, bit-identical.
template <int R, int NL, bool BF16, bool PRE = true>
__global__ __launch_bounds__(256) void lookup_conv_kernel(LookupArgs a, const float *__restrict__ wgt,
                                                          const float *__restrict__ bias, int cout,
                                                          int relu, float *__restrict__ out) {
    constexpr int T = 2 * R + 1, CIN = NL * T;
    const long long pblk = (long long)blockIdx.x * 256;
    const long long p = pblk + threadIdx.x;
    const bool active = p < a.P;
    const long long pp = active ? p : a.P - 1;
    const long long bimg = pp / a.HW, rem = pp - bimg * a.HW;
    const float x = pixel_x(a, bimg, rem, active);
    const long long lrow = pp - pblk;
    float corr[CIN];
    if constexpr (PRE) {
        LevelWindow<R, BF16> lw[NL];
#pragma unroll
        for (int i = 0; i < NL; ++i) issue_level<R, BF16, true>(lw[i], a, i, x, pblk, lrow);
#pragma unroll
        for (int i = 0; i < NL; ++i)
            finish_level<R, BF16>(lw[i], a, i, pblk, lrow, [&](int t, float v) { corr[i * T + t] = v; });
    } else {
#pragma unroll
        for (int i = 0; i < NL; ++i) {
            LevelWindow<R, BF16> lw;
            issue_level<R, BF16, true>(lw, a, i, x, pblk, lrow);
            finish_level<R, BF16>(lw, a, i, pblk, lrow, [&](int t, float v) { corr[i * T + t] = v; });
        }
    }
    float *op = out + bimg * (long long)cout * a.HW + rem;
    for (int c = 0; c < cout; ++c) {
        const float *wr = wgt + c * CIN;
        float acc = bias ? bias[c] : 0.0f;
#pragma unroll
        for (int k = 0; k < CIN; ++k) acc = fmaf(wr[k], corr[k], acc);
        if (relu) acc = fmaxf(acc, 0.0f);
        if (active) op[(long long)c * a.HW] = acc;
    }
}

template <int R, int M>
static hipError_t launch_chain_m(const LookupArgs &a, hipStream_t s, unsigned lds = 0) {
    const unsigned nblk = (unsigned)((a.P + 255) / 256);
    if (a.levels == 4)
        hipLaunchKernelGGL((lookup_chain_kernel<R, 4, M>), dim3(nblk), dim3(256), lds, s, a);
    else if (a.levels == 3)
        hipLaunchKernelGGL((lookup_chain_kernel<R, 3, M>), dim3(nblk), dim3(256), lds, s, a);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

#ifdef RAFTCORR_DEV
#include "dev/lookup_dev.inc"   // A/B variants and prototypes: libraftcorr_dev.so only
#endif

template <int R>
static hipError_t launch_pair_r(const LookupArgs &a, int bf16, hipStream_t s) {
    const unsigned nblk = (unsigned)((a.P + 255) / 256);
    if (a.rec_nr) {   // RC_LAYOUT_RECORDS (bf16, 4 levels: checked by the C-ABI)
        if (!bf16 || a.levels != 4) return hipErrorNotSupported;
#ifdef RAFTCORR_DEV
        if (const hipError_t e = dev_launch_records<R>(a, s); e != hipErrorNotSupported) return e;
#endif
        // the cooperative whole-record fetch: 118.4 vs 121.5 us per config-3
        // lookup (interleaved, bit-identical; profiles/r06/rec_o)
        if (a.out_cl) hipLaunchKernelGGL((lookup_records_kernel<R, true, 0, true>), dim3(nblk), dim3(256), 0, s, a);
        else hipLaunchKernelGGL((lookup_records_kernel<R, false, 0, true>), dim3(nblk), dim3(256), 0, s, a);
        return hipGetLastError();
    }
    if (a.shk[0]) {   // RC_LAYOUT_DISPARITY (fp32, NCHW output: checked by the C-ABI)
        if (bf16 || a.out_cl) return hipErrorNotSupported;
        if (a.levels == 4) hipLaunchKernelGGL((lookup_sheared_pair_kernel<R, 4>), dim3(nblk), dim3(256), 0, s, a);
        else if (a.levels == 2) hipLaunchKernelGGL((lookup_sheared_pair_kernel<R, 2>), dim3(nblk), dim3(256), 0, s, a);
        else return hipErrorInvalidValue;
        return hipGetLastError();
    }
#ifdef RAFTCORR_DEV
    if (const hipError_t e = dev_launch_pair<R>(a, bf16, s); e != hipErrorNotSupported) return e;
#endif
    const bool cl = a.out_cl != 0;
    if (a.levels == 4) {
        if (cl) {
            if (bf16) hipLaunchKernelGGL((lookup_pair_kernel<R, 4, 0, true, 1, true>), dim3(nblk), dim3(256), 0, s, a);
            else hipLaunchKernelGGL((lookup_pair_kernel<R, 4, 0, false, 1, true>), dim3(nblk), dim3(256), 0, s, a);
        } else {
            if (bf16) hipLaunchKernelGGL((lookup_pair_kernel<R, 4, 0, true>), dim3(nblk), dim3(256), 0, s, a);
            else hipLaunchKernelGGL((lookup_pair_kernel<R, 4>), dim3(nblk), dim3(256), 0, s, a);
        }
    } else if (a.levels == 2) {
        if (cl) {
            if (bf16) hipLaunchKernelGGL((lookup_pair_kernel<R, 2, 0, true, 1, true>), dim3(nblk), dim3(256), 0, s, a);
            else hipLaunchKernelGGL((lookup_pair_kernel<R, 2, 0, false, 1, true>), dim3(nblk), dim3(256), 0, s, a);
        } else {
            if (bf16) hipLaunchKernelGGL((lookup_pair_kernel<R, 2, 0, true>), dim3(nblk), dim3(256), 0, s, a);
            else hipLaunchKernelGGL((lookup_pair_kernel<R, 2>), dim3(nblk), dim3(256), 0, s, a);
        }
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <int R>
static hipError_t launch_chain_r(const LookupArgs &a, hipStream_t s) {
#ifdef RAFTCORR_DEV
    if (const hipError_t e = dev_launch_chain<R>(a, s); e != hipErrorNotSupported) return e;
#endif
    return launch_chain_m<R, 0>(a, s);
}

template <int R>
static hipError_t launch_conv_r(const LookupArgs &a, int bf16, const float *w, const float *b,
                                int cout, int relu, float *out, hipStream_t s) {
    const unsigned nblk = (unsigned)((a.P + 255) / 256);
#ifdef RAFTCORR_DEV
    if (const hipError_t e = dev_launch_conv<R>(a, bf16, w, b, cout, relu, out, s); e != hipErrorNotSupported)
        return e;
#endif
    if (a.levels == 4) {
        if (bf16) hipLaunchKernelGGL((lookup_conv_kernel<R, 4, true>), dim3(nblk), dim3(256), 0, s, a, w, b, cout, relu, out);
        else hipLaunchKernelGGL((lookup_conv_kernel<R, 4, false>), dim3(nblk), dim3(256), 0, s, a, w, b, cout, relu, out);
    } else if (a.levels == 3) {
        if (bf16) hipLaunchKernelGGL((lookup_conv_kernel<R, 3, true>), dim3(nblk), dim3(256), 0, s, a, w, b, cout, relu, out);
        else hipLaunchKernelGGL((lookup_conv_kernel<R, 3, false>), dim3(nblk), dim3(256), 0, s, a, w, b, cout, relu, out);
    } else if (a.levels == 2) {
        if (bf16) hipLaunchKernelGGL((lookup_conv_kernel<R, 2, true>), dim3(nblk), dim3(256), 0, s, a, w, b, cout, relu, out);
        else hipLaunchKernelGGL((lookup_conv_kernel<R, 2, false>), dim3(nblk), dim3(256), 0, s, a, w, b, cout, relu, out);
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <int R>
static hipError_t launch_r(const LookupArgs &a, int bf16, hipStream_t s) {
    // Default: runtime level loop (low VGPR count, 8 waves/SIMD) + exact-span
    // predicated loads; small problems: every level's loads up front (64-thread
    // blocks) or one wave per level (lookup_levelpar_kernel).  Measured
    // (tools/ablate.py) before choosing.
#ifdef RAFTCORR_DEV
    if (const hipError_t e = dev_launch_level<R>(a, bf16, s); e != hipErrorNotSupported) return e;
#endif
    const bool unroll = a.levels == 3 || a.levels == 4;
    if (a.P < kLevelParP && a.levels <= 4) {
        const unsigned nblk = (unsigned)((a.P + 63) / 64);
        if (bf16) hipLaunchKernelGGL((lookup_levelpar_kernel<R, true>), dim3(nblk), dim3(64 * a.levels), 0, s, a);
        else hipLaunchKernelGGL((lookup_levelpar_kernel<R, false>), dim3(nblk), dim3(64 * a.levels), 0, s, a);
    } else if (a.P < kSmallP && unroll) {
        if (a.levels == 4) {
            if (bf16) launch_k<R, 4, true, true, 64>(a, s);
            else launch_k<R, 4, false, true, 64>(a, s);
        } else {
            if (bf16) launch_k<R, 3, true, true, 64>(a, s);
            else launch_k<R, 3, false, true, 64>(a, s);
        }
    } else {
        if (bf16) launch_k<R, 0, true, true>(a, s);
        else launch_k<R, 0, false, true>(a, s);
    }
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

hipError_t rc_launch_lookup_pair(const rc::LookupArgs &a, int radius, int pyr_bf16, hipStream_t s) {
    if (a.P <= 0) return hipSuccess;
    switch (radius) {
        case 1: return rc::launch_pair_r<1>(a, pyr_bf16, s);
        case 2: return rc::launch_pair_r<2>(a, pyr_bf16, s);
        case 3: return rc::launch_pair_r<3>(a, pyr_bf16, s);
        case 4: return rc::launch_pair_r<4>(a, pyr_bf16, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t rc_launch_lookup_chain(const rc::LookupArgs &a, int radius, hipStream_t s) {
    if (a.P <= 0) return hipSuccess;
    switch (radius) {
        case 1: return rc::launch_chain_r<1>(a, s);
        case 2: return rc::launch_chain_r<2>(a, s);
        case 3: return rc::launch_chain_r<3>(a, s);
        case 4: return rc::launch_chain_r<4>(a, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t rc_launch_lookup_conv(const rc::LookupArgs &a, int radius, int pyr_bf16, const float *w,
                                 const float *b, int cout, int relu, float *out, hipStream_t s) {
    if (a.P <= 0) return hipSuccess;
    switch (radius) {
        case 1: return rc::launch_conv_r<1>(a, pyr_bf16, w, b, cout, relu, out, s);
        case 2: return rc::launch_conv_r<2>(a, pyr_bf16, w, b, cout, relu, out, s);
        case 3: return rc::launch_conv_r<3>(a, pyr_bf16, w, b, cout, relu, out, s);
        case 4: return rc::launch_conv_r<4>(a, pyr_bf16, w, b, cout, relu, out, s);
        default: return hipErrorInvalidValue;
    }
}
