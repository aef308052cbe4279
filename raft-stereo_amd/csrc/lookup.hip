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

#ifdef RAFTCORR_DEV
// Level-0 chain (dev variant 220): every level 0..NL-1
// derived from ONE span of level 0 -- the top level's 2r+4 window scaled by
// S = 2^(NL-1) (96 elements at L = 4, r = 4), exact-span predicated -- so the
// lookups read level 0 only (249 MB at config 2 instead of levels 0 + 2 and the
// level-2 copy) at the cost of more 64-B sectors per pixel (4.7 vs 3.7
// simulated).  Level i window element jj is the pool_tree of 2^i level-0
// elements, the fp32 ops of avg_pool2d applied i times (model.py:294).
template <int R, int NL>
__global__ __launch_bounds__(256) void lookup_l0chain_kernel(LookupArgs a) {
    constexpr int T = 2 * R + 1, NW = 2 * R + 4, TOP = NL - 1, S = 1 << TOP;
    constexpr int NE0 = S * NW, NC0 = NE0 / 4;
    static_assert(S % 4 == 0, "span start must be 16-B aligned");
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const long long pblk = (long long)blk * 256;
    const long long p = pblk + threadIdx.x;
    const bool active = p < a.P;
    const long long pp = active ? p : a.P - 1;
    const long long bimg = pp / a.HW, rem = pp - bimg * a.HW;
    const float x = pixel_x(a, bimg, rem, active);
    float *outp = a.out + bimg * (long long)(NL * T) * a.HW + rem;
    const long long lrow = pp - pblk;
    const float xtop = x / (float)(1 << TOP);
    const bool inwin = (xtop > -(float)(R + 4)) && (xtop < (float)(a.W[TOP] + R + 4));
    const float ntop = inwin ? floorf(xtop) : 0.0f;
    const int e0 = S * ((int)ntop - R - 1);
    int lo = 0x7FFFFFFF, hi = -1;
    if (inwin) {
#pragma unroll
        for (int i = 0; i <= TOP; ++i) {
            int f, l;
            tap_span<R>(x / (float)(1 << i), a.W[i], f, l);
            if (f <= l) {
                lo = min(lo, f << i);
                hi = max(hi, ((l + 1) << i) - 1);
            }
        }
    }
    const long long ld0 = a.ld[0];
    const float *lvl0 = static_cast<const float *>(a.lvl[0]);
    const auto rs0 = make_rsrc(lvl0 + pblk * ld0, clamp_bytes((a.P - pblk) * ld0 * 4));
    float s0[NE0];
#pragma unroll
    for (int k = 0; k < NC0; ++k) {
        const int cs = e0 + 4 * k;
        const bool ok = cs <= hi && cs + 3 >= lo;
        const f32x4 v = ld4(rs0, ok ? (uint32_t)((lrow * ld0 + cs) * 4) : 0xFFFFFF00u);
#pragma unroll
        for (int c = 0; c < 4; ++c) s0[4 * k + c] = v[c];
    }
    const float *row0 = lvl0 + pp * ld0;
    auto level = [&](auto ic) {
        constexpr int i = decltype(ic)::value;
        constexpr int SI = 1 << i, NDD = 1 << (TOP - i);
        const int W = a.W[i];
        const float Wm1 = (float)(W - 1), half = Wm1 / 2.0f;
        const DivRN dv = div_prep(Wm1);
        const float xl = x / (float)(1 << i);
        const float n = inwin ? floorf(xl) : 0.0f;
        const int dd = inwin ? (int)n - NDD * (int)ntop : 0;
        const bool valid = inwin && dd >= 0 && dd < NDD;
        float w[NW];
#pragma unroll
        for (int jj = 0; jj < NW; ++jj) {
            float val = 0.0f;
#pragma unroll
            for (int d = 0; d < NDD; ++d) {
                constexpr int base = (R + 1) * (S - SI);
                const float v = pool_tree<SI>(s0 + base + SI * (d + jj));
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
            float e0_ = w[t], e1_ = w[t + 1], e2_ = w[t + 2], e3_ = w[t + 3];
            asm("" : "+v"(e0_), "+v"(e1_), "+v"(e2_), "+v"(e3_));
            const float a0 = lo_ ? e0_ : (hi_ ? e2_ : e1_);
            const float a1 = lo_ ? e1_ : (hi_ ? e3_ : e2_);
            const bool ok0 = (x0 >= 0.0f) && (x0 <= Wm1);
            const bool ok1 = (x0 + 1.0f >= 0.0f) && (x0 + 1.0f <= Wm1);
            bad |= inwin && (!valid || x0 < nt - 1.0f || x0 > nt + 1.0f);
            res[t] = fmaf(w1, ok1 ? a1 : 0.0f, w0 * (ok0 ? a0 : 0.0f));
        }
        if (__builtin_expect(bad, 0)) {
            for (int t = 0; t < T; ++t) {
                const float xt = (float)(t - R) + xl;
                const float xn = div_rn(2.0f * xt, dv) - 1.0f;
                const float xp = (xn + 1.0f) * half;
                const float x0 = floorf(xp);
                const float w1 = xp - x0, w0 = 1.0f - w1;
                const bool ok0 = (x0 >= 0.0f) && (x0 <= Wm1);
                const bool ok1 = (x0 + 1.0f >= 0.0f) && (x0 + 1.0f <= Wm1);
                const float v0 = ok0 ? derived_elem<SI>(row0, (long long)x0) : 0.0f;
                const float v1 = ok1 ? derived_elem<SI>(row0, (long long)x0 + 1) : 0.0f;
                res[t] = fmaf(w1, v1, w0 * v0);
            }
        }
        if (active) {
#pragma unroll
            for (int t = 0; t < T; ++t) outp[(long long)(i * T + t) * a.HW] = res[t];
        }
    };
    level(std::integral_constant<int, 0>{});
    level(std::integral_constant<int, 1>{});
    level(std::integral_constant<int, 2>{});
    if constexpr (TOP >= 3) level(std::integral_constant<int, 3>{});
}
#endif

// PH (dev-only timing probes; the values read are NOT the span's): 1 = read
// each span at +64 B when that touches fewer 128-B lines (what a second,
// half-line-shifted copy of the level would give), 2 = move every span to a
// 128-B line start (lower bound: the fewest lines any layout could give).
template <int R, bool BF16 = false, int PH = 0>
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
    if (shb != 0 || PH != 0) {
        const unsigned long long b0 =
            (unsigned long long)(uintptr_t)(lvl + ((pblk + lrow) * ld + (lo_e & ~(PS::EPC - 1))) * PS::ES);
        const unsigned long long b1 = (unsigned long long)(uintptr_t)(lvl + ((pblk + lrow) * ld + hi_e) * PS::ES);
        if (lo_e <= hi_e) {
            if constexpr (PH == 2) {     // dev probe: line-aligned spans
                phase = (uint32_t)((128 - (b0 & 127)) & 127);
            } else {
                const unsigned long long sh = PH == 1 ? 64ull : (unsigned long long)shb;
                const long long l0 = (long long)(b1 >> 7) - (long long)(b0 >> 7);
                const long long l1 = (long long)((b1 + sh) >> 7) - (long long)((b0 + sh) >> 7);
                phase = l1 < l0 ? (uint32_t)sh : 0u;
            }
        }
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
// M: dev-only ablation (RAFTCORR_LOOKUP_VARIANT 201-204, dev library):
// 1 = no output stores, 2 = no fallback path, 3 / 4 = issue_pair's line-phase
// probes PH 1 / 2 (timing only: wrong values), 5 = hardware block order
// (no XCD remap; same values), 6 = PH 1, 7 = non-temporal output stores;
// the WPE parameter (dev variants 208/209) caps registers for 5/6 waves/SIMD;
// 9 (variant 211) = the channels-last store path writing into an NCHW
// buffer (timing A/B of the two layouts on the same output tensor).
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
        issue_pair<R, BF16, (M == 3 || M == 6) ? 1 : (M == 4 ? 2 : 0)>(sp[k], a, 2 * k, q.x, q.pblk, q.lrow);
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

#ifdef RAFTCORR_DEV
// Disparity-major ("sheared") pair lookup (dev only): the
// pair kernel's arithmetic (levels 0 and 2 stored, 1 and 3 their pairwise
// means, finish_pair) over levels stored as S_i[b,h][k][w1] with
// k = (w1 >> i) - j + W_i - 1 (lookup_sheared.hip's layout), so the lanes of
// a wave whose pixels look at the same disparity read one contiguous run of
// a row per span element -- coalesced along w1 -- instead of a 16-B piece of
// 64 different pixel rows.  A span is 2(2r+4) dword loads per lane (exact-
// span predicated).  No memory fallback (finish_pair NOFALLBACK): the probe
// feeds no subnormal coordinates.
template <int R>
__global__ __launch_bounds__(256) void lookup_sheared_pair_kernel(LookupArgs a, const float *s0, const float *s2,
                                                                  long long K0, long long K2, long long ldw) {
    constexpr int NS = PairSpan<R>::NS;
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
    float *outp = a.out + bimg * (long long)(4 * (2 * R + 1)) * a.HW + rem;
    auto sink = [&](int ch, float v) {
        if (active) outp[(long long)ch * a.HW] = v;
    };
    PairSpan<R> sp[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
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
        const long long K = k ? K2 : K0;
        const float *lv = k ? s2 : s0;
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
#pragma unroll
    for (int k = 0; k < 2; ++k) finish_pair<R, true>(sp[k], a, 2 * k, x, pp, sink);
}
#endif

// Persistent pair lookup (dev variants 215-219 while measured).  The one-round
// grid of lookup_pair_kernel puts every wave in the same phase: all spans are
// requested at launch and each wave's output stores follow its own loads.
// Here each wave walks 64-pixel groups g, g + S, g + 2S, ... of its XCD's
// contiguous share of the image (S = waves on that XCD), and with PIPE the
// spans of group n+1 are requested before group n's tap math and stores, so a
// wave's stores overlap its own next loads; the x of group n+2 is loaded one
// stage ahead, so issuing the next spans never waits on the current ones.
// Same PairSpan / finish_pair as the pair kernel: bit-identical output.
__device__ __forceinline__ float group_x(const LookupArgs &a, long long g, int lane) {
    const long long p = g * 64 + lane;
    const long long pp = p < a.P ? p : a.P - 1;
    const long long bimg = pp / a.HW, rem = pp - bimg * a.HW;
    return pixel_x(a, bimg, rem, p < a.P);
}

template <int R, int NL, bool BF16, bool PIPE, int WPE = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void lookup_pair_persist_kernel(LookupArgs a) {
    static_assert(NL == 2 || NL == 4, "pair lookup: 2 or 4 levels");
    constexpr int NP = NL / 2;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const long long NG = (a.P + 63) >> 6;
    const int nb = gridDim.x, xcd = blockIdx.x & 7, kb = blockIdx.x >> 3;
    const int nbx = (nb >> 3) + (xcd < (nb & 7) ? 1 : 0);          // blocks on this XCD
    const long long gq = NG >> 3, gr = NG & 7;
    const long long g0 = xcd * gq + (xcd < gr ? xcd : gr);
    const long long g1 = g0 + gq + (xcd < gr ? 1 : 0);              // this XCD's groups [g0, g1)
    const long long S = 4LL * nbx;
    long long g = g0 + 4LL * kb + w;
    if (g >= g1) return;
    auto pix = [&](long long gg, float x) {
        PairPixel q;
        q.pblk = gg * 64;
        const long long p = q.pblk + lane;
        q.active = p < a.P;
        q.pp = q.active ? p : a.P - 1;
        const long long bimg = q.pp / a.HW, rem = q.pp - bimg * a.HW;
        q.x = x;
        q.outp = a.out + bimg * (long long)(NL * (2 * R + 1)) * a.HW + rem;
        q.lrow = lane;
        return q;
    };
    auto sink_of = [&](const PairPixel &q) {
        return [&a, q](int ch, float v) {
            if (q.active) q.outp[(long long)ch * a.HW] = v;
        };
    };
    if constexpr (!PIPE) {
        for (; g < g1; g += S) {
            const PairPixel q = pix(g, group_x(a, g, lane));
            PairSpan<R, BF16> sp[NP];
#pragma unroll
            for (int k = 0; k < NP; ++k) issue_pair<R, BF16>(sp[k], a, 2 * k, q.x, q.pblk, q.lrow);
#pragma unroll
            for (int k = 0; k < NP; ++k) finish_pair<R, false, BF16>(sp[k], a, 2 * k, q.x, q.pp, sink_of(q));
        }
    } else {
        PairPixel qa = pix(g, group_x(a, g, lane));
        float xn = g + S < g1 ? group_x(a, g + S, lane) : 0.0f;   // x of the next group
        PairSpan<R, BF16> sa[NP];
#pragma unroll
        for (int k = 0; k < NP; ++k) issue_pair<R, BF16>(sa[k], a, 2 * k, qa.x, qa.pblk, qa.lrow);
        for (;;) {
            const long long gn = g + S;
            const bool more = gn < g1;                               // wave-uniform
            PairPixel qb;
            PairSpan<R, BF16> sb[NP];
            if (more) {
                const float x2 = gn + S < g1 ? group_x(a, gn + S, lane) : 0.0f;
                qb = pix(gn, xn);
#pragma unroll
                for (int k = 0; k < NP; ++k) issue_pair<R, BF16>(sb[k], a, 2 * k, qb.x, qb.pblk, qb.lrow);
                xn = x2;
            }
#pragma unroll
            for (int k = 0; k < NP; ++k) finish_pair<R, false, BF16>(sa[k], a, 2 * k, qa.x, qa.pp, sink_of(qa));
            if (!more) break;
            qa = qb;
#pragma unroll
            for (int k = 0; k < NP; ++k) sa[k] = sb[k];
            g = gn;
        }
    }
}

template <int R, bool PIPE, int WPE>
static void launch_pair_persist(const LookupArgs &a, int bf16, int blocks_per_cu, hipStream_t s) {
    const long long NG = (a.P + 63) >> 6;
    long long nblk = 256LL * blocks_per_cu;                         // MI355X: 256 CUs
    if (nblk * 4 > NG) nblk = (NG + 3) / 4;
    if (a.levels == 4) {
        if (bf16) hipLaunchKernelGGL((lookup_pair_persist_kernel<R, 4, true, PIPE, WPE>), dim3(nblk), dim3(256), 0, s, a);
        else hipLaunchKernelGGL((lookup_pair_persist_kernel<R, 4, false, PIPE, WPE>), dim3(nblk), dim3(256), 0, s, a);
    } else {
        if (bf16) hipLaunchKernelGGL((lookup_pair_persist_kernel<R, 2, true, PIPE, WPE>), dim3(nblk), dim3(256), 0, s, a);
        else hipLaunchKernelGGL((lookup_pair_persist_kernel<R, 2, false, PIPE, WPE>), dim3(nblk), dim3(256), 0, s, a);
    }
}

// Cooperative span loads (dev variants 212-214 while measured).  The pair
// kernel above has each lane fetch its own two spans with 7 (fp32) 16-B
// loads: every wave-instruction then touches 64 different rows, and a span's
// 128-B line is requested as two 64-B sectors by two different instructions.
// Here LPS lanes load one span together (LPS x 16 B covers the span's
// chunks), so one instruction covers 64 / LPS spans and asks for each line
// once; the chunks land in LDS by buffer->LDS DMA (no VGPRs held while in
// flight), and each pixel's lane reads its span back with NC ds_read_b128.
// Same PairSpan fields and the same finish_pair, so the output is the pair
// kernel's bit for bit.
template <int R, bool BF16>
struct CoopGeom {
    typedef PairSpan<R, BF16> PS;
    static constexpr int LPS = PS::NC <= 4 ? 4 : 8;   // lanes per span (16-B chunks)
    static constexpr int SPI = 64 / LPS;              // spans per wave-instruction
    static constexpr int NI = 64 / SPI;               // instructions per wave and level pair
    static constexpr int SPAN_B = 64 * 16 * NI;       // LDS bytes per wave and level pair (1 KB per instr)
    static_assert(PS::NC <= LPS, "span chunks exceed the lanes per span");
    // chunk-position swizzle: lanes p and p + 8 of a ds_read_b128 lane group
    // would hit the same banks with 8 lanes per span
    __device__ static __forceinline__ int swz(int j) { return LPS == 8 ? (j & 1) : 0; }
    // LDS byte offset of chunk c of the span of the wave's pixel p
    __device__ static __forceinline__ int at(int p, int c) {
        const int j = p / SPI;
        return j * 1024 + ((c ^ swz(j)) * SPI + (p % SPI)) * 16;
    }
};

// As issue_pair, but returns the span's byte offset (chunk 0) and the mask of
// chunks to fetch instead of loading them.
template <int R, bool BF16 = false>
__device__ __forceinline__ uint32_t plan_pair(PairSpan<R, BF16> &ps, const LookupArgs &a, int lo, float x,
                                              long long pblk, long long lrow) {
    typedef PairSpan<R, BF16> PS;
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
    const int sa = 2 * ((int)ps.m - R - 1);
    const int ea = sa & ~(PS::EPC - 1);
    ps.sh = sa - ea;
    const long long ld = a.ld[lo];
    const char *lvl = static_cast<const char *>(a.lvl[lo]);
    const long long shb = a.shadow[lo];
    uint32_t phase = 0;
    if (shb != 0 && lo_e <= hi_e) {
        const unsigned long long b0 =
            (unsigned long long)(uintptr_t)(lvl + ((pblk + lrow) * ld + (lo_e & ~(PS::EPC - 1))) * PS::ES);
        const unsigned long long b1 = (unsigned long long)(uintptr_t)(lvl + ((pblk + lrow) * ld + hi_e) * PS::ES);
        const long long l0 = (long long)(b1 >> 7) - (long long)(b0 >> 7);
        const long long l1 = (long long)((b1 + shb) >> 7) - (long long)((b0 + shb) >> 7);
        phase = l1 < l0 ? 1u : 0u;
    }
    // the chunks [first, last] hold [lo_e, hi_e] (none: first > last)
    int first = 7, last = 0;
    if (lo_e <= hi_e) {
        first = max((lo_e - ea) / PS::EPC, 0);
        last = min((hi_e - ea) / PS::EPC, PS::NC - 1);
    }
    // packed plan: bits 0-22 the byte offset / 16 of chunk `first` (>= 0;
    // lrow < 64, ld*ES <= 2^18: < 2^20), bit 23 shadow copy, bits 24-26 first
    // chunk, 27-29 last chunk.  (Chunk 0 may start before the row: ea < 0.)
    const uint32_t loc = first <= last ? (uint32_t)((lrow * ld + ea + PS::EPC * first) * PS::ES) >> 4 : 0u;
    return loc | (phase << 23) | ((uint32_t)first << 24) | ((uint32_t)last << 27);
}

// One wave's cooperative fetch of the spans of level pair `lo` for its 64
// pixels into `sbuf` (SPAN_B bytes): instruction j loads the spans of pixels
// SPI*j .. SPI*j + SPI-1, lane l chunk (l / SPI) ^ swz(j) of pixel SPI*j + l % SPI.
// Each pixel's plan travels in one dword (`pk`, see coop_pack): all the
// wave's ds_bpermutes issue before its loads.
template <int R, bool BF16>
__device__ __forceinline__ void coop_fetch(const LookupArgs &a, int lo, long long pblk, uint32_t pk,
                                           __attribute__((address_space(3))) char *sbuf) {
    typedef CoopGeom<R, BF16> G;
    typedef PairSpan<R, BF16> PS;
    const int lane = threadIdx.x & 63;
    const long long ld = a.ld[lo];
    const uint32_t shb = (uint32_t)a.shadow[lo];
    const auto rs = make_rsrc(static_cast<const char *>(a.lvl[lo]) + pblk * ld * PS::ES,
                              clamp_bytes((a.P - pblk) * ld * PS::ES + a.shadow[lo]));
    uint32_t v[G::NI];
#pragma unroll
    for (int j = 0; j < G::NI; ++j) v[j] = (uint32_t)__shfl((int)pk, G::SPI * j + lane % G::SPI, 64);
#pragma unroll
    for (int j = 0; j < G::NI; ++j) {
        const int c = (lane / G::SPI) ^ G::swz(j);
        const uint32_t first = (v[j] >> 24) & 7u, last = (v[j] >> 27) & 7u;
        const uint32_t o = ((v[j] & 0x7FFFFFu) << 4) + ((v[j] >> 23) & 1u ? shb : 0u) + 16u * ((uint32_t)c - first);
        const uint32_t off = ((uint32_t)c >= first && (uint32_t)c <= last) ? o : 0xFFFFFF00u;
#if defined(__HIP_DEVICE_COMPILE__)   // the LDS-pointer builtin has no host form
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void *)(sbuf + j * 1024),
                                                 16, (int)off, 0, 0, 0);
#else
        (void)rs; (void)off;
#endif
    }
}

template <int R, bool BF16>
__device__ __forceinline__ void coop_read(PairSpan<R, BF16> &ps, const char *sbuf) {
    typedef CoopGeom<R, BF16> G;
    const int p = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < PairSpan<R, BF16>::NC; ++k) {
        const uint4 v = *reinterpret_cast<const uint4 *>(sbuf + G::at(p, k));
        ps.q[k][0] = v.x; ps.q[k][1] = v.y; ps.q[k][2] = v.z; ps.q[k][3] = v.w;
    }
}

template <int R, int NL, int WPB, bool BF16 = false>
__global__ __launch_bounds__(64 * WPB) void lookup_pair_coop_kernel(LookupArgs a) {
    static_assert(NL == 2 || NL == 4, "pair lookup: 2 or 4 levels");
    typedef CoopGeom<R, BF16> G;
    constexpr int NP = NL / 2;
    __shared__ __attribute__((aligned(16))) char sbuf[WPB][NP][G::SPAN_B];
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    const long long pblk = (long long)blk * 64 * WPB;
    const PairPixel q = pair_pixel<R, NL>(a, pblk);
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const long long pw = pblk + 64 * w;             // the wave's first pixel (wave-uniform)
    PairSpan<R, BF16> sp[NP];
    uint32_t pk[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) pk[k] = plan_pair<R, BF16>(sp[k], a, 2 * k, q.x, pw, q.pp - pw);
#pragma unroll
    for (int k = 0; k < NP; ++k)
        coop_fetch<R, BF16>(a, 2 * k, pw, pk[k], (__attribute__((address_space(3))) char *)sbuf[w][k]);
    // both spans back into registers before any output store: a store is
    // counted in vmcnt, so a later LDS read would wait for it too
#pragma unroll
    for (int k = 0; k < NP; ++k) coop_read<R, BF16>(sp[k], sbuf[w][k]);
    auto sink = [&](int ch, float v) {
        if (q.active) q.outp[(long long)ch * a.HW] = v;
    };
#pragma unroll
    for (int k = 0; k < NP; ++k) finish_pair<R, false, BF16>(sp[k], a, 2 * k, q.x, q.pp, sink);
}

template <int R, int WPB>
static void launch_pair_coop(const LookupArgs &a, int bf16, hipStream_t s) {
    const unsigned nblk = (unsigned)((a.P + 64 * WPB - 1) / (64 * WPB));
    if (a.levels == 4) {
        if (bf16) hipLaunchKernelGGL((lookup_pair_coop_kernel<R, 4, WPB, true>), dim3(nblk), dim3(64 * WPB), 0, s, a);
        else hipLaunchKernelGGL((lookup_pair_coop_kernel<R, 4, WPB>), dim3(nblk), dim3(64 * WPB), 0, s, a);
    } else {
        if (bf16) hipLaunchKernelGGL((lookup_pair_coop_kernel<R, 2, WPB, true>), dim3(nblk), dim3(64 * WPB), 0, s, a);
        else hipLaunchKernelGGL((lookup_pair_coop_kernel<R, 2, WPB>), dim3(nblk), dim3(64 * WPB), 0, s, a);
    }
}

#ifdef RAFTCORR_DEV
__device__ __forceinline__ unsigned long long rtc_stamp() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}

// Diagnostic build of the 4-level pair kernel (dev library, variant 210):
// lane 0 of every wave records s_memrealtime (100 MHz) at
//   0 start, 1 loads issued, 2 span 0 landed, 3 pair 0 done (math + stores
//   issued), 4 span 2 landed, 5 pair 2 done, 6 all stores drained,
// plus HW_ID, into dbg[wave * 8 + k].  Its run time is not the product's
// (the waits forbid overlaps); read shares and distributions only.
template <int R>
__global__ __launch_bounds__(256) void lookup_pair_stamped_kernel(LookupArgs a) {
    unsigned long long st[7];
    st[0] = rtc_stamp();
    const PairPixel q = pair_pixel<R, 4>(a, (long long)blockIdx.x * 256);
    PairSpan<R> s0, s2;
    issue_pair<R>(s0, a, 0, q.x, q.pblk, q.lrow);
    issue_pair<R>(s2, a, 2, q.x, q.pblk, q.lrow);
    st[1] = rtc_stamp();
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PairSpan<R>::NC) : "memory");
    st[2] = rtc_stamp();
    auto sink = [&](int ch, float v) {
        if (q.active) q.outp[(long long)ch * a.HW] = v;
    };
    finish_pair<R>(s0, a, 0, q.x, q.pp, sink);
    st[3] = rtc_stamp();
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (2 * R + 1)) : "memory");
    st[4] = rtc_stamp();
    finish_pair<R>(s2, a, 2, q.x, q.pp, sink);
    st[5] = rtc_stamp();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    st[6] = rtc_stamp();
    unsigned hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    if ((threadIdx.x & 63) == 0) {
        unsigned long long *d = a.dbg + ((long long)blockIdx.x * 4 + (threadIdx.x >> 6)) * 8;
#pragma unroll
        for (int k = 0; k < 7; ++k) d[k] = st[k];
        d[7] = hw;
    }
}
#endif

template <int R>
static hipError_t launch_pair_r(const LookupArgs &a, int bf16, hipStream_t s) {
    const unsigned nblk = (unsigned)((a.P + 255) / 256);
#ifdef RAFTCORR_DEV
    if constexpr (R == 4) {
        const int v = dev_knob("RAFTCORR_LOOKUP_VARIANT");
        if ((a.levels == 4 || a.levels == 2) && !a.out_cl && v >= 212 && v <= 214) {
            if (v == 212) launch_pair_coop<R, 1>(a, bf16, s);
            if (v == 213) launch_pair_coop<R, 2>(a, bf16, s);
            if (v == 214) launch_pair_coop<R, 4>(a, bf16, s);
            return hipGetLastError();
        }
        // persistent pair lookup: 215 = one group at a time, 2 blocks/CU;
        // 216 / 217 = pipelined, 1 / 2 blocks per CU (more spill to scratch)
        if ((a.levels == 4 || a.levels == 2) && !a.out_cl && v >= 215 && v <= 217) {
            if (v == 215) launch_pair_persist<R, false, 2>(a, bf16, 2, s);
            if (v == 216) launch_pair_persist<R, true, 1>(a, bf16, 1, s);
            if (v == 217) launch_pair_persist<R, true, 2>(a, bf16, 2, s);
            return hipGetLastError();
        }
        // 220: level-0 chain (reads level 0 only; fp32, 4 levels)
        if (a.levels == 4 && !bf16 && !a.out_cl && v == 220) {
            hipLaunchKernelGGL((lookup_l0chain_kernel<R, 4>), dim3(nblk), dim3(256), 0, s, a);
            return hipGetLastError();
        }
        if (a.levels == 4 && v == 210 && a.dbg) {
            hipLaunchKernelGGL((lookup_pair_stamped_kernel<R>), dim3(nblk), dim3(256), 0, s, a);
            return hipGetLastError();
        }
        if (a.levels == 4 && v >= 201 && v <= 211) {
            if (v == 211 && !bf16) hipLaunchKernelGGL((lookup_pair_kernel<R, 4, 9>), dim3(nblk), dim3(256), 0, s, a);
            if (v == 211 && bf16) hipLaunchKernelGGL((lookup_pair_kernel<R, 4, 9, true>), dim3(nblk), dim3(256), 0, s, a);
            // 208 / 209: at least 5 / 6 waves per SIMD (register cap)
            if (v == 208 && !bf16) hipLaunchKernelGGL((lookup_pair_kernel<R, 4, 0, false, 5>), dim3(nblk), dim3(256), 0, s, a);
            if (v == 208 && bf16) hipLaunchKernelGGL((lookup_pair_kernel<R, 4, 0, true, 5>), dim3(nblk), dim3(256), 0, s, a);
            if (v == 209 && !bf16) hipLaunchKernelGGL((lookup_pair_kernel<R, 4, 0, false, 6>), dim3(nblk), dim3(256), 0, s, a);
            if (v == 209 && bf16) hipLaunchKernelGGL((lookup_pair_kernel<R, 4, 0, true, 6>), dim3(nblk), dim3(256), 0, s, a);
            if (v == 207 && !bf16) hipLaunchKernelGGL((lookup_pair_kernel<R, 4, 7>), dim3(nblk), dim3(256), 0, s, a);
            if (v == 207 && bf16) hipLaunchKernelGGL((lookup_pair_kernel<R, 4, 7, true>), dim3(nblk), dim3(256), 0, s, a);
            if (v == 205 && !bf16) hipLaunchKernelGGL((lookup_pair_kernel<R, 4, 5>), dim3(nblk), dim3(256), 0, s, a);
            if (v == 206 && !bf16) hipLaunchKernelGGL((lookup_pair_kernel<R, 4, 6>), dim3(nblk), dim3(256), 0, s, a);
            if (v == 205 && bf16) hipLaunchKernelGGL((lookup_pair_kernel<R, 4, 5, true>), dim3(nblk), dim3(256), 0, s, a);
            if (v == 206 && bf16) hipLaunchKernelGGL((lookup_pair_kernel<R, 4, 6, true>), dim3(nblk), dim3(256), 0, s, a);
            // every variant in the pyramid's own element type (an fp32 kernel
            // on a bf16 pyramid reads past the end of its buffers)
            if (v == 201 && !bf16) hipLaunchKernelGGL((lookup_pair_kernel<R, 4, 1>), dim3(nblk), dim3(256), 0, s, a);
            if (v == 202 && !bf16) hipLaunchKernelGGL((lookup_pair_kernel<R, 4, 2>), dim3(nblk), dim3(256), 0, s, a);
            if (v == 201 && bf16) hipLaunchKernelGGL((lookup_pair_kernel<R, 4, 1, true>), dim3(nblk), dim3(256), 0, s, a);
            if (v == 202 && bf16) hipLaunchKernelGGL((lookup_pair_kernel<R, 4, 2, true>), dim3(nblk), dim3(256), 0, s, a);
            if (v == 203 && !bf16) hipLaunchKernelGGL((lookup_pair_kernel<R, 4, 3>), dim3(nblk), dim3(256), 0, s, a);
            if (v == 204 && !bf16) hipLaunchKernelGGL((lookup_pair_kernel<R, 4, 4>), dim3(nblk), dim3(256), 0, s, a);
            if (v == 203 && bf16) hipLaunchKernelGGL((lookup_pair_kernel<R, 4, 3, true>), dim3(nblk), dim3(256), 0, s, a);
            if (v == 204 && bf16) hipLaunchKernelGGL((lookup_pair_kernel<R, 4, 4, true>), dim3(nblk), dim3(256), 0, s, a);
            return hipGetLastError();
        }
    }
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

template <int R>
static hipError_t launch_chain_r(const LookupArgs &a, hipStream_t s) {
#ifdef RAFTCORR_DEV
    if constexpr (R == 4) {   // ablation variants (dev library), config-2 radius
        const int variant = dev_knob("RAFTCORR_LOOKUP_VARIANT");
        if (variant == 101) return launch_chain_m<R, 1>(a, s);
        if (variant == 102) return launch_chain_m<R, 2>(a, s);
        if (variant == 103) return launch_chain_m<R, 3>(a, s);
        if (variant == 104) return launch_chain_m<R, 4>(a, s);
        if (variant == 105) return launch_chain_m<R, 5>(a, s);   // non-temporal output stores
    }
#endif
    return launch_chain_m<R, 0>(a, s);
}

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

template <int R>
static hipError_t launch_conv_r(const LookupArgs &a, int bf16, const float *w, const float *b,
                                int cout, int relu, float *out, hipStream_t s) {
    const unsigned nblk = (unsigned)((a.P + 255) / 256);
#ifdef RAFTCORR_DEV
    if (dev_knob("RAFTCORR_CONV_VARIANT") == 1 && a.levels == 4 && !bf16) {   // one level at a time
        hipLaunchKernelGGL((lookup_conv_kernel<R, 4, false, false>), dim3(nblk), dim3(256), 0, s, a, w, b, cout, relu, out);
        return hipGetLastError();
    }
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

template <int R>
static hipError_t launch_r(const LookupArgs &a, int bf16, int variant, hipStream_t s) {
    // Default: runtime level loop (low VGPR count, 8 waves/SIMD) + exact-span
    // predicated loads.  Variant 1: full windows; 3: levels unrolled (all
    // loads first; ~130 VGPRs).  Measured (tools/ablate.py) before choosing.
    const bool unroll = a.levels == 3 || a.levels == 4;
#ifndef RAFTCORR_DEV
    variant = 0;
#endif
    if (variant == 0 && a.P < kLevelParP && a.levels <= 4) {
        const unsigned nblk = (unsigned)((a.P + 63) / 64);
        if (bf16) hipLaunchKernelGGL((lookup_levelpar_kernel<R, true>), dim3(nblk), dim3(64 * a.levels), 0, s, a);
        else hipLaunchKernelGGL((lookup_levelpar_kernel<R, false>), dim3(nblk), dim3(64 * a.levels), 0, s, a);
    } else if (variant == 0 && a.P < kSmallP && unroll) {
        if (a.levels == 4) {
            if (bf16) launch_k<R, 4, true, true, 64>(a, s);
            else launch_k<R, 4, false, true, 64>(a, s);
        } else {
            if (bf16) launch_k<R, 3, true, true, 64>(a, s);
            else launch_k<R, 3, false, true, 64>(a, s);
        }
#ifdef RAFTCORR_DEV
    } else if (variant == 6 && a.P < kLevelParP && a.levels <= 4) {   // blocks in launch order
        const unsigned nblk = (unsigned)((a.P + 63) / 64);
        if (bf16) hipLaunchKernelGGL((lookup_levelpar_kernel<R, true, false>), dim3(nblk), dim3(64 * a.levels), 0, s, a);
        else hipLaunchKernelGGL((lookup_levelpar_kernel<R, false, false>), dim3(nblk), dim3(64 * a.levels), 0, s, a);
    } else if (variant == 1) {
        if (bf16) launch_k<R, 0, true, false>(a, s);
        else launch_k<R, 0, false, false>(a, s);
    } else if (variant == 4 && a.levels == 4) {
        if (bf16) launch_k<R, 4, true, true, 256, 4>(a, s);
        else launch_k<R, 4, false, true, 256, 4>(a, s);
    } else if (variant == 3 && a.levels == 4) {
        if (bf16) launch_k<R, 4, true, true>(a, s);
        else launch_k<R, 4, false, true>(a, s);
#endif
    } else {
        if (bf16) launch_k<R, 0, true, true>(a, s);
        else launch_k<R, 0, false, true>(a, s);
    }
    return hipGetLastError();
}

}  // namespace rc

// RAFTCORR_LOOKUP_VARIANT (dev library only, read per call): see launch_r.
hipError_t rc_launch_lookup(const rc::LookupArgs &a, int radius, int pyr_bf16, hipStream_t s) {
    if (a.P <= 0) return hipSuccess;
#ifdef RAFTCORR_DEV
    const int variant = rc::dev_knob("RAFTCORR_LOOKUP_VARIANT");
#else
    const int variant = 0;
#endif
    switch (radius) {
        case 1: return rc::launch_r<1>(a, pyr_bf16, variant, s);
        case 2: return rc::launch_r<2>(a, pyr_bf16, variant, s);
        case 3: return rc::launch_r<3>(a, pyr_bf16, variant, s);
        case 4: return rc::launch_r<4>(a, pyr_bf16, variant, s);
        case 5: return rc::launch_r<5>(a, pyr_bf16, variant, s);
        case 6: return rc::launch_r<6>(a, pyr_bf16, variant, s);
        case 7: return rc::launch_r<7>(a, pyr_bf16, variant, s);
        case 8: return rc::launch_r<8>(a, pyr_bf16, variant, s);
        default: return hipErrorInvalidValue;
    }
}

#ifdef RAFTCORR_DEV
// Dev-only entry: the sheared pair lookup (fp32, 4 levels, r = 4) over levels
// 0 and 2 stored as S_i[b,h][k][w1] (K0 / K2 rows of ldw floats per image row).
extern "C" int rc_dev_lookup_sheared_pair(const void *lvl0, const void *lvl2, long K0, long K2, long ldw,
                                          const int *widths, const float *coords_x, long cbs, int B, int H,
                                          int W1, float *out, void *stream) {
    rc::LookupArgs a{};
    for (int i = 0; i < 4; ++i) a.W[i] = widths[i];
    a.coords = coords_x;
    a.cbs = cbs;
    a.out = out;
    a.P = (long long)B * H * W1;
    a.HW = H * W1;
    a.W1 = W1;
    a.levels = 4;
    if (a.P <= 0) return 0;
    const unsigned nblk = (unsigned)((a.P + 255) / 256);
    hipLaunchKernelGGL((rc::lookup_sheared_pair_kernel<4>), dim3(nblk), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), a, static_cast<const float *>(lvl0),
                       static_cast<const float *>(lvl2), (long long)K0, (long long)K2, (long long)ldw);
    return hipGetLastError() == hipSuccess ? 0 : 3;
}
#endif

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
