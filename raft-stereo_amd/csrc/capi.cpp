// C-ABI entry points declared in include/raftcorr.h.
//
// Validation mirrors the reference's failure modes where it has them
// (e.g. W2 < 2^num_levels makes avg_pool2d raise at model.py:294), then
// launches on the caller's stream.  Nothing here allocates or synchronises, so
// every entry point is safe inside hipStreamBeginCapture.
#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#include "../../include/raftcorr.h"
#include "common.h"

namespace {
thread_local char g_err[512] = "";

int fail(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}

int hip_rc(hipError_t e, const char *what) {
    if (e == hipSuccess) return RC_OK;
    return fail(RC_EHIP, "%s: %s", what, hipGetErrorString(e));
}

bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// RC_SHADOW (ABI v5): byte offset from a stored level's base to its copy.
long long shadow_offset(long long rows, long long ld, int esize) { return RC_SHADOW_OFFSET(rows, ld, esize); }

// pyr_dtype bits an entry point accepts: the element type (low byte), the
// RC_SHADOW_LEVEL bits and, where the pair kernel serves it, RC_OUT_CHANNELS_LAST.
int check_flags(const char *who, int pyr_dtype, bool allow_cl, bool build = false, bool allow_disp = false,
                bool allow_rec = false) {
    const unsigned known = 0xFFu | RC_SHADOW | (allow_cl ? (unsigned)RC_OUT_CHANNELS_LAST : 0u) |
                           (build ? (unsigned)RC_BUILD_EXACT_F32 : 0u) |
                           (allow_disp ? (unsigned)RC_LAYOUT_DISPARITY : 0u) |
                           (allow_rec ? (unsigned)RC_LAYOUT_RECORDS : 0u);
    if (!allow_cl && (pyr_dtype & RC_OUT_CHANNELS_LAST))
        return fail(RC_EUNSUPPORTED, "%s: RC_OUT_CHANNELS_LAST is only defined for "
                    "rc_corr_lookup_chain / rc_corr_lookup_step", who);
    if (!allow_disp && (pyr_dtype & RC_LAYOUT_DISPARITY))
        return fail(RC_EUNSUPPORTED, "%s: RC_LAYOUT_DISPARITY is only defined for "
                    "rc_corr_build / rc_corr_lookup_chain", who);
    if (!allow_rec && (pyr_dtype & RC_LAYOUT_RECORDS))
        return fail(RC_EUNSUPPORTED, "%s: RC_LAYOUT_RECORDS is only defined for "
                    "rc_corr_build / rc_corr_lookup_chain / rc_corr_lookup_step", who);
    if ((pyr_dtype & RC_LAYOUT_DISPARITY) && (pyr_dtype & RC_LAYOUT_RECORDS))
        return fail(RC_EINVAL, "%s: RC_LAYOUT_DISPARITY and RC_LAYOUT_RECORDS exclude each other", who);
    if ((unsigned)pyr_dtype & ~known)
        return fail(RC_EINVAL, "%s: unknown pyr_dtype flag bits 0x%x", who, (unsigned)pyr_dtype & ~known);
    return RC_OK;
}

bool is_pow2_float(float v) {
    int e;
    return std::frexp(v, &e) == 0.5f;
}
}  // namespace


extern "C" int rc_abi_version(void) { return RC_ABI_VERSION; }

extern "C" const char *rc_last_error(void) { return g_err; }

extern "C" int rc_corr_build(const void *fmap1, const void *fmap2, int fmap_dtype, int B, int D,
                             int H, int W1, int W2, void *const *pyr, const long *pyr_ld, int nbuf,
                             int pyr_dtype, void *stream) {
    g_err[0] = 0;
    if (int e = check_flags("rc_corr_build", pyr_dtype, false, true, true, true)) return e;
    const bool exact_f32 = (pyr_dtype & RC_BUILD_EXACT_F32) != 0;
    const bool disp = (pyr_dtype & RC_LAYOUT_DISPARITY) != 0;
    const bool rec = (pyr_dtype & RC_LAYOUT_RECORDS) != 0;
    const unsigned shmask = ((unsigned)pyr_dtype >> 8) & 0xFFu;   // RC_SHADOW_LEVEL bits
    pyr_dtype &= 0xFF;
    if (B < 0 || D <= 0 || H < 0 || W1 < 0 || W2 <= 0)
        return fail(RC_EINVAL, "rc_corr_build: bad shape B=%d D=%d H=%d W1=%d W2=%d", B, D, H, W1, W2);

    if (nbuf < 1 || nbuf > RC_MAX_LEVELS)
        return fail(RC_EINVAL, "rc_corr_build: nbuf=%d outside 1..%d", nbuf, RC_MAX_LEVELS);
    if ((W2 >> (nbuf - 1)) < 1)
        return fail(RC_EINVAL,
                    "rc_corr_build: pyramid level %d of width %d would be empty "
                    "(avg_pool2d output size too small, model.py:294)",
                    nbuf - 1, W2);
    if (fmap_dtype != RC_F32 && fmap_dtype != RC_BF16)
        return fail(RC_EINVAL, "rc_corr_build: unknown fmap dtype %d", fmap_dtype);
    if (pyr_dtype != RC_F32 && pyr_dtype != RC_BF16)
        return fail(RC_EINVAL, "rc_corr_build: unknown pyramid dtype %d", pyr_dtype);
    if (!pyr) return fail(RC_EINVAL, "rc_corr_build: null pyramid array");
    if (disp) {   // RC_LAYOUT_DISPARITY: the split build's pair layout only
        if (fmap_dtype != RC_F32 || pyr_dtype != RC_F32 || exact_f32 || shmask)
            return fail(RC_EUNSUPPORTED, "rc_corr_build: RC_LAYOUT_DISPARITY needs fp32 fmaps and pyramid, "
                        "the split build and no shadow copies");
        if (!(nbuf == 1 || (nbuf == 3 && !pyr[1])))
            return fail(RC_EUNSUPPORTED, "rc_corr_build: RC_LAYOUT_DISPARITY stores the pair layout: "
                        "nbuf 1, or 3 with pyr[1] NULL");
        if (W1 % 4 || W2 % 4)
            return fail(RC_EUNSUPPORTED, "rc_corr_build: RC_LAYOUT_DISPARITY needs W1, W2 multiples of 4");
        if (!pyr_ld) return fail(RC_EINVAL, "rc_corr_build: RC_LAYOUT_DISPARITY needs pyr_ld");
        for (int l = 0; l < nbuf; l += 2) {
            if (pyr_ld[l] < W1 || pyr_ld[l] % 4)
                return fail(RC_EINVAL, "rc_corr_build: disparity-major row stride %ld of level %d must be "
                            ">= W1 = %d and a multiple of 4", pyr_ld[l], l, W1);
            if ((long long)B * H * RC_SHEAR_ROWS(W2, W1, l) * pyr_ld[l] * 4 >= 0xFFFFFF00LL)
                return fail(RC_EUNSUPPORTED, "rc_corr_build: disparity-major level %d exceeds 4 GiB", l);
        }
    }
    if (rec) {   // RC_LAYOUT_RECORDS: the bf16 ring build's deferred epilogue, one tile per row
        if (fmap_dtype != RC_BF16 || pyr_dtype != RC_BF16 || exact_f32 || shmask)
            return fail(RC_EUNSUPPORTED, "rc_corr_build: RC_LAYOUT_RECORDS needs bf16 fmaps and pyramid "
                        "and no shadow copies");
        if (nbuf != 3 || pyr[1] || pyr[2])
            return fail(RC_EUNSUPPORTED, "rc_corr_build: RC_LAYOUT_RECORDS stores the 4-level pair layout: "
                        "nbuf 3 with pyr[0] the records and pyr[1], pyr[2] NULL");
        if (W2 <= 64 || W2 > 320 || D <= 224)
            return fail(RC_EUNSUPPORTED, "rc_corr_build: RC_LAYOUT_RECORDS needs 64 < W2 <= 320 and D > 224 "
                        "(W2=%d D=%d)", W2, D);
        if ((long long)D * H * (W1 > W2 ? W1 : W2) * 2 >= (1LL << 30))
            return fail(RC_EUNSUPPORTED, "rc_corr_build: RC_LAYOUT_RECORDS: fmap image over 1 GiB");
    }
    if ((long long)B * H * W1 == 0) return RC_OK;
    if (!fmap1 || !fmap2 || !aligned16(fmap1) || !aligned16(fmap2))
        return fail(RC_EINVAL, "rc_corr_build: feature maps must be non-null and 16-byte aligned");
    const int nfused = nbuf < 7 ? nbuf : 7;
    for (int l = 0; l < nbuf; ++l) {
        // a NULL level l >= 1 inside the fused epilogue is computed (the next
        // level needs it) but not stored; later levels are pooled from memory
        const bool may_skip = l >= 1 && l < nfused && (nbuf <= 7 || l < 6);
        if (!pyr[l] && may_skip) continue;
        if (!pyr[l] || !aligned16(pyr[l]))
            return fail(RC_EINVAL, "rc_corr_build: pyramid buffer %d null or not 16-byte aligned", l);
        if (!disp && !rec && pyr_ld && pyr_ld[l] < (long)(W2 >> l))
            return fail(RC_EINVAL, "rc_corr_build: row stride %ld of level %d < width %d", pyr_ld[l],
                        l, W2 >> l);
    }

    rc::BuildArgs a{};
    a.f1 = fmap1;
    a.f2 = fmap2;
    a.B = B; a.D = D; a.H = H; a.W1 = W1; a.W2 = W2;
    a.nfused = nfused;
    if (rec) {
        a.rec = pyr[0];
        a.rec_nr = RC_REC_COUNT(W2);
    }
    for (int l = 0; l < a.nfused && !rec; ++l) {
        a.lvl[l] = pyr[l];
        a.ld[l] = pyr_ld ? pyr_ld[l] : (W2 >> l);
        if ((shmask >> l & 1u) && pyr[l])
            a.shadow[l] = shadow_offset((long long)B * H * W1, a.ld[l], pyr_dtype == RC_BF16 ? 2 : 4);
        if (disp && pyr[l]) a.shk[l] = RC_SHEAR_ROWS(W2, W1, l);
    }
    a.tiles_m = (W1 + 127) / 128;
    a.tiles_n = (W2 + 127) / 128;
    a.sq = std::sqrt((float)D);                 // torch.sqrt(torch.tensor(D).float()), :326
    a.pow2 = is_pow2_float(a.sq) ? 1 : 0;
    a.scale = 1.0f / a.sq;                      // exact when pow2
    a.pyr_bf16 = pyr_dtype == RC_BF16;
#ifdef RAFTCORR_DEV
    a.stagger = rc::dev_knob("RAFTCORR_STAGGER");
#endif
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    // fp32 fmaps + fp32 pyramid: exact fp32 MFMA.  bf16 fmaps, or a bf16
    // pyramid (bf16-level tolerance requested), take the bf16 MFMA kernel.
    const bool bf16_mma = fmap_dtype == RC_BF16 || pyr_dtype == RC_BF16;
    // fp32: the split-bf16 kernel (fp32 accuracy, volume_split.hip) unless the
    // exact fp32 MFMA kernel is asked for or the shape is outside the split
    // kernel's addressing (hipErrorNotSupported: nothing was launched)
    hipError_t e = hipErrorNotSupported;
    if (bf16_mma) e = rc_launch_build_bf16mma(a, fmap_dtype == RC_BF16, s);
    else if (!exact_f32) e = rc_launch_build_split(a, s);
    if (e == hipErrorNotSupported && disp)
        return fail(RC_EUNSUPPORTED, "rc_corr_build: RC_LAYOUT_DISPARITY: shape outside the split build");
    if (e == hipErrorNotSupported && rec)
        return fail(RC_EUNSUPPORTED, "rc_corr_build: RC_LAYOUT_RECORDS: shape outside the records build");
    if (e == hipErrorNotSupported && !bf16_mma) e = rc_launch_build_f32(a, s);
    int rc = hip_rc(e, "rc_corr_build: volume launch");
    if (rc) return rc;
    const long rows = (long)B * H * W1;
    for (int l = a.nfused; l < nbuf; ++l) {
        const long long ldi = pyr_ld ? pyr_ld[l - 1] : (W2 >> (l - 1));
        const long long ldo = pyr_ld ? pyr_ld[l] : (W2 >> l);
        rc = hip_rc(rc_launch_pool(pyr[l - 1], ldi, pyr[l], ldo, rows, W2 >> (l - 1), a.pyr_bf16, s),
                    "rc_corr_build: pool launch");
        if (rc) return rc;
        if ((shmask >> l & 1u) && pyr[l]) {   // the same pooling step once more, into the level's shadow copy
            void *sh = static_cast<char *>(pyr[l]) + shadow_offset(rows, ldo, a.pyr_bf16 ? 2 : 4);
            rc = hip_rc(rc_launch_pool(pyr[l - 1], ldi, sh, ldo, rows, W2 >> (l - 1), a.pyr_bf16, s),
                        "rc_corr_build: pool launch");
            if (rc) return rc;
        }
    }
    return RC_OK;
}

extern "C" int rc_corr_pool(const void *in, long ld_in, void *out, long ld_out, long rows,
                            int W_in, int dtype, void *stream) {
    g_err[0] = 0;
    if (int e = check_flags("rc_corr_pool", dtype, false)) return e;
    dtype &= 0xFF;    // pools the primary copy; a shadow is not written
    if (rows < 0 || W_in < 2 || ld_in < W_in || ld_out < W_in / 2)
        return fail(RC_EINVAL, "rc_corr_pool: bad shape rows=%ld W_in=%d ld_in=%ld ld_out=%ld", rows,
                    W_in, ld_in, ld_out);
    if (dtype != RC_F32 && dtype != RC_BF16)
        return fail(RC_EINVAL, "rc_corr_pool: unknown dtype %d", dtype);
    if (rows == 0) return RC_OK;
    if (!in || !out) return fail(RC_EINVAL, "rc_corr_pool: null pointer");
    return hip_rc(rc_launch_pool(in, ld_in, out, ld_out, rows, W_in, dtype == RC_BF16,
                                 reinterpret_cast<hipStream_t>(stream)),
                  "rc_corr_pool: launch");
}

namespace {
// Shared validation of the lookup entry points; fills `a` or returns an error.
int prep_lookup(const char *who, const void *const *pyr, const int *widths, const long *pyr_ld,
                int pyr_dtype, int levels, int radius, const float *coords_x,
                long coord_batch_stride, int B, int H, int W1, const float *out, rc::LookupArgs &a,
                bool *empty, bool allow_null = false) {
    *empty = false;
    const bool disp = (pyr_dtype & RC_LAYOUT_DISPARITY) != 0;     // rows of W1 (or more) per diagonal
    const bool rec = (pyr_dtype & RC_LAYOUT_RECORDS) != 0;        // pyr[0] = the records
    const unsigned shmask = ((unsigned)pyr_dtype >> 8) & 0xFFu;   // RC_SHADOW_LEVEL bits
    pyr_dtype &= 0xFF;
    if (levels < 1 || levels > RC_MAX_LEVELS)
        return fail(RC_EINVAL, "%s: levels=%d outside 1..%d", who, levels, RC_MAX_LEVELS);
    if (radius < 1 || radius > 8)
        return fail(RC_EUNSUPPORTED, "%s: radius=%d outside 1..8", who, radius);
    if (pyr_dtype != RC_F32 && pyr_dtype != RC_BF16)
        return fail(RC_EINVAL, "%s: unknown pyramid dtype %d", who, pyr_dtype);
    if (B < 0 || H < 0 || W1 < 0)
        return fail(RC_EINVAL, "%s: bad shape B=%d H=%d W1=%d", who, B, H, W1);
    if (!pyr || !widths) return fail(RC_EINVAL, "%s: null pyramid/width array", who);
    const long long P = (long long)B * H * W1;
    if (P == 0) {
        *empty = true;
        return RC_OK;
    }
    if ((long long)H * W1 > 0x7FFFFFFF) return fail(RC_EUNSUPPORTED, "%s: H*W1 too large", who);
    if (!coords_x || !out) return fail(RC_EINVAL, "%s: null coords/out", who);
    a = rc::LookupArgs{};
    for (int i = 0; i < levels; ++i) {
        if (widths[i] < 1) return fail(RC_EINVAL, "%s: level %d width %d", who, i, widths[i]);
        if (!pyr[i] && allow_null && i > 0) {      // recomputed by the kernel, never read
            a.lvl[i] = nullptr;
            a.W[i] = widths[i];
            a.ld[i] = widths[i];
            continue;
        }
        if (!pyr[i] || !aligned16(pyr[i]))
            return fail(RC_EINVAL, "%s: level %d null or not 16-byte aligned", who, i);
        a.lvl[i] = pyr[i];
        a.W[i] = widths[i];
        a.ld[i] = pyr_ld ? pyr_ld[i] : widths[i];
        if (rec) {
            if (i > 0) return fail(RC_EINVAL, "%s: RC_LAYOUT_RECORDS: pyr[%d] must be NULL", who, i);
            a.ld[0] = widths[0];
            a.rec_nr = RC_REC_COUNT(widths[0]);
            continue;
        }
        if (disp) {
            if (a.ld[i] < W1 || a.ld[i] % 4)
                return fail(RC_EINVAL, "%s: disparity-major row stride %lld of level %d must be >= W1 = %d "
                            "and a multiple of 4", who, a.ld[i], i, W1);
            a.shk[i] = RC_SHEAR_ROWS(widths[0], W1, i);
            if ((long long)B * H * a.shk[i] * a.ld[i] * 4 >= 0xFFFFFF00LL)
                return fail(RC_EUNSUPPORTED, "%s: disparity-major level %d exceeds 4 GiB", who, i);
            continue;
        }
        if (a.ld[i] < widths[i])
            return fail(RC_EINVAL, "%s: level %d row stride %lld < width %d", who, i, a.ld[i],
                        widths[i]);
        if (shmask >> i & 1u) {
            const int es = pyr_dtype == RC_BF16 ? 2 : 4;
            a.shadow[i] = shadow_offset(P, a.ld[i], es);
            // the pair kernel addresses both copies with 32-bit buffer offsets
            if (a.shadow[i] + P * a.ld[i] * es > 0xFFFFFF00LL)
                return fail(RC_EUNSUPPORTED, "%s: level %d with its shadow copy exceeds 4 GiB", who, i);
        }
    }
    a.coords = coords_x;
    a.cbs = coord_batch_stride;
    a.P = P;
    a.HW = H * W1;
    a.W1 = W1;
    a.levels = levels;
    return RC_OK;
}
}  // namespace

namespace {
// Which pool-chain kernel serves a request (rc_corr_lookup_chain and the
// chain mode of rc_corr_lookup_step): the pair kernel (reads levels 0 and 2)
// for 2 levels, or for 4 levels when level 2 is given; otherwise the level-1
// chain kernel (reads levels 0 and 1) for 3-4 levels.
int chain_kind(const char *who, const void *const *pyr, const int *widths, int levels, int radius,
               bool *pair, bool rec = false) {
    if (levels < 2 || levels > 4 || radius < 1 || radius > 4)
        return fail(RC_EUNSUPPORTED, "%s: levels 2..4 and radius 1..4 only", who);
    for (int i = 1; i < levels; ++i)
        if (widths[i] != widths[i - 1] / 2)
            return fail(RC_EINVAL, "%s: width %d of level %d is not floor(%d/2)", who, widths[i], i,
                        widths[i - 1]);
    *pair = levels == 2 || (levels == 4 && (pyr[2] != nullptr || rec));
    // the pair kernel's window argument holds for widths up to 2^16 (lookup.hip)
    if (*pair && widths[0] > 65536)
        return fail(RC_EUNSUPPORTED, "%s: level-0 width %d > 65536 for the pair kernel", who,
                    widths[0]);
    if (!*pair && !pyr[1])
        return fail(RC_EINVAL, "%s: %d levels need level 1 (or level 2 with 4 levels)", who, levels);
    if (!*pair && levels < 3)
        return fail(RC_EUNSUPPORTED, "%s: the level-1 chain needs 3..4 levels", who);
    return RC_OK;
}

// Row strides the chain kernels read with 16-B chunks must be whole chunks
// (multiples of 4 fp32 / 8 bf16 elements).
int chain_strides(const char *who, const rc::LookupArgs &a, bool pair, bool bf16 = false) {
    const int need[2] = {0, pair ? 2 : 1};
    const int epc = bf16 ? 8 : 4;
    for (int k = 0; k < 2; ++k) {
        const int i = need[k];
        if (i < a.levels && a.ld[i] % epc != 0)
            return fail(RC_EINVAL, "%s: level-%d row stride %lld is not a multiple of %d", who, i,
                        a.ld[i], epc);
    }
    return RC_OK;
}
}  // namespace

extern "C" int rc_corr_lookup(const void *const *pyr, const int *widths, const long *pyr_ld,
                              int pyr_dtype, int levels, int radius, const float *coords_x,
                              long coord_batch_stride, int B, int H, int W1, float *out,
                              void *stream) {
    g_err[0] = 0;
    rc::LookupArgs a;
    bool empty;
    if (int e = check_flags("rc_corr_lookup", pyr_dtype, false)) return e;
    int rc = prep_lookup("rc_corr_lookup", pyr, widths, pyr_ld, pyr_dtype, levels, radius, coords_x,
                         coord_batch_stride, B, H, W1, out, a, &empty);
    if (rc || empty) return rc;
    pyr_dtype &= 0xFF;
    a.out = out;
    return hip_rc(rc_launch_lookup(a, radius, pyr_dtype == RC_BF16,
                                   reinterpret_cast<hipStream_t>(stream)),
                  "rc_corr_lookup: launch");
}

extern "C" int rc_corr_lookup_chain(const void *const *pyr, const int *widths, const long *pyr_ld,
                                    int pyr_dtype, int levels, int radius, const float *coords_x,
                                    long coord_batch_stride, int B, int H, int W1, float *out,
                                    void *stream) {
    g_err[0] = 0;
    rc::LookupArgs a;
    bool empty;
    if (int e = check_flags("rc_corr_lookup_chain", pyr_dtype, true, false, true, true)) return e;
    int rc = prep_lookup("rc_corr_lookup_chain", pyr, widths, pyr_ld, pyr_dtype, levels, radius,
                         coords_x, coord_batch_stride, B, H, W1, out, a, &empty, true);
    if (rc) return rc;
    const bool cl = (pyr_dtype & RC_OUT_CHANNELS_LAST) != 0;
    const bool disp = (pyr_dtype & RC_LAYOUT_DISPARITY) != 0;
    const bool rec = (pyr_dtype & RC_LAYOUT_RECORDS) != 0;
    const bool shadowed = ((unsigned)pyr_dtype & RC_SHADOW) != 0;
    pyr_dtype &= 0xFF;
    bool pair;
    if ((rc = chain_kind("rc_corr_lookup_chain", pyr, widths, levels, radius, &pair, rec))) return rc;
    if (rec && (levels != 4 || pyr_dtype != RC_BF16 || shadowed))
        return fail(RC_EUNSUPPORTED, "rc_corr_lookup_chain: RC_LAYOUT_RECORDS needs the 4-level bf16 pair "
                    "layout and no shadow copies");
    if (disp && (!pair || pyr_dtype != RC_F32 || cl || shadowed))
        return fail(RC_EUNSUPPORTED, "rc_corr_lookup_chain: RC_LAYOUT_DISPARITY needs the fp32 pair layout "
                    "(2 levels, or 4 with level 2 given), NCHW output and no shadow copies");
    if (pyr_dtype == RC_BF16 && !pair)
        return fail(RC_EUNSUPPORTED, "rc_corr_lookup_chain: a bf16 pyramid needs the pair layout "
                    "(2 levels, or 4 with level 2 given)");
    if (cl && !pair)
        return fail(RC_EUNSUPPORTED, "rc_corr_lookup_chain: RC_OUT_CHANNELS_LAST needs the pair layout");
    if (empty) return RC_OK;
    a.out = out;
    a.out_cl = cl;
    if (!rec && (rc = chain_strides("rc_corr_lookup_chain", a, pair, pyr_dtype == RC_BF16))) return rc;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    return hip_rc(pair ? rc_launch_lookup_pair(a, radius, pyr_dtype == RC_BF16, s)
                       : rc_launch_lookup_chain(a, radius, s),
                  "rc_corr_lookup_chain: launch");
}

extern "C" int rc_corr_lookup_step(const void *const *pyr, const int *widths, const long *pyr_ld,
                                   int pyr_dtype, int levels, int radius, int chain,
                                   const float *coords1, const float *delta, float *coords1_out,
                                   float *flow_out, int B, int H, int W1, float *out,
                                   void *stream) {
    g_err[0] = 0;
    rc::LookupArgs a;
    bool empty;
    if (int e = check_flags("rc_corr_lookup_step", pyr_dtype, true, false, false, true)) return e;
    const bool rec = (pyr_dtype & RC_LAYOUT_RECORDS) != 0;
    const bool shadowed = ((unsigned)pyr_dtype & RC_SHADOW) != 0;
    if (rec && !chain) return fail(RC_EUNSUPPORTED, "rc_corr_lookup_step: RC_LAYOUT_RECORDS needs chain != 0");
    int rc = prep_lookup("rc_corr_lookup_step", pyr, widths, pyr_ld, pyr_dtype, levels, radius,
                         coords1, 2L * H * W1, B, H, W1, out, a, &empty, chain != 0);
    if (rc || empty) return rc;
    const bool cl = (pyr_dtype & RC_OUT_CHANNELS_LAST) != 0;
    pyr_dtype &= 0xFF;
    if (!coords1_out || !flow_out)
        return fail(RC_EINVAL, "rc_corr_lookup_step: null coords1_out / flow_out");
    bool pair = false;
    if (chain) {
        if ((rc = chain_kind("rc_corr_lookup_step", pyr, widths, levels, radius, &pair, rec))) return rc;
        if (pyr_dtype != RC_F32 && !pair)
            return fail(RC_EUNSUPPORTED, "rc_corr_lookup_step: a bf16 pyramid needs the pair layout");
        if (rec && (levels != 4 || pyr_dtype != RC_BF16 || shadowed))
            return fail(RC_EUNSUPPORTED, "rc_corr_lookup_step: RC_LAYOUT_RECORDS needs the 4-level bf16 pair "
                        "layout and no shadow copies");
        if (!rec && (rc = chain_strides("rc_corr_lookup_step", a, pair, pyr_dtype == RC_BF16))) return rc;
    }
    if (cl && !pair)
        return fail(RC_EUNSUPPORTED, "rc_corr_lookup_step: RC_OUT_CHANNELS_LAST needs the pair layout");
    a.out = out;
    a.out_cl = cl;
    a.step = 1;
    a.W1 = W1;
    a.delta = delta;
    a.coords_out = coords1_out;
    a.flow_out = flow_out;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    return hip_rc(chain ? (pair ? rc_launch_lookup_pair(a, radius, pyr_dtype == RC_BF16, s)
                                : rc_launch_lookup_chain(a, radius, s))
                        : rc_launch_lookup(a, radius, pyr_dtype == RC_BF16, s),
                  "rc_corr_lookup_step: launch");
}

namespace {
// Validation shared by rc_corr_lookup_backward and rc_corr_lookup_backward_calls.
int prep_lookup_bwd(const char *who, void *const *grad_pyr, const int *widths, const long *grad_ld,
                    int levels, int radius, const float *coords_x, long coord_batch_stride, int B,
                    int H, int W1, const float *grad_out, rc::LookupBwdArgs &a, bool *empty,
                    bool *pair_out) {
    // RC_SHADOW_LEVEL(l) bits above the level count: gradient copies (pair layout)
    const unsigned shmask = ((unsigned)levels >> 8) & 0xFFu;
    levels &= 0xFF;
    rc::LookupArgs la;
    int rc = prep_lookup(who, grad_pyr, widths, grad_ld, RC_F32, levels, radius, coords_x,
                         coord_batch_stride, B, H, W1, grad_out, la, empty, true);
    if (rc || *empty) return rc;
    // pair-folded buffers: levels 1 and 3 NULL, their gradients folded into
    // levels 0 and 2 (2 or 4 levels, radius 1..4, widths halving, W <= 2^16)
    const bool pair = levels >= 2 && !grad_pyr[1];
    *pair_out = pair;
    if (pair) {
        bool ok = (levels == 2 || (levels == 4 && grad_pyr[2] && !grad_pyr[3])) && radius <= 4 &&
                  widths[0] <= 65536;
        for (int i = 1; i < levels; ++i) ok = ok && widths[i] == widths[i - 1] / 2;
        if (!ok)
            return fail(RC_EINVAL, "%s: NULL gradient levels need the pair layout (levels 2 or 4, "
                        "level 1 [and 3] NULL, radius <= 4, halving widths)", who);
        if (shmask && (levels != 4 || (shmask & ~0x5u)))
            return fail(RC_EUNSUPPORTED, "%s: RC_SHADOW gradient copies are levels 0 and 2 of the "
                        "4-level pair layout", who);
    } else if (shmask) {
        return fail(RC_EUNSUPPORTED, "%s: RC_SHADOW needs the pair layout", who);
    } else {
        for (int i = 1; i < levels; ++i)
            if (!grad_pyr[i]) return fail(RC_EINVAL, "%s: level %d null", who, i);
    }
    a = rc::LookupBwdArgs{};
    for (int i = 0; i < levels; ++i) {
        a.W[i] = la.W[i];
        a.ld[i] = la.ld[i];
        if (!grad_pyr[i]) {
            a.g[i] = nullptr;
            continue;
        }
        if (la.ld[i] % 4 != 0)
            return fail(RC_EINVAL, "%s: row stride %lld of level %d is not a multiple of 4", who,
                        la.ld[i], i);
        a.g[i] = static_cast<float *>(const_cast<void *>(la.lvl[i]));
        if (shmask >> i & 1u) {
            a.shadow[i] = shadow_offset(la.P, la.ld[i], 4);
            if (a.shadow[i] + la.P * la.ld[i] * 4 > 0xFFFFFF00LL)
                return fail(RC_EUNSUPPORTED, "%s: level %d with its shadow copy exceeds 4 GiB", who, i);
        }
    }
    a.coords = coords_x;
    a.cbs = coord_batch_stride;
    a.grad_out = grad_out;
    a.P = la.P;
    a.HW = la.HW;
    a.levels = levels;
    return RC_OK;
}
}  // namespace

extern "C" int rc_corr_lookup_backward(void *const *grad_pyr, const int *widths,
                                       const long *grad_ld, int levels, int radius,
                                       const float *coords_x, long coord_batch_stride, int B,
                                       int H, int W1, const float *grad_out, void *stream) {
    g_err[0] = 0;
    if (levels & ~0xFFFF)
        return fail(RC_EINVAL, "rc_corr_lookup_backward: unknown flag bits 0x%x", levels & ~0xFFFF);
    rc::LookupBwdArgs a;
    bool empty = false, pair = false;
    int rc = prep_lookup_bwd("rc_corr_lookup_backward", grad_pyr, widths, grad_ld, levels, radius,
                             coords_x, coord_batch_stride, B, H, W1, grad_out, a, &empty, &pair);
    if (rc || empty) return rc;
    return hip_rc(rc_launch_lookup_bwd(a, radius, reinterpret_cast<hipStream_t>(stream)),
                  "rc_corr_lookup_backward: launch");
}

extern "C" int rc_corr_lookup_backward_calls(void *const *grad_pyr, const int *widths,
                                             const long *grad_ld, int levels, int radius,
                                             int n_calls, const float *const *coords_x,
                                             const long *coord_batch_stride, int B, int H, int W1,
                                             const float *const *grad_out, void *stream) {
    g_err[0] = 0;
    const char *who = "rc_corr_lookup_backward_calls";
    const bool overwrite = (levels & RC_GRAD_OVERWRITE) != 0;
    levels &= ~RC_GRAD_OVERWRITE;
    if (levels & ~0xFFFF) return fail(RC_EINVAL, "%s: unknown flag bits 0x%x", who, levels & ~0xFFFF);
    if (n_calls < 0) return fail(RC_EINVAL, "%s: n_calls=%d", who, n_calls);
    if (n_calls > 0 && (!coords_x || !coord_batch_stride || !grad_out))
        return fail(RC_EINVAL, "%s: null coords / stride / grad_out array", who);
    if (levels & 0xFF00) return fail(RC_EUNSUPPORTED, "%s: RC_SHADOW gradient copies", who);
    const hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    rc::LookupBwdArgs a;
    bool empty = false, pair = false;
    for (int c = 0; c < n_calls; ++c) {       // every call validated before any launch
        int rc = prep_lookup_bwd(who, grad_pyr, widths, grad_ld, levels, radius, coords_x[c],
                                 coord_batch_stride[c], B, H, W1, grad_out[c], a, &empty, &pair);
        if (rc || empty) return rc;
    }
    if (n_calls == 0) {
        if (overwrite) return fail(RC_EINVAL, "%s: RC_GRAD_OVERWRITE with no calls", who);
        return RC_OK;
    }
    auto per_call = [&]() -> int {
        // per-level layout, or rows too wide for LDS: zero if asked, then one
        // rc_corr_lookup_backward launch per call
        if (overwrite)
            for (int i = 0; i < a.levels; ++i)
                if (a.g[i]) {
                    hipError_t e = hipMemsetAsync(a.g[i], 0, (size_t)(a.P * a.ld[i]) * 4, s);
                    if (e != hipSuccess) return hip_rc(e, "rc_corr_lookup_backward_calls: memset");
                }
        for (int c = 0; c < n_calls; ++c) {
            a.coords = coords_x[c];
            a.cbs = coord_batch_stride[c];
            a.grad_out = grad_out[c];
            hipError_t e = rc_launch_lookup_bwd(a, radius, s);
            if (e != hipSuccess) return hip_rc(e, "rc_corr_lookup_backward_calls: launch");
        }
        return RC_OK;
    };
    if (!pair) return per_call();
    rc::LookupBwdCallsArgs ca{};
    ca.g[0] = a.g[0];
    ca.ld[0] = a.ld[0];
    if (a.levels == 4) {
        ca.g[1] = a.g[2];
        ca.ld[1] = a.ld[2];
    }
    for (int i = 0; i < a.levels; ++i) ca.W[i] = a.W[i];
    ca.P = a.P;
    ca.HW = a.HW;
    // fused or per-call for the WHOLE request, decided before any launch
    if (!rc_lookup_bwd_calls_fits(ca, radius, a.levels, coord_batch_stride, n_calls)) return per_call();
    for (int c0 = 0; c0 < n_calls; c0 += rc::kMaxBwdCalls) {
        ca.ncalls = std::min(rc::kMaxBwdCalls, n_calls - c0);
        ca.accumulate = (c0 > 0 || !overwrite) ? 1 : 0;
        for (int c = 0; c < ca.ncalls; ++c) {
            ca.coords[c] = coords_x[c0 + c];
            ca.cbs[c] = coord_batch_stride[c0 + c];
            ca.grad_out[c] = grad_out[c0 + c];
        }
        hipError_t e = rc_launch_lookup_bwd_calls(ca, radius, a.levels, s);
        if (e != hipSuccess) return hip_rc(e, "rc_corr_lookup_backward_calls: launch");
    }
    return RC_OK;
}

extern "C" int rc_corr_build_backward(const void *fmap1, const void *fmap2, int fmap_dtype, int B,
                                      int D, int H, int W1, int W2, const void *const *grad_pyr,
                                      const long *grad_ld, int levels, float *grad_fmap1,
                                      float *grad_fmap2, void *stream) {
    g_err[0] = 0;
    const unsigned shmask = ((unsigned)levels >> 8) & 0xFFu;   // RC_SHADOW_LEVEL bits (pair layout)
    levels &= 0xFF;
    if (B < 0 || D <= 0 || H < 0 || W1 < 0 || W2 <= 0)
        return fail(RC_EINVAL, "rc_corr_build_backward: bad shape B=%d D=%d H=%d W1=%d W2=%d", B, D,
                    H, W1, W2);
    const bool exact_f32 = (fmap_dtype & RC_BUILD_EXACT_F32) != 0;
    fmap_dtype &= ~RC_BUILD_EXACT_F32;
    if (fmap_dtype != RC_F32)
        return fail(RC_EUNSUPPORTED, "rc_corr_build_backward: fp32 feature maps only");
    if (levels < 1 || levels > RC_MAX_LEVELS || (W2 >> (levels - 1)) < 1)
        return fail(RC_EINVAL, "rc_corr_build_backward: levels=%d invalid for W2=%d", levels, W2);
    if (!grad_pyr) return fail(RC_EINVAL, "rc_corr_build_backward: null gradient array");
    if ((long long)B * H * W1 == 0) return RC_OK;   // nothing to reduce; outputs are empty
    if (!fmap1 || !fmap2 || !grad_fmap1 || !grad_fmap2 || !aligned16(fmap1) || !aligned16(fmap2) ||
        !aligned16(grad_fmap1) || !aligned16(grad_fmap2))
        return fail(RC_EINVAL, "rc_corr_build_backward: feature maps and their gradients must be "
                    "non-null and 16-byte aligned");
    rc::BuildBwdArgs a{};
    // levels == 3 with grad_pyr[1] NULL: pair-folded gradients (levels 0, 2)
    const bool pair = levels == 3 && !grad_pyr[1];
    if (shmask && (!pair || (shmask & ~0x5u)))
        return fail(RC_EUNSUPPORTED, "rc_corr_build_backward: RC_SHADOW copies are levels 0 and 2 of "
                    "the pair layout");
    for (int l = 0; l < levels; ++l) {
        const long ld = grad_ld ? grad_ld[l] : (long)(W2 >> l);
        if (pair && l == 1) {
            a.g[1] = nullptr;
            a.ld[1] = W2 >> 1;
            a.Wl[1] = W2 >> 1;
            continue;
        }
        if (!grad_pyr[l] || !aligned16(grad_pyr[l]))
            return fail(RC_EINVAL, "rc_corr_build_backward: level gradient %d null or not 16-byte "
                        "aligned", l);
        if (ld < (long)(W2 >> l))
            return fail(RC_EINVAL, "rc_corr_build_backward: row stride %ld of level %d < width %d",
                        ld, l, W2 >> l);
        a.g[l] = static_cast<const float *>(grad_pyr[l]);
        a.ld[l] = ld;
        a.Wl[l] = W2 >> l;
        if (shmask >> l & 1u) a.shadow[l] = shadow_offset((long long)B * H * W1, ld, 4) / 4;
    }
    if (a.ld[0] % 4 != 0)
        return fail(RC_EINVAL, "rc_corr_build_backward: level-0 row stride %lld is not a multiple "
                    "of 4", a.ld[0]);
    a.nlev = levels;
    a.exact = exact_f32 ? 1 : 0;
    a.f1 = static_cast<const float *>(fmap1);
    a.f2 = static_cast<const float *>(fmap2);
    a.df1 = grad_fmap1;
    a.df2 = grad_fmap2;
    a.B = B; a.D = D; a.H = H; a.W1 = W1; a.W2 = W2;
    a.tm = (D + 127) / 128;
    a.tn1 = (W1 + 127) / 128;
    a.tn2 = (W2 + 127) / 128;
    a.sq = std::sqrt((float)D);                 // :326 divides by sqrt(float(D))
    a.pow2 = is_pow2_float(a.sq) ? 1 : 0;
    a.scale = 1.0f / a.sq;
    return hip_rc(rc_launch_volume_bwd(a, reinterpret_cast<hipStream_t>(stream)),
                  "rc_corr_build_backward: launch");
}

extern "C" int rc_corr_lookup_conv(const void *const *pyr, const int *widths, const long *pyr_ld,
                                   int pyr_dtype, int levels, int radius, const float *coords_x,
                                   long coord_batch_stride, int B, int H, int W1,
                                   const float *weight, const float *bias, int cout, int relu,
                                   float *out, void *stream) {
    g_err[0] = 0;
    rc::LookupArgs a;
    bool empty;
    if (int e = check_flags("rc_corr_lookup_conv", pyr_dtype, false)) return e;
    int rc = prep_lookup("rc_corr_lookup_conv", pyr, widths, pyr_ld, pyr_dtype, levels, radius,
                         coords_x, coord_batch_stride, B, H, W1, out, a, &empty);
    if (rc) return rc;
    pyr_dtype &= 0xFF;
    if (levels < 2 || levels > 4 || radius > 4)
        return fail(RC_EUNSUPPORTED, "rc_corr_lookup_conv: levels 2..4 and radius 1..4 only");
    if (cout < 1) return fail(RC_EINVAL, "rc_corr_lookup_conv: cout=%d", cout);
    if (empty) return RC_OK;
    if (!weight) return fail(RC_EINVAL, "rc_corr_lookup_conv: null weight");
    return hip_rc(rc_launch_lookup_conv(a, radius, pyr_dtype == RC_BF16, weight, bias, cout, relu,
                                        out, reinterpret_cast<hipStream_t>(stream)),
                  "rc_corr_lookup_conv: launch");
}

extern "C" int rc_convex_upsample(const float *flow, const float *mask, int N, int C, int H, int W,
                                  int factor, float *out, void *stream) {
    g_err[0] = 0;
    if (N < 0 || C < 1 || H < 0 || W < 0)
        return fail(RC_EINVAL, "rc_convex_upsample: bad shape N=%d C=%d H=%d W=%d", N, C, H, W);
    if (factor != 1 && factor != 2 && factor != 4 && factor != 8)
        return fail(RC_EUNSUPPORTED, "rc_convex_upsample: factor %d (1, 2, 4 or 8)", factor);
    if ((long long)N * H * W == 0) return RC_OK;
    if (!flow || !mask || !out) return fail(RC_EINVAL, "rc_convex_upsample: null pointer");
    return hip_rc(rc_launch_convex_upsample(flow, mask, N, C, H, W, factor, out,
                                            reinterpret_cast<hipStream_t>(stream)),
                  "rc_convex_upsample: launch");
}
