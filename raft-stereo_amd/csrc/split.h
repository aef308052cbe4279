// The exact three-way bf16 split of fp32 operands shared by the split-bf16
// MFMA kernels (volume_split.hip: the forward volume; backward.hip: the
// volume backward): x = h + m + l exactly for finite |x| < 3.39e38, and the
// six leading products of (h+m+l)(h'+m'+l') on v_mfma_f32_16x16x32_bf16
// (DESIGN.md §3.1c).
#pragma once
#include "common.h"
#include "epilogue.h"

namespace rc {

typedef unsigned u32x4s __attribute__((ext_vector_type(4)));
typedef __bf16 sp_bf16x2 __attribute__((ext_vector_type(2)));

// two fp32 -> packed bf16 (RNE), and back to fp32
__device__ __forceinline__ uint32_t sp_pack(float lo, float hi) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{lo, hi}, sp_bf16x2));   // v_cvt_pk_bf16_f32
}
__device__ __forceinline__ float sp_lo(uint32_t p) { return __builtin_bit_cast(float, p << 16); }
__device__ __forceinline__ float sp_hi(uint32_t p) { return __builtin_bit_cast(float, p & 0xFFFF0000u); }

struct SplitFrag {
    bf16x8 h, m, l;
};

// a - b as ONE scalar v_sub_f32: opaque to the SLP vectorizer, which would
// pair the residuals of two elements into v_pk_add_f32 -- beside MFMAs a
// packed f32 op costs ~4x the issue slots of two scalar ones
// (MI355X_MICROARCH.md, constants table: "an anti-lever beside MFMAs")
__device__ __forceinline__ float sp_sub(float a, float b) {
    float r;
    asm("v_sub_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// 8 consecutive d of one w -> head, middle and low bf16 pieces (each exact
// residual of the previous: x = h + m + l for finite |x| < 3.39e38).
// SCALAR (default): residuals by sp_sub (v_sub_f32); false: as the compiler
// packs them (the dev A/B kModePackedSub; config 2 build 286 vs 280 us,
// bit-identical, profiles/r04/d/build_ablate.log).
template <bool SCALAR = true>
__device__ __forceinline__ SplitFrag sp_split(const float (&x)[8]) {
    u32x4s h, m, l;
    auto sub = [](float a, float b) { return SCALAR ? sp_sub(a, b) : a - b; };
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t hp = sp_pack(x[2 * k], x[2 * k + 1]);
        const float r0 = sub(x[2 * k], sp_lo(hp)), r1 = sub(x[2 * k + 1], sp_hi(hp));   // exact
        const uint32_t mp = sp_pack(r0, r1);
        const float s0 = sub(r0, sp_lo(mp)), s1 = sub(r1, sp_hi(mp));                  // exact
        h[k] = hp;
        m[k] = mp;
        l[k] = sp_pack(s0, s1);
    }
    return SplitFrag{__builtin_bit_cast(bf16x8, h), __builtin_bit_cast(bf16x8, m), __builtin_bit_cast(bf16x8, l)};
}

// c += a * b to fp32 accuracy: the six leading piece products, small terms
// first (mm + hl + lh + hm + mh + hh); ml, lm, ll (< 2^-27 |a||b|) dropped.
__device__ __forceinline__ void sp_mma6(f32x4 &c, const SplitFrag &x, const SplitFrag &y) {
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x.m, y.m, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x.h, y.l, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x.l, y.h, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x.h, y.m, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x.m, y.h, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x.h, y.h, c, 0, 0, 0);
}

}  // namespace rc
