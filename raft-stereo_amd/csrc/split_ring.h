// Pieces of the split-bf16 volume kernel (volume_split.hip): the LDS-DMA
// ring's geometry and a lane's fragment read + split.
#pragma once
#include "common.h"
#include "epilogue.h"
#include "split.h"

namespace rc {

constexpr int kSpBK = 16;                   // d per ring stage (two per K step)
constexpr int kSpMaxFused = 5;              // levels the epilogue writes (more: pooled from memory)

// Ring geometry for stage rows TW floats wide (the tile width in w; 16 | TW,
// TW <= 128) and SL slots (stages; SL / 2 K steps: one in use, the rest in
// flight).  A DMA block holds two rows (2 TW fp32 = TW / 2 lanes x 16 B) plus
// 16 B of padding, so rows d and d + 8 (4 blocks apart) fall on different
// ds_read_b32 banks: 4 (8 TW + 16) / 4 = 16 mod 32 dwords for TW % 16 == 0.
//   TW 128, SL 4: the product, 66.5 KB -- two workgroups per CU;
//   TW 80, SL 6 / SL 4 (dev A/B, tiles of at most 5 fragments, W <= 160):
//   61.5 KB, two K steps in flight at the same two workgroups per CU / 41 KB,
//   three workgroups per CU.  Realtime graph step 61.8 / 61.5 vs 60.7 us:
//   not kept.
template <int TW, int SL>
struct SpRing {
    static_assert(TW % 16 == 0 && TW <= 128 && SL % 2 == 0 && SL >= 4, "split ring geometry");
    static constexpr int Blk = 8 * TW + 16;   // bytes per DMA block: 2 rows + 16 B pad
    static constexpr int Op = 8 * Blk;        // one operand tile of a stage: 16 rows
    static constexpr int Slot = 2 * Op;       // F1 + F2
    static constexpr int Bytes = SL * Slot;
    static constexpr int Wave = Bytes / 4;    // per-wave epilogue staging once the ring drains
    static constexpr int KA = SL / 2;         // K steps the ring holds
};
constexpr int kSpStb = 16 * (64 + 4) * 4;     // per-wave epilogue staging (epilogue_swapped, WT 64)
static_assert(4 * kSpStb <= SpRing<128, 4>::Bytes && 4 * kSpStb <= SpRing<80, 4>::Bytes,
              "epilogue staging aliases the ring");
// the pair epilogue (kModePairEpi, dev, wide ring only): two columns of levels
// 0-2 per wave, at WT = 64
static_assert(2 * 16 * ((64 + 4) + (32 + 4) + (16 + 4)) * 4 <= SpRing<128, 4>::Wave, "pair staging per wave");
// levels 0-2 of one column (the fast epilogue), at the narrow ring's WT <= 48
static_assert(16 * ((48 + 4) + (24 + 4) + (12 + 4)) * 4 <= SpRing<80, 4>::Wave, "staging per wave");

// One lane's fragment: rows r0..r0+7 (d inside the stage) of w column w of an
// operand tile at LDS byte address base.  Row d of the tile sits in block
// d >> 1 at +4 TW bytes for odd d.
template <int MODE, int TW = 128>
__device__ __forceinline__ SplitFrag sp_read(const char *base) {
    constexpr int Blk = SpRing<TW, 4>::Blk;
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = *reinterpret_cast<const float *>(base + (j >> 1) * Blk + (j & 1) * 4 * TW);
    if constexpr (MODE & kModeNoSplit) {     // dev timing probe: head piece only, reused thrice
        u32x4s h;
#pragma unroll
        for (int k = 0; k < 4; ++k) h[k] = sp_pack(x[2 * k], x[2 * k + 1]);
        const bf16x8 hb = __builtin_bit_cast(bf16x8, h);
        return SplitFrag{hb, hb, hb};
    }
    return sp_split<(MODE & kModePackedSub) == 0>(x);
}

}  // namespace rc
