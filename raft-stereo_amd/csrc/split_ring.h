// Pieces of the split-bf16 volume kernel (volume_split.hip): the LDS-DMA
// ring's geometry and a lane's fragment read + split.
#pragma once
#include "common.h"
#include "epilogue.h"
#include "split.h"

namespace rc {

constexpr int kSpBK = 16;                   // d per ring stage (two per K step)
constexpr int kSpBlk = 1040;                // bytes per DMA block: 2 rows of 128 fp32 + 16 B pad
constexpr int kSpOp = 8 * kSpBlk;           // one operand tile of a stage: 16 rows
constexpr int kSpSlot = 2 * kSpOp;          // F1 + F2
constexpr int kSpSL = 4;                    // ring slots (stages): one K step in flight, one in use
constexpr int kSpMaxFused = 5;              // levels the epilogue writes (more: pooled from memory)
constexpr int kSpStb = 16 * (64 + 4) * 4;   // per-wave epilogue staging (epilogue_swapped, WT 64)
static_assert(4 * kSpStb <= kSpSL * kSpSlot, "epilogue staging aliases the ring");
// the pair epilogue (kModePairEpi): two columns of levels 0-2 per wave, at WT = 64
static_assert(2 * 16 * ((64 + 4) + (32 + 4) + (16 + 4)) * 4 <= kSpSL * kSpSlot / 4, "pair staging per wave");

// One lane's fragment: rows r0..r0+7 (d inside the stage) of w column w of an
// operand tile at LDS byte address base.  Row d of the tile sits in block
// d >> 1 at +512 B for odd d.
template <int MODE>
__device__ __forceinline__ SplitFrag sp_read(const char *base) {
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = *reinterpret_cast<const float *>(base + (j >> 1) * kSpBlk + (j & 1) * 512);
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
