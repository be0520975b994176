// x3_split.h -- fp32 value -> (hi, lo) fp16 pair for the 3-product split MFMA (gfx950).
//
// x = hi + lo with hi = fp16(x), lo = fp16(x - hi); a product w x is then carried as
// w_hi x_hi + w_hi x_lo + w_lo x_hi in fp32 MFMA accumulators (22 significant bits per factor,
// the dropped w_lo x_lo term <= 2^-22 |w x|).  Included inside sgn::{anonymous}.
#pragma once
#include "agg_device.h"

namespace sgn {
namespace {

struct X3Pair {
    h8 hi, lo;
};

// (t * scale) -> (hi, lo) for a power-of-two `scale` (so t * scale is exact): each fp16 half is one
// v_fma_mix{lo,hi}_f16 (an fp32 FMA rounded once to fp16), 4 instructions per 2 values
__device__ __forceinline__ X3Pair split8_scaled(const float (&t)[8], float scale) {
    u32x4 hi, lo;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        uint32_t h, l;
        asm("v_fma_mixlo_f16 %0, %1, %2, 0" : "=v"(h) : "v"(t[2 * q]), "v"(scale));
        asm("v_fma_mixhi_f16 %0, %1, %2, 0" : "+v"(h) : "v"(t[2 * q + 1]), "v"(scale));
        asm("v_fma_mixlo_f16 %0, %1, %2, -%3 op_sel_hi:[0,0,1]" : "=v"(l) : "v"(t[2 * q]), "v"(scale), "v"(h));
        asm("v_fma_mixhi_f16 %0, %1, %2, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
            : "+v"(l) : "v"(t[2 * q + 1]), "v"(scale), "v"(h));
        hi[q] = h;
        lo[q] = l;
    }
    return X3Pair{__builtin_bit_cast(h8, hi), __builtin_bit_cast(h8, lo)};
}

}  // namespace
}  // namespace sgn
