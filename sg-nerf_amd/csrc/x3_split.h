// x3_split.h -- fp32 value -> (hi, lo) fp16 pair for the 3-product split MFMA (gfx950).
//
// x = hi + lo with hi = fp16(x), lo = fp16(x - hi); a product w x is then carried as
// w_hi x_hi + w_hi x_lo + w_lo x_hi in fp32 MFMA accumulators (22 significant bits per factor,
// the dropped w_lo x_lo term <= 2^-22 |w x|).  Also the accurate sin / cos of the positional
// encodings (networks.py:175-192 uses torch.sin / torch.cos in fp32).
#pragma once
#include "agg_device.h"

namespace sgn {
namespace {

struct X3Pair {
    h8 hi, lo;
};

// (t * scale) -> (hi, lo) for a power-of-two `scale` (so t * scale is exact): each fp16 half is one
// v_fma_mix{lo,hi}_f16 (an fp32 FMA rounded once to fp16), 4 instructions per 2 values.  Inline asm
// (the compiler turns the same fmas into multiply / move / convert chains), so its hazard wait states
// are not inserted: use it only where no MFMA accumulates in VGPRs the outputs could land on (the
// training GEMMs keep their accumulators in AGPRs; tools/asm_hazards.py checks the built code)
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
// x -> (hi, lo) without scaling: v_cvt_pk_f16_f32 for hi and lo, and the difference x - hi as one
// v_fma_mix_f32 per value reading hi's fp16 half in place (the compiler forms a convert and a
// subtract instead).  The asm writes only into x's own register ("+v", tied): that register's last
// writer is a compiler-visible instruction, which already waited out any MFMA still reading it, so
// the asm needs no hazard wait states of its own (an asm VALU writing a fresh register can land on
// a register an in-flight MFMA still reads as its accumulator input -- the hazard recognizer does not
// see inline asm).
__device__ __forceinline__ X3Pair split8_unit(const float (&v)[8]) {
    X3Pair r;
    r.hi = pack8(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]);
    const u32x4 hp = __builtin_bit_cast(u32x4, r.hi);
    float d[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        d[2 * q] = v[2 * q];
        d[2 * q + 1] = v[2 * q + 1];
        asm("v_fma_mix_f32 %0, %1, -1.0, %0 op_sel_hi:[1,0,0]" : "+v"(d[2 * q]) : "v"(hp[q]));
        asm("v_fma_mix_f32 %0, %1, -1.0, %0 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(d[2 * q + 1]) : "v"(hp[q]));
    }
    r.lo = pack8(d[0], d[1], d[2], d[3], d[4], d[5], d[6], d[7]);
    return r;
}

// sin and cos of x (fp32, within ~1 ulp): quadrant q = rint(x 2/pi), r = x - q pi/2 in double
// (exact to far below fp32 resolution for |x| < 2^20), cephes' minimax polynomials on
// [-pi/4, pi/4]; |x| >= 2^20 (never met by the encodings' arguments) takes the library sincosf.
__device__ __forceinline__ void sincos_acc_fast(float x, float &s, float &c) {  // |x| < 2^20
    const float qf = __builtin_rintf(x * 0.63661977236758134f);
    const float r = (float)__builtin_fma((double)qf, -1.5707963267948966, (double)x);
    const float z = r * r;
    const float sp = __builtin_fmaf(__builtin_fmaf(__builtin_fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z,
                                                   -1.6666654611e-1f), z * r, r);
    const float cp = __builtin_fmaf(__builtin_fmaf(__builtin_fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z,
                                                   4.166664568298827e-2f), z * z, __builtin_fmaf(-0.5f, z, 1.f));
    const int q = (int)qf;
    const float s0 = (q & 1) ? cp : sp, c0 = (q & 1) ? sp : cp;
    s = (q & 2) ? -s0 : s0;
    c = ((q + 1) & 2) ? -c0 : c0;
}
__device__ __forceinline__ void sincos_acc(float x, float &s, float &c) {
    if (__builtin_expect(__builtin_fabsf(x) >= 1048576.f, 0)) {
        sincosf(x, &s, &c);
        return;
    }
    sincos_acc_fast(x, s, c);
}

}  // namespace
}  // namespace sgn
