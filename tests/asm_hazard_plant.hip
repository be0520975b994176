// A deliberately planted inline-asm / MFMA hazard (TEST INPUT ONLY: compiled to assembly by
// tests/test_asm_hazards.py, never linked or run).  The asm VALU reads the MFMA's result right after
// the MFMA; the compiler's hazard recognizer does not look inside inline asm, which is the class of
// bug tools/asm_hazards.py guards against (63962d3).
#include <hip/hip_runtime.h>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void k_plant(const h8 *a, const h8 *b, f4 *out) {
    const int t = threadIdx.x;
    f4 c = out[t];
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[t], b[t], c, 0, 0, 0);
    float r;
    asm volatile("v_add_f32 %0, %1, %1" : "=v"(r) : "v"(c[0]));
    out[t] = f4{r, c[1], c[2], c[3]};
}
