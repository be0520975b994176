// Probe (not product): v_mfma_f32_32x32x16_f16 fed by ds_read_b64_tr_b16 vs by plain 16-B reads of the
// same k-contiguous fragments: D = A B with A[i][k] = i + 100 k, B = ones (D[i][j] = 16 i + 100 * 120).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short s4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16x __attribute__((ext_vector_type(16)));
__global__ void k(float *out) {
    __shared__ _Float16 sm[16 * 32];   // [k][i] row-major: 16 k rows of 32 columns (64 B rows)
    __shared__ _Float16 st[32 * 16];   // [i][k]: k-contiguous
    for (int t = threadIdx.x; t < 512; t += 64) {
        const int kk = t / 32, i = t % 32;
        sm[t] = (_Float16)(i + 100 * kk);
        st[i * 16 + kk] = (_Float16)(i + 100 * kk);
    }
    __syncthreads();
    const int l = threadIdx.x, g = l >> 4, i16 = l & 15, q = i16 >> 2, p = i16 & 3;
    const int row = 8 * (g >> 1) + q, col = 16 * (g & 1) + 4 * p;
    s4 a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4 *)(sm + row * 32 + col));
    s4 a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4 *)(sm + (row + 4) * 32 + col));
    h8 at = __builtin_bit_cast(h8, __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7));
    h8 an = *(h8 *)(st + (l & 31) * 16 + 8 * (l >> 5));
    h8 ones;
    for (int e = 0; e < 8; ++e) ones[e] = (_Float16)1.f;
    f16x z = {};
    f16x dt = __builtin_amdgcn_mfma_f32_32x32x16_f16(at, ones, z, 0, 0, 0);
    f16x dn = __builtin_amdgcn_mfma_f32_32x32x16_f16(an, ones, z, 0, 0, 0);
    for (int r = 0; r < 16; ++r) {
        out[l * 16 + r] = dt[r];
        out[1024 + l * 16 + r] = dn[r];
    }
    for (int e = 0; e < 8; ++e) {
        out[2048 + l * 8 + e] = (float)at[e];
        out[2560 + l * 8 + e] = (float)an[e];
    }
}
int main() {
    float *d;
    (void)hipMalloc(&d, 4096 * 4);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    float h[4096];
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l)
        for (int e = 0; e < 8; ++e) bad += h[2048 + l * 8 + e] != h[2560 + l * 8 + e];
    printf("fragments differ at %d of 512 values\n", bad);
    for (int l : {0, 1, 2, 3, 4, 33})
        printf("lane %d: tr D r0..3 %g %g %g %g | plain D r0..3 %g %g %g %g\n", l, h[l * 16], h[l * 16 + 1], h[l * 16 + 2],
               h[l * 16 + 3], h[1024 + l * 16], h[1024 + l * 16 + 1], h[1024 + l * 16 + 2], h[1024 + l * 16 + 3]);
    return 0;
}
