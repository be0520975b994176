// Probe (not product): what ds_read_b64_tr_b16 returns per lane for a [rows][64] fp16 LDS tile holding
// row*64 + col, when lane 4q+p (of each 16-lane group) supplies row q (+ 4 * group), cols 4p..4p+3.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short s4 __attribute__((ext_vector_type(4)));
__global__ void k(short *out) {
    __shared__ short sm[16 * 64];
    for (int i = threadIdx.x; i < 16 * 64; i += 64) sm[i] = (short)i;
    __syncthreads();
    const int l = threadIdx.x, g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
    const int row = 4 * g + q, col = 4 * p;
    s4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4 *)(sm + row * 64 + col));
    for (int e = 0; e < 4; ++e) out[l * 4 + e] = v[e];
}
int main() {
    short *d; hipMalloc(&d, 64 * 4 * 2);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    short h[256]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    for (int l = 0; l < 64; ++l) {
        printf("lane %2d:", l);
        for (int e = 0; e < 4; ++e) printf(" (r%d,c%d)", h[l * 4 + e] / 64, h[l * 4 + e] % 64);
        printf("\n");
    }
    return 0;
}
