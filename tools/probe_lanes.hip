// Probe of lane-exchange / MFMA operand semantics used by k_agg_rows (debug tool).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void k_swap(unsigned *o) {
    int l = threadIdx.x;
    unsigned a = 1000 + l, b = 2000 + l;
    auto r16 = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    auto r32 = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    o[l] = r16[0]; o[64 + l] = r16[1]; o[128 + l] = r32[0]; o[192 + l] = r32[1];
}

// D = mfma(A, B): A[m][k] = fa(m,k), B[k][n] = fb(k,n); write acc regs
__global__ void k_mfma(float *o, int trans) {
    int l = threadIdx.x;
    h8 a, b;
    for (int e = 0; e < 8; ++e) {
        int k = 8 * (l >> 5) + e, i = l & 31;
        a[e] = (_Float16)((i * 3 + k * 7) % 11 - 5);   // "weights": A[m=i][k]
        b[e] = (_Float16)((i * 5 + k * 3) % 13 - 6);   // "acts":    B[k][n=i]
    }
    f32x16 c = {};
    c = trans ? __builtin_amdgcn_mfma_f32_32x32x16_f16(b, a, c, 0, 0, 0)
              : __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
    for (int r = 0; r < 16; ++r) o[l * 16 + r] = c[r];
}

int main() {
    unsigned *d; hipMalloc(&d, 256 * 4);
    k_swap<<<1, 64>>>(d);
    std::vector<unsigned> h(256);
    hipMemcpy(h.data(), d, 256 * 4, hipMemcpyDeviceToHost);
    const char *nm[4] = {"p16[0]", "p16[1]", "p32[0]", "p32[1]"};
    for (int v = 0; v < 4; ++v) {
        printf("%s:", nm[v]);
        for (int l = 0; l < 64; l += 4) printf(" %u", h[v * 64 + l]);
        printf("\n");
    }
    float *df; hipMalloc(&df, 64 * 16 * 4);
    std::vector<float> o(64 * 16);
    for (int trans = 0; trans < 2; ++trans) {
        k_mfma<<<1, 64>>>(df, trans);
        hipMemcpy(o.data(), df, o.size() * 4, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int l = 0; l < 64; ++l)
            for (int r = 0; r < 16; ++r) {
                int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), col = l & 31;
                // non-trans: D[m=row][n=col] = sum_k A[row][k] B[k][col]
                // trans:     D[m=row][n=col] = sum_k B'[row][k] A'[k][col] with B' = acts as A
                double ref = 0;
                for (int k = 0; k < 16; ++k) {
                    double A = ((row * 3 + k * 7) % 11 - 5), B = ((col * 5 + k * 3) % 13 - 6);
                    double At = ((col * 3 + k * 7) % 11 - 5), Bt = ((row * 5 + k * 3) % 13 - 6);
                    ref += trans ? Bt * At : A * B;
                }
                if (std::fabs(ref - o[l * 16 + r]) > 1e-3) ++bad;
            }
        printf("mfma trans=%d: %d mismatches\n", trans, bad);
    }
    return 0;
}
