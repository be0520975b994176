// optim.hip -- the training step's streaming kernels outside the MLP: the Adam update of
// the neural-point parameters and the bias-gradient column sums.
//
// Adam: torch.optim.Adam (the reference's two groups, mvs_points_volumetric_model.py:100-108,
// betas (0.9, 0.999), eps 1e-8, no weight decay / amsgrad), the per-element math of torch's
// fused implementation:
//   m = b1 m + (1 - b1) g;  v = b2 v + (1 - b2) g^2
//   p -= (lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps)
// The point group is ~47 M fp32 elements per step (embedding 32 + colour 3 + dir 3 + conf 1
// per point): pure HBM streaming, 16 B read + 12 B written per element (+4 B when the kernel
// also clears the gradient for the next step, which replaces a separate fill pass).
// One thread per float4, every access a 16-B vector load/store.
//
// Column sums: db_l = sum over rows of the fp16 delta tile [rows][cols] (fp32 accumulate),
// in two deterministic passes (fixed row slabs per workgroup, then the slabs in order), all
// layers of the step in the same two launches.
#include <algorithm>
#include <cmath>
#include <hip/hip_fp16.h>

#include "sgn_common.h"

namespace sgn {
namespace {

struct AdamArgs {
    float *p, *g, *m, *v;
    int64_t n;
    float b1, b2, omb1, omb2, step_size, bc2_sqrt, eps;
    int zero_grad;
};

__device__ __forceinline__ void adam1(float &p, float &g, float &m, float &v, const AdamArgs &a) {
    m = a.b1 * m + a.omb1 * g;
    v = a.b2 * v + a.omb2 * g * g;
    const float denom = sqrtf(v) / a.bc2_sqrt + a.eps;
    p -= a.step_size * m / denom;
}

__global__ __launch_bounds__(256) void k_adam(AdamArgs a) {
    const int64_t n4 = a.n >> 2;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += stride) {
        float4 p = reinterpret_cast<const float4 *>(a.p)[i];
        float4 g = reinterpret_cast<const float4 *>(a.g)[i];
        float4 m = reinterpret_cast<const float4 *>(a.m)[i];
        float4 v = reinterpret_cast<const float4 *>(a.v)[i];
        adam1(p.x, g.x, m.x, v.x, a);
        adam1(p.y, g.y, m.y, v.y, a);
        adam1(p.z, g.z, m.z, v.z, a);
        adam1(p.w, g.w, m.w, v.w, a);
        reinterpret_cast<float4 *>(a.p)[i] = p;
        reinterpret_cast<float4 *>(a.m)[i] = m;
        reinterpret_cast<float4 *>(a.v)[i] = v;
        if (a.zero_grad) reinterpret_cast<float4 *>(a.g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    // ragged tail (n % 4 elements), first workgroup only
    if (blockIdx.x == 0 && threadIdx.x < (a.n & 3)) {
        const int64_t j = (n4 << 2) + threadIdx.x;
        float p = a.p[j], g = a.g[j], m = a.m[j], v = a.v[j];
        adam1(p, g, m, v, a);
        a.p[j] = p;
        a.m[j] = m;
        a.v[j] = v;
        if (a.zero_grad) a.g[j] = 0.f;
    }
}

constexpr int kMaxColsumMats = 8;
constexpr int kColsumCols = 256;    // columns per tile (the MLP width)
constexpr int kColsumSlabs = 512;   // row slabs (workgroups) per matrix

struct ColsumArgs {
    const __half *x[kMaxColsumMats];
    int64_t rows, slab;   // rows per slab
    float *ws;            // [count][kColsumSlabs][256]
    float *out;           // [count][256]
};

// grid (kColsumSlabs, count), 256 threads: 32 lanes x 8 columns cover a row, 8 rows at a time
__global__ __launch_bounds__(256) void k_colsum_part(ColsumArgs a) {
    const int mat = blockIdx.y;
    const int c8 = threadIdx.x & 31, r8 = threadIdx.x >> 5;
    const int64_t r0 = blockIdx.x * a.slab;
    const int64_t r1 = min(r0 + a.slab, a.rows);
    const __half *x = a.x[mat];
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int64_t r = r0 + r8; r < r1; r += 8) {
        const uint4 w = *reinterpret_cast<const uint4 *>(x + r * kColsumCols + c8 * 8);
        const __half2 *h = reinterpret_cast<const __half2 *>(&w);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float2 f = __half22float2(h[j]);
            acc[2 * j] += f.x;
            acc[2 * j + 1] += f.y;
        }
    }
    __shared__ float red[8][kColsumCols];
#pragma unroll
    for (int j = 0; j < 8; ++j) red[r8][c8 * 8 + j] = acc[j];
    __syncthreads();
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += red[k][threadIdx.x];
    a.ws[((int64_t)mat * kColsumSlabs + blockIdx.x) * kColsumCols + threadIdx.x] = s;
}

// grid (count), 256 threads: the slabs summed in slab order
__global__ __launch_bounds__(256) void k_colsum_final(ColsumArgs a) {
    const int mat = blockIdx.x;
    const float *w = a.ws + (int64_t)mat * kColsumSlabs * kColsumCols + threadIdx.x;
    float s = 0.f;
    for (int b = 0; b < kColsumSlabs; ++b) s += w[b * kColsumCols];
    a.out[mat * kColsumCols + threadIdx.x] = s;
}

}  // namespace
}  // namespace sgn

using namespace sgn;

extern "C" {

int sgn_adam_step(float *d_param, float *d_grad, float *d_exp_avg, float *d_exp_avg_sq, int64_t n, double lr,
                  double beta1, double beta2, double eps, int64_t step, int32_t zero_grad, sgn_stream_t stream) {
    SGN_REQUIRE(n >= 0 && step >= 1, "sgn_adam_step: n >= 0 and step >= 1 required");
    if (n == 0) return 0;
    SGN_REQUIRE(d_param && d_grad && d_exp_avg && d_exp_avg_sq, "sgn_adam_step: null buffer");
    for (const void *q : {(const void *)d_param, (const void *)d_grad, (const void *)d_exp_avg,
                          (const void *)d_exp_avg_sq})
        SGN_REQUIRE(!(reinterpret_cast<uintptr_t>(q) & 15), "sgn_adam_step: buffers must be 16-B aligned");
    AdamArgs a;
    a.p = d_param;
    a.g = d_grad;
    a.m = d_exp_avg;
    a.v = d_exp_avg_sq;
    a.n = n;
    // host-side scalars in double and rounded once to fp32, as torch does with its Python
    // float hyper-parameters (1 - beta2 = 0.001, not 1 - 0.999f)
    a.b1 = (float)beta1;
    a.b2 = (float)beta2;
    a.omb1 = (float)(1.0 - beta1);
    a.omb2 = (float)(1.0 - beta2);
    const double bc1 = 1.0 - std::pow(beta1, (double)step);
    const double bc2 = 1.0 - std::pow(beta2, (double)step);
    a.step_size = (float)(lr / bc1);
    a.bc2_sqrt = (float)std::sqrt(bc2);
    a.eps = (float)eps;
    a.zero_grad = zero_grad ? 1 : 0;
    const int64_t n4 = n >> 2;
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((n4 + 255) / 256, 256 * 32));
    hipLaunchKernelGGL(k_adam, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), a);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

size_t sgn_colsum_workspace_bytes(int32_t count) {
    return (size_t)std::max(count, 0) * kColsumSlabs * kColsumCols * sizeof(float);
}

int sgn_colsum_f16(int32_t count, const void *const *d_x, int64_t rows, int32_t cols, float *d_ws, float *d_out,
                   sgn_stream_t stream) {
    SGN_REQUIRE(count >= 1 && count <= kMaxColsumMats, "sgn_colsum_f16: 1 <= count <= 8");
    SGN_REQUIRE(cols == kColsumCols, "sgn_colsum_f16: cols must be 256");
    SGN_REQUIRE(rows >= 0, "sgn_colsum_f16: rows < 0");
    SGN_REQUIRE(d_x && d_ws && d_out, "sgn_colsum_f16: null buffer");
    ColsumArgs a;
    for (int i = 0; i < count; ++i) {
        SGN_REQUIRE(d_x[i] != nullptr, "sgn_colsum_f16: null matrix");
        SGN_REQUIRE(!(reinterpret_cast<uintptr_t>(d_x[i]) & 15), "sgn_colsum_f16: matrices must be 16-B aligned");
        a.x[i] = static_cast<const __half *>(d_x[i]);
    }
    a.rows = rows;
    a.slab = (rows + kColsumSlabs - 1) / kColsumSlabs;
    a.ws = d_ws;
    a.out = d_out;
    hipLaunchKernelGGL(k_colsum_part, dim3(kColsumSlabs, count), dim3(256), 0, as_stream(stream), a);
    SGN_CHECK_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_colsum_final, dim3(count), dim3(256), 0, as_stream(stream), a);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

}  // extern "C"
