// optim.hip -- the training step's streaming kernels outside the MLP: the Adam update of
// the neural-point parameters and the bias-gradient column sums.
//
// Adam: torch.optim.Adam (the reference's two groups, mvs_points_volumetric_model.py:100-108,
// betas (0.9, 0.999), eps 1e-8, no weight decay / amsgrad), the per-element math of torch's
// fused implementation:
//   m = b1 m + (1 - b1) g;  v = b2 v + (1 - b2) g^2
//   p -= (lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps)
// The point group is ~47 M fp32 elements per step (embedding 32 + colour 3 + dir 3 + conf 1
// per point): pure HBM streaming, 16 B read + 12 B written per element (+4 B for the elements
// whose gradient is non-zero when the kernel also clears the gradient for the next step, which
// replaces a separate fill pass).
// One thread per float4, every access a 16-B vector load/store.
//
// Column sums: db_l = sum over rows of the fp16 delta tile [rows][cols] (fp32 accumulate),
// in two deterministic passes (fixed row slabs per workgroup, then the slabs in order), all
// layers of the step in the same two launches.
//
// Segment kernels (one launch for up to 16 segments): the weight-gradient epilogue (split-K
// partials summed, unpermuted from the MFMA storage order, unscaled and added into the flat
// gradient -- the accumulation autograd does into nn.Linear's .grad), clearing padded tails and
// the index gathers that re-pack the MFMA weight blobs from the flat parameter.
#include <algorithm>
#include <cmath>
#include <hip/hip_fp16.h>

#include "sgn_common.h"

namespace sgn {
namespace {

constexpr int kMaxAdamTensors = 8;

struct AdamArgs {
    float *p[kMaxAdamTensors], *g[kMaxAdamTensors], *m[kMaxAdamTensors], *v[kMaxAdamTensors];
    int64_t n[kMaxAdamTensors];
    int64_t off4[kMaxAdamTensors + 1];   // prefix sums of the tensors' whole float4 counts
    int nt;
    float b1, b2, omb1, omb2, step_size, bc2_sqrt, eps;
    int zero_grad;
};

// one element's update; every Adam kernel here runs exactly this sequence of fp32 operations, so
// the row-sparse path below reproduces the dense one bit for bit
__device__ __forceinline__ void adam_el(float &p, float g, float &m, float &v, float b1, float b2, float omb1,
                                        float omb2, float step_size, float bc2_sqrt, float eps) {
    m = b1 * m + omb1 * g;
    v = b2 * v + omb2 * g * g;
    const float denom = sqrtf(v) / bc2_sqrt + eps;
    p -= step_size * m / denom;
}

__device__ __forceinline__ void adam1(float &p, float &g, float &m, float &v, const AdamArgs &a) {
    adam_el(p, g, m, v, a.b1, a.b2, a.omb1, a.omb2, a.step_size, a.bc2_sqrt, a.eps);
}

// float4 number i of the group's concatenated tensors -> (tensor, float4 index in it)
__device__ __forceinline__ int adam_tensor(const AdamArgs &a, int64_t i) {
    int t = 0;
#pragma unroll
    for (int k = 1; k < kMaxAdamTensors; ++k) t += (k < a.nt && i >= a.off4[k]);
    return t;
}

struct Adam4 {
    float4 p, g, m, v;
    int t;
    int64_t j;
};

__device__ __forceinline__ void adam_load(const AdamArgs &a, int64_t i, Adam4 &x) {
    x.t = adam_tensor(a, i);
    x.j = i - a.off4[x.t];
    x.p = reinterpret_cast<const float4 *>(a.p[x.t])[x.j];
    x.g = reinterpret_cast<const float4 *>(a.g[x.t])[x.j];
    x.m = reinterpret_cast<const float4 *>(a.m[x.t])[x.j];
    x.v = reinterpret_cast<const float4 *>(a.v[x.t])[x.j];
}

__device__ __forceinline__ void adam_store(const AdamArgs &a, Adam4 &x) {
    const bool gz = x.g.x != 0.f || x.g.y != 0.f || x.g.z != 0.f || x.g.w != 0.f;
    adam1(x.p.x, x.g.x, x.m.x, x.v.x, a);
    adam1(x.p.y, x.g.y, x.m.y, x.v.y, a);
    adam1(x.p.z, x.g.z, x.m.z, x.v.z, a);
    adam1(x.p.w, x.g.w, x.m.w, x.v.w, a);
    reinterpret_cast<float4 *>(a.p[x.t])[x.j] = x.p;
    reinterpret_cast<float4 *>(a.m[x.t])[x.j] = x.m;
    reinterpret_cast<float4 *>(a.v[x.t])[x.j] = x.v;
    // most rows' gradients are already zero (a step touches ~50 k of 1.2 M points): store only
    // the others, 4 of the 32 B per element skipped for the untouched rows
    if (a.zero_grad && gz) reinterpret_cast<float4 *>(a.g[x.t])[x.j] = make_float4(0.f, 0.f, 0.f, 0.f);
}

// one launch per parameter group: every tensor's float4s as one range, two per thread per trip
// (both loaded before either is computed: 128 B in flight per thread)
__global__ __launch_bounds__(256) void k_adam(AdamArgs a) {
    const int64_t n4 = a.off4[a.nt];
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    for (; i + stride < n4; i += 2 * stride) {
        Adam4 x, y;
        adam_load(a, i, x);
        adam_load(a, i + stride, y);
        adam_store(a, x);
        adam_store(a, y);
    }
    if (i < n4) {
        Adam4 x;
        adam_load(a, i, x);
        adam_store(a, x);
    }
    // ragged tails (n % 4 elements of each tensor), first workgroup only
    if (blockIdx.x == 0) {
        for (int t = 0; t < a.nt; ++t) {
            if (threadIdx.x >= (a.n[t] & 3)) continue;
            const int64_t j = ((a.n[t] >> 2) << 2) + threadIdx.x;
            float p = a.p[t][j], g = a.g[t][j], m = a.m[t][j], v = a.v[t][j];
            adam1(p, g, m, v, a);
            a.p[t][j] = p;
            a.m[t][j] = m;
            a.v[t][j] = v;
            if (a.zero_grad) a.g[t][j] = 0.f;
        }
    }
}

// ---- row-sparse exact Adam (the point group) -------------------------------------------------
// A step's gradient touches ~50 k of the 1.2 M points; the dense update of the other rows is the
// zero-gradient recurrence m = b1 m, v = b2 v, p -= step_size_k m / (sqrt(v) / bc2_sqrt_k + eps),
// deterministic per element.  Each row records the step it holds (last[r]); a listed row replays the
// steps it missed with adam_el at g = 0 and each step's constants (sched[k - 1] = (step_size_k,
// bc2_sqrt_k)), then (apply) takes step `target` with the gradient buffer's value (zero for a row the
// step did not touch, which is that step's zero-gradient update): the same operations in the same
// order as the dense kernel, so a row equals the dense update bit for bit once brought forward.
// Two launches: k_rows_claim takes each listed row once (a claim tag per launch; the lists may repeat
// rows and hold -1) into a compact (row, step held) list -- and, for list 1 and row 0, once more into
// the `pend` list of distinct rows (the rows whose gradient the coming step writes, also the f32
// step's projection subset); k_rows_update then runs one thread per (row, element) of the compact list.
constexpr int kMaxRowTensors = 4;
struct AdamRowsArgs {
    float *p[kMaxRowTensors], *g[kMaxRowTensors], *m[kMaxRowTensors], *v[kMaxRowTensors];
    int32_t w[kMaxRowTensors];     // elements per row
    int32_t ms[kMaxRowTensors];    // row stride of exp_avg / exp_avg_sq (>= w: narrow tensors' moments packed)
    int32_t nt, wsum;              // tensors, elements per row in all
    const int32_t *rows;           // list 1 (duplicates and -1 allowed), or null: rows 0 .. n_max - 1
    const void *d_count;           // device count of list 1 (int32 or int64, times count_mul; null: n_max)
    int32_t count_is64, count_mul, row0;   // row0: row 0 as one more list-1 entry
    int64_t n_max, n_rows;
    const int32_t *rows2;          // list 2 (a previous pend list), device int64 count at d_count2
    const int64_t *d_count2;
    int64_t n_max2;
    int32_t *last, *claim, *claim2;   // [n_rows]: step the row holds; this launch's claim tags
    int32_t tag;
    int32_t *ws;                   // [0] count, rows at ws + 4, steps held at ws + 4 + cap
    int64_t cap;
    int64_t *pend;                 // [0] count, [1] list-1 ids >= n_rows met; rows (int32) at pend + 2
    float2 *sched;                 // [k - 1] = (step_size_k, bc2_sqrt_k), k = 1 .. target
    int32_t target, apply;         // bring rows to step `target`; apply: that step with the gradient
    float b1, b2, omb1, omb2, eps, ss_t, bs_t;   // ss_t, bs_t: step `target`'s constants
    int32_t zero_grad;
};

// exclusive prefix over the workgroup (256 threads, 4 waves, lane-major) of two per-thread bit sets'
// popcounts, and their totals: ballots within a wave, one barrier across the four
__device__ __forceinline__ void wg_scan2(uint32_t wm, uint32_t pm, int *sc, int &ew, int &ep, int &tw, int &tp) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t lt = (1ull << lane) - 1;
    int xw = 0, xp = 0, sw = 0, sp = 0;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const uint64_t bw = __ballot(wm >> e & 1), bp = __ballot(pm >> e & 1);
        xw += __popcll(bw & lt), sw += __popcll(bw);
        xp += __popcll(bp & lt), sp += __popcll(bp);
    }
    if (lane == 0) sc[wv] = sw, sc[4 + wv] = sp;
    __syncthreads();
    int ow = 0, op = 0;
    tw = tp = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const int cw = sc[w], cp = sc[4 + w];
        ow += w < wv ? cw : 0, op += w < wv ? cp : 0;
        tw += cw, tp += cp;
    }
    ew = ow + xw, ep = op + xp;
}

// A workgroup takes CLAIM_PER entries (CLAIM_PER / 256 per thread): the row's first claimant records
// (row, last[row]) and sets last[row]; the winners are appended with one counter atomic per workgroup
// and list (one per wave serialised ~3.6 k atomics on each counter: 60 us)
constexpr int CLAIM_EPT = 2, CLAIM_PER = 256 * CLAIM_EPT;
__global__ __launch_bounds__(256) void k_rows_claim(AdamRowsArgs a) {
    __shared__ int sc[8];
    __shared__ int base_s[2];
    int64_t n1 = a.n_max;
    if (a.d_count) {
        const int64_t c = a.count_is64 ? *(const int64_t *)a.d_count : (int64_t)*(const int32_t *)a.d_count;
        n1 = min(n1, c * a.count_mul);
    }
    const int64_t n2 = a.rows2 ? min(a.n_max2, *a.d_count2) : 0;
    const int64_t n = n1 + n2 + a.row0;
    int32_t *prow = a.pend ? (int32_t *)(a.pend + 2) : nullptr;
    for (int64_t b0 = (int64_t)blockIdx.x * CLAIM_PER; b0 < n; b0 += (int64_t)gridDim.x * CLAIM_PER) {
        int rr[CLAIM_EPT], fr[CLAIM_EPT];
        uint32_t wm = 0, pm = 0;   // this thread's winners / pend entries (bit e)
        int oob = 0;
#pragma unroll
        for (int e = 0; e < CLAIM_EPT; ++e) {
            const int64_t i = b0 + e * 256 + threadIdx.x;
            int r = -1;
            bool l1 = false;
            if (i < n1) r = a.rows ? a.rows[i] : (int)i, l1 = true;
            else if (i < n1 + n2) r = a.rows2[i - n1];
            else if (i < n) r = 0, l1 = true;
            const bool valid = r >= 0 && r < a.n_rows;
            oob += l1 && r >= a.n_rows;
            rr[e] = r;
            fr[e] = 0;
            // test, then test-and-set (a point repeats across many samples' neighbour lists)
            if (valid && __builtin_nontemporal_load(a.claim + r) != a.tag && atomicExch(a.claim + r, a.tag) != a.tag) {
                fr[e] = a.last[r];
                a.last[r] = a.target;
                wm |= 1u << e;
            }
            if (a.pend && l1 && valid && __builtin_nontemporal_load(a.claim2 + r) != a.tag &&
                atomicExch(a.claim2 + r, a.tag) != a.tag)
                pm |= 1u << e;
        }
        if (a.pend && oob) atomicAdd((unsigned long long *)(a.pend + 1), (unsigned long long)oob);
        int tw, tp, ew, ep;
        wg_scan2(wm, pm, sc, ew, ep, tw, tp);
        if (threadIdx.x == 0) {
            base_s[0] = tw ? atomicAdd(a.ws, tw) : 0;
            base_s[1] = a.pend && tp ? (int)atomicAdd((unsigned long long *)a.pend, (unsigned long long)tp) : 0;
        }
        __syncthreads();
        int sw = base_s[0] + ew, sp = base_s[1] + ep;
        __syncthreads();
#pragma unroll
        for (int e = 0; e < CLAIM_EPT; ++e) {
            if (wm >> e & 1) {
                a.ws[4 + sw] = rr[e];
                a.ws[4 + a.cap + sw] = fr[e];
                ++sw;
            }
            if (pm >> e & 1) prow[sp++] = rr[e];
        }
    }
}

// one thread per (compact row, element): replay the missed steps, then (apply) step `target`.
// The constants of the last kSchedWin steps are staged in LDS (a row lags at most the flush
// interval); older steps are read from the table itself.
constexpr int kSchedWin = 1024;
__global__ __launch_bounds__(256) void k_rows_update(AdamRowsArgs a) {
    __shared__ float2 win[kSchedWin];
    const int upto = a.apply ? a.target - 1 : a.target;  // zero-gradient steps from + 1 .. upto
    const int lo = max(0, upto - kSchedWin);            // win[k - 1 - lo] = sched[k - 1], k > lo
    for (int i = threadIdx.x; i < upto - lo; i += blockDim.x) win[i] = a.sched[lo + i];
    __syncthreads();
    // the step's constants for later catch-ups (this launch's replays stop one step short of it)
    if (a.apply && blockIdx.x == 0 && threadIdx.x == 0) a.sched[a.target - 1] = make_float2(a.ss_t, a.bs_t);
    const int nw = a.ws[0] * a.wsum;
    const int stride = gridDim.x * blockDim.x;
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < nw; j += stride) {
        const int w = j / a.wsum;
        int c = j - w * a.wsum, t = 0;
        while (t + 1 < a.nt && c >= a.w[t]) c -= a.w[t++];
        const int r = a.ws[4 + w];
        const int from = a.ws[4 + a.cap + w];
        const int64_t e = (int64_t)r * a.w[t] + c, em = (int64_t)r * a.ms[t] + c;
        const bool app = a.apply && from < a.target;
        float p = a.p[t][e], m = a.m[t][em], v = a.v[t][em];
        const float g = app ? a.g[t][e] : 0.f;   // with p, m, v: one memory round trip, not two
        // two loops, so the common one reads LDS only (one loop selecting between LDS and the table
        // compiled to a flat load and a full wait per step)
        int k = from + 1;
        for (; k <= min(upto, lo); ++k) {
            const float2 sc = a.sched[k - 1];
            adam_el(p, 0.f, m, v, a.b1, a.b2, a.omb1, a.omb2, sc.x, sc.y, a.eps);
        }
        for (; k <= upto; ++k) {
            const float2 sc = win[k - 1 - lo];
            adam_el(p, 0.f, m, v, a.b1, a.b2, a.omb1, a.omb2, sc.x, sc.y, a.eps);
        }
        if (app) {
            adam_el(p, g, m, v, a.b1, a.b2, a.omb1, a.omb2, a.ss_t, a.bs_t, a.eps);
            if (a.zero_grad && g != 0.f) a.g[t][e] = 0.f;
        }
        a.p[t][e] = p;
        a.m[t][em] = m;
        a.v[t][em] = v;
    }
}

constexpr int kMaxColsumMats = 8;
constexpr int kColsumCols = 256;    // columns per tile (the MLP width)
constexpr int kColsumSlabs = SGN_COLSUM_SLABS;   // row slabs (workgroups) per matrix

struct ColsumArgs {
    const __half *x[kMaxColsumMats];
    const float *rw[kMaxColsumMats];   // per-row weights (null: 1)
    int64_t rows, slab;   // rows per slab
    int count;
    float *ws;            // [count][kColsumSlabs][256], then [count][kColsumSlabs] row-weight sums
    float *out;           // [count][256] (null: partials only)
};

template <bool W>
__device__ __forceinline__ void colsum_rows(const __half *x, const float *rw, int64_t r, int64_t r1, int c8,
                                            float (&acc)[8], float &wsum) {
#pragma unroll 2
    for (; r < r1; r += 8) {
        const uint4 w = *reinterpret_cast<const uint4 *>(x + r * kColsumCols + c8 * 8);
        const float s = W ? rw[r] : 1.f;
        if (W) wsum += s;
        const __half2 *h = reinterpret_cast<const __half2 *>(&w);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float2 f = __half22float2(h[j]);
            if (W) {
                acc[2 * j] += f.x * s;
                acc[2 * j + 1] += f.y * s;
            } else {
                acc[2 * j] += f.x;
                acc[2 * j + 1] += f.y;
            }
        }
    }
}

// grid (kColsumSlabs, count), 256 threads: 32 lanes x 8 columns cover a row, 8 rows at a time
__global__ __launch_bounds__(256) void k_colsum_part(ColsumArgs a) {
    const int mat = blockIdx.y;
    const int c8 = threadIdx.x & 31, r8 = threadIdx.x >> 5;
    const int64_t r0 = blockIdx.x * a.slab;
    const int64_t r1 = min(r0 + a.slab, a.rows);
    const __half *x = a.x[mat];
    const float *rw = a.rw[mat];
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float wsum = 0.f;   // this thread's rows' weights (every c8 lane of a row group holds the same)
    if (rw)   // workgroup-uniform: two loops, no branch inside
        colsum_rows<true>(x, rw, r0 + r8, r1, c8, acc, wsum);
    else
        colsum_rows<false>(x, rw, r0 + r8, r1, c8, acc, wsum);
    __shared__ float red[8][kColsumCols];
    __shared__ float wred[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) red[r8][c8 * 8 + j] = acc[j];
    if (c8 == 0) wred[r8] = wsum;
    __syncthreads();
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += red[k][threadIdx.x];
    a.ws[((int64_t)mat * kColsumSlabs + blockIdx.x) * kColsumCols + threadIdx.x] = s;
    if (rw && threadIdx.x == 0) {
        float t = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) t += wred[k];
        a.ws[(int64_t)a.count * kColsumSlabs * kColsumCols + (int64_t)mat * kColsumSlabs + blockIdx.x] = t;
    }
}

// grid (count), 256 threads: the slabs summed in slab order
__global__ __launch_bounds__(256) void k_colsum_final(ColsumArgs a) {
    const int mat = blockIdx.x;
    const float *w = a.ws + (int64_t)mat * kColsumSlabs * kColsumCols + threadIdx.x;
    float s = 0.f;
    for (int b = 0; b < kColsumSlabs; ++b) s += w[b * kColsumCols];
    a.out[mat * kColsumCols + threadIdx.x] = s;
}

// ---- segment kernels: the step's small gathers / clears / gradient epilogues, one launch each
// (grid.y = segment).  Replace ~40 per-tensor torch launches of the training step.
constexpr int kMaxSegs = 16;
constexpr int32_t kGradPer = 32;   // partials per group of k_grad_accumulate (its float atomics)

struct GradArgs {
    sgn_grad_segment s[kMaxSegs];
    const float *scale;   // device loss scale (power of two) or null
    float *grad;
    int32_t per;          // partials per group (at least kGradPer)
};

__device__ __forceinline__ bool grad_seg_vec4(const sgn_grad_segment &g) {
    return !((g.n | g.stride) & 3) && !(reinterpret_cast<uintptr_t>(g.src) & 15) &&
           !(reinterpret_cast<uintptr_t>(g.tail) & 15) && !(reinterpret_cast<uintptr_t>(g.dst) & 15);
}

__device__ __forceinline__ void grad_add(float *p, float v, bool atomic) {
    if (atomic)
        atomicAdd(p, v);
    else
        *p += v;
}

// grad[dst[j]] += (sum over b < nb of src[b * stride + j] (+ tail[j])) / scale; dst[j] < 0: skipped.
// grid (units, segments, partial groups): group z sums its share of the nb partials in order and
// adds it with a float atomic when there is more than one group (else a plain read-modify-write:
// the destinations are distinct across all segments -- each reference weight has one stored
// element).  Four consecutive elements per thread (16-B loads) when the segment allows it.
__global__ __launch_bounds__(256) void k_grad_accumulate(GradArgs a) {
    const sgn_grad_segment &g = a.s[blockIdx.y];
    const int32_t per = max(a.per, (g.nb + (int32_t)gridDim.z - 1) / (int32_t)gridDim.z);
    const int32_t b0 = (int32_t)blockIdx.z * per, b1 = min(g.nb, b0 + per);
    if (b0 >= b1) return;
    const bool atomic = gridDim.z > 1;
    const bool tail = g.tail && blockIdx.z == 0;
    const float inv = a.scale ? 1.f / a.scale[0] : 1.f;
    const int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (grad_seg_vec4(g)) {
        const int64_t j = u * 4;
        if (j >= g.n) return;
        const float4 *src = reinterpret_cast<const float4 *>(g.src + j);
        const int64_t st4 = g.stride / 4;
        float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 4
        for (int32_t b = b0; b < b1; ++b) {
            const float4 v = src[(int64_t)b * st4];
            s.x += v.x;
            s.y += v.y;
            s.z += v.z;
            s.w += v.w;
        }
        if (tail) {
            const float4 v = *reinterpret_cast<const float4 *>(g.tail + j);
            s.x += v.x;
            s.y += v.y;
            s.z += v.z;
            s.w += v.w;
        }
        const int4 d = *reinterpret_cast<const int4 *>(g.dst + j);
        if (d.x >= 0) grad_add(a.grad + d.x, s.x * inv, atomic);
        if (d.y >= 0) grad_add(a.grad + d.y, s.y * inv, atomic);
        if (d.z >= 0) grad_add(a.grad + d.z, s.z * inv, atomic);
        if (d.w >= 0) grad_add(a.grad + d.w, s.w * inv, atomic);
        return;
    }
    if (u >= g.n) return;
    const int32_t d = g.dst[u];
    if (d < 0) return;
    float s = 0.f;
    for (int32_t b = b0; b < b1; ++b) s += g.src[(int64_t)b * g.stride + u];
    if (tail) s += g.tail[u];
    grad_add(a.grad + d, s * inv, atomic);
}

struct ZeroArgs {
    uint4 *p[kMaxSegs];
    int64_t n16[kMaxSegs];
};

__global__ __launch_bounds__(256) void k_zero_segments(ZeroArgs a) {
    uint4 *p = a.p[blockIdx.y];
    const int64_t n = a.n16[blockIdx.y];
    const uint4 z = make_uint4(0u, 0u, 0u, 0u);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) p[i] = z;
}

struct CopyArgs {
    const char *src[kMaxSegs];   // null: clear
    char *dst[kMaxSegs];
    int64_t bytes[kMaxSegs];
};

// dst = src (or zeros) per segment, in 16-B, 4-B or single-byte units as the segment's alignment allows
__global__ __launch_bounds__(256) void k_copy_segments(CopyArgs a) {
    const int sg = blockIdx.y;
    const char *src = a.src[sg];
    char *dst = a.dst[sg];
    const int64_t n = a.bytes[sg];
    const int64_t t0 = (int64_t)blockIdx.x * 256 + threadIdx.x, st = (int64_t)gridDim.x * 256;
    const uintptr_t al = reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst) | (uintptr_t)n;
    if (!(al & 15)) {
        for (int64_t i = t0; i < n / 16; i += st)
            reinterpret_cast<uint4 *>(dst)[i] = src ? reinterpret_cast<const uint4 *>(src)[i] : make_uint4(0u, 0u, 0u, 0u);
    } else if (!(al & 3)) {
        for (int64_t i = t0; i < n / 4; i += st)
            reinterpret_cast<uint32_t *>(dst)[i] = src ? reinterpret_cast<const uint32_t *>(src)[i] : 0u;
    } else {
        for (int64_t i = t0; i < n; i += st) dst[i] = src ? src[i] : (char)0;
    }
}

struct GatherArgs {
    sgn_gather_segment s[kMaxSegs];
    const float *src;
    int64_t n_src;
};

// dst[j] = idx[j] in [0, n_src) ? src[idx[j]] : 0, stored as fp32 or fp16 (round to nearest even)
__global__ __launch_bounds__(256) void k_gather_segments(GatherArgs a) {
    const sgn_gather_segment &g = a.s[blockIdx.y];
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= g.n) return;
    const int32_t i = g.idx[j];
    const float v = (i >= 0 && i < a.n_src) ? a.src[i] : 0.f;
    if (g.fp16)
        static_cast<__half *>(g.dst)[j] = __float2half_rn(v);
    else
        static_cast<float *>(g.dst)[j] = v;
}

// ---- power-of-two loss scale: 2^-floor(log2(max(max|a|, max|b|, 1e-30))) -----------------
// max |x| as the max of the sign-cleared bit patterns (NaN > inf > every finite value, so a NaN
// propagates as torch.amax / torch.maximum would), per-workgroup partials then one workgroup.
constexpr int kScaleBlocks = 256;

__device__ __forceinline__ uint32_t block_max_u32(uint32_t v) {
    __shared__ uint32_t red[256];
    red[threadIdx.x] = v;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] = max(red[threadIdx.x], red[threadIdx.x + s]);
        __syncthreads();
    }
    return red[0];
}

__global__ __launch_bounds__(256) void k_absmax_part(const float *a, int64_t na, const float *b, int64_t nb,
                                                     uint32_t *ws) {
    uint32_t m = 0;
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < na; i += stride)
        m = max(m, __float_as_uint(a[i]) & 0x7fffffffu);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nb; i += stride)
        m = max(m, __float_as_uint(b[i]) & 0x7fffffffu);
    m = block_max_u32(m);
    if (threadIdx.x == 0) ws[blockIdx.x] = m;
}

__global__ __launch_bounds__(256) void k_pow2_scale(const uint32_t *ws, float *out) {
    const uint32_t m = block_max_u32(ws[threadIdx.x]);
    if (threadIdx.x == 0) {
        const float f = __uint_as_float(m);
        const float c = (f != f) ? f : fmaxf(f, 1e-30f);   // torch.clamp(min=1e-30) keeps a NaN
        out[0] = exp2f(-floorf(log2f(c)));
    }
}

// ---- fp32-faithful blob re-pack from the flat parameter (one shift launch + one pack launch) --
// per layer l: s_l = 14 - e with max |W_l| = f 2^e (frexp; 0 for an all-zero or non-finite max),
// then per fp16 fragment element v = W 2^s_l, hi = fp16(v), lo = fp16(v - hi), and the fp32
// section by kind (mlp_x3.hip Y32Kind: weight, bias, bias 2^s, 2^-s, 1, weight 2^-s_3).
constexpr int kMaxPackLayers = 16;

struct PackArgs {
    const float *flat;
    int64_t woff[kMaxPackLayers], wlen[kMaxPackLayers];
    const int32_t *code16, *code32;
    int64_t n16, n32;
    int32_t *shift;
    __half *out16;
    float *out32;
};

// one 1024-thread workgroup per layer; four independent max chains per thread keep several loads
// in flight (the largest layer, block1.2 / block3.0, is ~73k weights)
constexpr int SHIFT_TPB = 1024;
__global__ __launch_bounds__(SHIFT_TPB) void k_layer_shift(PackArgs a) {
    __shared__ uint32_t red[SHIFT_TPB / 64];
    const float *w = a.flat + a.woff[blockIdx.x];
    const int64_t n = a.wlen[blockIdx.x];
    uint32_t m[4] = {0u, 0u, 0u, 0u};
    int64_t i = threadIdx.x;
    for (; i + 3 * SHIFT_TPB < n; i += 4 * SHIFT_TPB) {
#pragma unroll
        for (int q = 0; q < 4; ++q) m[q] = max(m[q], __float_as_uint(w[i + q * SHIFT_TPB]) & 0x7fffffffu);
    }
    for (; i < n; i += SHIFT_TPB) m[0] = max(m[0], __float_as_uint(w[i]) & 0x7fffffffu);
    uint32_t v = max(max(m[0], m[1]), max(m[2], m[3]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t mm = 0;
        for (int q = 0; q < SHIFT_TPB / 64; ++q) mm = max(mm, red[q]);
        const float f = __uint_as_float(mm);
        int e = 0;
        if (f > 0.f && __builtin_isfinite(f)) frexpf(f, &e);
        a.shift[blockIdx.x] = (f > 0.f && __builtin_isfinite(f)) ? 14 - e : 0;
    }
}

// codes: fp16 element idx | layer << 22 | lo << 26 (-1: zero); fp32 element idx | layer << 22 | kind << 26
__global__ __launch_bounds__(256) void k_pack_scaled(PackArgs a) {
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (blockIdx.y == 0) {
        if (j >= a.n16) return;
        const int32_t c = a.code16[j];
        float v = 0.f;
        if (c >= 0) v = a.flat[c & 0x3fffff] * ldexpf(1.f, a.shift[(c >> 22) & 15]);
        const __half hi = __float2half_rn(v);
        a.out16[j] = (c >= 0 && ((c >> 26) & 1)) ? __float2half_rn(v - __half2float(hi)) : hi;
        return;
    }
    if (j >= a.n32) return;
    const int32_t c = a.code32[j];
    const int idx = c & 0x3fffff, l = (c >> 22) & 15, k = (c >> 26) & 7;
    float y = 0.f;
    switch (k) {
    case 1: y = a.flat[idx]; break;                                   // YK_W
    case 2: y = a.flat[idx]; break;                                   // YK_B
    case 3: y = a.flat[idx] * ldexpf(1.f, a.shift[l]); break;         // YK_BS
    case 4: y = ldexpf(1.f, -a.shift[l]); break;                      // YK_INV
    case 5: y = 1.f; break;                                           // YK_ONE
    case 6: y = a.flat[idx] * ldexpf(1.f, -a.shift[3]); break;        // YK_WINV
    default: break;                                                   // YK_ZERO
    }
    a.out32[j] = y;
}

// ---- the captured loss stage's inputs over the batch's item capacity: item i < counters[1] takes
// its blended features (fp16 -> fp32), its sample's alpha, its ray's direction and its sample id;
// padding items zeros, ray 0 and the sentinel sample s_cap.  32 threads per item (8 columns each).
struct ColourInArgs {
    const int32_t *counters, *work, *samp_ray;
    int64_t n_cap, s_cap;
    const __half *fs16;
    const float *feat, *raydir;
    float *fs32, *al32, *v;
    int32_t *samp;
    float *vpe;   // [n_cap][32] PE(viewdir) | 1 | 0 or null
};

__global__ __launch_bounds__(256) void k_colour_inputs(ColourInArgs a) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t i = t >> 5;
    const int c8 = (int)(t & 31);
    if (i >= a.n_cap) return;
    const bool ok = i < (int64_t)a.counters[1];
    float4 lo = make_float4(0.f, 0.f, 0.f, 0.f), hi = lo;
    if (ok) {
        const uint4 w = *reinterpret_cast<const uint4 *>(a.fs16 + i * 256 + c8 * 8);
        const __half2 *h = reinterpret_cast<const __half2 *>(&w);
        const float2 f0 = __half22float2(h[0]), f1 = __half22float2(h[1]), f2 = __half22float2(h[2]),
                     f3 = __half22float2(h[3]);
        lo = make_float4(f0.x, f0.y, f1.x, f1.y);
        hi = make_float4(f2.x, f2.y, f3.x, f3.y);
    }
    float4 *o = reinterpret_cast<float4 *>(a.fs32 + i * 256 + c8 * 8);
    o[0] = lo;
    o[1] = hi;
    if (c8 == 0) {
        const int32_t s = ok ? a.work[i] : 0;
        const int64_t r = ok ? (int64_t)a.samp_ray[s] : 0;
        a.al32[i] = ok ? a.feat[(int64_t)s * 4] : 0.f;
        a.v[i * 3 + 0] = a.raydir[r * 3 + 0];
        a.v[i * 3 + 1] = a.raydir[r * 3 + 1];
        a.v[i * 3 + 2] = a.raydir[r * 3 + 2];
        a.samp[i] = ok ? s : (int32_t)a.s_cap;
    }
    if (a.vpe) {   // PE(viewdir), ori=True without the raw v (point_aggregators.py:772-780): sin | cos of v 2^f
        float x = c8 == 24 ? 1.f : 0.f;
        if (c8 < 24) {
            const int jj = c8 < 12 ? c8 : c8 - 12, c = jj >> 2, f = jj & 3;
            const int32_t s = ok ? a.work[i] : 0;
            const int64_t r = ok ? (int64_t)a.samp_ray[s] : 0;
            float sn, cs;
            sincosf(a.raydir[r * 3 + c] * (float)(1 << f), &sn, &cs);
            x = c8 < 12 ? sn : cs;
        }
        a.vpe[i * 32 + c8] = x;
    }
}

// The distinct points a training step touches: point 0 (the conf read of empty neighbour slots),
// then every neighbour pidx[e] >= 0 of the first S = counters[0] samples.  stamp[p] == step marks
// a point already listed this step (the first lane to swap the stamp in owns it), so the table is
// never cleared; a wave appends its fresh points with one atomic on the count.  The list order
// follows the atomics (the consumers are order-free); its contents are deterministic.
__global__ void __launch_bounds__(256) k_touched_points(const int32_t *__restrict__ pidx,
                                                        const int32_t *__restrict__ counters, int64_t cap_slots,
                                                        int32_t K, int64_t n_points, int32_t step, int32_t *stamp,
                                                        int32_t *__restrict__ idx, unsigned long long *cnt,
                                                        unsigned long long *cnt_next, unsigned long long *n_bad) {
    int64_t n = (int64_t)counters[0] * K;
    n = (n < cap_slots ? n : cap_slots) + 1;   // virtual slot 0 is point 0
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    if (blockIdx.x == 0 && threadIdx.x == 0) *cnt_next = 0;   // the other step parity's count
    const int lane = threadIdx.x & 63;
    for (int64_t v0 = (int64_t)blockIdx.x * blockDim.x; v0 < n; v0 += stride) {
        const int64_t v = v0 + threadIdx.x;
        int32_t p = -1;
        bool fresh = false;
        if (v < n) {
            p = v == 0 ? 0 : pidx[v - 1];
            if (p >= n_points) atomicAdd(n_bad, 1ull);   // never expected: reported, not projected
            if (p >= 0 && p < n_points && stamp[p] != step)
                fresh = atomicExch(&stamp[p], step) != step;
        }
        const uint64_t m = __ballot(fresh);
        if (m == 0) continue;
        const int leader = __ffsll((unsigned long long)m) - 1;
        int base = 0;
        if (lane == leader) base = (int)atomicAdd(cnt, (unsigned long long)__popcll(m));
        base = __shfl(base, leader);
        if (fresh) {
            const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
            idx[base + below] = p;
        }
    }
}

// The distinct points a render frame's samples name (sgn_frame_points): a frame's ~28 M neighbour
// slots name ~0.2 M points ~100 times each, so they are byte marks by plain stores (idempotent, no
// atomics, no read before the store), then one thread per 4-byte word of marks compacts and clears them.
__device__ __forceinline__ void mark_point(int32_t p, int64_t n_points, uint8_t *mark, unsigned &bad) {
    if (p >= 0 && p < n_points) mark[p] = 1;
    else if (p >= n_points) ++bad;
}

__global__ void __launch_bounds__(256) k_mark_points(const int32_t *__restrict__ pidx,
                                                     const int32_t *__restrict__ counters, int64_t cap_slots,
                                                     int32_t K, int64_t n_points, uint8_t *mark,
                                                     unsigned long long *cnt) {
    int64_t n = (int64_t)counters[0] * K;
    n = n < cap_slots ? n : cap_slots;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        mark[0] = 1;   // point 0, as sgn_touched_points has it
        cnt[0] = 0;    // the compaction's counter (it runs after this kernel on the stream)
    }
    unsigned bad = 0;
    const int64_t n4 = n >> 2, stride = (int64_t)gridDim.x * blockDim.x;
    const int4 *p4 = reinterpret_cast<const int4 *>(pidx);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        const int4 v = p4[i];
        mark_point(v.x, n_points, mark, bad);
        mark_point(v.y, n_points, mark, bad);
        mark_point(v.z, n_points, mark, bad);
        mark_point(v.w, n_points, mark, bad);
    }
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) mark_point(pidx[4 * n4 + threadIdx.x], n_points, mark, bad);
    if (bad) atomicAdd(cnt + 1, (unsigned long long)bad);
}

// K = 8 (the configs' neighbour count): one thread per sample, whose slots are stored unless the
// previous sample (the thread before it) holds the same point -- consecutive samples along a ray share
// most of their neighbours, and a point that sample holds is marked by that thread.
__global__ void __launch_bounds__(256) k_mark_points8(const int32_t *__restrict__ pidx,
                                                      const int32_t *__restrict__ counters, int64_t cap_samples,
                                                      int64_t n_points, uint8_t *mark, unsigned long long *cnt) {
    int64_t S = counters[0];
    S = S < cap_samples ? S : cap_samples;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        mark[0] = 1;
        cnt[0] = 0;
    }
    unsigned bad = 0;
    const int4 *p4 = reinterpret_cast<const int4 *>(pidx);
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < S; s += (int64_t)gridDim.x * blockDim.x) {
        const int4 a = p4[2 * s], b = p4[2 * s + 1];
        int4 pa = make_int4(-1, -1, -1, -1), pb = pa;
        if (s > 0) pa = p4[2 * s - 2], pb = p4[2 * s - 1];
        const int cur[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        const int prv[8] = {pa.x, pa.y, pa.z, pa.w, pb.x, pb.y, pb.z, pb.w};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int p = cur[k];
            bool dup = false;
#pragma unroll
            for (int j = 0; j < 8; ++j) dup |= p == prv[j];
            if (p >= n_points) ++bad;
            else if (p >= 0 && !dup) mark[p] = 1;
        }
    }
    if (bad) atomicAdd(cnt + 1, (unsigned long long)bad);
}

__global__ void __launch_bounds__(256) k_compact_points(uint8_t *mark, int64_t n_points, int32_t *__restrict__ idx,
                                                        unsigned long long *cnt) {
    __shared__ int sc[4];
    __shared__ int base_s;
    const int64_t nw = (n_points + 3) >> 2;
    uint32_t *mw = reinterpret_cast<uint32_t *>(mark);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int64_t w0 = (int64_t)blockIdx.x * blockDim.x; w0 < nw; w0 += (int64_t)gridDim.x * blockDim.x) {
        const int64_t w = w0 + threadIdx.x;
        uint32_t m = w < nw ? mw[w] : 0u;
        if (m) mw[w] = 0u;
        const uint32_t bits = (uint32_t)((m & 0xffu) != 0) | (uint32_t)((m & 0xff00u) != 0) << 1 |
                              (uint32_t)((m & 0xff0000u) != 0) << 2 | (uint32_t)((m & 0xff000000u) != 0) << 3;
        const int c = __popc(bits);
        int x = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        if (lane == 63) sc[wv] = x;
        __syncthreads();
        int off = 0, tot = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            off += k < wv ? sc[k] : 0;
            tot += sc[k];
        }
        if (threadIdx.x == 0) base_s = tot ? (int)atomicAdd(cnt, (unsigned long long)tot) : 0;
        __syncthreads();
        int pos = base_s + off + x - c;
        __syncthreads();
        uint32_t b = bits;
        while (b) {
            idx[pos++] = (int32_t)(4 * w + __ffs(b) - 1);
            b &= b - 1;
        }
    }
}

}  // namespace
}  // namespace sgn

using namespace sgn;

extern "C" {

int sgn_adam_step_multi(int32_t n_t, float *const *d_param, float *const *d_grad, float *const *d_exp_avg,
                        float *const *d_exp_avg_sq, const int64_t *n, double lr, double beta1, double beta2, double eps,
                        int64_t step, int32_t zero_grad, sgn_stream_t stream) {
    SGN_REQUIRE(n_t >= 0 && n_t <= kMaxAdamTensors, "sgn_adam_step_multi: 0 <= n_t <= 8");
    SGN_REQUIRE(step >= 1, "sgn_adam_step: step >= 1 required");
    if (n_t == 0) return 0;
    SGN_REQUIRE(d_param && d_grad && d_exp_avg && d_exp_avg_sq && n, "sgn_adam_step_multi: null argument");
    AdamArgs a;
    a.nt = n_t;
    a.off4[0] = 0;
    for (int t = 0; t < n_t; ++t) {
        SGN_REQUIRE(n[t] >= 0, "sgn_adam_step: n >= 0 required");
        SGN_REQUIRE(n[t] == 0 || (d_param[t] && d_grad[t] && d_exp_avg[t] && d_exp_avg_sq[t]),
                    "sgn_adam_step: null buffer");
        for (const void *q : {(const void *)d_param[t], (const void *)d_grad[t], (const void *)d_exp_avg[t],
                              (const void *)d_exp_avg_sq[t]})
            SGN_REQUIRE(!(reinterpret_cast<uintptr_t>(q) & 15), "sgn_adam_step: buffers must be 16-B aligned");
        a.p[t] = d_param[t];
        a.g[t] = d_grad[t];
        a.m[t] = d_exp_avg[t];
        a.v[t] = d_exp_avg_sq[t];
        a.n[t] = n[t];
        a.off4[t + 1] = a.off4[t] + (n[t] >> 2);
    }
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
    const int64_t n4 = a.off4[n_t];
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((n4 + 511) / 512, 256 * 16));
    hipLaunchKernelGGL(k_adam, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), a);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

size_t sgn_adam_rows_workspace_bytes(int64_t n_entries) {
    return (size_t)(2 * std::max<int64_t>(n_entries, 0) + 4) * 4;
}
size_t sgn_adam_rows_pend_bytes(int64_t n_entries) { return (size_t)(std::max<int64_t>(n_entries, 0) + 4) * 4; }

int sgn_adam_rows(int32_t n_t, float *const *d_param, float *const *d_grad, float *const *d_exp_avg,
                  float *const *d_exp_avg_sq, const int32_t *row_width, const int32_t *mv_stride, int64_t n_rows,
                  const int32_t *d_rows,
                  const void *d_count, int32_t count_is64, int32_t count_mul, int64_t n_max, int32_t row0,
                  const int32_t *d_rows2, const int64_t *d_count2, int64_t n_max2, int32_t *d_last,
                  int32_t *d_claim, int32_t *d_claim2, int32_t tag, void *d_ws, size_t ws_bytes, void *d_pend,
                  size_t pend_bytes, float *d_sched, double lr, double beta1, double beta2, double eps, int64_t step,
                  int32_t apply, int32_t zero_grad, sgn_stream_t stream) {
    SGN_REQUIRE(n_t >= 1 && n_t <= kMaxRowTensors, "sgn_adam_rows: 1 <= n_t <= 4");
    SGN_REQUIRE(step >= (apply ? 1 : 0) && step < (1ll << 31), "sgn_adam_rows: 0 <= step < 2^31 (apply: >= 1)");
    SGN_REQUIRE(d_param && d_exp_avg && d_exp_avg_sq && row_width && d_last && d_claim && d_sched && d_ws,
                "sgn_adam_rows: null argument");
    SGN_REQUIRE(!apply || d_grad, "sgn_adam_rows: apply needs the gradients");
    SGN_REQUIRE(n_max >= 0 && n_max2 >= 0 && (d_rows || n_max <= n_rows), "sgn_adam_rows: n_max");
    SGN_REQUIRE(!d_rows2 || d_count2, "sgn_adam_rows: list 2 needs its device count");
    SGN_REQUIRE(!d_pend || d_claim2, "sgn_adam_rows: the pend list needs the second claim array");
    const int64_t entries = n_max + (d_rows2 ? n_max2 : 0) + (row0 ? 1 : 0);
    SGN_REQUIRE(ws_bytes >= sgn_adam_rows_workspace_bytes(std::min<int64_t>(entries, n_rows)),
                "sgn_adam_rows: workspace too small");
    SGN_REQUIRE(!d_pend || pend_bytes >= sgn_adam_rows_pend_bytes(std::min<int64_t>(n_max + 1, n_rows)),
                "sgn_adam_rows: pend list too small");
    SGN_REQUIRE(!d_count || count_mul >= 1, "sgn_adam_rows: count_mul >= 1");
    AdamRowsArgs a{};
    a.nt = n_t;
    a.wsum = 0;
    for (int t = 0; t < n_t; ++t) {
        SGN_REQUIRE(row_width[t] >= 1 && d_param[t] && d_exp_avg[t] && d_exp_avg_sq[t] && (!apply || d_grad[t]),
                    "sgn_adam_rows: empty tensor");
        a.p[t] = d_param[t];
        a.g[t] = apply ? d_grad[t] : nullptr;
        a.m[t] = d_exp_avg[t];
        a.v[t] = d_exp_avg_sq[t];
        SGN_REQUIRE(!mv_stride || mv_stride[t] >= row_width[t], "sgn_adam_rows: mv_stride[t] >= row_width[t]");
        a.w[t] = row_width[t];
        a.ms[t] = mv_stride ? mv_stride[t] : row_width[t];
        a.wsum += row_width[t];
    }
    a.rows = d_rows;
    a.d_count = d_count;
    a.count_is64 = count_is64 ? 1 : 0;
    a.count_mul = count_mul;
    a.row0 = row0 ? 1 : 0;
    a.n_max = n_max;
    a.n_rows = n_rows;
    a.rows2 = d_rows2;
    a.d_count2 = d_count2;
    a.n_max2 = n_max2;
    a.last = d_last;
    a.claim = d_claim;
    a.claim2 = d_claim2;
    a.tag = tag;
    a.ws = static_cast<int32_t *>(d_ws);
    a.cap = std::min<int64_t>(entries, n_rows);
    a.pend = static_cast<int64_t *>(d_pend);
    a.sched = reinterpret_cast<float2 *>(d_sched);
    a.target = (int32_t)step;
    a.apply = apply ? 1 : 0;
    // the scalars exactly as sgn_adam_step_multi forms them
    a.b1 = (float)beta1;
    a.b2 = (float)beta2;
    a.omb1 = (float)(1.0 - beta1);
    a.omb2 = (float)(1.0 - beta2);
    a.ss_t = apply ? (float)(lr / (1.0 - std::pow(beta1, (double)step))) : 0.f;
    a.bs_t = apply ? (float)std::sqrt(1.0 - std::pow(beta2, (double)step)) : 0.f;
    a.eps = (float)eps;
    a.zero_grad = zero_grad ? 1 : 0;
    SGN_REQUIRE(a.cap * a.wsum < (1ll << 31), "sgn_adam_rows: rows x elements < 2^31");
    hipStream_t st = as_stream(stream);
    SGN_CHECK_HIP(hipMemsetAsync(d_ws, 0, 4, st));
    if (d_pend) SGN_CHECK_HIP(hipMemsetAsync(d_pend, 0, 16, st));
    const int64_t cblocks = std::max<int64_t>(1, std::min<int64_t>((entries + CLAIM_PER - 1) / CLAIM_PER, 256 * 4));
    hipLaunchKernelGGL(k_rows_claim, dim3((unsigned)cblocks), dim3(256), 0, st, a);
    SGN_CHECK_HIP(hipGetLastError());
    const int64_t ublocks = std::max<int64_t>(1, std::min<int64_t>((a.cap * a.wsum + 255) / 256, 256 * 64));
    hipLaunchKernelGGL(k_rows_update, dim3((unsigned)ublocks), dim3(256), 0, st, a);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

int sgn_adam_step(float *d_param, float *d_grad, float *d_exp_avg, float *d_exp_avg_sq, int64_t n, double lr,
                  double beta1, double beta2, double eps, int64_t step, int32_t zero_grad, sgn_stream_t stream) {
    SGN_REQUIRE(n >= 0 && step >= 1, "sgn_adam_step: n >= 0 and step >= 1 required");
    if (n == 0) return 0;
    SGN_REQUIRE(d_param && d_grad && d_exp_avg && d_exp_avg_sq, "sgn_adam_step: null buffer");
    return sgn_adam_step_multi(1, &d_param, &d_grad, &d_exp_avg, &d_exp_avg_sq, &n, lr, beta1, beta2, eps, step,
                               zero_grad, stream);
}

size_t sgn_colsum_workspace_bytes(int32_t count) {
    return (size_t)std::max(count, 0) * kColsumSlabs * (kColsumCols + 1) * sizeof(float);
}

int sgn_colsum_f16(int32_t count, const void *const *d_x, int64_t rows, int32_t cols, float *d_ws, float *d_out,
                   sgn_stream_t stream) {
    return sgn_colsum_f16_weighted(count, d_x, nullptr, rows, cols, d_ws, d_out, stream);
}

namespace {
int colsum_launch(int32_t count, const void *const *d_x, const float *const *d_rw, int64_t rows, int32_t cols,
                  float *d_ws, float *d_out, sgn_stream_t stream) {
    SGN_REQUIRE(count >= 1 && count <= kMaxColsumMats, "sgn_colsum_f16: 1 <= count <= 8");
    SGN_REQUIRE(cols == kColsumCols, "sgn_colsum_f16: cols must be 256");
    SGN_REQUIRE(rows >= 0, "sgn_colsum_f16: rows < 0");
    SGN_REQUIRE(d_x && d_ws, "sgn_colsum_f16: null buffer");
    ColsumArgs a;
    for (int i = 0; i < count; ++i) {
        SGN_REQUIRE(d_x[i] != nullptr, "sgn_colsum_f16: null matrix");
        SGN_REQUIRE(!(reinterpret_cast<uintptr_t>(d_x[i]) & 15), "sgn_colsum_f16: matrices must be 16-B aligned");
        a.x[i] = static_cast<const __half *>(d_x[i]);
        a.rw[i] = d_rw ? d_rw[i] : nullptr;
    }
    a.rows = rows;
    a.slab = (rows + kColsumSlabs - 1) / kColsumSlabs;
    a.count = count;
    a.ws = d_ws;
    a.out = d_out;
    hipLaunchKernelGGL(k_colsum_part, dim3(kColsumSlabs, count), dim3(256), 0, as_stream(stream), a);
    SGN_CHECK_HIP(hipGetLastError());
    if (d_out) {
        hipLaunchKernelGGL(k_colsum_final, dim3(count), dim3(256), 0, as_stream(stream), a);
        SGN_CHECK_HIP(hipGetLastError());
    }
    return 0;
}
}  // namespace

int sgn_colsum_f16_weighted(int32_t count, const void *const *d_x, const float *const *d_rw, int64_t rows, int32_t cols,
                            float *d_ws, float *d_out, sgn_stream_t stream) {
    SGN_REQUIRE(d_out, "sgn_colsum_f16: null output");
    return colsum_launch(count, d_x, d_rw, rows, cols, d_ws, d_out, stream);
}

int sgn_colsum_f16_weighted_parts(int32_t count, const void *const *d_x, const float *const *d_rw, int64_t rows,
                                  int32_t cols, float *d_ws, sgn_stream_t stream) {
    return colsum_launch(count, d_x, d_rw, rows, cols, d_ws, nullptr, stream);
}

int sgn_grad_accumulate(int32_t n_seg, const sgn_grad_segment *segs, const float *d_scale, float *d_grad,
                        sgn_stream_t stream) {
    SGN_REQUIRE(n_seg >= 0 && n_seg <= kMaxSegs, "sgn_grad_accumulate: 0 <= n_seg <= 16");
    if (n_seg == 0) return 0;
    SGN_REQUIRE(segs && d_grad, "sgn_grad_accumulate: null argument");
    GradArgs a;
    int64_t umax = 0;
    int32_t nbmax = 1;
    for (int i = 0; i < n_seg; ++i) {
        const sgn_grad_segment &g = segs[i];
        SGN_REQUIRE(g.n >= 0 && g.nb >= 1 && g.stride >= g.n, "sgn_grad_accumulate: n >= 0, nb >= 1, stride >= n");
        SGN_REQUIRE(g.n == 0 || (g.src && g.dst), "sgn_grad_accumulate: null segment buffer");
        a.s[i] = g;
        // work units as the kernel counts them (grad_seg_vec4)
        const bool vec = !((g.n | g.stride) & 3) && !(reinterpret_cast<uintptr_t>(g.src) & 15) &&
                         !(reinterpret_cast<uintptr_t>(g.tail) & 15) && !(reinterpret_cast<uintptr_t>(g.dst) & 15);
        umax = std::max(umax, vec ? g.n / 4 : g.n);
        if (g.n > 0) nbmax = std::max(nbmax, g.nb);
    }
    if (umax == 0) return 0;
    SGN_REQUIRE(umax <= (int64_t)256 * 0x7fffffff, "sgn_grad_accumulate: segment too long");
    a.scale = d_scale;
    a.grad = d_grad;
    // partial groups of at least kGradPer partials each, at most 32 groups (one group: deterministic order);
    // a segment with fewer partials than the largest uses fewer groups (fewer atomics), the rest exit
    a.per = kGradPer;
    const int groups = std::min(32, std::max(1, (nbmax + kGradPer - 1) / kGradPer));
    hipLaunchKernelGGL(k_grad_accumulate, dim3((unsigned)((umax + 255) / 256), n_seg, groups), dim3(256), 0,
                       as_stream(stream), a);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

int sgn_zero_segments(int32_t n_seg, void *const *d_ptr, const int64_t *bytes, sgn_stream_t stream) {
    SGN_REQUIRE(n_seg >= 0 && n_seg <= kMaxSegs, "sgn_zero_segments: 0 <= n_seg <= 16");
    if (n_seg == 0) return 0;
    SGN_REQUIRE(d_ptr && bytes, "sgn_zero_segments: null argument");
    ZeroArgs a;
    int64_t nmax = 0;
    for (int i = 0; i < n_seg; ++i) {
        SGN_REQUIRE(bytes[i] >= 0 && bytes[i] % 16 == 0, "sgn_zero_segments: byte counts must be multiples of 16");
        SGN_REQUIRE(bytes[i] == 0 || (d_ptr[i] && !(reinterpret_cast<uintptr_t>(d_ptr[i]) & 15)),
                    "sgn_zero_segments: regions must be 16-B aligned");
        a.p[i] = static_cast<uint4 *>(d_ptr[i]);
        a.n16[i] = bytes[i] / 16;
        nmax = std::max(nmax, a.n16[i]);
    }
    if (nmax == 0) return 0;
    const int64_t blocks = std::min<int64_t>((nmax + 255) / 256, 1024);
    hipLaunchKernelGGL(k_zero_segments, dim3((unsigned)blocks, n_seg), dim3(256), 0, as_stream(stream), a);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

int sgn_copy_segments(int32_t n_seg, const void *const *d_src, void *const *d_dst, const int64_t *bytes,
                      sgn_stream_t stream) {
    SGN_REQUIRE(n_seg >= 0 && n_seg <= kMaxSegs, "sgn_copy_segments: 0 <= n_seg <= 16");
    if (n_seg == 0) return 0;
    SGN_REQUIRE(d_src && d_dst && bytes, "sgn_copy_segments: null argument");
    CopyArgs a;
    int64_t nmax = 0;
    for (int i = 0; i < n_seg; ++i) {
        SGN_REQUIRE(bytes[i] >= 0 && (bytes[i] == 0 || d_dst[i]), "sgn_copy_segments: bad segment");
        a.src[i] = static_cast<const char *>(d_src[i]);
        a.dst[i] = static_cast<char *>(d_dst[i]);
        a.bytes[i] = bytes[i];
        const uintptr_t al = reinterpret_cast<uintptr_t>(d_src[i]) | reinterpret_cast<uintptr_t>(d_dst[i]) | (uintptr_t)bytes[i];
        nmax = std::max(nmax, (al & 15) == 0 ? bytes[i] / 16 : (al & 3) == 0 ? bytes[i] / 4 : bytes[i]);
    }
    if (nmax == 0) return 0;
    const int64_t blocks = std::min<int64_t>((nmax + 255) / 256, 1024);
    hipLaunchKernelGGL(k_copy_segments, dim3((unsigned)blocks, n_seg), dim3(256), 0, as_stream(stream), a);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

int sgn_gather_segments(int32_t n_seg, const sgn_gather_segment *segs, const float *d_src, int64_t n_src,
                        sgn_stream_t stream) {
    SGN_REQUIRE(n_seg >= 0 && n_seg <= kMaxSegs, "sgn_gather_segments: 0 <= n_seg <= 16");
    if (n_seg == 0) return 0;
    SGN_REQUIRE(segs && n_src >= 0 && (d_src || n_src == 0), "sgn_gather_segments: null argument");
    GatherArgs a;
    int64_t nmax = 0;
    for (int i = 0; i < n_seg; ++i) {
        const sgn_gather_segment &g = segs[i];
        SGN_REQUIRE(g.n >= 0 && (g.n == 0 || (g.idx && g.dst)), "sgn_gather_segments: bad segment");
        a.s[i] = g;
        nmax = std::max(nmax, g.n);
    }
    if (nmax == 0) return 0;
    SGN_REQUIRE(nmax <= (int64_t)256 * 0x7fffffff, "sgn_gather_segments: segment too long");
    a.src = d_src;
    a.n_src = n_src;
    hipLaunchKernelGGL(k_gather_segments, dim3((unsigned)((nmax + 255) / 256), n_seg), dim3(256), 0,
                       as_stream(stream), a);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

int sgn_pack_scaled_f32(const float *d_flat, int64_t n_flat, int32_t n_layers, const int64_t *w_off,
                        const int64_t *w_len, const int32_t *d_code16, int64_t n16, const int32_t *d_code32, int64_t n32,
                        int32_t *d_shift, void *d_out16, float *d_out32, sgn_stream_t stream) {
    SGN_REQUIRE(n_layers >= 1 && n_layers <= kMaxPackLayers, "sgn_pack_scaled_f32: 1 <= n_layers <= 16");
    SGN_REQUIRE(d_flat && w_off && w_len && d_shift && n16 >= 0 && n32 >= 0, "sgn_pack_scaled_f32: null argument");
    SGN_REQUIRE(n_flat <= 0x3fffff, "sgn_pack_scaled_f32: flat parameter above 2^22 elements");
    SGN_REQUIRE((n16 == 0 || (d_code16 && d_out16)) && (n32 == 0 || (d_code32 && d_out32)),
                "sgn_pack_scaled_f32: null section buffer");
    PackArgs a;
    for (int l = 0; l < n_layers; ++l) {
        SGN_REQUIRE(w_off[l] >= 0 && w_len[l] >= 0 && w_off[l] + w_len[l] <= n_flat,
                    "sgn_pack_scaled_f32: layer span outside the flat parameter");
        a.woff[l] = w_off[l];
        a.wlen[l] = w_len[l];
    }
    a.flat = d_flat;
    a.code16 = d_code16;
    a.code32 = d_code32;
    a.n16 = n16;
    a.n32 = n32;
    a.shift = d_shift;
    a.out16 = static_cast<__half *>(d_out16);
    a.out32 = d_out32;
    hipLaunchKernelGGL(k_layer_shift, dim3(n_layers), dim3(SHIFT_TPB), 0, as_stream(stream), a);
    SGN_CHECK_HIP(hipGetLastError());
    const int64_t nmax = std::max<int64_t>(std::max(n16, n32), 1);
    hipLaunchKernelGGL(k_pack_scaled, dim3((unsigned)((nmax + 255) / 256), 2), dim3(256), 0, as_stream(stream), a);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

int sgn_colour_inputs(const int32_t *d_counters, const int32_t *d_work, const int32_t *d_samp_ray, int64_t n_cap,
                      int64_t s_cap, const void *d_fs16, const float *d_feat, const float *d_raydir, float *d_fs32,
                      float *d_al32, float *d_v, int32_t *d_samp, float *d_vpe, sgn_stream_t stream) {
    SGN_REQUIRE(n_cap >= 0 && s_cap >= 0 && s_cap < 0x7fffffff, "sgn_colour_inputs: bad capacity");
    if (n_cap == 0) return 0;
    SGN_REQUIRE(d_counters && d_work && d_samp_ray && d_fs16 && d_feat && d_raydir && d_fs32 && d_al32 && d_v && d_samp,
                "sgn_colour_inputs: null buffer");
    SGN_REQUIRE(!(reinterpret_cast<uintptr_t>(d_fs16) & 15) && !(reinterpret_cast<uintptr_t>(d_fs32) & 15),
                "sgn_colour_inputs: feature rows must be 16-B aligned");
    ColourInArgs a;
    a.counters = d_counters;
    a.work = d_work;
    a.samp_ray = d_samp_ray;
    a.n_cap = n_cap;
    a.s_cap = s_cap;
    a.fs16 = static_cast<const __half *>(d_fs16);
    a.feat = d_feat;
    a.raydir = d_raydir;
    a.fs32 = d_fs32;
    a.al32 = d_al32;
    a.v = d_v;
    a.samp = d_samp;
    a.vpe = d_vpe;
    hipLaunchKernelGGL(k_colour_inputs, dim3((unsigned)((n_cap * 32 + 255) / 256)), dim3(256), 0, as_stream(stream), a);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

int sgn_touched_points(const int32_t *d_pidx, const int32_t *d_counters, int64_t s_cap, int32_t K, int64_t n_points,
                       int32_t step, int32_t *d_stamp, int32_t *d_idx, int64_t *d_count2, sgn_stream_t stream) {
    SGN_REQUIRE(s_cap >= 0 && K >= 1 && n_points >= 1 && step >= 0, "sgn_touched_points: bad size");
    SGN_REQUIRE(d_pidx && d_counters && d_stamp && d_idx && d_count2, "sgn_touched_points: null buffer");
    const int64_t slots = s_cap * K + 1;
    int64_t blocks = (slots + 255) / 256;
    blocks = blocks < 2048 ? blocks : 2048;
    auto *c = reinterpret_cast<unsigned long long *>(d_count2);
    hipLaunchKernelGGL(k_touched_points, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), d_pidx, d_counters,
                       s_cap * K, K, n_points, step, d_stamp, d_idx, c + (step & 1), c + ((step + 1) & 1), c + 2);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

size_t sgn_frame_points_mark_bytes(int64_t n_points) {
    return (size_t)((std::max<int64_t>(n_points, 1) + 15) / 16 * 16);
}

int sgn_frame_points(const int32_t *d_pidx, const int32_t *d_counters, int64_t s_cap, int32_t K, int64_t n_points,
                     uint8_t *d_mark, int32_t *d_idx, int64_t *d_count, sgn_stream_t stream) {
    SGN_REQUIRE(s_cap >= 0 && K >= 1 && n_points >= 1 && n_points < (1ll << 31), "sgn_frame_points: bad size");
    SGN_REQUIRE(d_pidx && d_counters && d_mark && d_idx && d_count, "sgn_frame_points: null buffer");
    SGN_REQUIRE(!(reinterpret_cast<uintptr_t>(d_pidx) & 15) && !(reinterpret_cast<uintptr_t>(d_mark) & 3),
                "sgn_frame_points: d_pidx 16-B and d_mark 4-B aligned");
    const int64_t slots4 = (s_cap * K + 3) / 4;
    auto *c = reinterpret_cast<unsigned long long *>(d_count);
    if (K == 8) {
        const int64_t mblocks = std::max<int64_t>(1, std::min<int64_t>((s_cap + 255) / 256, 256 * 16));
        hipLaunchKernelGGL(k_mark_points8, dim3((unsigned)mblocks), dim3(256), 0, as_stream(stream), d_pidx, d_counters,
                           s_cap, n_points, d_mark, c);
    } else {
        const int64_t mblocks = std::max<int64_t>(1, std::min<int64_t>((slots4 + 255) / 256, 256 * 16));
        hipLaunchKernelGGL(k_mark_points, dim3((unsigned)mblocks), dim3(256), 0, as_stream(stream), d_pidx,
                           d_counters, s_cap * K, K, n_points, d_mark, c);
    }
    SGN_CHECK_HIP(hipGetLastError());
    const int64_t nw = (n_points + 3) / 4;
    const int64_t kblocks = std::max<int64_t>(1, std::min<int64_t>((nw + 255) / 256, 256 * 4));
    hipLaunchKernelGGL(k_compact_points, dim3((unsigned)kblocks), dim3(256), 0, as_stream(stream), d_mark, n_points,
                       d_idx, c);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

size_t sgn_pow2_scale_workspace_bytes(void) { return kScaleBlocks * sizeof(uint32_t); }

int sgn_pow2_scale(const float *d_a, int64_t na, const float *d_b, int64_t nb, void *d_ws, float *d_out,
                   sgn_stream_t stream) {
    SGN_REQUIRE(na >= 0 && nb >= 0 && na + nb >= 1, "sgn_pow2_scale: at least one element");
    SGN_REQUIRE((d_a || na == 0) && (d_b || nb == 0) && d_ws && d_out, "sgn_pow2_scale: null buffer");
    hipLaunchKernelGGL(k_absmax_part, dim3(kScaleBlocks), dim3(256), 0, as_stream(stream), d_a, na, d_b, nb,
                       static_cast<uint32_t *>(d_ws));
    SGN_CHECK_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_pow2_scale, dim3(1), dim3(256), 0, as_stream(stream), static_cast<const uint32_t *>(d_ws),
                       d_out);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

}  // extern "C"
