// train_x3.hip -- the fp32 training step's backward (and the colour MLP's training forward) on
// hand-written gfx950 kernels, at the reference's fp32 arithmetic.
//
// The reference differentiates PointAggregator.forward / viewmlp (models/aggregators/
// point_aggregators.py:868-959, :561-786) and the NeuralPoints gather (models/neural_points/
// neural_points.py:942-988) with torch autograd in fp32 (optimize_parameters,
// models/base_rendering_model.py:534-664; models/mvs_points_volumetric_model.py:116-141).  Here the
// step is a fixed sequence of launches over compact rows (one per valid (sample, neighbour) pair,
// sample-major) and work items (one per sample with a neighbour, sample order):
//
//   k_lists_count / k_lists_write  deterministic work list (samples with a neighbour, ascending) and
//                                  the compact row offset of every sample (prefix sum of samp_nnb)
//   k_rows16 (mlp_x3.hip, save)    the forward; z1 / z2 / z3 (SG: + zb) pre-activations at the rows
//   k_row_inputs                   per row: block1.0's input x0 = [emb | PE(emb) | PE(dists) | 1],
//                                  block3.0's extra channels [colour | dir - v | <dir, v> | 1], the
//                                  blend weights (w conf, w); per item PE(viewdir) | 1 (the colour
//                                  MLP's 24 extra inputs)
//   k_row_gather                   SG: the rows' BPNet embedding (block2_bpnet.0's second input)
//   k_x3rows / k_x3tn              every nn.Linear product: rows mode = forward (x W^T) and backward
//                                  data (dy W, masked by LeakyReLU' of the saved activation), the
//                                  weight block resident in LDS; split-K mode = weight gradients
//                                  (dy^T x as fixed-order partials, bias through a ones column)
//   k_colour_head / _bwd           color_branch.6 + sigmoid (fp32 FMA), and its backward
//   k_row_head                     block3.2's LeakyReLU, the alpha branch, the K-blend backward:
//                                  delta4, d conf through the straight-through clamp, dWa partials
//   k_row_tail                     d points_embeding through PE(emb), d colour / dir
//   k_reduce_partials              partials summed in a fixed order into the flat gradient
//
// Every GEMM is the 3-product split: x = hi + lo (fp16), w = hi + lo, w x ~ w_hi x_hi + w_hi x_lo +
// w_lo x_hi on v_mfma_f32_32x32x16_f16 with fp32 accumulation.  Operands are scaled by powers of two
// before the split so hi stays below 2^14 and lo stays a normal fp16 number: weights by the packer's
// per-layer shift, deltas by the amax word their producer wrote (max |x| via atomicMax), forward
// activations not at all (they are inside fp16 range, as the forward kernel requires).  Results are
// deterministic: no float atomics except the per-point gradients (the reference's index_add).
#include <cmath>
#include <type_traits>
#include <vector>

#include "agg_device.h"
#include "x3_split.h"

namespace sgn {
namespace {
namespace tx {

constexpr int TPB = 256;
constexpr int FRAG = 1024;  // one fragment: 64 lanes x 16 B

// ---- the split-K / rows GEMM ------------------------------------------------------------

struct Opnd {
    const float *p, *p2;
    int64_t ld, ld2;
    int32_t csplit, ncols, ones_col, act, kmajor, nrows, dyn, vec;
    const uint32_t *amax;
    const int32_t *shift;
};

struct GemmK {
    Opnd A, B;
    int32_t M, N, K;
    const int32_t *d_rows;
    const float *bias;
    int32_t act;
    const float *mask;
    int64_t ldm;
    float *out;
    int64_t ldo;
    int32_t out_cols;
    float *out2;
    int64_t ldo2;
    uint32_t *amax_out, *amax_out2;
    float *part;
    int32_t splits;   // split-K mode: row runs; rows mode: row-tile strides (the grid is splits x blocks, 1-D)
    char *bpack;      // rows mode: the weight blocks pre-converted by k_x3bpack (or null: each workgroup converts)
};

// 1-D block id -> (output column block, split / row-tile start).  Blocks b and b + 8 run on one XCD
// (its own L2), so the column blocks of a split go to the same XCD: they read the same rows of the
// shared operand at about the same time, and the second and third reads hit that L2, not HBM.
// Splits past the last multiple of 8 keep the plain order (correct, no sharing).
__device__ __forceinline__ void tn_block(int nblk, int splits, int &blk, int &split) {
    const int b = blockIdx.x;
    const int q = splits / 8, base = 8 * nblk * q;
    if (b < base) {
        const int xcd = b & 7, k = b >> 3;
        blk = k % nblk;
        split = (k / nblk) * 8 + xcd;
    } else {
        const int t = b - base;
        blk = t % nblk;
        split = 8 * q + t / nblk;
    }
}

__device__ __forceinline__ int op_shift(const Opnd &o) {
    if (o.shift) return o.shift[0];
    if (o.amax) {
        const float m = __builtin_bit_cast(float, o.amax[0]);
        if (!(m > 0.f) || !(m < 3.0e38f)) return 0;
        int e;
        frexpf(m, &e);  // m < 2^e
        return 14 - e;
    }
    return 0;
}

__device__ __forceinline__ float lrelu_ref(float x) { return x > 0.f ? x : x * 0.01f; }
// the same value as max(x, 0.01 x) in two instructions (one v_max: no canonicalising max of a loaded value)
__device__ __forceinline__ float lrelu_max(float x) {
    float t = x * 0.01f;
    asm("v_max_f32 %0, %1, %0" : "+v"(t) : "v"(x));
    return t;
}

// ---- split-K mode: C[m][n] = sum over rows r of A(m, r) B(n, r) ---------------------------------
// Both operands are row-major [rows][cols] (kmajor).  A stage is 32 rows; thread t of an operand loads
// 4 consecutive columns (a quad) of 8 consecutive rows (an octet) as 8 float4, which transpose in
// registers into the lane fragments of those 4 columns (8 k values each).  Stages are loaded two ahead
// into registers, converted into LDS (two buffers), then 2 k-steps of MFMAs: 4 waves split M, each
// wave WM x WN 32x32 tiles.
// Buffer view of an operand's rows [0, rows): loads past them return 0 (the hardware range check),
// stores past them are dropped -- no per-row branches in the loops.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc(const void *p, int64_t ld, int64_t rows) {
    int64_t bytes = rows * ld * 4;
    bytes = bytes < 0 ? 0 : bytes > 0x7fffffff ? 0x7fffffff : bytes;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
}
constexpr uint32_t OOB = 0x80000000u;  // a byte offset past every operand buffer: loads 0, stores dropped

__device__ __forceinline__ float4 ld4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

// A split-K operand's two sources as buffers over the split's rows [0, r1) (p2: the columns >= csplit)
struct OpRs {
    __amdgpu_buffer_rsrc_t r1, r2;
};
__device__ __forceinline__ OpRs op_rsrc(const Opnd &o, int r1) {
    return OpRs{rows_rsrc(o.p, o.ld, r1), rows_rsrc(o.p2 ? o.p2 : o.p, o.p2 ? o.ld2 : o.ld, r1)};
}

// element (i, k .. k + 7) of an operand (i: the M / N index, k: the reduction index, a multiple of 8)
// through its buffers over the matrix rows [0, lim) (rows past them read 0): kmajor 0: matrix row i,
// columns k..k+7; kmajor 1: rows k..k+7, column i.  Both sources are read and one selected per lane (the
// weight staging of the rows mode, once per workgroup), no branches.
__device__ __forceinline__ void load8(const Opnd &o, const OpRs &rs, int i, int k, int lim, float (&v)[8]) {
    if (!o.kmajor) {
        const bool s1 = k < o.csplit;  // csplit % 8 == 0: the octet has one source
        const int64_t rb1 = (int64_t)i * o.ld, rb2 = (int64_t)i * (o.p2 ? o.ld2 : o.ld);
        const uint32_t a1 = s1 ? (uint32_t)((rb1 + k) * 4) : OOB, a2 = s1 ? OOB : (uint32_t)((rb2 + k - o.csplit) * 4);
        const float4 x1 = ld4(rs.r1, a1), y1 = ld4(rs.r1, a1 + 16), x2 = ld4(rs.r2, a2), y2 = ld4(rs.r2, a2 + 16);
        const float4 x = s1 ? x1 : x2, y = s1 ? y1 : y2;
        v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
        v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
        const bool rok = i < lim;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int c = k + e;
            float u = c == o.ones_col ? (rok ? 1.f : 0.f) : c < o.ncols ? v[e] : 0.f;
            if (o.act && s1 && c != o.ones_col) u = lrelu_ref(u);
            v[e] = u;
        }
    } else {
        const bool s1 = i < o.csplit;
        const int c2 = s1 ? 0 : i - o.csplit;
        const bool cok = i < o.ncols && i != o.ones_col;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int r = k + e;
            const uint32_t a1 = s1 ? (uint32_t)(((int64_t)r * o.ld + i) * 4) : OOB;
            const uint32_t a2 = s1 ? OOB : (uint32_t)(((int64_t)r * (o.p2 ? o.ld2 : o.ld) + c2) * 4);
            const float x1 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs.r1, a1, 0, 0));
            const float x2 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs.r2, a2, 0, 0));
            float u = i == o.ones_col ? (r < lim ? 1.f : 0.f) : cok ? (s1 ? x1 : x2) : 0.f;
            if (o.act && s1 && cok) u = lrelu_ref(u);
            v[e] = u;
        }
    }
}

template <int Q>  // column quads of the operand's block
struct QStage {
    float4 v[8];
    // thread t loads the column quad c0 + 4 (t % Q) of rows r0 + 8 (t / Q) .. + 7 as 8 float4 (rows past the
    // split's end read 0 through the buffer range).  Lanes whose quad is special (a column past ncols, the
    // ones column) patch it only in waves that hold one (wave-uniform branch); LeakyReLU on p's columns.
    __device__ __forceinline__ void load(const Opnd &o, const OpRs &rs, int c0, int r0, int rend, int tid) {
        if (tid >= 4 * Q) return;
        const int q = tid % Q, oc = tid / Q;
        const int c = c0 + 4 * q, r = r0 + 8 * oc;
        const bool s1 = c < o.csplit;
        const int cc = s1 ? c : c - o.csplit;
        const int64_t ld = s1 ? o.ld : o.ld2;
        const bool cin = c < o.ncols;
        const uint32_t step = (uint32_t)(ld * 4);
        uint32_t off = (uint32_t)(((int64_t)r * ld + (cin ? cc : 0)) * 4);
        const bool mixed = __ballot(!s1) != 0 && o.p2;   // wave-uniform: a p2 quad in this wave
        if (!mixed) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = ld4(rs.r1, off + e * step);
        } else {
            const uint32_t o1 = s1 ? off : OOB, o2 = s1 ? OOB : off;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float4 a = ld4(rs.r1, o1 + e * step), b = ld4(rs.r2, o2 + e * step);
                v[e] = s1 ? a : b;
            }
        }
        if (o.act && s1) {
#pragma unroll
            for (int e = 0; e < 8; ++e)
                v[e] = make_float4(lrelu_ref(v[e].x), lrelu_ref(v[e].y), lrelu_ref(v[e].z), lrelu_ref(v[e].w));
        }
        const bool spec = c + 4 > o.ncols || (o.ones_col >= c && o.ones_col < c + 4);
        if (__ballot(spec) != 0) {   // wave-uniform
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const bool rok = r + e < rend;
                float x[4] = {v[e].x, v[e].y, v[e].z, v[e].w};
#pragma unroll
                for (int j = 0; j < 4; ++j) x[j] = c + j == o.ones_col ? (rok ? 1.f : 0.f) : c + j < o.ncols ? x[j] : 0.f;
                v[e] = make_float4(x[0], x[1], x[2], x[3]);
            }
        }
    }
    // lane fragments (column 4 q + j, octet oc) -> LDS ((tile * 2 + kstep) * 2 + hi/lo) * FRAG + L * 16
    template <bool P1 = false>
    __device__ __forceinline__ void store(char *base, float scale, int tid) const {
        if (tid >= 4 * Q) return;
        const int q = tid % Q, oc = tid / Q;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float x[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) x[e] = j == 0 ? v[e].x : j == 1 ? v[e].y : j == 2 ? v[e].z : v[e].w;
            const int m = 4 * q + j;
            const int t = m >> 5, L = (m & 31) + 32 * (oc & 1), s = oc >> 1;
            const X3Pair p = split8_scaled(x, scale);
            char *d = base + ((t * 2 + s) * 2) * FRAG + L * 16;
            *(h8 *)d = p.hi;
            if (!P1) *(h8 *)(d + FRAG) = p.lo;
        }
    }
};

// P1: the hi halves only (one fp16 product per fp32 product: the f16 training step's accuracy)
template <int WM, int WN, bool P1 = false>
__global__ __launch_bounds__(TPB, 1) void k_x3tn(GemmK g) {
    constexpr int TA = 4 * WM, TB = WN, BM = 32 * TA, BN = 32 * TB;
    constexpr int ABYTES = TA * 4 * FRAG, STAGE = (TA + TB) * 4 * FRAG;
    static_assert(BM / 4 * 4 <= TPB && BN / 4 * 4 <= TPB, "one quad-octet per thread");
    __shared__ __attribute__((aligned(16))) char lds[2 * STAGE];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int sa = op_shift(g.A), sb = op_shift(g.B);
    const float fa = ldexpf(1.f, sa), fb = ldexpf(1.f, sb), osc = ldexpf(1.f, -(sa + sb));
    const int nb_n = (g.N + BN - 1) / BN, nb_m = (g.M + BM - 1) / BM;
    int blk, split;
    tn_block(nb_m * nb_n, g.splits, blk, split);
    const int m0 = (blk / nb_n) * BM, n0 = (blk % nb_n) * BN;
    const int rows = min(g.d_rows ? *g.d_rows : 0x7fffffff, g.K);
    const int per = ((rows + g.splits - 1) / g.splits + 31) / 32 * 32;
    const int r0 = split * per, r1 = min(rows, r0 + per);
    const int nkb = r1 > r0 ? (r1 - r0 + 31) / 32 : 0;
    const OpRs ra = op_rsrc(g.A, r1), rb = op_rsrc(g.B, r1);
    f32x16 acc[WM][WN];
#pragma unroll
    for (int a = 0; a < WM; ++a)
#pragma unroll
        for (int b = 0; b < WN; ++b) acc[a][b] = f32x16{};
    QStage<BM / 4> a0, a1;
    QStage<BN / 4> b0, b1;
    auto compute = [&](const char *st) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            h8 ah[WM], al[WM];
#pragma unroll
            for (int a = 0; a < WM; ++a) {
                const char *p = st + (((w * WM + a) * 2 + s) * 2) * FRAG + lane * 16;
                ah[a] = *(const h8 *)p;
                al[a] = *(const h8 *)(p + FRAG);
            }
#pragma unroll
            for (int b = 0; b < WN; ++b) {
                const char *p = st + ABYTES + ((b * 2 + s) * 2) * FRAG + lane * 16;
                const h8 bh = *(const h8 *)p, bl = *(const h8 *)(p + FRAG);
#pragma unroll
                for (int a = 0; a < WM; ++a) {
                    if (!P1) {
                        acc[a][b] = mfma32(al[a], bh, acc[a][b]);
                        acc[a][b] = mfma32(ah[a], bl, acc[a][b]);
                    }
                    acc[a][b] = mfma32(ah[a], bh, acc[a][b]);
                }
            }
        }
    };
    if (nkb > 0) {
        a0.load(g.A, ra, m0, r0, r1, tid);
        b0.load(g.B, rb, n0, r0, r1, tid);
        if (nkb > 1) {
            a1.load(g.A, ra, m0, r0 + 32, r1, tid);
            b1.load(g.B, rb, n0, r0 + 32, r1, tid);
        }
        a0.template store<P1>(lds, fa, tid);
        b0.template store<P1>(lds + ABYTES, fb, tid);
        __syncthreads();
        // two stages per trip, so the register sets keep static names: stage kb in LDS buffer kb & 1,
        // stage kb + 1 in registers, stage kb + 2 loading
        for (int kb = 0; kb < nkb; kb += 2) {
            if (kb + 2 < nkb) {
                a0.load(g.A, ra, m0, r0 + 32 * (kb + 2), r1, tid);
                b0.load(g.B, rb, n0, r0 + 32 * (kb + 2), r1, tid);
            }
            compute(lds);
            if (kb + 1 < nkb) {
                a1.template store<P1>(lds + STAGE, fa, tid);
                b1.template store<P1>(lds + STAGE + ABYTES, fb, tid);
            }
            __syncthreads();
            if (kb + 1 >= nkb) break;
            if (kb + 3 < nkb) {
                a1.load(g.A, ra, m0, r0 + 32 * (kb + 3), r1, tid);
                b1.load(g.B, rb, n0, r0 + 32 * (kb + 3), r1, tid);
            }
            compute(lds + STAGE);
            if (kb + 2 < nkb) {
                a0.template store<P1>(lds, fa, tid);
                b0.template store<P1>(lds + ABYTES, fb, tid);
            }
            __syncthreads();
        }
    }
    // this split's partial [M][N] through a buffer: elements outside it are dropped, not branched around
    const __amdgpu_buffer_rsrc_t pr = rows_rsrc(g.part + (int64_t)split * g.M * g.N, g.N, g.M);
#pragma unroll
    for (int a = 0; a < WM; ++a)
#pragma unroll
        for (int b = 0; b < WN; ++b) {
            const int n = n0 + b * 32 + (lane & 31);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + (w * WM + a) * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                const uint32_t off = n < g.N ? (uint32_t)((m * g.N + n) * 4) : OOB;
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, acc[a][b][r] * osc), pr, off, 0, 0);
            }
        }
}

// ---- split-K weight gradients of the row layers (M = 256), LDS-DMA staged ------------------------
// part[split][m][n] = sum over the split's rows r of A(m, r) B(n, r): A = a delta [rows][256] (no column
// split, ones column or activation), B = the layer input ([rows][<= ld], column split, ones column and
// LeakyReLU as k_x3tn).  The raw fp32 rows of A (all 256 columns) and of B's 96-column block stream into
// two 3-slot LDS rings by LDS-DMA (rows past the split's end land as zeros through the buffer range
// check), A two stages ahead of its MFMAs, B three: B's stage is converted one stage ahead, once per
// workgroup (each wave a quarter: LeakyReLU, the ones column, the (hi, lo) split) into a fragment image
// the 8 waves share, while A's fragments are read straight from the raw stage by the wave that owns
// them (8 rows of one column per lane) and split in registers (the compiler's v_fma_mix).  18 MFMAs per
// 32-row stage and wave: waves own 32 rows of M, all 96 columns of the block; two waves per SIMD hide
// each other's LDS latencies.
constexpr int DW_ROWS = 32, DW_BN = 96, DW_NST = 3;
constexpr int DW_ABYTES = DW_ROWS * 256 * 4;       // 32 KiB: a raw A stage
constexpr int DW_BBYTES = DW_ROWS * DW_BN * 4;     // 12 KiB: a raw B stage
constexpr int DW_FBYTES = 2 * 3 * 2 * FRAG;        // 12 KiB: a stage's B fragments ((k-step 3 + tile) 2 + hi/lo)
constexpr int DW_LDS = DW_NST * (DW_ABYTES + DW_BBYTES) + 2 * DW_FBYTES;   // 156 KiB
constexpr int DW_TPB = 512;   // 8 waves

typedef _Float16 h4 __attribute__((ext_vector_type(4)));

// (t * scale) -> (hi, lo) fp16 halves (scale a power of two): v_fma_mix{lo,hi}_f16 the compiler forms itself
__device__ __forceinline__ X3Pair split8_mix(const float (&t)[8], float scale) {
    _Float16 h[8], l[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) h[j] = (_Float16)__builtin_fmaf(t[j], scale, 0.f);
#pragma unroll
    for (int j = 0; j < 8; ++j) l[j] = (_Float16)__builtin_fmaf(t[j], scale, -(float)h[j]);
    return X3Pair{h8{h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7]}, h8{l[0], l[1], l[2], l[3], l[4], l[5], l[6], l[7]}};
}

// 16 B per lane at byte voff (per lane) + soff (uniform) of buffer r into LDS ldsdst + 16 lane
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char *ldsdst, uint32_t voff, uint32_t soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void *)ldsdst, 16, voff, soff, 0, 0);
}

// this wave's DMAs but the last n issued have landed, its LDS writes are done, then the workgroup barrier
// (after it every wave's have); the asm's memory clobber keeps the compiler's LDS accesses on their side
// (a wave's last DMA group: A's 4 rows, then 1 or 2 B chunks -- each one or two exec-masked instructions
// -- so "all but the last 5" is a safe bound for every wave: it may wait for a little more, never less)
template <int N>
__device__ __forceinline__ void dw_wait_barrier() {
    static_assert(N == 5 || N == 4 || N == 0, "");
    if constexpr (N == 5) asm volatile("s_waitcnt vmcnt(5) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <bool BACT>   // LeakyReLU on B's p columns
__global__ __launch_bounds__(DW_TPB, 1) void k_x3dw(GemmK g) {
    __shared__ __attribute__((aligned(16))) char lds[DW_LDS];
    char *const la = lds, *const lb = lds + DW_NST * DW_ABYTES, *const lf = lb + DW_NST * DW_BBYTES;
    const int tid = threadIdx.x, lane = tid & 63, L = lane & 31, hk = lane >> 5;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int sa = op_shift(g.A), sb = op_shift(g.B);
    const float fa = ldexpf(1.f, sa), fb = ldexpf(1.f, sb), osc = ldexpf(1.f, -(sa + sb));
    const int nb_n = (g.N + DW_BN - 1) / DW_BN;
    int blk, split;
    tn_block(nb_n, g.splits, blk, split);
    const int n0 = blk * DW_BN;
    const int rows = min(g.d_rows ? *g.d_rows : 0x7fffffff, g.K);
    const int per = ((rows + g.splits - 1) / g.splits + 31) / 32 * 32;
    const int r0 = split * per, r1 = min(rows, r0 + per);
    const int nst = r1 > r0 ? (r1 - r0 + DW_ROWS - 1) / DW_ROWS : 0;
    const OpRs ra = op_rsrc(g.A, r1), rb = op_rsrc(g.B, r1);
    // B's DMA: chunk ci = 64 j + lane (j = w, w + 8 < 12) of the dense [32][96] stage, 16 B each: stage row
    // ci / 24, columns n0 + 4 (ci % 24) .. + 3 from p (columns < csplit) or p2; columns past ncols load 0
    // per-lane byte offsets relative to the stage's first row (the stage adds a uniform soffset)
    const uint32_t ald = (uint32_t)(g.A.ld * 4), bld1 = (uint32_t)(g.B.ld * 4),
                   bld2 = (uint32_t)((g.B.p2 ? g.B.ld2 : g.B.ld) * 4);
    uint32_t bv1[2], bv2[2];
    bool bs1[2];
    const bool two = w + 8 < 12;   // wave-uniform: a second chunk
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
        const int ci = 64 * (jj == 0 || two ? w + 8 * jj : w) + lane, rr = ci / 24, c = n0 + 4 * (ci % 24);
        bs1[jj] = c < g.B.csplit;
        const bool ok = c < g.B.ncols;
        bv1[jj] = ok && bs1[jj] ? (uint32_t)rr * bld1 + (uint32_t)(c * 4) : OOB;
        bv2[jj] = ok && !bs1[jj] ? (uint32_t)rr * bld2 + (uint32_t)((c - g.B.csplit) * 4) : OOB;
    }
    const bool bmixed = __ballot(!(bs1[0] && bs1[1])) != 0;   // wave-uniform: a p2 chunk in this wave
    // a mixed wave issues a chunk's p lanes and p2 lanes as two exec-masked instructions (at least one of
    // them has a lane: one or two instructions per chunk)
    const uint32_t av = (uint32_t)(4 * w) * ald + lane * 16;
    auto issue_a = [&](int st) {   // A rows r0 + 32 st .. into A slot st % 3: 4 rows per wave, a 1-KiB row each
        char *slot = la + (st % DW_NST) * DW_ABYTES;
        const uint32_t rs = (uint32_t)(r0 + DW_ROWS * st);
#pragma unroll
        for (int e = 0; e < 4; ++e) dma16(ra.r1, slot + (4 * w + e) * 1024, av, (rs + e) * ald);
    };
    auto issue_b = [&](int st) {   // B's block of those rows into B slot st % 3
        char *slot = lb + (st % DW_NST) * DW_BBYTES;
        const uint32_t rs = (uint32_t)(r0 + DW_ROWS * st);
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
            if (jj == 1 && !two) break;
            char *dst = slot + (w + 8 * jj) * 1024;
            if (!bmixed) {
                dma16(rb.r1, dst, bv1[jj], rs * bld1);
            } else {   // p and p2 lanes in separate exec-masked instructions
                if (bs1[jj]) dma16(rb.r1, dst, bv1[jj], rs * bld1);
                else dma16(rb.r2, dst, bv2[jj], rs * bld2);
            }
        }
    };
    // B's conversion: wave w takes half (w & 1) -- stage rows + 4 .. + 3 -- of the fragments kb = (w >> 1) + 4 j
    // < 6 (k-step kb / 3, tile kb % 3), j < 2 (waves w and w + 4 share a SIMD: 3 halves per SIMD); lane (L,
    // hk): column n0 + 32 (kb % 3) + L, rows 16 (kb / 3) + 8 hk + 4 half .. + 3.  x -> max(x, m x) is LeakyReLU (m = 0.01) or the identity (m = 1); columns past ncols
    // arrived as zeros; the ones column is patched in its wave only.
    const int half = w & 1;
    float cm[2];
    bool cone[2];
    int crow[2], ccol[2], cimg[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int kb = min((w >> 1) + 4 * j, 5), ks = kb / 3, b = kb % 3;
        const int c = n0 + 32 * b + L;
        cone[j] = c == g.B.ones_col;
        cm[j] = c < g.B.csplit ? 0.01f : 1.f;
        crow[j] = 16 * ks + 8 * hk + 4 * half;
        ccol[j] = 32 * b + L;
        cimg[j] = (kb * 2) * FRAG + lane * 16 + 8 * half;
    }
    const bool cspec = __ballot(cone[0] || (two && cone[1])) != 0;   // wave-uniform
    auto convert = [&](int st) {   // raw B slot st % 3 -> fragment image st & 1
        const float *src = (const float *)(lb + (st % DW_NST) * DW_BBYTES);
        char *dst = lf + (st & 1) * DW_FBYTES;
        const int rs = r0 + DW_ROWS * st;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            if (j == 1 && !two) break;
            float v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = src[(crow[j] + e) * DW_BN + ccol[j]];
            if (BACT) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {   // max(x, m x) as one v_max (no canonicalising max of the LDS value)
                    float t = v[e] * cm[j];
                    asm("v_max_f32 %0, %1, %0" : "+v"(t) : "v"(v[e]));
                    v[e] = t;
                }
            }
            if (cspec) {   // the ones column: 1 on the split's rows
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = cone[j] && rs + crow[j] + e < r1 ? 1.f : v[e];
            }
            _Float16 h[4], l[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) h[e] = (_Float16)__builtin_fmaf(v[e], fb, 0.f);
#pragma unroll
            for (int e = 0; e < 4; ++e) l[e] = (_Float16)__builtin_fmaf(v[e], fb, -(float)h[e]);
            *(h4 *)(dst + cimg[j]) = h4{h[0], h[1], h[2], h[3]};
            *(h4 *)(dst + cimg[j] + FRAG) = h4{l[0], l[1], l[2], l[3]};
        }
    };
    f32x16 acc[3];
#pragma unroll
    for (int b = 0; b < 3; ++b) acc[b] = f32x16{};
    // prologue: B(0) landed and converted; then A(0), B(1), A(1), B(2) in flight -- the loop's DMA groups
    // are (A(st + 2), B(st + 3)) in that order, so at stage st the last group issued may stay in flight
    if (nst > 0) {
        issue_b(0);
        dw_wait_barrier<0>();
        convert(0);
        issue_a(0);
        if (nst > 1) issue_b(1);
        if (nst > 1) issue_a(1);
        if (nst > 2) issue_b(2);
    }
    // stage st: A(st) and B(st + 1) landed (this wave's; the group issued last may stay in flight), every
    // wave's after the barrier, and every wave is done with stage st - 1 (its A slot, which A(st + 2)
    // reuses, and its fragment image, which B(st + 1)'s conversion reuses) and has converted B(st).
    // TAIL: one of the last three stages (fewer loads ahead)
    auto stage = [&](int st, auto tailc) {
        constexpr bool TAIL = decltype(tailc)::value;
        if constexpr (!TAIL) {
            dw_wait_barrier<5>();
            issue_a(st + 2);
            issue_b(st + 3);
            convert(st + 1);
        } else {
            if (st + 1 < nst) dw_wait_barrier<4>();
            else dw_wait_barrier<0>();
            if (st + 2 < nst) issue_a(st + 2);
            if (st + 1 < nst) convert(st + 1);
        }
        const char *slot = la + (st % DW_NST) * DW_ABYTES;
        const char *fr = lf + (st & 1) * DW_FBYTES + lane * 16;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int rr = 16 * ks + 8 * hk;   // this lane's 8 stage rows rr .. rr + 7
            X3Pair af, bf[3];
            {
                const float *src = (const float *)(slot + rr * 1024) + 32 * w + L;
                float v[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = src[256 * e];
                af = split8_mix(v, fa);
            }
#pragma unroll
            for (int b = 0; b < 3; ++b) {
                bf[b].hi = *(const h8 *)(fr + ((ks * 3 + b) * 2) * FRAG);
                bf[b].lo = *(const h8 *)(fr + ((ks * 3 + b) * 2 + 1) * FRAG);
            }
#pragma unroll
            for (int b = 0; b < 3; ++b) {
                acc[b] = mfma32(af.lo, bf[b].hi, acc[b]);
                acc[b] = mfma32(af.hi, bf[b].lo, acc[b]);
                acc[b] = mfma32(af.hi, bf[b].hi, acc[b]);
            }
        }
    };
    int st = 0;
    for (; st + 3 < nst; ++st) stage(st, std::false_type{});
    for (; st < nst; ++st) stage(st, std::true_type{});
    const __amdgpu_buffer_rsrc_t pr = rows_rsrc(g.part + (int64_t)split * g.M * g.N, g.N, g.M);
#pragma unroll
    for (int b = 0; b < 3; ++b) {
        const int n = n0 + b * 32 + L;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = 32 * w + (r & 3) + 8 * (r >> 2) + 4 * hk;
            const uint32_t off = n < g.N ? (uint32_t)((m * g.N + n) * 4) : OOB;
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, acc[b][r] * osc), pr, off, 0, 0);
        }
    }
}

// ---- rows mode, weights resident ----------------------------------------------------------------
// Y[r][n] = sum_k A(r, k) B(n, k) for the 32 WN columns of block blockIdx.x: the workgroup's block of
// B (KS k-steps of 16 x WN tiles of 32, hi / lo fp16 fragments, 2 KiB per (k-step, tile)) is DMA'd
// into LDS once (pre-split by k_x3bpack) or converted there, then the workgroup walks row tiles of 256
// rows (one 32-row MFMA tile per wave) with the A fragments loaded straight into registers: lane l holds
// row l & 31, k = 16 s + 8 (l >> 5) .. + 7 of k-step s, RT_PD k-steps ahead of the MFMAs.  One
// workgroup of 8 waves per CU (the weight block is up to 144 KiB): two waves per SIMD, one's epilogue
// (mask loads, stores) under the other's MFMAs.
constexpr int RT_W = 8, RT_TPB = 64 * RT_W, RT_ROWS = 32 * RT_W, RT_PD = 4;

// the A operand of the rows mode: row-major, 16-B aligned rows, columns in whole octets, the column
// split at a multiple of 16 (host-checked), read through buffers over the valid rows (rows past them
// read 0): lane's row offset in each source; k-step kb's source choice is wave-uniform
template <bool HASP2, bool ACT>   // the operand has a second source (columns >= csplit); LeakyReLU on p's
struct ARow {
    __amdgpu_buffer_rsrc_t r1, r2;
    uint32_t o1, o2;
    int csplit, ncols;
    __device__ __forceinline__ void load(int kb, int hk, float (&v)[8]) const {
        const int k = kb + 8 * hk;
        const bool s1 = !HASP2 || kb < csplit;  // wave-uniform
        const uint32_t off = k >= ncols ? OOB : s1 ? o1 + (uint32_t)k * 4 : o2 + (uint32_t)(k - csplit) * 4;
        const float4 x = ld4(s1 ? r1 : r2, off), y = ld4(s1 ? r1 : r2, off + 16);
        v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
        v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
        if (ACT && s1) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = lrelu_max(v[e]);
        }
    }
};
template <bool HASP2, bool ACT>
__device__ __forceinline__ ARow<HASP2, ACT> arow(const Opnd &o, const OpRs &rs, int row) {
    ARow<HASP2, ACT> a;
    a.r1 = rs.r1;
    a.r2 = rs.r2;
    a.o1 = (uint32_t)((int64_t)row * o.ld * 4);
    a.o2 = o.p2 ? (uint32_t)((int64_t)row * o.ld2 * 4) : a.o1;
    a.csplit = o.csplit;
    a.ncols = o.ncols;
    return a;
}

// HASP2: operand A has a second source; ACT: LeakyReLU on A; O2: the launch writes out2 (host-dispatched)
template <int KS, int WN, bool P1, bool HASP2, bool ACT, bool O2>
__global__ __launch_bounds__(RT_TPB, 1) void k_x3rows(GemmK g) {
    __shared__ __attribute__((aligned(16))) char lds[KS * WN * 2 * FRAG];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int sa = op_shift(g.A), sb = op_shift(g.B);
    const float fa = ldexpf(1.f, sa), fb = ldexpf(1.f, sb), osc = ldexpf(1.f, -(sa + sb));
    const int rows = min(g.d_rows ? *g.d_rows : 0x7fffffff, g.M);
    const int limA = min(rows, g.A.nrows);
    int nblk, rt;
    tn_block((g.N + 32 * WN - 1) / (32 * WN), g.splits, nblk, rt);
    const int gy = g.splits;
    const int n0 = nblk * (32 * WN);
    const int L = lane & 31, hk = lane >> 5;
    const OpRs rsA = op_rsrc(g.A, limA);
    // weights: lane fragment f = (k-step s, tile t, lane) -> ((s WN + t) 2 + hi/lo) FRAG + lane 16
    if (g.bpack) {   // the block's image, converted once per launch by k_x3bpack: 1 KiB per wave and instruction
        constexpr int BYTES = KS * WN * 2 * FRAG, NCH = BYTES / 1024;
        const __amdgpu_buffer_rsrc_t rp =
            __builtin_amdgcn_make_buffer_rsrc(g.bpack + (int64_t)nblk * BYTES, (short)0, BYTES, 0x00020000);
#pragma unroll
        for (int j = 0; j < (NCH + RT_W - 1) / RT_W; ++j)
            if (NCH % RT_W == 0 || RT_W * j + w < NCH)
                dma16(rp, lds + (RT_W * j + w) * 1024, lane * 16 + w * 1024, j * (RT_W * 1024));
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        const OpRs rsB = op_rsrc(g.B, g.B.nrows);
        for (int f = tid; f < KS * WN * 64; f += RT_TPB) {
            const int fl = f & 63, t = (f >> 6) % WN, s = f / (64 * WN);
            float v[8];
            load8(g.B, rsB, n0 + 32 * t + (fl & 31), 16 * s + 8 * (fl >> 5), g.B.nrows, v);
            const X3Pair x = split8_scaled(v, fb);
            char *d = lds + ((s * WN + t) * 2) * FRAG + fl * 16;
            *(h8 *)d = x.hi;
            if (!P1) *(h8 *)(d + FRAG) = x.lo;
        }
    }
    __syncthreads();
    float am1 = 0.f, am2 = 0.f;
    // outputs, mask and bias through buffers over the valid rows / columns (no per-value branches)
    const __amdgpu_buffer_rsrc_t ro1 = rows_rsrc(g.out, g.ldo, rows);
    const __amdgpu_buffer_rsrc_t ro2 = rows_rsrc(O2 ? g.out2 : g.out, O2 ? g.ldo2 : g.ldo, O2 ? rows : 0);
    const __amdgpu_buffer_rsrc_t rmk = rows_rsrc(g.mask ? g.mask : g.out, g.ldm, g.mask ? rows : 0);
    const __amdgpu_buffer_rsrc_t rbs = rows_rsrc(g.bias ? g.bias : g.out, 1, g.bias ? g.N : 0);
    for (; rt * RT_ROWS < rows; rt += gy) {
        const int m0 = rt * RT_ROWS + 32 * w;
        const ARow<HASP2, ACT> ar = arow<HASP2, ACT>(g.A, rsA, m0 + L);
        // A: k-steps s .. s + RT_PD - 1 in flight while k-step s's MFMAs run (a ring of RT_PD octets)
        float a[RT_PD][8];
#pragma unroll
        for (int s = 0; s < RT_PD; ++s) ar.load(16 * s, hk, a[s]);
        f32x16 acc[WN];
#pragma unroll
        for (int t = 0; t < WN; ++t) acc[t] = f32x16{};
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const X3Pair x = split8_mix(a[s % RT_PD], fa);   // compiler-formed: its hazard recognizer sees it
            if (s + RT_PD < KS) ar.load(16 * (s + RT_PD), hk, a[s % RT_PD]);
            const char *p = lds + (s * WN * 2) * FRAG + lane * 16;
#pragma unroll
            for (int t = 0; t < WN; ++t) {
                const h8 bh = *(const h8 *)(p + (2 * t) * FRAG);
                if (!P1) {
                    const h8 bl = *(const h8 *)(p + (2 * t + 1) * FRAG);
                    acc[t] = mfma32(x.lo, bh, acc[t]);
                    acc[t] = mfma32(x.hi, bl, acc[t]);
                }
                acc[t] = mfma32(x.hi, bh, acc[t]);
            }
            __builtin_amdgcn_sched_barrier(0);   // k-steps in order: the A ring's registers stay bounded
        }
        // epilogue per 32-column tile: its 16 mask values loaded before any is used (columns past out_cols read
        // 0: only out's columns are masked); lane offsets of the tile's first row with the row terms as scalar
        // offsets; rows past the valid ones read 0 / are dropped by the buffer ranges and, in the one tile that
        // has them (FULL false), kept out of the amax words; columns past N are 0 (zero B rows, no bias)
        auto epilogue = [&](auto fullc) {
            constexpr bool FULL = decltype(fullc)::value;
            const uint32_t rb = (uint32_t)(m0 + 4 * hk);
#pragma unroll
            for (int t = 0; t < WN; ++t) {
                const int n = n0 + 32 * t + L;
                const float bv =
                    __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rbs, n < g.N ? (uint32_t)n * 4 : OOB, 0, 0));
                const bool o1 = n < g.out_cols, o2 = O2 && !o1 && n < g.N;
                const uint32_t b1 = o1 ? (rb * (uint32_t)g.ldo + (uint32_t)n) * 4 : OOB;
                const uint32_t bm = o1 ? (rb * (uint32_t)g.ldm + (uint32_t)n) * 4 : OOB;
                const uint32_t b2 = o2 ? (rb * (uint32_t)g.ldo2 + (uint32_t)(n - g.out_cols)) * 4 : OOB;
                float mk[16];
                if (g.mask) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const uint32_t rr = (r & 3) + 8 * (r >> 2);
                        mk[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rmk, bm, rr * (uint32_t)g.ldm * 4, 0));
                    }
                }
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const uint32_t rr = (r & 3) + 8 * (r >> 2);
                    float v = acc[t][r] * osc + bv;
                    if (g.mask && (!O2 || o1) && !(mk[r] > 0.f)) v *= 0.01f;
                    const float v1 = g.act ? lrelu_max(v) : v;
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v1), ro1, b1, rr * (uint32_t)g.ldo * 4, 0);
                    const bool rok = FULL || (int)(rb + rr) < rows;
                    am1 = fmaxf(am1, (!O2 || o1) && rok ? fabsf(v1) : 0.f);
                    if constexpr (O2) {
                        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), ro2, b2,
                                                              rr * (uint32_t)g.ldo2 * 4, 0);
                        am2 = fmaxf(am2, o2 && rok ? fabsf(v) : 0.f);
                    }
                }
            }
        };
        if (m0 + 32 <= rows) epilogue(std::true_type{});   // wave-uniform
        else epilogue(std::false_type{});
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        am1 = fmaxf(am1, __shfl_xor(am1, o));
        am2 = fmaxf(am2, __shfl_xor(am2, o));
    }
    if (lane == 0) {
        if (g.amax_out) atomicMax(g.amax_out, __builtin_bit_cast(uint32_t, am1));
        if (g.amax_out2) atomicMax(g.amax_out2, __builtin_bit_cast(uint32_t, am2));
    }
}

// The weight blocks of a rows-mode launch in the LDS image k_x3rows stages: block b at b KS WN 2 FRAG
// bytes, one thread per lane fragment (the same load8 / split as the in-workgroup conversion).
template <int KS, int WN, bool P1>
__global__ __launch_bounds__(TPB) void k_x3bpack(GemmK g) {
    constexpr int PER = KS * WN * 64;
    const int f = blockIdx.x * TPB + threadIdx.x;
    const int nb = (g.N + 32 * WN - 1) / (32 * WN);
    if (f >= nb * PER) return;
    const int b = f / PER, fr = f % PER;
    const int fl = fr & 63, t = (fr >> 6) % WN, s = fr / (64 * WN);
    const float fb = ldexpf(1.f, op_shift(g.B));
    const OpRs rsB = op_rsrc(g.B, g.B.nrows);
    float v[8];
    load8(g.B, rsB, b * 32 * WN + 32 * t + (fl & 31), 16 * s + 8 * (fl >> 5), g.B.nrows, v);
    const X3Pair x = split8_scaled(v, fb);
    char *d = g.bpack + (int64_t)b * (KS * WN * 2 * FRAG) + ((s * WN + t) * 2) * FRAG + fl * 16;
    *(h8 *)d = x.hi;
    if (!P1) *(h8 *)(d + FRAG) = x.lo;
}

// ---- deterministic work list and compact row offsets ---------------------------------------

constexpr int LIST_PER_BLOCK = 1024;  // samples per block (4 per thread)

// exclusive scan of one int2 per thread over the workgroup, in thread order; returns the total
__device__ __forceinline__ int2 block_scan2(int2 v, int2 &excl, int2 *sh) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int2 inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int x = __shfl_up(inc.x, o), y = __shfl_up(inc.y, o);
        if (lane >= o) {
            inc.x += x;
            inc.y += y;
        }
    }
    if (lane == 63) sh[w] = inc;
    __syncthreads();
    int2 base = make_int2(0, 0), tot = make_int2(0, 0);
    for (int i = 0; i < TPB / 64; ++i) {
        if (i < w) {
            base.x += sh[i].x;
            base.y += sh[i].y;
        }
        tot.x += sh[i].x;
        tot.y += sh[i].y;
    }
    excl = make_int2(base.x + inc.x - v.x, base.y + inc.y - v.y);
    __syncthreads();
    return tot;
}

__device__ __forceinline__ int2 count4(const int32_t *nnb, int s0, int S, int (&n)[4]) {
    int2 c = make_int2(0, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int s = s0 + j;
        n[j] = s < S ? nnb[s] : 0;
        c.x += n[j] > 0;
        c.y += n[j];
    }
    return c;
}

__global__ __launch_bounds__(TPB) void k_lists_count(const int32_t *counters, const int32_t *nnb, int2 *bsum) {
    __shared__ int2 sh[TPB / 64];
    const int S = counters[0];
    int n[4];
    const int2 c = count4(nnb, blockIdx.x * LIST_PER_BLOCK + threadIdx.x * 4, S, n);
    int2 ex;
    const int2 tot = block_scan2(c, ex, sh);
    if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(TPB) void k_lists_write(const int32_t *counters, const int32_t *nnb, const int2 *bsum,
                                                     int32_t *work, int32_t *row_off, float4 *feat, int32_t *tl) {
    __shared__ int2 sh[TPB / 64];
    __shared__ int2 bb[TPB / 64];
    const int S = counters[0];
    const int s_blk = blockIdx.x * LIST_PER_BLOCK;
    // base = sum of the previous blocks' totals (fixed order: per-thread strided sums, then waves)
    int2 pb = make_int2(0, 0);
    for (int b = threadIdx.x; b < (int)blockIdx.x; b += TPB) {
        pb.x += bsum[b].x;
        pb.y += bsum[b].y;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        pb.x += __shfl_xor(pb.x, o);
        pb.y += __shfl_xor(pb.y, o);
    }
    if ((threadIdx.x & 63) == 0) bb[threadIdx.x >> 6] = pb;
    __syncthreads();
    int2 base = make_int2(0, 0);
    for (int i = 0; i < TPB / 64; ++i) {
        base.x += bb[i].x;
        base.y += bb[i].y;
    }
    int n[4];
    const int s0 = s_blk + threadIdx.x * 4;
    const int2 c = count4(nnb, s0, S, n);
    int2 ex;
    const int2 tot = block_scan2(c, ex, sh);
    int it = base.x + ex.x, ro = base.y + ex.y;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int s = s0 + j;
        if (s < S) {
            row_off[s] = ro;
            if (n[j] > 0) work[it++] = s;
            ro += n[j];
            feat[s] = make_float4(0.f, 0.f, 0.f, 0.f);  // the forward writes alpha / rgb of items only
        }
    }
    // the block holding the last sample (block 0 when there are none) publishes the totals
    const int last = S > 0 ? S - 1 : 0;
    if (threadIdx.x == 0 && last >= s_blk && last < s_blk + LIST_PER_BLOCK) {
        tl[0] = base.x + tot.x;
        tl[1] = base.y + tot.y;
    }
}

// ---- per-row / per-item kernels (one wave per work item, its rows in turn) ------------------

struct RowArgs {
    const float *xyz, *emb, *color, *dir, *conf, *campos, *rot, *raydir;
    const int32_t *counters, *work, *samp_ray, *samp_nnb, *pidx, *row_off, *tl;
    const float *samp_locw;
    int32_t K;
};

__device__ __forceinline__ int n_items(const RowArgs &r) { return r.tl[0]; }

// x0 columns c0..c0+3 (c0 % 4 == 0) of a row (point_aggregators.py:594-621: [emb | PE(emb, 3) |
// PE(dists, 5)], then the ones column 284 that carries block1.0's bias gradient, zero padding to
// 288).  PE columns come in (sin, cos) pairs of one argument: pair p of PE(emb) is channel p / 3 at
// frequency 2^(p % 3), of PE(dists) channel p / 5 at 2^(p % 5) (networks.py:175-192)
__device__ __forceinline__ f32x4 x0_quad(int c0, const float *e, const float (&d)[6]) {
    f32x4 v;
    if (c0 < 32) return *(const f32x4 *)(e + c0);
    if (c0 >= 284) {
        v[0] = 1.f; v[1] = v[2] = v[3] = 0.f;
        return v;
    }
    const bool pe_emb = c0 < 224;
    const int p0 = (c0 - (pe_emb ? 32 : 224)) >> 1;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int p = p0 + h;
        const int ch = pe_emb ? p / 3 : p / 5, f = pe_emb ? p % 3 : p % 5;
        const float base = pe_emb ? e[ch] : d[ch];
        float sn, cs;
        sincos_acc(base * (float)(1 << f), sn, cs);
        v[2 * h] = sn;
        v[2 * h + 1] = cs;
    }
    return v;
}

// dists of a row and the sample's linear-kernel weights (point_aggregators.py:494-502, :868-953;
// the same arithmetic as the forward's gather_row): lane k < K of the wave holds row k's
__device__ __forceinline__ void row_geometry(const RowArgs &a, const Cam &cam, int s, int pid, float (&d)[6], float &wn,
                                             float &wgt) {
    const float lx = a.samp_locw[(int64_t)s * 3], ly = a.samp_locw[(int64_t)s * 3 + 1], lz = a.samp_locw[(int64_t)s * 3 + 2];
    const bool m = pid >= 0;
    float px = 0.f, py = 0.f, pz = 0.f, cf = 0.f;
    if (m) {
        px = a.xyz[(int64_t)pid * 3]; py = a.xyz[(int64_t)pid * 3 + 1]; pz = a.xyz[(int64_t)pid * 3 + 2];
        cf = a.conf[pid];
    }
    const float dwx = __fsub_rn(px, lx), dwy = __fsub_rn(py, ly), dwz = __fsub_rn(pz, lz);
    float xp = 0.f, yp = 0.f, zp = 0.f, xl, yl, zl;
    if (m) cam.pers(px, py, pz, xp, yp, zp);
    cam.pers(lx, ly, lz, xl, yl, zl);
    d[0] = m ? dwx : 0.f; d[1] = m ? dwy : 0.f; d[2] = m ? dwz : 0.f;
    d[3] = m ? __fsub_rn(__fmul_rn(xp, zp), __fmul_rn(xl, zl)) : 0.f;
    d[4] = m ? __fsub_rn(__fmul_rn(yp, zp), __fmul_rn(yl, zl)) : 0.f;
    d[5] = m ? __fsub_rn(zp, zl) : 0.f;
    float w = 0.f;
    if (m) {
        const float n2 = __fadd_rn(__fadd_rn(__fmul_rn(dwx, dwx), __fmul_rn(dwy, dwy)), __fmul_rn(dwz, dwz));
        w = 1.f / fmaxf(sqrtf(n2), 1e-6f);
    }
    wn = w;
    wgt = cf;
}

// x0 as 72 quads + ext as 2 quads per row: the item's rows x quads are one flat task list over the
// wave's lanes (row geometry from lane k by a lane-indexed shuffle)
constexpr int X0_QUADS = 72, ROW_QUADS = 74;

__global__ __launch_bounds__(TPB) void k_row_inputs(RowArgs a, float *x0, float *ext, float2 *rw, float *vpe) {
    // Two items per wave, one per half-wave (lanes 32 h .. 32 h + 31): the items' dependent index chains
    // (work -> sample -> neighbours -> point records) are in flight together, so a wave pays that
    // latency once per two items.  The items' rows' embeddings are staged in LDS once (the PE tasks
    // read them there instead of issuing a dependent global load per task).
    __shared__ __attribute__((aligned(16))) float se[TPB / 64][2][8 * 32];  // K <= 8 rows per item
    const int lane = threadIdx.x & 63, wl = threadIdx.x >> 6, h = lane >> 5, l32 = lane & 31;
    const int wv = blockIdx.x * (TPB / 64) + wl, nw = gridDim.x * (TPB / 64);
    const Cam cam = load_cam(a.campos, a.rot);
    const int n = n_items(a);
    for (int i2 = wv; 2 * i2 < n; i2 += nw) {
        const int it = 2 * i2 + h;
        const bool iv = it < n;
        const int s = iv ? a.work[it] : 0;
        const int nnb = iv ? a.samp_nnb[s] : 0, ro = iv ? a.row_off[s] : 0;
        const int ray = iv ? a.samp_ray[s] : 0;
        // lanes k < K of each half: row k's geometry and weight; normalised over the sample's rows
        const int kl = l32 < a.K ? l32 : 0;
        const int pidl = l32 < nnb ? a.pidx[(int64_t)s * a.K + kl] : -1;
        float dl[6], w, cf;
        row_geometry(a, cam, s, pidl, dl, w, cf);
        float wsum = w;
#pragma unroll
        for (int o = 1; o < 8; o <<= 1) wsum += __shfl_xor(wsum, o);  // lanes 32 h .. 32 h + 7 (K <= 8)
        wsum = __shfl(wsum, 32 * h);
        const float wn = w / fmaxf(wsum, 1e-8f);
        const float wgt = wn * fminf(fmaxf(cf, 1e-4f), 1.f);
        if (l32 < nnb) rw[ro + l32] = make_float2(wgt, wn);
        const float vx = a.raydir[(int64_t)ray * 3], vy = a.raydir[(int64_t)ray * 3 + 1], vz = a.raydir[(int64_t)ray * 3 + 2];
        if (iv) {  // the item's PE(viewdir) for the colour MLP (:772-780), ones column 24
            float v = l32 == 24 ? 1.f : 0.f;
            if (l32 < 24) {
                const int jj = l32 < 12 ? l32 : l32 - 12, c = jj >> 2, f = jj & 3;
                float sn, cs;
                sincos_acc((c == 0 ? vx : c == 1 ? vy : vz) * (float)(1 << f), sn, cs);
                v = l32 < 12 ? sn : cs;
            }
            vpe[(int64_t)it * 32 + l32] = v;
        }
        {   // half-lane l: floats 8 (l & 3) .. + 7 of row l >> 2
            const int k = l32 >> 2;
            const int pk = __shfl(pidl, 32 * h + k);
            f32x4 e0 = {0.f, 0.f, 0.f, 0.f}, e1 = e0;
            if (k < nnb && pk >= 0) {
                const f32x4 *src = (const f32x4 *)(a.emb + (int64_t)pk * 32 + 8 * (l32 & 3));
                e0 = src[0];
                e1 = src[1];
            }
            *(f32x4 *)&se[wl][h][32 * k + 8 * (l32 & 3)] = e0;
            *(f32x4 *)&se[wl][h][32 * k + 8 * (l32 & 3) + 4] = e1;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // one wave: its own writes are every lane's
        }
        const int ntask = nnb * ROW_QUADS;
        const int nmax = max(ntask, __shfl_xor(ntask, 32));
        for (int t0 = 0; t0 < nmax; t0 += 32) {  // wave-uniform trip count: the shuffles see every lane
            const int t = t0 + l32;
            const bool act = t < ntask;
            const int k = act ? t / ROW_QUADS : 0, q = t - k * ROW_QUADS;
            const int pid = __shfl(pidl, 32 * h + k);
            float d[6];
#pragma unroll
            for (int c = 0; c < 6; ++c) d[c] = __shfl(dl[c], 32 * h + k);
            if (!act) continue;
            const int64_t row = ro + k;
            const int64_t pb = (int64_t)pid * 3;
            if (q < X0_QUADS) {
                *(f32x4 *)(x0 + row * 288 + 4 * q) = x0_quad(4 * q, &se[wl][h][32 * k], d);
            } else if (q == X0_QUADS) {  // block3.0's extra channels (:639-652): colour, dir - v
                f32x4 u;
                u[0] = a.color[pb]; u[1] = a.color[pb + 1]; u[2] = a.color[pb + 2];
                u[3] = __fsub_rn(a.dir[pb], vx);
                *(f32x4 *)(ext + row * 8) = u;
            } else {  // dir - v, <dir, v>, and the ones column of block3.0's bias
                const float d0 = a.dir[pb], d1 = a.dir[pb + 1], d2 = a.dir[pb + 2];
                f32x4 u;
                u[0] = __fsub_rn(d1, vy);
                u[1] = __fsub_rn(d2, vz);
                u[2] = __fadd_rn(__fadd_rn(__fmul_rn(d0, vx), __fmul_rn(d1, vy)), __fmul_rn(d2, vz));
                u[3] = 1.f;
                *(f32x4 *)(ext + row * 8 + 4) = u;
            }
        }
    }
}

// d_dst[row] = d_src[pid of the row] (dim floats, as quads): the item's rows x quads as one flat list
__global__ __launch_bounds__(TPB) void k_row_gather(RowArgs a, const float *src, int dim, float *dst) {
    const int lane = threadIdx.x & 63;
    const int wv = blockIdx.x * (TPB / 64) + (threadIdx.x >> 6), nw = gridDim.x * (TPB / 64);
    const int n = n_items(a), nq = dim >> 2;
    for (int it = wv; it < n; it += nw) {
        const int s = a.work[it];
        const int nnb = a.samp_nnb[s], ro = a.row_off[s];
        for (int t = lane; t < nnb * nq; t += 64) {
            const int k = t / nq, q = t - k * nq;
            const int pid = a.pidx[(int64_t)s * a.K + k];
            *(f32x4 *)(dst + (int64_t)(ro + k) * dim + 4 * q) = *(const f32x4 *)(src + (int64_t)pid * dim + 4 * q);
        }
    }
}

// wave-wide sum
__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    return x;
}

// color_branch.6 (128 -> 3) + sigmoid * (1 + 2e-3) - 1e-3 in fp32; rgb into feat[s].yzw
__global__ __launch_bounds__(TPB) void k_colour_head(RowArgs a, const float *h3, const float *w6, const float *b6,
                                                     float4 *feat) {
    const int lane = threadIdx.x & 63;
    const int wv = blockIdx.x * (TPB / 64) + (threadIdx.x >> 6), nw = gridDim.x * (TPB / 64);
    const int n = n_items(a);
    for (int it = wv; it < n; it += nw) {
        const float2 h = *(const float2 *)(h3 + (int64_t)it * 128 + 2 * lane);
        float y[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) y[c] = wave_sum(h.x * w6[c * 128 + 2 * lane] + h.y * w6[c * 128 + 2 * lane + 1]) + b6[c];
        if (lane == 0) {
            const int s = a.work[it];
            float4 f = feat[s];
            f.y = 1.f / (1.f + expf(-y[0])) * 1.002f - 0.001f;
            f.z = 1.f / (1.f + expf(-y[1])) * 1.002f - 0.001f;
            f.w = 1.f / (1.f + expf(-y[2])) * 1.002f - 0.001f;
            feat[s] = f;
        }
    }
}

constexpr int HEAD_BLOCKS = 256;
// k_row_head's workgroups (its partials: [ROW_HEAD_BLOCKS][257], summed in a fixed order by k_reduce_wide):
// 1024 took the head 132 -> 101 us per config-5 step (one wave walks ~4 items instead of ~15)
constexpr int ROW_HEAD_BLOCKS = 1024;

// backward of k_colour_head: dy4 = d rgb 1.002 sig (1 - sig); dy3 = (W6^T dy4) LReLU'(h3); the
// weight / bias gradient of color_branch.6 as one fixed-order partial per workgroup
// ([HEAD_BLOCKS][3][129]: 128 weights then the bias)
__global__ __launch_bounds__(TPB) void k_colour_head_bwd(RowArgs a, const float *h3, const float *w6, const float *b6,
                                                         const float4 *dfeat, float *dy3, uint32_t *amax, float *part) {
    __shared__ float sh[TPB / 64][3][130];
    const int lane = threadIdx.x & 63, wl = threadIdx.x >> 6;
    const int wv = blockIdx.x * (TPB / 64) + wl, nw = gridDim.x * (TPB / 64);
    const int n = n_items(a);
    float gw[3][2] = {}, gb[3] = {}, am = 0.f;
    for (int it = wv; it < n; it += nw) {
        const float2 h = *(const float2 *)(h3 + (int64_t)it * 128 + 2 * lane);
        const float4 df = dfeat[a.work[it]];
        const float dr[3] = {df.y, df.z, df.w};
        float dy[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float y = wave_sum(h.x * w6[c * 128 + 2 * lane] + h.y * w6[c * 128 + 2 * lane + 1]) + b6[c];
            const float sg = 1.f / (1.f + expf(-y));
            dy[c] = dr[c] * 1.002f * (sg * (1.f - sg));
            gw[c][0] += dy[c] * h.x;
            gw[c][1] += dy[c] * h.y;
            gb[c] += dy[c];
        }
        float d0 = dy[0] * w6[2 * lane] + dy[1] * w6[128 + 2 * lane] + dy[2] * w6[256 + 2 * lane];
        float d1 = dy[0] * w6[2 * lane + 1] + dy[1] * w6[128 + 2 * lane + 1] + dy[2] * w6[256 + 2 * lane + 1];
        d0 = h.x > 0.f ? d0 : d0 * 0.01f;
        d1 = h.y > 0.f ? d1 : d1 * 0.01f;
        *(float2 *)(dy3 + (int64_t)it * 128 + 2 * lane) = make_float2(d0, d1);
        am = fmaxf(am, fmaxf(fabsf(d0), fabsf(d1)));
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        sh[wl][c][2 * lane] = gw[c][0];
        sh[wl][c][2 * lane + 1] = gw[c][1];
        if (lane == 0) sh[wl][c][128] = gb[c];
    }
    __syncthreads();
    for (int j = threadIdx.x; j < 3 * 129; j += TPB) {
        const int c = j / 129, u = j % 129;
        float v = 0.f;
        for (int q = 0; q < TPB / 64; ++q) v += sh[q][c][u];
        part[(int64_t)blockIdx.x * 3 * 129 + j] = v;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) am = fmaxf(am, __shfl_xor(am, o));
    if (lane == 0) atomicMax(amax, __builtin_bit_cast(uint32_t, am));
}

__device__ __forceinline__ float softplus_ref(float x) { return x > 20.f ? x : log1pf(expf(x)); }

// block3.2's output and everything between it and the blended feature (point_aggregators.py:
// 640-653, :743-770): h4 = LReLU(z4); alpha = softplus(wa h4 + ba - 1); f_s = sum_k w_k h4_k,
// alpha_s = sum_k w_k alpha_k.  Backward per row: dza = w dalpha_s sigmoid(za - 1);
// d w = <h4, d f_s> + alpha dalpha_s (-> d conf = d w * w_norm through the straight-through clamp);
// delta4 = (w d f_s + dza wa) LReLU'(z4) (in place over z4).  dWa / dba partial per workgroup
// ([HEAD_BLOCKS][257]).
// 16 wave-wide sums at once, reduce-scatter style (17 cross-lane moves instead of 96): on return,
// the sum of v[j] over the wave sits in lane 4 j of v[0] (fixed order, deterministic)
__device__ __forceinline__ void wave_sum16(float (&v)[16], int lane) {
#pragma unroll
    for (int h = 8; h >= 1; h >>= 1) {  // exchange distance 32, 16, 8, 4 halves the live values
        const int o = 4 * h;
        const bool up = lane & o;
#pragma unroll
        for (int i = 0; i < h; ++i) {
            const float send = up ? v[i] : v[i + h];
            const float keep = up ? v[i + h] : v[i];
            v[i] = keep + __shfl_xor(send, o);
        }
    }
    v[0] += __shfl_xor(v[0], 2);
    v[0] += __shfl_xor(v[0], 1);
}
__device__ __forceinline__ float lane_value(float x, int l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), l));
}

constexpr int MAX_K = 8;

__global__ __launch_bounds__(TPB) void k_row_head(RowArgs a, float *z4d4, const float *dfs, const float4 *dfeat,
                                                  const float2 *rw, const float *wa, const float *ba, float *g_conf,
                                                  uint32_t *amax, float *part) {
    __shared__ float sh[TPB / 64][260];
    const int lane = threadIdx.x & 63, wl = threadIdx.x >> 6;
    const int wv = blockIdx.x * (TPB / 64) + wl, nw = gridDim.x * (TPB / 64);
    const int n = n_items(a);
    const f32x4 wa4 = *(const f32x4 *)(wa + 4 * lane);
    const float bav = ba[0];
    f32x4 gw = {0.f, 0.f, 0.f, 0.f};
    float gb = 0.f, am = 0.f;
    for (int it = wv; it < n; it += nw) {
        const int s = a.work[it];
        const int nnb = a.samp_nnb[s], ro = a.row_off[s];
        const float das = dfeat[s].x;
        const f32x4 df = *(const f32x4 *)(dfs + (int64_t)it * 256 + 4 * lane);
        // all rows' z4 in flight at once, then their two dot products in one batched reduction
        f32x4 z[MAX_K];
        float red[16];
#pragma unroll
        for (int k = 0; k < MAX_K; ++k) {
            z[k] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (k < nnb) z[k] = *(const f32x4 *)(z4d4 + (int64_t)(ro + k) * 256 + 4 * lane);
        }
        const float2 wwl = lane < nnb ? rw[ro + lane] : make_float2(0.f, 0.f);
#pragma unroll
        for (int k = 0; k < MAX_K; ++k) {
            float pa = 0.f, pd = 0.f;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float h = lrelu_ref(z[k][q]);
                pa += wa4[q] * h;
                pd += h * df[q];
            }
            red[k] = pa;
            red[MAX_K + k] = pd;
        }
        wave_sum16(red, lane);
        float gc = 0.f;
#pragma unroll
        for (int k = 0; k < MAX_K; ++k) {
            if (k >= nnb) break;
            const float za = lane_value(red[0], 4 * k) + bav;
            const float dot = lane_value(red[0], 4 * (MAX_K + k));
            const float x = za - 1.f;
            const float al = softplus_ref(x), sg = x > 20.f ? 1.f : 1.f / (1.f + expf(-x));
            const float wk = lane_value(wwl.x, k), wnk = lane_value(wwl.y, k);
            const float dza = wk * das * sg;
            const float dw = dot + al * das;
            f32x4 d;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float h = lrelu_ref(z[k][q]);
                const float t = wk * df[q] + dza * wa4[q];
                d[q] = z[k][q] > 0.f ? t : t * 0.01f;
                am = fmaxf(am, fabsf(d[q]));
                gw[q] += dza * h;
            }
            gb += dza;
            *(f32x4 *)(z4d4 + (int64_t)(ro + k) * 256 + 4 * lane) = d;
            if (lane == k) gc = dw * wnk;
        }
        if (lane < nnb) atomicAdd(g_conf + a.pidx[(int64_t)s * a.K + lane], gc);
    }
    *(f32x4 *)&sh[wl][4 * lane] = gw;
    if (lane == 0) sh[wl][256] = gb;
    __syncthreads();
    for (int j = threadIdx.x; j < 257; j += TPB) {
        float v = 0.f;
        for (int q = 0; q < TPB / 64; ++q) v += sh[q][j];
        part[(int64_t)blockIdx.x * 257 + j] = v;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) am = fmaxf(am, __shfl_xor(am, o));
    if (lane == 0) atomicMax(amax, __builtin_bit_cast(uint32_t, am));
}

// the point gradients of a row: d emb through [emb | PE(emb)] (networks.py:175-192) from block1.0's
// input gradient dx0 [rows][224]; d colour, d dir from block3.0's extra-channel gradient dext
// [rows][8] (d (dir - v) + v d <dir, v>)
// tasks per row: 32 embedding channels, then colour (3) and dir (3); the item's rows x tasks are
// one flat list over the wave's lanes
constexpr int TAIL_TASKS = 38;

__global__ __launch_bounds__(TPB) void k_row_tail(RowArgs a, const float *dx0, const float *dext, float *g_emb,
                                                  float *g_color, float *g_dir) {
    const int lane = threadIdx.x & 63;
    const int wv = blockIdx.x * (TPB / 64) + (threadIdx.x >> 6), nw = gridDim.x * (TPB / 64);
    const int n = n_items(a);
    for (int it = wv; it < n; it += nw) {
        const int s = a.work[it];
        const int nnb = a.samp_nnb[s], ro = a.row_off[s];
        const int ray = a.samp_ray[s];
        const int ntask = nnb * TAIL_TASKS;
        for (int t = lane; t < ntask; t += 64) {
            const int k = t / TAIL_TASKS, c = t - k * TAIL_TASKS;
            const int64_t j = ro + k;
            const int pid = a.pidx[(int64_t)s * a.K + k];
            if (c < 32) {
                const float *g = dx0 + j * 224;
                const float e = a.emb[(int64_t)pid * 32 + c];
                float de = g[c];
#pragma unroll
                for (int f = 0; f < 3; ++f) {
                    const float sc = (float)(1 << f);
                    float sn, cs;
                    sincos_acc(e * sc, sn, cs);
                    const int col = 32 + 2 * (3 * c + f);
                    de += g[col] * cs * sc - g[col + 1] * sn * sc;
                }
                atomicAdd(g_emb + (int64_t)pid * 32 + c, de);
            } else {
                const int u = c - 32;
                const float *g = dext + j * 8;
                if (u < 3) {
                    atomicAdd(g_color + (int64_t)pid * 3 + u, g[u]);
                } else {
                    const float v = a.raydir[(int64_t)ray * 3 + u - 3];
                    atomicAdd(g_dir + (int64_t)pid * 3 + u - 3, g[u] + g[6] * v);
                }
            }
        }
    }
}

// ---- partials -> flat gradient ---------------------------------------------------------------

struct RedSeg {
    const float *part;
    int32_t splits, M, N, n_in, bias_col, ldw;
    float *dst_w, *dst_b;
};
constexpr int MAX_RED = 16;
struct RedArgs {
    RedSeg s[MAX_RED];
    int64_t start[MAX_RED + 1];
    int32_t n_seg;
};

__global__ __launch_bounds__(TPB) void k_reduce_partials(RedArgs r) {
    const int64_t t = blockIdx.x * (int64_t)TPB + threadIdx.x;
    if (t >= r.start[r.n_seg]) return;
    int q = 0;
    while (q + 1 < r.n_seg && t >= r.start[q + 1]) ++q;
    const RedSeg &s = r.s[q];
    const int64_t e = t - r.start[q];
    const int m = (int)(e / s.N), c = (int)(e % s.N);
    const int64_t stride = (int64_t)s.M * s.N;
    // four interleaved chains (fixed order: split i into chain i % 4, chains summed pairwise)
    const float *p = s.part + e;
    float v0 = 0.f, v1 = 0.f, v2 = 0.f, v3 = 0.f;
    int i = 0;
    for (; i + 3 < s.splits; i += 4) {
        v0 += p[i * stride];
        v1 += p[(i + 1) * stride];
        v2 += p[(i + 2) * stride];
        v3 += p[(i + 3) * stride];
    }
    if (i < s.splits) v0 += p[i * stride];
    if (i + 1 < s.splits) v1 += p[(i + 1) * stride];
    if (i + 2 < s.splits) v2 += p[(i + 2) * stride];
    const float v = (v0 + v1) + (v2 + v3);
    if (c < s.n_in) s.dst_w[(int64_t)m * s.ldw + c] += v;
    else if (c == s.bias_col) s.dst_b[m] += v;
}

// segments with many splits and few outputs (k_row_head's [ROW_HEAD_BLOCKS][257]): one workgroup per
// output, thread i sums splits i, i + TPB, .. in order, then a fixed LDS tree (deterministic); one
// thread per output walked the splits serially (128 us for 1024 splits)
constexpr int WIDE_SPLITS = 512;
__global__ __launch_bounds__(TPB) void k_reduce_wide(RedSeg s) {
    __shared__ float red[TPB];
    const int64_t e = blockIdx.x;
    const int m = (int)(e / s.N), c = (int)(e % s.N);
    const int64_t stride = (int64_t)s.M * s.N;
    float v = 0.f;
    for (int i = threadIdx.x; i < s.splits; i += TPB) v += s.part[e + i * stride];
    red[threadIdx.x] = v;
    __syncthreads();
#pragma unroll
    for (int o = TPB / 2; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        if (c < s.n_in) s.dst_w[(int64_t)m * s.ldw + c] += red[0];
        else if (c == s.bias_col) s.dst_b[m] += red[0];
    }
}

}  // namespace tx
}  // namespace
}  // namespace sgn

namespace {
// rows mode: column block 128 wide unless 96 covers N with less padding (one workgroup per CU); k-steps
// of 16 as instantiated (8, 16 or 18)
void rows_shape(int N, int K, bool &w96, int &ks, int &nb) {
    w96 = ((N + 95) / 96) * 96 < ((N + 127) / 128) * 128;
    nb = (N + (w96 ? 96 : 128) - 1) / (w96 ? 96 : 128);
    const int k16 = (K + 15) / 16;
    ks = k16 <= 8 ? 8 : k16 <= 16 ? 16 : 18;
}
}  // namespace

extern "C" {

size_t sgn_x3_gemm_bpack_bytes(const sgn_x3_gemm_args *g) {
    if (!g || g->mode != 0 || g->N <= 0 || g->K < 0 || g->K > 288) return 0;
    bool w96;
    int ks, nb;
    rows_shape(g->N, g->K, w96, ks, nb);
    return (size_t)nb * ks * (w96 ? 3 : 4) * 2 * sgn::tx::FRAG;
}

int sgn_x3_gemm(const sgn_x3_gemm_args *ga, sgn_stream_t stream) {
    using namespace sgn;
    using namespace sgn::tx;
    SGN_REQUIRE(ga, "null argument");
    const sgn_x3_gemm_args &g = *ga;
    SGN_REQUIRE(g.mode == 0 || g.mode == 1, "mode: 0 rows, 1 split-K partials");
    SGN_REQUIRE(g.M >= 0 && g.N > 0 && g.K >= 0, "bad extents");
    SGN_REQUIRE(g.a.p && g.b.p, "null operand");
    auto conv = [](const sgn_x3_operand &o, int dyn, int nrows, Opnd &d) -> int {
        if ((o.csplit < o.ncols) && (!o.p2 || o.csplit % 8 != 0)) return -1;
        if (o.amax && o.shift) return -1;
        d.p = o.p; d.p2 = o.p2; d.ld = o.ld; d.ld2 = o.ld2;
        d.csplit = o.csplit < o.ncols ? o.csplit : 0x7fffffff;
        d.ncols = o.ncols; d.ones_col = o.ones_col; d.act = o.act; d.kmajor = o.kmajor;
        d.nrows = nrows; d.dyn = dyn; d.amax = o.amax; d.shift = o.shift;
        const bool al1 = ((uintptr_t)o.p & 15) == 0 && o.ld % 4 == 0;
        const bool al2 = !o.p2 || (((uintptr_t)o.p2 & 15) == 0 && o.ld2 % 4 == 0);
        d.vec = al1 && al2;
        return 0;
    };
    GemmK k{};
    // the data rows: mode 0 = A's rows (M, device count); mode 1 = the reduction (K, device count)
    SGN_REQUIRE(conv(g.a, 1, g.mode == 0 ? g.M : g.K, k.A) == 0, "operand a: bad column split or scale source");
    SGN_REQUIRE(conv(g.b, g.mode == 1, g.mode == 0 ? (g.b.kmajor ? g.K : g.N) : g.K, k.B) == 0,
                "operand b: bad column split or scale source");
    if (g.mode == 0) {
        SGN_REQUIRE(!g.a.kmajor, "mode 0: operand a is row-major [rows][K]");
        SGN_REQUIRE(g.out && g.out_cols > 0 && (g.out_cols >= g.N || g.out2), "mode 0: out (and out2 past out_cols)");
        // B's "rows": kmajor 0 -> its i = n < N; kmajor 1 -> its k < K
        k.B.nrows = g.b.kmajor ? g.K : g.N;
    } else {
        SGN_REQUIRE(g.a.kmajor && g.b.kmajor, "mode 1: both operands [rows][...] (kmajor)");
        SGN_REQUIRE(k.A.vec && k.B.vec && (g.a.csplit >= g.a.ncols || g.a.csplit % 4 == 0) &&
                        (g.b.csplit >= g.b.ncols || g.b.csplit % 4 == 0),
                    "mode 1: 16-B aligned rows (ld % 4 == 0) and column splits at a multiple of 4");
        SGN_REQUIRE(g.part && g.splits >= 1 && g.splits <= 4096, "mode 1: partials and 1..4096 splits");
    }
    k.M = g.M; k.N = g.N; k.K = g.K;
    k.d_rows = g.d_rows;
    k.bias = g.bias; k.act = g.act; k.mask = g.mask; k.ldm = g.ldm;
    k.out = g.out; k.ldo = g.ldo; k.out_cols = g.out_cols < g.N ? g.out_cols : g.N;
    k.out2 = g.out2; k.ldo2 = g.ldo2; k.amax_out = g.amax_out; k.amax_out2 = g.amax_out2;
    k.part = g.part;
    SGN_REQUIRE(g.products == 0 || g.products == 1 || g.products == 3, "products: 3 (0) or 1");
    const bool p1 = g.products == 1;
    hipStream_t st = as_stream(stream);
    if (g.mode == 0) {
        if (g.M == 0) return 0;
        SGN_REQUIRE(g.K <= 288, "mode 0: K <= 288 (the weight block lives in LDS)");
        SGN_REQUIRE(k.A.vec && g.a.ncols % 8 == 0 && g.a.ones_col < 0 && (g.a.csplit >= g.a.ncols || g.a.csplit % 16 == 0),
                    "mode 0: operand a needs 16-B aligned rows (ld % 4 == 0), ncols % 8 == 0, a column split at a multiple "
                    "of 16, no ones column");
        bool w96;
        int ks, nb;
        rows_shape(g.N, g.K, w96, ks, nb);
        const int tiles = (g.M + RT_ROWS - 1) / RT_ROWS;
        int gy = 256 / nb;
        gy = gy < 1 ? 1 : gy > tiles ? tiles : gy;
        k.splits = gy;
        const dim3 grid(nb * gy);
        if (p1) SGN_REQUIRE(!w96 && ks != 16, "products 1: the colour layers' shapes (K <= 128 or 272..288, N > 96)");
        if (g.bpack) {
            SGN_REQUIRE(((uintptr_t)g.bpack & 15) == 0, "bpack: 16-B aligned");
            k.bpack = (char *)g.bpack;
        }
        // (KS, WN, P1): the weight conversion (with a workspace) then the row tiles
        const bool hasp2 = g.a.p2 && g.a.csplit < g.a.ncols, o2 = g.out2 != nullptr, act = g.a.act != 0;
        if (p1) SGN_REQUIRE(!hasp2 && !o2 && !act, "products 1: one-source operand a without activation, no out2");
        // 32-bit buffer offsets: every rows-mode operand / output below 2 GiB
        auto fits = [&](int64_t ld, int64_t cols) { return (int64_t)g.M * ld * 4 + cols * 4 < 0x7fffffff; };
        SGN_REQUIRE(fits(g.a.ld, 0) && (!hasp2 || fits(g.a.ld2, 0)) && fits(g.ldo, 0) && (!g.mask || fits(g.ldm, 0)) &&
                        (!o2 || fits(g.ldo2, 0)),
                    "mode 0: operands and outputs must stay below 2 GiB");
        auto launch = [&](auto ks_c, auto wn_c, auto p1_c) {
            constexpr int KS = decltype(ks_c)::value, WN = decltype(wn_c)::value;
            constexpr bool P1 = decltype(p1_c)::value;
            if (k.bpack) {
                const int nf = nb * KS * WN * 64;
                hipLaunchKernelGGL((k_x3bpack<KS, WN, P1>), dim3((nf + TPB - 1) / TPB), dim3(TPB), 0, st, k);
            }
            if constexpr (P1) {
                hipLaunchKernelGGL((k_x3rows<KS, WN, P1, false, false, false>), grid, dim3(RT_TPB), 0, st, k);
            } else {
                auto go = [&](auto hc, auto ac, auto oc) {
                    hipLaunchKernelGGL((k_x3rows<KS, WN, P1, decltype(hc)::value, decltype(ac)::value, decltype(oc)::value>),
                                       grid, dim3(RT_TPB), 0, st, k);
                };
                using T = std::true_type;
                using F = std::false_type;
                if (hasp2) {
                    if (act) o2 ? go(T{}, T{}, T{}) : go(T{}, T{}, F{});
                    else o2 ? go(T{}, F{}, T{}) : go(T{}, F{}, F{});
                } else {
                    if (act) o2 ? go(F{}, T{}, T{}) : go(F{}, T{}, F{});
                    else o2 ? go(F{}, F{}, T{}) : go(F{}, F{}, F{});
                }
            }
        };
        using I8 = std::integral_constant<int, 8>;
        using I16 = std::integral_constant<int, 16>;
        using I18 = std::integral_constant<int, 18>;
        using W3 = std::integral_constant<int, 3>;
        using W4 = std::integral_constant<int, 4>;
        if (p1) {
            if (ks <= 8) launch(I8{}, W4{}, std::true_type{});
            else launch(I18{}, W4{}, std::true_type{});
        } else if (ks <= 8) {
            if (w96) launch(I8{}, W3{}, std::false_type{});
            else launch(I8{}, W4{}, std::false_type{});
        } else if (ks <= 16) {
            if (w96) launch(I16{}, W3{}, std::false_type{});
            else launch(I16{}, W4{}, std::false_type{});
        } else {
            if (w96) launch(I18{}, W3{}, std::false_type{});
            else launch(I18{}, W4{}, std::false_type{});
        }
    } else {
        // M block 256 (or 128 for M <= 128); N block 96, 160 (M <= 128: the colour layers' 129
        // columns in one block) or 32 (narrow N)
        const int BM = g.M > 128 ? 256 : 128;
        const int BN = g.N <= 32 ? 32 : (BM == 128 && g.N <= 160) ? 160 : 96;
        const int nbm = (g.M + BM - 1) / BM, nbn = (g.N + BN - 1) / BN;
        k.splits = g.splits;
        const dim3 grid(nbm * nbn * g.splits);
        if (p1) {
            SGN_REQUIRE(BM == 128 && (BN == 160 || BN == 96), "products 1: the colour layers' shapes (M <= 128, N > 32)");
            if (BN == 160) hipLaunchKernelGGL((k_x3tn<1, 5, true>), grid, dim3(TPB), 0, st, k);
            else hipLaunchKernelGGL((k_x3tn<1, 3, true>), grid, dim3(TPB), 0, st, k);
        } else if (BM == 256 && BN == 96 && g.M == 256 && !g.a.p2 && g.a.ones_col < 0 && !g.a.act && g.a.ncols >= 256 &&
                   g.a.ld >= 256) {
            // the row layers' weight gradients
            if (g.b.act) hipLaunchKernelGGL(k_x3dw<true>, grid, dim3(DW_TPB), 0, st, k);
            else hipLaunchKernelGGL(k_x3dw<false>, grid, dim3(DW_TPB), 0, st, k);
        } else if (BM == 256 && BN == 96) hipLaunchKernelGGL((k_x3tn<2, 3>), grid, dim3(TPB), 0, st, k);
        else if (BM == 256) hipLaunchKernelGGL((k_x3tn<2, 1>), grid, dim3(TPB), 0, st, k);
        else if (BN == 160) hipLaunchKernelGGL((k_x3tn<1, 5>), grid, dim3(TPB), 0, st, k);
        else if (BN == 96) hipLaunchKernelGGL((k_x3tn<1, 3>), grid, dim3(TPB), 0, st, k);
        else hipLaunchKernelGGL((k_x3tn<1, 1>), grid, dim3(TPB), 0, st, k);
    }
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

int sgn_train_lists(const int32_t *d_counters, const int32_t *d_samp_nnb, int64_t s_cap, int32_t *d_work,
                    int32_t *d_row_off, float *d_feat, int32_t *d_counts, void *d_ws, sgn_stream_t stream) {
    using namespace sgn;
    using namespace sgn::tx;
    SGN_REQUIRE(d_counters && d_samp_nnb && d_work && d_row_off && d_feat && d_counts && d_ws, "null argument");
    SGN_REQUIRE(s_cap >= 1 && s_cap < (1 << 30), "s_cap out of range");
    const int nb = (int)((s_cap + LIST_PER_BLOCK - 1) / LIST_PER_BLOCK);
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(k_lists_count, dim3(nb), dim3(TPB), 0, st, d_counters, d_samp_nnb, (int2 *)d_ws);
    hipLaunchKernelGGL(k_lists_write, dim3(nb), dim3(TPB), 0, st, d_counters, d_samp_nnb, (const int2 *)d_ws, d_work,
                       d_row_off, (float4 *)d_feat, d_counts);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

size_t sgn_train_lists_workspace_bytes(int64_t s_cap) {
    return (size_t)((s_cap + sgn::tx::LIST_PER_BLOCK - 1) / sgn::tx::LIST_PER_BLOCK + 1) * 8;
}

namespace {
sgn::tx::RowArgs row_args(const sgn_point_tables *pt, const sgn_query_out *q, int32_t K, const int32_t *row_off,
                          const int32_t *counts) {
    sgn::tx::RowArgs a{};
    a.xyz = pt->xyz; a.emb = pt->embedding; a.color = pt->color; a.dir = pt->dir; a.conf = pt->conf;
    a.campos = pt->campos; a.rot = pt->camrotc2w; a.raydir = pt->raydir;
    a.counters = q->counters; a.work = q->work; a.samp_ray = q->samp_ray; a.samp_nnb = q->samp_nnb; a.pidx = q->pidx;
    a.samp_locw = q->samp_locw; a.row_off = row_off; a.tl = counts; a.K = K;
    return a;
}
// one wave per work item, grid-stride: 16 waves per CU (4096 x 4) keep enough items' dependent load chains
// in flight (1024 workgroups: k_row_inputs 153 -> 138 us, k_row_tail 88 -> 61 us per config-5 step)
constexpr int ROW_GRID = 4096;
}  // namespace

int sgn_train_row_inputs(const sgn_point_tables *pt, const sgn_query_out *q, int32_t K, const int32_t *d_row_off,
                         const int32_t *d_counts, float *d_x0, float *d_ext, float *d_rw, float *d_vpe,
                         sgn_stream_t stream) {
    using namespace sgn;
    using namespace sgn::tx;
    SGN_REQUIRE(pt && q && d_row_off && d_counts && d_x0 && d_ext && d_rw && d_vpe, "null argument");
    SGN_REQUIRE(K >= 1 && K <= 8, "K = 1 .. 8");
    SGN_REQUIRE(pt->campos && pt->camrotc2w && pt->raydir && !pt->pers, "camera required, no precomputed pers");
    SGN_REQUIRE(((uintptr_t)d_x0 & 15) == 0 && ((uintptr_t)d_rw & 7) == 0, "aligned x0 / rw required");
    const RowArgs a = row_args(pt, q, K, d_row_off, d_counts);
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(k_row_inputs, dim3(ROW_GRID), dim3(TPB), 0, st, a, d_x0, d_ext, (float2 *)d_rw, d_vpe);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

int sgn_train_row_gather(const sgn_query_out *q, int32_t K, const int32_t *d_row_off, const int32_t *d_counts,
                         const float *d_src, int32_t dim, float *d_dst, sgn_stream_t stream) {
    using namespace sgn;
    using namespace sgn::tx;
    SGN_REQUIRE(q && d_row_off && d_counts && d_src && d_dst, "null argument");
    SGN_REQUIRE(K >= 1 && K <= 8, "K = 1 .. 8");
    SGN_REQUIRE(dim > 0 && dim % 4 == 0 && ((uintptr_t)d_src & 15) == 0 && ((uintptr_t)d_dst & 15) == 0,
                "dim % 4 == 0 and 16-B aligned tables");
    RowArgs a{};
    a.work = q->work; a.samp_nnb = q->samp_nnb; a.pidx = q->pidx; a.row_off = d_row_off; a.tl = d_counts; a.K = K;
    hipLaunchKernelGGL(k_row_gather, dim3(ROW_GRID), dim3(TPB), 0, as_stream(stream), a, d_src, dim, d_dst);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

int sgn_train_colour_head(const sgn_query_out *q, const int32_t *d_counts, const float *d_h3, const float *d_w6,
                          const float *d_b6, float *d_feat, sgn_stream_t stream) {
    using namespace sgn;
    using namespace sgn::tx;
    SGN_REQUIRE(q && d_counts && d_h3 && d_w6 && d_b6 && d_feat, "null argument");
    SGN_REQUIRE(((uintptr_t)d_h3 & 7) == 0, "aligned h3 required");
    RowArgs a{};
    a.work = q->work; a.tl = d_counts;
    hipLaunchKernelGGL(k_colour_head, dim3(ROW_GRID), dim3(TPB), 0, as_stream(stream), a, d_h3, d_w6, d_b6,
                       (float4 *)d_feat);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

size_t sgn_train_head_partial_floats(int32_t which) {
    return which == 0 ? (size_t)sgn::tx::HEAD_BLOCKS * 3 * 129 : (size_t)sgn::tx::ROW_HEAD_BLOCKS * 257;
}

int sgn_train_colour_head_bwd(const sgn_query_out *q, const int32_t *d_counts, const float *d_h3, const float *d_w6,
                              const float *d_b6, const float *d_dfeat, float *d_dy3, uint32_t *d_amax, float *d_part,
                              sgn_stream_t stream) {
    using namespace sgn;
    using namespace sgn::tx;
    SGN_REQUIRE(q && d_counts && d_h3 && d_w6 && d_b6 && d_dfeat && d_dy3 && d_amax && d_part, "null argument");
    RowArgs a{};
    a.work = q->work; a.tl = d_counts;
    hipLaunchKernelGGL(k_colour_head_bwd, dim3(HEAD_BLOCKS), dim3(TPB), 0, as_stream(stream), a, d_h3, d_w6, d_b6,
                       (const float4 *)d_dfeat, d_dy3, d_amax, d_part);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

int sgn_train_row_head(const sgn_point_tables *pt, const sgn_query_out *q, int32_t K, const int32_t *d_row_off,
                       const int32_t *d_counts, float *d_z4_delta4, const float *d_dfs, const float *d_dfeat,
                       const float *d_rw, const float *d_wa, const float *d_ba, float *d_gconf, uint32_t *d_amax,
                       float *d_part, sgn_stream_t stream) {
    using namespace sgn;
    using namespace sgn::tx;
    SGN_REQUIRE(pt && q && d_row_off && d_counts && d_z4_delta4 && d_dfs && d_dfeat && d_rw && d_wa && d_ba && d_gconf &&
                    d_amax && d_part,
                "null argument");
    SGN_REQUIRE(K >= 1 && K <= 8, "K = 1 .. 8");
    const RowArgs a = row_args(pt, q, K, d_row_off, d_counts);
    hipLaunchKernelGGL(k_row_head, dim3(ROW_HEAD_BLOCKS), dim3(TPB), 0, as_stream(stream), a, d_z4_delta4, d_dfs,
                       (const float4 *)d_dfeat, (const float2 *)d_rw, d_wa, d_ba, d_gconf, d_amax, d_part);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

int sgn_train_row_tail(const sgn_point_tables *pt, const sgn_query_out *q, int32_t K, const int32_t *d_row_off,
                       const int32_t *d_counts, const float *d_dx0, const float *d_dext, const sgn_point_grads *grads,
                       sgn_stream_t stream) {
    using namespace sgn;
    using namespace sgn::tx;
    SGN_REQUIRE(pt && q && d_row_off && d_counts && d_dx0 && d_dext && grads, "null argument");
    SGN_REQUIRE(grads->embedding && grads->color && grads->dir, "null gradient outputs");
    SGN_REQUIRE(K >= 1 && K <= 8, "K = 1 .. 8");
    const RowArgs a = row_args(pt, q, K, d_row_off, d_counts);
    hipLaunchKernelGGL(k_row_tail, dim3(ROW_GRID), dim3(TPB), 0, as_stream(stream), a, d_dx0, d_dext, grads->embedding,
                       grads->color, grads->dir);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

int sgn_reduce_partials(int32_t n_seg, const sgn_partial_segment *segs, sgn_stream_t stream) {
    using namespace sgn;
    using namespace sgn::tx;
    SGN_REQUIRE(segs && n_seg >= 1 && n_seg <= MAX_RED, "1..16 segments");
    RedArgs r{};
    r.n_seg = 0;
    r.start[0] = 0;
    for (int i = 0; i < n_seg; ++i) {
        const sgn_partial_segment &s = segs[i];
        SGN_REQUIRE(s.part && s.splits >= 1 && s.M >= 1 && s.N >= 1 && s.dst_w, "bad segment");
        SGN_REQUIRE(s.n_in <= s.N && (s.bias_col < 0 || (s.bias_col < s.N && s.dst_b)), "bad segment columns");
        const RedSeg g{s.part, s.splits, s.M, s.N, s.n_in, s.bias_col, s.ldw, s.dst_w, s.dst_b};
        if (s.splits >= WIDE_SPLITS && (int64_t)s.M * s.N <= 4096) {
            hipLaunchKernelGGL(k_reduce_wide, dim3((unsigned)(s.M * s.N)), dim3(TPB), 0, as_stream(stream), g);
            SGN_CHECK_HIP(hipGetLastError());
            continue;
        }
        r.s[r.n_seg] = g;
        r.start[r.n_seg + 1] = r.start[r.n_seg] + (int64_t)s.M * s.N;
        ++r.n_seg;
    }
    if (r.n_seg == 0) return 0;
    const int64_t blocks = (r.start[r.n_seg] + TPB - 1) / TPB;
    hipLaunchKernelGGL(k_reduce_partials, dim3((unsigned)blocks), dim3(TPB), 0, as_stream(stream), r);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

}  // extern "C"
