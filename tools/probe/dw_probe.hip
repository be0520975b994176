// dw_f16.hip -- the f16 training step's row-layer weight gradients on a hand-written kernel.
//
// The reference differentiates the aggregator's row MLP with torch autograd (PointAggregator.forward,
// models/aggregators/point_aggregators.py:868-959, from optimize_parameters,
// models/base_rendering_model.py:534-664): dW_l = delta_l^T x_l over every (sample, neighbour) row.
// In the f16 step (train_hip.HipTrainer, precision "f16") k_agg_bwd leaves delta_l and x_l as fp16
// rows; this kernel forms dW_l as fixed-order split-K partials (fp32 accumulation of the exact fp16
// products) that sgn_grad_accumulate sums, unscales and unpermutes into the flat gradient.
//
// k_f16dw: part[s][m][n] = sum over the rows r of run s of d[r][m] x[r][n], m < 256, n < ncols.  A
// workgroup (8 waves) owns one run and one 128-column block of x: the run's raw fp16 rows of d (all
// 256 columns) and of x's block stream into a 4-slot LDS ring by LDS-DMA three 32-row stages ahead
// (rows past the run land as zeros through the buffer range check); every wave reads its MFMA
// fragments straight from the raw stage with ds_read_b64_tr_b16 (the transposed read gives each lane 4
// consecutive rows of one column: the k-contiguous operand of v_mfma_f32_32x32x16_f16 without any
// register transpose or conversion).  The 16-B chunks of a row sit XOR-swizzled by 4 (row & 3) --
// chosen through the DMA's per-lane global offsets -- so the four rows of a transposed read fall in
// four different 16-bank windows (conflict-free).  Wave w owns rows 32 w .. + 31 of m and the block's
// four 32-column tiles: 8 MFMAs per stage.
#include "agg_device.h"

namespace sgn {
namespace {
namespace f16dw {

constexpr int ROWS = 32, BN = 128, NST = 4, NW = 8, TPB = 64 * NW;
constexpr int ABYTES = ROWS * 512;     // 16 KiB: 32 rows x 256 fp16
constexpr int BBYTES = ROWS * BN * 2;  // 8 KiB: 32 rows x 128 fp16
constexpr int STAGE = ABYTES + BBYTES;
constexpr uint32_t OOB = 0x80000000u;

typedef short s4 __attribute__((ext_vector_type(4)));

struct Args {
    const char *d, *x;
    uint32_t ldd2, ldx2;   // row strides in bytes
    int32_t ncols, n_rows, splits;
    float *part;
};

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char *ldsdst, uint32_t voff, uint32_t soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void *)ldsdst, 16, voff, soff, 0, 0);
}

__device__ __forceinline__ s4 tr4(const char *p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4 *)p);
}

// this wave's DMAs but the last N landed, then the workgroup barrier (every wave's have, after it); the
// memory clobber keeps the compiler's LDS reads after it
template <int N>
__device__ __forceinline__ void wait_barrier() {
    static_assert(N == 6 || N == 3 || N == 0, "");
    if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)\n\ts_barrier" ::: "memory");
    else if constexpr (N == 3) asm volatile("s_waitcnt vmcnt(3)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
}

// 1-D block id -> (column block, run): the column blocks of a run on one XCD (blocks b and b + 8 share
// it), so the run's d rows are read from HBM once and hit that XCD's L2 for the other blocks
__device__ __forceinline__ void xcd_block(int nblk, int splits, int &blk, int &split) {
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

__global__ __launch_bounds__(TPB, 1) void k_f16dw(Args g) {
    __shared__ __attribute__((aligned(16))) char lds[NST * STAGE];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nb = (g.ncols + BN - 1) / BN;
    int blk, split;
    xcd_block(nb, g.splits, blk, split);
    const int n0 = blk * BN;
    const int per = ((g.n_rows + g.splits - 1) / g.splits + ROWS - 1) / ROWS * ROWS;
    const int r0 = split * per, r1 = min(g.n_rows, r0 + per);
    const int nst = r1 > r0 ? (r1 - r0 + ROWS - 1) / ROWS : 0;
    auto rsrc = [](const char *p, int64_t bytes) {
        bytes = bytes < 0 ? 0 : bytes > 0x7fffffff ? 0x7fffffff : bytes;
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(p), (short)0, (int)bytes, 0x00020000);
    };
    const __amdgpu_buffer_rsrc_t ra = rsrc(g.d, (int64_t)r1 * g.ldd2), rb = rsrc(g.x, (int64_t)r1 * g.ldx2);
    // DMA per-lane global offsets relative to the stage's first row (the stage adds a uniform soffset).
    // d: wave w's instruction e fills stage rows 4 w + 2 e + (lane >> 5), LDS chunk (lane & 31), which holds
    // the row's global chunk (lane & 31) ^ 4 (row & 3).  x: wave w fills stage rows 4 w + (lane >> 4),
    // LDS chunk (lane & 15) <- columns n0 + 8 ((lane & 15) ^ 4 (row & 3)) .. + 7 (past ncols: zeros).
    uint32_t av[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const int row = 4 * w + 2 * e + (lane >> 5);
        av[e] = (uint32_t)row * g.ldd2 + (uint32_t)(((lane & 31) ^ (4 * (row & 3))) * 16);
    }
    uint32_t bv;
    {
        const int row = 4 * w + (lane >> 4);
        const int c = n0 + 8 * ((lane & 15) ^ (4 * (row & 3)));
        bv = c < g.ncols ? (uint32_t)row * g.ldx2 + (uint32_t)c * 2 : OOB;
    }
    auto issue = [&](int st) {   // stage st (rows r0 + 32 st ..) into slot st % 4: 3 instructions per wave
        char *slot = lds + (st % NST) * STAGE;
        const uint32_t rs = (uint32_t)(r0 + ROWS * st);
#pragma unroll
        for (int e = 0; e < 2; ++e) dma16(ra, slot + (4 * w + 2 * e) * 512, av[e], rs * g.ldd2);
        dma16(rb, slot + ABYTES + w * 1024, bv, rs * g.ldx2);
    };
    // transposed-read addresses: lane l (group gq = l >> 4, i = l & 15, q = i >> 2, p = i & 3) supplies row
    // 8 (gq >> 1) + q (+ 16 ks + 4 h) of the stage, columns 16 (gq & 1) + 4 p .. + 3 of its 32-column tile;
    // the row's chunk is XOR-swizzled by 4 q (the row's low bits: 16 ks + 4 h keep them)
    const int gq = lane >> 4, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
    const int trow = 8 * (gq >> 1) + q;
    const int csub = 2 * (gq & 1) + (p >> 1), cbyte = (p & 1) * 8;   // chunk within the tile, byte within it
    const uint32_t aoff = (uint32_t)(trow * 512 + ((4 * w + csub) ^ (4 * q)) * 16 + cbyte);
    uint32_t boff[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) boff[b] = (uint32_t)(ABYTES + trow * 256 + ((4 * b + csub) ^ (4 * q)) * 16 + cbyte);
    f32x16 acc[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[b] = f32x16{};
    for (int st = 0; st < 3 && st < nst; ++st) issue(st);
    // stage st: this wave's DMAs of stage st landed (those of st + 1, st + 2 may stay in flight), every wave's
    // after the barrier, and every wave is done with stage st - 1, whose slot stage st + 3 reuses
    auto stage = [&](int st, auto tailc) {
        constexpr bool TAIL = decltype(tailc)::value;
        if constexpr (!TAIL) {
            wait_barrier<6>();
            issue(st + 3);
        } else {
            if (st + 2 < nst) wait_barrier<6>();
            else if (st + 1 < nst) wait_barrier<3>();
            else wait_barrier<0>();
        }
        const char *slot = lds + (st % NST) * STAGE;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int ro = (16 * ks) * 512, rob = (16 * ks) * 256;
            const s4 a0 = tr4(slot + aoff + ro), a1 = tr4(slot + aoff + ro + 4 * 512);
            const h8 af = __builtin_bit_cast(h8, __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const s4 b0 = tr4(slot + boff[b] + rob), b1 = tr4(slot + boff[b] + rob + 4 * 256);
                const h8 bf = __builtin_bit_cast(h8, __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7));
                acc[b] = mfma32(af, bf, acc[b]);
            }
        }
    };
    int st = 0;
    for (; st + 3 < nst; ++st) stage(st, std::false_type{});
    for (; st < nst; ++st) stage(st, std::true_type{});
    if (w == 0 && blockIdx.x == 0)
        for (int e = 0; e < 16; ++e) g.part[256 * g.ncols * g.splits + lane * 16 + e] = acc[0][e];
    // this run's partial [256][ncols] (columns past ncols dropped by the buffer range, not branched around)
    const int L = lane & 31, hk = lane >> 5;
    const __amdgpu_buffer_rsrc_t pr =
        rsrc((const char *)(g.part + (int64_t)split * 256 * g.ncols), (int64_t)256 * g.ncols * 4);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const int n = n0 + 32 * b + L;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = 32 * w + (r & 3) + 8 * (r >> 2) + 4 * hk;
            const uint32_t off = n < g.ncols ? (uint32_t)((m * g.ncols + n) * 4) : OOB;
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, acc[b][r]), pr, off, 0, 0);
        }
    }
}

}  // namespace f16dw
}  // namespace
}  // namespace sgn

extern "C" {

int probe_f16_weight_grad(const void *d, int64_t ldd, const void *x, int64_t ldx, int32_t ncols, int32_t n_rows,
                        int32_t splits, float *part, sgn_stream_t stream) {
    using namespace sgn;
    SGN_REQUIRE(d && x && part, "null pointer");
    SGN_REQUIRE(ncols > 0 && ncols % 8 == 0 && ldx >= ncols && ldx % 8 == 0 && ldd >= 256 && ldd % 8 == 0,
                "x: ncols % 8 == 0, ldx >= ncols, 16-B aligned rows; d: ldd >= 256");
    SGN_REQUIRE((((uintptr_t)d | (uintptr_t)x) & 15) == 0, "16-B aligned operands");
    SGN_REQUIRE(n_rows >= 0 && splits >= 1 && splits <= 4096, "n_rows >= 0, 1..4096 splits");
    SGN_REQUIRE((int64_t)n_rows * ldd * 2 < 0x7fffffff && (int64_t)n_rows * ldx * 2 < 0x7fffffff,
                "operands below 2 GiB");
    f16dw::Args a;
    a.d = (const char *)d;
    a.x = (const char *)x;
    a.ldd2 = (uint32_t)(ldd * 2);
    a.ldx2 = (uint32_t)(ldx * 2);
    a.ncols = ncols;
    a.n_rows = n_rows;
    a.splits = splits;
    a.part = part;
    const int nb = (ncols + f16dw::BN - 1) / f16dw::BN;
    hipLaunchKernelGGL(f16dw::k_f16dw, dim3(nb * splits), dim3(f16dw::TPB), 0, as_stream(stream), a);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

}  // extern "C"
