// agg_train.hip -- training backward of the fused neural-point aggregator.
//
// Gradients of PointAggregator.forward / viewmlp (models/aggregators/point_aggregators.py:
// 868-959, :561-786) and of the NeuralPoints gather (models/neural_points/neural_points.py:
// 942-988) w.r.t. the per-point parameters (points_embeding, points_color, points_dir,
// points_conf through the straight-through clamp :863-865), given d loss / d f_s (the
// blended 256-d features) and d loss / d alpha_s from the colour MLP + ray march (those
// are per-sample and small; the host differentiates them).
//
// Forward (mlp.hip, k_agg_rows<0, true>) saved per row: block1.0 inputs x0, block1.2
// inputs h1, block3.0 inputs [h2 | ext], block3.2 inputs h3 (fp16, fragment column order).
//
// k_agg_bwd, one wave per 32-row tile (4 samples x 8 neighbours), everything on MFMA
// v_mfma_f32_32x32x16_f16:
//   recompute z4 = W3 h3 + b3 (h4 = LReLU(z4)), the alpha logit za = wa . h4 + ba
//   d za  = w * d alpha_s * sigmoid(za - 1)                     (softplus(za - 1), :298-304)
//   d w   = <h4, d f_s> + alpha * d alpha_s                      (K-blend, :743-770)
//   delta4 = (w d f_s + d za wa) * LReLU'(z4)
//   delta3 = (W3^T delta4) * LReLU'(h3), delta2 = (W2^T delta3)[:256] * LReLU'(h2), ext grads
//   delta1 = (W1^T delta2) * LReLU'(h1), d x0 = W0^T delta1 -> d feat through PE(feat)
// The accumulator of one product is converted in registers into the B operand of the next
// (the k permutation lives in the transposed weight blob, as in the forward).  Weight
// gradients dW_l = delta_l^T x_l are plain GEMMs over the saved [rows][C] tiles (host side,
// hipBLASLt); the deltas are written for them.  Gradients are computed with a loss scale
// (device scalar) so fp16 deltas keep their precision; point gradients leave unscaled.
#include <vector>

#include "agg_device.h"

namespace sgn {
namespace {

using namespace mlp;

// transposed-weight blob: fragment (row tile t, k-step ks) of layer L at OFF_T[L] + (t*16 + ks)*FRAG;
// rows = the layer's input units, k = its output units in chain order (16 k-steps)
constexpr int TT0 = 9, TT1 = 8, TT2 = 9, TT3 = 8;  // row tiles (inputs 288 / 256 / 263 / 256)
constexpr size_t OFF_T3 = 0;
constexpr size_t OFF_T2 = OFF_T3 + (size_t)TT3 * 16 * FRAG;
constexpr size_t OFF_T1 = OFF_T2 + (size_t)TT2 * 16 * FRAG;
constexpr size_t OFF_T0 = OFF_T1 + (size_t)TT1 * 16 * FRAG;
// SG: block2_bpnet.0's first 256 inputs (the block1 output h; the BPNet embedding is not trained)
constexpr int TTB = 8;
constexpr size_t OFF_TB = OFF_T0 + (size_t)TT0 * 16 * FRAG;
constexpr size_t T_BYTES = OFF_TB + (size_t)TTB * 16 * FRAG;

struct BwdArgs {
    AggArgs a;                 // point tables, query, forward blob (gather + W3 recompute)
    const void *tblob;         // transposed weights
    const _Float16 *sh1, *sh2, *sh3;
    const float *dfs;          // [n_items][256] d loss / d f_s (natural unit order)
    const float *dalpha;       // [n_items]      d loss / d alpha_s
    const float *scale;        // device scalar loss scale
    _Float16 *d4, *d3, *d2, *d1;  // [rows][256] scaled deltas, chain column order
    _Float16 *h4;              // [rows][256] block3.2 outputs, chain column order
    float *dza;                // [rows] scaled d alpha-logit
    float *g_emb, *g_color, *g_dir, *g_conf;  // [N,32] [N,3] [N,3] [N] (atomic add, unscaled)
    int32_t n_items;
    const _Float16 *sh2b;      // SG: [rows][256] block2_bpnet inputs h (chain order)
    _Float16 *db;              // SG: [rows][256] scaled block2_bpnet deltas (chain order)
};

// A wave's window onto rows [row0, row0 + 32) of a [rows][C] fp16 tile: the descriptor's range ends
// at the last row of a work item (rows of items past the end read 0 and drop their stores), so the
// epilogues load and store without a branch per fragment (a branch around each load made hipcc wait
// vmcnt(0) per fragment: 8 dependent round trips per product).
struct Tile {
    __amdgpu_buffer_rsrc_t r;
    uint32_t lo;  // lane offset (lane & 31) * C * 2 + (lane >> 5) * 16
    __device__ __forceinline__ h8 load(int s) const {
        return __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(r, lo, s * 32, 0));
    }
    __device__ __forceinline__ void store(int s, h8 v) const {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, lo, s * 32, 0);
    }
};
// buffer descriptor of a wave-uniform range (readfirstlane keeps it in SGPRs: a VGPR descriptor
// is a waterfall loop around every access)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_u(const void *ptr, int bytes) {
    const uint64_t p = (uint64_t)ptr;
    const uint32_t plo = __builtin_amdgcn_readfirstlane((uint32_t)p), phi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)phi << 32) | plo), (short)0,
                                             __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// nrow: rows of this wave's tile that belong to work items (a multiple of 8, wave-uniform)
__device__ __forceinline__ Tile tile_of(const _Float16 *base, int C, int64_t row0, int nrow, int lane) {
    Tile t;
    t.r = rsrc_u(base + row0 * C, nrow * C * 2);
    t.lo = (uint32_t)((lane & 31) * C * 2 + (lane >> 5) * 16);
    return t;
}

// delta (fp32 accumulator registers 8 s2 .. 8 s2 + 7) * LReLU'(h) with h the saved fp16 fragment
__device__ __forceinline__ h8 mask_frag(const f32x16 &acc, int s2, h8 hv) {
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const float d = acc[8 * s2 + e];
        v[e] = (float)hv[e] > 0.f ? d : 0.01f * d;
    }
    return pack8(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]);
}

__device__ __forceinline__ h8 plain_frag(const f32x16 &acc, int s2) {
    const int r = 8 * s2;
    return pack8(acc[r], acc[r + 1], acc[r + 2], acc[r + 3], acc[r + 4], acc[r + 5], acc[r + 6], acc[r + 7]);
}

// The workgroup's 4 waves (one per SIMD) run the same sequence of 12 weight products per tile
// on different rows.  Each product's NT x 16 fragments are staged once per workgroup in LDS by
// LDS-DMA and read there by all four waves; two slots, the next product's DMA in flight while
// the current one multiplies (boundary = counted vmcnt + raw barrier, then issue the next DMA
// into the slot read one product ago).  Read one by one from L2 instead, the MFMAs waited on
// every fragment (one wave per SIMD, ~5 % of the MFMA rate).
constexpr int BWD_TPB = 256;
constexpr int BWD_SLOT = 4 * 16 * (int)FRAG;  // the largest product: 4 tiles x 16 k-steps
constexpr int BWD_LDS = 2 * BWD_SLOT;
// product I: 0-1 block3.2 recompute (W3, tiles 4I..), 2-3 W3^T, 4-5 W2^T, 6 W2^T's input tile 8
// (colour / dir channels), [SG: 7-8 W_B^T], then W1^T (2 products), W0^T (3, 3 row tiles each)
__host__ __device__ constexpr int n_prod(bool sg) { return sg ? 14 : 12; }
__host__ __device__ constexpr int prod_w1(bool sg) { return sg ? 9 : 7; }
__host__ __device__ constexpr int prod_w0(bool sg) { return sg ? 11 : 9; }
__host__ __device__ constexpr int prod_nt(int I, bool sg = false) { return I == 6 ? 1 : I >= prod_w0(sg) ? 3 : 4; }
__host__ __device__ constexpr uint32_t prod_off(int I, int ks, int t, bool sg = false) {
    return (uint32_t)(I < 2 ? OFF_W3 + ((size_t)(I * KS_HID + ks) * 4 + t) * FRAG
                    : I < 4 ? OFF_T3 + ((size_t)((I - 2) * 4 + t) * 16 + ks) * FRAG
                    : I < 6 ? OFF_T2 + ((size_t)((I - 4) * 4 + t) * 16 + ks) * FRAG
                    : I == 6 ? OFF_T2 + ((size_t)(8 + t) * 16 + ks) * FRAG
                    : (sg && I < 9) ? OFF_TB + ((size_t)((I - 7) * 4 + t) * 16 + ks) * FRAG
                    : I < prod_w0(sg) ? OFF_T1 + ((size_t)((I - prod_w1(sg)) * 4 + t) * 16 + ks) * FRAG
                                      : OFF_T0 + ((size_t)((I - prod_w0(sg)) * 3 + t) * 16 + ks) * FRAG);
}

// A product's NT x 16 fragments are contiguous in their blob (prod_off(I, 0, 0) on), W3 k-step-major,
// the transposed layers row-tile-major; the slot mirrors that order, so fragment (ks, t) sits at
// slot index prod_m(I, ks, t) and the DMA piece i of wave w moves index w + 4 i.
template <int I, bool SG = false>
__host__ __device__ constexpr int prod_m(int ks, int t) { return I < 2 ? ks * prod_nt(I, SG) + t : t * 16 + ks; }

template <int I, bool SG = false>
__device__ __forceinline__ void prod_dma(char *lds, const WBlob &wb, const WBlob &tb, int w, int lane) {
    constexpr int NT = prod_nt(I, SG), NF = 16 * NT;
    static_assert(NF % 4 == 0 && NF * (int)FRAG <= BWD_SLOT, "staging slot");
    const WBlob &src = I < 2 ? wb : tb;
    // wo: this wave's first index in bytes, opaque per product, so each piece's LDS address and blob
    // offset are one SALU add here (hoisted out of the tile loop, the pieces' addresses were spilled to
    // VGPR lanes and read back with a readlane and hazard nops each)
    uint32_t wo = (uint32_t)w * (uint32_t)FRAG;
    asm volatile("" : "+s"(wo));
    char *dst = lds + (I & 1) * BWD_SLOT + wo;
    const uint32_t src0 = (uint32_t)prod_off(I, 0, 0, SG) + wo;
#pragma unroll
    for (int i = 0; i < NF / 4; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(src.rsrc, (__attribute__((address_space(3))) void *)(dst + 4 * i * (int)FRAG),
                                                 16, lane * 16, src0 + 4 * i * (uint32_t)FRAG, 0, 0);
}

// LDS: the two weight slots, then one 8 KB region per wave (MR): at a tile's start this wave's
// d f_s rows (4 items x 1 KB, rows MR_DFS apart so the items' lanes read different banks) and its
// copy of block3.2's bias and the alpha weight; from product 2 on, the saved activations whose
// LReLU' masks the current product's epilogue (8 fragments, LDS-DMA'd with the product's weights
// instead of loaded to registers in the epilogue: hipcc waits vmcnt(0) -- the weight DMA in flight
// included -- at every use of a global load while a DMA is outstanding).  One LDS array: a second
// __shared__ object makes hipcc wait vmcnt(0) for the DMA before every LDS read.
constexpr int MRW = 8192;
constexpr int MR_DFS = 1040;
constexpr int MR_F = 4 * MR_DFS;  // b3 [256] fp32, then wa [256]
static_assert(MR_F + 2 * HID * 4 <= MRW, "per-wave region");
constexpr int BWD_LDS_ALL = BWD_LDS + 4 * MRW;  // 160 KB: the CU's whole LDS

// Product boundary: this wave's DMA pieces of product I have landed -- the VM vector-memory
// operations it issued after them (the previous epilogue's stores) may stay in flight, vmcnt
// retires in order -- and its LDS reads are done; then the barrier (every wave's pieces landed,
// every wave done with the slot the next DMA overwrites).  Not __syncthreads(): its fence waits
// vmcnt(0), draining the stores.
template <int VM>
__device__ __forceinline__ void boundary() {
    static_assert(VM >= 0 && VM < 64, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(VM) : "memory");
}

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char *dst, uint32_t voff, uint32_t soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void *)dst, 16, voff, soff, 0, 0);
}

// the 8 saved fragments k0 .. k0 + 7 of this wave's tile -> its region, fragment k0 + i at i KB
__device__ __forceinline__ void mask_dma(char *mr, const Tile &t, int k0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) dma16(t.r, mr + i * 1024, t.lo, (uint32_t)(k0 + i) * 32);
}

// acc[t] (+)= sum_ks W_I(t, ks) * in[ks].  VM: boundary allowance (the stores of product I - 1's
// epilogue); mask: the tile whose fragments k0 .. k0 + 7 product I's epilogue reads from the
// region; `more`: the workgroup has another tile (the last product's successor is the next tile's
// product 0)
template <int I, int NT, bool SG, int VM>
__device__ __forceinline__ void prod_mul(char *lds, const WBlob &wb, const WBlob &tb, const h8 (&in)[16],
                                         f32x16 (&acc)[NT], int w, int lane, bool more,
                                         const Tile *mask = nullptr, int k0 = 0) {
    static_assert(NT == prod_nt(I, SG), "product width");
    boundary<VM>();
    if (mask) mask_dma(lds + BWD_LDS + w * MRW, *mask, k0);
    asm volatile("" ::: "memory");  // the masks' pieces stay older than the weights' (mask_wait counts)
    if constexpr (I + 1 < n_prod(SG)) prod_dma<I + 1, SG>(lds, wb, tb, w, lane);
    else if (more) prod_dma<0, SG>(lds, wb, tb, w, lane);
    asm volatile("" ::: "memory");  // and the epilogue's stores younger than both (boundary counts)
    // opaque per product: hipcc hoisted every fragment's address out of the tile loop into its own
    // VGPR (64 of them); one base VGPR + the read's 16-bit immediate offset instead
    uint32_t voff = (uint32_t)((I & 1) * BWD_SLOT + lane * 16);
    asm volatile("" : "+v"(voff));
    const char *sl = lds + voff;
    // fragment n = ks * NT + t read PF ahead of its MFMA: one read in flight per MFMA left the MFMAs
    // waiting out the LDS latency one by one (the scheduler, short of registers, chose that)
    constexpr int NF = 16 * NT, PF = 4;
    h8 fr[NF];
#pragma unroll
    for (int n = 0; n < PF; ++n) fr[n] = *(const h8 *)(sl + prod_m<I, SG>(n / NT, n % NT) * (int)FRAG);
    // program order pinned (sched_barrier after each pair): the scheduler otherwise regrouped the
    // MFMAs by accumulator -- a dependent chain -- each behind its own read
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int n = 0; n < NF; ++n) {
        if (n + PF < NF) {
            const int m = n + PF;
            fr[m] = *(const h8 *)(sl + prod_m<I, SG>(m / NT, m % NT) * (int)FRAG);
        }
        acc[n % NT] = mfma32(fr[n], in[n / NT], acc[n % NT]);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// acc[t] = sum_ks T[t0 + t][ks] * in[ks] for the NT row tiles of transposed product I
template <int I, int NT, bool SG, int VM>
__device__ __forceinline__ void tmul(char *lds, const WBlob &wb, const WBlob &tb, const h8 (&in)[16],
                                     f32x16 (&acc)[NT], int w, int lane, bool more, const Tile *mask = nullptr,
                                     int k0 = 0) {
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x16{};
    prod_mul<I, NT, SG, VM>(lds, wb, tb, in, acc, w, lane, more, mask, k0);
}

// product I's epilogue reads its masks: the DMA pieces issued after them (product I + 1's
// weights, 4 per row tile) may stay in flight
template <int I, bool SG>
__device__ __forceinline__ void mask_wait() {
    static_assert(I + 1 < n_prod(SG), "a masked product has a successor in the tile");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * prod_nt(I + 1, SG)) : "memory");
}

// d feat[c] contribution of layer-0 local channel C (mlp_layout.h l0 order): PE(feat) chain rule
template <int C>
__device__ __forceinline__ void l0_backward(float d, const float (&feat)[16], float (&df)[16]) {
    if constexpr (C < 16) {
        df[C] += d;
    } else if constexpr (C < 112) {
        constexpr int m = C - 16, dd = m / 6, f = (m % 6) / 2, sc = m % 2;
        float sv, cv;
        sincos_pow2<f>(feat[dd], sv, cv);
        df[dd] += sc ? -d * sv * (float)(1 << f) : d * cv * (float)(1 << f);
    }
    // C >= 112: PE(dists) -> point xyz / sample positions (not trained)
}

// one masked product pair's epilogue: delta = acc * LReLU'(saved), kept for the next product and stored
template <int P>
__device__ __forceinline__ void masked_epilogue(const char *lds, int w, const f32x16 (&ac)[4], h8 (&out)[16],
                                                const Tile &dst, int lane) {
    uint32_t voff = (uint32_t)(BWD_LDS + w * MRW + lane * 16);
    asm volatile("" : "+v"(voff));
    const char *mr = lds + voff;
#pragma unroll
    for (int tt = 0; tt < 4; ++tt)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
            const int i = 2 * tt + s2, k = 8 * P + i;
            out[k] = mask_frag(ac[tt], s2, *(const h8 *)(mr + i * 1024));
            dst.store(k, out[k]);
        }
}

template <bool SG>
__global__ __launch_bounds__(BWD_TPB) void k_agg_bwd(BwdArgs b) {
    constexpr int IW1 = prod_w1(SG), IW0 = prod_w0(SG);
    __shared__ __attribute__((aligned(16))) char lds[BWD_LDS_ALL];
    const AggArgs &a = b.a;
    const int lane = threadIdx.x & 63;
    const int h = lane >> 5, j = lane & 31, q = j >> 3;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    char *mr = lds + BWD_LDS + w * MRW;
    const Cam cam = load_cam(a.campos, a.rot);
    const WBlob wb = make_blob(a.blob, a.blob_bytes);
    const WBlob tb = make_blob(b.tblob, T_BYTES);
    const float ba = ((const float *)((const char *)a.blob + OFF_F32))[F_BA];
    const float scale = *b.scale, inv = 1.f / scale;
    const int end = b.n_items;
    if (blockIdx.x * 16 < end) prod_dma<0, SG>(lds, wb, tb, w, lane);  // stream prologue
    // trip count uniform over the workgroup (its waves meet at the staging barriers); rows past
    // the end are masked (ok = false) and out of the tiles' range
    for (int bbase = blockIdx.x * 16; bbase < end; bbase += gridDim.x * 16) {
        const int base = bbase + w * 4;
        const bool more = bbase + (int)gridDim.x * 16 < end;
        const int item = base + q;
        const int64_t row0 = (int64_t)base * 8;
        const int nrow = min(max(end - base, 0), 4) * 8;
        // this wave's d f_s rows and the fp32 constants -> its region (landed at product 0's boundary;
        // the region's last readers, the previous tile's block1.2 epilogue, are past 3 boundaries)
        {
            const __amdgpu_buffer_rsrc_t rd = rsrc_u(b.dfs + (int64_t)base * HID, nrow / 8 * HID * 4);
#pragma unroll
            for (int i = 0; i < 4; ++i) dma16(rd, mr + i * MR_DFS, lane * 16, i * HID * 4);
            dma16(wb.rsrc, mr + MR_F, lane * 16, (uint32_t)(OFF_F32 + F_B3 * 4));
            dma16(wb.rsrc, mr + MR_F + HID * 4, lane * 16, (uint32_t)(OFF_F32 + F_WA * 4));
        }
        float feat[16], dist[3];
        h8 ext;
        const RowIdx ix = row_index(a, item, end, lane);
        const RowIn ri = gather_row(a, cam, ix, lane, feat, dist, ext);
        const bool ok = ri.sval;
        const int it = ok ? item : 0;
        // this row's ray direction (the dir gradient of product 6), loaded with the gather
        const float vr[3] = {a.raydir[(int64_t)ix.ray * 3], a.raydir[(int64_t)ix.ray * 3 + 1],
                             a.raydir[(int64_t)ix.ray * 3 + 2]};
        const float dal = b.dalpha[it];
        const Tile t3 = tile_of(b.sh3, 256, row0, nrow, lane);
        // ---- recompute block3.2: z4 = W3 h3 + b3 ------------------------------------------
        f32x16 acc[8];
        {
            h8 x3[16];
#pragma unroll
            for (int s = 0; s < 16; ++s) x3[s] = t3.load(s);
#pragma unroll
            for (int t = 0; t < 8; ++t) acc[t] = f32x16{};
            prod_mul<0, 4, SG, 0>(lds, wb, tb, x3, *(f32x16(*)[4])&acc[0], w, lane, more);
            prod_mul<1, 4, SG, 0>(lds, wb, tb, x3, *(f32x16(*)[4])&acc[4], w, lane, more);
        }
        // ---- pass 1: h4, alpha logit, <h4, d f_s> ------------------------------------------
        const float *dfl = (const float *)(mr + q * MR_DFS);
        const float *Fb3 = (const float *)(mr + MR_F), *Fwa = Fb3 + HID;
        float za = 0.f, dwv = 0.f;
#pragma unroll
        for (int t = 0; t < 8; ++t)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int u0 = 32 * t + 8 * g + 4 * h;
                const f32x4 df4 = *(const f32x4 *)(dfl + u0);
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const int r = 4 * g + c, u = u0 + c;
                    const float z = acc[t][r] + Fb3[u];
                    const float hv = z > 0.f ? z : 0.01f * z;
                    acc[t][r] = hv;
                    za = fmaf(Fwa[u], hv, za);
                    dwv = fmaf(hv, df4[c], dwv);
                }
            }
        za += __shfl_xor(za, 32) + ba;
        dwv = (dwv + __shfl_xor(dwv, 32)) * scale;
        const float x1 = za - 1.f;
        const float alpha_row = softplus(x1);
        const float sig = 1.f / (1.f + expf(-x1));
        const float das = ok ? dal * scale : 0.f;
        const float wgt = ri.wgt;  // 0 for masked neighbours and padding rows
        const float dz = wgt * das * sig;
        const float dwgt = dwv + alpha_row * das;  // scaled d loss / d (weight * conf) of this row
        // ---- pass 2: delta4 = (w d f_s + dz wa) * LReLU'(z4); save h4 / delta4 (33 stores) ----
        h8 dl[16];
        {
            const Tile th4 = tile_of(b.h4, 256, row0, nrow, lane), td4 = tile_of(b.d4, 256, row0, nrow, lane);
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                f32x16 dv;
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int u0 = 32 * t + 8 * g + 4 * h;
                    const f32x4 df4 = *(const f32x4 *)(dfl + u0);
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        const int r = 4 * g + c, u = u0 + c;
                        const float hv = acc[t][r];
                        const float d = fmaf(wgt * scale, df4[c], dz * Fwa[u]);
                        dv[r] = hv > 0.f ? d : 0.01f * d;
                    }
                }
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    dl[2 * t + s2] = plain_frag(dv, s2);
                    th4.store(2 * t + s2, plain_frag(acc[t], s2));
                    td4.store(2 * t + s2, dl[2 * t + s2]);
                }
            }
            // lane-half 1 stores out of range (dropped): one store instruction either way
            const __amdgpu_buffer_rsrc_t rz = rsrc_u(b.dza + row0, nrow * 4);
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, dz), rz, h ? 0x40000000u : j * 4u, 0, 0);
        }
        // ---- block3.2 backward: delta3 = (W3^T delta4) * LReLU'(h3) ----------------------
        h8 dn[16];
        {
            const Tile td3 = tile_of(b.d3, 256, row0, nrow, lane);
            f32x16 ac[4];
            tmul<2, 4, SG, 33>(lds, wb, tb, dl, ac, w, lane, more, &t3, 0);
            mask_wait<2, SG>();
            masked_epilogue<0>(lds, w, ac, dn, td3, lane);
            tmul<3, 4, SG, 8>(lds, wb, tb, dl, ac, w, lane, more, &t3, 8);
            mask_wait<3, SG>();
            masked_epilogue<1>(lds, w, ac, dn, td3, lane);
        }
        // ---- block3.0 backward: delta2 = (W2^T delta3)[:256] * LReLU'(h2); ext grads -------
        // (SG: h2 is the block2_bpnet output, so this is block2_bpnet's delta, saved to db)
        {
            const Tile t2 = tile_of(b.sh2, KS_L2 * 16, row0, nrow, lane);
            const Tile td2 = tile_of(SG ? b.db : b.d2, 256, row0, nrow, lane);
            f32x16 ac[4];
            tmul<4, 4, SG, 8>(lds, wb, tb, dn, ac, w, lane, more, &t2, 0);
            mask_wait<4, SG>();
            masked_epilogue<0>(lds, w, ac, dl, td2, lane);
            tmul<5, 4, SG, 8>(lds, wb, tb, dn, ac, w, lane, more, &t2, 8);
            mask_wait<5, SG>();
            masked_epilogue<1>(lds, w, ac, dl, td2, lane);
        }
        {
            f32x16 ae[1];
            tmul<6, 1, SG, 8>(lds, wb, tb, dn, ae, w, lane, more);
            // tile 8 = inputs 256..262: half 0 regs 0..3 -> colour 0..2, (dir - v)_0;
            // half 1 regs 0..2 -> (dir - v)_1, (dir - v)_2, <dir, v>   (:639-652)
            const float o0 = __shfl_xor(ae[0][0], 32), o1 = __shfl_xor(ae[0][1], 32), o2 = __shfl_xor(ae[0][2], 32);
            if (ok && ri.pid >= 0 && h == 0) {
                const float ddiff[3] = {ae[0][3], o0, o1};
                const int64_t pb = (int64_t)ri.pid * 3;
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    atomicAdd(b.g_color + pb + c, ae[0][c] * inv);
                    atomicAdd(b.g_dir + pb + c, fmaf(o2, vr[c], ddiff[c]) * inv);
                }
                atomicAdd(b.g_conf + ri.pid, dwgt * ri.wn * inv);  // straight-through clamp (:863-865)
            }
        }
        // (the atomics are conditional: the next boundary drains vmcnt)
        // ---- SG block2_bpnet backward: delta2 = (W_B[:, :256]^T delta_B) * LReLU'(h) ------
        if constexpr (SG) {
            const Tile tb2 = tile_of(b.sh2b, 256, row0, nrow, lane);
            const Tile td2 = tile_of(b.d2, 256, row0, nrow, lane);
            f32x16 ac[4];
            tmul<7, 4, SG, 0>(lds, wb, tb, dl, ac, w, lane, more, &tb2, 0);
            mask_wait<7, SG>();
            masked_epilogue<0>(lds, w, ac, dn, td2, lane);
            tmul<8, 4, SG, 8>(lds, wb, tb, dl, ac, w, lane, more, &tb2, 8);
            mask_wait<8, SG>();
            masked_epilogue<1>(lds, w, ac, dn, td2, lane);
#pragma unroll
            for (int k = 0; k < 16; ++k) dl[k] = dn[k];
        }
        // ---- block1.2 backward: delta1 = (W1^T delta2) * LReLU'(h1) ----------------------
        {
            const Tile t1 = tile_of(b.sh1, 256, row0, nrow, lane);
            const Tile td1 = tile_of(b.d1, 256, row0, nrow, lane);
            f32x16 ac[4];
            tmul<IW1, 4, SG, SG ? 8 : 0>(lds, wb, tb, dl, ac, w, lane, more, &t1, 0);
            mask_wait<IW1, SG>();
            masked_epilogue<0>(lds, w, ac, dn, td1, lane);
            tmul<IW1 + 1, 4, SG, 8>(lds, wb, tb, dl, ac, w, lane, more, &t1, 8);
            mask_wait<IW1 + 1, SG>();
            masked_epilogue<1>(lds, w, ac, dn, td1, lane);
        }
        // ---- block1.0 backward: d x0 = W0^T delta1 -> d feat through PE(feat) --------------
        float dfe[16];
#pragma unroll
        for (int c = 0; c < 16; ++c) dfe[c] = 0.f;
        static_for<3>([&](auto pp) {
            constexpr int P = decltype(pp)::value;
            f32x16 ac[3];
            tmul<IW0 + P, 3, SG, P == 0 ? 8 : 0>(lds, wb, tb, dn, ac, w, lane, more);
            static_for<3>([&](auto ttc) {
                constexpr int T = 3 * P + decltype(ttc)::value;
                static_for<16>([&](auto rr) {
                    constexpr int R = decltype(rr)::value;
                    l0_backward<16 * T + R>(ac[T - 3 * P][R], feat, dfe);
                });
            });
        });
        if (ok && ri.pid >= 0) {
            float *ge = b.g_emb + (int64_t)ri.pid * 32 + 16 * h;
#pragma unroll
            for (int c = 0; c < 16; ++c) atomicAdd(ge + c, dfe[c] * inv);
        }
    }
}

// ---- host-side packing of the transposed blob -------------------------------------------

// M: [n_rows][n_cols] row-major fp32; fragment (t, ks), lane, e <- M[rowfn(32 t + (lane & 31))][colfn(ks, 8 (lane >> 5) + e)]
template <typename T, typename RowFn, typename ColFn>
void pack_t(T *dst, const float *M, int n_rows, int n_cols, int n_tiles, RowFn rowfn, ColFn colfn) {
    for (int t = 0; t < n_tiles; ++t)
        for (int ks = 0; ks < 16; ++ks)
            for (int lane = 0; lane < 64; ++lane)
                for (int e = 0; e < 8; ++e) {
                    const int r = rowfn(32 * t + (lane & 31));
                    const int c = colfn(ks, 8 * (lane >> 5) + e);
                    const float v = (r >= 0 && r < n_rows && c >= 0 && c < n_cols) ? M[(size_t)r * n_cols + c] : 0.f;
                    dst[(((size_t)t * 16 + ks) * 64 + lane) * 8 + e] = (T)v;
                }
}

std::vector<float> transpose(const float *W, int n_out, int n_in) {
    std::vector<float> T((size_t)n_out * n_in);
    for (int o = 0; o < n_out; ++o)
        for (int i = 0; i < n_in; ++i) T[(size_t)i * n_out + o] = W[(size_t)o * n_in + i];
    return T;
}

int chain_col(int ks, int p) { return 16 * ks + perm_acc(p); }
// layer-0 transposed rows: tile position 32 t + jj holds local channel 16 t + r of lane-half hh,
// (hh, r) = ((jj >> 2) & 1, (jj & 3) + 4 (jj >> 3)) -- the inverse of acc_unit
int t0_row(int pos) {
    const int t = pos >> 5, jj = pos & 31;
    return l0_ref_col((jj >> 2) & 1, 16 * t + (jj & 3) + 4 * (jj >> 3));
}

// w: block1.0, block1.2, block3.0, block3.2 weights, and (SG, wb != nullptr) block2_bpnet.0's
// [256][256 + bpnet_dim] weight, of which the first 256 input columns are transposed
template <typename T>
void pack_tblob(const float *const *w, T *e, const float *wb = nullptr, int bpnet_dim = 0) {
    const auto idr = [](int r) { return r; };
    std::vector<float> t3 = transpose(w[3], 256, 256), t2 = transpose(w[2], 256, 263), t1 = transpose(w[1], 256, 256),
                       t0 = transpose(w[0], 256, 284);
    pack_t(e + OFF_T3 / 2, t3.data(), 256, 256, TT3, idr, chain_col);
    pack_t(e + OFF_T2 / 2, t2.data(), 263, 256, TT2, idr, chain_col);
    pack_t(e + OFF_T1 / 2, t1.data(), 256, 256, TT1, idr, chain_col);
    pack_t(e + OFF_T0 / 2, t0.data(), 284, 256, TT0, t0_row, chain_col);
    if (wb) {
        std::vector<float> h((size_t)256 * 256);
        for (int o = 0; o < 256; ++o)
            for (int i = 0; i < 256; ++i) h[(size_t)o * 256 + i] = wb[(size_t)o * (256 + bpnet_dim) + i];
        std::vector<float> tbp = transpose(h.data(), 256, 256);
        pack_t(e + OFF_TB / 2, tbp.data(), 256, 256, TTB, idr, chain_col);
    }
}

}  // namespace
}  // namespace sgn

extern "C" {

size_t sgn_train_tblob_bytes(void) { return sgn::T_BYTES; }

/* Index map of the transposed blob over the flat parameter vector (as sgn_mlp_pack_index):
 * n = sgn_train_tblob_bytes() / 2 elements, value = flat index + 1, 0 = zero. */
int sgn_train_pack_index(int32_t *out, int64_t n) {
    using namespace sgn;
    SGN_REQUIRE(out && n == (int64_t)(T_BYTES / 2), "sgn_train_pack_index: bad size");
    // flat offsets of block1.0 / block1.2 / block3.0 / block3.2 weights (LAYERS order: w, b per layer)
    const int64_t o0 = 0, o1 = o0 + 256 * 284 + 256, o2 = o1 + 256 * 256 + 256, o3 = o2 + 256 * 263 + 256;
    const int64_t offs[4] = {o0, o1, o2, o3};
    const int sz[4] = {256 * 284, 256 * 256, 256 * 263, 256 * 256};
    std::vector<std::vector<float>> wi(4);
    std::vector<const float *> wp(4);
    for (int L = 0; L < 4; ++L) {
        wi[L].resize(sz[L]);
        for (int i = 0; i < sz[L]; ++i) wi[L][i] = (float)(offs[L] + i + 1);
        wp[L] = wi[L].data();
    }
    std::vector<float> e(T_BYTES / 2, 0.f);
    pack_tblob(wp.data(), e.data());
    for (int64_t i = 0; i < n; ++i) out[i] = (int32_t)e[(size_t)i];
    return 0;
}

/* As sgn_train_pack_index for the SG flat vector (the 9 base layers, then block2_bpnet.0 weight
 * [256][256 + bpnet_dim] and bias): the block2_bpnet section of the transposed blob maps too. */
int sgn_train_pack_index_sg(int32_t bpnet_dim, int32_t *out, int64_t n) {
    using namespace sgn;
    SGN_REQUIRE(bpnet_dim == 0 || bpnet_dim == mlp::BP_DIM, "bpnet_dim must be 0 or 96");
    SGN_REQUIRE(out && n == (int64_t)(T_BYTES / 2), "sgn_train_pack_index_sg: bad size");
    const int64_t o0 = 0, o1 = o0 + 256 * 284 + 256, o2 = o1 + 256 * 256 + 256, o3 = o2 + 256 * 263 + 256;
    const int64_t ob = 341764;  // after the 9 base layers (weights.N_PARAMS)
    const int64_t offs[5] = {o0, o1, o2, o3, ob};
    const int64_t sz[5] = {256 * 284, 256 * 256, 256 * 263, 256 * 256, (int64_t)256 * (256 + bpnet_dim)};
    std::vector<std::vector<float>> wi(5);
    std::vector<const float *> wp(5);
    for (int L = 0; L < 5; ++L) {
        wi[L].resize((size_t)sz[L]);
        for (int64_t i = 0; i < sz[L]; ++i) wi[L][(size_t)i] = (float)(offs[L] + i + 1);
        wp[L] = wi[L].data();
    }
    std::vector<float> e(T_BYTES / 2, 0.f);
    pack_tblob(wp.data(), e.data(), wp[4], bpnet_dim);
    for (int64_t i = 0; i < n; ++i) out[i] = (int32_t)e[(size_t)i];
    return 0;
}

int sgn_train_pack_t_sg(const float *const *w, int32_t bpnet_dim, void *d_tblob, sgn_stream_t stream) {
    using namespace sgn;
    SGN_REQUIRE(w && w[0] && w[1] && w[2] && w[3] && w[4], "null weights");
    SGN_REQUIRE(bpnet_dim == 0 || bpnet_dim == mlp::BP_DIM, "bpnet_dim must be 0 or 96");
    std::vector<uint8_t> blob(T_BYTES, 0);
    pack_tblob(w, (_Float16 *)blob.data(), w[4], bpnet_dim);
    hipStream_t st = as_stream(stream);
    SGN_CHECK_HIP(hipMemcpyAsync(d_tblob, blob.data(), T_BYTES, hipMemcpyHostToDevice, st));
    SGN_CHECK_HIP(hipStreamSynchronize(st));
    return 0;
}

int sgn_train_pack_t(const float *const *w, void *d_tblob, sgn_stream_t stream) {
    using namespace sgn;
    using namespace sgn::mlp;
    SGN_REQUIRE(w && w[0] && w[1] && w[2] && w[3], "null weights");
    std::vector<uint8_t> blob(T_BYTES, 0);
    pack_tblob(w, (_Float16 *)blob.data());
    hipStream_t st = as_stream(stream);
    SGN_CHECK_HIP(hipMemcpyAsync(d_tblob, blob.data(), T_BYTES, hipMemcpyHostToDevice, st));
    SGN_CHECK_HIP(hipStreamSynchronize(st));
    return 0;
}

/* Column maps of the saved / delta tiles -> reference indices (-1 = padding):
 * which 0: chain columns (256) -> unit; 1: block1.0 inputs (288) -> block1.0 input column;
 * 2: block3.0 inputs (272) -> block3.0 input column. */
int sgn_train_colmap(int32_t which, int32_t *out, int32_t n) {
    using namespace sgn::mlp;
    const int want = which == 0 ? 256 : which == 1 ? KS_L0 * 16 : which == 2 ? KS_L2 * 16 : -1;
    SGN_REQUIRE(want > 0 && out && n == want, "sgn_train_colmap: bad map id or size");
    for (int p = 0; p < n; ++p) {
        const int ks = p >> 4, hh = (p >> 3) & 1, e = p & 7;
        if (which == 1) out[p] = l0_ref_col(hh, 8 * ks + e);
        else if (ks < 16) out[p] = 16 * ks + perm_acc(p & 15);
        else out[p] = (hh == 0 && e < 7) ? 256 + e : -1;
    }
    return 0;
}

int sgn_aggregate_backward(const sgn_point_tables *pt, const sgn_query_out *q, int32_t n_items, int32_t K,
                           const void *d_packed, const void *d_tblob, const sgn_agg_saved *saved,
                           const float *d_dfs, const float *d_dalpha, const float *d_scale,
                           const sgn_agg_deltas *deltas, const sgn_point_grads *grads, sgn_stream_t stream) {
    using namespace sgn;
    SGN_REQUIRE(pt && q && d_packed && d_tblob && saved && deltas && grads && d_scale, "null argument");
    SGN_REQUIRE(n_items >= 0, "n_items < 0");
    SGN_REQUIRE(K >= 1 && K <= 8, "the MFMA aggregator takes K = 1 .. 8 neighbours per sample");
    SGN_REQUIRE(pt->campos && pt->camrotc2w && pt->raydir && !pt->pers, "camera required, no precomputed pers");
    if (n_items == 0) return 0;
    SGN_REQUIRE(d_dfs && d_dalpha && saved->h1 && saved->h2 && saved->h3, "null saved/input tensors");
    SGN_REQUIRE(deltas->d1 && deltas->d2 && deltas->d3 && deltas->d4 && deltas->h4 && deltas->dza, "null delta outputs");
    SGN_REQUIRE(grads->embedding && grads->color && grads->dir && grads->conf, "null gradient outputs");
    BwdArgs b{};
    AggArgs &a = b.a;
    a.xyz = pt->xyz; a.emb = pt->embedding; a.color = pt->color; a.dir = pt->dir; a.conf = pt->conf;
    a.campos = pt->campos; a.rot = pt->camrotc2w; a.raydir = pt->raydir;
    a.pers = nullptr; a.samp_pers = nullptr;
    a.counters = q->counters; a.work = q->work; a.samp_ray = q->samp_ray; a.pidx = q->pidx;
    a.samp_locw = q->samp_locw;
    a.K = K;
    a.blob = d_packed; a.blob_bytes = mlp::TOTAL_BYTES;
    a.blend = nullptr; a.wnorm = nullptr;
    b.tblob = d_tblob;
    b.sh1 = (const _Float16 *)saved->h1; b.sh2 = (const _Float16 *)saved->h2; b.sh3 = (const _Float16 *)saved->h3;
    b.dfs = d_dfs; b.dalpha = d_dalpha; b.scale = d_scale;
    b.d4 = (_Float16 *)deltas->d4; b.d3 = (_Float16 *)deltas->d3; b.d2 = (_Float16 *)deltas->d2;
    b.d1 = (_Float16 *)deltas->d1; b.h4 = (_Float16 *)deltas->h4; b.dza = deltas->dza;
    b.g_emb = grads->embedding; b.g_color = grads->color; b.g_dir = grads->dir; b.g_conf = grads->conf;
    b.n_items = n_items;
    const int64_t waves = ((int64_t)n_items + 3) / 4;
    const int64_t blocks = (waves + 3) / 4;
    hipLaunchKernelGGL(k_agg_bwd<false>, dim3((unsigned)(blocks < 2048 ? blocks : 2048)), dim3(BWD_TPB), 0,
                       as_stream(stream), b);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

int sgn_aggregate_backward_sg(int32_t bpnet_layers, int32_t bpnet_dim, const sgn_point_tables *pt,
                              const sgn_query_out *q, int32_t n_items, int32_t K, const void *d_packed,
                              const void *d_tblob,
                              const sgn_agg_saved *saved, const void *d_h2b, const float *d_dfs, const float *d_dalpha,
                              const float *d_scale, const sgn_agg_deltas *deltas, void *d_db,
                              const sgn_point_grads *grads, sgn_stream_t stream) {
    using namespace sgn;
    if (bpnet_layers == 0)
        return sgn_aggregate_backward(pt, q, n_items, K, d_packed, d_tblob, saved, d_dfs, d_dalpha, d_scale, deltas,
                                      grads, stream);
    SGN_REQUIRE(bpnet_layers == 1 && (bpnet_dim == 0 || bpnet_dim == mlp::BP_DIM),
                "block2_bpnet: supported are 0 layers, or 1 layer with bpnet_dim 0 or 96");
    SGN_REQUIRE(pt && q && d_packed && d_tblob && saved && deltas && grads && d_scale && d_h2b && d_db, "null argument");
    SGN_REQUIRE(n_items >= 0, "n_items < 0");
    SGN_REQUIRE(K >= 1 && K <= 8, "the MFMA aggregator takes K = 1 .. 8 neighbours per sample");
    SGN_REQUIRE(pt->campos && pt->camrotc2w && pt->raydir && !pt->pers, "camera required, no precomputed pers");
    if (n_items == 0) return 0;
    SGN_REQUIRE(d_dfs && d_dalpha && saved->h1 && saved->h2 && saved->h3, "null saved/input tensors");
    SGN_REQUIRE(deltas->d1 && deltas->d2 && deltas->d3 && deltas->d4 && deltas->h4 && deltas->dza, "null delta outputs");
    SGN_REQUIRE(grads->embedding && grads->color && grads->dir && grads->conf, "null gradient outputs");
    BwdArgs b{};
    AggArgs &a = b.a;
    a.xyz = pt->xyz; a.emb = pt->embedding; a.color = pt->color; a.dir = pt->dir; a.conf = pt->conf;
    a.campos = pt->campos; a.rot = pt->camrotc2w; a.raydir = pt->raydir;
    a.pers = nullptr; a.samp_pers = nullptr;
    a.counters = q->counters; a.work = q->work; a.samp_ray = q->samp_ray; a.pidx = q->pidx;
    a.samp_locw = q->samp_locw;
    a.K = K;
    a.blob = d_packed; a.blob_bytes = mlp::total_bytes_sg(mlp::ks_bp(bpnet_dim));
    a.blend = nullptr; a.wnorm = nullptr;
    b.tblob = d_tblob;
    b.sh1 = (const _Float16 *)saved->h1; b.sh2 = (const _Float16 *)saved->h2; b.sh3 = (const _Float16 *)saved->h3;
    b.sh2b = (const _Float16 *)d_h2b; b.db = (_Float16 *)d_db;
    b.dfs = d_dfs; b.dalpha = d_dalpha; b.scale = d_scale;
    b.d4 = (_Float16 *)deltas->d4; b.d3 = (_Float16 *)deltas->d3; b.d2 = (_Float16 *)deltas->d2;
    b.d1 = (_Float16 *)deltas->d1; b.h4 = (_Float16 *)deltas->h4; b.dza = deltas->dza;
    b.g_emb = grads->embedding; b.g_color = grads->color; b.g_dir = grads->dir; b.g_conf = grads->conf;
    b.n_items = n_items;
    const int64_t waves = ((int64_t)n_items + 3) / 4;
    const int64_t blocks = (waves + 3) / 4;
    hipLaunchKernelGGL(k_agg_bwd<true>, dim3((unsigned)(blocks < 2048 ? blocks : 2048)), dim3(BWD_TPB), 0,
                       as_stream(stream), b);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

}  // extern "C"
