// mlp.hip -- fused neural-point aggregator on MFMA (gfx950, fp16 in / fp32 accumulate).
//
// Replaces NeuralPoints.forward's gather (neural_points.py:942-988) and
// PointAggregator.forward + viewmlp (point_aggregators.py:868-959, :561-786) for the
// ScanNet configuration (agg_dist_pers 20, linear kernel, agg_intrp_order 2).
//
// k_point_proj: P[point] = W0a [feat | PE(feat)] + b0, block1.0's 224 per-point input
//   channels, once per frame (fp16, accumulator order).
// k_agg_rows: one wave owns a 32-row column tile = 4 shading samples x K=8 neighbours; a
//   512-thread workgroup (8 waves) = one 256-row work tile.
//   prologue : gather point records by index, pers transform, 6-d dists, inverse-distance
//              weights normalised over the 8 rows of a sample (lane butterflies), conf
//              clamp; accumulators start at P[pid]
//   block1   : PE(dists) -> 256 (layer 0, 4 k-steps) -> 256; block3: 263 -> 256 -> 256, as
//              MFMA chains; each layer's accumulator tile is converted in place into the
//              next layer's B operand (the k permutation lives in the packed weights)
//   block3.2 : transposed, so the alpha dot product and the K-blend f_s = sum_k w_k h_k are
//              per-lane FMAs; f_s leaves as fp16 rows for k_color
// k_color: one wave = 32 samples: [f_s | PE(viewdir)] -> 128 -> 128 -> 128 -> 3, sigmoid.
//
// Weights stream through an LDS ring filled by LDS-DMA and shared by the workgroup's 8 waves;
// activations never leave registers between layers.  DESIGN.md section 3.1 has the timing.
#include <cstdio>
#include <cstdlib>
#include <utility>
#include <vector>

#include "agg_device.h"

namespace sgn {
namespace {


// ---- workgroup-shared weight stream, k-outer ---------------------------------------
// A workgroup = 8 waves (2 per SIMD) = 32 samples x 8 neighbours = 256 rows, 32 rows per
// wave.  Per layer pass each wave keeps its output tiles as MFMA accumulators and walks the
// input k-steps in order, so an input fragment dies as soon as it has been multiplied into the
// pass's tiles (layer-0 fragments are generated just in time from the row's dists).  The
// weights (424 fragments of 1 KiB per tile, packed [layer][pass][k-step][tile]) stream through
// a 2-slot LDS ring of chunks of up to 36 fragments filled by LDS-DMA (buffer_load ... lds),
// the next chunk in flight while the current one is read; one barrier per chunk.  Every
// fragment fetched into LDS feeds 8 waves.
constexpr int ROWS_TPB = 512;
constexpr int WG_WAVES = ROWS_TPB / 64;
constexpr int WG_SAMPLES = WG_WAVES * 4;  // 32
constexpr int CHUNK_FRAGS = 32;  // fragments per LDS chunk (k-steps x tiles of a pass)
constexpr int FRAG_PD = 3;  // weight fragments in flight per wave (LDS -> VGPR queue)
// output tiles per pass: layer 0 runs all 8 tiles in one pass (its inputs are generated on
// the fly and never stored), the chained layers run two passes of 4 (their input fragments
// stay in registers, the accumulators of 8 tiles would not fit beside them)
__host__ __device__ constexpr int layer_tp(int L) { return L == 0 ? 8 : 4; }
__host__ __device__ constexpr int layer_np(int L) { return 8 / layer_tp(L); }
// block3.0 (17 k-steps: 256 chained + the colour/dir channels) goes in chunks of 9 + 8 k-steps
// instead of 8 + 8 + 1: a 4-fragment tail chunk cost a whole boundary (~2.3 k cycles for 4
// MFMAs per wave, measured with clock stamps in round 2)
__host__ __device__ constexpr int layer_kc(int L) { return L == 2 ? 9 : CHUNK_FRAGS / layer_tp(L); }
constexpr int MAX_CHUNK_FRAGS = 9 * 4 > CHUNK_FRAGS ? 9 * 4 : CHUNK_FRAGS;
constexpr int SLOT_BYTES = MAX_CHUNK_FRAGS * (int)FRAG;
constexpr int PF_MAX = (MAX_CHUNK_FRAGS + WG_WAVES - 1) / WG_WAVES;  // LDS-DMA pieces per wave per chunk (max)
constexpr int NSLOT = 2;  // ring slots: the next chunk in flight while the current one is read (two
                          // in flight measured 12 % slower: k_agg_rows 13.65 vs 11.97 ms, same box)
constexpr int LDS_F32_OFF = NSLOT * SLOT_BYTES;
// blended features leave through a per-wave LDS transpose as one 16-B store per lane and
// block3.2 pass (full 128-B lines) instead of eight 2-B scattered stores
constexpr int FSW_OFF = LDS_F32_OFF + (int)(N_F32 + HID) * 4;  // after the fp32 section + block2_bpnet bias (SG)
constexpr int FSW_BYTES = WG_WAVES * 1024;  // [wave][4 samples][128 units] fp16
constexpr int LDS_BYTES = FSW_OFF + FSW_BYTES;
static_assert(CHUNK_FRAGS % WG_WAVES == 0, "chunk must split evenly over the waves");


// Layers of the row stream: 0 block1.0, 1 block1.2, 2 block3.0, 3 block3.2, 4 block2_bpnet.0
// (SG variant only).  Variant code V = KSB + 256 * SPLIT: KSB = k-steps of block2_bpnet.0
// (0: variant absent), SPLIT = per-point block1.0 projection (layer 0 = W0b only, 4 k-steps).
// Stream order: 0, 1, [4], 2, 3.  (The stream helpers below take V in their KSB argument.)
__host__ __device__ constexpr int vksb(int V) { return V & 255; }
__host__ __device__ constexpr bool vsplit(int V) { return (V >> 8) != 0; }
__host__ __device__ constexpr int layer_ks(int V, int L) {
    return L == 0 ? (vsplit(V) ? KS_L0S : KS_L0) : L == 2 ? KS_L2 : L == 4 ? vksb(V) : KS_HID;
}
__host__ __device__ constexpr int layer_nch(int KSB, int L) {
    return (layer_ks(KSB, L) + layer_kc(L) - 1) / layer_kc(L);
}
__host__ __device__ constexpr size_t layer_off(int V, int L) {
    return L == 0 ? (vsplit(V) ? OFF_W0B : OFF_W0) : L == 1 ? OFF_W1 : L == 2 ? OFF_W2 : L == 3 ? OFF_W3 : OFF_WB;
}
__host__ __device__ constexpr int chunk_nk(int KSB, int L, int c) {
    return (layer_ks(KSB, L) - c * layer_kc(L)) < layer_kc(L) ? (layer_ks(KSB, L) - c * layer_kc(L)) : layer_kc(L);
}
// stream position: layer L, pass P (tiles TP*P..), chunk C (k-steps C*KC..) -> blob offset
__host__ __device__ constexpr uint32_t chunk_off(int KSB, int L, int P, int C) {
    return (uint32_t)(layer_off(KSB, L) + ((size_t)P * layer_ks(KSB, L) * layer_tp(L) +
                                      (size_t)C * layer_kc(L) * layer_tp(L)) * FRAG);
}

// ---- chunk stream ---------------------------------------------------------------
// Per work tile the stream is: layer 0 (1 pass x 9 chunks), then the chained layers
// (2 passes each) in stream order.
__host__ __device__ constexpr int n_stream(int V) { return vksb(V) ? 5 : 4; }
__host__ __device__ constexpr int stream_layer(int V, int i) { return vksb(V) ? (i < 2 ? i : i == 2 ? 4 : i - 1) : i; }
__host__ __device__ constexpr int stream_pos(int V, int L) { return vksb(V) ? (L < 2 ? L : L == 4 ? 2 : L + 1) : L; }
__host__ __device__ constexpr int pass_chunks(int KSB, int L) { return layer_nch(KSB, L); }
__host__ __device__ constexpr int layer_chunks(int KSB, int L) { return layer_np(L) * layer_nch(KSB, L); }
__host__ __device__ constexpr int pos_base(int KSB, int i) {
    return i == 0 ? 0 : pos_base(KSB, i - 1) + layer_chunks(KSB, stream_layer(KSB, i - 1));
}
__host__ __device__ constexpr int chunk_base(int KSB, int L) { return pos_base(KSB, stream_pos(KSB, L)); }
__host__ __device__ constexpr int n_chunks(int KSB) { return pos_base(KSB, n_stream(KSB)); }
__host__ __device__ constexpr int chunk_index(int KSB, int L, int P, int C) {
    return chunk_base(KSB, L) + P * pass_chunks(KSB, L) + C;
}
__host__ __device__ constexpr int chunk_pos(int KSB, int n, int i = 0) {
    return (i + 1 >= n_stream(KSB) || n < pos_base(KSB, i + 1)) ? i : chunk_pos(KSB, n, i + 1);
}
__host__ __device__ constexpr int chunk_L(int KSB, int n) { return stream_layer(KSB, chunk_pos(KSB, n)); }
__host__ __device__ constexpr int chunk_P(int KSB, int n) {
    return (n - chunk_base(KSB, chunk_L(KSB, n))) / pass_chunks(KSB, chunk_L(KSB, n));
}
__host__ __device__ constexpr int chunk_C(int KSB, int n) {
    return (n - chunk_base(KSB, chunk_L(KSB, n))) % pass_chunks(KSB, chunk_L(KSB, n));
}
static_assert(n_chunks(0) == 5 + 2 * (2 + 2 + 2), "base stream");
static_assert((chunk_L(ks_bp(BP_DIM), 9) == 4 && chunk_L(ks_bp(BP_DIM), 8) == 1 &&
                   chunk_L(ks_bp(BP_DIM), 15) == 2 && n_chunks(ks_bp(BP_DIM)) == 23),
              "SG stream order");
static_assert((n_chunks(256) == 1 + 2 * (2 + 2 + 2) && chunk_L(256, 1) == 1),
              "split stream");

// Issue the LDS-DMA of stream chunk N into LDS slot `dst`: each wave moves fragments
// w + WG_WAVES*j (1 KiB, lane-linear) with buffer_load ... lds; the boundary waits for vmcnt(0).
template <int KSB, int N>
__device__ __forceinline__ void dma_chunk(const WBlob &wb, char *dst, int w, int lane, int lz) {
    constexpr int L = chunk_L(KSB, N), P = chunk_P(KSB, N), C = chunk_C(KSB, N);
    constexpr int nf = chunk_nk(KSB, L, C) * layer_tp(L);
    static_for<PF_MAX>([&](auto jj) {
        constexpr int J = decltype(jj)::value;
        if constexpr (WG_WAVES * J < nf) {
            const int i = w + WG_WAVES * J;
            if (WG_WAVES * (J + 1) <= nf || i < nf) {  // wave-uniform
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    wb.rsrc, (__attribute__((address_space(3))) void *)(dst + i * (int)FRAG), 16,
                    lane * 16, chunk_off(KSB, L, P, C) + (uint32_t)(i * (int)FRAG + lz), 0, 0);
            }
        }
    });
}

// Chunk boundary: wait for this wave's DMAs of the chunk about to be read, drain LDS reads,
// barrier; then start the next chunk's DMA into the slot read one chunk ago.
template <int KSB, int N>
__device__ __forceinline__ void chunk_enter(const WBlob &wb, char *lds, int &slot, int w, int lane, int lz) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    dma_chunk<KSB, (N + 1) % n_chunks(KSB)>(wb, lds + (slot ^ 1) * SLOT_BYTES, w, lane, lz);
}

// One pass of a layer, k-outer: acc[t] = bias + sum_k W[TP*P+t][k] * in(k), chunk by chunk.
// TRANS: the activations are the A operand and the weights the B operand, so the
// accumulators hold D^T (lane = output unit, registers = rows) and start at zero (the bias
// is added in the epilogue, where it is one value per lane).
struct NoHook {
    __device__ void operator()() const {}
};

// post(): called once, right after the boundary of the pass's chunk HOOK_C -- stores of the previous
// phase issued there are waited for by the NEXT boundary's vmcnt(0), one chunk of MFMAs later,
// instead of stalling the boundary that follows them directly.
template <int KSB, int L, int P, bool TRANS = false, bool PREINIT = false, int HOOK_C = 0, class InFn,
          class PostFn = NoHook>
__device__ __forceinline__ void run_pass(const WBlob &wb, char *lds, int &slot, int w, int lane, int lz,
                                         const float *Fl, size_t fb, f32x16 (&acc)[layer_tp(L)], InFn &&in,
                                         PostFn &&post = PostFn{}) {
    constexpr int TP = layer_tp(L), KC = layer_kc(L);
    const int h = lane >> 5;
#pragma unroll
    for (int tt = 0; tt < TP; ++tt) {
        if constexpr (PREINIT) {
            // accumulators already hold the per-point partial sums (split block1.0)
        } else if constexpr (TRANS) {
            acc[tt] = f32x16{};
        } else {  // accumulators start at the bias (acc order, LDS)
            const f32x4 *b = (const f32x4 *)(Fl + fb + ((TP * P + tt) * 2 + h) * 16);
            const f32x4 b0 = b[0], b1 = b[1], b2 = b[2], b3 = b[3];
            acc[tt] = f32x16{b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3],
                             b2[0], b2[1], b2[2], b2[3], b3[0], b3[1], b3[2], b3[3]};
        }
    }
    static_for<layer_nch(KSB, L)>([&](auto cc) {
        constexpr int C = decltype(cc)::value;
        chunk_enter<KSB, chunk_index(KSB, L, P, C)>(wb, lds, slot, w, lane, lz);
        if constexpr (C == HOOK_C) post();
        const char *sl = lds + slot * SLOT_BYTES;
        // weight fragments through a register queue PD deep, so LDS latency overlaps PD MFMAs
        constexpr int NF = chunk_nk(KSB, L, C) * TP, PD = NF < FRAG_PD ? NF : FRAG_PD;
        auto frag = [&](int f) { return *(const h8 *)(sl + f * (int)FRAG + lane * 16); };
        h8 fr[PD];
#pragma unroll
        for (int f = 0; f < PD; ++f) fr[f] = frag(f);
        __builtin_amdgcn_sched_group_barrier(0x100, PD, 0);  // PD LDS reads in flight first
        static_for<chunk_nk(KSB, L, C)>([&](auto kk) {
            constexpr int KK = decltype(kk)::value;
            const h8 B = in(std::integral_constant<int, C * KC + KK>{});
            static_for<TP>([&](auto tt) {
                constexpr int t = decltype(tt)::value, F = KK * TP + t;
                const h8 A = fr[F % PD];
                if constexpr (F + PD < NF) fr[F % PD] = frag(F + PD);
                acc[t] = TRANS ? mfma32(B, A, acc[t]) : mfma32(A, B, acc[t]);
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // then one LDS read
            });
        });
        slot = slot + 1 == NSLOT ? 0 : slot + 1;
        __builtin_amdgcn_sched_barrier(0);
    });
}

// Split block1.0, per row: acc[t] = P[pid][t] + W0b[t] PE(dists) (4 k-steps, one stream chunk).
// P (fp16, [point][tile t][lane-half h][16], so the two lanes of a row read one 64-B run per
// load) is loaded at entry; tiles go in pairs, k-outer inside a pair, so P of the later tiles
// lands while the earlier tiles multiply and only the first pair waits on the gather.
// P[pid] of this lane's row -> 16 B fragments in accumulator order (layout: run_split_l0)
__device__ __forceinline__ void load_proj(const _Float16 *proj, int pid, int lane, h8 (&pv)[16]) {
    const int h = lane >> 5;
    const h8 *src = (const h8 *)(proj + (int64_t)(pid < 0 ? 0 : pid) * HID);
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        pv[2 * t] = src[(2 * t + h) * 2];
        pv[2 * t + 1] = src[(2 * t + h) * 2 + 1];
    }
}

// pv: the rows' P, loaded a tile ahead (k_agg_rows issues it during the previous tile's last
// chunk): the scattered 16-B P reads cost the vector-memory path ~8k cycles per workgroup
// tile, which then overlap that chunk's MFMAs instead of stalling this tile's first barrier.
template <int V, class PostFn>
__device__ __forceinline__ void run_split_l0(const WBlob &wb, char *lds, int &slot, int w, int lane, int lz,
                                             const h8 (&pv)[16], const float (&feat)[16],
                                             const float (&dist)[3], f32x16 (&acc)[8], PostFn &&post) {
    static_assert(layer_nch(V, 0) == 1 && layer_ks(V, 0) == 4, "split layer 0 is one chunk of 4 k-steps");
    h8 B[4];
    static_for<4>([&](auto kk) { B[decltype(kk)::value] = l0_step<KS_P0 + decltype(kk)::value>(feat, dist); });
    chunk_enter<V, chunk_index(V, 0, 0, 0)>(wb, lds, slot, w, lane, lz);
    post();
    const char *sl = lds + slot * SLOT_BYTES;
    // stream position n -> fragment (k-step k, tile t): pair p = n / 8, k = (n % 8) / 2, t = 2p + n % 2
    auto fidx = [](int n) { return ((n & 7) >> 1) * 8 + 2 * (n >> 3) + (n & 1); };
    auto frag = [&](int f) { return *(const h8 *)(sl + f * (int)FRAG + lane * 16); };
    constexpr int NF = 32, PD = FRAG_PD;
    h8 fr[PD];
#pragma unroll
    for (int f = 0; f < PD; ++f) fr[f] = frag(fidx(f));
    __builtin_amdgcn_sched_group_barrier(0x100, PD, 0);
    static_for<4>([&](auto pp) {
        constexpr int P = decltype(pp)::value;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int t = 2 * P + u;
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                acc[t][r] = (float)pv[2 * t][r];
                acc[t][r + 8] = (float)pv[2 * t + 1][r];
            }
        }
        static_for<8>([&](auto nn) {
            constexpr int N = 8 * P + decltype(nn)::value, K = (N & 7) >> 1, T = 2 * P + (N & 1);
            const h8 A = fr[N % PD];
            if constexpr (N + PD < NF) fr[N % PD] = frag(fidx(N + PD));
            acc[T] = mfma32(A, B[K], acc[T]);
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        });
    });
    slot = slot + 1 == NSLOT ? 0 : slot + 1;
    __builtin_amdgcn_sched_barrier(0);
}

// LeakyReLU + fp16 pack: pass accumulators (bias included) -> next-layer fragments
template <int TP, int P>
__device__ __forceinline__ void chain_out(const f32x16 (&acc)[TP], h8 (&out)[16]) {
#pragma unroll
    for (int tt = 0; tt < TP; ++tt)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
            const int t = TP * P + tt, r = 8 * s2;
            const u32x4 u = {lrelu_pk(acc[tt][r + 0], acc[tt][r + 1]), lrelu_pk(acc[tt][r + 2], acc[tt][r + 3]),
                             lrelu_pk(acc[tt][r + 4], acc[tt][r + 5]), lrelu_pk(acc[tt][r + 6], acc[tt][r + 7])};
            out[2 * t + s2] = __builtin_bit_cast(h8, u);
        }
}

template <int V, bool SAVE = false>
__global__ __launch_bounds__(ROWS_TPB, 1) void k_agg_rows(AggArgs a) {
    constexpr int KSB = vksb(V);
    constexpr bool SPLIT = vsplit(V);
    static_assert(!(SPLIT && SAVE), "the training save mode runs the unsplit block1.0");
    constexpr int NBP = KSB > KS_HID ? KSB - KS_HID : 0;  // BPNet k-steps (SG, predict_semantic = 1)
    __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES + WG_WAVES * NBP * (int)FRAG];
    const int lane = threadIdx.x & 63;
    const int h = lane >> 5, kk = lane & 7, q = (lane & 31) >> 3;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nwork = a.counters[1];
    const int end = min(nwork, a.item0 + a.n_items);
    const Cam cam = load_cam(a.campos, a.rot);
    const WBlob wb = make_blob(a.blob, a.blob_bytes);
    const __amdgpu_buffer_rsrc_t bp_rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)a.bpnet, (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t fs_rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)a.fs, (short)0, 0x7fffffff, 0x00020000);
    {   // fp32 parameters (biases, alpha weights) -> LDS once
        const float *src = (const float *)((const char *)a.blob + OFF_F32);
        float *dst = (float *)(lds + LDS_F32_OFF);
        for (int i = threadIdx.x; i < (int)N_F32; i += ROWS_TPB) dst[i] = src[i];
        if constexpr (KSB > 0) {  // block2_bpnet.0 bias (acc order) after the base section
            const float *bb = (const float *)((const char *)a.blob + off_bb(KSB));
            for (int i = threadIdx.x; i < HID; i += ROWS_TPB) dst[F_BB + i] = bb[i];
        }
    }
    __syncthreads();  // parameters visible before the first tile's bias reads
    int slot = 0;
    // stream prologue: chunk 0 in flight (chunk_enter<n> issues chunk n + 1)
    dma_chunk<V, 0>(wb, lds, w, lane, 0);
    // Phase stagger: every workgroup runs identical tiles, so without it all CUs gather their
    // tiles' point records (~150 KB per CU) in the same microseconds and the chip-wide burst
    // (~38 MB of random reads) sets the tile-start latency.  Eight start phases, one per
    // group of CUs on every XCD (workgroups go round-robin over the 8 XCDs), ~1/8 tile apart.
    for (int i = (blockIdx.x >> 3) & 7; i > 0; --i) __builtin_amdgcn_s_sleep(127);
    // index chain of this wave's rows, one work tile ahead (issued mid-tile, see block1.2)
    RowIdx nx = row_index(a, a.item0 + blockIdx.x * WG_SAMPLES + w * 4 + q, end, lane);
    asm volatile("" : "+v"(nx.s), "+v"(nx.pid), "+v"(nx.ray));  // waited for here (once), see block3.0
    h8 pnext[16];  // split block1.0: the next tile's P rows (see run_split_l0)
    if constexpr (SPLIT) {
        if (a.item0 + (int)blockIdx.x * WG_SAMPLES < end) load_proj(a.proj, nx.pid, lane, pnext);  // P[0] exists
    }
    // blended features of a block3.2 pass as fp16 pairs (tile tt, half k2) -> pf[tt]; pass 0's
    // are stored after block3.2 pass 1's first chunk boundary (see run_pass), pass 1's at once
    // (the next tile's first boundary waits on its gather loads anyway)
    const int jl = lane & 31;
    uint32_t pf0[4], pf1[4];
    // stores as wave ww; drop = true sends them out of the buffer's range (discarded by the
    // hardware) so the wave-role choice below needs no branch (a branch here costs ~20 spills)
    auto flush_fs = [&](const uint32_t (&pv)[4], int pbase, int P, int ww) {
        // lane (unit jl, half h) holds samples h (lo) and h + 2 (hi) of tiles 4P + tt
        _Float16 *st = (_Float16 *)(lds + FSW_OFF + w * 1024);
#pragma unroll
        for (int tt = 0; tt < 4; ++tt) {
            st[h * 128 + 32 * tt + jl] = __builtin_bit_cast(_Float16, (unsigned short)(pv[tt] & 0xffff));
            st[(h + 2) * 128 + 32 * tt + jl] = __builtin_bit_cast(_Float16, (unsigned short)(pv[tt] >> 16));
        }
        // lane L: sample L >> 4, units 8 (L & 15) .. +7 of the pass (16 B)
        const u32x4 v = *(const u32x4 *)(st + (lane >> 4) * 128 + 8 * (lane & 15));
        const int it = pbase + ww * 4 + (lane >> 4);
        const uint32_t off = it < end ? (uint32_t)((it - a.item0) * HID + 128 * P + 8 * (lane & 15)) * 2 : 0xFFFF0000u;
        __builtin_amdgcn_raw_buffer_store_b128(v, fs_rsrc, off, 0, 0);
    };

    for (int base = a.item0 + blockIdx.x * WG_SAMPLES; base < end; base += gridDim.x * WG_SAMPLES) {
        // opaque zero per iteration: keeps LDS parameter reads and weight offsets inside the loop
        int lz = 0;
        asm volatile("" : "+s"(lz));
        char *ldsi = lds + lz;
        const float *Fl = (const float *)(ldsi + LDS_F32_OFF);
        const int item = base + w * 4 + q;
        float feat[16], dist[3];
        h8 ext;
        const RowIn ri = gather_row<!SPLIT>(a, cam, nx, lane, feat, dist, ext);
        const int nitem = item + gridDim.x * WG_SAMPLES;

        const int64_t srow0 = (int64_t)(base + w * 4 - a.item0) * 8;  // first saved row of this wave (SAVE)
        // SG: this row's BPNet embedding -> the wave's LDS area as ready-made B fragments
        // (LDS-DMA, one 1-KiB fragment per k-step; lane (row, half h) <- channels 16j+8h..+7).
        // Its vmcnt is covered by the chunk waits before block2_bpnet (older than those DMAs).
        char *bpl = ldsi + LDS_BYTES + w * NBP * (int)FRAG;
        if constexpr (KSB > KS_HID) {
            const uint32_t rb = (uint32_t)(ri.pid < 0 ? 0 : ri.pid) * (NBP * 32) + 16 * h;
#pragma unroll
            for (int j = 0; j < NBP; ++j)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    bp_rsrc, (__attribute__((address_space(3))) void *)(bpl + j * (int)FRAG), 16, rb + 32 * j, 0, 0, 0);
        }
        h8 actA[16], actB[16];
        {   // block1.0: 284 -> 256, one pass over 8 tiles, inputs generated per k-step
            f32x16 acc0[8];
            if constexpr (SPLIT) {
                run_split_l0<V>(wb, ldsi, slot, w, lane, lz, pnext, feat, dist, acc0, NoHook{});
            } else {
                run_pass<V, 0, 0>(wb, ldsi, slot, w, lane, lz, Fl, F_B0, acc0, [&](auto k) {
                    const h8 v = l0_step<decltype(k)::value>(feat, dist);
                    if constexpr (SAVE) save_frag(a.sx0, KS_L0 * 16, srow0, decltype(k)::value, v, lane, ri.sval);
                    return v;
                });
            }
            chain_out<8, 0>(acc0, actA);
            if constexpr (SAVE) {
#pragma unroll
                for (int s2 = 0; s2 < 16; ++s2) save_frag(a.sh1, 256, srow0, s2, actA[s2], lane, ri.sval);
            }
        }
        f32x16 acc[4];
        // block1.2: 256 -> 256
        auto inA = [&](auto k) { return actA[decltype(k)::value]; };
        run_pass<V, 1, 0>(wb, ldsi, slot, w, lane, lz, Fl, F_B1, acc, inA);
        chain_out<4, 0>(acc, actB);
        if constexpr (SAVE) {
#pragma unroll
            for (int s2 = 0; s2 < 8; ++s2) {
                if constexpr (KSB > 0) save_frag(a.sh2b, 256, srow0, s2, actB[s2], lane, ri.sval);
                else save_frag(a.sh2, KS_L2 * 16, srow0, s2, actB[s2], lane, ri.sval);
            }
        }
        run_pass<V, 1, 1>(wb, ldsi, slot, w, lane, lz, Fl, F_B1, acc, inA);
        // next tile's index chain: work entry now, neighbour / ray indices one pass later
        const int s_next = nitem < end ? a.work[nitem] : 0;
        chain_out<4, 1>(acc, actB);
        if constexpr (SAVE) {
#pragma unroll
            for (int s2 = 8; s2 < 16; ++s2) {
                if constexpr (KSB > 0) save_frag(a.sh2b, 256, srow0, s2, actB[s2], lane, ri.sval);
                else save_frag(a.sh2, KS_L2 * 16, srow0, s2, actB[s2], lane, ri.sval);
            }
            if constexpr (KSB == 0) save_frag(a.sh2, KS_L2 * 16, srow0, 16, ext, lane, ri.sval);
        }
        if constexpr (KSB > 0) {
            // block2_bpnet.0 (SG): [h 256 | BPNet embedding] -> 256 (point_aggregators.py:629-636)
            auto inBP = [&](auto k) {
                constexpr int K = decltype(k)::value;
                if constexpr (K < 16) return actB[K];
                else return *(const h8 *)(bpl + (K - 16) * (int)FRAG + lane * 16);
            };
            run_pass<V, 4, 0>(wb, ldsi, slot, w, lane, lz, Fl, F_BB, acc, inBP);
            chain_out<4, 0>(acc, actA);
            run_pass<V, 4, 1>(wb, ldsi, slot, w, lane, lz, Fl, F_BB, acc, inBP);
            chain_out<4, 1>(acc, actA);
            if constexpr (SAVE) {  // block3.0's inputs: the block2_bpnet output + the extra channels
#pragma unroll
                for (int s2 = 0; s2 < 16; ++s2) save_frag(a.sh2, KS_L2 * 16, srow0, s2, actA[s2], lane, ri.sval);
                save_frag(a.sh2, KS_L2 * 16, srow0, 16, ext, lane, ri.sval);
            }
        }
        // block3.0: [h 256 | colour, dir - v, <dir, v>] -> 256 (input in actB, or actA after block2_bpnet)
        auto &in3 = pick<(KSB > 0)>(actA, actB);
        auto &out3 = pick<(KSB > 0)>(actB, actA);
        auto in3f = [&](auto k) {
            constexpr int K = decltype(k)::value;
            if constexpr (K < 16) return in3[K]; else return ext;
        };
        run_pass<V, 2, 0>(wb, ldsi, slot, w, lane, lz, Fl, F_B2, acc, in3f);
        nx.sval = nitem < end;
        nx.s = s_next;
        nx.pid = nx.sval && kk < a.K ? a.pidx[(int64_t)s_next * a.K + kk] : -1;
        nx.ray = a.samp_ray[s_next];
        chain_out<4, 0>(acc, out3);
        run_pass<V, 2, 1>(wb, ldsi, slot, w, lane, lz, Fl, F_B2, acc, in3f);
        // the next tile's indices have landed (this pass's boundaries drained vmcnt); hide their
        // loads from the compiler's wait tracking, which otherwise -- with more VMEM ops in
        // between than vmcnt can count -- waits for every younger load (the next tile's P) at
        // the loop head
        asm volatile("" : "+v"(nx.s), "+v"(nx.pid), "+v"(nx.ray));
        chain_out<4, 1>(acc, out3);
        if constexpr (SAVE) {
#pragma unroll
            for (int s2 = 0; s2 < 16; ++s2) save_frag(a.sh3, 256, srow0, s2, out3[s2], lane, ri.sval);
        }
        // block3.2: 256 -> 256, transposed (lane = output unit j = lane & 31 of tile t,
        // register i = row (i & 3) + 8 (i >> 2) + 4h, i.e. sample i >> 2), so the K-blend
        // and the alpha dot product are per-lane FMAs over registers
        float wv[16];      // K-blend weight of the row in register i
#pragma unroll
        for (int i = 0; i < 16; ++i)
            wv[i] = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(
                                                  ((i & 3) + 8 * (i >> 2) + 4 * h) * 4, __builtin_bit_cast(int, ri.wgt)));
        f32x2 ap2[8] = {};  // alpha logit partials of rows (2p, 2p+1) over this lane's units
        const int j = lane & 31;
        auto l3_epilogue = [&](auto pp) {
            constexpr int P = decltype(pp)::value, TP = 4;
#pragma unroll
            for (int tt = 0; tt < TP; ++tt) {
                const int t = TP * P + tt;
                const float bu = Fl[F_B3 + 32 * t + j], wau = Fl[F_WA + 32 * t + j];
                // register pairs (i, i+1) as packed fp32 (v_pk_add/mul/fma_f32)
                f32x2 fg2[4] = {};
#pragma unroll
                for (int i = 0; i < 16; i += 2) {
                    const f32x2 y = f32x2{acc[tt][i], acc[tt][i + 1]} + f32x2{bu, bu};
                    const f32x2 z = y * f32x2{0.01f, 0.01f};
                    const f32x2 hv = {fmaxf(y[0], z[0]), fmaxf(y[1], z[1])};
                    ap2[i >> 1] = __builtin_elementwise_fma(f32x2{wau, wau}, hv, ap2[i >> 1]);
                    fg2[i >> 2] = __builtin_elementwise_fma(f32x2{wv[i], wv[i + 1]}, hv, fg2[i >> 2]);
                }
                float fg[4];
#pragma unroll
                for (int g = 0; g < 4; ++g) fg[g] = fg2[g][0] + fg2[g][1];
                // halves hold rows 4h..4h+3 of each sample: lanes 0-31 <- samples 0 / 2,
                // lanes 32-63 <- samples 1 / 3 (v_permlane32_swap)
                float x0 = fg[0], y0 = fg[1], x1 = fg[2], y1 = fg[3];
                permlane32_swap(x0, y0);
                permlane32_swap(x1, y1);
                typedef _Float16 h2 __attribute__((ext_vector_type(2)));
                const h2 pk = {(_Float16)(x0 + y0), (_Float16)(x1 + y1)};
                pick<P == 0>(pf0, pf1)[tt] = __builtin_bit_cast(uint32_t, pk);
                (void)t;
            }
        };
        auto inA3 = [&](auto k) { return out3[decltype(k)::value]; };
        run_pass<V, 3, 0, true>(wb, ldsi, slot, w, lane, lz, Fl, F_B3, acc, inA3);
        l3_epilogue(std::integral_constant<int, 0>{});
        flush_fs(pf0, base, 0, w);
        run_pass<V, 3, 1, true, false, layer_nch(V, 3) - 1>(wb, ldsi, slot, w, lane, lz, Fl, F_B3, acc, inA3, [&]() {
            if constexpr (SPLIT) load_proj(a.proj, nx.pid, lane, pnext);  // next tile's P (its last chunk)
        });
        l3_epilogue(std::integral_constant<int, 1>{});
        flush_fs(pf1, base, 1, w);
        // alpha: reduce the 16 row partials over the 32 lanes (units) of each half,
        // reduce-scatter style; lane j ends with row index i = 8 b1 + 4 b2 + 2 b3 + b4 (b = bits of j)
        float bq[8];
#pragma unroll
        for (int p2 = 0; p2 < 8; ++p2) {  // lanes j, j^16 (v_permlane16_swap)
            float x = ap2[p2][0], y = ap2[p2][1];
            permlane16_swap(x, y);
            bq[p2] = x + y;
        }
        auto rs_step = [&](float lo, float hi, bool upper, auto ctrl) {
            const float keep = upper ? hi : lo, send = upper ? lo : hi;
            return keep + __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, send),
                                                                             decltype(ctrl)::value, 0xF, 0xF, true));
        };
        float cq[4], dq[2];
#pragma unroll
        for (int u = 0; u < 4; ++u)  // lanes j, j^8 (row_ror:8)
            cq[u] = rs_step(bq[2 * u], bq[2 * u + 1], (j & 8) != 0, std::integral_constant<int, 0x128>{});
#pragma unroll
        for (int v = 0; v < 2; ++v)  // lanes j, 7-j within 8 (row_half_mirror)
            dq[v] = rs_step(cq[2 * v], cq[2 * v + 1], (j & 4) != 0, std::integral_constant<int, 0x141>{});
        float eq = rs_step(dq[0], dq[1], (j & 2) != 0, std::integral_constant<int, 0x4E>{});  // j, j^2
        eq += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, eq), 0xB1, 0xF, 0xF, true));
        const float alpha_val = softplus(eq + Fl[F_BA] - 1.f);
        // back to lane = row: row r lives in half (r >> 2) & 1 at register i = (r & 3) + 4 (r >> 3)
        const int ri_ = (j & 3) + 4 * (j >> 3);
        const int src = 32 * ((j >> 2) & 1) + 2 * ((ri_ >> 3) & 1) + 4 * ((ri_ >> 2) & 1) + 8 * ((ri_ >> 1) & 1) +
                        16 * (ri_ & 1);
        const float alpha_row =
            __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src * 4, __builtin_bit_cast(int, alpha_val)));
        const float alpha_s = dpp_sum8(ri.wgt * alpha_row);
        if (ri.sval && kk == 0 && h == 0) a.feat[(int64_t)ri.s * 4 + 0] = alpha_s;
    }
    // the stream ran one chunk ahead: let those LDS-DMAs land before the workgroup retires
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
struct ColorArgs {
    const int32_t *counters, *work, *samp_ray;
    const float *raydir;
    const void *blob;
    const _Float16 *fs;
    float *feat;
    int32_t item0, n_items;
};

// Colour MLP, one 512-thread workgroup per CU: the 136 colour fragments (C0..C2, 136 KiB)
// and the colour fp32 parameters are copied into LDS once (LDS-DMA), then every wave runs
// 32 samples at a time: [f_s | PE(viewdir)] -> 128 -> 128 -> 128 (MFMA, A from LDS) -> 3.
constexpr int COL_TPB = 512;
constexpr int COL_FRAGS = T_CHID * (KS_C0 + 2 * KS_CH);  // 136
constexpr int COL_F32 = (int)(N_F32 - F_CB0);             // colour biases + output layer
constexpr int COL_LDS = COL_FRAGS * (int)FRAG + COL_F32 * 4;
static_assert(COL_FRAGS % (COL_TPB / 64) == 0, "colour fragments split evenly over the waves");
static_assert(OFF_C1 == OFF_C0 + (size_t)T_CHID * KS_C0 * FRAG && OFF_C2 == OFF_C1 + (size_t)T_CHID * KS_CH * FRAG,
              "colour layers are contiguous");

template <int KS, int NIN>
__device__ __forceinline__ void color_layer(const char *wl, const float *bl, const h8 (&in)[NIN], h8 (&out)[8],
                                            int lane) {
    const int h = lane >> 5;
#pragma unroll
    for (int t = 0; t < T_CHID; ++t) {
        f32x16 acc = {};
#pragma unroll
        for (int k = 0; k < KS; ++k)
            acc = mfma32(*(const h8 *)(wl + (t * KS + k) * (int)FRAG + lane * 16), in[k], acc);
        const float *b = bl + (t * 2 + h) * 16;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
            const int r = 8 * s2;
            const u32x4 u = {lrelu_pk(acc[r + 0] + b[r + 0], acc[r + 1] + b[r + 1]),
                             lrelu_pk(acc[r + 2] + b[r + 2], acc[r + 3] + b[r + 3]),
                             lrelu_pk(acc[r + 4] + b[r + 4], acc[r + 5] + b[r + 5]),
                             lrelu_pk(acc[r + 6] + b[r + 6], acc[r + 7] + b[r + 7])};
            out[2 * t + s2] = __builtin_bit_cast(h8, u);
        }
    }
}

__global__ __launch_bounds__(COL_TPB, 1) void k_color(ColorArgs a) {
    __shared__ __attribute__((aligned(16))) char lds[COL_LDS];
    const int lane = threadIdx.x & 63;
    const int h = lane >> 5, j = lane & 31;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nwork = a.counters[1];
    const int end = min(nwork, a.item0 + a.n_items);
    const WBlob wb = make_blob(a.blob);
#pragma unroll
    for (int i = 0; i < COL_FRAGS / (COL_TPB / 64); ++i) {  // colour fragments -> LDS
        const int f = w + (COL_TPB / 64) * i;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            wb.rsrc, (__attribute__((address_space(3))) void *)(lds + f * (int)FRAG), 16, lane * 16,
            (uint32_t)(OFF_C0 + (size_t)f * FRAG), 0, 0);
    }
    {   // f32 section from F_CB0
        float *dst = (float *)(lds + COL_FRAGS * (int)FRAG);
        const float *src = (const float *)((const char *)a.blob + OFF_F32) + F_CB0;
        for (int i = threadIdx.x; i < COL_F32; i += COL_TPB) dst[i] = src[i];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int wave = blockIdx.x * (COL_TPB / 64) + w;
    const int nwaves = gridDim.x * (COL_TPB / 64);
    for (int base = a.item0 + wave * 32; base < end; base += nwaves * 32) {
        // opaque zero: keeps the (loop-invariant) LDS fragment reads inside the loop
        int lz = 0;
        asm volatile("" : "+s"(lz));
        const char *W0 = lds + lz, *W1 = W0 + T_CHID * KS_C0 * (int)FRAG, *W2 = W1 + T_CHID * KS_CH * (int)FRAG;
        const float *Fc = (const float *)(lds + lz + COL_FRAGS * (int)FRAG);
        const int item = base + j;
        const bool sval = item < end;
        const int s = sval ? a.work[item] : 0;
        const int ray = a.samp_ray[s];
        h8 x[KS_C0];
        const h8 *row = (const h8 *)(a.fs + (int64_t)(sval ? item - a.item0 : 0) * HID);
#pragma unroll
        for (int k = 0; k < 16; ++k) x[k] = row[2 * k + h];
        // PE(viewdir) ori=True, channels [3:] (point_aggregators.py:579-585, networks.py:175-192):
        // pe[d*4+f] = sin(v_d 2^f), pe[12+d*4+f] = cos(v_d 2^f)
        const float v[3] = {a.raydir[(int64_t)ray * 3], a.raydir[(int64_t)ray * 3 + 1], a.raydir[(int64_t)ray * 3 + 2]};
        float pe[24];
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            float s0, c0;
            sincos_pow2<0>(v[d], s0, c0);
            pe[d * 4] = s0;
            pe[12 + d * 4] = c0;
#pragma unroll
            for (int f = 1; f < 4; ++f) {
                const float s1 = 2.f * s0 * c0, c1 = (c0 - s0) * (c0 + s0);
                s0 = s1;
                c0 = c1;
                pe[d * 4 + f] = s0;
                pe[12 + d * 4 + f] = c0;
            }
        }
        x[16] = h ? pack8(pe[8], pe[9], pe[10], pe[11], pe[12], pe[13], pe[14], pe[15])
                  : pack8(pe[0], pe[1], pe[2], pe[3], pe[4], pe[5], pe[6], pe[7]);
        x[17] = h ? h8{} : pack8(pe[16], pe[17], pe[18], pe[19], pe[20], pe[21], pe[22], pe[23]);
        h8 y1[KS_CH], y2[KS_CH];
        color_layer<KS_C0, KS_C0>(W0, Fc + (F_CB0 - F_CB0), x, y1, lane);
        color_layer<KS_CH, KS_CH>(W1, Fc + (F_CB1 - F_CB0), y1, y2, lane);
        float o[3] = {0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < T_CHID; ++t) {
            f32x16 acc = {};
#pragma unroll
            for (int k = 0; k < KS_CH; ++k)
                acc = mfma32(*(const h8 *)(W2 + (t * KS_CH + k) * (int)FRAG + lane * 16), y2[k], acc);
            const float *b = Fc + (F_CB2 - F_CB0) + (t * 2 + h) * 16;
            const float *w0 = Fc + (F_WC3 - F_CB0) + (t * 2 + h) * 16;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float y = acc[r] + b[r];
                const float hv = fmaxf(y, 0.01f * y);
                o[0] = fmaf(w0[r], hv, o[0]);
                o[1] = fmaf(w0[128 + r], hv, o[1]);
                o[2] = fmaf(w0[256 + r], hv, o[2]);
            }
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float z = o[c] + __shfl_xor(o[c], 32) + Fc[F_BC3 - F_CB0 + c];
            o[c] = (1.f / (1.f + expf(-z))) * (1.f + 2.f * 0.001f) - 0.001f;
        }
        if (sval && h == 0) {
            a.feat[(int64_t)s * 4 + 1] = o[0];
            a.feat[(int64_t)s * 4 + 2] = o[1];
            a.feat[(int64_t)s * 4 + 3] = o[2];
        }
    }
}

// ---- per-point block1.0 projection (split block1.0) ---------------------------------
// P[p] = W0a [feat_p | PE(feat_p)] + b0 for every point (the 224 point-only channels of the
// 284 block1.0 inputs, mlp_layout.h), fp16 in accumulator order per lane-half: P[p][h][t][r] =
// unit 32 t + acc_unit(r, h).  One 512-thread workgroup per CU keeps W0a (112 KiB) and b0 in
// LDS; each wave takes 32 points at a time, lane = point, k-outer over 14 k-steps.
constexpr int PROJ_TPB = 512;
constexpr int PROJ_FRAGS = T_HID * KS_P0;  // 112
constexpr int PROJ_LDS = PROJ_FRAGS * (int)FRAG + HID * 4;
static_assert(PROJ_FRAGS % (PROJ_TPB / 64) == 0, "projection fragments split evenly over the waves");

struct ProjArgs {
    const float *emb;
    int64_t n;
    const void *blob;
    _Float16 *proj;
    const int32_t *idx = nullptr;    // subset: the points idx[0 .. *count) only
    const int64_t *count = nullptr;
};

__global__ __launch_bounds__(PROJ_TPB, 1) void k_point_proj(ProjArgs a) {
    __shared__ __attribute__((aligned(16))) char lds[PROJ_LDS];
    const int lane = threadIdx.x & 63, h = lane >> 5;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const WBlob wb = make_blob(a.blob);
#pragma unroll
    for (int i = 0; i < PROJ_FRAGS / (PROJ_TPB / 64); ++i) {  // W0a fragments -> LDS (LDS-DMA)
        const int f = w + (PROJ_TPB / 64) * i;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(wb.rsrc, (__attribute__((address_space(3))) void *)(lds + f * (int)FRAG),
                                                 16, lane * 16, (uint32_t)(OFF_W0A + (size_t)f * FRAG), 0, 0);
    }
    {
        float *dst = (float *)(lds + PROJ_FRAGS * (int)FRAG);
        const float *src = (const float *)((const char *)a.blob + OFF_F32) + F_B0;
        for (int i = threadIdx.x; i < HID; i += PROJ_TPB) dst[i] = src[i];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int64_t n = a.idx ? (*a.count < a.n ? *a.count : a.n) : a.n;
    const int64_t nt = (n + 31) / 32;
    for (int64_t tile = (int64_t)blockIdx.x * (PROJ_TPB / 64) + w; tile < nt; tile += (int64_t)gridDim.x * (PROJ_TPB / 64)) {
        int lz = 0;
        asm volatile("" : "+s"(lz));
        const char *W = lds + lz;
        const float *B = (const float *)(lds + lz + PROJ_FRAGS * (int)FRAG);
        const int64_t q = tile * 32 + (lane & 31);
        const bool ok = q < n;
        const int64_t p = a.idx ? (ok ? (int64_t)a.idx[q] : 0) : q;
        float feat[16], dist[3] = {0.f, 0.f, 0.f};
        {
            const f32x4 *e4 = (const f32x4 *)(a.emb + (ok ? p : 0) * 32 + 16 * h);
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const f32x4 v = e4[g];
                feat[4 * g] = v[0]; feat[4 * g + 1] = v[1]; feat[4 * g + 2] = v[2]; feat[4 * g + 3] = v[3];
            }
        }
        f32x16 acc[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const f32x4 *b = (const f32x4 *)(B + (t * 2 + h) * 16);
            const f32x4 b0 = b[0], b1 = b[1], b2 = b[2], b3 = b[3];
            acc[t] = f32x16{b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3],
                            b2[0], b2[1], b2[2], b2[3], b3[0], b3[1], b3[2], b3[3]};
        }
        static_for<KS_P0>([&](auto kk) {
            constexpr int KK = decltype(kk)::value;
            const h8 x = l0_step<KK>(feat, dist);
#pragma unroll
            for (int t = 0; t < 8; ++t)
                acc[t] = mfma32(*(const h8 *)(W + (t * KS_P0 + KK) * (int)FRAG + lane * 16), x, acc[t]);
        });
        if (ok) {
            h8 *dst = (h8 *)(a.proj + p * HID);  // [t][h][16]: see run_split_l0
#pragma unroll
            for (int t = 0; t < 8; ++t)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    const int r = 8 * s2;
                    dst[(2 * t + h) * 2 + s2] = pack8(acc[t][r], acc[t][r + 1], acc[t][r + 2], acc[t][r + 3], acc[t][r + 4],
                                            acc[t][r + 5], acc[t][r + 6], acc[t][r + 7]);
                }
        }
    }
}

// fp32 -> fp16 point table (BPNet embedding of the SG variant): 4 values per thread
__global__ __launch_bounds__(256) void k_to_f16(const float *__restrict__ src, _Float16 *__restrict__ dst, int64_t n) {
    for (int64_t i = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) * 4; i < n; i += (int64_t)gridDim.x * blockDim.x * 4) {
        if (i + 4 <= n) {
            const f32x4 v = *(const f32x4 *)(src + i);
            typedef _Float16 h4 __attribute__((ext_vector_type(4)));
            *(h4 *)(dst + i) = h4{(_Float16)v[0], (_Float16)v[1], (_Float16)v[2], (_Float16)v[3]};
        } else {
            for (int64_t k = i; k < n; ++k) dst[k] = (_Float16)src[k];
        }
    }
}

// ---- host-side packing ---------------------------------------------------------

// column of the reference weight matrix feeding B position p of k-step ks (-1: zero)
int col_l0(int ks, int p) { return l0_ref_col(p >> 3, 8 * ks + (p & 7)); }
int col_chain(int ks, int p) { return 16 * ks + perm_acc(p); }
int col_l2(int ks, int p) { return ks < 16 ? col_chain(ks, p) : (p < 7 ? 256 + p : -1); }
int col_l0b(int ks, int p) { return l0_ref_col(p >> 3, 8 * (KS_P0 + ks) + (p & 7)); }
int col_l0a(int ks, int p) { return l0_ref_col(p >> 3, 8 * ks + (p & 7)); }
int col_bp(int ks, int p) { return ks < 16 ? col_chain(ks, p) : 256 + 16 * (ks - 16) + p; }
int col_c0(int ks, int p) { return ks < 16 ? 16 * ks + p : (16 * (ks - 16) + p < 24 ? 256 + 16 * (ks - 16) + p : -1); }

// kouter: fragment (t, ks) at index ks*n_tiles + t (block1/block3 stream order), else t*KS + ks
template <typename T, typename ColFn>
void pack_frags(T *dst, const float *W, int n_out, int n_in, int n_tiles, int KS, ColFn col, int kouter) {
    for (int t = 0; t < n_tiles; ++t)
        for (int ks = 0; ks < KS; ++ks)
            for (int lane = 0; lane < 64; ++lane)
                for (int e = 0; e < 8; ++e) {
                    int row = 32 * t + (lane & 31);
                    int c = col(ks, 8 * (lane >> 5) + e);
                    float v = (row < n_out && c >= 0 && c < n_in) ? W[(size_t)row * n_in + c] : 0.f;
                    // kouter > 0: [pass = t/kouter][ks][t%kouter] (k-outer stream of k_agg_rows)
                    size_t f = kouter ? ((size_t)(t / kouter) * KS + ks) * kouter + (t % kouter)
                                      : (size_t)t * KS + ks;
                    dst[(f * 64 + lane) * 8 + e] = (T)v;
                }
}

void pack_acc_order(float *dst, const float *v, int n_tiles) {
    for (int t = 0; t < n_tiles; ++t)
        for (int h = 0; h < 2; ++h)
            for (int r = 0; r < 16; ++r) dst[(t * 2 + h) * 16 + r] = v[32 * t + acc_unit(r, h)];
}

// The whole blob: fragment part as elements of e16 (element i = byte 2 i), fp32 section F,
// block2_bpnet bias Fbb (SG).  T16 = _Float16 packs weights; T16 = float packs index maps.
template <typename T16>
void pack_blob(int ksb, int bpnet_dim, const float *const *w, const float *const *b, T16 *e16, float *F, float *Fbb) {
    auto frag = [&](size_t off) { return e16 + off / 2; };
    pack_frags(frag(OFF_W0), w[0], 256, 284, T_HID, KS_L0, col_l0, layer_tp(0));
    pack_frags(frag(OFF_W1), w[1], 256, 256, T_HID, KS_HID, col_chain, layer_tp(1));
    pack_frags(frag(OFF_W2), w[2], 256, 263, T_HID, KS_L2, col_l2, layer_tp(2));
    pack_frags(frag(OFF_W3), w[3], 256, 256, T_HID, KS_HID, col_chain, layer_tp(3));
    pack_frags(frag(OFF_C0), w[5], 128, 280, T_CHID, KS_C0, col_c0, 0);
    pack_frags(frag(OFF_C1), w[6], 128, 128, T_CHID, KS_CH, col_chain, 0);
    pack_frags(frag(OFF_C2), w[7], 128, 128, T_CHID, KS_CH, col_chain, 0);
    pack_frags(frag(OFF_W0B), w[0], 256, 284, T_HID, KS_L0S, col_l0b, layer_tp(0));  // split block1.0, per row
    pack_frags(frag(OFF_W0A), w[0], 256, 284, T_HID, KS_P0, col_l0a, 0);             // split block1.0, per point
    pack_acc_order(F + F_B0, b[0], T_HID);
    pack_acc_order(F + F_B1, b[1], T_HID);
    pack_acc_order(F + F_B2, b[2], T_HID);
    for (int u = 0; u < HID; ++u) F[F_B3 + u] = b[3][u];  // natural order: block3.2 runs transposed
    pack_acc_order(F + F_CB0, b[5], T_CHID);
    pack_acc_order(F + F_CB1, b[6], T_CHID);
    pack_acc_order(F + F_CB2, b[7], T_CHID);
    for (int u = 0; u < HID; ++u) F[F_WA + u] = w[4][u];
    F[F_BA] = b[4][0];
    for (int c = 0; c < 3; ++c) {
        pack_acc_order(F + F_WC3 + c * 128, w[8] + c * 128, T_CHID);
        F[F_BC3 + c] = b[8][c];
    }
    if (ksb > 0) {  // block2_bpnet.0 = w[9] [256, 256 + bpnet_dim], b[9] [256]
        pack_frags(frag(OFF_WB), w[9], 256, 256 + bpnet_dim, T_HID, ksb, col_bp, layer_tp(4));
        pack_acc_order(Fbb, b[9], T_HID);
    }
}

}  // namespace
}  // namespace sgn

extern "C" {

size_t sgn_mlp_packed_bytes(void) { return sgn::mlp::TOTAL_BYTES; }

size_t sgn_mlp_section(int32_t which) {
    using namespace sgn::mlp;
    return which == 0 ? OFF_F32 : which == 1 ? OFF_W0B : which == 2 ? TOTAL_BYTES : 0;
}

size_t sgn_point_proj_bytes(int64_t n_points) { return (size_t)(n_points > 0 ? n_points : 0) * sgn::mlp::PROJ_BYTES_PER_POINT; }

int sgn_point_project_subset(const sgn_point_tables *pt, const void *d_packed, const int32_t *d_idx,
                             const int64_t *d_count, void *d_proj, sgn_stream_t stream) {
    using namespace sgn;
    using namespace sgn::mlp;
    SGN_REQUIRE(pt && d_packed && d_proj && d_idx && d_count, "null argument");
    SGN_REQUIRE(pt->n_points >= 0 && (pt->n_points == 0 || pt->embedding), "embedding required");
    if (pt->n_points == 0) return 0;
    ProjArgs a{pt->embedding, pt->n_points, d_packed, (_Float16 *)d_proj, d_idx, d_count};
    // persistent grid over the device count (a frame names ~19 % of the points)
    const int64_t waves = (pt->n_points + 31) / 32;
    const int64_t wg = (waves + PROJ_TPB / 64 - 1) / (PROJ_TPB / 64);
    hipLaunchKernelGGL(k_point_proj, dim3((unsigned)(wg < 256 ? wg : 256)), dim3(PROJ_TPB), 0, as_stream(stream), a);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

int sgn_point_project(const sgn_point_tables *pt, const void *d_packed, void *d_proj, sgn_stream_t stream) {
    using namespace sgn;
    using namespace sgn::mlp;
    SGN_REQUIRE(pt && d_packed && d_proj, "null argument");
    SGN_REQUIRE(pt->n_points >= 0 && (pt->n_points == 0 || pt->embedding), "embedding required");
    if (pt->n_points == 0) return 0;
    ProjArgs a{pt->embedding, pt->n_points, d_packed, (_Float16 *)d_proj};
    const int64_t waves = (pt->n_points + 31) / 32;
    const int64_t wg = (waves + PROJ_TPB / 64 - 1) / (PROJ_TPB / 64);
    hipLaunchKernelGGL(k_point_proj, dim3((unsigned)(wg < 256 ? wg : 256)), dim3(PROJ_TPB), 0, as_stream(stream), a);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

static int mlp_variant_ksb(int32_t bpnet_layers, int32_t bpnet_dim) {
    if (bpnet_layers == 0) return 0;
    if (bpnet_layers == 1 && (bpnet_dim == 0 || bpnet_dim == sgn::mlp::BP_DIM)) return sgn::mlp::ks_bp(bpnet_dim);
    return -1;
}

size_t sgn_mlp_packed_bytes_sg(int32_t bpnet_layers, int32_t bpnet_dim) {
    const int ksb = mlp_variant_ksb(bpnet_layers, bpnet_dim);
    return ksb < 0 ? 0 : sgn::mlp::total_bytes_sg(ksb);
}

int sgn_mlp_pack_sg(int32_t bpnet_layers, int32_t bpnet_dim, const float *const *w, const float *const *b,
                    void *d_packed, sgn_stream_t stream) {
    using namespace sgn;
    using namespace sgn::mlp;
    SGN_REQUIRE(w && b && d_packed, "null argument");
    const int ksb = mlp_variant_ksb(bpnet_layers, bpnet_dim);
    SGN_REQUIRE(ksb >= 0, "block2_bpnet: supported are 0 layers, or 1 layer with bpnet_dim 0 or 96");
    if (ksb > 0) SGN_REQUIRE(w[9] && b[9], "block2_bpnet.0 weights missing");
    std::vector<uint8_t> blob(total_bytes_sg(ksb), 0);
    pack_blob(ksb, bpnet_dim, w, b, (_Float16 *)blob.data(), (float *)(blob.data() + OFF_F32),
              ksb > 0 ? (float *)(blob.data() + off_bb(ksb)) : nullptr);
    hipStream_t st = as_stream(stream);
    SGN_CHECK_HIP(hipMemcpyAsync(d_packed, blob.data(), blob.size(), hipMemcpyHostToDevice, st));
    SGN_CHECK_HIP(hipStreamSynchronize(st));
    return 0;
}

int sgn_mlp_pack(const float *const *w, const float *const *b, void *d_packed, sgn_stream_t stream) {
    return sgn_mlp_pack_sg(0, 0, w, b, d_packed, stream);
}

/* Index maps of the base forward blob over the flat parameter vector (LAYERS order, each
 * layer weight row-major then bias): out[i] = flat index + 1, 0 = zero padding.
 * which 0: fragment part (OFF_F32 / 2 fp16 elements), 1: fp32 section (N_F32),
 * 2: split block1.0 sections [OFF_W0B, TOTAL_BYTES) as fp16 elements. */
int sgn_mlp_pack_index(int32_t which, int32_t *out, int64_t n) {
    using namespace sgn;
    using namespace sgn::mlp;
    const int64_t want = which == 0 ? (int64_t)(OFF_F32 / 2) : which == 1 ? (int64_t)N_F32
                       : which == 2 ? (int64_t)((TOTAL_BYTES - OFF_W0B) / 2) : -1;
    SGN_REQUIRE(out && n == want, "sgn_mlp_pack_index: bad map id or size");
    static const int shape[9][2] = {{256, 284}, {256, 256}, {256, 263}, {256, 256}, {1, 256},
                                    {128, 280}, {128, 128}, {128, 128}, {3, 128}};
    std::vector<std::vector<float>> wi(9), bi(9);
    std::vector<const float *> wp(9), bp(9);
    int64_t off = 0;
    for (int L = 0; L < 9; ++L) {
        wi[L].resize((size_t)shape[L][0] * shape[L][1]);
        for (size_t i = 0; i < wi[L].size(); ++i) wi[L][i] = (float)(off + (int64_t)i + 1);
        off += (int64_t)wi[L].size();
        bi[L].resize(shape[L][0]);
        for (size_t i = 0; i < bi[L].size(); ++i) bi[L][i] = (float)(off + (int64_t)i + 1);
        off += (int64_t)bi[L].size();
        wp[L] = wi[L].data();
        bp[L] = bi[L].data();
    }
    std::vector<float> e16(TOTAL_BYTES / 2, 0.f), F(N_F32, 0.f);
    pack_blob<float>(0, 0, wp.data(), bp.data(), e16.data(), F.data(), nullptr);
    const float *src = which == 0 ? e16.data() : which == 1 ? F.data() : e16.data() + OFF_W0B / 2;
    for (int64_t i = 0; i < n; ++i) out[i] = (int32_t)src[i];
    return 0;
}

// Work items per launch: the blended features are stored through a buffer descriptor (31-bit
// byte range) based at the launch's first item, so at most 2^31 / 512 B items per launch.
constexpr int64_t F16_MAX_CHUNK = ((int64_t)0x7fffffff / (sgn::mlp::HID * 2)) / 32 * 32;

size_t sgn_aggregate_workspace_bytes(int64_t S) {
    // blended-feature rows of every work item (fp16, 512 B each), so the two stages may be called
    // separately; a smaller workspace is accepted with stages = 3 (both stages per chunk)
    if (S < 32) S = 32;
    return (size_t)S * sgn::mlp::HID * sizeof(_Float16);
}

int sgn_aggregate_sg(int32_t bpnet_layers, int32_t bpnet_dim, const void *d_bpnet_f16, const void *d_point_proj,
                     const sgn_point_tables *pt, const sgn_query_out *q, int64_t S_capacity, int32_t K,
                     const void *d_packed, float *d_out_feat, float *d_out_blend, float *d_out_wnorm,
                     void *d_workspace, size_t workspace_bytes, int32_t stages, sgn_stream_t stream) {
    using namespace sgn;
    using namespace sgn::mlp;
    SGN_REQUIRE(pt && q && d_packed && d_out_feat && d_workspace, "null argument");
    const int ksb = mlp_variant_ksb(bpnet_layers, bpnet_dim);
    SGN_REQUIRE(ksb >= 0, "block2_bpnet: supported are 0 layers, or 1 layer with bpnet_dim 0 or 96");
    SGN_REQUIRE(ksb <= KS_HID || d_bpnet_f16, "bpnet_dim > 0 needs the fp16 BPNet point embedding");
    SGN_REQUIRE(K >= 1 && K <= 8, "the MFMA aggregator takes K = 1 .. 8 neighbours per sample");
    hipStream_t st = as_stream(stream);
    const int64_t ws_items = (int64_t)(workspace_bytes / (HID * sizeof(_Float16)));
    SGN_REQUIRE(ws_items >= 32, "aggregate workspace too small");
    SGN_REQUIRE(stages == 3 || ws_items >= S_capacity,
                "stages 1 and 2 called separately need a workspace for all S_capacity items");
    // chunk = items per launch; with a full-size workspace chunk c keeps its rows at item c * chunk
    const bool full = ws_items >= S_capacity;
    const int64_t chunk = ws_items < F16_MAX_CHUNK ? ws_items : F16_MAX_CHUNK;
    const uint8_t *P = (const uint8_t *)d_packed;
    AggArgs a;
    a.xyz = pt->xyz; a.emb = pt->embedding; a.color = pt->color; a.dir = pt->dir; a.conf = pt->conf;
    a.campos = pt->campos; a.rot = pt->camrotc2w; a.raydir = pt->raydir;
    a.pers = pt->pers; a.samp_pers = pt->samp_pers;
    SGN_REQUIRE((pt->pers == nullptr) == (pt->samp_pers == nullptr), "pers and samp_pers go together");
    SGN_REQUIRE(pt->campos && pt->camrotc2w && pt->raydir, "camera (campos, camrotc2w, raydir) required");
    a.counters = q->counters; a.work = q->work; a.samp_ray = q->samp_ray; a.pidx = q->pidx;
    a.samp_locw = q->samp_locw;
    a.K = K;
    a.blob = P;
    a.blob_bytes = total_bytes_sg(ksb);
    a.bpnet = (const _Float16 *)d_bpnet_f16;
    a.proj = (const _Float16 *)d_point_proj;
    a.feat = d_out_feat; a.blend = d_out_blend; a.wnorm = d_out_wnorm; a.fs = (_Float16 *)d_workspace;
    ColorArgs c;
    c.counters = q->counters; c.work = q->work; c.samp_ray = q->samp_ray; c.raydir = pt->raydir;
    c.blob = P; c.fs = a.fs; c.feat = d_out_feat;
    for (int64_t i0 = 0; i0 < S_capacity; i0 += chunk) {
        int64_t n = S_capacity - i0 < chunk ? S_capacity - i0 : chunk;
        a.item0 = c.item0 = (int32_t)i0;
        a.n_items = c.n_items = (int32_t)n;
        a.fs = (_Float16 *)d_workspace + (full ? i0 * HID : 0);
        c.fs = a.fs;
        int64_t wg = (n + WG_SAMPLES - 1) / WG_SAMPLES;  // persistent: one workgroup per CU
        dim3 g1((unsigned)(wg < 256 ? wg : 256));
        if (stages & 1) {
            constexpr int SP = 256;  // split block1.0 (per-point projection given)
            constexpr int KB = ks_bp(BP_DIM);
            auto kern = d_point_proj ? (ksb == 0 ? k_agg_rows<SP> : ksb == KS_HID ? k_agg_rows<KS_HID + SP>
                                                                                : k_agg_rows<KB + SP>)
                                     : (ksb == 0 ? k_agg_rows<0> : ksb == KS_HID ? k_agg_rows<KS_HID>
                                                                                : k_agg_rows<KB>);
            hipLaunchKernelGGL(kern, g1, dim3(ROWS_TPB), 0, st, a);
        }
        int64_t wg2 = (n + 32 * (COL_TPB / 64) - 1) / (32 * (COL_TPB / 64));  // 32 samples per wave
        dim3 g2((unsigned)(wg2 < 256 ? wg2 : 256));  // persistent: colour weights loaded once per CU
        if (stages & 2) hipLaunchKernelGGL(k_color, g2, dim3(COL_TPB), 0, st, c);
    }
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

int sgn_aggregate_train_fwd(const sgn_point_tables *pt, const sgn_query_out *q, int64_t S_capacity, int32_t K,
                            const void *d_packed, float *d_out_feat, void *d_fs, const sgn_agg_saved *saved,
                            sgn_stream_t stream) {
    using namespace sgn;
    using namespace sgn::mlp;
    SGN_REQUIRE(pt && q && d_packed && d_out_feat && d_fs && saved, "null argument");
    SGN_REQUIRE(saved->x0 && saved->h1 && saved->h2 && saved->h3, "null saved-activation buffer");
    SGN_REQUIRE(K >= 1 && K <= 8, "the MFMA aggregator takes K = 1 .. 8 neighbours per sample");
    SGN_REQUIRE(pt->campos && pt->camrotc2w && pt->raydir && !pt->pers, "camera required, no precomputed pers");
    SGN_REQUIRE(S_capacity >= 0 && S_capacity < (1 << 27), "S_capacity out of range");
    if (S_capacity == 0) return 0;
    AggArgs a{};
    a.xyz = pt->xyz; a.emb = pt->embedding; a.color = pt->color; a.dir = pt->dir; a.conf = pt->conf;
    a.campos = pt->campos; a.rot = pt->camrotc2w; a.raydir = pt->raydir;
    a.counters = q->counters; a.work = q->work; a.samp_ray = q->samp_ray; a.pidx = q->pidx;
    a.samp_locw = q->samp_locw;
    a.K = K;
    a.blob = d_packed; a.blob_bytes = TOTAL_BYTES;
    a.feat = d_out_feat; a.fs = (_Float16 *)d_fs;
    a.item0 = 0; a.n_items = (int32_t)S_capacity;
    a.sx0 = (_Float16 *)saved->x0; a.sh1 = (_Float16 *)saved->h1; a.sh2 = (_Float16 *)saved->h2;
    a.sh3 = (_Float16 *)saved->h3;
    int64_t wg = (S_capacity + WG_SAMPLES - 1) / WG_SAMPLES;
    hipLaunchKernelGGL((k_agg_rows<0, true>), dim3((unsigned)(wg < 256 ? wg : 256)), dim3(ROWS_TPB), 0, as_stream(stream), a);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

int sgn_aggregate_train_fwd_sg(int32_t bpnet_layers, int32_t bpnet_dim, const void *d_bpnet_f16,
                               const sgn_point_tables *pt, const sgn_query_out *q, int64_t S_capacity, int32_t K,
                               const void *d_packed, float *d_out_feat, void *d_fs, const sgn_agg_saved *saved,
                               void *d_h2b, sgn_stream_t stream) {
    using namespace sgn;
    using namespace sgn::mlp;
    const int ksb = mlp_variant_ksb(bpnet_layers, bpnet_dim);
    SGN_REQUIRE(ksb >= 0, "block2_bpnet: supported are 0 layers, or 1 layer with bpnet_dim 0 or 96");
    if (ksb == 0)
        return sgn_aggregate_train_fwd(pt, q, S_capacity, K, d_packed, d_out_feat, d_fs, saved, stream);
    SGN_REQUIRE(pt && q && d_packed && d_out_feat && d_fs && saved && d_h2b, "null argument");
    SGN_REQUIRE(saved->x0 && saved->h1 && saved->h2 && saved->h3, "null saved-activation buffer");
    SGN_REQUIRE(ksb <= KS_HID || (d_bpnet_f16 && ((uintptr_t)d_bpnet_f16 & 15) == 0),
                "bpnet_dim > 0 needs the 16-byte aligned fp16 BPNet point embedding");
    SGN_REQUIRE(K >= 1 && K <= 8, "the MFMA aggregator takes K = 1 .. 8 neighbours per sample");
    SGN_REQUIRE(pt->campos && pt->camrotc2w && pt->raydir && !pt->pers, "camera required, no precomputed pers");
    SGN_REQUIRE(S_capacity >= 0 && S_capacity < (1 << 27), "S_capacity out of range");
    if (S_capacity == 0) return 0;
    AggArgs a{};
    a.xyz = pt->xyz; a.emb = pt->embedding; a.color = pt->color; a.dir = pt->dir; a.conf = pt->conf;
    a.campos = pt->campos; a.rot = pt->camrotc2w; a.raydir = pt->raydir;
    a.counters = q->counters; a.work = q->work; a.samp_ray = q->samp_ray; a.pidx = q->pidx;
    a.samp_locw = q->samp_locw;
    a.K = K;
    a.blob = d_packed; a.blob_bytes = total_bytes_sg(ksb);
    a.bpnet = (const _Float16 *)d_bpnet_f16;
    a.feat = d_out_feat; a.fs = (_Float16 *)d_fs;
    a.item0 = 0; a.n_items = (int32_t)S_capacity;
    a.sx0 = (_Float16 *)saved->x0; a.sh1 = (_Float16 *)saved->h1; a.sh2 = (_Float16 *)saved->h2;
    a.sh3 = (_Float16 *)saved->h3; a.sh2b = (_Float16 *)d_h2b;
    const int64_t wg = (S_capacity + WG_SAMPLES - 1) / WG_SAMPLES;
    auto kern = ksb == KS_HID ? k_agg_rows<KS_HID, true> : k_agg_rows<ks_bp(BP_DIM), true>;
    hipLaunchKernelGGL(kern, dim3((unsigned)(wg < 256 ? wg : 256)), dim3(ROWS_TPB), 0, as_stream(stream), a);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

/* Index maps of the SG blob's block2_bpnet sections over the flat parameter vector (the 9 base
 * layers, then block2_bpnet.0 weight [256][256 + bpnet_dim] and bias): which 3: fragments
 * [OFF_WB, off_bb) as fp16 elements, 4: the bias (HID fp32, accumulator order). */
int sgn_mlp_pack_index_sg(int32_t bpnet_layers, int32_t bpnet_dim, int32_t which, int32_t *out, int64_t n) {
    using namespace sgn;
    using namespace sgn::mlp;
    const int ksb = mlp_variant_ksb(bpnet_layers, bpnet_dim);
    SGN_REQUIRE(ksb > 0, "sgn_mlp_pack_index_sg: block2_bpnet variant required");
    const int64_t want = which == 3 ? (int64_t)((off_bb(ksb) - OFF_WB) / 2) : which == 4 ? (int64_t)HID : -1;
    SGN_REQUIRE(out && n == want, "sgn_mlp_pack_index_sg: bad map id or size");
    static const int shape[9][2] = {{256, 284}, {256, 256}, {256, 263}, {256, 256}, {1, 256},
                                    {128, 280}, {128, 128}, {128, 128}, {3, 128}};
    std::vector<std::vector<float>> wi(10), bi(10);
    std::vector<const float *> wp(10), bp(10);
    int64_t off = 0;
    for (int L = 0; L < 10; ++L) {
        const int o = L < 9 ? shape[L][0] : 256, i = L < 9 ? shape[L][1] : 256 + bpnet_dim;
        wi[L].resize((size_t)o * i);
        for (size_t j = 0; j < wi[L].size(); ++j) wi[L][j] = (float)(off + (int64_t)j + 1);
        off += (int64_t)wi[L].size();
        bi[L].resize(o);
        for (size_t j = 0; j < bi[L].size(); ++j) bi[L][j] = (float)(off + (int64_t)j + 1);
        off += (int64_t)bi[L].size();
        wp[L] = wi[L].data();
        bp[L] = bi[L].data();
    }
    std::vector<float> e16(total_bytes_sg(ksb) / 2, 0.f), F(N_F32, 0.f), BB(HID, 0.f);
    pack_blob<float>(ksb, bpnet_dim, wp.data(), bp.data(), e16.data(), F.data(), BB.data());
    const float *src = which == 3 ? e16.data() + OFF_WB / 2 : BB.data();
    for (int64_t j = 0; j < n; ++j) out[j] = (int32_t)src[j];
    return 0;
}

int sgn_bpnet_pack(const float *d_embedding, int64_t n_points, int32_t bpnet_dim, void *d_out_f16,
                   sgn_stream_t stream) {
    using namespace sgn;
    SGN_REQUIRE(n_points >= 0 && bpnet_dim == mlp::BP_DIM, "bpnet_dim must be 96");
    SGN_REQUIRE(n_points == 0 || (d_embedding && d_out_f16), "null argument");
    SGN_REQUIRE(((uintptr_t)d_embedding & 15) == 0 && ((uintptr_t)d_out_f16 & 15) == 0, "16-byte alignment required");
    const int64_t n = n_points * bpnet_dim;
    if (n == 0) return 0;
    int64_t blocks = (n / 4 + 255) / 256;
    hipLaunchKernelGGL(k_to_f16, dim3((unsigned)(blocks < 4096 ? blocks : 4096)), dim3(256), 0, as_stream(stream),
                       d_embedding, (_Float16 *)d_out_f16, n);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

int sgn_aggregate(const sgn_point_tables *pt, const sgn_query_out *q, int64_t S_capacity, int32_t K,
                  const void *d_packed, float *d_out_feat, float *d_out_blend, float *d_out_wnorm,
                  void *d_workspace, size_t workspace_bytes, int32_t stages, sgn_stream_t stream) {
    return sgn_aggregate_sg(0, 0, nullptr, nullptr, pt, q, S_capacity, K, d_packed, d_out_feat, d_out_blend, d_out_wnorm,
                            d_workspace, workspace_bytes, stages, stream);
}

}  // extern "C"
