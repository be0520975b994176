// mlp_x3.hip -- fp32-faithful neural-point aggregator on fp16 MFMA (gfx950): every fp32
// product of the reference's nn.Linear layers is carried as three fp16 MFMA products.
//
// Path: NeuralPoints gather (neural_points.py:942-988), PointAggregator.forward / viewmlp
// (point_aggregators.py:868-959, :561-786), at the reference's arithmetic precision:
//
//   w = 2^-s (w_hi + w_lo), x = x_hi + x_lo, all four fp16; w x ~ 2^-s (w_hi x_hi + w_hi x_lo + w_lo x_hi)
//
// with fp32 accumulation (an fp16 x fp16 product is exact in fp32).  The weights of each layer are
// pre-scaled by a power of two 2^s (max |w| 2^s < 2^14) so w_lo stays a normal fp16 number; the
// epilogue multiplies by 2^-s exactly.  Per product the representation error is <= 2^-22 |w x|
// (+ 2^-25 |w| for activations below fp16's normal range), the dropped w_lo x_lo term <= 2^-22
// |w x|: the layer sums agree with an fp32 evaluation to a few fp32 ulps of sum |w x|.
// Activations must stay inside fp16's range (|x| < 65504): an activation outside it turns into
// inf / NaN in the MFMA operands, which k_color16 detects on the sample's decoded features and
// reports through the sticky range flag (counters[3], sgn_aggregate_check) -- never silently.
// The positional encodings use accurate sin/cos of the scaled argument (x 2^f is exact), as
// torch.sin does (networks.py:175-192).  dtype of this path: "f32 (3xf16 split MFMA, fp32
// accumulate)"; 3 MFMAs per product, so its MFMA ceiling is 1/3 of the fp16 dense peak.
//
// Kernels (v_mfma_f32_16x16x32_f16, 8 waves per 512-thread workgroup, two per SIMD):
//   k_point_proj16 : P[p] = 2^s0 (W0a [feat | PE(feat)] + b0) fp32 [256] + the packed 64-B point
//                    record, once per point-cloud version
//   k_pair_slots   : packs two samples whose neighbour counts sum to <= 8 into one 8-row half
//   k_rows16       : 16 samples x 8 neighbours per tile: block1.0's PE(dists) part on top of
//                    P[pid], block1.2, (block2_bpnet), block3.0, block3.2 (transposed), alpha,
//                    K-blend -> f_s fp32
//   k_color16      : 8 waves x 16 samples: [f_s | PE(viewdir)] -> 128 -> 128 -> 128 -> 3, sigmoid
// Weight fragment pairs (hi, lo) stream through a 2-slot LDS ring of 64-KiB chunks filled by
// LDS-DMA, shared by the workgroup's 8 waves.
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cmath>
#include <utility>
#include <vector>

#include "agg_device.h"
#include "x3_split.h"

namespace sgn {
namespace {
namespace x3 {

constexpr int NW16 = 8, TPB16 = NW16 * 64;
constexpr int PAIR = 2048;        // hi fragment (1 KiB) then lo fragment (1 KiB)
constexpr int SLOT_PAIRS = 32;
constexpr int SLOT = SLOT_PAIRS * PAIR;  // 64 KiB
constexpr int NSLOT = 2;
constexpr int PD = 2;     // fragment pairs in flight per wave (LDS -> VGPR queue)
constexpr size_t PROJ_BYTES_PER_POINT = HID * 4;  // P row: fp32 [256], natural unit order
struct XL {
    int ks, tp, np, kc;
    uint32_t off;
};
__host__ __device__ constexpr int nch(XL l) { return (l.ks + l.kc - 1) / l.kc; }
__host__ __device__ constexpr int nk(XL l, int c) { return l.ks - c * l.kc < l.kc ? l.ks - c * l.kc : l.kc; }

template <class Net>
struct Sched {
    static constexpr int layer_chunks(int l) { return Net::L[l].np * nch(Net::L[l]); }
    static constexpr int base(int l) { return l == 0 ? 0 : base(l - 1) + layer_chunks(l - 1); }
    static constexpr int total() { return base(Net::NL); }
    static constexpr int idx(int l, int p, int c) { return base(l) + p * nch(Net::L[l]) + c; }
    static constexpr int cl(int n, int l = 0) { return (l + 1 >= Net::NL || n < base(l + 1)) ? l : cl(n, l + 1); }
    static constexpr int cp(int n) { return (n - base(cl(n))) / nch(Net::L[cl(n)]); }
    static constexpr int cc(int n) { return (n - base(cl(n))) % nch(Net::L[cl(n)]); }
    static constexpr uint32_t off(int n) {
        return Net::L[cl(n)].off +
               (uint32_t)((cp(n) * Net::L[cl(n)].ks + cc(n) * Net::L[cl(n)].kc) * Net::L[cl(n)].tp) * PAIR;
    }
    static constexpr int pairs(int n) { return nk(Net::L[cl(n)], cc(n)) * Net::L[cl(n)].tp; }
};
struct X3B {
    h8 hi, lo;
};

// x -> (hi, lo): hi = fp16(x), lo = fp16(x - hi) (the difference is exact in fp32)
__device__ __forceinline__ X3B split8(const float (&v)[8]) {
    const X3Pair p = split8_unit(v);
    return X3B{p.hi, p.lo};
}

// LeakyReLU(0.01) exactly as the reference (x, or fp32(0.01 x) below zero): max(x, 0.01 x) as one
// v_max_f32 in inline asm -- fmaxf on an MFMA result makes the compiler canonicalise the operand with an
// extra v_max_f32 x, x, x first (IEEE mode); NaN / inf still propagate (the fp16-range guard).  The asm
// writes into the register of 0.01 x ("+v", tied; see split8_unit for why)
__device__ __forceinline__ float lrelu_x3(float a) {
    float r = 0.01f * a;
    asm("v_max_f32 %0, %1, %0" : "+v"(r) : "v"(a));
    return r;
}
// LeakyReLU(2^-s a) as the next layer's (hi, lo) fragment (LeakyReLU commutes with the exact
// power-of-two scaling)
__device__ __forceinline__ X3B lrelu_split8(const float (&a)[8], float inv) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = lrelu_x3(a[j] * inv);
    return split8(v);
}

// one 1-KiB LDS-DMA piece of wave w: 16 B per lane from blob byte offset soff + w * 1024 + lane * 16 into
// LDS dst + w * 1024 (+ lane * 16).  The constant part of the offset is made opaque at its use, so the
// compiler materialises it right there (one s_mov) instead of hoisting ~70 per-tile offsets into
// SGPRs that then spill into VGPR lanes.
__device__ __forceinline__ void lds_dma_1k(const WBlob &wb, char *dst, int w, int lane, uint32_t soff) {
    asm volatile("" : "+s"(soff));
    __builtin_amdgcn_raw_ptr_buffer_load_lds(wb.rsrc, (__attribute__((address_space(3))) void *)(dst + w * 1024), 16,
                                             lane * 16 + w * 1024, soff, 0, 0);
}

// LDS-DMA of stream chunk N into `dst`: 2 * pairs 1-KiB pieces, wave w (of NWv) moves pieces
// w + NWv j
template <class Net, int N, int NWv = NW16>
__device__ __forceinline__ void dma_chunk(const WBlob &wb, char *dst, int w, int lane, int) {
    using S = Sched<Net>;
    constexpr int nf = 2 * S::pairs(N);
    static_for<(nf + NWv - 1) / NWv>([&](auto jj) {
        constexpr int J = decltype(jj)::value;
        const int i = w + NWv * J;
        if (NWv * (J + 1) <= nf || i < nf)  // wave-uniform
            lds_dma_1k(wb, dst + NWv * J * 1024, w, lane, S::off(N) + (uint32_t)(NWv * J * 1024));
    });
}

// piece J (of this wave's PW = ceil(2 pairs / NWv)) of chunk N: wave w moves the contiguous pieces
// w PW .. w PW + PW - 1, so four consecutive pieces share one soffset / M0 and the instruction offset
// (0 .. 3 KiB, applied to the blob address and the LDS address alike) steps through them: one s_mov pair per
// four pieces instead of per piece (the initial dma_chunk keeps the interleaved assignment)
template <class Net, int N, int J, int NWv = NW16>
__device__ __forceinline__ void dma_piece(const WBlob &wb, char *dst, int w, int lane, int) {
    using S = Sched<Net>;
    constexpr int nf = 2 * S::pairs(N);
    constexpr int PW = (nf + NWv - 1) / NWv;
    const int i = w * PW + J;
    if (nf % NWv == 0 || i < nf) {  // wave-uniform
        uint32_t soff = S::off(N) + (uint32_t)((J & ~3) * 1024);
        asm volatile("" : "+s"(soff));
        __builtin_amdgcn_raw_ptr_buffer_load_lds(wb.rsrc,
                                                 (__attribute__((address_space(3))) void *)(dst + (w * PW + (J & ~3)) * 1024),
                                                 16, lane * 16 + w * PW * 1024, soff, (J & 3) * 1024, 0);
    }
}
template <class Net, int N, int NWv = NW16>
constexpr int dma_pieces() { return (2 * Sched<Net>::pairs(N) + NWv - 1) / NWv; }

__device__ __forceinline__ int cur_slot(int s) { return s; }
__device__ __forceinline__ int dma_slot(int s) { return s ^ 1; }
__device__ __forceinline__ void chunk_exit(int &s, int) { s ^= 1; }

// chunk boundary: this wave's DMAs of chunk N landed, LDS reads drained, barrier; then chunk N+1
// goes into the slot every wave finished reading one chunk ago (its pieces are spread over the
// chunk's MFMAs by run_layer16)
// VM: vector-memory operations this wave is guaranteed to have issued after its last DMA piece of
// the chunk being entered (loads placed at the end of the previous chunk, stores): they may stay in
// flight across the boundary (vmcnt retires in order, so the DMA has landed once at most VM remain)
template <class Net, int N, int NWv = NW16, int VM = 0>
__device__ __forceinline__ void chunk_enter(const WBlob &, char *, int, int, int, int) {
    static_assert(VM >= 0 && VM < 64, "vmcnt range");
    if constexpr (VM == 0)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else  // vmcnt[3:0] | expcnt 7 | lgkmcnt 15 | vmcnt[5:4] << 14 (gfx9 encoding: wait on vmcnt only)
        __builtin_amdgcn_s_waitcnt((VM & 15) | (7 << 4) | (15 << 8) | ((VM >> 4) << 14));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
}

struct NoHook {
    template <class C>
    __device__ void operator()(C) const {}
};
// vmcnt allowance at the entry of chunk C of a layer (chunk_enter's VM)
struct VmZero {
    static constexpr int vm(int) { return 0; }
};


// accurate sin/cos of x 2^F (the scaling is exact; torch.sin on the product, networks.py:186)
template <int F>
__device__ __forceinline__ void sincos_f(float x, float &s, float &c) {
    sincos_acc(x * (float)(1 << F), s, c);
}
// =====================================================================================
// 2 waves per SIMD: v_mfma_f32_16x16x32_f16, 8 waves x 16 rows (2 samples x K = 8) per
// 128-row workgroup tile.  A wave's registers hold 16 rows (hi/lo layer input 64, all 16 output
// tiles' accumulators 64), so two waves share a SIMD and hide each other's LDS-DMA issue,
// epilogue VALU and gather latency.  Each 1-KiB weight fragment (16 units x 32 inputs) serves
// 8 waves.  Lane l: row r = l & 15, group g = l >> 4.  A operand: A[unit l&15][k 8g+j];
// B operand: B[k 8g+j][row l&15]; D: lane holds D[unit 4g+i][row l&15] (i = 0..3) of its tile,
// i.e. units 16 t + 4 g + i of tile t -- natural order, so P and the biases are natural-order
// vectors.  Chained layers: k-step s of the next layer takes tiles 2s, 2s+1 of this one as
// element j <- unit 16 (j >> 2) + 4 g + (j & 3) (perm16, folded into the packed weights).
// =====================================================================================
constexpr uint32_t OFF16_BASE = 0;
constexpr uint32_t OFF16_W0B = OFF16_BASE;                  // block1.0 PE(dists): 2 ks x 16 tiles
constexpr uint32_t OFF16_W1 = OFF16_W0B + 32 * PAIR;        // block1.2: 8 x 16
constexpr uint32_t OFF16_W2 = OFF16_W1 + 128 * PAIR;        // block3.0: 9 x 16
constexpr uint32_t OFF16_W3 = OFF16_W2 + 144 * PAIR;        // block3.2: 8 x 16 (transposed use)
constexpr uint32_t OFF16_W0A = OFF16_W3 + 128 * PAIR;       // block1.0 per point: 7 x 16
constexpr uint32_t OFF16_WB = OFF16_W0A + 112 * PAIR;       // block2_bpnet.0 (SG): 8 + 3 x 16
constexpr uint32_t OFF16_C0 = OFF16_WB + 176 * PAIR;        // colour 0: [f_s | PE(v)] 280 -> 128: 9 x 8
constexpr uint32_t OFF16_C1 = OFF16_C0 + 72 * PAIR;         // colour 1: 128 -> 128: 4 x 8
constexpr uint32_t OFF16_C2 = OFF16_C1 + 32 * PAIR;         // colour 2: 4 x 8
constexpr uint32_t OFF16_F32 = OFF16_C2 + 32 * PAIR;
// natural-order fp32 section of the 16x16 kernels
constexpr int Y_B0 = 0, Y_B1 = 256, Y_B2 = 512, Y_B3 = 768, Y_WA = 1024, Y_BB = 1280, Y_BA = 1536, Y_INV = 1537;
// colour (k_color16): biases of colour 0..2 (scaled by 2^s), the output layer [3][128] and its bias
constexpr int Y_CB0 = Y_INV + 8 + 3, Y_CB1 = Y_CB0 + 128, Y_CB2 = Y_CB1 + 128, Y_CW3 = Y_CB2 + 128, Y_CB3 = Y_CW3 + 384;
constexpr int N_Y32 = Y_CB3 + 4;  // 2320 (multiple of 4)
constexpr size_t BLOB_BYTES_ALL = OFF16_F32 + (size_t)N_Y32 * 4;
__host__ __device__ constexpr size_t blob_bytes_sg(int) { return BLOB_BYTES_ALL; }
static_assert(N_Y32 % 4 == 0, "fp32 section in 16-B units");

// block3.2 in two passes of 8 output tiles: pass 0 converts the input once and keeps it
// as (hi, lo) fragments, and the epilogue (K-blend, alpha) of its 8 tiles runs between pass 1's MFMAs
// Row kernel workgroup (4 waves): 4 waves (one per SIMD) with a 2 x 32-KiB ring, so two
// workgroups share a CU and their waves pair up on each SIMD without a common barrier (the barrier
// of one chunk boundary no longer holds the other workgroup's wave of the SIMD: while one runs its
// tile transition or epilogue VALU, the other's MFMAs keep the matrix pipe busy)
constexpr int NWR = 4;                            // row waves
constexpr int NSLR = NSLOT;                       // row ring slots
static_assert(NWR == 4, "row workgroup: 4 waves");
// ring slot of SP fragment pairs: 16 (NS = 1, two workgroups per CU) or 32 (NS = 2, one per CU);
// KC = SP / 16 k-steps of 16 tiles per chunk
template <int SP_>
struct NetR16T {
    static constexpr int NW = NWR, SP = SP_;  // waves sharing the ring, fragment pairs per ring slot
    static constexpr int KC = SP_ / 16;
    static constexpr int NL = 4;
    static constexpr XL L[NL] = {{2, 16, 1, KC, OFF16_W0B}, {8, 16, 1, KC, OFF16_W1}, {9, 16, 1, KC, OFF16_W2},
                                 {8, 8, 2, 2 * KC, OFF16_W3}};
};
template <int KB, int SP_>
struct NetR16SGT {
    static constexpr int NW = NWR, SP = SP_;
    static constexpr int KC = SP_ / 16;
    static constexpr int NL = 5;
    static constexpr XL L[NL] = {{2, 16, 1, KC, OFF16_W0B}, {8, 16, 1, KC, OFF16_W1}, {KB, 16, 1, KC, OFF16_WB},
                                 {9, 16, 1, KC, OFF16_W2}, {8, 8, 2, 2 * KC, OFF16_W3}};
};
struct NetProj16 {
    static constexpr int NW = NW16, SP = SLOT_PAIRS;
    static constexpr int NL = 1;
    static constexpr XL L[NL] = {{7, 16, 1, 2, OFF16_W0A}};
};
// colour kernel workgroup (8 waves), as the row kernel's
constexpr int NWC = 8, SPC = NWC == 4 ? 16 : 32, KCC = SPC / 8;
static_assert(NWC == 4 || NWC == 8, "colour workgroup: 4 or 8 waves");
struct NetColor16 {
    static constexpr int NW = NWC, SP = SPC;
    static constexpr int NL = 3;
    static constexpr XL L[NL] = {{9, 8, 1, KCC, OFF16_C0}, {4, 8, 1, KCC, OFF16_C1}, {4, 8, 1, KCC, OFF16_C2}};
};
static_assert(Sched<NetR16T<16>>::total() == 27 && Sched<NetR16T<32>>::total() == 14 &&
                  Sched<NetR16T<32>>::pairs(9) == 16, "16x16 row stream");
static_assert(NWC == 4 ? Sched<NetColor16>::total() == 9 && Sched<NetColor16>::pairs(4) == 8
                       : Sched<NetColor16>::total() == 5 && Sched<NetColor16>::pairs(2) == 8, "16x16 colour stream");

__device__ __forceinline__ f32x4 mfma16(h8 a, h8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// the B fragments of one k-step for NS row sets of 16 rows each
template <int NS>
struct X3S {
    X3B b[NS];
};

// One layer, k-outer over all output tiles of pass P: acc[s][AOFF + t] += W[t] in(k).b[s], three MFMAs
// per (k-step, tile, row set), next chunk's LDS-DMA pieces spread over the first pairs.  Each weight
// fragment pair read from LDS feeds 3 NS MFMAs.  TRANS: activations are the A operand (acc[s][t]
// holds D[row 4g+i][unit 16t + (l & 15)]).
// mid(integral_constant F) runs after pair F's MFMAs of every chunk (F counted over the layer: k-step
// K, tile t -> F = K TP + t), so per-pair VALU work of another stage can ride between the MFMAs.
// PIPE: k-step K + 1's input (in) is converted halfway through k-step K's MFMAs (k-step 0's before the
// layer's first chunk boundary), so a chunk's MFMAs start right after its boundary instead of behind the
// conversion VALU.  Per pair the lo fragment (read after hi) feeds the first MFMA, so one lgkmcnt wait
// covers both fragments.
template <class Net, int L, bool TRANS = false, class Vm = VmZero, int P = 0, int AOFF = 0, bool PIPE = false,
          int NS, int NA, class SlotT, class InFn, class PostFn = NoHook, class EndFn = NoHook, class MidFn = NoHook>
__device__ __forceinline__ void run_layer_ns(const WBlob &wb, char *lds, SlotT &slot, int w, int lane, int lz,
                                             f32x4 (&acc)[NS][NA], InFn &&in, PostFn &&post = PostFn{},
                                             EndFn &&end = EndFn{}, MidFn &&mid = MidFn{}) {
    constexpr XL ly = Net::L[L];
    constexpr int TP = ly.tp;
    static_assert((TP == 16 || TP == 8) && P < ly.np, "passes of 16 or 8 output tiles");
    static_assert(AOFF + TP <= NA, "accumulator view");
    X3S<NS> Bn;
    if constexpr (PIPE) Bn = in(std::integral_constant<int, 0>{});
    static_for<nch(ly)>([&](auto cc) {
        constexpr int C = decltype(cc)::value;
        constexpr int N = Sched<Net>::idx(L, P, C), NN = (N + 1) % Sched<Net>::total();
        constexpr int NWv = Net::NW, SLOTv = Net::SP * PAIR;
        static_assert(nk(ly, C) * TP <= Net::SP, "chunk larger than a ring slot");
        chunk_enter<Net, N, NWv, Vm::vm(C)>(wb, lds, slot, w, lane, lz);
        post(cc);
        const char *sl = lds + cur_slot(slot) * SLOTv;
        char *dnext = lds + dma_slot(slot) * SLOTv;
        constexpr int NF = nk(ly, C) * TP;
        constexpr int PW = dma_pieces<Net, NN, NWv>();
        auto frag = [&](int f, int part) { return *(const h8 *)(sl + (2 * f + part) * 1024 + lane * 16); };
        h8 fh[PD], fl[PD];
#pragma unroll
        for (int f = 0; f < PD; ++f) {
            fh[f] = frag(f, 0);
            fl[f] = frag(f, 1);
        }
        __builtin_amdgcn_sched_group_barrier(0x100, 2 * PD, 0);
        static_for<nk(ly, C)>([&](auto kk) {
            constexpr int KK = decltype(kk)::value;
            // NS = 2 without PIPE (the save mode): a k-step's input conversion stays inside its k-step, so
            // the B fragments of two k-steps are never live together
            constexpr int KS = C * ly.kc + KK;
            if constexpr (NS > 1 && KK > 0 && !PIPE) __builtin_amdgcn_sched_barrier(0);
            X3S<NS> B;
            if constexpr (PIPE) B = Bn;
            else B = in(std::integral_constant<int, KS>{});
            static_for<TP>([&](auto tt) {
                constexpr int t = decltype(tt)::value, F = KK * TP + t;
                const h8 Ah = fh[F % PD], Al = fl[F % PD];
                if constexpr (F + PD < NF) {
                    fh[F % PD] = frag(F + PD, 0);
                    fl[F % PD] = frag(F + PD, 1);
                }
#pragma unroll
                for (int s = 0; s < NS; ++s) {
                    f32x4 &c = acc[s][AOFF + t];
                    if constexpr (TRANS) {
                        c = mfma16(B.b[s].hi, Al, c);
                        c = mfma16(B.b[s].lo, Ah, c);
                        c = mfma16(B.b[s].hi, Ah, c);
                    } else {
                        c = mfma16(Al, B.b[s].hi, c);
                        c = mfma16(Ah, B.b[s].lo, c);
                        c = mfma16(Ah, B.b[s].hi, c);
                    }
                }
                constexpr int NSP = NF / 2 > 0 ? NF / 2 : 1;
                if constexpr (F < NSP) {
                    static_for<(F + 1) * PW / NSP - F * PW / NSP>([&](auto jj) {
                        dma_piece<Net, NN, F * PW / NSP + decltype(jj)::value, NWv>(wb, dnext, w, lane, lz);
                    });
                }
                mid(std::integral_constant<int, (C * ly.kc + KK) * TP + t>{});
                // (the clamped index keeps the discarded instantiation of the last k-step in range)
                if constexpr (PIPE && t == TP / 2 - 1 && KS + 1 < ly.ks)
                    Bn = in(std::integral_constant<int, (KS + 1 < ly.ks ? KS + 1 : KS)>{});
                if constexpr (NS == 1) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                } else {
                    __builtin_amdgcn_sched_group_barrier(0x008, 3 * NS / 2, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 3 * NS - 3 * NS / 2, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                }
            });
        });
        __builtin_amdgcn_sched_barrier(0);
        end(cc);  // after every DMA piece of the chunk: loads here may stay in flight one boundary
        chunk_exit(slot, lane);
        __builtin_amdgcn_sched_barrier(0);
    });
}

// one row set (16 rows / units of the accumulators): the layer loop above with NS = 1
template <class Net, int L, bool TRANS = false, class Vm = VmZero, int P = 0, class SlotT, class InFn,
          class PostFn = NoHook, class EndFn = NoHook, class MidFn = NoHook>
__device__ __forceinline__ void run_layer16(const WBlob &wb, char *lds, SlotT &slot, int w, int lane, int lz,
                                            f32x4 (&acc)[Net::L[L].tp], InFn &&in, PostFn &&post = PostFn{},
                                            EndFn &&end = EndFn{}, MidFn &&mid = MidFn{}) {
    constexpr int TP = Net::L[L].tp;
    run_layer_ns<Net, L, TRANS, Vm, P, 0>(wb, lds, slot, w, lane, lz, reinterpret_cast<f32x4(&)[1][TP]>(acc),
                                          [&](auto k) { return X3S<1>{{in(k)}}; }, post, end, mid);
}

// LeakyReLU(2^-s acc + add) of 16 tiles -> the next layer's 8 k-step B fragments (hi/lo)
template <bool ADD>
__device__ __forceinline__ void chain_out16(const f32x4 (&acc)[16], const f32x4 (&add)[16], float inv, X3B (&out)[8]) {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float a = acc[2 * s + (j >> 2)][j & 3];
            const float y = ADD ? (a + add[2 * s + (j >> 2)][j & 3]) * inv : a * inv;
            v[j] = fmaxf(y, 0.01f * y);
        }
        out[s] = split8(v);
    }
}

// ---- per-point block1.0 projection (16x16): P[p] fp32 [256] in natural unit order ----
struct Proj16Args {
    const float *emb;
    int64_t n;
    const void *blob;
    float *proj;
    const float *xyz, *color, *dir, *conf;
    float *rec;  // [n][16] packed point records (AggArgs::rec), after P in the projection buffer
    const int32_t *idx;    // optional: project only points idx[0 .. *n_dev) (a training step's touched rows)
    const int64_t *n_dev;  // device count of idx (<= n)
};
constexpr int REC16_FLOATS = 16;
constexpr int Y_LDS_OFF = NSLOT * SLOT;
constexpr int PROJ16_LDS = Y_LDS_OFF + N_Y32 * 4;

__global__ __launch_bounds__(TPB16, 1) void k_point_proj16(Proj16Args a) {
    __shared__ __attribute__((aligned(16))) char lds[PROJ16_LDS];
    const int lane = threadIdx.x & 63, g = lane >> 4;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const WBlob wb = make_blob(a.blob, BLOB_BYTES_ALL);
    {
        const float *src = (const float *)((const char *)a.blob + OFF16_F32);
        float *dst = (float *)(lds + Y_LDS_OFF);
        for (int i = threadIdx.x; i < N_Y32; i += TPB16) dst[i] = src[i];
    }
    __syncthreads();
    int slot = 0;
    dma_chunk<NetProj16, 0, NW16>(wb, lds, w, lane, 0);
    const int64_t n = a.idx ? min(*a.n_dev, a.n) : a.n;
    const int64_t ntile = (n + 16 * NW16 - 1) / (16 * NW16);
    for (int64_t tile = blockIdx.x; tile < ntile; tile += gridDim.x) {
        int lz = 0;
        asm volatile("" : "+s"(lz));
        const float *Yl = (const float *)(lds + lz + Y_LDS_OFF);
        const int64_t j = tile * (16 * NW16) + w * 16 + (lane & 15);
        const bool ok = j < n;
        const int64_t p = a.idx ? (ok ? (int64_t)a.idx[j] : 0) : j;
        // lane group g owns features 8 g .. 8 g + 7: k-step 0 slot j = feat[8 g + j]; k-step S >= 1
        // slot j = PE channel q = 8 (S - 1) + j of those features (feature 8 g + q / 6, frequency
        // (q % 6) / 2, sin / cos for even / odd q) -- col_proj16 maps it to the reference column
        float f8[8];
        {
            const f32x4 *e4 = (const f32x4 *)(a.emb + (ok ? p : 0) * 32 + 8 * g);
            const f32x4 u0 = e4[0], u1 = e4[1];
            f8[0] = u0[0]; f8[1] = u0[1]; f8[2] = u0[2]; f8[3] = u0[3];
            f8[4] = u1[0]; f8[5] = u1[1]; f8[6] = u1[2]; f8[7] = u1[3];
        }
        f32x4 acc[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) acc[t] = *(const f32x4 *)(Yl + Y_B0 + 16 * t + 4 * g);
        auto in = [&](auto k) {
            constexpr int S = decltype(k)::value;
            float v[8];
            if constexpr (S == 0) {
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = f8[j];
            } else {
                static_for<4>([&](auto jp) {
                    constexpr int q = 8 * (S - 1) + 2 * decltype(jp)::value, dl = q / 6, f = (q % 6) / 2;
                    float sv, cv;
                    sincos_f<f>(f8[dl], sv, cv);
                    v[2 * decltype(jp)::value] = sv;
                    v[2 * decltype(jp)::value + 1] = cv;
                });
            }
            return split8(v);
        };
        // the point's packed record, lane group g's 16-B quarter: loaded here, stored after the
        // MFMAs (which hide the loads)
        f32x4 q{};
        {
            const float *src = g == 0 ? a.xyz : g == 1 ? a.color : a.dir;
            const int64_t pc = ok ? p : 0;
            if (g < 3) q = f32x4{src[pc * 3], src[pc * 3 + 1], src[pc * 3 + 2], g == 0 ? a.conf[pc] : 0.f};
        }
        run_layer16<NetProj16, 0>(wb, lds + lz, slot, w, lane, lz, acc, in);
        if (ok) {  // natural unit order: tile t of lane group g at 16 t + 4 g (64 B per point per store)
            float *dst = a.proj + p * HID + 4 * g;
#pragma unroll
            for (int t = 0; t < 16; ++t) *(f32x4 *)(dst + 16 * t) = acc[t];
            *(f32x4 *)(a.rec + p * REC16_FLOATS + 4 * g) = q;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---- per-neighbour rows (16x16) -------------------------------------------------------------
constexpr int WG16_SAMPLES = NWR * 2;            // halves (16 rows, 2 per wave) per workgroup tile
constexpr int TPBR = NWR * 64;
// the row kernel's LDS: ring (NSLR slots of SP pairs), fp32 section, then [unit r][20] 2^s3 b3
// (t = 0..15) and [r][20] 2^-s3 alpha w
__host__ __device__ constexpr int yr_off(int sp) { return NSLR * sp * PAIR; }
__host__ __device__ constexpr int yt16_off(int sp) { return yr_off(sp) + N_Y32 * 4; }
__host__ __device__ constexpr int rows16_lds(int sp) { return yt16_off(sp) + 2 * 16 * 20 * 4; }
static_assert(2 * rows16_lds(16) <= 163840, "LDS budget (16x16 rows)");

// row r's point record, its sample position and view direction (+ the caller's pers
// coordinates on the compatibility path)
template <bool PERS>
struct Rec16 {
    float p[3], col[3], dir[3], cf, l[3], v[3];
    float pp[PERS ? 3 : 1], pl[PERS ? 3 : 1];  // the caller's pers coordinates (PointAggregator path only)
};
// Rows without a work item (ix.sval false: the tail of the work list, or a launch with no
// samples at all, where samp_ray holds no written entry) read nothing.
// The point's attributes come from its packed 64-B record (three 16-B loads on one cache line,
// instead of ten dword gathers from four tables).
// The nine loads of the record, sample position and ray direction are issued unconditionally (rows
// without a work item or neighbour read the weight blob instead and select zeros), so a caller may
// count them (REC16_LOADS) in a chunk boundary's vmcnt allowance.
constexpr int REC16_LOADS = 9;
template <bool PERS>
__device__ __forceinline__ Rec16<PERS> load_rec16(const AggArgs &a, const RowIdx &ix) {
    Rec16<PERS> r;
    const bool v = ix.sval;
    const int pid = ix.pid, s = ix.s, ray = ix.ray;
    const bool m = v && pid >= 0;
    const float *dummy = (const float *)a.blob;
    const f32x4 *rp = (const f32x4 *)(m ? a.rec + (int64_t)pid * REC16_FLOATS : dummy);
    const float *lp = v ? a.samp_locw + (int64_t)s * 3 : dummy;
    const float *vp = v ? a.raydir + (int64_t)ray * 3 : dummy;
    const f32x4 q0 = rp[0], q1 = rp[1], q2 = rp[2];
    float l3[3], v3[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        l3[c] = lp[c];
        v3[c] = vp[c];
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        r.p[c] = m ? q0[c] : 0.f;
        r.col[c] = m ? q1[c] : 0.f;
        r.dir[c] = m ? q2[c] : 0.f;
        r.l[c] = v ? l3[c] : 0.f;
        r.v[c] = v ? v3[c] : 0.f;
        if constexpr (PERS) {
            r.pp[c] = m ? a.pers[(int64_t)pid * 3 + c] : 0.f;
            r.pl[c] = v ? a.samp_pers[(int64_t)s * 3 + c] : 0.f;
        }
    }
    r.cf = m ? q0[3] : 0.f;
    return r;
}
// vmcnt allowances of k_rows16's boundaries (chunk_enter VM), per row set of the wave: block3.2 ends its
// first chunk with the next tile's record (REC16_LOADS loads) and this tile's slot entry (1), the
// youngest; after block3.2 come the next tile's 16 P loads (and the epilogue's f_s stores, masked per
// segment, so not counted), all younger than block1.0's DMA
// The save mode (training) waits vmcnt(0) at every boundary instead: its z stores inside the k-loops
// let these counts pass with a weight LDS-DMA piece still in flight (a few samples a frame read stale
// block3.2 weights, run to run; tools/f32_repeat.py)
template <int NS>
struct VmL3P0 {
    static constexpr int vm(int c) { return c == 1 ? NS * (REC16_LOADS + 1) : 0; }
};
template <int NS>
struct VmL0 {  // the P loads follow only the DMA of block1.0's first chunk
    static constexpr int vm(int c) { return c == 0 ? 16 * NS : 0; }
};

// ---- paired samples: k_rows16's 8-row halves ----------------------------------------------------
// A work item with n < 8 valid neighbours (a prefix of its K slots, KBuf) leaves 8 - n rows of its
// half idle: 11 % of the rows at config 2, where 21 % of the samples have 1..7 neighbours, about
// evenly spread over 1..7.  Two samples whose counts sum to <= 8 share one half: sample A on rows
// 0..nA-1, sample B on rows oB..oB+nB-1, oB = max(nA, 4), so B never spans the two lane groups of
// 4 rows the K-blend chains run in (the K-blend, the weight normalisation and alpha are then
// two-segment sums with the same bits as for a sample alone, see k_rows16).  Per 1024 consecutive work items (neighbours in the work list
// are neighbours in the frame, so the P gathers keep their locality) the items are ranked per count
// (stable), then paired 7+1, 6+2, 5+3, 4+4 in rank order and the leftover 1..4s consecutively;
// 8s and unpaired 5..7s run alone.  Writes per slot (half) the row table rows[8 slot + kk] =
// s * 8 + k (-1: idle row; s * 8 + k is the pidx index of the row) and the entry
// {A item | nA << 28, B item | nB << 28, A sample, B sample} (items relative to item0, < 2^28);
// slots of a block are contiguous, blocks in atomic order (a sample's values depend only on its
// block, so results do not depend on that order).
constexpr int PAIR_TPB = 1024, PAIR_NW = PAIR_TPB / 64;
__global__ __launch_bounds__(PAIR_TPB) void k_pair_slots(const int32_t *__restrict__ counters,
                                                         const int32_t *__restrict__ work,
                                                         const int32_t *__restrict__ nnb, int32_t item0,
                                                         int32_t n_items, int32_t pair, int32_t *__restrict__ rows,
                                                         int4 *__restrict__ slots, int32_t *__restrict__ slot_n) {
    __shared__ int wc[PAIR_NW][9], nt[9];  // per-wave counts -> exclusive per-wave offsets; totals
    __shared__ int16_t blist[9][PAIR_TPB];  // count -> rank -> thread
    __shared__ int ss[PAIR_TPB];            // thread -> sample
    __shared__ int8_t sc[PAIR_TPB];         // thread -> count
    __shared__ int wl[PAIR_NW], sbase;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int end = min(counters[1], item0 + n_items);
    // grid-stride over 1024-item blocks of the work list (the grid is sized for the capacity, the
    // list is known on the device only)
    for (int rel0 = blockIdx.x * PAIR_TPB; item0 + rel0 < end; rel0 += gridDim.x * PAIR_TPB) {
        __syncthreads();  // the previous block's LDS tables are read
        const int item = item0 + rel0 + tid;
        const bool ok = item < end;
        const int s = ok ? work[item] : 0;
        const int c = ok ? min(max(nnb[s], 1), 8) : 0;
        ss[tid] = s;
        sc[tid] = (int8_t)c;
        const uint64_t below = (1ull << lane) - 1ull;
        int rank = 0;
#pragma unroll
        for (int b = 1; b <= 8; ++b) {
            const uint64_t m = __ballot(c == b);
            if (c == b) rank = __popcll(m & below);
            if (lane == 0) wc[wv][b] = __popcll(m);
        }
        __syncthreads();
        if (tid >= 1 && tid <= 8) {  // one thread per count: offsets over the waves, the block's total
            int tot = 0;
            for (int q = 0; q < PAIR_NW; ++q) {
                const int v = wc[q][tid];
                wc[q][tid] = tot;
                tot += v;
            }
            nt[tid] = tot;
        }
        __syncthreads();
        if (ok) rank += wc[wv][c];
        int n[9];
#pragma unroll
        for (int b = 1; b <= 8; ++b) n[b] = nt[b];
        if (ok) blist[c][rank] = (int16_t)tid;
        __syncthreads();
        const int p17 = min(n[1], n[7]), p26 = min(n[2], n[6]), p35 = min(n[3], n[5]), p44 = n[4] / 2;
        const int L1 = n[1] - p17, L2 = n[2] - p26, L3 = n[3] - p35, L4 = n[4] - 2 * p44;
        const int Lt = L1 + L2 + L3 + L4;
        auto left = [&](int j) -> int {  // leftover j (counts 1..4 in count, rank order) -> thread
            if (j < L1) return blist[1][p17 + j];
            j -= L1;
            if (j < L2) return blist[2][p26 + j];
            j -= L2;
            if (j < L3) return blist[3][p35 + j];
            return blist[4][2 * p44 + j - L3];
        };
        bool lead = ok;
        int partner = -1;
        if (ok && c >= 5 && c <= 7) {
            const int pc = c == 7 ? p17 : c == 6 ? p26 : p35;
            if (rank < pc) partner = blist[8 - c][rank];
        } else if (ok && c <= 4) {
            const int pc = c == 1 ? p17 : c == 2 ? p26 : c == 3 ? p35 : 2 * p44;
            if (rank < pc) {
                if (c < 4 || (rank & 1)) lead = false;  // the 7, 6, 5 (or the even-ranked 4) leads
                else partner = blist[4][rank + 1];
            } else {
                const int j = (c == 1 ? 0 : c == 2 ? L1 : c == 3 ? L1 + L2 : L1 + L2 + L3) + rank - pc;
                if (j & 1) lead = false;
                else if (j + 1 < Lt) partner = left(j + 1);
            }
        }
        if (!pair) {  // pairing off (SGN_PAIR=0): every sample alone in its half
            lead = ok;
            partner = -1;
        }
        const uint64_t lm = __ballot(lead);
        int idx = __popcll(lm & below);
        if (lane == 0) wl[wv] = __popcll(lm);
        __syncthreads();
        if (tid == 0) {
            int tot = 0;
            for (int q = 0; q < PAIR_NW; ++q) tot += wl[q];
            sbase = tot ? atomicAdd(slot_n, tot) : 0;
        }
        for (int q = 0; q < wv; ++q) idx += wl[q];
        __syncthreads();
        if (lead) {
            const int slot = sbase + idx;
            const int nb = partner >= 0 ? sc[partner] : 0, sb = partner >= 0 ? ss[partner] : 0;
            int r8[8];
            const int ob = c > 4 ? c : 4;  // B's first row: never across the 4-row lane-group boundary
#pragma unroll
            for (int k = 0; k < 8; ++k) r8[k] = k < c ? s * 8 + k : (k >= ob && k < ob + nb ? sb * 8 + (k - ob) : -1);
            int4 *rp = (int4 *)(rows + (int64_t)slot * 8);
            rp[0] = make_int4(r8[0], r8[1], r8[2], r8[3]);
            rp[1] = make_int4(r8[4], r8[5], r8[6], r8[7]);
            slots[slot] = make_int4((int)((uint32_t)(rel0 + tid) | ((uint32_t)c << 28)),
                                    partner >= 0 ? (int)((uint32_t)(rel0 + partner) | ((uint32_t)nb << 28)) : 0, s, sb);
        }
    }
}

// a row-table entry s * 8 + k -> the pidx index s * K + k of that neighbour
__device__ __forceinline__ int64_t pidx_of(const AggArgs &a, int v) { return (int64_t)(v >> 3) * a.K + (v & 7); }

// the lane's row of slot `slot` (half of the wave), row kk of the half: rows table -> pidx index
__device__ __forceinline__ RowIdx row_index16(const AggArgs &a, int slot, int nslots, int kk) {
    RowIdx x;
    const int v = slot < nslots ? a.rows[(int64_t)slot * 8 + kk] : -1;
    x.sval = v >= 0;
    x.s = x.sval ? v >> 3 : 0;
    x.a = (v & 7) == kk;  // B rows sit nA rows after their k
    x.pid = x.sval ? a.pidx[pidx_of(a, v)] : -1;
    x.ray = x.sval ? a.samp_ray[x.s] : 0;
    return x;
}

// dists (point_aggregators.py:917-925): d[0..2] world offsets, d[3..5] pers-space terms; the
// linear-kernel weight normalised over the sample's 8 rows times the clamped conf (:946-953)
struct Row16 {
    float d[6];
    float wgt, wn;
};
template <bool PERS>
__device__ __forceinline__ Row16 row_math16(const Cam &cam, const Rec16<PERS> &rc, bool m, bool isA,
                                            int nA, bool waveB) {
    Row16 o;
    const float dwx = __fsub_rn(rc.p[0], rc.l[0]), dwy = __fsub_rn(rc.p[1], rc.l[1]), dwz = __fsub_rn(rc.p[2], rc.l[2]);
    o.d[0] = m ? dwx : 0.f;
    o.d[1] = m ? dwy : 0.f;
    o.d[2] = m ? dwz : 0.f;
    float xp, yp, zp, xl, yl, zl;
    if constexpr (PERS) {
        xp = rc.pp[0]; yp = rc.pp[1]; zp = rc.pp[2];
        xl = rc.pl[0]; yl = rc.pl[1]; zl = rc.pl[2];
    } else {
        cam.pers(rc.p[0], rc.p[1], rc.p[2], xp, yp, zp);
        cam.pers(rc.l[0], rc.l[1], rc.l[2], xl, yl, zl);
    }
    o.d[3] = m ? __fsub_rn(__fmul_rn(xp, zp), __fmul_rn(xl, zl)) : 0.f;
    o.d[4] = m ? __fsub_rn(__fmul_rn(yp, zp), __fmul_rn(yl, zl)) : 0.f;
    o.d[5] = m ? __fsub_rn(zp, zl) : 0.f;
    float w = 0.f;
    if (m) {
        const float n2 = __fadd_rn(__fadd_rn(__fmul_rn(dwx, dwx), __fmul_rn(dwy, dwy)), __fmul_rn(dwz, dwz));
        w = 1.f / fmaxf(sqrtf(n2), 1e-6f);
    }
    // normalised over the rows of the row's own sample (A: rows 0..nA-1 of the half, B: rows
    // oB = max(nA, 4) .. 7, always in the upper quad; idle rows carry w = 0).  B's weights are first
    // rotated inside that quad so its rows start at row 4 (the rows rotated in are A's or idle: 0),
    // so both samples sum in the same tree as alone in a half: a sample's values do not depend on its
    // partner.
    // (waveB: the wave holds a B sample, else every row is A's or idle and one sum does)
    float wsum;
    if (waveB) {
        const float wb0 = isA ? 0.f : w;
        const int rb0 = __builtin_bit_cast(int, wb0);
        const int r1 = __builtin_amdgcn_mov_dpp(rb0, 0x39, 0xF, 0xF, true);  // quad_perm [1,2,3,0]
        const int r2 = __builtin_amdgcn_mov_dpp(rb0, 0x4E, 0xF, 0xF, true);  // [2,3,0,1]
        const int r3 = __builtin_amdgcn_mov_dpp(rb0, 0x93, 0xF, 0xF, true);  // [3,0,1,2]
        const int rot = nA > 4 ? nA - 4 : 0;
        const float wbs = __builtin_bit_cast(float, rot == 0 ? rb0 : rot == 1 ? r1 : rot == 2 ? r2 : r3);
        const float wsa = dpp_sum8(isA ? w : 0.f), wsb = dpp_sum8(wbs);
        wsum = isA ? wsa : wsb;
    } else {
        wsum = dpp_sum8(w);
    }
    w = w / fmaxf(wsum, 1e-8f);
    o.wn = w;
    o.wgt = w * fminf(fmaxf(rc.cf, 1e-4f), 1.f);
    return o;
}

// PE(dists) of the row (networks.py:175-192, 6 values x 5 frequencies, sin / cos interleaved): pair
// slot c = 0..7 of lane group g (k-step c / 4, B slots 2 (c % 4), 2 (c % 4) + 1 = sin, cos) holds
//   c < 5 : component g,           frequency c
//   c = 5 : component 4 + (g & 1), frequency (g >= 2)        c = 6 : the same, frequency 2 + (g >= 2)
//   c = 7 : component 4 + (g & 1), frequency 4 (g < 2; padding for g >= 2)
// so every frequency is a compile-time power of two and a lane selects only its two components once
// per tile (PeRow); col_l0b16 maps the slots to the reference columns.
struct PeRow {
    float lo, hi, shi;  // d[g], d[4 + (g & 1)], 2 if g >= 2 else 1
};
__device__ __forceinline__ PeRow pe_row16(const float (&d)[6], int g) {
    PeRow r;
    r.lo = g == 0 ? d[0] : g == 1 ? d[1] : g == 2 ? d[2] : d[3];
    r.hi = (g & 1) ? d[5] : d[4];
    r.shi = g >= 2 ? 2.f : 1.f;
    return r;
}
// slot c's argument: the component times its frequency 2^f (exact scaling, as positions * freq_bands)
template <int C>
__device__ __forceinline__ float pe_arg16(const PeRow &r) {
    if constexpr (C < 5) return r.lo * (float)(1 << C);
    else if constexpr (C == 7) return r.hi * 16.f;
    else return r.hi * (r.shi * (float)(1 << (2 * (C - 5))));
}
// k-step S's fragment: slots c = 4 S .. 4 S + 3 (block1.0 computes it inside its k-loop, so the
// second k-step's sin / cos overlap the first one's MFMAs).  Arguments of 2^20 and above (never met
// by the aggregator's distances) take the library sincosf, behind one wave-uniform branch.
template <int S>
__device__ __forceinline__ X3B pe_dists16_k(const PeRow &r) {
    float x[4], u[8];
    static_for<4>([&](auto cc) { x[decltype(cc)::value] = pe_arg16<4 * S + decltype(cc)::value>(r); });
    const float m = fmaxf(fmaxf(__builtin_fabsf(x[0]), __builtin_fabsf(x[1])), fmaxf(__builtin_fabsf(x[2]), __builtin_fabsf(x[3])));
    if (__builtin_expect(__ballot(!(m < 1048576.f)) != 0, 0)) {
#pragma unroll
        for (int q = 0; q < 4; ++q) sincosf(x[q], &u[2 * q], &u[2 * q + 1]);
    } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) sincos_acc_fast(x[q], u[2 * q], u[2 * q + 1]);
    }
    return split8(u);
}

// block3.2 epilogue of a tile (K-blend -> f_s, alpha), per lane: rows 4 g + i of half g >> 1
struct Epi16 {
    float wsa[4], wsb[4];   // the rows' blend weights split by segment (A: positions < nA, B: the rest),
                            // times 2^-s3 (block3.2's accumulators hold 2^s3 (W x + b))
    float ap[4];            // alpha partials of the 4 rows over this lane's units
    float fsv[4];           // blended features of units 16 t + r, t = 4 (T / 4) .. + 3, stored per 4
    float *fs_dst;
    bool fs_have;
    float inv3;
};

// a workgroup's tiles: first, first + step, ... < end (grid-stride; an XCD-contiguous order measured
// within +-1 %)
struct Tiles {
    int first, end, step;
};
__device__ __forceinline__ Tiles grid_tiles(int ntiles) { return Tiles{(int)blockIdx.x, ntiles, (int)gridDim.x}; }

// KB: k-steps of block2_bpnet.0 in 16x16 steps (0: base viewmlp; 8: bpnet_dim 0; 11: dim 96)
// SAVE (training): the pre-activations of block1.0 / 1.2 / 3.0 go to a.z1 / z2 / z3 as the next
// layer converts them (chain_k); SG: block2_bpnet.0's to a.zb
// NS: row sets of 16 rows per wave.  NS = 2: 32 rows per wave, each LDS weight fragment pair feeds
// six MFMAs (half the LDS reads and weight DMA per MFMA of NS = 1), one workgroup per CU and one
// wave per SIMD (the accumulators of two layers, 256 registers, sit in AGPRs)
template <int KB, bool PERS, bool SAVE = false, int NS = 1, int SP = 16>
__global__ __launch_bounds__(TPBR, NS == 1 ? 8 / NWR : 1) void k_rows16(AggArgs a) {
    using Net = std::conditional_t<(KB > 0), NetR16SGT<KB, SP>, NetR16T<SP>>;
    constexpr int YR_OFF = yr_off(SP), YT16_OFF = yt16_off(SP), ROWS16_LDS = rows16_lds(SP);
    constexpr int LB = 2, L2 = KB ? 3 : 2, L3 = KB ? 4 : 3;
    constexpr int NBP = KB > 8 ? KB - 8 : 0;  // BPNet k-steps (32 channels each)
    constexpr int WGS = WG16_SAMPLES * NS;    // halves per workgroup tile
    __shared__ __attribute__((aligned(16))) char lds[ROWS16_LDS];
    const int lane = threadIdx.x & 63;
    const int g = lane >> 4, r = lane & 15, kk = lane & 7, sc = r >> 3;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nslots = a.slot_n[0];  // paired halves (k_pair_slots), 2 per row set and tile
    const Cam cam = load_cam(a.campos, a.rot);
    const WBlob wb = make_blob(a.blob, BLOB_BYTES_ALL);
    const float *proj = (const float *)a.proj;
    {
        const float *src = (const float *)((const char *)a.blob + OFF16_F32);
        float *dst = (float *)(lds + YR_OFF);
        for (int i = threadIdx.x; i < N_Y32; i += TPBR) dst[i] = src[i];
        {
            // row stride 20 floats: the 16 lanes' 16-B reads of one column quad hit disjoint banks
            float *yt = (float *)(lds + YT16_OFF);
            for (int i = threadIdx.x; i < 512; i += TPBR) {
                const int which = i >> 8, u = i & 255, t = u >> 4, rr = u & 15;
                yt[which * 320 + rr * 20 + t] = src[(which ? Y_WA : Y_B3) + 16 * t + rr];
            }
        }
    }
    __syncthreads();
    int slot = 0;
    dma_chunk<Net, 0, NWR>(wb, lds, w, lane, 0);
    // The next tile's chain, prefetched inside the current tile so each step lands under MFMAs:
    // row-table entry (block1.2), neighbour / ray index (block3.0), point record + sample position
    // and the P row (block3.2).  First tile: here.  Row set q of wave w: halves w 2 NS + 2 q (+ sc).
    const Tiles xt = grid_tiles((nslots + WGS - 1) / WGS);
    RowIdx nx[NS];
    Rec16<PERS> rnext[NS];
#pragma unroll
    for (int q = 0; q < NS; ++q) {
        nx[q] = row_index16(a, xt.first * WGS + w * 2 * NS + 2 * q + sc, nslots, kk);
        rnext[q] = load_rec16<PERS>(a, nx[q]);
    }
    // P row of point pid into `dst`: natural unit order, tile t of lane group g at 16 t + 4 g, so the
    // 4 lanes of a row read one contiguous 64 B per load instruction
    auto load_p = [&](int pid, f32x4 (&dst)[16]) {
        const float *src = proj + (int64_t)(pid < 0 ? 0 : pid) * HID + 4 * g;
#pragma unroll
        for (int t = 0; t < 16; ++t) dst[t] = *(const f32x4 *)(src + 16 * t);
    };
    // accA: block1.0's accumulators start at P[pid]; the next tile's P is loaded into the array
    // block3.0 accumulated in (dead once block3.2 has consumed it), so it lands during the
    // block3.2 epilogue and the tile transition without extra registers
    f32x4 accA[NS][16], accB[NS][16];
#pragma unroll
    for (int q = 0; q < NS; ++q) load_p(nx[q].pid, pick<(KB > 0)>(accB[q], accA[q]));  // SG: where the tile loop copies it from

    // epilogue pieces (LDS reads through the tile's opaque base)
    auto epi_begin = [&](Epi16 &e, const char *ldsi, float wgt, int nA, int nB, int2 ce, bool ok) {
        const float inv3 = ((const float *)(ldsi + YR_OFF))[Y_INV + 3];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float wi = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute((4 * g + i) * 4, __builtin_bit_cast(int, wgt)));
            const bool inA = 4 * (g & 1) + i < nA;
            const float ws = wi;
            e.wsa[i] = inA ? ws : 0.f;
            e.wsb[i] = inA ? 0.f : ws;
            e.ap[i] = 0.f;
        }
        e.fs_have = ((g & 1) ? nB > 0 : nA > 0) && ok;
        e.inv3 = inv3;
        e.fs_dst = (float *)a.fs + (int64_t)((uint32_t)((g & 1) ? ce.y : ce.x) & 0x0FFFFFFFu) * HID + r;
    };
    // block3.2 output tile T of accumulators `ac` (2^s3 (W x + b)): LeakyReLU, alpha partials, K-blend
    auto epi_step = [&](Epi16 &e, const char *ldsi, const f32x4 (&ac)[16], auto tc) {
        constexpr int T = decltype(tc)::value;
        const float wau = ((const float *)(ldsi + YT16_OFF))[320 + r * 20 + T];  // 2^-s3 alpha weight
        float fa = 0.f, fb = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float hv = lrelu_x3(__builtin_fmaf(ac[T][i], e.inv3, ((const float *)(ldsi + YT16_OFF))[r * 20 + T]));
            e.ap[i] = __builtin_fmaf(wau, hv, e.ap[i]);
            fa = __builtin_fmaf(e.wsa[i], hv, fa);
            fb = __builtin_fmaf(e.wsb[i], hv, fb);
        }
        // + the half's other 4 rows (lane group g ^ 1, 16 lanes away): the swap leaves A's pair of chains
        // in the even groups and B's in the odd ones.  Per sample this is (chain over its rows 0..3) +
        // (chain over rows 4..7) at any offset: B sits in one group (zero-weight rows leave a chain
        // unchanged, the other group's chain is 0)
        permlane16_swap(fa, fb);
        e.fsv[T & 3] = fa + fb;
        if constexpr ((T & 3) == 3) {  // 16 lanes write 64 contiguous bytes of the work item's row, per 4
            if (e.fs_have) {
#pragma unroll
                for (int u = 0; u < 4; ++u) e.fs_dst[16 * (T - 3 + u)] = e.fsv[u];
            }
        }
    };
    auto epi_end = [&](Epi16 &e, const char *ldsi, int nA, int nB, int s_ix) {
        // alpha: row logits summed over the 16 lanes (units) of the group, softplus(x + b - 1), blended
        // over the segment's rows like f_s
        const float ba = ((const float *)(ldsi + YR_OFF))[Y_BA];
        float xr[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float x = dpp_sum8(e.ap[i]);
            x += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0x128, 0xF, 0xF, true));
            xr[i] = x;
        }
        // one softplus per lane: lane r takes row 4 g + (r & 3), and each lane then reads the four rows'
        // values from its quad (quad_perm broadcasts) -- 16x fewer log1p / exp than every lane
        // evaluating its four rows
        const int q4 = r & 3;
        const float spm = softplus((q4 == 0 ? xr[0] : q4 == 1 ? xr[1] : q4 == 2 ? xr[2] : xr[3]) + ba - 1.f);
        const int spi = __builtin_bit_cast(int, spm);
        const float sp4[4] = {__builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(spi, 0x00, 0xF, 0xF, true)),
                              __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(spi, 0x55, 0xF, 0xF, true)),
                              __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(spi, 0xAA, 0xF, 0xF, true)),
                              __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(spi, 0xFF, 0xF, 0xF, true))};
        float asa = 0.f, asb = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {  // the rows' weights
            asa = __builtin_fmaf(e.wsa[i], sp4[i], asa);
            asb = __builtin_fmaf(e.wsb[i], sp4[i], asb);
        }
        permlane16_swap(asa, asb);
        const float as = asa + asb;  // even groups: A's alpha, odd groups: B's
        // the segment's sample: row 0 (A) or row max(nA, 4) (B) of the half (lanes 0..15 hold rows)
        const int s_of = __builtin_amdgcn_ds_bpermute((8 * (g >> 1) + ((g & 1) ? (nA > 4 ? nA : 4) : 0)) * 4, s_ix);
        if (r == 0 && ((g & 1) ? nB > 0 : nA > 0)) a.feat[(int64_t)s_of * 4 + 0] = as;
    };

    for (int tile = xt.first; tile < xt.end; tile += xt.step) {
        const int base = tile * WGS;
        int lz = 0;
        asm volatile("" : "+s"(lz));
        char *ldsi = lds + lz;
        const float *Yl = (const float *)(ldsi + YR_OFF);
        RowIdx ix[NS];
        Row16 rw[NS];
        int nslot[NS], nA[NS], nB[NS];
        uint64_t mrowA[NS], mrowB[NS];
        int64_t vrow[NS];
        X3B ext[NS];
        const int hsh = 8 * (g >> 1);  // half g >> 1's row bits
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            const int hslot = base + w * 2 * NS + 2 * q + sc;  // this lane's half (the LDS ring slot is `slot`)
            nslot[q] = tile + xt.step < xt.end ? hslot + xt.step * WGS : nslots;  // next tile's half
            ix[q] = nx[q];
            const bool m = ix[q].pid >= 0;
            const Rec16<PERS> rc = rnext[q];
            // rows of the two segments (lane group 0 = rows 0..15): bits 8 h .. 8 h + 7 are half h's
            mrowA[q] = __ballot(ix[q].sval && ix[q].a);
            mrowB[q] = __ballot(ix[q].sval && !ix[q].a);
            const int nA0 = __popc((uint32_t)mrowA[q] & 0xFFu), nA1 = __popc(((uint32_t)mrowA[q] >> 8) & 0xFFu);
            const bool waveB = (mrowB[q] & 0xFFFFull) != 0;  // wave-uniform: a B sample in either half
            rw[q] = row_math16<PERS>(cam, rc, m, ix[q].a, sc ? nA1 : nA0, waveB);
            nA[q] = __popcll((mrowA[q] >> hsh) & 0xFFull);
            nB[q] = __popcll((mrowB[q] >> hsh) & 0xFFull);
            // SAVE: the row's pidx index s * K + k (from the slot's row table entry s * 8 + k), or its
            // compact row row_off[s] + k; -1 for rows without a neighbour
            vrow[q] = -1;
            if (SAVE && ix[q].sval && m) {
                const int e = a.rows[(int64_t)hslot * 8 + kk];
                vrow[q] = a.row_off ? (int64_t)a.row_off[e >> 3] + (e & 7) : pidx_of(a, e);
            }
            if ((a.blend || a.wnorm) && ix[q].sval) {  // optional outputs: the row's pidx index from the table
                const int64_t v = pidx_of(a, a.rows[(int64_t)hslot * 8 + kk]);
                if (a.blend && g == 0) a.blend[v] = rw[q].wgt;
                if (a.wnorm && g == 1) a.wnorm[v] = rw[q].wn;
            }
            {   // block3 extra channels: colour, dir - v, <dir, v> (:639-652), lane group 0
                const bool e = g == 0 && m;
                float u[8];
                u[0] = e ? rc.col[0] : 0.f; u[1] = e ? rc.col[1] : 0.f; u[2] = e ? rc.col[2] : 0.f;
                u[3] = e ? __fsub_rn(rc.dir[0], rc.v[0]) : 0.f;
                u[4] = e ? __fsub_rn(rc.dir[1], rc.v[1]) : 0.f;
                u[5] = e ? __fsub_rn(rc.dir[2], rc.v[2]) : 0.f;
                u[6] = e ? __fadd_rn(__fadd_rn(__fmul_rn(rc.dir[0], rc.v[0]), __fmul_rn(rc.dir[1], rc.v[1])),
                                     __fmul_rn(rc.dir[2], rc.v[2])) : 0.f;
                u[7] = 0.f;
                ext[q] = split8(u);
            }
        }
        // Each layer's epilogue (LeakyReLU + hi/lo split of its accumulators) runs lazily inside the
        // next layer's k-loop: k-step k converts tiles 2k, 2k+1 only, so the VALU work overlaps the
        // MFMAs in flight instead of idling the matrix pipe between layers.
        auto chain_k = [&](int q, const f32x4 (&ac)[16], float inv, auto kc, float *zsave = nullptr) {
            constexpr int S = decltype(kc)::value;
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = ac[2 * S + (j >> 2)][j & 3];
            if constexpr (SAVE) {  // units 16 t + 4 g .. + 3 of tiles t = 2 S, 2 S + 1
                if (zsave && vrow[q] >= 0) {
                    float *zr = zsave + vrow[q] * HID + 4 * g;
                    *(f32x4 *)(zr + 32 * S) = f32x4{v[0] * inv, v[1] * inv, v[2] * inv, v[3] * inv};
                    *(f32x4 *)(zr + 32 * S + 16) = f32x4{v[4] * inv, v[5] * inv, v[6] * inv, v[7] * inv};
                }
            }
            return lrelu_split8(v, inv);
        };
        auto bias_init = [&](f32x4 (&ac)[16], int yb) {
#pragma unroll
            for (int t = 0; t < 16; ++t) ac[t] = *(const f32x4 *)(Yl + yb + 16 * t + 4 * g);
        };
        {   // block1.0: W0b PE(dists) on MFMA, + P[pid] (W0a [feat | PE(feat)] + b0, k_point_proj16)
            PeRow pr[NS];
#pragma unroll
            for (int q = 0; q < NS; ++q) {
                pr[q] = pe_row16(rw[q].d, g);
                if constexpr (KB > 0) {  // SG: five layers, the P array alternates -- copy it back
#pragma unroll
                    for (int t = 0; t < 16; ++t) accA[q][t] = accB[q][t];
                }
            }
            run_layer_ns<Net, 0, false, std::conditional_t<SAVE, VmZero, VmL0<NS>>, 0, 0, !SAVE>(
                wb, ldsi, slot, w, lane, lz, accA, [&](auto k) {
                    X3S<NS> o;
#pragma unroll
                    for (int q = 0; q < NS; ++q) o.b[q] = pe_dists16_k<decltype(k)::value>(pr[q]);
                    return o;
                }, NoHook{});
        }
        // block1.2: 256 -> 256 (input: block1.0 accumulators)
        const float inv0 = Yl[Y_INV + 0], inv1 = Yl[Y_INV + 1], inv2 = Yl[Y_INV + 2], inv7 = Yl[Y_INV + 7];
#pragma unroll
        for (int q = 0; q < NS; ++q) bias_init(accB[q], Y_B1);
        int v_next[NS];
        run_layer_ns<Net, 1, false, VmZero, 0, 0, !SAVE>(wb, ldsi, slot, w, lane, lz, accB, [&](auto k) {
            X3S<NS> o;
#pragma unroll
            for (int q = 0; q < NS; ++q) o.b[q] = chain_k(q, accA[q], inv0, k, a.z1);
            return o;
        }, [&](auto c) {
            if constexpr (decltype(c)::value == 0) {
#pragma unroll
                for (int q = 0; q < NS; ++q) v_next[q] = nslot[q] < nslots ? a.rows[(int64_t)nslot[q] * 8 + kk] : -1;
            }
        });
        if constexpr (KB > 0) {
            // block2_bpnet.0 (SG): [h 256 | BPNet embedding] -> 256; the row's fp32 embedding
            // (channels 32 m + 8 g .. +7 for k-step 8 + m) gathered and split here
            X3B bpv[NS][NBP > 0 ? NBP : 1];
            if constexpr (NBP > 0) {
#pragma unroll
                for (int q = 0; q < NS; ++q) {
                    const float *src = a.bpnet32 + (int64_t)(ix[q].pid >= 0 ? ix[q].pid : 0) * (NBP * 32) + 8 * g;
#pragma unroll
                    for (int j = 0; j < NBP; ++j) {
                        const f32x4 u0 = *(const f32x4 *)(src + 32 * j), u1 = *(const f32x4 *)(src + 32 * j + 4);
                        const float v[8] = {u0[0], u0[1], u0[2], u0[3], u1[0], u1[1], u1[2], u1[3]};
                        bpv[q][j] = split8(v);
                    }
                }
            }
#pragma unroll
            for (int q = 0; q < NS; ++q) bias_init(accA[q], Y_BB);
            run_layer_ns<Net, LB>(wb, ldsi, slot, w, lane, lz, accA, [&](auto k) {
                constexpr int K = decltype(k)::value;
                X3S<NS> o;
#pragma unroll
                for (int q = 0; q < NS; ++q) {
                    if constexpr (K < 8) o.b[q] = chain_k(q, accB[q], inv1, k, a.z2);
                    else o.b[q] = bpv[q][K - 8];
                }
                return o;
            }, NoHook{});
        }
        // block3.0: [h 256 | colour, dir - v, <dir, v>] -> 256 (input: block1.2 or block2_bpnet)
        auto &in2 = pick<(KB > 0)>(accA, accB);
        auto &acc2 = pick<(KB > 0)>(accB, accA);
        const float inv_in2 = KB > 0 ? inv7 : inv1;
#pragma unroll
        for (int q = 0; q < NS; ++q) bias_init(acc2[q], Y_B2);
        run_layer_ns<Net, L2, false, VmZero, 0, 0, !SAVE>(wb, ldsi, slot, w, lane, lz, acc2, [&](auto k) {
            constexpr int K = decltype(k)::value;
            X3S<NS> o;
#pragma unroll
            for (int q = 0; q < NS; ++q) {
                if constexpr (K < 8) o.b[q] = chain_k(q, in2[q], inv_in2, k, KB > 0 ? a.zb : a.z2);
                else o.b[q] = ext[q];
            }
            return o;
        }, [&](auto c) {
            constexpr int C = decltype(c)::value;
            if constexpr (C == 0) {  // v_next landed at the previous boundaries
#pragma unroll
                for (int q = 0; q < NS; ++q) {
                    nx[q].sval = v_next[q] >= 0;
                    nx[q].s = nx[q].sval ? v_next[q] >> 3 : 0;
                    nx[q].a = (v_next[q] & 7) == kk;
                    nx[q].pid = nx[q].sval ? a.pidx[pidx_of(a, v_next[q])] : -1;
                    nx[q].ray = nx[q].sval ? a.samp_ray[nx[q].s] : 0;
                }
            }
        });
        // block3.2: 256 -> 256 transposed: acc[t][i] = h[row 4 g + i][unit 16 t + (l & 15)]
        auto &acc = in2;  // block3.0's input is dead: its registers take block3.2's accumulators
#pragma unroll
        for (int q = 0; q < NS; ++q)
#pragma unroll
            for (int t = 0; t < 16; ++t) acc[q][t] = f32x4{};  // the bias joins in the epilogue (epi_step)
        // the next tile's record (and this tile's slot entry for the epilogue: half g >> 1's
        // {A item | nA << 28, B item | nB << 28, ..}) go out at the end of block3.2's first chunk, after
        // the chunk's DMA pieces, so they stay in flight across one boundary (VmL3P0)
        int2 ce[NS];
        int eslot[NS];
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            ce[q] = make_int2(0, 0);
            eslot[q] = base + w * 2 * NS + 2 * q + (g >> 1);
        }
        auto first_chunk_loads = [&](auto c) {
            if constexpr (decltype(c)::value == 0) {
#pragma unroll
                for (int q = 0; q < NS; ++q) {
                    rnext[q] = load_rec16<PERS>(a, nx[q]);
                    ce[q] = *(const int2 *)(a.slots + (eslot[q] < nslots ? eslot[q] : 0));
                }
            }
        };
        Epi16 e[NS];
        {
            // pass 0 (output tiles 0..7) converts block3.0's output once into (hi, lo) fragments (in the
            // registers it frees) and pass 1 (tiles 8..15) reuses them; pass 1 carries the epilogue of
            // pass 0's tiles, output tile T after k-step T (one per 8 MFMA pairs)
            X3B in3[NS][8];
            run_layer_ns<Net, L3, true, std::conditional_t<SAVE, VmZero, VmL3P0<NS>>, 0, 0, !SAVE>(
                wb, ldsi, slot, w, lane, lz, acc, [&](auto k) {
                    constexpr int K = decltype(k)::value;
                    X3S<NS> o;
#pragma unroll
                    for (int q = 0; q < NS; ++q) {
                        in3[q][K] = chain_k(q, acc2[q], inv2, k, a.z3);
                        o.b[q] = in3[q][K];
                    }
                    return o;
                }, NoHook{}, first_chunk_loads);
#pragma unroll
            for (int q = 0; q < NS; ++q) epi_begin(e[q], ldsi, rw[q].wgt, nA[q], nB[q], ce[q], eslot[q] < nslots);
            run_layer_ns<Net, L3, true, VmZero, 1, 8>(wb, ldsi, slot, w, lane, lz, acc, [&](auto k) {
                X3S<NS> o;
#pragma unroll
                for (int q = 0; q < NS; ++q) o.b[q] = in3[q][decltype(k)::value];
                return o;
            }, NoHook{}, NoHook{}, [&](auto f) {
                constexpr int F = decltype(f)::value;
                if constexpr ((F & 7) == 7) {
#pragma unroll
                    for (int q = 0; q < NS; ++q) epi_step(e[q], ldsi, acc[q], std::integral_constant<int, F / 8>{});
                }
            });
        }
        // everything prefetched has landed (the chunk boundaries waited vmcnt(0)): hide the loads
        // from the compiler's wait tracking, which would otherwise wait for the epilogue's stores
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            asm volatile("" : "+v"(nx[q].s), "+v"(nx[q].pid), "+v"(nx[q].ray));
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                asm volatile("" : "+v"(rnext[q].p[c]), "+v"(rnext[q].col[c]), "+v"(rnext[q].dir[c]), "+v"(rnext[q].l[c]),
                             "+v"(rnext[q].v[c]));
                if constexpr (PERS) asm volatile("" : "+v"(rnext[q].pp[c]), "+v"(rnext[q].pl[c]));
            }
            asm volatile("" : "+v"(rnext[q].cf));
        }
        {   // the rest of the epilogue; the next tile's P rows (see accA) go out first, into block3.2's
            // consumed input registers, and land under it
            constexpr int NE = 8, PPE = 16 / NE;  // epilogue steps left, P loads per step and row set
            static_for<NE>([&](auto tc) {  // the loads spread between the steps (a burst stalls the issue)
                constexpr int J = decltype(tc)::value;
#pragma unroll
                for (int q = 0; q < NS; ++q) {
                    const float *psrc = proj + (int64_t)(nx[q].pid < 0 ? 0 : nx[q].pid) * HID + 4 * g;
#pragma unroll
                    for (int u = 0; u < PPE; ++u) acc2[q][PPE * J + u] = *(const f32x4 *)(psrc + 16 * (PPE * J + u));
                    epi_step(e[q], ldsi, acc[q], std::integral_constant<int, (16 - NE) + J>{});
                }
            });
#pragma unroll
            for (int q = 0; q < NS; ++q) epi_end(e[q], ldsi, nA[q], nB[q], ix[q].s);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---- host packing of the 16x16 sections -------------------------------------------------
// B position p = 8 g + j of a chained k-step -> unit offset inside the 32-wide step
int perm16(int p) { return 16 * ((p & 7) >> 2) + 4 * (p >> 3) + (p & 3); }
int col_chain16(int ks, int p) { return 32 * ks + perm16(p); }
int col_l2_16(int ks, int p) { return ks < 8 ? col_chain16(ks, p) : (p < 7 ? 256 + p : -1); }
int col_l0b16(int s, int p) {  // pe_dists16_k: slot c = 4 s + e / 2 of lane group g, sin / cos by e parity
    const int g = p >> 3, c = 4 * s + ((p & 7) >> 1);
    int comp, f;
    if (c < 5) {
        comp = g;
        f = c;
    } else {
        comp = 4 + (g & 1);
        f = c == 5 ? (g >= 2) : c == 6 ? 2 + (g >= 2) : 4;
        if (c == 7 && g >= 2) return -1;  // padding
    }
    return 224 + 2 * (5 * comp + f) + (p & 1);
}
int col_proj16(int s, int p) { return s == 0 ? p : 32 + 48 * (p >> 3) + 8 * (s - 1) + (p & 7); }
int col_bp16(int ks, int p) { return ks < 8 ? col_chain16(ks, p) : 256 + 32 * (ks - 8) + p; }
int col_c016(int ks, int p) {  // k-step 8: lane group g = p / 8 < 3 holds sin, cos of v_g 2^f at slots 2 f, 2 f + 1
    if (ks < 8) return 32 * ks + p;
    const int g = p >> 3, f = (p & 7) >> 1;
    return g < 3 ? 256 + ((p & 1) ? 12 : 0) + 4 * g + f : -1;
}

// 16 output tiles of 16 units, one pass, k-outer: pair f = ks * 16 + t; A[unit][k] fragment
// lane l: unit 16 t + (l & 15), input col(ks, 8 (l >> 4) + e)
template <typename ColFn>
void pack_pairs16(_Float16 *dst, const float *W, int n_out, int n_in, int KS, int shift, ColFn col, int NT = 16,
                  int NP = 1) {
    const float sc = ldexpf(1.f, shift);
    const int TPP = NT / NP;  // output tiles per pass: pair f = (pass KS + ks) TPP + t % TPP
    for (int t = 0; t < NT; ++t)
        for (int ks = 0; ks < KS; ++ks) {
            const size_t f = ((size_t)(t / TPP) * KS + ks) * TPP + t % TPP;
            for (int lane = 0; lane < 64; ++lane)
                for (int e = 0; e < 8; ++e) {
                    const int row = 16 * t + (lane & 15);
                    const int c = col(ks, 8 * (lane >> 4) + e);
                    const float v = (row < n_out && c >= 0 && c < n_in) ? W[(size_t)row * n_in + c] * sc : 0.f;
                    const _Float16 hi = (_Float16)v;
                    const _Float16 lo = (_Float16)(v - (float)hi);
                    dst[((2 * f) * 64 + lane) * 8 + e] = hi;
                    dst[((2 * f + 1) * 64 + lane) * 8 + e] = lo;
                }
        }
}

// The blob's layout, once: pairs(off, layer, n_out, n_in, KS, col, NT, NP) places layer's weights as
// (hi, lo) fragment pairs of 2^s w, f32(Y index, kind, layer, element) an fp32-section entry.  Layers are
// the w[] / b[] order of sgn_mlp_pack_f32 (weights.LAYERS, then block2_bpnet.0 as 9).
enum Y32Kind { YK_ZERO = 0, YK_W = 1, YK_B = 2, YK_BS = 3, YK_INV = 4, YK_ONE = 5, YK_WINV = 6, YK_BS_OR_B = 7 };
template <class Pairs, class F32>
void layout_blob16(int ksb, int bpnet_dim, Pairs &&pairs, F32 &&f32) {
    pairs(OFF16_W0B, 0, 256, 284, 2, col_l0b16, 16, 1);
    pairs(OFF16_W1, 1, 256, 256, 8, col_chain16, 16, 1);
    pairs(OFF16_W2, 2, 256, 263, 9, col_l2_16, 16, 1);
    pairs(OFF16_W3, 3, 256, 256, 8, col_chain16, 16, 2);  // block3.2 in two passes of 8 tiles
    pairs(OFF16_W0A, 0, 256, 284, 7, col_proj16, 16, 1);
    for (int u = 0; u < HID; ++u) {
        f32(Y_B0 + u, YK_BS, 0, u);
        f32(Y_B1 + u, YK_BS, 1, u);
        f32(Y_B2 + u, YK_BS, 2, u);
        f32(Y_B3 + u, YK_B, 3, u);  // block3.2's bias, added in the row kernel's epilogue
        f32(Y_WA + u, YK_W, 4, u);
    }
    f32(Y_BA, YK_B, 4, 0);
    const int li[7] = {0, 1, 2, 3, 5, 6, 7};
    for (int i = 0; i < 7; ++i) f32(Y_INV + i, YK_INV, li[i], 0);
    f32(Y_INV + 7, ksb > 0 ? YK_INV : YK_ONE, 9, 0);
    if (ksb > 0) {
        pairs(OFF16_WB, 9, 256, 256 + bpnet_dim, 8 + bpnet_dim / 32, col_bp16, 16, 1);
        for (int u = 0; u < HID; ++u) f32(Y_BB + u, YK_BS, 9, u);
    }
    // colour MLP (k_color16): 8 output tiles per layer; k-step 8 of colour 0 holds PE(v)
    pairs(OFF16_C0, 5, 128, 280, 9, col_c016, 8, 1);
    pairs(OFF16_C1, 6, 128, 128, 4, col_chain16, 8, 1);
    pairs(OFF16_C2, 7, 128, 128, 4, col_chain16, 8, 1);
    for (int u = 0; u < 128; ++u) {
        f32(Y_CB0 + u, YK_BS, 5, u);
        f32(Y_CB1 + u, YK_BS, 6, u);
        f32(Y_CB2 + u, YK_BS, 7, u);
        for (int c = 0; c < 3; ++c) f32(Y_CW3 + 128 * c + u, YK_W, 8, c * 128 + u);
    }
    for (int c = 0; c < 3; ++c) f32(Y_CB3 + c, YK_B, 8, c);
}

void pack_blob16(int ksb, int bpnet_dim, const float *const *w, const float *const *b, const int *s, int sb,
                 uint8_t *blob) {
    auto shift = [&](int L) { return L == 9 ? sb : s[L]; };
    float *Y = (float *)(blob + OFF16_F32);
    layout_blob16(ksb, bpnet_dim,
                  [&](uint32_t off, int L, int n_out, int n_in, int KS, auto col, int NT, int NP) {
                      pack_pairs16((_Float16 *)(blob + off), w[L], n_out, n_in, KS, shift(L), col, NT, NP);
                  },
                  [&](int yi, int kind, int L, int e) {
                      float v = 0.f;
                      switch (kind) {
                          case YK_W: v = w[L][e]; break;
                          case YK_B: v = b[L][e]; break;
                          case YK_BS: v = b[L][e] * ldexpf(1.f, shift(L)); break;
                          case YK_INV: v = ldexpf(1.f, -shift(L)); break;
                          case YK_ONE: v = 1.f; break;
                          case YK_WINV: v = w[L][e] * ldexpf(1.f, -shift(3)); break;
                          default: break;
                      }
                      Y[yi] = v;
                  });
}

// Index maps of the same layout, for packing on the device from a flat parameter (train_hip):
// fp16 element i of the fragment section -> (layer << 20 | element) | (1 << 30 for the lo part),
// -1 for padding; fp32 entry j -> kind << 26 | layer << 20 | element (kind 0: zero)
void index_blob16(int ksb, int bpnet_dim, int32_t *i16, size_t n16, int32_t *i32, size_t n32) {
    for (size_t i = 0; i < n16; ++i) i16[i] = -1;
    for (size_t i = 0; i < n32; ++i) i32[i] = 0;
    layout_blob16(ksb, bpnet_dim,
                  [&](uint32_t off, int L, int n_out, int n_in, int KS, auto col, int NT, int NP) {
                      const int TPP = NT / NP;
                      int32_t *dst = i16 + off / 2;
                      for (int t = 0; t < NT; ++t)
                          for (int ks = 0; ks < KS; ++ks) {
                              const size_t f = ((size_t)(t / TPP) * KS + ks) * TPP + t % TPP;
                              for (int lane = 0; lane < 64; ++lane)
                                  for (int e = 0; e < 8; ++e) {
                                      const int row = 16 * t + (lane & 15);
                                      const int c = col(ks, 8 * (lane >> 4) + e);
                                      const bool ok = row < n_out && c >= 0 && c < n_in;
                                      const int32_t code = ok ? (L << 20) | (row * n_in + c) : -1;
                                      dst[((2 * f) * 64 + lane) * 8 + e] = code;
                                      dst[((2 * f + 1) * 64 + lane) * 8 + e] = ok ? code | (1 << 30) : -1;
                                  }
                          }
                  },
                  [&](int yi, int kind, int L, int e) { i32[yi] = (kind << 26) | (L << 20) | e; });
}
// ---- colour MLP ------------------------------------------------------------------------
struct ColorArgs {
    const int32_t *counters, *work, *samp_ray;
    const float *raydir;
    const void *blob;
    const float *fs;
    float *feat;
    int32_t *range_flag;  // set to 1 when a sample's decoded features are not finite (fp16 range exceeded)
    int32_t item0, n_items;
};
// ---- colour MLP, 16x16 (2 waves per SIMD): 8 waves x 16 samples per 128-sample tile --------
// Lane (sample r = l & 15, group g = l >> 4).  Colour 0's k-step s < 8 takes f_s units 32 s + 8 g + j
// (natural order, two 16-B loads per lane), k-step 8 the PE(viewdir) channels 8 g + j < 24; colour
// 1 and 2 chain lazily as in k_rows16 (k-step s converts tiles 2 s, 2 s + 1 of the previous layer).
// The output layer (128 -> 3) and the sigmoid are per-lane FMAs over the 32 units a lane holds
// plus two cross-group shuffles.
constexpr int YC_OFF = NSLOT * SPC * PAIR, TPBC = NWC * 64;
constexpr int COL16_LDS = YC_OFF + N_Y32 * 4;
static_assert(COL16_LDS * (8 / NWC) <= 163840, "LDS budget (colour, 8 / NWC workgroups per CU)");

__global__ __launch_bounds__(TPBC, 8 / NWC) void k_color16(ColorArgs a) {
    __shared__ __attribute__((aligned(16))) char lds[COL16_LDS];
    const int lane = threadIdx.x & 63;
    const int g = lane >> 4, r = lane & 15;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nwork = a.counters[1];
    const int end = min(nwork, a.item0 + a.n_items);
    const WBlob wb = make_blob(a.blob, BLOB_BYTES_ALL);
    {
        const float *src = (const float *)((const char *)a.blob + OFF16_F32);
        float *dst = (float *)(lds + YC_OFF);
        for (int i = threadIdx.x; i < N_Y32; i += TPBC) dst[i] = src[i];
    }
    __syncthreads();
    int slot = 0;
    dma_chunk<NetColor16, 0, NWC>(wb, lds, w, lane, 0);
    // The tile's f_s rows go out in four quarters (k-steps 2 q, 2 q + 1 of colour 0), each at a chunk
    // boundary after its registers were consumed and a chunk before they are needed: the next tile's
    // quarter 0 in colour 0's second chunk, quarter 1 (and the sample ids) in colour 1, quarter 2 (and
    // the ray ids) in colour 2, quarter 3 in the tile's own first chunk with its ray directions.  The
    // rows as one 16 KiB-per-wave burst had to land within one chunk (vmcnt retires in order: the next
    // boundary's wait for its weight pieces waits for them too), and did not (colour stage -23 % without
    // them, tools/x3_variant.py cabl_fs).
    f32x4 fr[16];
    float vd[3];
    int sn = 0, rn = 0;
    // The quarters are asm loads, outside the compiler's wait tracking: with an LDS-DMA outstanding it
    // waits vmcnt(0) at the first use of any load result, which would drain a quarter right after it
    // was issued.  A quarter issued in a chunk's hook is older than the next chunk's weight pieces, so
    // that chunk's boundary wait has retired it; its first use re-reads the registers through an empty
    // asm after that boundary (in order with the boundary's asm), so no read moves above it.
    auto load_q = [&](auto qc, int item) {
        constexpr int Q = decltype(qc)::value;
        const bool ok = item < end;
        const f32x4 *row = (const f32x4 *)(a.fs + (int64_t)(ok ? item - a.item0 : 0) * HID + 8 * g) + 16 * Q;
        f32x4 t0, t1, t2, t3;
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(t0) : "v"(row));
        asm volatile("global_load_dwordx4 %0, %1, off offset:16" : "=v"(t1) : "v"(row));
        asm volatile("global_load_dwordx4 %0, %1, off offset:128" : "=v"(t2) : "v"(row));
        asm volatile("global_load_dwordx4 %0, %1, off offset:144" : "=v"(t3) : "v"(row));
        fr[4 * Q] = t0;
        fr[4 * Q + 1] = t1;
        fr[4 * Q + 2] = t2;
        fr[4 * Q + 3] = t3;
    };
    auto load_sid = [&](int item) { sn = item < end ? a.work[item] : 0; };
    auto load_ray = [&]() { rn = a.samp_ray[sn]; };
    auto load_dir = [&]() {
#pragma unroll
        for (int c = 0; c < 3; ++c) vd[c] = a.raydir[(int64_t)rn * 3 + c];
    };
    {
        const int item = a.item0 + blockIdx.x * (16 * NWC) + w * 16 + r;
        load_sid(item);
        load_q(std::integral_constant<int, 0>{}, item);
        load_q(std::integral_constant<int, 1>{}, item);
        load_q(std::integral_constant<int, 2>{}, item);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the first tile's quarters (no boundary between)
    }
    load_ray();
    for (int base = a.item0 + blockIdx.x * (16 * NWC); base < end; base += gridDim.x * (16 * NWC)) {
        int lz = 0;
        asm volatile("" : "+s"(lz));
        char *ldsi = lds + lz;
        const float *Yl = (const float *)(ldsi + YC_OFF);
        const int item = base + w * 16 + r;
        const bool sval = item < end;
        const int s = sn;
        auto bias = [&](f32x4 (&ac)[8], int yb) {
#pragma unroll
            for (int t = 0; t < 8; ++t) ac[t] = *(const f32x4 *)(Yl + yb + 16 * t + 4 * g);
        };
        auto chain = [&](const f32x4 (&ac)[8], float inv, auto kc) {
            constexpr int S = decltype(kc)::value;
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = ac[2 * S + (j >> 2)][j & 3];
            return lrelu_split8(v, inv);
        };
        f32x4 c0[8], c1[8];
        bias(c0, Y_CB0);
        run_layer16<NetColor16, 0>(wb, ldsi, slot, w, lane, lz, c0, [&](auto k) {
            constexpr int K = decltype(k)::value;
            float v[8];
            if constexpr (K < 8) {
                f32x4 u0 = fr[2 * K], u1 = fr[2 * K + 1];
                asm volatile("" : "+v"(u0), "+v"(u1));   // after the boundary that retired them
                v[0] = u0[0]; v[1] = u0[1]; v[2] = u0[2]; v[3] = u0[3];
                v[4] = u1[0]; v[5] = u1[1]; v[6] = u1[2]; v[7] = u1[3];
            } else {
                // PE(viewdir) ori=True (point_aggregators.py:579-585, networks.py:175-192): lane group g < 3
                // holds sin, cos of v_g 2^f, f = 0..3 (slots 2 f, 2 f + 1; col_c016 maps them to the
                // reference's sin block [0, 12) and cos block [12, 24)), group 3 is padding: 4 sincos per
                // lane with compile-time frequencies and both results used
                const float x = g == 0 ? vd[0] : g == 1 ? vd[1] : vd[2];
                float y[4];
#pragma unroll
                for (int f = 0; f < 4; ++f) y[f] = x * (float)(1 << f);
                const float m = fmaxf(fmaxf(__builtin_fabsf(y[0]), __builtin_fabsf(y[1])),
                                      fmaxf(__builtin_fabsf(y[2]), __builtin_fabsf(y[3])));
                if (__builtin_expect(__ballot(!(m < 1048576.f)) != 0, 0)) {
#pragma unroll
                    for (int f = 0; f < 4; ++f) sincosf(y[f], &v[2 * f], &v[2 * f + 1]);
                } else {
#pragma unroll
                    for (int f = 0; f < 4; ++f) sincos_acc_fast(y[f], v[2 * f], v[2 * f + 1]);
                }
            }
            return split8(v);
        }, [&](auto c) {
            constexpr int C = decltype(c)::value;
            if constexpr (C == 0) {
                load_q(std::integral_constant<int, 3>{}, item);   // this tile's k-steps 6, 7 (next chunk)
                load_dir();                                        // this tile's directions (k-step 8)
            }
            if constexpr (C == 1) load_q(std::integral_constant<int, 0>{}, item + gridDim.x * (16 * NWC));
        });
        bias(c1, Y_CB1);
        const float inv4 = Yl[Y_INV + 4], inv5 = Yl[Y_INV + 5], inv6 = Yl[Y_INV + 6];
        // colour 0 consumed fr: the next tile's quarters 1, 2 go out at colour 1's and colour 2's boundaries
        run_layer16<NetColor16, 1>(wb, ldsi, slot, w, lane, lz, c1, [&](auto k) { return chain(c0, inv4, k); },
                                   [&](auto c) {
                                       if constexpr (decltype(c)::value == 0) {
                                           load_q(std::integral_constant<int, 1>{}, item + gridDim.x * (16 * NWC));
                                           load_sid(item + gridDim.x * (16 * NWC));
                                       }
                                   });
        bias(c0, Y_CB2);
        run_layer16<NetColor16, 2>(wb, ldsi, slot, w, lane, lz, c0, [&](auto k) { return chain(c1, inv5, k); },
                                   [&](auto c) {
                                       if constexpr (decltype(c)::value == 0) {
                                           load_q(std::integral_constant<int, 2>{}, item + gridDim.x * (16 * NWC));
                                           load_ray();  // the next tile's ray ids
                                       }
                                   });
        // output layer: units 16 t + 4 g + i of this lane, summed over the 4 lane groups (the four
        // weights of a (t, c) as one 16-B LDS read: this file is built without SLP vectorisation)
        float o[3] = {0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            f32x4 wc[3];
#pragma unroll
            for (int c = 0; c < 3; ++c) wc[c] = *(const f32x4 *)(Yl + Y_CW3 + 128 * c + 16 * t + 4 * g);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float y = c0[t][i] * inv6;
                const float hv = lrelu_x3(y);
#pragma unroll
                for (int c = 0; c < 3; ++c) o[c] = __builtin_fmaf(wc[c][i], hv, o[c]);
            }
        }
        bool fin = true;  // the logits (the sigmoid maps +-inf to finite values) and k_rows16's alpha
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            float x = o[c] + __shfl_xor(o[c], 16);
            x += __shfl_xor(x, 32);
            const float z = x + Yl[Y_CB3 + c];
            fin = fin && __builtin_isfinite(z);
            o[c] = (1.f / (1.f + expf(-z))) * (1.f + 2.f * 0.001f) - 0.001f;
        }
        if (sval && g == 0) {
            a.feat[(int64_t)s * 4 + 1] = o[0];
            a.feat[(int64_t)s * 4 + 2] = o[1];
            a.feat[(int64_t)s * 4 + 3] = o[2];
            // fp16-range guard: an activation >= 65504 became inf in its hi part and NaN / inf in
            // every layer after it (mlp_x3.hip header); flag the call instead of returning it
            if (!(fin && __builtin_isfinite(a.feat[(int64_t)s * 4]))) *a.range_flag = 1;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
// ---- host-side packing ---------------------------------------------------------------------
// power of two 2^s with max |W| 2^s < 2^14 (so lo parts stay normal fp16 numbers)
int layer_shift(const float *W, size_t n) {
    float m = 0.f;
    for (size_t i = 0; i < n; ++i) m = fmaxf(m, fabsf(W[i]));
    if (!(m > 0.f) || !std::isfinite(m)) return 0;
    int e;
    frexpf(m, &e);  // m < 2^e
    return 14 - e;
}
// ksb > 0: w[9] / b[9] = block2_bpnet.0 ([256][256 + bpnet_dim], [256])
void pack_blob_x3(int ksb, int bpnet_dim, const float *const *w, const float *const *b, uint8_t *blob) {
    static const int shape[9][2] = {{256, 284}, {256, 256}, {256, 263}, {256, 256}, {1, 256},
                                    {128, 280}, {128, 128}, {128, 128}, {3, 128}};
    int s[9] = {};
    for (int L : {0, 1, 2, 3, 5, 6, 7}) s[L] = layer_shift(w[L], (size_t)shape[L][0] * shape[L][1]);
    const int sb = ksb > 0 ? layer_shift(w[9], (size_t)256 * (256 + bpnet_dim)) : 0;
    pack_blob16(ksb, bpnet_dim, w, b, s, sb, blob);
}

int variant_ksb(int32_t bpnet_layers, int32_t bpnet_dim) {
    if (bpnet_layers == 0) return 0;
    if (bpnet_layers == 1 && (bpnet_dim == 0 || bpnet_dim == BP_DIM)) return ks_bp(bpnet_dim);
    return -1;
}

}  // namespace x3
}  // namespace
}  // namespace sgn
extern "C" {

size_t sgn_mlp_packed_bytes_f32(int32_t bpnet_layers, int32_t bpnet_dim) {
    const int ksb = sgn::x3::variant_ksb(bpnet_layers, bpnet_dim);
    return ksb < 0 ? 0 : sgn::x3::blob_bytes_sg(ksb);
}

int sgn_mlp_pack_f32(int32_t bpnet_layers, int32_t bpnet_dim, const float *const *w, const float *const *b,
                     void *d_packed, sgn_stream_t stream) {
    using namespace sgn;
    SGN_REQUIRE(w && b && d_packed, "null argument");
    const int ksb = x3::variant_ksb(bpnet_layers, bpnet_dim);
    SGN_REQUIRE(ksb >= 0, "block2_bpnet: supported are 0 layers, or 1 layer with bpnet_dim 0 or 96");
    for (int L = 0; L < (ksb ? 10 : 9); ++L) SGN_REQUIRE(w[L] && b[L], "null layer pointer");
    std::vector<uint8_t> blob(x3::blob_bytes_sg(ksb), 0);
    x3::pack_blob_x3(ksb, bpnet_dim, w, b, blob.data());
    hipStream_t st = as_stream(stream);
    SGN_CHECK_HIP(hipMemcpyAsync(d_packed, blob.data(), blob.size(), hipMemcpyHostToDevice, st));
    SGN_CHECK_HIP(hipStreamSynchronize(st));
    return 0;
}

int sgn_mlp_pack_f32_host(int32_t bpnet_layers, int32_t bpnet_dim, const float *const *w, const float *const *b,
                          void *h_packed) {
    using namespace sgn;
    SGN_REQUIRE(w && b && h_packed, "null argument");
    const int ksb = x3::variant_ksb(bpnet_layers, bpnet_dim);
    SGN_REQUIRE(ksb >= 0, "block2_bpnet: supported are 0 layers, or 1 layer with bpnet_dim 0 or 96");
    for (int L = 0; L < (ksb ? 10 : 9); ++L) SGN_REQUIRE(w[L] && b[L], "null layer pointer");
    std::fill_n((uint8_t *)h_packed, x3::blob_bytes_sg(ksb), (uint8_t)0);
    x3::pack_blob_x3(ksb, bpnet_dim, w, b, (uint8_t *)h_packed);
    return 0;
}

int sgn_point_project_f32_subset(const sgn_point_tables *pt, const void *d_packed, const int32_t *d_idx,
                                 const int64_t *d_count, void *d_proj, sgn_stream_t stream) {
    using namespace sgn;
    SGN_REQUIRE(pt && d_packed && d_proj && d_idx && d_count, "null argument");
    SGN_REQUIRE(pt->n_points >= 0 && (pt->n_points == 0 || pt->embedding), "embedding required");
    SGN_REQUIRE(((uintptr_t)d_proj & 15) == 0 && ((uintptr_t)pt->embedding & 15) == 0, "16-byte alignment required");
    if (pt->n_points == 0) return 0;
    SGN_REQUIRE(pt->xyz && pt->color && pt->dir && pt->conf, "point tables (xyz, color, dir, conf) required");
    float *rec = (float *)((char *)d_proj + (size_t)pt->n_points * x3::PROJ_BYTES_PER_POINT);
    x3::Proj16Args a{pt->embedding, pt->n_points, d_packed, (float *)d_proj, pt->xyz, pt->color, pt->dir,
                     pt->conf, rec, d_idx, d_count};
    // persistent grid over the device count (a training step touches ~50 k of 1.2 M points)
    const int64_t tiles = (pt->n_points + 16 * x3::NW16 - 1) / (16 * x3::NW16);
    hipLaunchKernelGGL(x3::k_point_proj16, dim3((unsigned)(tiles < 256 ? tiles : 256)), dim3(x3::TPB16), 0,
                       as_stream(stream), a);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

size_t sgn_point_proj_bytes_f32(int64_t n_points) {
    // P rows, then the packed 64-B point records
    return (size_t)(n_points > 0 ? n_points : 0) * (sgn::x3::PROJ_BYTES_PER_POINT + sgn::x3::REC16_FLOATS * 4);
}

int sgn_point_project_f32(const sgn_point_tables *pt, const void *d_packed, void *d_proj, sgn_stream_t stream) {
    using namespace sgn;
    SGN_REQUIRE(pt && d_packed && d_proj, "null argument");
    SGN_REQUIRE(pt->n_points >= 0 && (pt->n_points == 0 || pt->embedding), "embedding required");
    SGN_REQUIRE(((uintptr_t)d_proj & 15) == 0 && ((uintptr_t)pt->embedding & 15) == 0, "16-byte alignment required");
    if (pt->n_points == 0) return 0;
    SGN_REQUIRE(pt->xyz && pt->color && pt->dir && pt->conf, "point tables (xyz, color, dir, conf) required");
    float *rec = (float *)((char *)d_proj + (size_t)pt->n_points * x3::PROJ_BYTES_PER_POINT);
    x3::Proj16Args a{pt->embedding, pt->n_points, d_packed, (float *)d_proj, pt->xyz, pt->color, pt->dir,
                     pt->conf, rec, nullptr, nullptr};
    const int64_t tiles = (pt->n_points + 16 * x3::NW16 - 1) / (16 * x3::NW16);
    hipLaunchKernelGGL(x3::k_point_proj16, dim3((unsigned)(tiles < 256 ? tiles : 256)), dim3(x3::TPB16), 0,
                       as_stream(stream), a);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

// Workspace: blended features of every work item (fp32, 1 KiB each), so the two stages may be
// called separately, then k_pair_slots' row table (32 B) and slot entries (16 B) per item, then a
// 2-KiB tail: [0] the slot count, [1] the fp16-range flag (k_color16; sgn_aggregate_check_f32).
// A smaller workspace is accepted with stages = 3 (both stages per chunk).
constexpr int64_t WS_PER_ITEM = sgn::mlp::HID * 4 + 32 + 16, WS_TAIL = 2048;
size_t sgn_aggregate_workspace_bytes_f32(int64_t S) {
    if (S < 32) S = 32;
    return (size_t)(S * WS_PER_ITEM + WS_TAIL);
}

namespace {
int32_t *ws_tail(void *d_workspace, size_t workspace_bytes) {
    const int64_t ws_items = workspace_bytes > (size_t)WS_TAIL ? (int64_t)((workspace_bytes - WS_TAIL) / WS_PER_ITEM) : 0;
    return (int32_t *)((char *)d_workspace + ws_items * WS_PER_ITEM);
}
}  // namespace

}  // extern "C"

namespace {
int aggregate_f32(int32_t bpnet_layers, int32_t bpnet_dim, const float *d_bpnet, const void *d_point_proj,
                  const sgn_point_tables *pt, const sgn_query_out *q, int64_t S_capacity, int32_t K,
                  const void *d_packed, float *d_out_feat, float *d_out_blend, float *d_out_wnorm,
                  void *d_workspace, size_t workspace_bytes, int32_t stages, sgn_stream_t stream,
                  float *const *z = nullptr, const int32_t *row_off = nullptr) {
    using namespace sgn;
    using namespace sgn::mlp;
    SGN_REQUIRE(pt && q && d_packed && d_out_feat && d_workspace && d_point_proj, "null argument");
    SGN_REQUIRE(stages >= 1 && stages <= 3, "stages must be 1 (rows), 2 (colour) or 3 (both)");
    const int ksb = x3::variant_ksb(bpnet_layers, bpnet_dim);
    SGN_REQUIRE(ksb >= 0, "block2_bpnet: supported are 0 layers, or 1 layer with bpnet_dim 0 or 96");
    SGN_REQUIRE(bpnet_dim == 0 || (d_bpnet && ((uintptr_t)d_bpnet & 15) == 0),
                "bpnet_dim > 0 needs the 16-byte aligned fp32 BPNet point embedding");
    SGN_REQUIRE(K >= 1 && K <= 8, "the fp32 MFMA aggregator takes K = 1 .. 8 neighbours per sample");
    SGN_REQUIRE(pt->campos && pt->camrotc2w && pt->raydir, "camera (campos, camrotc2w, raydir) required");
    SGN_REQUIRE((pt->pers == nullptr) == (pt->samp_pers == nullptr), "pers and samp_pers go together");
    SGN_REQUIRE(S_capacity >= 0 && S_capacity < (1 << 30), "S_capacity out of range");
    SGN_REQUIRE(((uintptr_t)d_workspace & 15) == 0 && ((uintptr_t)d_point_proj & 15) == 0, "16-byte alignment required");
    hipStream_t st = as_stream(stream);
    const int64_t ws_items = workspace_bytes > (size_t)WS_TAIL ? (int64_t)((workspace_bytes - WS_TAIL) / WS_PER_ITEM) : 0;
    SGN_REQUIRE(ws_items >= 32, "aggregate workspace too small");
    SGN_REQUIRE(stages == 3 || ws_items >= S_capacity,
                "stages 1 and 2 called separately need a workspace for all S_capacity items");
    // chunk = items per launch; with a full-size workspace chunk c keeps its rows at item c * chunk.
    // k_rows16 bases its f_s descriptor per tile (one launch per stage for any frame); k_pair_slots
    // packs chunk-relative items in 28 bits
    const bool full = ws_items >= S_capacity;
    const int64_t lim = ws_items < (1 << 27) ? ws_items : (1 << 27);
    const int64_t chunk = lim < S_capacity ? lim : (S_capacity > 32 ? S_capacity : 32);
    AggArgs a{};
    a.xyz = pt->xyz; a.emb = pt->embedding; a.color = pt->color; a.dir = pt->dir; a.conf = pt->conf;
    a.campos = pt->campos; a.rot = pt->camrotc2w; a.raydir = pt->raydir;
    a.pers = pt->pers; a.samp_pers = pt->samp_pers;
    a.counters = q->counters; a.work = q->work; a.samp_ray = q->samp_ray; a.pidx = q->pidx;
    a.samp_locw = q->samp_locw;
    a.K = K;
    a.blob = d_packed; a.blob_bytes = x3::blob_bytes_sg(ksb);
    a.bpnet32 = d_bpnet;
    a.proj = (const _Float16 *)d_point_proj;  // fp32 P table (k_rows16 reads it as float)
    a.rec = (const float *)((const char *)d_point_proj + (size_t)pt->n_points * x3::PROJ_BYTES_PER_POINT);
    a.feat = d_out_feat; a.blend = d_out_blend; a.wnorm = d_out_wnorm; a.fs = (_Float16 *)d_workspace;
    int32_t *tail = ws_tail(d_workspace, workspace_bytes);
    int32_t *rows = (int32_t *)((char *)d_workspace + ws_items * mlp::HID * 4);
    int4 *slots = (int4 *)(rows + ws_items * 8);
    int32_t *slot_n = tail;
    a.rows = rows; a.slots = slots; a.slot_n = slot_n;
    if (z) {
        a.z1 = z[0]; a.z2 = z[1]; a.z3 = z[2]; a.zb = z[3];
        a.row_off = row_off;
    }
    // SGN_PAIR=0 runs every sample alone in its k_rows16 half (same results, bit for bit; tests)
    const char *pe = getenv("SGN_PAIR");
    const int32_t pair = !(pe && pe[0] == '0');
    if (stages & 1) {
        // a paired half writes only its samples' valid rows: the optional per-slot outputs start at 0
        if (d_out_blend) SGN_CHECK_HIP(hipMemsetAsync(d_out_blend, 0, (size_t)S_capacity * K * 4, st));
        if (d_out_wnorm) SGN_CHECK_HIP(hipMemsetAsync(d_out_wnorm, 0, (size_t)S_capacity * K * 4, st));
    }
    // the fp16-range flag covers the samples of this call's colour stage (cleared with its first chunk)
    if (stages & 2) SGN_CHECK_HIP(hipMemsetAsync(tail + 1, 0, 4, st));
    x3::ColorArgs c{q->counters, q->work, q->samp_ray, pt->raydir, d_packed, (const float *)d_workspace, d_out_feat,
                    tail + 1, 0, 0};
    for (int64_t i0 = 0; i0 < S_capacity; i0 += chunk) {
        const int64_t n = S_capacity - i0 < chunk ? S_capacity - i0 : chunk;
        a.item0 = c.item0 = (int32_t)i0;
        a.n_items = c.n_items = (int32_t)n;
        float *fs = (float *)d_workspace + (full ? i0 * mlp::HID : 0);
        a.fs = (_Float16 *)fs;
        c.fs = fs;
        if (stages & 1) {
            SGN_CHECK_HIP(hipMemsetAsync(slot_n, 0, 4, st));
            const int64_t pb = (n + x3::PAIR_TPB - 1) / x3::PAIR_TPB;
            hipLaunchKernelGGL(x3::k_pair_slots, dim3((unsigned)(pb < 1024 ? pb : 1024)),
                               dim3(x3::PAIR_TPB), 0, st, q->counters, q->work, q->samp_nnb, (int32_t)i0, (int32_t)n,
                               pair, rows, slots, slot_n);
            // inference rows: 32 rows per wave (NS = 2; 0.94x the time of NS = 1 at config 2,
            // profiles/r04_v2_bench_rows_ns*.json); the save mode (training) keeps NS = 1
            const int ns = z ? 1 : 2;
            auto kern = z ? (ksb == 0 ? x3::k_rows16<0, false, true> : ksb == KS_HID ? x3::k_rows16<8, false, true>
                                                                                  : x3::k_rows16<11, false, true>)
                          : pt->pers ? (ksb == 0 ? x3::k_rows16<0, true, false, 2> : ksb == KS_HID ? x3::k_rows16<8, true, false, 2>
                                                                                      : x3::k_rows16<11, true, false, 2>)
                                     : (ksb == 0 ? x3::k_rows16<0, false, false, 2> : ksb == KS_HID ? x3::k_rows16<8, false, false, 2>
                                                                                        : x3::k_rows16<11, false, false, 2>);
            const int64_t wg16 = (n + x3::WG16_SAMPLES * ns - 1) / (x3::WG16_SAMPLES * ns),
                          wmax = ns == 1 ? 256 * (8 / x3::NWR) : 256;
            hipLaunchKernelGGL(kern, dim3((unsigned)(wg16 < wmax ? wg16 : wmax)), dim3(x3::TPBR), 0, st, a);
        }
        if (stages & 2) {
            const int64_t wgc = (n + 16 * x3::NWC - 1) / (16 * x3::NWC), wcmax = 256 * (8 / x3::NWC);
            hipLaunchKernelGGL(x3::k_color16, dim3((unsigned)(wgc < wcmax ? wgc : wcmax)), dim3(x3::TPBC), 0, st, c);
        }
    }
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

}  // namespace

extern "C" {

int sgn_aggregate_f32(int32_t bpnet_layers, int32_t bpnet_dim, const float *d_bpnet, const void *d_point_proj,
                      const sgn_point_tables *pt, const sgn_query_out *q, int64_t S_capacity, int32_t K,
                      const void *d_packed, float *d_out_feat, float *d_out_blend, float *d_out_wnorm,
                      void *d_workspace, size_t workspace_bytes, int32_t stages, sgn_stream_t stream) {
    return aggregate_f32(bpnet_layers, bpnet_dim, d_bpnet, d_point_proj, pt, q, S_capacity, K, d_packed, d_out_feat,
                         d_out_blend, d_out_wnorm, d_workspace, workspace_bytes, stages, stream);
}

int sgn_aggregate_train_fwd_f32(const void *d_point_proj, const sgn_point_tables *pt, const sgn_query_out *q,
                                int64_t S_capacity, int32_t K, const void *d_packed, float *d_out_feat,
                                float *d_z1, float *d_z2, float *d_z3, const int32_t *d_row_off, void *d_workspace,
                                size_t workspace_bytes, sgn_stream_t stream) {
    SGN_REQUIRE(d_z1 && d_z2 && d_z3 && ((uintptr_t)d_z1 & 15) == 0 && ((uintptr_t)d_z2 & 15) == 0 &&
                    ((uintptr_t)d_z3 & 15) == 0,
                "16-byte aligned pre-activation buffers z1, z2, z3 required");
    SGN_REQUIRE(pt && pt->pers == nullptr, "the training forward computes the pers coordinates itself");
    float *const z[4] = {d_z1, d_z2, d_z3, nullptr};
    return aggregate_f32(0, 0, nullptr, d_point_proj, pt, q, S_capacity, K, d_packed, d_out_feat, nullptr, nullptr,
                         d_workspace, workspace_bytes, 1, stream, z, d_row_off);
}

int sgn_aggregate_train_fwd_f32_sg(int32_t bpnet_layers, int32_t bpnet_dim, const float *d_bpnet,
                                   const void *d_point_proj, const sgn_point_tables *pt, const sgn_query_out *q,
                                   int64_t S_capacity, int32_t K, const void *d_packed, float *d_out_feat, float *d_z1,
                                   float *d_z2, float *d_zb, float *d_z3, const int32_t *d_row_off, void *d_workspace,
                                   size_t workspace_bytes, sgn_stream_t stream) {
    SGN_REQUIRE(bpnet_layers == 1, "the SG training forward has one block2_bpnet layer");
    SGN_REQUIRE(d_z1 && d_z2 && d_zb && d_z3 && ((uintptr_t)d_z1 & 15) == 0 && ((uintptr_t)d_z2 & 15) == 0 &&
                    ((uintptr_t)d_zb & 15) == 0 && ((uintptr_t)d_z3 & 15) == 0,
                "16-byte aligned pre-activation buffers z1, z2, zb, z3 required");
    SGN_REQUIRE(pt && pt->pers == nullptr, "the training forward computes the pers coordinates itself");
    float *const z[4] = {d_z1, d_z2, d_z3, d_zb};
    return aggregate_f32(bpnet_layers, bpnet_dim, d_bpnet, d_point_proj, pt, q, S_capacity, K, d_packed, d_out_feat,
                         nullptr, nullptr, d_workspace, workspace_bytes, 1, stream, z, d_row_off);
}

int sgn_mlp_pack_index_f32(int32_t bpnet_layers, int32_t bpnet_dim, int32_t which, int32_t *out, int64_t n) {
    using namespace sgn;
    const int ksb = x3::variant_ksb(bpnet_layers, bpnet_dim);
    SGN_REQUIRE(ksb >= 0, "block2_bpnet: supported are 0 layers, or 1 layer with bpnet_dim 0 or 96");
    SGN_REQUIRE(out && (which == 0 || which == 1), "which: 0 fragment section, 1 fp32 section");
    const size_t n16 = x3::OFF16_F32 / 2, n32 = x3::N_Y32;
    SGN_REQUIRE((size_t)n == (which == 0 ? n16 : n32), "index map length (sgn_mlp_layout_f32)");
    std::vector<int32_t> a(n16), b(n32);
    x3::index_blob16(ksb, bpnet_dim, a.data(), n16, b.data(), n32);
    const std::vector<int32_t> &src = which == 0 ? a : b;
    for (size_t i = 0; i < src.size(); ++i) out[i] = src[i];
    return 0;
}

int64_t sgn_mlp_layout_f32(int32_t which) {
    // 0: bytes of the fragment section (= byte offset of the fp32 section), 1: fp32 entries after it
    return which == 0 ? (int64_t)sgn::x3::OFF16_F32 : which == 1 ? (int64_t)sgn::x3::N_Y32 : -1;
}

int sgn_aggregate_check_f32(const void *d_workspace, size_t workspace_bytes, sgn_stream_t stream) {
    using namespace sgn;
    SGN_REQUIRE(d_workspace && workspace_bytes >= (size_t)(32 * WS_PER_ITEM + WS_TAIL), "null or too small workspace");
    const int32_t *flag = ws_tail(const_cast<void *>(d_workspace), workspace_bytes) + 1;
    int32_t h = 0;
    hipStream_t st = as_stream(stream);
    SGN_CHECK_HIP(hipMemcpyAsync(&h, flag, 4, hipMemcpyDeviceToHost, st));
    SGN_CHECK_HIP(hipStreamSynchronize(st));
    SGN_REQUIRE(h == 0, "fp16 range exceeded: an aggregator activation or point feature reached |x| >= 65504, so "
                        "the split-fp16 MFMA operands overflowed and the decoded features of the last "
                        "sgn_aggregate_f32 call are not finite");
    return 0;
}

int64_t sgn_aggregate_fs_offset_f32(size_t workspace_bytes, int64_t S_capacity) {
    // aggregate_f32 keeps item i's f_s at d_workspace + i * 1 KiB when the workspace holds every item
    // (`full`), else it reuses the first rows chunk by chunk
    const int64_t ws_items = workspace_bytes > (size_t)WS_TAIL ? (int64_t)((workspace_bytes - WS_TAIL) / WS_PER_ITEM) : 0;
    return S_capacity >= 0 && ws_items >= 32 && ws_items >= S_capacity ? 0 : -1;
}

size_t sgn_aggregate_flag_offset_f32(size_t workspace_bytes) {
    const int64_t ws_items = workspace_bytes > (size_t)WS_TAIL ? (int64_t)((workspace_bytes - WS_TAIL) / WS_PER_ITEM) : 0;
    return (size_t)(ws_items * WS_PER_ITEM + 4);
}

}  // extern "C"
