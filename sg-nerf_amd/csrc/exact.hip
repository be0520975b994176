// exact.hip -- the aggregator and colour MLP in plain fp32 on v_mfma_f32_16x16x4_f32: the f32
// mode's range fallback.
//
// The fast fp32-faithful kernels (mlp_x3.hip) carry every activation as an fp16 (hi, lo) pair, so
// an activation with |x| >= 65504 cannot be represented there; k_color16 flags such a frame
// (counters / sgn_aggregate_check_f32).  The reference has no such limit: nn.Linear in fp32
// (point_aggregators.py:561-786 viewmlp, :868-959 forward).  The host re-runs a flagged frame's
// aggregation here: the same gather, dists, weights and K-blend, every nn.Linear as fp32 MFMAs
// with fp32 operands (each MFMA a k-ordered fmaf chain: exact fp32 products, fp32 sums) on the
// weights exactly as the checkpoint holds them -- no power-of-two scaling, no fp16 anywhere, so
// any activation fp32 holds is carried.  Slower than the split path (the fp32-input MFMA peak is
// 1/16 of the fp16 one), and only used for frames the split path cannot represent.
//
// Layout: a wave owns 16 rows (2 samples x 8 neighbour slots; row k >= K or without a neighbour
// is idle); lane l holds row r = l & 15 and, per output tile U of 16 units, units 16 U + 4 g + i
// (g = l >> 4, i = 0..3) -- the 16x16x4 accumulator layout.  The next layer's k-step (T, i) takes
// channel 16 T + 4 g + i of the row from the lane's own accumulator register, so activations
// never move; the weight operand W[16 U + r][16 T + 4 g + i] is read from a chunk of W^T staged in
// LDS (row stride 260 floats: the four lane groups of one read hit disjoint banks).
#include <vector>

#include "agg_device.h"
#include "x3_split.h"

namespace sgn {
namespace {
namespace xe {

constexpr int NW = 4, TPB = NW * 64;
constexpr int KCH = 32;                 // W^T rows (input channels) per staged chunk
constexpr int LSTR = 256 + 4;           // floats per staged row
constexpr int NL = 10;                  // block1.0, block1.2, block2_bpnet.0, block3.0, block3.2, alpha,
                                        // colour 0, 2, 4, 6
enum { LB10 = 0, LB12, LBP, LB30, LB32, LA, LC0, LC2, LC4, LC6 };

// per layer: in (reference width), in_pad (multiple of 16), out; wt = W^T [in_pad][out] and b [out]
// (float offsets into the exact blob); alpha / colour 6 keep W [out][in] (per-lane dot products)
struct XLayer {
    int in, in_pad, out;
    uint32_t wt, b;
};
struct XLayout {
    XLayer l[NL];
    uint32_t floats;
};

__host__ __device__ inline XLayout x_layout(int bpnet_layers, int bpnet_dim) {
    XLayout x{};
    const int shape[NL][2] = {{284, 256}, {256, 256}, {256 + bpnet_dim, 256}, {263, 256}, {256, 256},
                              {256, 1},   {280, 128}, {128, 128},             {128, 128}, {128, 3}};
    uint32_t off = 0;
    for (int L = 0; L < NL; ++L) {
        XLayer &y = x.l[L];
        y.in = shape[L][0];
        y.out = shape[L][1];
        y.in_pad = (y.in + 15) / 16 * 16;
        if (L == LBP && bpnet_layers == 0) y.in = y.in_pad = y.out = 0;
        y.wt = off;
        off += (uint32_t)(y.in_pad * y.out);
        y.b = off;
        off += (uint32_t)((y.out + 3) / 4 * 4);
    }
    x.floats = off;
    return x;
}

struct XArgs {
    AggArgs a;
    const float *w;  // exact blob
    XLayout lay;
    float *fs;       // [items of the chunk][256] blended features
    int bpnet_dim;
};

__device__ __forceinline__ float lrelu_x(float x) { return fmaxf(x, 0.01f * x); }

// value c (0..5, runtime) of d[6]
__device__ __forceinline__ float pick6(const float (&d)[6], int c) {
    float v = d[0];
#pragma unroll
    for (int j = 1; j < 6; ++j) v = c == j ? d[j] : v;
    return v;
}

// acc[U] += W x over input tiles T = 0 .. NT - 1: in(T) returns this lane's four channels
// 16 T + 4 g + i of its row; W^T rows come from global memory through LDS, KCH at a time.
template <int NU, int NT, class In>
__device__ __forceinline__ void layer_x(const float *__restrict__ wt, float *lds, f32x4 (&acc)[NU], int g, int r,
                                        In &&in) {
    constexpr int OUT = 16 * NU, Q4 = OUT / 4;
    static_for<(NT + 1) / 2>([&](auto cc) {
        constexpr int C0 = 2 * decltype(cc)::value, NTC = NT - C0 < 2 ? NT - C0 : 2;
        constexpr int NQ = NTC * 16 * Q4;
        __builtin_amdgcn_sched_barrier(0);
        __syncthreads();  // every wave is done with the previous chunk
        __builtin_amdgcn_sched_barrier(0);  // (the staging loads stay here, not hoisted chunks ahead)
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));  // the chunk's staging addresses are computed here, not hoisted
        for (int q = tid; q < NQ; q += TPB) {
            const int row = q / Q4, c4 = q - row * Q4;
            *(f32x4 *)(lds + row * LSTR + 4 * c4) = *(const f32x4 *)(wt + (size_t)(16 * C0 + row) * OUT + 4 * c4);
        }
        __builtin_amdgcn_sched_barrier(0);
        __syncthreads();
        static_for<NTC>([&](auto tt) {
            constexpr int T = C0 + decltype(tt)::value;
            const f32x4 x = in(std::integral_constant<int, T>{});
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                // one k-step at a time: without the fence the scheduler hoists the whole chunk's LDS
                // reads ahead of its MFMAs and spills
                __builtin_amdgcn_sched_barrier(0);
                const float *wl = lds + (16 * (T - C0) + 4 * g + i) * LSTR + r;
#pragma unroll
                for (int U = 0; U < NU; ++U) acc[U] = __builtin_amdgcn_mfma_f32_16x16x4f32(wl[16 * U], x[i], acc[U], 0, 0, 0);
            }
        });
    });
}

template <int NU>
__device__ __forceinline__ void bias_x(f32x4 (&acc)[NU], const float *b, int g) {
#pragma unroll
    for (int U = 0; U < NU; ++U) acc[U] = *(const f32x4 *)(b + 16 * U + 4 * g);
}

// one row per lane group position: (item, slot) -> gather, dists, weights (point_aggregators.py:868-953)
struct XRow {
    bool sval, m;
    int s, pid, ray;
    float d[6], ext[8], wgt;
};

template <bool PERS>
__device__ __forceinline__ XRow x_row(const AggArgs &a, const Cam &cam, int item, int end, int k) {
    XRow x;
    x.sval = item < end;
    x.s = x.sval ? a.work[item] : 0;
    x.pid = x.sval && k < a.K ? a.pidx[(int64_t)x.s * a.K + k] : -1;
    x.m = x.pid >= 0;
    x.ray = x.sval ? a.samp_ray[x.s] : 0;
    const int64_t s = x.s, pid = x.m ? x.pid : 0;
    const float lx = a.samp_locw[s * 3], ly = a.samp_locw[s * 3 + 1], lz = a.samp_locw[s * 3 + 2];
    const float vx = a.raydir[(int64_t)x.ray * 3], vy = a.raydir[(int64_t)x.ray * 3 + 1],
                vz = a.raydir[(int64_t)x.ray * 3 + 2];
    const float px = a.xyz[pid * 3], py = a.xyz[pid * 3 + 1], pz = a.xyz[pid * 3 + 2];
    const float dwx = __fsub_rn(px, lx), dwy = __fsub_rn(py, ly), dwz = __fsub_rn(pz, lz);
    float xp, yp, zp, xl, yl, zl;
    if constexpr (PERS) {
        xp = a.pers[pid * 3]; yp = a.pers[pid * 3 + 1]; zp = a.pers[pid * 3 + 2];
        xl = a.samp_pers[s * 3]; yl = a.samp_pers[s * 3 + 1]; zl = a.samp_pers[s * 3 + 2];
    } else {
        cam.pers(px, py, pz, xp, yp, zp);
        cam.pers(lx, ly, lz, xl, yl, zl);
    }
    x.d[0] = x.m ? dwx : 0.f;
    x.d[1] = x.m ? dwy : 0.f;
    x.d[2] = x.m ? dwz : 0.f;
    x.d[3] = x.m ? __fsub_rn(__fmul_rn(xp, zp), __fmul_rn(xl, zl)) : 0.f;
    x.d[4] = x.m ? __fsub_rn(__fmul_rn(yp, zp), __fmul_rn(yl, zl)) : 0.f;
    x.d[5] = x.m ? __fsub_rn(zp, zl) : 0.f;
    float w = 0.f;
    if (x.m) {
        const float n2 = __fadd_rn(__fadd_rn(__fmul_rn(dwx, dwx), __fmul_rn(dwy, dwy)), __fmul_rn(dwz, dwz));
        w = 1.f / fmaxf(sqrtf(n2), 1e-6f);
    }
    const float wsum = dpp_sum8(w);  // the sample's 8 slots are 8 consecutive lanes
    w = w / fmaxf(wsum, 1e-8f);
    const float cf = x.m ? a.conf[pid] : 0.f;
    x.wgt = w * fminf(fmaxf(cf, 1e-4f), 1.f);
    if (x.sval && k < a.K && (threadIdx.x & 63) < 16) {
        if (a.blend) a.blend[s * a.K + k] = x.wgt;
        if (a.wnorm) a.wnorm[s * a.K + k] = w;
    }
    // block3's extra channels: colour, dir - v, <dir, v> (:639-652)
    const float c0 = a.color[pid * 3], c1 = a.color[pid * 3 + 1], c2 = a.color[pid * 3 + 2];
    const float e0 = a.dir[pid * 3], e1 = a.dir[pid * 3 + 1], e2 = a.dir[pid * 3 + 2];
    x.ext[0] = x.m ? c0 : 0.f;
    x.ext[1] = x.m ? c1 : 0.f;
    x.ext[2] = x.m ? c2 : 0.f;
    x.ext[3] = x.m ? __fsub_rn(e0, vx) : 0.f;
    x.ext[4] = x.m ? __fsub_rn(e1, vy) : 0.f;
    x.ext[5] = x.m ? __fsub_rn(e2, vz) : 0.f;
    x.ext[6] = x.m ? __fadd_rn(__fadd_rn(__fmul_rn(e0, vx), __fmul_rn(e1, vy)), __fmul_rn(e2, vz)) : 0.f;
    x.ext[7] = 0.f;
    return x;
}

// SG: KSG > 0 adds block2_bpnet.0 ([h | BPNet embedding of bpnet_dim] -> 256) between block1.2
// and block3.0 (point_aggregators.py:345-354, :629-636)
template <bool PERS, int NTB>
__global__ __launch_bounds__(TPB, 1) void k_rows_exact(XArgs xa) {
    __shared__ __attribute__((aligned(16))) float lds[KCH * LSTR];
    const AggArgs &a = xa.a;
    const XLayout &ly = xa.lay;
    const int lane = threadIdx.x & 63, r = lane & 15, k = r & 7;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int end = min(a.counters[1], a.item0 + a.n_items);
    const Cam cam = load_cam(a.campos, a.rot);
    const int ntile = (a.n_items + 2 * NW - 1) / (2 * NW);
    for (int tile = blockIdx.x; tile < ntile; tile += gridDim.x) {  // workgroup-uniform trip count
        // g opaque per tile: the per-lane channel arithmetic of the encodings is recomputed where it is
        // used instead of hoisted out of the loop (hundreds of loop-invariant registers, spilled)
        int g = lane >> 4;
        asm volatile("" : "+v"(g));
        const int item = a.item0 + tile * 2 * NW + 2 * w + (r >> 3);
        const XRow x = x_row<PERS>(a, cam, item, end, k);
        const int64_t pid = x.m ? x.pid : 0;
        const float *emb = a.emb + pid * 32;
        // block1.0: [feat 32 | PE(feat, 3) 192 | PE(dists, 5) 60] (networks.py:175-192: sin / cos
        // interleaved per (component, frequency)) -> 256
        f32x4 h0[16];
        bias_x(h0, xa.w + ly.l[LB10].b, g);
        layer_x<16, 18>(xa.w + ly.l[LB10].wt, lds, h0, g, r, [&](auto tc) {
            constexpr int T = decltype(tc)::value;
            f32x4 v{};
            if constexpr (T < 2) {
                v = x.m ? *(const f32x4 *)(emb + 16 * T + 4 * g) : f32x4{};
            } else if constexpr (T < 14) {
                // channels 32 + 2 (3 c + f) + {sin, cos}: lane pairs (i = 0, 1) and (2, 3) share an argument
#pragma unroll
                for (int hp = 0; hp < 2; ++hp) {
                    const int q = (16 * T + 4 * g + 2 * hp - 32) >> 1, c = q / 3, f = q - 3 * c;
                    float sv, cv;
                    sincos_acc(emb[c] * (float)(1 << f), sv, cv);
                    v[2 * hp] = x.m ? sv : 0.f;
                    v[2 * hp + 1] = x.m ? cv : 0.f;
                }
            } else {
#pragma unroll
                for (int hp = 0; hp < 2; ++hp) {
                    const int j = 16 * T + 4 * g + 2 * hp - 224;
                    if (j < 60) {
                        const int q = j >> 1, c = q / 5, f = q - 5 * c;
                        float sv, cv;
                        sincos_acc(pick6(x.d, c) * (float)(1 << f), sv, cv);
                        v[2 * hp] = x.m ? sv : 0.f;
                        v[2 * hp + 1] = x.m ? cv : 0.f;
                    }
                }
            }
            return v;
        });
        auto chain = [](const f32x4 (&h)[16]) {
            return [&h](auto tc) {
                constexpr int T = decltype(tc)::value;
                f32x4 v;
#pragma unroll
                for (int i = 0; i < 4; ++i) v[i] = lrelu_x(h[T][i]);
                return v;
            };
        };
        f32x4 h1[16];
        bias_x(h1, xa.w + ly.l[LB12].b, g);
        layer_x<16, 16>(xa.w + ly.l[LB12].wt, lds, h1, g, r, chain(h0));
        if constexpr (NTB > 0) {  // block2_bpnet.0 into h0
            bias_x(h0, xa.w + ly.l[LBP].b, g);
            const float *bp = a.bpnet32 ? a.bpnet32 + pid * xa.bpnet_dim : nullptr;
            layer_x<16, NTB>(xa.w + ly.l[LBP].wt, lds, h0, g, r, [&](auto tc) {
                constexpr int T = decltype(tc)::value;
                f32x4 v;
                if constexpr (T < 16) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) v[i] = lrelu_x(h1[T][i]);
                } else {
                    v = x.m && bp ? *(const f32x4 *)(bp + 16 * (T - 16) + 4 * g) : f32x4{};
                }
                return v;
            });
        }
        auto &hin = pick<(NTB > 0)>(h0, h1);
        // block3.0: [h 256 | colour, dir - v, <dir, v>] -> 256, into the array block1.2 / block2_bpnet left
        f32x4 h2[16];
        bias_x(h2, xa.w + ly.l[LB30].b, g);
        layer_x<16, 17>(xa.w + ly.l[LB30].wt, lds, h2, g, r, [&](auto tc) {
            constexpr int T = decltype(tc)::value;
            f32x4 v;
            if constexpr (T < 16) {
#pragma unroll
                for (int i = 0; i < 4; ++i) v[i] = lrelu_x(hin[T][i]);
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) v[i] = g == 0 ? x.ext[i] : g == 1 ? x.ext[4 + i] : 0.f;
            }
            return v;
        });
        f32x4 h3[16];
        bias_x(h3, xa.w + ly.l[LB32].b, g);
        layer_x<16, 16>(xa.w + ly.l[LB32].wt, lds, h3, g, r, chain(h2));
        // epilogue (:743-770): h = LReLU(block3.2), alpha = softplus(W_a h + b_a - 1), K-blend of
        // h and alpha over the sample's rows with weight * conf
        const float *wa = xa.w + ly.l[LA].wt;
        float dot = 0.f;
#pragma unroll
        for (int U = 0; U < 16; ++U) {
            const f32x4 wv = *(const f32x4 *)(wa + 16 * U + 4 * g);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                h3[U][i] = lrelu_x(h3[U][i]);
                dot = __builtin_fmaf(wv[i], h3[U][i], dot);
            }
        }
        dot += __shfl_xor(dot, 16);
        dot += __shfl_xor(dot, 32);
        const float alpha = softplus(dot + xa.w[ly.l[LA].b] - 1.f);
        const float as = dpp_sum8(x.m ? x.wgt * alpha : 0.f);
        const bool lead = x.sval && k == 0;
        if (lead && g == 0) a.feat[(int64_t)x.s * 4] = as;
        float *fs = xa.fs + (int64_t)(item - a.item0) * HID;
#pragma unroll
        for (int U = 0; U < 16; ++U) {
            f32x4 o;
#pragma unroll
            for (int i = 0; i < 4; ++i) o[i] = dpp_sum8(x.m ? x.wgt * h3[U][i] : 0.f);
            if (lead) *(f32x4 *)(fs + 16 * U + 4 * g) = o;
        }
    }
}

// colour MLP (point_aggregators.py:779-786): [f_s | PE(viewdir, 4) sin 12 | cos 12] -> 128 -> 128
// -> 128 -> 3, sigmoid * (1 + 2e-3) - 1e-3; 16 work items per wave, one per lane row
__global__ __launch_bounds__(TPB, 1) void k_color_exact(XArgs xa) {
    __shared__ __attribute__((aligned(16))) float lds[KCH * LSTR];
    const AggArgs &a = xa.a;
    const XLayout &ly = xa.lay;
    const int lane = threadIdx.x & 63, g = lane >> 4, r = lane & 15;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int end = min(a.counters[1], a.item0 + a.n_items);
    const int ntile = (a.n_items + 16 * NW - 1) / (16 * NW);
    for (int tile = blockIdx.x; tile < ntile; tile += gridDim.x) {
        const int item = a.item0 + tile * 16 * NW + 16 * w + r;
        const bool sval = item < end;
        const int s = sval ? a.work[item] : 0;
        const int ray = a.samp_ray[s];
        const float v3[3] = {a.raydir[(int64_t)ray * 3], a.raydir[(int64_t)ray * 3 + 1], a.raydir[(int64_t)ray * 3 + 2]};
        const float *fs = xa.fs + (int64_t)(sval ? item - a.item0 : 0) * HID;
        f32x4 c0[8], c1[8];
        bias_x(c0, xa.w + ly.l[LC0].b, g);
        layer_x<8, 18>(xa.w + ly.l[LC0].wt, lds, c0, g, r, [&](auto tc) {
            constexpr int T = decltype(tc)::value;
            f32x4 v{};
            if constexpr (T < 16) {
                v = *(const f32x4 *)(fs + 16 * T + 4 * g);
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int j = 16 * (T - 16) + 4 * g + i;  // 0..11 sin, 12..23 cos of v_c 2^f, c = q / 4
                    if (j < 24) {
                        const int q = j < 12 ? j : j - 12, c = q >> 2, f = q & 3;
                        const float vc = c == 0 ? v3[0] : c == 1 ? v3[1] : v3[2];
                        float sv, cv;
                        sincos_acc(vc * (float)(1 << f), sv, cv);
                        v[i] = j < 12 ? sv : cv;
                    }
                }
            }
            return v;
        });
        auto chain8 = [](const f32x4 (&h)[8]) {
            return [&h](auto tc) {
                constexpr int T = decltype(tc)::value;
                f32x4 v;
#pragma unroll
                for (int i = 0; i < 4; ++i) v[i] = lrelu_x(h[T][i]);
                return v;
            };
        };
        bias_x(c1, xa.w + ly.l[LC2].b, g);
        layer_x<8, 8>(xa.w + ly.l[LC2].wt, lds, c1, g, r, chain8(c0));
        bias_x(c0, xa.w + ly.l[LC4].b, g);
        layer_x<8, 8>(xa.w + ly.l[LC4].wt, lds, c0, g, r, chain8(c1));
        const float *w6 = xa.w + ly.l[LC6].wt, *b6 = xa.w + ly.l[LC6].b;
        float o[3] = {0.f, 0.f, 0.f};
#pragma unroll
        for (int U = 0; U < 8; ++U) {
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const f32x4 wv = *(const f32x4 *)(w6 + c * 128 + 16 * U + 4 * g);
#pragma unroll
                for (int i = 0; i < 4; ++i) o[c] = __builtin_fmaf(wv[i], lrelu_x(c0[U][i]), o[c]);
            }
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            float z = o[c] + __shfl_xor(o[c], 16);
            z += __shfl_xor(z, 32);
            z += b6[c];
            o[c] = (1.f / (1.f + expf(-z))) * (1.f + 2.f * 0.001f) - 0.001f;
        }
        if (sval && g == 0) {
            a.feat[(int64_t)s * 4 + 1] = o[0];
            a.feat[(int64_t)s * 4 + 2] = o[1];
            a.feat[(int64_t)s * 4 + 3] = o[2];
        }
    }
}

}  // namespace xe
}  // namespace
}  // namespace sgn

extern "C" {

size_t sgn_mlp_packed_bytes_exact(int32_t bpnet_layers, int32_t bpnet_dim) {
    if (!(bpnet_layers == 0 || (bpnet_layers == 1 && (bpnet_dim == 0 || bpnet_dim == 96)))) return 0;
    return (size_t)sgn::xe::x_layout(bpnet_layers, bpnet_dim).floats * 4;
}

// weights in the order of sgn_mlp_pack_f32: block1.0, block1.2, block3.0, block3.2, alpha_branch.0,
// color_branch.0, .2, .4, .6 (+ block2_bpnet.0 as 9); W [out][in] row-major fp32 as nn.Linear holds it
int sgn_mlp_pack_exact(int32_t bpnet_layers, int32_t bpnet_dim, const float *const *w, const float *const *b,
                       void *d_packed, sgn_stream_t stream) {
    using namespace sgn;
    using namespace sgn::xe;
    SGN_REQUIRE(w && b && d_packed, "null argument");
    SGN_REQUIRE(bpnet_layers == 0 || (bpnet_layers == 1 && (bpnet_dim == 0 || bpnet_dim == 96)),
                "block2_bpnet: supported are 0 layers, or 1 layer with bpnet_dim 0 or 96");
    const XLayout ly = x_layout(bpnet_layers, bpnet_dim);
    const int src[NL] = {0, 1, 9, 2, 3, 4, 5, 6, 7, 8};  // x_layout layer -> argument index
    std::vector<float> blob(ly.floats, 0.f);
    for (int L = 0; L < NL; ++L) {
        const XLayer &y = ly.l[L];
        if (y.out == 0) continue;
        const float *W = w[src[L]], *B = b[src[L]];
        SGN_REQUIRE(W && B, "null layer pointer");
        if (L == LA || L == LC6) {  // W [out][in] for the per-lane dot products
            for (int o = 0; o < y.out; ++o)
                for (int i = 0; i < y.in; ++i) blob[y.wt + (size_t)o * y.in_pad + i] = W[(size_t)o * y.in + i];
        } else {  // W^T [in_pad][out]
            for (int o = 0; o < y.out; ++o)
                for (int i = 0; i < y.in; ++i) blob[y.wt + (size_t)i * y.out + o] = W[(size_t)o * y.in + i];
        }
        for (int o = 0; o < y.out; ++o) blob[y.b + o] = B[o];
    }
    hipStream_t st = as_stream(stream);
    SGN_CHECK_HIP(hipMemcpyAsync(d_packed, blob.data(), blob.size() * 4, hipMemcpyHostToDevice, st));
    SGN_CHECK_HIP(hipStreamSynchronize(st));
    return 0;
}

int sgn_aggregate_exact(int32_t bpnet_layers, int32_t bpnet_dim, const float *d_bpnet, const sgn_point_tables *pt,
                        const sgn_query_out *q, int64_t S_capacity, int32_t K, const void *d_packed_exact,
                        float *d_out_feat, float *d_out_blend, float *d_out_wnorm, void *d_workspace,
                        size_t workspace_bytes, sgn_stream_t stream) {
    using namespace sgn;
    using namespace sgn::xe;
    SGN_REQUIRE(pt && q && d_packed_exact && d_out_feat && d_workspace, "null argument");
    SGN_REQUIRE(bpnet_layers == 0 || (bpnet_layers == 1 && (bpnet_dim == 0 || bpnet_dim == 96)),
                "block2_bpnet: supported are 0 layers, or 1 layer with bpnet_dim 0 or 96");
    SGN_REQUIRE(bpnet_dim == 0 || (d_bpnet && ((uintptr_t)d_bpnet & 15) == 0),
                "bpnet_dim > 0 needs the 16-byte aligned fp32 BPNet point embedding");
    SGN_REQUIRE(K >= 1 && K <= 8, "the aggregator takes K = 1 .. 8 neighbours per sample");
    SGN_REQUIRE(pt->xyz && pt->embedding && pt->color && pt->dir && pt->conf, "point tables required");
    SGN_REQUIRE(((uintptr_t)pt->embedding & 15) == 0 && ((uintptr_t)d_packed_exact & 15) == 0 &&
                    ((uintptr_t)d_workspace & 15) == 0,
                "16-byte alignment required");
    SGN_REQUIRE(pt->campos && pt->camrotc2w && pt->raydir, "camera (campos, camrotc2w, raydir) required");
    SGN_REQUIRE((pt->pers == nullptr) == (pt->samp_pers == nullptr), "pers and samp_pers go together");
    SGN_REQUIRE(S_capacity >= 0 && S_capacity < (1 << 30), "S_capacity out of range");
    const int64_t ws_items = (int64_t)(workspace_bytes / (HID * 4));
    SGN_REQUIRE(ws_items >= 1, "exact aggregate workspace too small (1 KiB per work item of a chunk)");
    hipStream_t st = as_stream(stream);
    if (S_capacity == 0 || pt->n_points == 0) return 0;  // no neighbours: no work item
    XArgs x{};
    AggArgs &a = x.a;
    a.xyz = pt->xyz; a.emb = pt->embedding; a.color = pt->color; a.dir = pt->dir; a.conf = pt->conf;
    a.campos = pt->campos; a.rot = pt->camrotc2w; a.raydir = pt->raydir;
    a.pers = pt->pers; a.samp_pers = pt->samp_pers;
    a.counters = q->counters; a.work = q->work; a.samp_ray = q->samp_ray; a.pidx = q->pidx;
    a.samp_locw = q->samp_locw;
    a.K = K;
    a.bpnet32 = d_bpnet;
    a.feat = d_out_feat; a.blend = d_out_blend; a.wnorm = d_out_wnorm;
    x.w = (const float *)d_packed_exact;
    x.lay = x_layout(bpnet_layers, bpnet_dim);
    x.fs = (float *)d_workspace;
    x.bpnet_dim = bpnet_dim;
    const int ntb = bpnet_layers ? (256 + bpnet_dim) / 16 : 0;
    if (d_out_blend) SGN_CHECK_HIP(hipMemsetAsync(d_out_blend, 0, (size_t)S_capacity * K * 4, st));
    if (d_out_wnorm) SGN_CHECK_HIP(hipMemsetAsync(d_out_wnorm, 0, (size_t)S_capacity * K * 4, st));
    const int64_t chunk = ws_items < S_capacity ? ws_items : S_capacity;
    for (int64_t i0 = 0; i0 < S_capacity; i0 += chunk) {
        a.item0 = (int32_t)i0;
        a.n_items = (int32_t)(S_capacity - i0 < chunk ? S_capacity - i0 : chunk);
        const int64_t tr = (a.n_items + 2 * NW - 1) / (2 * NW), tc = (a.n_items + 16 * NW - 1) / (16 * NW);
        const dim3 gr((unsigned)(tr < 2048 ? tr : 2048)), gc((unsigned)(tc < 1024 ? tc : 1024));
        if (pt->pers) {
            if (ntb == 0) hipLaunchKernelGGL((k_rows_exact<true, 0>), gr, dim3(TPB), 0, st, x);
            else if (ntb == 16) hipLaunchKernelGGL((k_rows_exact<true, 16>), gr, dim3(TPB), 0, st, x);
            else hipLaunchKernelGGL((k_rows_exact<true, 22>), gr, dim3(TPB), 0, st, x);
        } else {
            if (ntb == 0) hipLaunchKernelGGL((k_rows_exact<false, 0>), gr, dim3(TPB), 0, st, x);
            else if (ntb == 16) hipLaunchKernelGGL((k_rows_exact<false, 16>), gr, dim3(TPB), 0, st, x);
            else hipLaunchKernelGGL((k_rows_exact<false, 22>), gr, dim3(TPB), 0, st, x);
        }
        hipLaunchKernelGGL(k_color_exact, gc, dim3(TPB), 0, st, x);
    }
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

}  // extern "C"
