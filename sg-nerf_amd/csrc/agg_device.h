// agg_device.h -- device helpers shared by the aggregator kernels (mlp.hip: forward,
// agg_train.hip: training forward-save / backward).  Included inside sgn::{anonymous}.
//
// NeuralPoints gather + PointAggregator prologue (neural_points.py:942-988,
// point_aggregators.py:868-953), positional encodings (networks.py:175-192), MFMA and
// lane-exchange primitives for v_mfma_f32_32x32x16_f16 fragments (mlp_layout.h).
#pragma once
#include <utility>

#include "mlp_layout.h"
#include "sgn_common.h"

namespace sgn {
namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

using namespace mlp;

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// Weight blob access through a buffer descriptor: one VGPR of per-lane offset plus a
// compile-time SGPR/immediate offset per fragment (flat 64-bit addresses per fragment
// would be hoisted out of the sample loop and spill).
struct WBlob {
    __amdgpu_buffer_rsrc_t rsrc;
    __device__ __forceinline__ h8 frag(uint32_t byte_off, int lane) const {
        return __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(rsrc, lane * 16, byte_off, 0));
    }
    // 4 fp32 of an accumulator-order vector: element (t*2 + h)*16 + 4g of f32 section offset `f`
    __device__ __forceinline__ f32x4 acc4(uint32_t f, int t, int g, int h) const {
        return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                             rsrc, h * 64, (uint32_t)(OFF_F32 + (f + t * 32 + 4 * g) * 4), 0));
    }
    __device__ __forceinline__ float scalar(uint32_t f) const {
        return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, 0, (uint32_t)(OFF_F32 + f * 4), 0));
    }
};

__device__ __forceinline__ WBlob make_blob(const void *p, size_t bytes = TOTAL_BYTES) {
    WBlob b;
    b.rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
    return b;
}

__device__ __forceinline__ f32x16 mfma32(h8 a, h8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float lrelu(float x) { return x > 0.f ? x : x * 0.01f; }
__device__ __forceinline__ float softplus(float x) { return x > 20.f ? x : log1pf(expf(x)); }
struct Cam {
    float cx, cy, cz;
    float r[9];  // camrotc2w row-major
    // w2pers (neural_points.py:845-850): c_j = sum_i R[i][j] * (p_i - campos_i)
    __device__ __forceinline__ void pers(float x, float y, float z, float &px, float &py, float &pz) const {
        float sx = __fsub_rn(x, cx), sy = __fsub_rn(y, cy), sz = __fsub_rn(z, cz);
        float c0 = __fadd_rn(__fadd_rn(__fmul_rn(r[0], sx), __fmul_rn(r[3], sy)), __fmul_rn(r[6], sz));
        float c1 = __fadd_rn(__fadd_rn(__fmul_rn(r[1], sx), __fmul_rn(r[4], sy)), __fmul_rn(r[7], sz));
        float c2 = __fadd_rn(__fadd_rn(__fmul_rn(r[2], sx), __fmul_rn(r[5], sy)), __fmul_rn(r[8], sz));
        px = __fdiv_rn(c0, c2);
        py = __fdiv_rn(c1, c2);
        pz = c2;
    }
};

__device__ __forceinline__ Cam load_cam(const float *campos, const float *rot) {
    Cam c;
    c.cx = campos[0]; c.cy = campos[1]; c.cz = campos[2];
#pragma unroll
    for (int i = 0; i < 9; ++i) c.r[i] = rot[i];
    return c;
}


struct AggArgs {
    // point tables
    const float *xyz, *emb, *color, *dir, *conf;
    const float *campos, *rot, *raydir;
    const float *pers, *samp_pers;  // optional precomputed pers coordinates
    // query
    const int32_t *counters, *work, *samp_ray, *pidx;
    const float *samp_locw;
    // weights
    const void *blob;
    size_t blob_bytes;
    const _Float16 *bpnet;  // [N, bpnet_dim] fp16 (SG variant with predict_semantic = 1), else null
    const float *bpnet32;   // [N, bpnet_dim] fp32 (the same table for the fp32-faithful kernels)
    // outputs
    float *feat;      // float4 per sample id: .x alpha written here
    float *blend;     // [S*8] weight * conf (optional)
    float *wnorm;     // [S*8] normalised weight (optional)
    _Float16 *fs;     // [chunk][256] blended features (natural unit order)
    const _Float16 *proj;  // split block1.0: P[point][2][128] = W0a [feat | PE(feat)] + b0, acc order
    int32_t item0, n_items;  // work-list chunk
    // training forward (save mode): per-row layer inputs, row = 8 * (item - item0) + k,
    // fp16 in fragment column order (mlp_layout.h: column 16 s + 8 h + e of k-step s)
    _Float16 *sx0;    // [rows][288] block1.0 inputs (layer-0 channel order)
    _Float16 *sh1;    // [rows][256] block1.2 inputs (chain order)
    _Float16 *sh2;    // [rows][272] block3.0 inputs (chain order | colour, dir - v, <dir, v>)
    _Float16 *sh3;    // [rows][256] block3.2 inputs (chain order)
    _Float16 *sh2b;   // [rows][256] block2_bpnet inputs h (chain order; SG save mode, where sh2 then
                      // holds block3.0's inputs [block2_bpnet output | colour, dir - v, <dir, v>])
    // packed point records of the fp32 16x16 kernels (k_point_proj16 writes them beside P):
    // 64 B per point = {x, y, z, conf}, {r, g, b, 0}, {dx, dy, dz, 0}, {0}; one cache line per row
    const float *rec;
    // paired sample slots of k_rows16 (k_pair_slots): per 8-row half the row table
    // rows[8 slot + kk] = s * 8 + k (-1: idle row) and the entry {A item | nA << 28,
    // B item | nB << 28, A sample, B sample} (items relative to item0); slot_n[0] = slots
    const int32_t *rows;
    const int4 *slots;
    const int32_t *slot_n;
    // fp32-faithful training forward (k_rows16 save mode): the pre-activations 2^-s acc of block1.0,
    // block1.2 and block3.0 (the inputs of the next layer before LeakyReLU), fp32 natural unit order,
    // row s * 8 + k (the row's pidx index); rows without a neighbour are not written.  SG: zb is
    // block2_bpnet.0's (block3.0's input), z2 stays block1.2's
    float *z1, *z2, *z3, *zb;
    // with row_off (sgn_train_lists): the rows are compact instead, row_off[s] + k
    const int32_t *row_off;
    // neighbours per sample of the query's pidx (1..8): a sample's row k < K reads pidx index s * K + k,
    // rows k >= K are empty (fp32 kernels: a row-table entry s * 8 + k names pidx index s * K + k)
    int32_t K;
};

// training save: one 16-byte fragment of a 32-row tile -> [rows][C] (C multiple of 16)
__device__ __forceinline__ void save_frag(_Float16 *base, int C, int64_t row0, int s, h8 v, int lane, bool ok) {
    if (ok) *(h8 *)(base + (row0 + (lane & 31)) * C + s * 16 + (lane >> 5) * 8) = v;
}

template <class F, int... I>
__device__ __forceinline__ void static_for_impl(F &&f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F &&f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// DPP butterflies: lanes j^1, j^2 (quad_perm), then the mirrored quad of the 8-lane half-row
__device__ __forceinline__ float dpp_sum8(float x) {
    x += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0xB1, 0xF, 0xF, true));
    x += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0x4E, 0xF, 0xF, true));
    x += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0x141, 0xF, 0xF, true));
    return x;
}

__device__ __forceinline__ h8 pack8(float a0, float a1, float a2, float a3, float a4, float a5, float a6,
                                    float a7) {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    const h2 p0 = {(_Float16)a0, (_Float16)a1}, p1 = {(_Float16)a2, (_Float16)a3};
    const h2 p2 = {(_Float16)a4, (_Float16)a5}, p3 = {(_Float16)a6, (_Float16)a7};
    const u32x4 u = {__builtin_bit_cast(uint32_t, p0), __builtin_bit_cast(uint32_t, p1),
                     __builtin_bit_cast(uint32_t, p2), __builtin_bit_cast(uint32_t, p3)};
    return __builtin_bit_cast(h8, u);
}

// sin/cos for the positional encodings: hardware v_sin/v_cos on the argument reduced to
// [-0.5, 0.5] revolutions (abs error ~1e-6, far below the fp16 rounding of the result)
__device__ __forceinline__ float pe_sin(float x) {
    float r = x * 0.15915494309189535f;
    r = r - rintf(r);
    return __builtin_amdgcn_sinf(r);
}
__device__ __forceinline__ float pe_cos(float x) {
    float r = x * 0.15915494309189535f;
    r = r - rintf(r);
    return __builtin_amdgcn_cosf(r);
}

// sin/cos of x * 2^F from one hardware sin/cos of x and F double-angle steps
// (sin 2a = 2 sin a cos a, cos 2a = (cos a - sin a)(cos a + sin a)); identical
// sub-expressions of the channels of one k-step are CSE'd by the compiler.
template <int F>
__device__ __forceinline__ void sincos_pow2(float x, float &s, float &c) {
    if constexpr (F == 0) {
        s = pe_sin(x);
        c = pe_cos(x);
    } else {
        float s0, c0;
        sincos_pow2<F - 1>(x, s0, c0);
        s = 2.f * s0 * c0;
        c = (c0 - s0) * (c0 + s0);
    }
}

// value of layer-0 channel C (0..143) of a lane-half (mlp_layout.h order)
template <int C>
__device__ __forceinline__ float l0_channel(const float (&feat)[16], const float (&dist)[3]) {
    if constexpr (C < 16) {
        return feat[C];
    } else if constexpr (C < 112) {
        constexpr int m = C - 16, d = m / 6, f = (m % 6) / 2, sc = m % 2;
        float sv, cv;
        sincos_pow2<f>(feat[d], sv, cv);
        return sc ? cv : sv;
    } else if constexpr (C < 142) {
        constexpr int m = C - 112, dd = m / 10, f = (m % 10) / 2, sc = m % 2;
        float sv, cv;
        sincos_pow2<f>(dist[dd], sv, cv);
        return sc ? cv : sv;
    } else {
        return 0.f;
    }
}

template <int K0>
__device__ __forceinline__ h8 l0_step(const float (&feat)[16], const float (&dist)[3]) {
    return pack8(l0_channel<8 * K0 + 0>(feat, dist), l0_channel<8 * K0 + 1>(feat, dist),
                 l0_channel<8 * K0 + 2>(feat, dist), l0_channel<8 * K0 + 3>(feat, dist),
                 l0_channel<8 * K0 + 4>(feat, dist), l0_channel<8 * K0 + 5>(feat, dist),
                 l0_channel<8 * K0 + 6>(feat, dist), l0_channel<8 * K0 + 7>(feat, dist));
}


// v_permlane{16,32}_swap as inline asm: this compiler's lowering of the two-result
// builtins returns the first result twice (seen in the ISA: v_add v48, v48, v48 after the
// swap).  x, y are swapped in place: permlane32: x.hi <-> y.lo; permlane16: odd rows of x
// <-> even rows of y.  The s_nops cover the VALU-write -> permlane-read hazard.
__device__ __forceinline__ void permlane32_swap(float &x, float &y) {
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\ts_nop 1" : "+v"(x), "+v"(y));
}
__device__ __forceinline__ void permlane16_swap(float &x, float &y) {
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\ts_nop 1" : "+v"(x), "+v"(y));
}

// LeakyReLU(0.01) = 0.505 x + 0.495 |x|: one v_mul with an |x| source modifier + one v_fma
// (no compare/select, no NaN canonicalisation); within 1 ulp of max(x, 0.01x)
__device__ __forceinline__ float lrelu_max(float x) { return __builtin_fmaf(0.505f, x, 0.495f * __builtin_fabsf(x)); }


// fp16 pack + LeakyReLU on the packed halves: v_cvt_pk_f16_f32, v_pk_mul_f16, v_pk_max_f16
// (1.5 instructions per value; lrelu(fp16(x)) differs from fp16(lrelu(x)) only by the
// rounding of 0.01x on negative inputs)
__device__ __forceinline__ uint32_t lrelu_pk(float x0, float x1) {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    const h2 v = {(_Float16)x0, (_Float16)x1};
    const h2 sl = v * h2{(_Float16)0.01f, (_Float16)0.01f};
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(v, sl));
}


template <bool C, class T>
__device__ __forceinline__ T &pick(T &a, T &b) {
    if constexpr (C) return a; else return b;
}

struct RowIn {
    int s;       // sample id
    bool sval;   // work item exists
    float wgt;   // normalised weight * conf of this row
    int pid;     // neighbour point index (-1: masked)
    float wn;    // normalised inverse-distance weight (before the conf factor)
};

// Gather + pers + dists + weights of this lane's row; raw features for the
// just-in-time layer-0 encodings, block3's extra channels.
// Index chain of a row (work item -> sample -> neighbour point, sample -> ray); k_agg_rows
// loads it one work tile ahead so the record gather below starts from resident indices.
struct RowIdx {
    int s, pid, ray;
    bool sval;
    bool a = true;  // k_rows16: the row belongs to its half's sample A (rows 0..nA-1)
};

__device__ __forceinline__ RowIdx row_index(const AggArgs &a, int item, int end, int lane) {
    RowIdx x;
    x.sval = item < end;
    x.s = x.sval ? a.work[item] : 0;
    x.pid = x.sval && (lane & 7) < a.K ? a.pidx[(int64_t)x.s * a.K + (lane & 7)] : -1;
    x.ray = x.sval ? a.samp_ray[x.s] : 0;  // no sample id to follow without a work item
    return x;
}

// FEAT = false: the point features are not needed (split block1.0).  Block3's extra channels
// (colour, dir - v, <dir, v>, 0; lane-half 0 only, zero on half 1) go to `ext` as fp16 or, with
// F32EXT, to `extf` in fp32 (the fp32-faithful kernels split them themselves).
template <bool FEAT, bool F32EXT>
__device__ __forceinline__ RowIn gather_row_impl(const AggArgs &a, const Cam &cam, const RowIdx &ix, int lane,
                                                 float (&feat)[16], float (&dist)[3], h8 &ext, float (&extf)[8]) {
    const int h = lane >> 5, kk = lane & 7;
    RowIn ri;
    ri.sval = ix.sval;
    ri.s = ix.s;
    const int s = ri.s;
    const int pid = ix.pid;
    const bool m = pid >= 0;
    ri.pid = pid;
    const float lx = a.samp_locw[(int64_t)s * 3 + 0], ly = a.samp_locw[(int64_t)s * 3 + 1],
                lz = a.samp_locw[(int64_t)s * 3 + 2];
    const int ray = ix.ray;
    const float vx = a.raydir[(int64_t)ray * 3 + 0], vy = a.raydir[(int64_t)ray * 3 + 1],
                vz = a.raydir[(int64_t)ray * 3 + 2];
    float px = 0.f, py = 0.f, pz = 0.f, cf = 0.f;
    float col[3] = {0.f, 0.f, 0.f}, pdr[3] = {0.f, 0.f, 0.f};
    if (m) {
        px = a.xyz[(int64_t)pid * 3 + 0]; py = a.xyz[(int64_t)pid * 3 + 1]; pz = a.xyz[(int64_t)pid * 3 + 2];
        if constexpr (FEAT) {
            const f32x4 *e4 = (const f32x4 *)(a.emb + (int64_t)pid * 32 + 16 * h);
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                f32x4 v = e4[g];
                feat[4 * g + 0] = v[0]; feat[4 * g + 1] = v[1]; feat[4 * g + 2] = v[2]; feat[4 * g + 3] = v[3];
            }
        } else {
#pragma unroll
            for (int c = 0; c < 16; ++c) feat[c] = 0.f;
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) { col[c] = a.color[(int64_t)pid * 3 + c]; pdr[c] = a.dir[(int64_t)pid * 3 + c]; }
        cf = a.conf[pid];
    } else {
#pragma unroll
        for (int c = 0; c < 16; ++c) feat[c] = 0.f;
    }
    // dists (point_aggregators.py:917-925): half 0 world offsets, half 1 pers-space terms
    const float dwx = __fsub_rn(px, lx), dwy = __fsub_rn(py, ly), dwz = __fsub_rn(pz, lz);
    dist[0] = m ? dwx : 0.f; dist[1] = m ? dwy : 0.f; dist[2] = m ? dwz : 0.f;
    if (h == 1) {
        float xp = 0.f, yp = 0.f, zp = 0.f, xl, yl, zl;
        if (a.pers) {
            if (m) { xp = a.pers[(int64_t)pid * 3]; yp = a.pers[(int64_t)pid * 3 + 1]; zp = a.pers[(int64_t)pid * 3 + 2]; }
            xl = a.samp_pers[(int64_t)s * 3]; yl = a.samp_pers[(int64_t)s * 3 + 1]; zl = a.samp_pers[(int64_t)s * 3 + 2];
        } else {
            if (m) cam.pers(px, py, pz, xp, yp, zp);
            cam.pers(lx, ly, lz, xl, yl, zl);
        }
        dist[0] = m ? __fsub_rn(__fmul_rn(xp, zp), __fmul_rn(xl, zl)) : 0.f;
        dist[1] = m ? __fsub_rn(__fmul_rn(yp, zp), __fmul_rn(yl, zl)) : 0.f;
        dist[2] = m ? __fsub_rn(zp, zl) : 0.f;
    }
    // linear kernel weights, normalised over the sample's 8 rows, times clamped conf
    float w = 0.f;
    if (m) {
        float n2 = __fadd_rn(__fadd_rn(__fmul_rn(dwx, dwx), __fmul_rn(dwy, dwy)), __fmul_rn(dwz, dwz));
        w = 1.f / fmaxf(sqrtf(n2), 1e-6f);
    }
    const float wsum = dpp_sum8(w);
    w = w / fmaxf(wsum, 1e-8f);
    ri.wn = w;
    ri.wgt = w * fminf(fmaxf(cf, 1e-4f), 1.f);
    if (a.blend && ri.sval && h == 0 && kk < a.K) a.blend[(int64_t)s * a.K + kk] = ri.wgt;
    if (a.wnorm && ri.sval && h == 1 && kk < a.K) a.wnorm[(int64_t)s * a.K + kk] = w;
    // block3 extra channels: colour, dir - v, <dir, v> (:639-652), lane-half 0 only
    if constexpr (F32EXT) {
        const bool e = h == 0 && m;
        extf[0] = e ? col[0] : 0.f;
        extf[1] = e ? col[1] : 0.f;
        extf[2] = e ? col[2] : 0.f;
        extf[3] = e ? __fsub_rn(pdr[0], vx) : 0.f;
        extf[4] = e ? __fsub_rn(pdr[1], vy) : 0.f;
        extf[5] = e ? __fsub_rn(pdr[2], vz) : 0.f;
        extf[6] = e ? __fadd_rn(__fadd_rn(__fmul_rn(pdr[0], vx), __fmul_rn(pdr[1], vy)), __fmul_rn(pdr[2], vz)) : 0.f;
        extf[7] = 0.f;
    } else {
        h8 e = {};
        if (h == 0 && m) {
            e = pack8(col[0], col[1], col[2], __fsub_rn(pdr[0], vx), __fsub_rn(pdr[1], vy), __fsub_rn(pdr[2], vz),
                      __fadd_rn(__fadd_rn(__fmul_rn(pdr[0], vx), __fmul_rn(pdr[1], vy)), __fmul_rn(pdr[2], vz)), 0.f);
        }
        ext = e;
    }
    return ri;
}

template <bool FEAT = true>
__device__ __forceinline__ RowIn gather_row(const AggArgs &a, const Cam &cam, const RowIdx &ix, int lane,
                                            float (&feat)[16], float (&dist)[3], h8 &ext) {
    float unused[8];
    return gather_row_impl<FEAT, false>(a, cam, ix, lane, feat, dist, ext, unused);
}

template <bool FEAT = true>
__device__ __forceinline__ RowIn gather_row_f(const AggArgs &a, const Cam &cam, const RowIdx &ix, int lane,
                                              float (&feat)[16], float (&dist)[3], float (&extf)[8]) {
    h8 unused;
    return gather_row_impl<FEAT, true>(a, cam, ix, lane, feat, dist, unused, extf);
}

template <bool FEAT = true>
__device__ __forceinline__ RowIn gather_row(const AggArgs &a, const Cam &cam, int item, int end, int lane,
                                            float (&feat)[16], float (&dist)[3], h8 &ext) {
    return gather_row<FEAT>(a, cam, row_index(a, item, end, lane), lane, feat, dist, ext);
}


}  // namespace
}  // namespace sgn
