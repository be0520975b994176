// loss.hip -- the training step's per-ray loss stage, forward and backward, on the device:
// ray_dist + ray_march + fill_invalid (as composite.hip), the masked colour MSE and the zero-one
// loss on the neighbours' confidence, and their gradients w.r.t. the per-sample features
// (alpha, r, g, b) and the points' conf.  Replaces the torch autograd of:
//   ray_dist          neural_points_volumetric_model.py:569-577
//   ray_march         diff_ray_marching.py:509-555 (alpha_blend, radiance_render,
//                     diff_render_func.py:36-49)
//   losses            base_rendering_model.py:534-664 (ray_masked_coarse_raycolor: MSE over the
//                     valid rays; ray_miss_coarse_raycolor / coarse_raycolor weight 0, logged),
//                     mvs_points_volumetric_model.py:607-614 (zero_one_loss on conf_coefficient over
//                     the dense [R'', SR, K] neighbour tensor of point_aggregators.py:951-958, empty
//                     entries reading conf at the clamped index 0, neural_points.py:956-967)
// Three launches, no host synchronisation (graph-capturable):
//   k_loss_fwd     8 lanes per ray: composite, per-slot (T, e, dist) kept in the workspace,
//                  block partial sums of the loss terms (fixed order)
//   k_loss_reduce  one workgroup: the partials in block order -> the four losses and the
//                  gradient scales (the valid-ray count is only known here)
//   k_loss_bwd     8 lanes per ray: reverse pass over the slots -> d feat per sample;
//                  zero-one gradients added into d conf (atomics; a ray's empty entries as one add)
#include "sgn_common.h"

namespace sgn {
namespace {

constexpr int LOSS_TPB = 256;
constexpr int LPR = 8;  // lanes per ray: the slot walk runs on all 8 (same values), the SR x K zero-one
                        // entries are split over them by neighbour k
constexpr int LOSS_NSUM = 5;  // masked se, missed se, all se, zero-one sum, valid rays

struct LossArgs {
    const float *campos, *rot;
    const int32_t *ray_ns, *ray_soff, *samp_nnb, *pidx;
    const float *samp_locw, *feat, *gt, *conf;
    int64_t R;
    int SR, K, unit;
    float vz, bg0, bg1, bg2, zo_w, zo_eps;
    const float *bg_ray;  // [R][3] per-ray background (ABI 16, inputs['bg_ray']) or null: (bg0, bg1, bg2)
    float *slot_ws;   // [R][SR][3]: T (transmittance before the slot), e = exp(-sigma dist), dist
    float *partial;   // [blocks][LOSS_NSUM]
    float *sums;      // [8]: l_col, l_zo, l_miss, l_all, 2 / max(3 n, 1), zo_w / max(n SR K, 1), n
    float *out_rgb;   // [R][3]
    int8_t *out_mask; // [R]
    float *dfeat;     // [S][4]
    float *dconf;     // [N]
};

// the ray's background colour: inputs['bg_ray'] when given (fill_invalid blends T_bg * bg_ray,
// neural_points_volumetric_model.py:175-177), else the constant bg
__device__ __forceinline__ void ray_bg(const LossArgs &a, int64_t r, float (&bg)[3]) {
    if (a.bg_ray) {
        bg[0] = a.bg_ray[r * 3]; bg[1] = a.bg_ray[r * 3 + 1]; bg[2] = a.bg_ray[r * 3 + 2];
    } else {
        bg[0] = a.bg0; bg[1] = a.bg1; bg[2] = a.bg2;
    }
}

__device__ __forceinline__ float pers_z(const float *campos, const float *rot, float x, float y, float z) {
    const float sx = __fsub_rn(x, campos[0]), sy = __fsub_rn(y, campos[1]), sz = __fsub_rn(z, campos[2]);
    return __fadd_rn(__fadd_rn(__fmul_rn(sx, rot[2]), __fmul_rn(sy, rot[5])), __fmul_rn(sz, rot[8]));
}

// zero-one term of one (slot, k) entry and its derivative w.r.t. the gathered conf (the straight-
// through clamp passes the gradient unchanged, point_aggregators.py:863-865)
__device__ __forceinline__ void zero_one(float cd, float eps, float &term, float &dterm) {
    const float cl = fminf(fmaxf(cd, 1e-4f), 1.f);
    const float cc = __fsub_rn(cd, __fsub_rn(cd, cl));
    const float val = fminf(fmaxf(cc, eps), 1.f - eps);
    term = logf(val) + logf(1.f - val);
    dterm = (cc >= eps && cc <= 1.f - eps) ? 1.f / val - 1.f / (1.f - val) : 0.f;
}

// Per ray forward: slot s of the ray (s < ns: sample soff + s; later slots are padding at the
// origin's depth) closes slot s - 1's interval (running cummax of pers z).
template <bool STORE>
__device__ void ray_forward(const LossArgs &a, int64_t r, bool store, float (&col)[3], float &T, bool &any_valid) {
    const int ns = a.ray_ns[r], off = a.ray_soff[r], SR = a.SR;
    const float z0 = pers_z(a.campos, a.rot, 0.f, 0.f, 0.f);
    float *ws = a.slot_ws + r * (int64_t)SR * 3;
    T = 1.f;
    col[0] = col[1] = col[2] = 0.f;
    any_valid = false;
    float prev_cm = 0.f;
    bool pv = false;
    float4 pf = make_float4(0.f, 0.f, 0.f, 0.f);
    auto process = [&](int slot, float dist) {
        const bool mask = dist < 1e-8f || (a.unit && dist > 2.f * a.vz);
        dist = mask ? a.vz : dist;
        const float valid = pv ? 1.f : 0.f;
        dist = dist * valid;
        const float sigma = pf.x * valid;
        const float e = expf(-sigma * dist);
        const float o = 1.f - e;
        const float wgt = o * T;
        col[0] += pf.y * wgt;
        col[1] += pf.z * wgt;
        col[2] += pf.w * wgt;
        if (STORE && store) {
            ws[3 * slot + 0] = T;
            ws[3 * slot + 1] = e;
            ws[3 * slot + 2] = dist;
        }
        T = T * (1.f - o + 1e-10f);
    };
    const int last = ns < SR ? ns : SR - 1;
    for (int s = 0; s <= last; ++s) {
        float z = z0;
        bool v = false;
        float4 f = make_float4(0.f, 0.f, 0.f, 0.f);
        if (s < ns) {
            const int64_t id = off + s;
            z = pers_z(a.campos, a.rot, a.samp_locw[id * 3], a.samp_locw[id * 3 + 1], a.samp_locw[id * 3 + 2]);
            v = a.samp_nnb[id] > 0;
            f = *(const float4 *)(a.feat + id * 4);  // zero features for samples without neighbours
        }
        const float cm = s == 0 ? z : fmaxf(prev_cm, z);
        if (s > 0) process(s - 1, cm - prev_cm);
        prev_cm = cm;
        pv = v;
        pf = f;
        any_valid |= v;
    }
    if (ns >= SR) process(SR - 1, a.vz);
}

__device__ __forceinline__ float block_sum(float v, float *red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    float t = 0.f;
    for (int i = 0; i < LOSS_TPB / 64; ++i) t += red[i];  // fixed order
    return t;
}

__global__ __launch_bounds__(LOSS_TPB) void k_loss_fwd(LossArgs a) {
    __shared__ float red[LOSS_TPB / 64];
    const int64_t r = ((int64_t)blockIdx.x * LOSS_TPB + threadIdx.x) / LPR;
    const int sub = threadIdx.x % LPR;
    float v[LOSS_NSUM] = {0.f, 0.f, 0.f, 0.f, 0.f};
    if (r < a.R) {
        float col[3], T;
        bool any;
        ray_forward<true>(a, r, sub == 0, col, T, any);
        float bg[3];
        ray_bg(a, r, bg);
        float se = 0.f;
        for (int c = 0; c < 3; ++c) {
            const float full = any ? col[c] + bg[c] * T : bg[c];
            if (sub == 0) a.out_rgb[r * 3 + c] = full;
            const float d = full - a.gt[r * 3 + c];
            se += d * d;
        }
        if (sub == 0) {
            a.out_mask[r] = any ? 1 : 0;
            v[0] = any ? se : 0.f;
            v[1] = any ? 0.f : se;
            v[2] = se;
            v[4] = any ? 1.f : 0.f;
        }
        if (any) {  // zero-one terms over the ray's SR x K entries, neighbour k = sub, sub + 8, ..
            const int ns = a.ray_ns[r], off = a.ray_soff[r];
            const int nv = ns < a.SR ? ns : a.SR;
            float t0, d0;
            zero_one(a.conf[0], a.zo_eps, t0, d0);
            float zs = 0.f;
            int n_empty = 0;
            for (int k = sub; k < a.K; k += LPR) {
                n_empty += a.SR - nv;
                for (int s2 = 0; s2 < nv; ++s2) {
                    const int p = a.pidx[(int64_t)(off + s2) * a.K + k];
                    if (p < 0) {
                        ++n_empty;
                        continue;
                    }
                    float t, d;
                    zero_one(a.conf[p], a.zo_eps, t, d);
                    zs += t;
                }
            }
            v[3] = zs + (float)n_empty * t0;
        }
    }
    for (int i = 0; i < LOSS_NSUM; ++i) {
        const float t = block_sum(v[i], red);
        if (threadIdx.x == 0) a.partial[(int64_t)blockIdx.x * LOSS_NSUM + i] = t;
    }
}

__global__ __launch_bounds__(LOSS_TPB) void k_loss_reduce(LossArgs a, int nblocks) {
    __shared__ float red[LOSS_TPB / 64];
    float t[LOSS_NSUM];
    for (int i = 0; i < LOSS_NSUM; ++i) {
        float v = 0.f;
        for (int b = threadIdx.x; b < nblocks; b += LOSS_TPB) v += a.partial[(int64_t)b * LOSS_NSUM + i];
        t[i] = block_sum(v, red);
    }
    if (threadIdx.x == 0) {
        const float n = t[4];
        const float den_c = fmaxf(3.f * n, 1.f), den_z = fmaxf(n * (float)(a.SR * a.K), 1.f);
        a.sums[0] = t[0] / den_c;
        a.sums[1] = t[3] / den_z;
        a.sums[2] = t[1] / 3.f;
        a.sums[3] = t[2] / (3.f * (float)a.R);
        a.sums[4] = 2.f / den_c;
        a.sums[5] = a.zo_w / den_z;
        a.sums[6] = n;
        a.sums[7] = 0.f;
    }
}

__global__ __launch_bounds__(LOSS_TPB) void k_loss_bwd(LossArgs a) {
    const int64_t r = ((int64_t)blockIdx.x * LOSS_TPB + threadIdx.x) / LPR;
    const int sub = threadIdx.x % LPR;
    if (r >= a.R) return;
    const int ns = a.ray_ns[r], off = a.ray_soff[r], SR = a.SR;
    const int nv = ns < SR ? ns : SR;
    if (!a.out_mask[r]) {  // fill_invalid: the background colour carries no gradient
        for (int s = sub; s < nv; s += LPR)
            *(float4 *)(a.dfeat + (int64_t)(off + s) * 4) = make_float4(0.f, 0.f, 0.f, 0.f);
        return;
    }
    if (sub == 0) {  // reverse pass over the slots (one lane of the ray)
        const float gs = a.sums[4];
        float g[3];
        for (int c = 0; c < 3; ++c) g[c] = gs * (a.out_rgb[r * 3 + c] - a.gt[r * 3 + c]);
        const float *ws = a.slot_ws + r * (int64_t)SR * 3;
        // T after every slot (the padding slots' factors are exactly 1): from the last slot
        float Tend = 1.f;
        if (nv > 0) {
            const float Tl = ws[3 * (nv - 1)], el = ws[3 * (nv - 1) + 1];
            Tend = Tl * (1.f - (1.f - el) + 1e-10f);
        }
        // U = sum over later slots of g . c_i o_i T_i + g . bg T_end (d L / d a_s times a_s), from the end
        float bg[3];
        ray_bg(a, r, bg);
        float U = (g[0] * bg[0] + g[1] * bg[1] + g[2] * bg[2]) * Tend;
        for (int s = nv - 1; s >= 0; --s) {
            const int64_t id = off + s;
            const float T = ws[3 * s], e = ws[3 * s + 1], dist = ws[3 * s + 2];
            const float4 f = *(const float4 *)(a.feat + id * 4);
            const float o = 1.f - e;
            const float gc = g[0] * f.y + g[1] * f.z + g[2] * f.w;
            const float av = 1.f - o + 1e-10f;
            const float dO = gc * T - U / av;               // d L / d o_s
            const bool v = a.samp_nnb[id] > 0;
            const float dsig = dO * e * dist;              // o = 1 - exp(-sigma dist)
            const float w = o * T;
            *(float4 *)(a.dfeat + id * 4) = make_float4(v ? dsig : 0.f, g[0] * w, g[1] * w, g[2] * w);
            U += gc * w;
        }
    }
    // zero-one gradients, neighbour k = sub, sub + 8, ..; the empty entries all read conf[0]
    const float gz = a.sums[5];
    float t0, d0;
    zero_one(a.conf[0], a.zo_eps, t0, d0);
    int n_empty = 0;
    for (int k = sub; k < a.K; k += LPR) {
        n_empty += SR - nv;
        for (int s = 0; s < nv; ++s) {
            const int p = a.pidx[(int64_t)(off + s) * a.K + k];
            if (p < 0) {
                ++n_empty;
                continue;
            }
            float t, d;
            zero_one(a.conf[p], a.zo_eps, t, d);
            if (d != 0.f) atomicAdd(a.dconf + p, gz * d);
        }
    }
    if (n_empty > 0 && d0 != 0.f) atomicAdd(a.dconf, gz * d0 * (float)n_empty);
}

}  // namespace
}  // namespace sgn

extern "C" {

size_t sgn_loss_workspace_bytes(int64_t R, int32_t SR) {
    if (R < 0 || SR <= 0) return 0;
    const int64_t nb = (R * sgn::LPR + sgn::LOSS_TPB - 1) / sgn::LOSS_TPB;
    return (size_t)(R * SR * 3 * 4 + (nb + 1) * sgn::LOSS_NSUM * 4 + 64);
}

int sgn_loss_train(const sgn_loss_params *lp, const float *d_campos, const float *d_camrotc2w, int64_t R,
                   const sgn_query_out *q, const float *d_feat, const float *d_gt, const float *d_conf,
                   float *d_out_rgb, int8_t *d_out_mask, float *d_losses, float *d_dfeat, float *d_dconf,
                   void *d_workspace, size_t workspace_bytes, sgn_stream_t stream) {
    using namespace sgn;
    SGN_REQUIRE(lp && q && d_campos && d_camrotc2w && d_feat && d_gt && d_conf && d_out_rgb && d_out_mask &&
                    d_losses && d_dfeat && d_dconf && d_workspace,
                "null argument");
    SGN_REQUIRE(lp->SR > 0 && lp->K > 0, "SR and K must be positive");
    SGN_REQUIRE(R >= 0, "R must be non-negative");
    SGN_REQUIRE(workspace_bytes >= sgn_loss_workspace_bytes(R, lp->SR), "loss workspace too small");
    SGN_REQUIRE(((uintptr_t)d_feat & 15) == 0 && ((uintptr_t)d_dfeat & 15) == 0 && ((uintptr_t)d_workspace & 15) == 0,
                "16-byte alignment required");
    hipStream_t st = as_stream(stream);
    const int64_t nb = (R * LPR + LOSS_TPB - 1) / LOSS_TPB;
    LossArgs a{};
    a.campos = d_campos; a.rot = d_camrotc2w;
    a.ray_ns = q->ray_ns; a.ray_soff = q->ray_soff; a.samp_nnb = q->samp_nnb; a.pidx = q->pidx;
    a.samp_locw = q->samp_locw; a.feat = d_feat; a.gt = d_gt; a.conf = d_conf;
    a.R = R; a.SR = lp->SR; a.K = lp->K; a.unit = lp->raydist_mode_unit; a.vz = lp->vsize_z;
    a.bg0 = lp->bg[0]; a.bg1 = lp->bg[1]; a.bg2 = lp->bg[2];
    a.bg_ray = lp->bg_ray;
    a.zo_w = lp->zero_one_weight; a.zo_eps = lp->zero_one_eps;
    a.slot_ws = (float *)d_workspace;
    a.partial = a.slot_ws + R * lp->SR * 3;
    a.sums = d_losses;
    a.out_rgb = d_out_rgb; a.out_mask = d_out_mask; a.dfeat = d_dfeat; a.dconf = d_dconf;
    if (R == 0) {
        SGN_CHECK_HIP(hipMemsetAsync(d_losses, 0, 8 * sizeof(float), st));
        return 0;
    }
    hipLaunchKernelGGL(k_loss_fwd, dim3((unsigned)nb), dim3(LOSS_TPB), 0, st, a);
    hipLaunchKernelGGL(k_loss_reduce, dim3(1), dim3(LOSS_TPB), 0, st, a, (int)nb);
    hipLaunchKernelGGL(k_loss_bwd, dim3((unsigned)nb), dim3(LOSS_TPB), 0, st, a);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

}  // extern "C"
