// composite.hip -- per-ray ray_dist + front-to-back alpha composite + background fill.
//
// Replaces, for one ray r (sample slots 0..SR-1, selected samples first, then the
// zero-position padding slots of sample_loc_tensor, worldcoords.py:835):
//   ray_dist        neural_points_volumetric_model.py:569-577 (cummax of pers z, last
//                   interval vsize[2], raydist_mode_unit replacement, * ray_valid)
//   ray_march       diff_ray_marching.py:509-555 with alpha_blend / radiance_render
//                   (diff_render_func.py:36-49): o = 1 - exp(-sigma*dist),
//                   T = exclusive cumprod(1 - o + 1e-10), rgb = sum o*T*c + bg*T_last
//   fill_invalid    neural_points_volumetric_model.py:158-195 (rays without a valid
//                   sample get bg, coarse_is_background 1, ray_mask 0)
// One thread per ray, single pass over the slots (running cummax, running T).
#include "sgn_common.h"

namespace sgn {
namespace {

struct CompArgs {
    const float *campos, *rot, *raydir;
    const int32_t *ray_ns, *ray_soff, *samp_nnb;
    const float *samp_locw, *feat;
    int64_t R;
    int SR, unit;
    float vz, bg0, bg1, bg2;
    float *out_rgb, *out_bgT, *out_opacity, *out_blendw;
    int8_t *out_mask;
};

__device__ __forceinline__ float pers_z(const float *campos, const float *rot, float x, float y, float z) {
    float sx = __fsub_rn(x, campos[0]), sy = __fsub_rn(y, campos[1]), sz = __fsub_rn(z, campos[2]);
    return __fadd_rn(__fadd_rn(__fmul_rn(sx, rot[2]), __fmul_rn(sy, rot[5])), __fmul_rn(sz, rot[8]));
}

// One wave = 64 rays (lane = ray).  A ray's loop stops after its last selected sample: every
// later slot is a padding slot (sigma 0), whose opacity is exactly 0 and whose transmittance
// factor 1 - 0 + 1e-10 rounds to 1.0f, so skipping them changes no bit.  The [R, SR] opacity /
// blend-weight rows go out in column chunks of COMP_CW slots: the wave walks the chunks in step
// (each lane's ray state -- T, colour, running cummax, the previous slot -- stays in registers),
// stages a chunk's [64][COMP_CW] values in LDS (zero-filled, so padding slots cost nothing) and
// stores it as coalesced 16-B writes.  The LDS per workgroup (16.9 KiB) does not grow with SR, so
// a CU holds 9 such waves at any SR (a whole-row [64][SR + 1] staging took 66 KiB at SR 128).
constexpr int COMP_RAYS = 64, COMP_CW = 32, COMP_LD = COMP_CW + 1;
// one wave per workgroup: the chunk loop's barriers stage the wave's own rows only
static_assert(COMP_RAYS == 64, "k_composite: one wave64 per workgroup");

// chunk [c0, c0 + cw) of the wave's 64 x SR block (row stride SR) from st [64][COMP_LD]
__device__ __forceinline__ void store_chunk(float *dst, const float *st, int SR, int c0, int cw, int nrows,
                                            int lane) {
    if ((SR & 3) == 0 && cw == COMP_CW) {  // 16-B stores: 8 lanes per row chunk (128 B)
        for (int i = lane; i < nrows * (COMP_CW / 4); i += 64) {
            const int row = i >> 3, q = (i & 7) * 4;
            const float *p = st + row * COMP_LD + q;
            *(float4 *)(dst + (int64_t)row * SR + c0 + q) = make_float4(p[0], p[1], p[2], p[3]);
        }
    } else {
        for (int i = lane; i < nrows * cw; i += 64) {
            const int row = i / cw, col = i - row * cw;
            dst[(int64_t)row * SR + c0 + col] = st[row * COMP_LD + col];
        }
    }
}

__global__ __launch_bounds__(COMP_RAYS) void k_composite(CompArgs a) {
    __shared__ float st[2][COMP_RAYS * COMP_LD];  // chunk staging: opacity, blend weight
    const int lane = threadIdx.x;
    const int64_t r0 = (int64_t)blockIdx.x * COMP_RAYS, r = r0 + lane;
    const int nrows = a.R - r0 < COMP_RAYS ? (int)(a.R - r0) : COMP_RAYS;
    const int SR = a.SR;
    float *so = st[0] + lane * COMP_LD, *sb = st[1] + lane * COMP_LD;
    const bool want_o = a.out_opacity != nullptr, want_b = a.out_blendw != nullptr;
    const bool live = r < a.R;
    const int ns = live ? a.ray_ns[r] : 0, off = live ? a.ray_soff[r] : 0;
    const float z0 = pers_z(a.campos, a.rot, 0.f, 0.f, 0.f);
    float T = 1.f, cr = 0.f, cg = 0.f, cb = 0.f;
    bool any_valid = false;
    float prev_cm = 0.f;
    // slot s-1 state while slot s's z is read
    bool pv = false;
    float4 pf = make_float4(0.f, 0.f, 0.f, 0.f);
    int c0 = 0;  // the chunk being staged: slot s lands at column s - c0
    auto process = [&](int slot, float dist) {
        const bool mask = dist < 1e-8f || (a.unit && dist > 2.f * a.vz);
        dist = mask ? a.vz : dist;
        const float valid = pv ? 1.f : 0.f;
        dist = dist * valid;
        const float sigma = (pv ? pf.x : 0.f) * valid;
        const float o = 1.f - expf(-sigma * dist);
        const float wgt = o * T;
        if (pv) {
            cr += pf.y * wgt;
            cg += pf.z * wgt;
            cb += pf.w * wgt;
        }
        if (want_b) sb[slot - c0] = wgt;
        T = T * (1.f - o + 1e-10f);
        if (want_o) so[slot - c0] = o;
    };
    // iteration s reads slot s and closes slot s - 1's interval; slot ns (padding, z0) closes the last
    const int last = !live ? -1 : ns < SR ? ns : SR - 1;
    auto step = [&](int s) {
        float z = z0;
        bool v = false;
        float4 f = make_float4(0.f, 0.f, 0.f, 0.f);
        if (s < ns) {
            const int64_t id = off + s;
            z = pers_z(a.campos, a.rot, a.samp_locw[id * 3], a.samp_locw[id * 3 + 1], a.samp_locw[id * 3 + 2]);
            v = a.samp_nnb[id] > 0;
            if (v) f = *(const float4 *)(a.feat + id * 4);
        }
        const float cm = s == 0 ? z : fmaxf(prev_cm, z);
        if (s > 0) process(s - 1, cm - prev_cm);
        prev_cm = cm;
        pv = v;
        pf = f;
        any_valid |= v;
    };
    if (last >= 0) step(0);
    for (c0 = 0; c0 < SR; c0 += COMP_CW) {  // wave-uniform trip count (see the exit below)
        const int cw = SR - c0 < COMP_CW ? SR - c0 : COMP_CW;
        if (want_o)
            for (int c = 0; c < cw; ++c) so[c] = 0.f;
        if (want_b)
            for (int c = 0; c < cw; ++c) sb[c] = 0.f;
        // iterations whose closed slot s - 1 falls in this chunk
        const int s_end = last < c0 + cw ? last : c0 + cw;
        for (int s = c0 + 1; s <= s_end; ++s) step(s);
        if (live && ns >= SR && c0 + cw == SR) process(SR - 1, a.vz);  // a full ray's last slot: interval vsize[2]
        __syncthreads();
        if (want_o) store_chunk(a.out_opacity + r0 * SR, st[0], SR, c0, cw, nrows, lane);
        if (want_b) store_chunk(a.out_blendw + r0 * SR, st[1], SR, c0, cw, nrows, lane);
        __syncthreads();
        // nothing staged: stop once every lane's slots are done (a wave-uniform exit: the loop body holds
        // barriers; the extra iterations of lanes already past their last slot are no-ops)
        if (!want_o && !want_b && __all(c0 + cw > last)) break;
    }
    if (live) {
        a.out_mask[r] = any_valid ? 1 : 0;
        a.out_rgb[r * 3 + 0] = any_valid ? cr + a.bg0 * T : a.bg0;
        a.out_rgb[r * 3 + 1] = any_valid ? cg + a.bg1 * T : a.bg1;
        a.out_rgb[r * 3 + 2] = any_valid ? cb + a.bg2 * T : a.bg2;
        if (a.out_bgT) a.out_bgT[r] = any_valid ? T : 1.f;
    }
}

// ---- dense ray_march (compatibility sub-boundary, diff_ray_marching.py:509-555) ----------
struct MarchArgs {
    const float *ray_dist, *feat;
    const uint8_t *valid;
    int64_t R;
    int SR;
    float bg0, bg1, bg2;
    int has_bg;
    float *rgb, *opacity, *acc_t, *blendw, *bgT;
};

__global__ __launch_bounds__(256) void k_ray_march_dense(MarchArgs a) {
    const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (r >= a.R) return;
    float T = 1.f, cr = 0.f, cg = 0.f, cb = 0.f;
    for (int s = 0; s < a.SR; ++s) {
        const int64_t i = r * a.SR + s;
        const float v = a.valid[i] ? 1.f : 0.f;
        const float4 f = *(const float4 *)(a.feat + i * 4);
        const float sigma = f.x * v;
        const float o = 1.f - expf(-sigma * a.ray_dist[i]);
        const float wgt = o * T;
        cr += f.y * wgt;
        cg += f.z * wgt;
        cb += f.w * wgt;
        a.opacity[i] = o;
        a.acc_t[i] = T;
        a.blendw[i] = wgt;
        T = T * (1.f - o + 1e-10f);
    }
    a.bgT[r] = T;
    a.rgb[r * 3 + 0] = cr + (a.has_bg ? a.bg0 * T : 0.f);
    a.rgb[r * 3 + 1] = cg + (a.has_bg ? a.bg1 * T : 0.f);
    a.rgb[r * 3 + 2] = cb + (a.has_bg ? a.bg2 * T : 0.f);
}

}  // namespace
}  // namespace sgn

extern "C" int sgn_ray_march_dense(const float *d_ray_dist, const uint8_t *d_valid, const float *d_feat,
                                   int64_t R, int32_t SR, const float *bg, float *d_rgb, float *d_opacity,
                                   float *d_acc_t, float *d_blendw, float *d_bgT, sgn_stream_t stream) {
    using namespace sgn;
    SGN_REQUIRE(d_ray_dist && d_valid && d_feat && d_rgb && d_opacity && d_acc_t && d_blendw && d_bgT,
                "null argument");
    SGN_REQUIRE(SR > 0, "SR must be positive");
    if (R == 0) return 0;
    MarchArgs a;
    a.ray_dist = d_ray_dist; a.valid = d_valid; a.feat = d_feat; a.R = R; a.SR = SR;
    a.has_bg = bg != nullptr;
    a.bg0 = bg ? bg[0] : 0.f; a.bg1 = bg ? bg[1] : 0.f; a.bg2 = bg ? bg[2] : 0.f;
    a.rgb = d_rgb; a.opacity = d_opacity; a.acc_t = d_acc_t; a.blendw = d_blendw; a.bgT = d_bgT;
    hipLaunchKernelGGL(k_ray_march_dense, dim3((unsigned)((R + 255) / 256)), dim3(256), 0, as_stream(stream), a);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

extern "C" int sgn_composite(const sgn_composite_params *cp, const float *d_campos, const float *d_camrotc2w,
                             const float *d_raydir, int64_t R, const float *d_t_table, int32_t per_ray_t,
                             int32_t D, const sgn_query_out *q, const float *d_feat, float *d_out_rgb,
                             int8_t *d_out_mask, float *d_out_bgT, float *d_out_opacity, float *d_out_blendw,
                             sgn_stream_t stream) {
    using namespace sgn;
    (void)d_t_table; (void)per_ray_t; (void)D;
    SGN_REQUIRE(cp && q && d_feat && d_out_rgb && d_out_mask, "null argument");
    SGN_REQUIRE(cp->SR > 0, "SR must be positive");
    if (R == 0) return 0;
    CompArgs a;
    a.campos = d_campos; a.rot = d_camrotc2w; a.raydir = d_raydir;
    a.ray_ns = q->ray_ns; a.ray_soff = q->ray_soff; a.samp_nnb = q->samp_nnb;
    a.samp_locw = q->samp_locw; a.feat = d_feat;
    a.R = R; a.SR = cp->SR; a.unit = cp->raydist_mode_unit; a.vz = cp->vsize_z;
    a.bg0 = cp->bg[0]; a.bg1 = cp->bg[1]; a.bg2 = cp->bg[2];
    a.out_rgb = d_out_rgb; a.out_bgT = d_out_bgT; a.out_opacity = d_out_opacity; a.out_mask = d_out_mask;
    a.out_blendw = d_out_blendw;
    hipLaunchKernelGGL(k_composite, dim3((unsigned)((R + COMP_RAYS - 1) / COMP_RAYS)), dim3(COMP_RAYS), 0,
                       as_stream(stream), a);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}
