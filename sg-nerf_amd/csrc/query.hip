// query.hip -- ray march, shading-sample selection and layered kNN.
//
// Replaces lighting_fast_querier.query_grid_point_index
// (models/neural_points/query_point_indices_worldcoords.py:782-954):
//   mask_raypos (:413-437) + ray compaction / cumsum slot rule (:833-844) +
//   get_shadingloc (:439-461)                    -> k_march (one thread per ray)
//   query_neigh_along_ray_layered (:594-681) and the semantic-guidance variant
//   (:489-591)                                   -> k_knn (one thread per sample)
//
// Differences in structure (not in results):
//   * the [R, D, 3] candidate positions (3.07 GB at 800x800x400) are never
//     materialised: position d is recomputed as campos + raydir * t[d] with the
//     reference's two roundings;
//   * the march stops at the SR-th flagged candidate (later candidates can
//     never receive a slot: slot = cumsum - 1 <= SR - 1);
//   * samples are stored sample-major (prefix sum over rays) so the kNN runs
//     one thread per real sample instead of R*SR threads;
//   * a voxel's candidate points are one contiguous float4 run (grid.hip).
#include <hipcub/hipcub.hpp>
#include <cstdlib>
#include <utility>

#include "sgn_common.h"

namespace sgn {
namespace {

constexpr int TPB = 256;

// Ray batches up to this size march one wave per ray (k_march_wave), larger ones one thread
// per ray (k_march); SGN_MARCH_WAVE_MAX_RAYS overrides (0: always a thread per ray).
int64_t march_wave_max_rays() {
    const char *e = getenv("SGN_MARCH_WAVE_MAX_RAYS");
    return e ? (int64_t)atoll(e) : (int64_t)65536;
}

// ---- march -----------------------------------------------------------------
// [d_lo, d_hi]: the candidates of a ray inside its span through the grid box.
__device__ __forceinline__ void ray_span(const GridView &g, float cx, float cy, float cz, float dx, float dy,
                                         float dz, const float *__restrict__ tt, int D, int &d_lo_out,
                                         int &d_hi_out) {
    // Candidates whose t lies outside the ray's span through the grid box, widened by two voxels
    // on every side (far beyond the rounding of ray_coord / vox_coord), are out of the grid and
    // never flagged: the scan covers [d_lo, d_hi] only (the test inside is unchanged).
    float t_in = -INFINITY, t_out = INFINITY;
    {
        const float c[3] = {cx, cy, cz}, dv[3] = {dx, dy, dz};
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const float lo = g.shift[a] - 2.f * g.vs[a], hi = g.shift[a] + (g.dims[a] + 2.f) * g.vs[a];
            if (dv[a] != 0.f) {
                const float t1 = (lo - c[a]) / dv[a], t2 = (hi - c[a]) / dv[a];
                t_in = fmaxf(t_in, fminf(t1, t2));
                t_out = fminf(t_out, fmaxf(t1, t2));
            } else if (c[a] < lo || c[a] > hi) {
                t_out = -INFINITY;
            }
        }
    }
    int d_lo = 0, d_hi = -1;  // first / last candidate index with t in [t_in, t_out]
    if (t_in <= t_out) {
        int lo = 0, hi = D;  // first d with tt[d] >= t_in
        while (lo < hi) { const int m = (lo + hi) >> 1; if (tt[m] < t_in) lo = m + 1; else hi = m; }
        d_lo = lo;
        lo = d_lo; hi = D;  // first d with tt[d] > t_out
        while (lo < hi) { const int m = (lo + hi) >> 1; if (tt[m] <= t_out) lo = m + 1; else hi = m; }
        d_hi = lo - 1;
    }
    d_lo_out = d_lo;
    d_hi_out = d_hi;
}

// Candidate d of ray r is flagged when its voxel is inside the grid and
// coor_occ == 1 (vox != -2).  The first SR flagged candidates become slots.
template <bool PER_RAY_T>
__global__ __launch_bounds__(TPB) void k_march(GridView g, const float *__restrict__ campos,
                                               const float *__restrict__ raydir, int64_t R,
                                               const float *__restrict__ t_table, int D, int SR,
                                               int32_t *__restrict__ ray_ns,
                                               int16_t *__restrict__ ray_slot_d) {
    int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (r >= R) return;
    const float cx = campos[0], cy = campos[1], cz = campos[2];
    const float dx = raydir[r * 3 + 0], dy = raydir[r * 3 + 1], dz = raydir[r * 3 + 2];
    const float *tt = PER_RAY_T ? t_table + r * (int64_t)D : t_table;
    const int64_t plane = (int64_t)g.dims[1] * g.dims[2];
    int d_lo, d_hi;
    ray_span(g, cx, cy, cz, dx, dy, dz, tt, D, d_lo, d_hi);
    int cnt = 0;
    constexpr int U = 8;  // candidates whose grid words are in flight together
    for (int d0 = d_lo; d0 <= d_hi && cnt < SR; d0 += U) {
        int32_t word[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int d = d0 + u;
            word[u] = VOX_UNFLAGGED;
            if (d <= d_hi) {
                float t = tt[d];
                int ix = vox_coord(ray_coord(cx, dx, t), g.shift[0], g.vs[0]);
                int iy = vox_coord(ray_coord(cy, dy, t), g.shift[1], g.vs[1]);
                int iz = vox_coord(ray_coord(cz, dz, t), g.shift[2], g.vs[2]);
                if (ix >= 0 && ix < g.dims[0] && iy >= 0 && iy < g.dims[1] && iz >= 0 && iz < g.dims[2])
                    word[u] = g.vox[(int64_t)ix * plane + (int64_t)iy * g.dims[2] + iz];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (word[u] != VOX_UNFLAGGED && cnt < SR) {
                ray_slot_d[r * SR + cnt] = (int16_t)(d0 + u);
                ++cnt;
            }
        }
    }
    ray_ns[r] = cnt;
}

// Same slots as k_march, one 64-lane wave per ray (for small ray batches, e.g. the 4096-ray
// training step, where a thread per ray leaves most of the chip idle): lane l tests candidate
// base + l, a ballot and the lanes-below popcount give each flagged candidate its slot, so
// the first SR flagged candidates land in scan order exactly as in the serial loop.
template <bool PER_RAY_T>
__global__ __launch_bounds__(TPB) void k_march_wave(GridView g, const float *__restrict__ campos,
                                                    const float *__restrict__ raydir, int64_t R,
                                                    const float *__restrict__ t_table, int D, int SR,
                                                    int32_t *__restrict__ ray_ns,
                                                    int16_t *__restrict__ ray_slot_d) {
    const int lane = threadIdx.x & 63;
    const int64_t r = blockIdx.x * (int64_t)(TPB / 64) + (threadIdx.x >> 6);
    if (r >= R) return;  // wave-uniform
    const float cx = campos[0], cy = campos[1], cz = campos[2];
    const float dx = raydir[r * 3 + 0], dy = raydir[r * 3 + 1], dz = raydir[r * 3 + 2];
    const float *tt = PER_RAY_T ? t_table + r * (int64_t)D : t_table;
    const int64_t plane = (int64_t)g.dims[1] * g.dims[2];
    int d_lo, d_hi;
    ray_span(g, cx, cy, cz, dx, dy, dz, tt, D, d_lo, d_hi);
    int cnt = 0;
    for (int base = d_lo; base <= d_hi && cnt < SR; base += 64) {
        const int d = base + lane;
        int32_t word = VOX_UNFLAGGED;
        if (d <= d_hi) {
            const float t = tt[d];
            const int ix = vox_coord(ray_coord(cx, dx, t), g.shift[0], g.vs[0]);
            const int iy = vox_coord(ray_coord(cy, dy, t), g.shift[1], g.vs[1]);
            const int iz = vox_coord(ray_coord(cz, dz, t), g.shift[2], g.vs[2]);
            if (ix >= 0 && ix < g.dims[0] && iy >= 0 && iy < g.dims[1] && iz >= 0 && iz < g.dims[2])
                word = g.vox[(int64_t)ix * plane + (int64_t)iy * g.dims[2] + iz];
        }
        const bool flagged = word != VOX_UNFLAGGED;
        const uint64_t mask = __ballot(flagged);
        const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
        if (flagged && cnt + rank < SR) ray_slot_d[r * SR + cnt + rank] = (int16_t)d;
        cnt += __popcll(mask);
    }
    if (lane == 0) ray_ns[r] = cnt < SR ? cnt : SR;
}

__global__ void k_sample_total(const int32_t *__restrict__ soff, const int32_t *__restrict__ ns,
                               int64_t R, int32_t *__restrict__ counters) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        counters[0] = R > 0 ? soff[R - 1] + ns[R - 1] : 0;
        counters[1] = 0;
        counters[2] = 0;
        counters[3] = 0;
    }
}

__global__ __launch_bounds__(TPB) void k_emit_samples(const int32_t *__restrict__ ray_ns,
                                                      const int32_t *__restrict__ ray_soff,
                                                      const int16_t *__restrict__ ray_slot_d, int64_t R,
                                                      int SR, int32_t *__restrict__ samp_ray,
                                                      int32_t *__restrict__ samp_d) {
    int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (r >= R) return;
    int n = ray_ns[r], o = ray_soff[r];
    for (int j = 0; j < n; ++j) {
        samp_ray[o + j] = (int32_t)r;
        samp_d[o + j] = ray_slot_d[r * SR + j];
    }
}

// ---- layered kNN -------------------------------------------------------------
template <int K>
struct KBuf {
    int32_t id[K];
    float d2[K];
    int kid, far_ind;
    float far2;
    __device__ __forceinline__ void init() {
#pragma unroll
        for (int i = 0; i < K; ++i) { id[i] = -1; d2[i] = 0.f; }
        kid = 0; far_ind = 0; far2 = 0.f;
    }
    // :653-672, register-resident, static indices only
    __device__ __forceinline__ void push(int32_t pidx, float xyz2) {
        if (kid < K) {
#pragma unroll
            for (int i = 0; i < K; ++i)
                if (i == kid) { id[i] = pidx; d2[i] = xyz2; }
            if (xyz2 > far2) { far2 = xyz2; far_ind = kid; }
            ++kid;
        } else {
            ++kid;
            if (xyz2 < far2) {
#pragma unroll
                for (int i = 0; i < K; ++i)
                    if (i == far_ind) { id[i] = pidx; d2[i] = xyz2; }
                float f = xyz2;
                int fi = far_ind;
#pragma unroll
                for (int i = 0; i < K; ++i)
                    if (d2[i] > f) { f = d2[i]; fi = i; }
                far2 = f;
                far_ind = fi;
            }
        }
    }
};

template <int K, bool SEMANTIC, bool COUNT>
__global__ __launch_bounds__(TPB) void k_knn(GridView g, const float *__restrict__ campos,
                                             const float *__restrict__ raydir,
                                             const float *__restrict__ t_table, int D, int per_ray_t,
                                             int SR, float r2, int dense_out,
                                             const int32_t *__restrict__ point_labels,
                                             const int32_t *__restrict__ ray_labels, uint32_t sec_mod10,
                                             const int32_t *__restrict__ ray_soff,
                                             const int32_t *__restrict__ samp_ray,
                                             const int32_t *__restrict__ samp_d,
                                             int32_t *__restrict__ counters, float *__restrict__ samp_locw,
                                             int32_t *__restrict__ samp_nnb, int32_t *__restrict__ pidx_out,
                                             int32_t *__restrict__ work) {
    const int64_t S = counters[0];
    const int64_t plane = (int64_t)g.dims[1] * g.dims[2];
    int n_vox = 0, n_cand = 0;  // algorithmic-traffic counters (bench roofline), one atomic per wave
    for (int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; s < S;
         s += (int64_t)gridDim.x * blockDim.x) {
        const int32_t r = samp_ray[s];
        const int32_t d = samp_d[s];
        const float t = per_ray_t ? t_table[(int64_t)r * D + d] : t_table[d];
        const float ctr_x = ray_coord(campos[0], raydir[(int64_t)r * 3 + 0], t);
        const float ctr_y = ray_coord(campos[1], raydir[(int64_t)r * 3 + 1], t);
        const float ctr_z = ray_coord(campos[2], raydir[(int64_t)r * 3 + 2], t);
        const int fx = vox_coord(ctr_x, g.shift[0], g.vs[0]);
        const int fy = vox_coord(ctr_y, g.shift[1], g.vs[1]);
        const int fz = vox_coord(ctr_z, g.shift[2], g.vs[2]);
        int center_label = 0;
        if (SEMANTIC) center_label = ray_labels[r];
        KBuf<K> kb;
        kb.init();
        const int nlayer = (g.kernel0 + 1) / 2;
        for (int layer = 0; layer < nlayer; ++layer) {
            const int x0 = max(-fx, -layer), x1 = min(g.dims[0] - fx, layer + 1);
            const int y0 = max(-fy, -layer), y1 = min(g.dims[1] - fy, layer + 1);
            const int z0 = max(-fz, -layer), z1 = min(g.dims[2] - fz, layer + 1);
            for (int x = x0; x < x1; ++x)
                for (int y = y0; y < y1; ++y)
                    for (int z = z0; z < z1; ++z) {
                        if (max(abs(z), max(abs(x), abs(y))) != layer) continue;
                        const int32_t occ =
                            g.vox[(int64_t)(fx + x) * plane + (int64_t)(fy + y) * g.dims[2] + (fz + z)];
                        if (COUNT) ++n_vox;
                        if (occ < 0) continue;
                        const int32_t st = g.start[occ], n = g.cnt[occ];
                        if (COUNT) n_cand += n;
                        for (int q = 0; q < n; ++q) {
                            const float4 pt = g.pts[st + q];
                            const int32_t pid = __float_as_int(pt.w);
                            if (SEMANTIC) {
                                // :548-553 with label_prob == 0 (int tensor read as float, :916)
                                int lv = point_labels[pid];
                                bool pass = center_label == lv || lv == 0 || center_label == 0 || sec_mod10 <= 1u;
                                if (!pass) continue;
                            }
                            const float xv = __fsub_rn(pt.x, ctr_x);
                            const float yv = __fsub_rn(pt.y, ctr_y);
                            const float zv = __fsub_rn(pt.z, ctr_z);
                            const float xyz2 = __fmaf_rn(zv, zv, __fmaf_rn(yv, yv, __fmul_rn(xv, xv)));
                            if (r2 == 0.0f || xyz2 <= r2) kb.push(pid, xyz2);
                        }
                    }
            if (kb.kid >= K) break;
        }
        const int64_t ob = dense_out ? ((int64_t)r * SR + (s - ray_soff[r])) * K : s * K;
#pragma unroll
        for (int i = 0; i < K; ++i) pidx_out[ob + i] = kb.id[i];
        const int nnb = kb.kid < K ? kb.kid : K;
        samp_nnb[s] = nnb;
        samp_locw[s * 3 + 0] = ctr_x;
        samp_locw[s * 3 + 1] = ctr_y;
        samp_locw[s * 3 + 2] = ctr_z;
        if (nnb > 0) {
            int32_t w = atomicAdd(counters + 1, 1);
            work[w] = (int32_t)s;
        }
    }
    if constexpr (COUNT) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            n_vox += __shfl_xor(n_vox, o);
            n_cand += __shfl_xor(n_cand, o);
        }
        if ((threadIdx.x & 63) == 0) {
            atomicAdd(counters + 2, n_vox);
            atomicAdd((uint32_t *)counters + 3, (uint32_t)n_cand);
        }
    }
}

template <class F, int... I>
__device__ __forceinline__ void unroll_impl(F &&f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void unroll(F &&f) {  // f(integral_constant<0..N-1>), fully unrolled
    unroll_impl(f, std::make_integer_sequence<int, N>{});
}

// ---- layered kNN, query_size 3 (ScanNet / NeRF-synthetic configs) ----------------
// Same visit order and replacement rule as k_knn (layer 0 = the centre voxel, layer 1 = the 26
// others in x, y, z order; worldcoords.py:636-642), restructured for memory-level parallelism:
// the 27 grid words are loaded together, then the 27 {start, count} pairs together, so a
// sample waits on two dependent loads instead of 2 x 27 before its candidate runs; inside a
// voxel two candidates are in flight.  Out-of-grid neighbours read as empty, exactly like the
// reference's clipped loop bounds (:628-633).
template <int K, bool SEMANTIC>
__global__ __launch_bounds__(TPB) void k_knn27(GridView g, const float *__restrict__ campos,
                                               const float *__restrict__ raydir,
                                               const float *__restrict__ t_table, int D, int per_ray_t,
                                               int SR, float r2, int dense_out,
                                               const int32_t *__restrict__ point_labels,
                                               const int32_t *__restrict__ ray_labels, uint32_t sec_mod10,
                                               const int32_t *__restrict__ ray_soff,
                                               const int32_t *__restrict__ samp_ray,
                                               const int32_t *__restrict__ samp_d,
                                               int32_t *__restrict__ counters, float *__restrict__ samp_locw,
                                               int32_t *__restrict__ samp_nnb, int32_t *__restrict__ pidx_out,
                                               int32_t *__restrict__ work) {
    __shared__ uint32_t knn_runs[26 * TPB];
    const int64_t S = counters[0];
    const int64_t plane = (int64_t)g.dims[1] * g.dims[2];
    for (int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; s < S;
         s += (int64_t)gridDim.x * blockDim.x) {
        const int32_t r = samp_ray[s];
        const int32_t d = samp_d[s];
        const float t = per_ray_t ? t_table[(int64_t)r * D + d] : t_table[d];
        const float ctr_x = ray_coord(campos[0], raydir[(int64_t)r * 3 + 0], t);
        const float ctr_y = ray_coord(campos[1], raydir[(int64_t)r * 3 + 1], t);
        const float ctr_z = ray_coord(campos[2], raydir[(int64_t)r * 3 + 2], t);
        const int fx = vox_coord(ctr_x, g.shift[0], g.vs[0]);
        const int fy = vox_coord(ctr_y, g.shift[1], g.vs[1]);
        const int fz = vox_coord(ctr_z, g.shift[2], g.vs[2]);
        int center_label = 0;
        if (SEMANTIC) center_label = ray_labels[r];
        int2 sc[27];
        {
            // Branch-free: every load reads a valid address (clamped voxel, slot 0 for empty ones;
            // a sample exists only if some voxel is flagged, so slot 0 exists) and a select drops
            // it.  With `cond ? load : default` the compiler issued each {start, count} load in
            // its own branch and waited for it before the next: 27 serial memory latencies.
            int32_t wd[27];
#pragma unroll
            for (int v = 0; v < 27; ++v) {
                const int x = fx + v / 9 - 1, y = fy + (v / 3) % 3 - 1, z = fz + v % 3 - 1;
                const bool in = (unsigned)x < (unsigned)g.dims[0] && (unsigned)y < (unsigned)g.dims[1] &&
                                (unsigned)z < (unsigned)g.dims[2];
                const int xc = min(max(x, 0), g.dims[0] - 1), yc = min(max(y, 0), g.dims[1] - 1),
                          zc = min(max(z, 0), g.dims[2] - 1);
                const int32_t word = g.vox[(int64_t)xc * plane + (int64_t)yc * g.dims[2] + zc];
                wd[v] = in ? word : -1;
            }
            int2 e[27];
#pragma unroll
            for (int v = 0; v < 27; ++v) e[v] = g.sc[wd[v] >= 0 ? wd[v] : 0];
            // the empty asm consumes every result unconditionally, so the optimizer cannot sink a
            // load into a branch on its own condition (which serialised them)
#pragma unroll
            for (int v = 0; v < 27; ++v) asm volatile("" : "+v"(e[v].x), "+v"(e[v].y));
#pragma unroll
            for (int v = 0; v < 27; ++v) sc[v] = wd[v] >= 0 ? e[v] : make_int2(0, 0);
        }
        KBuf<K> kb;
        kb.init();
        auto consider = [&](float4 pt) {
            const int32_t pid = __float_as_int(pt.w);
            if (SEMANTIC) {
                const int lv = point_labels[pid];
                if (!(center_label == lv || lv == 0 || center_label == 0 || sec_mod10 <= 1u)) return;
            }
            const float xv = __fsub_rn(pt.x, ctr_x);
            const float yv = __fsub_rn(pt.y, ctr_y);
            const float zv = __fsub_rn(pt.z, ctr_z);
            const float xyz2 = __fmaf_rn(zv, zv, __fmaf_rn(yv, yv, __fmul_rn(xv, xv)));
            if (r2 == 0.0f || xyz2 <= r2) kb.push(pid, xyz2);
        };
        auto visit = [&](int2 c) {
            int q = 0;
            for (; q + 1 < c.y; q += 2) {
                const float4 p0 = g.pts[c.x + q], p1 = g.pts[c.x + q + 1];
                consider(p0);
                consider(p1);
            }
            if (q < c.y) consider(g.pts[c.x + q]);
        };
        visit(sc[13]);  // layer 0
        if (kb.kid < K) {
            // layer 1: the 26 neighbours' candidate runs concatenated in visit order and walked
            // with one cursor per lane, one candidate per iteration (next one's load in flight):
            // a wave iterates max over lanes of the sample's total instead of the sum over
            // voxels of the per-voxel maximum (~4x fewer iterations on surfaces).  The run
            // table is this lane's column of LDS ({start << 6 | count}, [26][TPB]).
            uint32_t *lst = knn_runs + threadIdx.x;
            int n = 0, total = 0;
            unroll<27>([&](auto vv) {
                constexpr int v = decltype(vv)::value;
                if constexpr (v != 13) {
                    if (sc[v].y > 0) {
                        lst[n * TPB] = ((uint32_t)sc[v].x << 6) | (uint32_t)sc[v].y;
                        ++n;
                        total += sc[v].y;
                    }
                }
            });
            int vi = 0, q = 0, st = 0, cnt = 0;
            if (n > 0) {
                const uint32_t e = lst[0];
                st = (int)(e >> 6);
                cnt = (int)(e & 63);
            }
            auto next_addr = [&]() {  // position of the next candidate; advances the cursor
                const int at = st + q;
                if (++q == cnt) {
                    q = 0;
                    if (++vi < n) {
                        const uint32_t e = lst[vi * TPB];
                        st = (int)(e >> 6);
                        cnt = (int)(e & 63);
                    }
                }
                return at;
            };
            if (total > 0) {
                float4 cur = g.pts[next_addr()];
                for (int j = 1; j < total; ++j) {
                    const float4 nxt = g.pts[next_addr()];
                    consider(cur);
                    cur = nxt;
                }
                consider(cur);
            }
        }
        const int64_t ob = dense_out ? ((int64_t)r * SR + (s - ray_soff[r])) * K : s * K;
#pragma unroll
        for (int i = 0; i < K; ++i) pidx_out[ob + i] = kb.id[i];
        const int nnb = kb.kid < K ? kb.kid : K;
        samp_nnb[s] = nnb;
        samp_locw[s * 3 + 0] = ctr_x;
        samp_locw[s * 3 + 1] = ctr_y;
        samp_locw[s * 3 + 2] = ctr_z;
        if (nnb > 0) {
            int32_t w = atomicAdd(counters + 1, 1);
            work[w] = (int32_t)s;
        }
    }
}

size_t scan_temp_bytes(int64_t R) {
    size_t tb = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tb, (const int32_t *)nullptr, (int32_t *)nullptr,
                                           (int)(R > 0 ? R : 1), (hipStream_t)0);
    return tb;
}

template <int K>
void launch_knn(dim3 grid, hipStream_t st, bool semantic, bool count, bool runs_fit, GridView g, const float *campos,
                const float *raydir, const float *t, int D, int per_ray_t, int SR, float r2,
                int dense, const int32_t *pl, const int32_t *rl, uint32_t sec,
                const sgn_query_out *o) {
    // k_knn27: query_size 3; its run table entries pack {start < 2^26, count < 64}
    const bool k27 = g.kernel0 == 3 && !count && runs_fit;
    auto kern = semantic ? (count ? k_knn<K, true, true> : k27 ? k_knn27<K, true> : k_knn<K, true, false>)
                         : (count ? k_knn<K, false, true> : k27 ? k_knn27<K, false> : k_knn<K, false, false>);
    hipLaunchKernelGGL(kern, grid, dim3(TPB), 0, st, g, campos, raydir, t, D, per_ray_t, SR, r2, dense, pl, rl, sec,
                       o->ray_soff, o->samp_ray, o->samp_d, o->counters, o->samp_locw, o->samp_nnb, o->pidx, o->work);
}

// ---- training-mode depth table (jitter > 0): near_far_linear_ray_generation,
// diff_ray_marching.py:349-393 -- tvals = linspace(0, 1, D + 1) (torch's two-sided linspace
// formula), t = near (1 - tvals) + far tvals, seg_i = (t_{i+1} - t_i) (1 + jitter (rnd_i - 0.5)),
// end = near + [0, cumsum(seg)], mid_i = (end_i + end_{i+1}) / 2.  One wave per ray, the cumsum as
// a wave scan per 64-segment chunk with the running sum carried across chunks (the torch
// sequence is ~17 launches over [R, D]).
__device__ __forceinline__ float linspace01(int i, int steps) {
    const float step = 1.0f / (float)(steps - 1);
    const int half = steps / 2;
    return i < half ? step * (float)i : 1.0f - step * (float)(steps - i - 1);
}

__global__ __launch_bounds__(256) void k_depth_jitter(float near, float far, int D, float jitter, int64_t R,
                                                      const float *__restrict__ rnd, float *__restrict__ t) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= R) return;
    const float *rr = rnd + r * D;
    float *tr = t + r * D;
    float carry = 0.f;   // cumsum of the segments before this chunk
    for (int c0 = 0; c0 < D; c0 += 64) {
        const int i = c0 + lane;
        float seg = 0.f;
        if (i < D) {
            const float ta = linspace01(i, D + 1), tb = linspace01(i + 1, D + 1);
            const float za = near * (1.0f - ta) + far * ta, zb = near * (1.0f - tb) + far * tb;
            seg = (zb - za) * (1.0f + jitter * (rr[i] - 0.5f));
        }
        float inc = seg;   // inclusive scan over the wave, in lane order
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const float v = __shfl_up(inc, o, 64);
            if (lane >= o) inc += v;
        }
        const float cs = carry + inc;                       // cumsum through segment i
        float prev = __shfl_up(cs, 1, 64);                  // cumsum through segment i - 1
        if (lane == 0) prev = carry;
        if (i < D) {
            const float e0 = (i == 0) ? near : near + prev, e1 = near + cs;
            tr[i] = (e0 + e1) / 2.0f;
        }
        carry = __shfl(cs, 63, 64);
    }
}

}  // namespace
}  // namespace sgn

extern "C" {

int sgn_depth_table_jitter(float near, float far, int32_t D, float jitter, int64_t R, const float *d_rnd, float *d_t,
                           sgn_stream_t stream) {
    SGN_REQUIRE(D >= 1 && R >= 0, "sgn_depth_table_jitter: D >= 1, R >= 0");
    if (R == 0) return 0;
    SGN_REQUIRE(d_rnd && d_t, "sgn_depth_table_jitter: null buffer");
    hipLaunchKernelGGL(sgn::k_depth_jitter, dim3((unsigned)((R + 3) / 4)), dim3(256), 0, sgn::as_stream(stream), near, far,
                       (int)D, jitter, R, d_rnd, d_t);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

size_t sgn_query_workspace_bytes(int64_t R) {
    // [R*SR_MAX int16 slot->depth table] is carved by the caller? no: kept here.
    size_t scan = sgn::scan_temp_bytes(R);
    size_t slots = (size_t)(R > 0 ? R : 1) * 128 * sizeof(int16_t);
    return ((scan + 255) / 256) * 256 + slots;
}

int sgn_query(const sgn_grid *grid, const sgn_query_params *qp, const float *d_campos,
              const float *d_raydir, int64_t R, const float *d_t_table, const int32_t *d_point_labels,
              const int32_t *d_ray_labels, const sgn_query_out *o, void *d_workspace,
              size_t workspace_bytes, sgn_stream_t stream) {
    using namespace sgn;
    SGN_REQUIRE(grid && qp && o, "null grid/params/out");
    SGN_REQUIRE(qp->SR > 0 && qp->SR <= 128, "SR must be in [1, 128]");
    SGN_REQUIRE(qp->K == 1 || qp->K == 4 || qp->K == 8 || qp->K == 16, "K must be 1, 4, 8 or 16");
    SGN_REQUIRE(qp->D > 0 && qp->D <= 32767, "D must be in [1, 32767]");
    SGN_REQUIRE(!qp->semantic || (d_point_labels && d_ray_labels), "semantic query needs labels");
    SGN_REQUIRE(R >= 0 && R * (int64_t)qp->SR < (int64_t)INT32_MAX, "R*SR must fit int32");
    SGN_REQUIRE(workspace_bytes >= sgn_query_workspace_bytes(R), "workspace too small");
    hipStream_t st = as_stream(stream);
    if (R == 0) {
        SGN_CHECK_HIP(hipMemsetAsync(o->counters, 0, 4 * sizeof(int32_t), st));
        return 0;
    }
    size_t scan = scan_temp_bytes(R);
    char *ws = (char *)d_workspace;
    int16_t *slot_d = (int16_t *)(ws + ((scan + 255) / 256) * 256);
    GridView g = grid->view();
    dim3 rg((unsigned)((R + TPB - 1) / TPB));
    if (R <= march_wave_max_rays()) {  // small batches: one wave per ray
        dim3 wg((unsigned)((R + TPB / 64 - 1) / (TPB / 64)));
        if (qp->per_ray_t)
            hipLaunchKernelGGL((k_march_wave<true>), wg, dim3(TPB), 0, st, g, d_campos, d_raydir, R, d_t_table,
                               qp->D, qp->SR, o->ray_ns, slot_d);
        else
            hipLaunchKernelGGL((k_march_wave<false>), wg, dim3(TPB), 0, st, g, d_campos, d_raydir, R, d_t_table,
                               qp->D, qp->SR, o->ray_ns, slot_d);
    } else if (qp->per_ray_t) {
        hipLaunchKernelGGL((k_march<true>), rg, dim3(TPB), 0, st, g, d_campos, d_raydir, R, d_t_table,
                           qp->D, qp->SR, o->ray_ns, slot_d);
    } else {
        hipLaunchKernelGGL((k_march<false>), rg, dim3(TPB), 0, st, g, d_campos, d_raydir, R, d_t_table,
                           qp->D, qp->SR, o->ray_ns, slot_d);
    }
    SGN_CHECK_HIP(hipcub::DeviceScan::ExclusiveSum(ws, scan, o->ray_ns, o->ray_soff, (int)R, st));
    hipLaunchKernelGGL(k_sample_total, dim3(1), dim3(64), 0, st, o->ray_soff, o->ray_ns, R, o->counters);
    hipLaunchKernelGGL(k_emit_samples, rg, dim3(TPB), 0, st, o->ray_ns, o->ray_soff, slot_d, R, qp->SR,
                       o->samp_ray, o->samp_d);
    int64_t cap = R * qp->SR;
    int64_t kb = (cap + TPB - 1) / TPB;
    dim3 kg((unsigned)(kb < 16384 ? kb : 16384));
    uint32_t sec = (uint32_t)(qp->seconds % 10);
    const bool runs_fit = grid->p.P <= 63 && grid->n_listed < ((int64_t)1 << 26);
    switch (qp->K) {
        case 1: launch_knn<1>(kg, st, qp->semantic, qp->count_traffic, runs_fit, g, d_campos, d_raydir, d_t_table, qp->D, qp->per_ray_t, qp->SR, qp->r2, qp->dense_out, d_point_labels, d_ray_labels, sec, o); break;
        case 4: launch_knn<4>(kg, st, qp->semantic, qp->count_traffic, runs_fit, g, d_campos, d_raydir, d_t_table, qp->D, qp->per_ray_t, qp->SR, qp->r2, qp->dense_out, d_point_labels, d_ray_labels, sec, o); break;
        case 8: launch_knn<8>(kg, st, qp->semantic, qp->count_traffic, runs_fit, g, d_campos, d_raydir, d_t_table, qp->D, qp->per_ray_t, qp->SR, qp->r2, qp->dense_out, d_point_labels, d_ray_labels, sec, o); break;
        default: launch_knn<16>(kg, st, qp->semantic, qp->count_traffic, runs_fit, g, d_campos, d_raydir, d_t_table, qp->D, qp->per_ray_t, qp->SR, qp->r2, qp->dense_out, d_point_labels, d_ray_labels, sec, o); break;
    }
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

}  // extern "C"
