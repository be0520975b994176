// grid.hip -- deterministic device build of the world-coordinate occupancy grid.
//
// Replaces lighting_fast_querier.build_occ_vox
// (models/neural_points/query_point_indices_worldcoords.py:706-778: claim_occ
// :265-326, map_coor2occ :328-363, fill_occ2pnts :365-410).  The reference
// rebuilds two dense int32 grids on every ray chunk (:797); here the grid is
// built once per point-cloud version and cached in an opaque sgn_grid.
//
// Layout (HBM):
//   vox       int32[vol]   one word per voxel: slot id >= 0 (occupied & mapped,
//                          hence flagged), -1 flagged-empty (coor_occ = 1),
//                          -2 unflagged.  One 4-byte read answers both the
//                          march test (mask_raypos :435) and the kNN lookup
//                          (coor_2_occ :644).
//   occ_start/occ_kept     int32[n_slots] CSR over slots.
//   cell_pts  float4[n_listed]  {x, y, z, bits(point index)} of every kept
//                          point, grouped by slot, in the reference's list
//                          order: a voxel's candidates are one contiguous run
//                          instead of P scattered 12-byte reads.
//
// Order ("parity mode"): claims and per-voxel lists in point-index order, the
// reservoir (:312-321, :400-407) resolved as a sequential Algorithm-R pass
// would resolve it (the latest ordinal wins a slot: atomicMax), draws from
// sgn::uniform01(seed, stream, point index).  Same rules as oracle/query_ref.c.
#include <hipcub/hipcub.hpp>
#include <climits>
#include <vector>

#include "sgn_common.h"

namespace sgn {

namespace {

constexpr int TPB = 256;

inline int blocks_for(int64_t n, int cap = 65536) {
    int64_t b = (n + TPB - 1) / TPB;
    if (b < 1) b = 1;
    return (int)(b < cap ? b : cap);
}

struct GridGeom {
    float sx, sy, sz, vx, vy, vz;
    int dx, dy, dz;
    __device__ __forceinline__ int64_t lin(int x, int y, int z) const {
        return (int64_t)x * ((int64_t)dy * dz) + (int64_t)y * dz + z;
    }
};

__global__ void k_point_keys(const float *__restrict__ pts, int64_t n, GridGeom g,
                             int32_t *__restrict__ key, int32_t *__restrict__ first) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        int cx = vox_coord(pts[i * 3 + 0], g.sx, g.vx);
        int cy = vox_coord(pts[i * 3 + 1], g.sy, g.vy);
        int cz = vox_coord(pts[i * 3 + 2], g.sz, g.vz);
        if (cx < 0 || cx >= g.dx || cy < 0 || cy >= g.dy || cz < 0 || cz >= g.dz) {
            key[i] = -1;
            continue;
        }
        int64_t l = g.lin(cx, cy, cz);
        key[i] = (int32_t)l;
        atomicMin(first + l, (int32_t)i);
    }
}

__global__ void k_is_first(const int32_t *__restrict__ key, const int32_t *__restrict__ first,
                           int64_t n, int32_t *__restrict__ flag) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        int32_t k = key[i];
        flag[i] = (k >= 0 && first[k] == (int32_t)i) ? 1 : 0;
    }
}

__global__ void k_total(const int32_t *__restrict__ excl, const int32_t *__restrict__ val,
                        int64_t n, int64_t *__restrict__ out) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *out = n > 0 ? (int64_t)excl[n - 1] + val[n - 1] : 0;
}

// claim_occ's slot assignment (:305-321): id t = claim rank; beyond max_o the
// reservoir draw picks a victim slot, the latest claimant (largest t) wins.
__global__ void k_assign_slots(const int32_t *__restrict__ key, const int32_t *__restrict__ flag,
                               const int32_t *__restrict__ rank, int64_t n, int32_t max_o,
                               uint64_t seed, int32_t *__restrict__ slot_vox,
                               unsigned long long *__restrict__ slot_win) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        if (!flag[i]) continue;
        int32_t t = rank[i];
        if (t < max_o) {
            slot_vox[t] = key[i];
        } else {
            float u = uniform01(seed, 1, (uint64_t)i);
            int insrt = (int)ceilf(__fmul_rn(u, (float)(t + 1))) - 1;
            if (insrt < max_o)
                atomicMax(slot_win + insrt,
                          ((unsigned long long)(uint32_t)t << 32) | (uint32_t)key[i]);
        }
    }
}

__global__ void k_map_slots(int32_t *__restrict__ slot_vox, const unsigned long long *__restrict__ slot_win,
                            int64_t n_slots, int32_t *__restrict__ vox) {
    for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n_slots;
         j += (int64_t)gridDim.x * blockDim.x) {
        unsigned long long w = slot_win[j];
        int32_t v = w ? (int32_t)(uint32_t)(w & 0xffffffffull) : slot_vox[j];
        slot_vox[j] = v;
        vox[v] = (int32_t)j;
    }
}

// map_coor2occ's neighbourhood flag (:353-361), query_size extent.
__global__ void k_flag(const int32_t *__restrict__ slot_vox, int64_t n_slots, GridGeom g, int3 qs,
                       int32_t *__restrict__ vox) {
    for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n_slots;
         j += (int64_t)gridDim.x * blockDim.x) {
        int64_t v = slot_vox[j];
        int64_t plane = (int64_t)g.dy * g.dz;
        int cx = (int)(v / plane), cy = (int)((v / g.dz) % g.dy), cz = (int)(v % g.dz);
        int x0 = max(0, cx - qs.x / 2), x1 = min(g.dx, cx + (qs.x + 1) / 2);
        int y0 = max(0, cy - qs.y / 2), y1 = min(g.dy, cy + (qs.y + 1) / 2);
        int z0 = max(0, cz - qs.z / 2), z1 = min(g.dz, cz + (qs.z + 1) / 2);
        for (int x = x0; x < x1; ++x)
            for (int y = y0; y < y1; ++y)
                for (int z = z0; z < z1; ++z) {
                    int32_t *c = vox + g.lin(x, y, z);
                    if (*c == VOX_UNFLAGGED) *c = VOX_FLAGGED;  // benign: all writers store -1
                }
    }
}

// fill_occ2pnts routing (:394-396): slot of the point's voxel, the `> 0` bug
// unless fix_occ0.  Unrouted points get the sentinel n_slots (sorted last).
__global__ void k_point_slot(const int32_t *__restrict__ key, const int32_t *__restrict__ vox,
                             int64_t n, int32_t n_slots, int32_t fix_occ0,
                             uint32_t *__restrict__ pslot, int32_t *__restrict__ pid) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        int32_t k = key[i];
        int32_t s = k >= 0 ? vox[k] : -1;
        bool ok = fix_occ0 ? (s >= 0) : (s > 0);
        pslot[i] = ok ? (uint32_t)s : (uint32_t)n_slots;
        pid[i] = (int32_t)i;
    }
}

__global__ void k_segments(const uint32_t *__restrict__ skey, int64_t n, uint32_t n_slots,
                           int32_t *__restrict__ seg_start, int32_t *__restrict__ seg_end) {
    for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n;
         q += (int64_t)gridDim.x * blockDim.x) {
        uint32_t s = skey[q];
        if (s >= n_slots) continue;
        if (q == 0 || skey[q - 1] != s) seg_start[s] = (int32_t)q;
        if (q == n - 1 || skey[q + 1] != s) seg_end[s] = (int32_t)(q + 1);
    }
}

__global__ void k_reservoir(const uint32_t *__restrict__ skey, const int32_t *__restrict__ sval,
                            int64_t n, uint32_t n_slots, const int32_t *__restrict__ seg_start,
                            int32_t P, uint64_t seed, int32_t *__restrict__ resv) {
    for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n;
         q += (int64_t)gridDim.x * blockDim.x) {
        uint32_t s = skey[q];
        if (s >= n_slots) continue;
        int32_t t = (int32_t)q - seg_start[s];
        if (t < P) continue;
        float u = uniform01(seed, 2, (uint64_t)sval[q]);
        int insrt = (int)ceilf(__fmul_rn(u, (float)(t + 1))) - 1;
        if (insrt < P) atomicMax(resv + (int64_t)s * P + insrt, t);
    }
}

__global__ void k_counts(const int32_t *__restrict__ seg_start, const int32_t *__restrict__ seg_end,
                         int64_t n_slots, int32_t P, int32_t *__restrict__ routed,
                         int32_t *__restrict__ kept) {
    for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n_slots;
         j += (int64_t)gridDim.x * blockDim.x) {
        int32_t r = seg_end[j] - seg_start[j];
        routed[j] = r;
        kept[j] = r < P ? r : P;
    }
}

__global__ void k_interleave_sc(const int32_t *__restrict__ start, const int32_t *__restrict__ kept, int64_t n_slots,
                                int2 *__restrict__ sc) {
    for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n_slots;
         j += (int64_t)gridDim.x * blockDim.x)
        sc[j] = make_int2(start[j], kept[j]);
}

__global__ void k_emit_points(const uint32_t *__restrict__ skey, const int32_t *__restrict__ sval,
                              int64_t n, uint32_t n_slots, const int32_t *__restrict__ seg_start,
                              const int32_t *__restrict__ resv, const int32_t *__restrict__ occ_start,
                              int32_t P, const float *__restrict__ pts, float4 *__restrict__ cell) {
    for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n;
         q += (int64_t)gridDim.x * blockDim.x) {
        uint32_t s = skey[q];
        if (s >= n_slots) continue;
        int32_t t = (int32_t)q - seg_start[s];
        if (t >= P) continue;
        int32_t w = resv[(int64_t)s * P + t];
        int32_t src = w >= 0 ? seg_start[s] + w : (int32_t)q;
        int32_t p = sval[src];
        cell[occ_start[s] + t] =
            make_float4(pts[(int64_t)p * 3], pts[(int64_t)p * 3 + 1], pts[(int64_t)p * 3 + 2],
                        __int_as_float(p));
    }
}

__global__ void k_export_grid(const int32_t *__restrict__ vox, int64_t vol, int32_t *__restrict__ coor_occ,
                              int32_t *__restrict__ coor_2_occ) {
    for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < vol;
         v += (int64_t)gridDim.x * blockDim.x) {
        int32_t x = vox[v];
        if (coor_occ) coor_occ[v] = x != VOX_UNFLAGGED ? 1 : 0;
        if (coor_2_occ) coor_2_occ[v] = x >= 0 ? x : -1;
    }
}

__global__ void k_export_lists(const int32_t *__restrict__ start, const int32_t *__restrict__ kept,
                               const int32_t *__restrict__ routed, const float4 *__restrict__ cell,
                               int64_t n_slots, int32_t max_o, int32_t P,
                               int32_t *__restrict__ numpnts, int32_t *__restrict__ lists) {
    for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < max_o;
         j += (int64_t)gridDim.x * blockDim.x) {
        int32_t k = j < n_slots ? kept[j] : 0;
        if (numpnts) numpnts[j] = j < n_slots ? routed[j] : 0;
        if (lists)
            for (int g = 0; g < P; ++g)
                lists[j * P + g] = g < k ? __float_as_int(cell[start[j] + g].w) : -1;
    }
}

template <typename T>
int dalloc(T **p, int64_t count, int64_t *acc = nullptr) {
    size_t bytes = (size_t)(count > 0 ? count : 1) * sizeof(T);
    SGN_CHECK_HIP(hipMalloc((void **)p, bytes));
    if (acc) *acc += (int64_t)bytes;
    return 0;
}

struct TmpBufs {
    std::vector<void *> ptrs;
    ~TmpBufs() {
        for (void *p : ptrs) (void)hipFree(p);
    }
    template <typename T>
    int get(T **p, int64_t count) {
        int rc = dalloc(p, count);
        if (rc == 0) ptrs.push_back(*p);
        return rc;
    }
};

}  // namespace

static int grid_build_impl(const float *d_points, int64_t n, const sgn_grid_params *prm,
                           hipStream_t st, sgn_grid *g) {
    g->p = *prm;
    g->n_points = n;
    g->vol = (int64_t)prm->dims[0] * prm->dims[1] * prm->dims[2];
    SGN_REQUIRE(prm->dims[0] > 0 && prm->dims[1] > 0 && prm->dims[2] > 0, "grid dims must be positive");
    SGN_REQUIRE(g->vol < (int64_t)INT_MAX, "grid volume must fit int32");
    SGN_REQUIRE(n >= 0 && n < (int64_t)INT_MAX, "point count must fit int32");
    SGN_REQUIRE(prm->max_o > 0 && prm->P > 0, "max_o and P must be positive");
    GridGeom geo{prm->shift[0], prm->shift[1], prm->shift[2], prm->vs[0], prm->vs[1], prm->vs[2],
                 prm->dims[0], prm->dims[1], prm->dims[2]};

    if (dalloc(&g->vox, g->vol, &g->device_bytes)) return -1;
    TmpBufs tmp;
    int32_t *key, *flag, *rank;
    int64_t *d_total;
    if (tmp.get(&key, n) || tmp.get(&flag, n) || tmp.get(&rank, n) || tmp.get(&d_total, 2)) return -1;

    // 1. voxel key per point, first point per voxel (vox used as scratch)
    SGN_CHECK_HIP(hipMemsetD32Async((hipDeviceptr_t)g->vox, INT_MAX, g->vol, st));
    if (n > 0) {
        hipLaunchKernelGGL(k_point_keys, dim3(blocks_for(n)), dim3(TPB), 0, st, d_points, n, geo, key, g->vox);
        hipLaunchKernelGGL(k_is_first, dim3(blocks_for(n)), dim3(TPB), 0, st, key, g->vox, n, flag);
    }
    // 2. claim rank = exclusive scan of first-point flags
    size_t tb = 0;
    void *tstore = nullptr;
    SGN_CHECK_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, flag, rank, (int)n, st));
    if (tmp.get((char **)&tstore, (int64_t)tb)) return -1;
    if (n > 0) {
        SGN_CHECK_HIP(hipcub::DeviceScan::ExclusiveSum(tstore, tb, flag, rank, (int)n, st));
    }
    hipLaunchKernelGGL(k_total, dim3(1), dim3(64), 0, st, rank, flag, n, d_total);
    int64_t n_claimed = 0;
    SGN_CHECK_HIP(hipMemcpyAsync(&n_claimed, d_total, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    SGN_CHECK_HIP(hipStreamSynchronize(st));
    g->n_claimed = n_claimed;
    g->n_slots = n_claimed < prm->max_o ? n_claimed : prm->max_o;
    const int64_t ns = g->n_slots;

    // 3. slots (claim_occ + reservoir), dense map, neighbourhood flags
    int32_t *slot_vox;
    unsigned long long *slot_win;
    if (tmp.get(&slot_vox, ns) || tmp.get(&slot_win, ns)) return -1;
    SGN_CHECK_HIP(hipMemsetAsync(slot_win, 0, sizeof(unsigned long long) * (size_t)(ns > 0 ? ns : 1), st));
    if (n > 0)
        hipLaunchKernelGGL(k_assign_slots, dim3(blocks_for(n)), dim3(TPB), 0, st, key, flag, rank, n,
                           prm->max_o, prm->seed, slot_vox, slot_win);
    SGN_CHECK_HIP(hipMemsetD32Async((hipDeviceptr_t)g->vox, (int)VOX_UNFLAGGED, g->vol, st));
    if (ns > 0) {
        hipLaunchKernelGGL(k_map_slots, dim3(blocks_for(ns)), dim3(TPB), 0, st, slot_vox, slot_win, ns, g->vox);
        hipLaunchKernelGGL(k_flag, dim3(blocks_for(ns)), dim3(TPB), 0, st, slot_vox, ns, geo,
                           make_int3(prm->query[0], prm->query[1], prm->query[2]), g->vox);
    }

    // 4. per-slot point lists in point-index order (stable radix sort by slot)
    uint32_t *pslot, *skey;
    int32_t *pid, *sval, *seg_start, *seg_end, *resv;
    if (tmp.get(&pslot, n) || tmp.get(&skey, n) || tmp.get(&pid, n) || tmp.get(&sval, n) ||
        tmp.get(&seg_start, ns) || tmp.get(&seg_end, ns) || tmp.get(&resv, ns * prm->P))
        return -1;
    if (dalloc(&g->occ_start, ns, &g->device_bytes) || dalloc(&g->occ_kept, ns, &g->device_bytes) ||
        dalloc(&g->occ_routed, ns, &g->device_bytes) || dalloc(&g->occ_sc, ns, &g->device_bytes))
        return -1;
    int end_bit = 1;
    while (end_bit < 32 && ((uint64_t)1 << end_bit) <= (uint64_t)ns) ++end_bit;
    if (n > 0) {
        hipLaunchKernelGGL(k_point_slot, dim3(blocks_for(n)), dim3(TPB), 0, st, key, g->vox, n,
                           (int32_t)ns, prm->fix_occ0, pslot, pid);
        size_t sb = 0;
        SGN_CHECK_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, sb, pslot, skey, pid, sval, (int)n, 0, end_bit, st));
        void *sstore;
        if (tmp.get((char **)&sstore, (int64_t)sb)) return -1;
        SGN_CHECK_HIP(hipcub::DeviceRadixSort::SortPairs(sstore, sb, pslot, skey, pid, sval, (int)n, 0, end_bit, st));
    }
    SGN_CHECK_HIP(hipMemsetAsync(seg_start, 0, sizeof(int32_t) * (size_t)(ns > 0 ? ns : 1), st));
    SGN_CHECK_HIP(hipMemsetAsync(seg_end, 0, sizeof(int32_t) * (size_t)(ns > 0 ? ns : 1), st));
    SGN_CHECK_HIP(hipMemsetD32Async((hipDeviceptr_t)resv, -1, (size_t)(ns > 0 ? ns : 1) * prm->P, st));
    if (n > 0) {
        hipLaunchKernelGGL(k_segments, dim3(blocks_for(n)), dim3(TPB), 0, st, skey, n, (uint32_t)ns, seg_start, seg_end);
        hipLaunchKernelGGL(k_reservoir, dim3(blocks_for(n)), dim3(TPB), 0, st, skey, sval, n, (uint32_t)ns,
                           seg_start, prm->P, prm->seed, resv);
    }
    if (ns > 0)
        hipLaunchKernelGGL(k_counts, dim3(blocks_for(ns)), dim3(TPB), 0, st, seg_start, seg_end, ns,
                           prm->P, g->occ_routed, g->occ_kept);
    size_t tb2 = 0;
    SGN_CHECK_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, g->occ_kept, g->occ_start, (int)ns, st));
    void *tstore2;
    if (tmp.get((char **)&tstore2, (int64_t)tb2)) return -1;
    if (ns > 0) SGN_CHECK_HIP(hipcub::DeviceScan::ExclusiveSum(tstore2, tb2, g->occ_kept, g->occ_start, (int)ns, st));
    hipLaunchKernelGGL(k_total, dim3(1), dim3(64), 0, st, g->occ_start, g->occ_kept, ns, d_total + 1);
    if (ns > 0)
        hipLaunchKernelGGL(k_interleave_sc, dim3(blocks_for(ns)), dim3(TPB), 0, st, g->occ_start, g->occ_kept, ns,
                           g->occ_sc);
    int64_t n_listed = 0;
    SGN_CHECK_HIP(hipMemcpyAsync(&n_listed, d_total + 1, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    SGN_CHECK_HIP(hipStreamSynchronize(st));
    g->n_listed = n_listed;
    if (dalloc(&g->cell_pts, n_listed, &g->device_bytes)) return -1;
    if (n > 0)
        hipLaunchKernelGGL(k_emit_points, dim3(blocks_for(n)), dim3(TPB), 0, st, skey, sval, n, (uint32_t)ns,
                           seg_start, resv, g->occ_start, prm->P, d_points, g->cell_pts);
    SGN_CHECK_HIP(hipGetLastError());
    SGN_CHECK_HIP(hipStreamSynchronize(st));  // temporaries are freed on return
    return 0;
}

}  // namespace sgn

extern "C" {

int sgn_grid_build(const float *d_points, int64_t n_points, const sgn_grid_params *params,
                   sgn_stream_t stream, sgn_grid **out_grid) {
    SGN_REQUIRE(params != nullptr && out_grid != nullptr, "null params/out_grid");
    SGN_REQUIRE(n_points == 0 || d_points != nullptr, "null points");
    sgn_grid *g = new sgn_grid();
    int rc = sgn::grid_build_impl(d_points, n_points, params, sgn::as_stream(stream), g);
    if (rc != 0) {
        sgn_grid_free(g);
        *out_grid = nullptr;
        return rc;
    }
    *out_grid = g;
    return 0;
}

int sgn_grid_free(sgn_grid *g) {
    if (!g) return 0;
    (void)hipFree(g->vox);
    (void)hipFree(g->occ_start);
    (void)hipFree(g->occ_kept);
    (void)hipFree(g->occ_routed);
    (void)hipFree(g->cell_pts);
    (void)hipFree(g->occ_sc);
    delete g;
    return 0;
}

int sgn_grid_get_info(const sgn_grid *g, sgn_grid_info *out) {
    SGN_REQUIRE(g && out, "null grid/out");
    out->n_points = g->n_points;
    out->n_claimed = g->n_claimed;
    out->n_slots = g->n_slots;
    out->n_listed = g->n_listed;
    out->volume = g->vol;
    out->device_bytes = g->device_bytes;
    return 0;
}

int sgn_grid_export(const sgn_grid *g, int32_t *d_coor_occ, int32_t *d_coor_2_occ,
                    int32_t *d_occ_numpnts, int32_t *d_occ_2_pnts, sgn_stream_t stream) {
    SGN_REQUIRE(g, "null grid");
    hipStream_t st = sgn::as_stream(stream);
    if (d_coor_occ || d_coor_2_occ)
        hipLaunchKernelGGL(sgn::k_export_grid, dim3(sgn::blocks_for(g->vol)), dim3(sgn::TPB), 0, st,
                           g->vox, g->vol, d_coor_occ, d_coor_2_occ);
    if (d_occ_numpnts || d_occ_2_pnts)
        hipLaunchKernelGGL(sgn::k_export_lists, dim3(sgn::blocks_for(g->p.max_o)), dim3(sgn::TPB), 0, st,
                           g->occ_start, g->occ_kept, g->occ_routed, g->cell_pts, g->n_slots,
                           g->p.max_o, g->p.P, d_occ_numpnts, d_occ_2_pnts);
    SGN_CHECK_HIP(hipGetLastError());
    return 0;
}

}  // extern "C"
