// sgn_common.h -- shared device helpers for libsgn_hip.so (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/sgn_hip.h"

namespace sgn {

// ---- error plumbing (thread-local message, negative return codes) --------
void set_error(const std::string &msg);
const char *get_error();

#define SGN_CHECK_HIP(expr)                                                             \
    do {                                                                                \
        hipError_t _e = (expr);                                                         \
        if (_e != hipSuccess) {                                                         \
            ::sgn::set_error(std::string(#expr) + ": " + hipGetErrorString(_e) + " @ " + \
                             __FILE__ + ":" + std::to_string(__LINE__));                \
            return -1;                                                                  \
        }                                                                               \
    } while (0)

#define SGN_REQUIRE(cond, msg)                                          \
    do {                                                                \
        if (!(cond)) {                                                  \
            ::sgn::set_error(std::string("invalid argument: ") + (msg)); \
            return -2;                                                  \
        }                                                               \
    } while (0)

inline hipStream_t as_stream(sgn_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// ---- parity-mode reservoir RNG (identical to oracle/query_ref.c) ----------
__host__ __device__ inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
// u in (0, 1], 24-bit resolution (curand_uniform's range, worldcoords.py:315)
__host__ __device__ inline float uniform01(uint64_t seed, uint64_t stream, uint64_t i) {
    uint64_t h = splitmix64(seed ^ splitmix64(stream * 0x2545F4914F6CDD1Dull + i));
    uint32_t b = (uint32_t)(h >> 40);
    return (float)(b + 1u) * (1.0f / 16777216.0f);
}

// (int) floor((p - shift) / vs), every op IEEE-rounded (worldcoords.py:288-290)
__device__ __forceinline__ int vox_coord(float p, float shift, float vs) {
    return (int)floorf(__fdiv_rn(__fsub_rn(p, shift), vs));
}

// raypos = campos + raydir * t, two roundings (diff_ray_marching.py:387)
__device__ __forceinline__ float ray_coord(float c, float d, float t) {
    return __fadd_rn(c, __fmul_rn(d, t));
}

struct GridView {
    const int32_t *vox;     // [vol]: >=0 occupancy slot, -1 flagged empty, -2 unflagged
    const int32_t *start;   // [n_slots] first kept point of the slot in pts
    const int32_t *cnt;     // [n_slots] kept points (min(P, routed))
    const float4 *pts;      // [n_listed] {x, y, z, bits(pidx)}
    const int2 *sc;         // [n_slots] {start, cnt}: one 8-B load per occupied voxel (k_knn27)
    float shift[3];
    float vs[3];
    int dims[3];
    int kernel0;            // kernel_size[0]
};

constexpr int32_t VOX_UNFLAGGED = -2;
constexpr int32_t VOX_FLAGGED = -1;

}  // namespace sgn

struct sgn_grid {
    sgn_grid_params p;
    int64_t vol = 0;
    int64_t n_points = 0, n_claimed = 0, n_slots = 0, n_listed = 0;
    int32_t *vox = nullptr;        // [vol]
    int32_t *occ_start = nullptr;  // [n_slots]
    int32_t *occ_kept = nullptr;   // [n_slots] min(P, routed)
    int32_t *occ_routed = nullptr; // [n_slots] routed points (reference occ_numpnts)
    float4 *cell_pts = nullptr;    // [n_listed]
    int2 *occ_sc = nullptr;        // [n_slots] {occ_start, occ_kept} interleaved
    int64_t device_bytes = 0;
    sgn::GridView view() const {
        sgn::GridView g;
        g.vox = vox; g.start = occ_start; g.cnt = occ_kept; g.pts = cell_pts; g.sc = occ_sc;
        for (int a = 0; a < 3; ++a) { g.shift[a] = p.shift[a]; g.vs[a] = p.vs[a]; g.dims[a] = p.dims[a]; }
        g.kernel0 = p.kernel[0];
        return g;
    }
};
