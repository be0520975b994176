/* oracle/query_ref.h -- TEST INFRASTRUCTURE ONLY (see query_ref.c header). */
#ifndef SGNREF_QUERY_REF_H
#define SGNREF_QUERY_REF_H
#include <stdint.h>

typedef struct {
    float shift[3];   /* d_coord_shift  = ranges[:3]               (:793) */
    float vs[3];      /* scaled voxel size (0.016 at ScanNet)      (:73)  */
    int dims[3];      /* scaled_vdim                               (:86)  */
    int kernel[3];    /* kernel_size: layered search radius        (:635) */
    int query[3];     /* query_size: coor_occ neighbourhood        (:797) */
    int max_o;
    int P;
    int K;
    int SR;
    float r2;         /* np.float32(radius_limit ** 2)             (:894) */
    uint64_t seed;    /* parity-mode reservoir seed                       */
    int fix_occ0;     /* 0 = reproduce `voxel_idx > 0` (:395)             */
} sgnref_params;

void sgnref_set_threads(int n);
float sgnref_uniform(uint64_t seed, uint64_t stream, uint64_t i);
int64_t sgnref_grid_volume(const sgnref_params *p);
int64_t sgnref_grid_build(const float *pts, int64_t n, const sgnref_params *p, int32_t *coor_occ,
                          int32_t *coor_2_occ, int32_t *occ_numpnts, int32_t *occ_2_pnts,
                          int32_t *occ_2_coor);
void sgnref_march(const sgnref_params *p, const int32_t *coor_occ, const float *campos,
                  const float *raydir, int64_t R, const float *t_table, int D, int per_ray_t,
                  int32_t *ray_ns, int32_t *ray_d);
int sgnref_knn_one(const sgnref_params *p, const float *pts, const int32_t *coor_2_occ,
                   const int32_t *occ_numpnts, const int32_t *occ_2_pnts, const float center[3],
                   int32_t *out_pidx, const int32_t *labels, int center_label, uint64_t seconds);
void sgnref_query(const sgnref_params *p, const float *pts, const int32_t *coor_occ,
                  const int32_t *coor_2_occ, const int32_t *occ_numpnts, const int32_t *occ_2_pnts,
                  const float *campos, const float *raydir, int64_t R, const float *t_table, int D,
                  int per_ray_t, int32_t *ray_ns, int32_t *ray_d, int32_t *pidx, float *loc_w,
                  const int32_t *point_labels, const int32_t *ray_labels, uint64_t seconds);
#endif
