/*
 * sgn_hip.h -- C ABI of libsgn_hip.so, the MI355X (gfx950) implementation of
 * the SG-NeRF / Point-NeRF per-ray rendering hot path:
 *
 *     neural-point grid  ->  ray march + shading-sample selection + layered kNN
 *     ->  per-neighbour aggregator MLP (MFMA)  ->  colour MLP  ->  alpha composite
 *
 * Every pointer named d_* is a DEVICE pointer owned by the caller (torch
 * tensors on the Python side); the library never allocates on the per-frame
 * path (sgn_query / sgn_aggregate / sgn_composite).  Only sgn_grid_build
 * allocates (once per point-cloud version) and sgn_grid_free releases.
 * Every call takes an explicit hipStream_t and is asynchronous w.r.t. the host
 * unless stated.  Return value: 0 on success, < 0 on error; sgn_last_error()
 * gives a message for the calling thread.
 *
 * Reference interfaces replaced (file:line in Quyans/SG-NeRF):
 *   sgn_grid_build   <- lighting_fast_querier.build_occ_vox
 *                       models/neural_points/query_point_indices_worldcoords.py:706-778
 *                       (claim_occ :265, map_coor2occ :328, fill_occ2pnts :365)
 *                       -- hoisted out of the per-chunk call (:797) and cached.
 *   sgn_query        <- lighting_fast_querier.query_grid_point_index :782-954
 *                       (mask_raypos :413, get_shadingloc :439,
 *                        query_neigh_along_ray_layered[_semantic_guidance] :594 / :489)
 *   sgn_aggregate    <- NeuralPoints.forward gather  neural_points.py:942-988
 *                       + PointAggregator.forward / viewmlp
 *                       models/aggregators/point_aggregators.py:868-959 / :561-786
 *   sgn_composite    <- NeuralPointsRayMarching.forward ray_dist + ray_march + fill_invalid
 *                       models/neural_points_volumetric_model.py:569-631, :158-195
 *                       models/rendering/diff_ray_marching.py:509-555
 */
#ifndef SGN_HIP_H
#define SGN_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void *sgn_stream_t; /* hipStream_t (torch.cuda.current_stream().cuda_stream) */
typedef struct sgn_grid sgn_grid; /* opaque, device-resident voxel grid of one point cloud */

#define SGN_ABI_VERSION 20

/* ---- grid ------------------------------------------------------------- */

typedef struct {
    float shift[3];      /* ranges[:3] after padding, fp32          (worldcoords.py:79,793) */
    float vs[3];         /* scaled voxel size = fl32(vsize*vscale)   (:73) */
    int32_t dims[3];     /* scaled_vdim                              (:86) */
    int32_t kernel[3];   /* kernel_size: layered kNN search extent   (:635) */
    int32_t query[3];    /* query_size: occupancy-flag neighbourhood (:797) */
    int32_t max_o;       /* max occupied voxels                      (:307) */
    int32_t P;           /* max points per voxel                     (:398) */
    int32_t fix_occ0;    /* 0 = reproduce `voxel_idx > 0` (:395); 1 = fixed */
    uint64_t seed;       /* reservoir seed (reference: wall clock)   (:314,:402) */
} sgn_grid_params;

typedef struct {
    int64_t n_points;    /* points given to the build */
    int64_t n_claimed;   /* occupied voxels (= reference occ_idx, may exceed max_o) */
    int64_t n_slots;     /* min(n_claimed, max_o) */
    int64_t n_listed;    /* points kept in per-voxel lists (sum of min(P, count)) */
    int64_t volume;      /* dims[0]*dims[1]*dims[2] */
    int64_t device_bytes;
} sgn_grid_info;

/* Builds the grid.  Synchronises `stream` twice (sizes read back). */
int sgn_grid_build(const float *d_points, int64_t n_points, const sgn_grid_params *params,
                   sgn_stream_t stream, sgn_grid **out_grid);
int sgn_grid_free(sgn_grid *grid);
int sgn_grid_get_info(const sgn_grid *grid, sgn_grid_info *out);
/* Writes the reference's own grid structures (for parity tests):
 * coor_occ/coor_2_occ int32[volume], occ_numpnts int32[max_o], occ_2_pnts int32[max_o*P]. */
int sgn_grid_export(const sgn_grid *grid, int32_t *d_coor_occ, int32_t *d_coor_2_occ,
                    int32_t *d_occ_numpnts, int32_t *d_occ_2_pnts, sgn_stream_t stream);

/* ---- query ------------------------------------------------------------ */

typedef struct {
    int32_t SR;          /* max shading samples per ray  (<= 128) */
    int32_t K;           /* neighbours per sample        (<= 16)  */
    int32_t D;           /* candidate depths per ray (z_depth_dim) */
    int32_t per_ray_t;   /* 0: t_table is [D]; 1: t_table is [R, D] (jittered training rays) */
    float r2;            /* np.float32(radius_limit ** 2); 0 disables the radius test */
    int32_t dense_out;   /* 0: pidx indexed by sample; 1: by ray*SR+slot (reference layout) */
    int32_t semantic;    /* 1: semantic-guidance filter (:489-591) */
    uint64_t seconds;    /* wall-clock value the semantic filter reads (:553) */
    int32_t count_traffic; /* 1: fill counters[2..3] (bench byte model; slower kNN) */
} sgn_query_params;

/* Sample-major outputs of one query call (all device, caller-allocated,
 * capacity R*SR samples unless noted):
 *   ray_ns    int32[R]        selected shading samples per ray (<= SR)
 *   ray_soff  int32[R]        exclusive prefix sum of ray_ns (first sample id of the ray)
 *   samp_ray  int32[S]        ray of each sample
 *   samp_d    int32[S]        candidate depth index of each sample
 *   samp_locw float[S*3]      sample position (world)
 *   samp_nnb  int32[S]        valid neighbours of the sample (0..K)
 *   pidx      int32[S*K] or [R*SR*K] (dense_out; caller pre-fills -1)
 *   work      int32[S]        ids of samples with samp_nnb > 0 (unordered)
 *   counters  int32[4]        [0] = S (total samples), [1] = work items; with count_traffic:
 *                             [2] voxel words and [3] (uint32) candidate points the kNN read
 */
typedef struct {
    int32_t *ray_ns, *ray_soff, *samp_ray, *samp_d, *samp_nnb, *pidx, *work, *counters;
    float *samp_locw;
} sgn_query_out;

/* Training-mode depth table (is_train: jittered linear depths), replacing the torch op sequence of
 * near_far_linear_ray_generation (models/rendering/diff_ray_marching.py:349-393) after its
 * torch.rand: d_rnd float[R*D] uniform [0, 1) in, d_t float[R*D] segment mid-point depths out
 * (the reference's middle_point_ts; sgn_query's per_ray_t = 1 table). */
int sgn_depth_table_jitter(float near, float far, int32_t D, float jitter, int64_t R, const float *d_rnd, float *d_t,
                           sgn_stream_t stream);

size_t sgn_query_workspace_bytes(int64_t R);
int sgn_query(const sgn_grid *grid, const sgn_query_params *qp, const float *d_campos,
              const float *d_raydir, int64_t R, const float *d_t_table,
              const int32_t *d_point_labels, const int32_t *d_ray_labels,
              const sgn_query_out *out, void *d_workspace, size_t workspace_bytes,
              sgn_stream_t stream);

/* ---- aggregator (per-neighbour MLP + K-blend, colour MLP) -------------- */

/* Size in bytes of the packed fp16 weight blob for the ScanNet-layout viewmlp
 * (block1 284->256->256, block3 263->256->256, alpha 256->1, colour 280->128x3->3). */
size_t sgn_mlp_packed_bytes(void);
/* Packs fp32 nn.Linear weights (row-major [out][in]) + biases into the
 * MFMA fragment-major fp16 layout.  Host pointers in, device pointer out
 * (synchronous copy). Order of `w`/`b`: block1.0, block1.2, block3.0,
 * block3.2, alpha_branch.0, color_branch.0, .2, .4, .6 (9 layers). */
int sgn_mlp_pack(const float *const *w, const float *const *b, void *d_packed,
                 sgn_stream_t stream);

typedef struct {
    /* point tables, row = neural point index */
    const float *xyz;        /* [N,3]  */
    const float *embedding;  /* [N,32] */
    const float *color;      /* [N,3]  */
    const float *dir;        /* [N,3]  */
    const float *conf;       /* [N]    */
    int64_t n_points;
    /* camera */
    const float *campos;     /* [3] */
    const float *camrotc2w;  /* [3,3] row-major */
    const float *raydir;     /* [rows of samp_ray's index space, 3]: per-ray view directions */
    /* optional precomputed camera-space ("pers") coordinates -- the compatibility path
     * (PointAggregator.forward on pre-gathered tensors) receives them from the caller;
     * NULL = compute from xyz and the camera (neural_points.py:838-850).  campos and
     * camrotc2w must still be valid pointers (unused values when pers is given). */
    const float *pers;       /* [N,3] or NULL */
    const float *samp_pers;  /* [S,3] or NULL (with pers) */
} sgn_point_tables;

/* out_feat: float4[S] = [alpha_s, r, g, b] for every work-list sample (samples
 * without a valid neighbour are not written; the composite ignores them).
 * Optional (NULL to skip): out_blend float[S*K] = normalised weight * conf
 * (the reference's `weight * conf_coefficient`), out_wnorm float[S*K] = normalised
 * weight alone (the reference's `weight` output, point_aggregators.py:946-958). */
size_t sgn_aggregate_workspace_bytes(int64_t S);
/* stages: bit 0 = per-neighbour MLP + K-blend (writes alpha), bit 1 = colour MLP (rgb). */
int sgn_aggregate(const sgn_point_tables *pt, const sgn_query_out *q, int64_t S_capacity,
                  int32_t K, const void *d_packed_mlp, float *d_out_feat, float *d_out_blend,
                  float *d_out_wnorm, void *d_workspace, size_t workspace_bytes, int32_t stages,
                  sgn_stream_t stream);

/* ---- split block1.0 (per-point projection) ----------------------------------
 * block1.0's inputs [feat | PE(feat) | PE(dists)] (point_aggregators.py:594-621) are per
 * point for the first 224 of 284 channels: sgn_point_project computes
 * P[p] = W0a [feat_p | PE(feat_p)] + b0 for every point once per frame (fp16,
 * sgn_point_proj_bytes(N)), and sgn_aggregate_sg(d_point_proj = P) then multiplies only the
 * 60 PE(dists) channels per (sample, neighbour) row.  Same sums, regrouped. */
size_t sgn_point_proj_bytes(int64_t n_points);
int sgn_point_project(const sgn_point_tables *pt, const void *d_packed_mlp, void *d_proj,
                      sgn_stream_t stream);
/* sgn_point_project for the points d_idx[0 .. *d_count) only (ABI 20; int32 indices < n_points, int64
 * device count, e.g. sgn_frame_points' list): the f16 renderer projects the points a frame's
 * samples name.  The other points' P rows are left as they are. */
int sgn_point_project_subset(const sgn_point_tables *pt, const void *d_packed, const int32_t *d_idx,
                             const int64_t *d_count, void *d_proj, sgn_stream_t stream);
/* Byte offsets inside the packed blob: 0 = fp32 section, 1 = split block1.0 sections,
 * 2 = end of the base blob (sgn_mlp_packed_bytes). */
size_t sgn_mlp_section(int32_t which);

/* ---- SG-NeRF variant: block2_bpnet (shading_feature_mlp_layer2_bpnet) ---
 * Replaces PointAggregator.block2_bpnet (models/aggregators/point_aggregators.py:345-354,
 * applied at :629-636) and the BPNet-embedding gather of NeuralPoints.forward
 * (models/neural_points/neural_points.py:970-972): Linear(256 + bpnet_dim -> 256) + LReLU
 * on [block1 output | bpnet_points_embedding[pidx]] between block1 and block3.
 * Supported: bpnet_layers 0 (= the base functions above), or 1 with bpnet_dim 96
 * (predict_semantic = 1, semantic_guidance = 1) or 0 (predict_semantic = 0).
 * Weight order: the 9 base layers, then block2_bpnet.0 ([256][256 + bpnet_dim]). */
size_t sgn_mlp_packed_bytes_sg(int32_t bpnet_layers, int32_t bpnet_dim); /* 0: unsupported */
int sgn_mlp_pack_sg(int32_t bpnet_layers, int32_t bpnet_dim, const float *const *w,
                    const float *const *b, void *d_packed, sgn_stream_t stream);
/* bpnet_points_embedding f32[N, 96] -> fp16 [N, 96] (the table sgn_aggregate_sg gathers;
 * the reference holds it detached, neural_points.py:662). 16-byte aligned pointers. */
int sgn_bpnet_pack(const float *d_embedding, int64_t n_points, int32_t bpnet_dim, void *d_out_f16,
                   sgn_stream_t stream);
int sgn_aggregate_sg(int32_t bpnet_layers, int32_t bpnet_dim, const void *d_bpnet_f16,
                     const void *d_point_proj, const sgn_point_tables *pt, const sgn_query_out *q, int64_t S_capacity,
                     int32_t K, const void *d_packed_mlp, float *d_out_feat, float *d_out_blend,
                     float *d_out_wnorm, void *d_workspace, size_t workspace_bytes,
                     int32_t stages, sgn_stream_t stream);

/* ---- fp32-faithful aggregator (the reference's arithmetic) -------------------------
 * Same operator as sgn_point_project + sgn_aggregate (PointAggregator.forward / viewmlp,
 * models/aggregators/point_aggregators.py:868-959, :561-786, at the reference's fp32 precision):
 * every fp32 product w x of the nn.Linear layers is carried as three fp16 MFMA products
 * 2^-s (w_hi x_hi + w_hi x_lo + w_lo x_hi) with fp32 accumulation (w pre-scaled by a per-layer
 * power of two 2^s; x = x_hi + x_lo), positional encodings from accurate sinf/cosf.  The results
 * agree with an fp32 evaluation to a few fp32 ulps of sum |w x| per layer.  Hidden activations
 * must stay inside fp16 range (|x| < 65504): one outside it makes the sample's decoded features
 * non-finite, which the colour stage records in a flag of the workspace (never returned silently:
 * sgn_aggregate_check_f32 reports it).  bpnet_layers / bpnet_dim select the SG-NeRF
 * block2_bpnet variant as in sgn_mlp_pack_sg (0/0 = base ScanNet viewmlp).
 *   sgn_mlp_pack_f32        : 9 (+ block2_bpnet.0) layers as sgn_mlp_pack_sg -> blob of
 *                             sgn_mlp_packed_bytes_f32(bpnet_layers, bpnet_dim) bytes (0: unsupported)
 *   sgn_point_project_f32   : P[p] fp32, the block1.0 per-point part, followed by a packed 64-B
 *                             record per point (xyz, conf, colour, dir) that the row kernel gathers
 *                             as one cache line (sgn_point_proj_bytes_f32(N) bytes; pt->xyz, color,
 *                             dir, conf and embedding required; opaque to the caller)
 *   sgn_aggregate_f32       : as sgn_aggregate_sg (same outputs, stages bits), d_point_proj required;
 *                             d_bpnet = fp32 [N, 96] BPNet point embedding when bpnet_dim = 96;
 *                             workspace sgn_aggregate_workspace_bytes_f32(S) (fp32 blended features
 *                             and the row kernel's paired-sample tables; opaque to the caller);
 *                             reads q->samp_nnb (valid neighbours are a prefix of each sample's K
 *                             slots, as sgn_query writes them); optional d_out_blend / d_out_wnorm are
 *                             zeroed by stage 1 before the valid rows are written
 *   sgn_aggregate_check_f32 : synchronises `stream` and returns -1 (sgn_last_error says why) when a
 *                             sample of the last colour stage run on this workspace had non-finite
 *                             decoded features (an activation outside fp16 range); 0 otherwise
 *   sgn_aggregate_flag_offset_f32 : byte offset of that int32 flag inside the workspace (for a
 *                             caller that reads it asynchronously, e.g. one frame later)
 *   sgn_aggregate_fs_offset_f32 (ABI 12) : byte offset inside the workspace of the blended features
 *                             f_s that stage 1 leaves for stage 2 -- fp32 [S_capacity][256], item i's
 *                             row at offset + 1024 i (a training step reads them) -- or -1 when a
 *                             workspace of workspace_bytes does not hold every item's row
 *   sgn_mlp_pack_f32_host   : sgn_mlp_pack_f32 into host memory (no device call; checkers)
 * 16-byte aligned device buffers. */
size_t sgn_mlp_packed_bytes_f32(int32_t bpnet_layers, int32_t bpnet_dim);
int sgn_mlp_pack_f32(int32_t bpnet_layers, int32_t bpnet_dim, const float *const *w, const float *const *b,
                     void *d_packed, sgn_stream_t stream);
int sgn_mlp_pack_f32_host(int32_t bpnet_layers, int32_t bpnet_dim, const float *const *w, const float *const *b,
                          void *h_packed);
size_t sgn_point_proj_bytes_f32(int64_t n_points);
int sgn_point_project_f32(const sgn_point_tables *pt, const void *d_packed_mlp, void *d_proj, sgn_stream_t stream);
size_t sgn_aggregate_workspace_bytes_f32(int64_t S);
int sgn_aggregate_f32(int32_t bpnet_layers, int32_t bpnet_dim, const float *d_bpnet, const void *d_point_proj,
                      const sgn_point_tables *pt, const sgn_query_out *q, int64_t S_capacity, int32_t K,
                      const void *d_packed_mlp, float *d_out_feat, float *d_out_blend, float *d_out_wnorm,
                      void *d_workspace, size_t workspace_bytes, int32_t stages, sgn_stream_t stream);
int sgn_aggregate_check_f32(const void *d_workspace, size_t workspace_bytes, sgn_stream_t stream);
size_t sgn_aggregate_flag_offset_f32(size_t workspace_bytes);
int64_t sgn_aggregate_fs_offset_f32(size_t workspace_bytes, int64_t S_capacity);

/* ---- plain-fp32 aggregator (ABI 16): the f32 mode's range fallback -----------------------
 * The same operator as sgn_aggregate_f32 (stages 1 + 2: alpha and colour of every work item,
 * optional blend / wnorm), every nn.Linear as v_mfma_f32_16x16x4_f32 on fp32 operands (exact fp32
 * products, fp32 sums) with the weights as the checkpoint holds them: no fp16 operand, so no range
 * limit below fp32's.  For frames whose activations leave fp16 range (sgn_aggregate_check_f32 /
 * the flag at sgn_aggregate_flag_offset_f32): the host re-runs them here instead of failing.  About
 * 1/5 of the split path's rate.  Needs no point projection (block1.0 is computed per row in full).
 *   sgn_mlp_pack_exact      : the 9 (+ block2_bpnet.0) layers in sgn_mlp_pack_f32's order -> fp32 blob of
 *                             sgn_mlp_packed_bytes_exact(bpnet_layers, bpnet_dim) bytes (W^T per layer)
 *   sgn_aggregate_exact     : workspace >= 1 KiB (1 KiB per work item of a chunk; a workspace holding
 *                             S_capacity items runs one chunk); d_bpnet fp32 [N, 96] when bpnet_dim = 96;
 *                             pt->pers / samp_pers optional as for sgn_aggregate_f32 */
size_t sgn_mlp_packed_bytes_exact(int32_t bpnet_layers, int32_t bpnet_dim);
int sgn_mlp_pack_exact(int32_t bpnet_layers, int32_t bpnet_dim, const float *const *w, const float *const *b,
                       void *d_packed, sgn_stream_t stream);
int sgn_aggregate_exact(int32_t bpnet_layers, int32_t bpnet_dim, const float *d_bpnet, const sgn_point_tables *pt,
                        const sgn_query_out *q, int64_t S_capacity, int32_t K, const void *d_packed_exact,
                        float *d_out_feat, float *d_out_blend, float *d_out_wnorm, void *d_workspace,
                        size_t workspace_bytes, sgn_stream_t stream);

/* sgn_point_project_f32 for the points d_idx[0 .. *d_count) only (int32 indices < n_points; the
 * count is a device int64): a training step re-projects the rows its rays touch after each weight
 * update instead of all N.  The other points' P rows and records are left as they are. */
int sgn_point_project_f32_subset(const sgn_point_tables *pt, const void *d_packed, const int32_t *d_idx,
                                 const int64_t *d_count, void *d_proj, sgn_stream_t stream);
/* fp32-faithful training forward (SURVEY §8 f1 at the reference's arithmetic): stage 1 of
 * sgn_aggregate_f32 for the base viewmlp that also writes the pre-activations of block1.0, block1.2
 * and block3.0 (2^-s (W x + b), before LeakyReLU) as fp32 [S_capacity * K][256] at row s * K + k
 * (the row's pidx index; rows without a neighbour are left unwritten), or, with d_row_off
 * (sgn_train_lists), at the compact row d_row_off[s] + k.  The backward through them runs on
 * sgn_x3_gemm and the row kernels below (train_hip, f32 mode).
 *   sgn_mlp_layout_f32(0 / 1)   : bytes of the blob's fragment section / fp32 entries after it
 *   sgn_mlp_pack_index_f32      : the blob as index maps, for packing it on the device from a flat
 *                                 parameter: which 0 -> per fp16 element (layer << 20 | element)
 *                                 (| 1 << 30 for the lo part, -1 padding); which 1 -> per fp32 entry
 *                                 kind << 26 | layer << 20 | element (kinds: see mlp_x3.hip Y32Kind) */
int sgn_aggregate_train_fwd_f32(const void *d_point_proj, const sgn_point_tables *pt, const sgn_query_out *q,
                                int64_t S_capacity, int32_t K, const void *d_packed_mlp, float *d_out_feat,
                                float *d_z1, float *d_z2, float *d_z3, const int32_t *d_row_off, void *d_workspace,
                                size_t workspace_bytes, sgn_stream_t stream);
/* The same for SG-NeRF's block2_bpnet.0 (point_aggregators.py:345-354, :629-636; bpnet_layers 1,
 * bpnet_dim 0 or 96 with d_bpnet the fp32 [N][96] BPNet embedding): d_z2 gets block1.2's
 * pre-activations, d_zb block2_bpnet.0's (block3.0's input).  d_packed_mlp: the SG fp32 blob. */
int sgn_aggregate_train_fwd_f32_sg(int32_t bpnet_layers, int32_t bpnet_dim, const float *d_bpnet,
                                   const void *d_point_proj, const sgn_point_tables *pt, const sgn_query_out *q,
                                   int64_t S_capacity, int32_t K, const void *d_packed_mlp, float *d_out_feat,
                                   float *d_z1, float *d_z2, float *d_zb, float *d_z3, const int32_t *d_row_off,
                                   void *d_workspace, size_t workspace_bytes, sgn_stream_t stream);
int64_t sgn_mlp_layout_f32(int32_t which);
int sgn_mlp_pack_index_f32(int32_t bpnet_layers, int32_t bpnet_dim, int32_t which, int32_t *out, int64_t n);

/* ---- training: forward with saved activations + backward ---
 * Gradients of PointAggregator.forward / viewmlp (point_aggregators.py:868-959, :561-786)
 * and of the NeuralPoints gather (neural_points.py:942-988) -- the reference gets them from
 * torch autograd in optimize_parameters (base_rendering_model.py:534-664).  Base ScanNet
 * layout only (no block2_bpnet). Rows: row = 8 * item + k (item = work-list position). */
typedef struct {
    void *x0;   /* fp16 [rows][288] block1.0 inputs           */
    void *h1;   /* fp16 [rows][256] block1.2 inputs           */
    void *h2;   /* fp16 [rows][272] block3.0 inputs (| ext)   */
    void *h3;   /* fp16 [rows][256] block3.2 inputs           */
} sgn_agg_saved;
typedef struct {
    void *d4, *d3, *d2, *d1;  /* fp16 [rows][256] scaled d loss / d pre-activation of block3.2,
                                 block3.0, block1.2, block1.0 outputs (sgn_train_colmap 0 order) */
    void *h4;                 /* fp16 [rows][256] block3.2 outputs (same order) */
    float *dza;               /* [rows] scaled d loss / d alpha-branch logit */
} sgn_agg_deltas;
typedef struct {
    float *embedding, *color, *dir, *conf;  /* [N,32] [N,3] [N,3] [N]: accumulated (+=), unscaled */
} sgn_point_grads;

/* Stage 1 of sgn_aggregate in one launch (items [0, S_capacity)), saving per-row layer
 * inputs.  d_fs: fp16 [S_capacity][256] blended features (the colour MLP's input). */
int sgn_aggregate_train_fwd(const sgn_point_tables *pt, const sgn_query_out *q, int64_t S_capacity,
                            int32_t K, const void *d_packed_mlp, float *d_out_feat, void *d_fs,
                            const sgn_agg_saved *saved, sgn_stream_t stream);
/* Transposed-weight blob of block1.0, block1.2, block3.0, block3.2 (w[0..3] as in
 * sgn_mlp_pack), host in, device out (synchronous). */
size_t sgn_train_tblob_bytes(void);
int sgn_train_pack_t(const float *const *w, void *d_tblob, sgn_stream_t stream);
/* Index maps for packing ON THE DEVICE from a flat fp32 parameter vector (the 9 base layers
 * in sgn_mlp_pack order, each weight row-major then its bias): out[i] = flat index + 1, 0 =
 * zero.  sgn_mlp_pack_index: which 0 = fp16 fragment part (n = OFF_F32 / 2 elements),
 * 1 = fp32 section (n = 2056); sgn_train_pack_index: transposed blob (n = tblob_bytes / 2). */
int sgn_mlp_pack_index(int32_t which, int32_t *out, int64_t n);  /* which 2: split block1.0 sections */
int sgn_train_pack_index(int32_t *out, int64_t n);
/* Column maps of the saved/delta tiles to reference indices (-1 = padding):
 * which 0: [256] chain order -> unit, 1: [288] -> block1.0 input, 2: [272] -> block3.0 input. */
int sgn_train_colmap(int32_t which, int32_t *out, int32_t n);
/* Backward for n_items work items: d_dfs f32 [n_items][256], d_dalpha f32 [n_items] (d loss
 * w.r.t. the blended features / alpha), d_scale: device scalar loss scale.  K (ABI 15): neighbours
 * per sample of q->pidx, 1 .. 8, as in the forward. */
int sgn_aggregate_backward(const sgn_point_tables *pt, const sgn_query_out *q, int32_t n_items, int32_t K,
                           const void *d_packed_mlp, const void *d_tblob, const sgn_agg_saved *saved,
                           const float *d_dfs, const float *d_dalpha, const float *d_scale,
                           const sgn_agg_deltas *deltas, const sgn_point_grads *grads,
                           sgn_stream_t stream);

/* ---- training of the SG-NeRF variant (block2_bpnet, point_aggregators.py:345-354, :629-636) ----
 * Gradients of block2_bpnet.0 = Linear(256 + bpnet_dim -> 256) + LReLU between block1 and
 * block3, on the fp16 blob of sgn_mlp_pack_sg (bpnet_layers 1, bpnet_dim 0 or 96; 0 layers =
 * the base functions).  The forward additionally saves block2_bpnet's inputs h (d_h2b, fp16
 * [rows][256], chain order) and saved->h2 holds block3.0's inputs (block2_bpnet's output + the
 * colour / dir channels); the backward writes block2_bpnet's scaled deltas (d_db, fp16
 * [rows][256]) and deltas->d2 = block1.2's.  The BPNet embedding is a detached input
 * (neural_points.py:662): it gets no gradient.  The transposed blob gains block2_bpnet.0's
 * first 256 input columns (sgn_train_pack_t_sg, w[0..3] and w[4] = block2_bpnet.0's weight). */
int sgn_aggregate_train_fwd_sg(int32_t bpnet_layers, int32_t bpnet_dim, const void *d_bpnet_f16,
                               const sgn_point_tables *pt, const sgn_query_out *q, int64_t S_capacity, int32_t K,
                               const void *d_packed_mlp, float *d_out_feat, void *d_fs, const sgn_agg_saved *saved,
                               void *d_h2b, sgn_stream_t stream);
int sgn_aggregate_backward_sg(int32_t bpnet_layers, int32_t bpnet_dim, const sgn_point_tables *pt,
                              const sgn_query_out *q, int32_t n_items, int32_t K, const void *d_packed_mlp,
                              const void *d_tblob,
                              const sgn_agg_saved *saved, const void *d_h2b, const float *d_dfs, const float *d_dalpha,
                              const float *d_scale, const sgn_agg_deltas *deltas, void *d_db,
                              const sgn_point_grads *grads, sgn_stream_t stream);
int sgn_train_pack_t_sg(const float *const *w, int32_t bpnet_dim, void *d_tblob, sgn_stream_t stream);
/* Index maps over the SG flat vector (the 9 base layers, then block2_bpnet.0 weight and bias):
 * sgn_mlp_pack_index_sg which 3 = block2_bpnet fragments (n = (bias offset - OFF_WB) / 2 fp16
 * elements), 4 = its bias (n = 256 fp32); sgn_train_pack_index_sg = the transposed blob. */
int sgn_mlp_pack_index_sg(int32_t bpnet_layers, int32_t bpnet_dim, int32_t which, int32_t *out, int64_t n);
int sgn_train_pack_index_sg(int32_t bpnet_dim, int32_t *out, int64_t n);

/* ---- training: point-parameter Adam and bias-gradient column sums ------------------
 * Replaces torch.optim.Adam.step for the neural-point group (the reference's optimizer,
 * models/mvs_points_volumetric_model.py:100-108; no weight decay, no amsgrad): one fp32
 * tensor of n elements, state tensors exp_avg / exp_avg_sq as torch keeps them, step =
 * the 1-based step count after this update.  zero_grad != 0 also clears d_grad (the next
 * step's zero_grad).  All buffers 16-B aligned. */
int sgn_adam_step(float *d_param, float *d_grad, float *d_exp_avg, float *d_exp_avg_sq, int64_t n, double lr,
                  double beta1, double beta2, double eps, int64_t step, int32_t zero_grad, sgn_stream_t stream);
/* The same update for n_t <= 8 tensors of one parameter group (host arrays of device pointers and
 * element counts; one lr / step for all) in one launch. */
int sgn_adam_step_multi(int32_t n_t, float *const *d_param, float *const *d_grad, float *const *d_exp_avg,
                        float *const *d_exp_avg_sq, const int64_t *n, double lr, double beta1, double beta2, double eps,
                        int64_t step, int32_t zero_grad, sgn_stream_t stream);
/* Row-sparse exact Adam for n_t <= 4 tensors sharing a row index (the point group: embedding,
 * colour, dir, conf; row_width[t] elements per row, <= 64 in all; n_rows rows).  Dense Adam
 * updates every row every step; a step's gradient touches few, and an untouched row's update is
 * the zero-gradient recurrence.  d_last[r] (int32, n_rows, zero at step 0) is the step row r holds.
 * A launch brings each listed row from d_last[r] to `step`: it replays the missed steps at zero
 * gradient with their constants from d_sched ([step][2] fp32, (lr_k / bc1_k, sqrt(bc2_k)), written
 * by each apply launch for its step), and with apply != 0 takes step `step` itself with the
 * gradient buffer's value (zero on rows the step did not touch: that step's zero-gradient update;
 * zero_grad clears it).  The same fp32 operations as sgn_adam_step_multi, so a row equals the
 * dense update's bit for bit once brought forward: read a row only then (d_rows null: every row,
 * n_max = n_rows).  List 1: d_rows[0 .. n) with n = min(n_max, count_mul * *d_count) (d_count int32
 * or int64 on the device, or null: n = n_max), -1 and duplicate entries allowed; row0 != 0 adds row
 * 0 (the loss stage reads point 0's conf for empty slots); list 2 (optional): d_rows2[0 ..
 * min(n_max2, *d_count2)) (int64 device count), e.g. a previous launch's pend list.  d_claim (int32
 * n_rows, initialised to a value no launch uses as its tag, e.g. 0) takes each row once per launch
 * under `tag` (unique per launch, != 0);
 * d_ws: sgn_adam_rows_workspace_bytes(min(entries, n_rows)) bytes of scratch (entries = n_max +
 * n_max2 + row0).  d_pend (optional, with d_claim2 like d_claim): sgn_adam_rows_pend_bytes(min(n_max
 * + 1, n_rows)) bytes receiving list 1's distinct valid rows and row 0 -- int64 count at [0], the
 * number of list-1 ids >= n_rows at [1] (a query / table mismatch), int32 rows from byte 16.
 * mv_stride (host, optional): row stride in floats of d_exp_avg[t] / d_exp_avg_sq[t] (>= row_width[t];
 * null: row_width) -- the narrow tensors' moments may share one packed [n_rows][16] buffer (ABI 18). */
size_t sgn_adam_rows_workspace_bytes(int64_t n_entries);
size_t sgn_adam_rows_pend_bytes(int64_t n_entries);
int sgn_adam_rows(int32_t n_t, float *const *d_param, float *const *d_grad, float *const *d_exp_avg,
                  float *const *d_exp_avg_sq, const int32_t *row_width, const int32_t *mv_stride, int64_t n_rows,
                  const int32_t *d_rows, const void *d_count, int32_t count_is64, int32_t count_mul, int64_t n_max,
                  int32_t row0, const int32_t *d_rows2, const int64_t *d_count2, int64_t n_max2, int32_t *d_last,
                  int32_t *d_claim, int32_t *d_claim2, int32_t tag, void *d_ws, size_t ws_bytes, void *d_pend,
                  size_t pend_bytes, float *d_sched, double lr, double beta1, double beta2, double eps, int64_t step,
                  int32_t apply, int32_t zero_grad, sgn_stream_t stream);
/* d_out[i][c] = sum over r < rows of d_x[i][r][c] (fp16 in, fp32 out, deterministic order),
 * for count <= 8 matrices [rows][256] (the bias gradients db = sum of the deltas,
 * torch.sum(d, 0) in the reference's autograd of nn.Linear).  d_x: host array of device
 * pointers; d_ws: sgn_colsum_workspace_bytes(count) of device scratch. */
size_t sgn_colsum_workspace_bytes(int32_t count);
int sgn_colsum_f16(int32_t count, const void *const *d_x, int64_t rows, int32_t cols, float *d_ws, float *d_out,
                   sgn_stream_t stream);
/* The same with per-row fp32 weights: d_out[i][c] = sum over r of d_rw[i][r] * d_x[i][r][c] (d_rw: host
 * array of device pointers, NULL entries = unweighted) -- the alpha branch's weight gradient
 * dza^T h4 (point_aggregators.py:650-653, nn.Linear(256, 1)) in the bias sums' launch. */
int sgn_colsum_f16_weighted(int32_t count, const void *const *d_x, const float *const *d_rw, int64_t rows,
                            int32_t cols, float *d_ws, float *d_out, sgn_stream_t stream);
/* ABI 14: the same sums left as SGN_COLSUM_SLABS fixed row-slab partials in d_ws (one launch, no final
 * pass), for sgn_grad_accumulate to add: column c of matrix i, slab b at
 * d_ws[(i * SGN_COLSUM_SLABS + b) * 256 + c]; for weighted matrices the slab's sum of the row weights
 * (the alpha branch's bias gradient sum(dza), point_aggregators.py:650-653) at
 * d_ws[count * SGN_COLSUM_SLABS * 256 + i * SGN_COLSUM_SLABS + b]. */
#define SGN_COLSUM_SLABS 512
int sgn_colsum_f16_weighted_parts(int32_t count, const void *const *d_x, const float *const *d_rw, int64_t rows,
                                  int32_t cols, float *d_ws, sgn_stream_t stream);

/* ---- training: segment kernels (one launch for up to 16 segments) --------------------
 * The gradient epilogue of the training step's weight GEMMs, i.e. the accumulation torch
 * autograd does into nn.Linear's weight/bias .grad (models/base_rendering_model.py:534-664 ->
 * loss.backward(); the layers of models/aggregators/point_aggregators.py:620-653, :772-780):
 * per segment, for j < n with dst[j] >= 0,
 *   d_grad[dst[j]] += (sum over b < nb of src[b * stride + j]  (+ tail[j] if tail)) / d_scale[0]
 * src: nb split-K partials (fp32, device); dst: int32 device map from the MFMA storage order to
 * the flat parameter (-1 = padding); d_scale: device loss scale or NULL (1).  Every dst entry of
 * a launch must be distinct (no two segments add into the same element).  Up to 16 partials the
 * sum runs in partial order; beyond, groups of ~16 partials add with float atomics, so the
 * fp32 sum order (not the set of terms) varies run to run.  The f16 training step uses it; the
 * fp32 step reduces through sgn_reduce_partials (fixed order, deterministic). */
typedef struct {
    const float *src;
    const float *tail;     /* optional [n] partial added after the nb slices (NULL: none) */
    const int32_t *dst;
    int64_t n;             /* elements per partial */
    int64_t stride;        /* elements between partials (>= n) */
    int32_t nb;            /* partials (>= 1) */
    int32_t reserved;
} sgn_grad_segment;
int sgn_grad_accumulate(int32_t n_seg, const sgn_grad_segment *segs, const float *d_scale, float *d_grad,
                        sgn_stream_t stream);
/* Clears n_seg device regions (d_ptr[i]: 16-B aligned, bytes[i] a multiple of 16; host arrays). */
int sgn_zero_segments(int32_t n_seg, void *const *d_ptr, const int64_t *bytes, sgn_stream_t stream);
/* Copies n_seg device regions in one launch: d_dst[i] = d_src[i] (bytes[i] bytes; d_src[i] null:
 * zeros), any alignment (16-B units where both ends and the length allow).  Host arrays.  The
 * training step's graph inputs / outputs and clears, instead of one copy or fill per tensor. */
int sgn_copy_segments(int32_t n_seg, const void *const *d_src, void *const *d_dst, const int64_t *bytes,
                      sgn_stream_t stream);
/* Index gathers from one fp32 source (the flat MLP parameter): dst[j] = src[idx[j]], 0 for idx
 * outside [0, n_src); stored as fp32 or, with fp16 != 0, rounded to fp16 (nearest even) -- the
 * device re-pack of the MFMA weight blobs each training step. */
typedef struct {
    const int32_t *idx;
    void *dst;
    int64_t n;
    int32_t fp16;
    int32_t reserved;
} sgn_gather_segment;
int sgn_gather_segments(int32_t n_seg, const sgn_gather_segment *segs, const float *d_src, int64_t n_src,
                        sgn_stream_t stream);
/* The fp32-faithful blob (sgn_mlp_pack_f32's layout) re-packed on the device from the flat fp32
 * parameter each training step: per layer l (w_off / w_len: host arrays, the weight span of layer
 * l in the flat vector, n_layers <= 16) the shift s_l = 14 - e, max |W_l| = f 2^e (frexp); then
 * the fp16 section (d_code16[j] = flat index | layer << 22 | lo << 26, -1 = zero: hi = fp16(W 2^s),
 * lo = fp16(W 2^s - hi)) and the fp32 section (d_code32[j] = flat index | layer << 22 | kind << 26,
 * kinds as the layout's sgn_mlp_pack_index_f32 map).  d_shift: int32[16] device scratch.  Bit-equal
 * to sgn_mlp_pack_f32 on the same weights. */
int sgn_pack_scaled_f32(const float *d_flat, int64_t n_flat, int32_t n_layers, const int64_t *w_off,
                        const int64_t *w_len, const int32_t *d_code16, int64_t n16, const int32_t *d_code32, int64_t n32,
                        int32_t *d_shift, void *d_out16, float *d_out32, sgn_stream_t stream);
/* The f16 training step's captured loss stage inputs over its item capacity n_cap: for item
 * i < d_counters[1] (sgn_query's work-item count) d_fs32[i] = fp32 of d_fs16[i] ([n_cap][256] fp16,
 * sgn_aggregate_train_fwd's blended features), d_al32[i] = d_feat[work[i]].alpha, d_v[i] = the
 * direction of the item's ray, d_samp[i] = work[i]; padding items get zeros, ray 0 and s_cap.
 * d_vpe (or NULL): [n_cap][32] the colour MLP's PE(viewdir) (sin | cos of v 2^f, f < 4, per
 * component; point_aggregators.py:772-780), 1 in column 24 (colour 0's bias column), zeros after. */
int sgn_colour_inputs(const int32_t *d_counters, const int32_t *d_work, const int32_t *d_samp_ray, int64_t n_cap,
                      int64_t s_cap, const void *d_fs16, const float *d_feat, const float *d_raydir, float *d_fs32,
                      float *d_al32, float *d_v, int32_t *d_samp, float *d_vpe, sgn_stream_t stream);
/* The backward's power-of-two loss scale: d_out[0] = 2^-floor(log2(max(max|a|, max|b|, 1e-30)))
 * over two fp32 device arrays (a NaN propagates), in two launches with no host sync; d_ws:
 * sgn_pow2_scale_workspace_bytes() of device scratch. */
size_t sgn_pow2_scale_workspace_bytes(void);
int sgn_pow2_scale(const float *d_a, int64_t na, const float *d_b, int64_t nb, void *d_ws, float *d_out,
                   sgn_stream_t stream);
/* The distinct points a training step's rays touch, on the device: point 0 (the conf read of empty
 * neighbour slots, train.composite_losses) and every neighbour d_pidx[e] >= 0, e < d_counters[0] * K
 * (sgn_query's sample count; s_cap bounds it).  Appends them to d_idx (int32 [n_points]) in no
 * particular order and writes their count to d_count2[step & 1]; d_count2[(step + 1) & 1] is
 * cleared for the next step; d_count2[2] (ABI 12) accumulates the neighbour indices >= n_points met
 * (a query / point-table mismatch: such a point is never projected), so a caller can assert it is 0.  d_stamp: int32 [n_points], -1 once at allocation, then owned by the
 * caller's step counter (step >= 0, increasing).  Replaces the torch touched_rows mask / scan /
 * scatter (train.py) on the single-GPU fp32 step's projection subset (sgn_point_project_f32_subset);
 * the neighbours come from the reference's query (neural_points.py:942-988). */
int sgn_touched_points(const int32_t *d_pidx, const int32_t *d_counters, int64_t s_cap, int32_t K, int64_t n_points,
                       int32_t step, int32_t *d_stamp, int32_t *d_idx, int64_t *d_count2, sgn_stream_t stream);

/* The distinct points a render frame's samples name (ABI 19), for sgn_point_project_f32_subset: the
 * block1.0 projection then runs over those points only (~19 % of the 1.2 M points of a config-2
 * frame) instead of all of them.  Point 0 and every neighbour d_pidx[e] >= 0, e < min(d_counters[0]
 * * K, s_cap * K), go to d_idx (int32 [n_points], no particular order) with their count at
 * d_count[0] (int64, device); d_count[1] accumulates neighbour indices >= n_points (a query / table
 * mismatch: never projected; the caller zeroes it once).  d_mark: sgn_frame_points_mark_bytes(
 * n_points) bytes, zero at allocation and left zero by every call.  d_pidx 16-B aligned. */
size_t sgn_frame_points_mark_bytes(int64_t n_points);
int sgn_frame_points(const int32_t *d_pidx, const int32_t *d_counters, int64_t s_cap, int32_t K, int64_t n_points,
                     uint8_t *d_mark, int32_t *d_idx, int64_t *d_count, sgn_stream_t stream);

/* ---- fp32 training step on hand-written kernels (ABI 9; SG entries ABI 10) -----------------------------------
 * The reference's fp32 autograd through PointAggregator / viewmlp and the NeuralPoints gather
 * (models/aggregators/point_aggregators.py:561-786, :868-959; neural_points.py:942-988; run from
 * optimize_parameters, base_rendering_model.py:534-664, mvs_points_volumetric_model.py:116-141) as
 * a fixed launch sequence over COMPACT rows (one per valid (sample, neighbour), sample-major) and
 * work items (samples with a neighbour, ascending): no host synchronisation, every count read on
 * the device (d_counts[0] = items, d_counts[1] = rows, from sgn_train_lists).
 *
 * sgn_x3_gemm: every nn.Linear product of the step (forward x W^T, backward data dy W, weight
 * gradient dy^T x) at fp32 accuracy on fp16 MFMA: each fp32 product as three fp16 products of
 * hi / lo halves (fp32 accumulate), operands scaled by powers of two before the split (weights by
 * d_shift -- the per-layer shifts sgn_pack_scaled_f32 writes -- deltas by the amax word their
 * producer wrote).  Operand element (i, k) (i: output row / column index, k: reduction index) is
 * element (r, c) of a row-major fp32 matrix, r = i, c = k (kmajor 0) or r = k, c = i (kmajor 1);
 * columns c >= csplit come from p2 (column c - csplit, no activation), c == ones_col reads 1 (the
 * bias gradient's column), c >= ncols reads 0; act = 1 applies LeakyReLU(0.01) to p's values.
 *   mode 0 (rows): out[r][n] (n < out_cols) / out2[r][n - out_cols] (n < N) = sum_k A(r, k) B(n, k)
 *     (+ bias[n]) for r < min(*d_rows, M); out is multiplied by LeakyReLU'(mask[r][n]) when mask is
 *     given (dz = dh * (z > 0 ? 1 : 0.01)), then LeakyReLU'd when act; *amax_out = max(|out|)
 *     (atomicMax of the bits; the caller zeroes it).  K = the weight matrix's reduction extent.
 *   mode 1 (split-K): part[s][m][n] = sum over rows r of split s of A(m, r) B(n, r), rows
 *     r < min(*d_rows, K) cut into `splits` equal 32-aligned runs (empty runs write zeros). */
typedef struct {
    const float *p, *p2;
    int64_t ld, ld2;
    int32_t csplit, ncols, ones_col, act, kmajor;
    const uint32_t *amax;   /* scale source: max |x| bits (or NULL) */
    const int32_t *shift;   /* or a power-of-two shift (or NULL: no scaling) */
} sgn_x3_operand;
typedef struct {
    sgn_x3_operand a, b;
    int32_t mode, M, N, K;
    const int32_t *d_rows;
    const float *bias;
    int32_t act;
    const float *mask;
    int64_t ldm;
    float *out;
    int64_t ldo;
    int32_t out_cols;
    float *out2;
    int64_t ldo2;
    uint32_t *amax_out, *amax_out2;
    float *part;
    int32_t splits;
    int32_t products;   /* 3 (or 0): hi/lo products, fp32 accuracy; 1: the hi halves only (fp16 operands,
                           the f16 training step's colour MLP; colour-layer shapes only) */
    void *bpack;        /* ABI 13, mode 0: NULL, or a 16-B aligned workspace of sgn_x3_gemm_bpack_bytes(g)
                           bytes: the weight blocks are split there once per call (one extra launch) and
                           every workgroup copies its block into LDS by DMA instead of converting it */
} sgn_x3_gemm_args;
int sgn_x3_gemm(const sgn_x3_gemm_args *g, sgn_stream_t stream);
size_t sgn_x3_gemm_bpack_bytes(const sgn_x3_gemm_args *g);   /* ABI 13; 0 unless mode 0 with K <= 288 */

/* The f16 training step's row-layer weight gradients (ABI 13; replaces the fp16 GEMMs of the
 * reference's autograd dW of the aggregator MLP, point_aggregators.py:868-959 under
 * base_rendering_model.py:534-664): part[s][m][n] = sum over the rows r of run s of d[r][m] x[r][n]
 * (fp32 accumulation of the exact fp16 products) for m < 256, n < ncols, the rows r < n_rows cut into
 * `splits` equal 32-aligned runs (empty runs write zeros); part is fp32 [splits][256][ncols].  d: fp16
 * [n_rows][ldd] (ldd >= 256), x: fp16 [n_rows][ldx], 16-B aligned rows, ncols % 8 == 0.  part_bias
 * (or NULL): fp32 [splits][256], the runs' column sums of d (the layer's bias gradient partials). */
int sgn_f16_weight_grad(const void *d, int64_t ldd, const void *x, int64_t ldx, int32_t ncols, int32_t n_rows,
                        int32_t splits, float *part, float *part_bias, sgn_stream_t stream);

/* Deterministic work list and compact row offsets after sgn_query: for s < d_counters[0],
 * d_row_off[s] = sum of samp_nnb over samples < s; d_work = the samples with samp_nnb > 0 in
 * ascending order (overwrites the query's unordered list: same set, same count); d_feat[s] = 0
 * (float4[s_cap]); d_counts[0] = items, [1] = rows.  d_ws: sgn_train_lists_workspace_bytes. */
size_t sgn_train_lists_workspace_bytes(int64_t s_cap);
int sgn_train_lists(const int32_t *d_counters, const int32_t *d_samp_nnb, int64_t s_cap, int32_t *d_work,
                    int32_t *d_row_off, float *d_feat, int32_t *d_counts, void *d_ws, sgn_stream_t stream);
/* Per row j (compact): d_x0[j] fp32[288] = block1.0's input [emb | PE(emb) | PE(dists)] (:594-621)
 * with 1 in column 284 (bias) and 0 after; d_ext[j] fp32[8] = block3.0's extra inputs [colour |
 * dir - v | <dir, v>] (:639-652) and 1; d_rw[j] fp32[2] = (normalised weight * clamped conf,
 * normalised weight).  Per item i: d_vpe[i] fp32[32] = PE(viewdir, 4) (sin | cos, :772-780), 1
 * in column 24, 0 after. */
int sgn_train_row_inputs(const sgn_point_tables *pt, const sgn_query_out *q, int32_t K, const int32_t *d_row_off,
                         const int32_t *d_counts, float *d_x0, float *d_ext, float *d_rw, float *d_vpe,
                         sgn_stream_t stream);
/* Per compact row j (sample s, neighbour k): d_dst[j][0..dim) = d_src[pidx[s K + k]][0..dim) --
 * SG's BPNet embedding rows, block2_bpnet.0's second input, for its weight gradient (dim % 4 == 0,
 * 16-B aligned tables). */
int sgn_train_row_gather(const sgn_query_out *q, int32_t K, const int32_t *d_row_off, const int32_t *d_counts,
                         const float *d_src, int32_t dim, float *d_dst, sgn_stream_t stream);
/* color_branch.6 + sigmoid * 1.002 - 0.001 (fp32) on the items' last hidden layer d_h3 [items][128]
 * (d_w6 [3][128], d_b6 [3]): d_feat[work[i]].rgb. */
int sgn_train_colour_head(const sgn_query_out *q, const int32_t *d_counts, const float *d_h3, const float *d_w6,
                          const float *d_b6, float *d_feat, sgn_stream_t stream);
/* Its backward from d_dfeat float4[S] (the loss stage's d feat): d_dy3 [items][128] = d loss / d
 * color_branch.4's pre-activation, *d_amax = max |dy3|, d_part = color_branch.6's weight / bias
 * gradient as sgn_train_head_partial_floats(0) floats ([blocks][3][129]). */
size_t sgn_train_head_partial_floats(int32_t which);
int sgn_train_colour_head_bwd(const sgn_query_out *q, const int32_t *d_counts, const float *d_h3, const float *d_w6,
                              const float *d_b6, const float *d_dfeat, float *d_dy3, uint32_t *d_amax, float *d_part,
                              sgn_stream_t stream);
/* block3.2's LeakyReLU, the alpha branch and the K-blend backward per row: d_z4_delta4 holds
 * block3.2's pre-activation [rows][256] and is overwritten with its delta; d_dfs [items][256]
 * = d loss / d f_s; d_dfeat.x = d loss / d alpha_s; d_rw from sgn_train_row_inputs; d_wa [256],
 * d_ba [1] alpha_branch.0; d_gconf[N] += d conf (straight-through clamp, :863-865); *d_amax =
 * max |delta4|; d_part = alpha_branch.0's weight / bias gradient, sgn_train_head_partial_floats(1)
 * floats ([blocks][257]). */
int sgn_train_row_head(const sgn_point_tables *pt, const sgn_query_out *q, int32_t K, const int32_t *d_row_off,
                       const int32_t *d_counts, float *d_z4_delta4, const float *d_dfs, const float *d_dfeat,
                       const float *d_rw, const float *d_wa, const float *d_ba, float *d_gconf, uint32_t *d_amax,
                       float *d_part, sgn_stream_t stream);
/* Point gradients of the rows (atomic adds, like the reference's index_add): d_dx0 [rows][224] =
 * d loss / d [emb | PE(emb)] -> points_embeding; d_dext [rows][8] -> points_color, points_dir. */
int sgn_train_row_tail(const sgn_point_tables *pt, const sgn_query_out *q, int32_t K, const int32_t *d_row_off,
                       const int32_t *d_counts, const float *d_dx0, const float *d_dext, const sgn_point_grads *grads,
                       sgn_stream_t stream);
/* Partials -> flat gradient, in a fixed order: per segment, for m < M, c < N,
 * v = sum over s < splits of part[s][m][c]; dst_w[m * ldw + c] += v (c < n_in), dst_b[m] += v
 * (c == bias_col).  Up to 16 segments per launch; no two may add into the same element. */
typedef struct {
    const float *part;
    int32_t splits, M, N, n_in, bias_col, ldw;
    float *dst_w, *dst_b;
} sgn_partial_segment;
int sgn_reduce_partials(int32_t n_seg, const sgn_partial_segment *segs, sgn_stream_t stream);

/* ---- composite --------------------------------------------------------- */

typedef struct {
    int32_t SR;
    float vsize_z;        /* vsize[2] (0.008): last-interval / replacement distance */
    int32_t raydist_mode_unit;
    float bg[3];          /* bg_color (tone map off) */
} sgn_composite_params;

/* Per ray: out_rgb float[R*3] (bg for invalid rays), out_mask int8[R]
 * (reference ray_mask after masked_valid_ray), out_bgT float[R] (background
 * transmission; 1 for invalid rays), out_opacity / out_blendw float[R*SR]
 * (opacity and alpha-blend weight per slot; may be NULL). */
int sgn_composite(const sgn_composite_params *cp, const float *d_campos, const float *d_camrotc2w,
                  const float *d_raydir, int64_t R, const float *d_t_table, int32_t per_ray_t,
                  int32_t D, const sgn_query_out *q, const float *d_feat, float *d_out_rgb,
                  int8_t *d_out_mask, float *d_out_bgT, float *d_out_opacity, float *d_out_blendw,
                  sgn_stream_t stream);

/* ray_march on dense [R, SR] inputs (diff_ray_marching.py:509-555, alpha blend +
 * radiance render): ray_dist/valid/feat(float4) in, rgb[R*3] (+ bg*T if bg != NULL,
 * host pointer to 3 floats), opacity/acc_transmission/blend_weight[R*SR], bg T[R]. */
int sgn_ray_march_dense(const float *d_ray_dist, const uint8_t *d_valid, const float *d_feat, int64_t R,
                        int32_t SR, const float *bg, float *d_rgb, float *d_opacity, float *d_acc_t,
                        float *d_blendw, float *d_bgT, sgn_stream_t stream);

/* ---- training loss stage (forward + backward) ----------------------------
 * Replaces the torch autograd of ray_dist + ray_march + fill_invalid and the training losses:
 *   models/neural_points_volumetric_model.py:569-577, models/rendering/diff_ray_marching.py:509-555,
 *   models/base_rendering_model.py:534-664 (ray_masked_coarse_raycolor; ray_miss / coarse logged),
 *   models/mvs_points_volumetric_model.py:607-614 (zero_one_loss on conf_coefficient). */
typedef struct {
    int32_t SR, K;
    float vsize_z;             /* vsize[2] */
    int32_t raydist_mode_unit;
    float bg[3];
    float zero_one_weight;     /* 1e-4 (train_ft) */
    float zero_one_eps;        /* 1e-3 */
    const float *bg_ray;       /* ABI 16: device float[R*3], the rays' background (inputs['bg_ray'] of the
                                  plane background model, fill_invalid's T_bg * bg_ray,
                                  neural_points_volumetric_model.py:175-177); NULL: bg[3] for every ray */
} sgn_loss_params;

size_t sgn_loss_workspace_bytes(int64_t R, int32_t SR);
/* d_feat float4[S] per sample (alpha, r, g, b; zeros for samples without neighbours) in; per ray
 * d_out_rgb float[R*3] (bg for rays without a valid sample) and d_out_mask int8[R]; d_losses
 * float[8] (device): ray_masked_coarse_raycolor, conf_coefficient (zero-one), ray_miss_coarse_raycolor,
 * coarse_raycolor, then the gradient scales; d_dfeat float4[S] = d total / d feat of every sample of
 * the rays (written); d_dconf float[N] += d total / d conf (atomics).  total = d_losses[0] + 3e-6 +
 * zero_one_weight * d_losses[1].  No host synchronisation. */
int sgn_loss_train(const sgn_loss_params *lp, const float *d_campos, const float *d_camrotc2w, int64_t R,
                   const sgn_query_out *q, const float *d_feat, const float *d_gt, const float *d_conf,
                   float *d_out_rgb, int8_t *d_out_mask, float *d_losses, float *d_dfeat, float *d_dconf,
                   void *d_workspace, size_t workspace_bytes, sgn_stream_t stream);

/* ---- misc -------------------------------------------------------------- */
int sgn_abi_version(void);
const char *sgn_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* SGN_HIP_H */
