// mlp_layout.h -- packed layout of the viewmlp weights for the MFMA kernels.
//
// Reference network (models/aggregators/point_aggregators.py:312-421, ScanNet):
//   block1: Linear(284,256) LReLU Linear(256,256) LReLU          per (sample, neighbour) row
//   block3: Linear(263,256) LReLU Linear(256,256) LReLU          per row
//   alpha_branch: Linear(256,1) -> softplus(x - 1)               per row, then K-blend
//   color_branch: Linear(280,128) LReLU x3 ... Linear(128,3)      per sample, sigmoid*1.002-0.001
//
// MFMA: v_mfma_f32_32x32x16_f16, D[32 out units][32 rows] += A[32 out][16 in] * B[16 in][32 rows].
// Lane l: A row (l & 31), k = 8*(l>>5) + e; B col (l & 31), k = 8*(l>>5) + e; D unit
// (reg&3) + 8*(reg>>2) + 4*(l>>5) of the 32-unit tile, row (l & 31).
//
// A fragments are stored fragment-major: [tile t][k-step][lane 0..63][8 x f16] (1 KiB per
// fragment, one 16-byte load per lane).  The in-register chaining of layer outputs into
// the next layer's B operand permutes k inside each 16-wide step (see perm_acc below);
// the permutation is folded into the packed A columns so nothing moves at run time.
#pragma once
#include <stddef.h>

namespace sgn {
namespace mlp {

constexpr int HID = 256;      // shading_feature_num
constexpr int CHID = 128;     // colour hidden
constexpr int T_HID = HID / 32;
constexpr int T_CHID = CHID / 32;
constexpr int KS_L0 = 18;     // 284 -> 288 inputs (custom per-half channel order)
constexpr int KS_HID = 16;    // 256 inputs
constexpr int KS_L2 = 17;     // 256 + 7 (colour, dir - v, <dir, v>) -> 272
constexpr int KS_C0 = 18;     // 256 + 24 (PE(viewdir)) -> 288
constexpr int KS_CH = 8;      // 128 inputs
constexpr size_t FRAG = 1024; // bytes per A fragment

constexpr size_t OFF_W0 = 0;
constexpr size_t OFF_W1 = OFF_W0 + (size_t)T_HID * KS_L0 * FRAG;
constexpr size_t OFF_W2 = OFF_W1 + (size_t)T_HID * KS_HID * FRAG;
constexpr size_t OFF_W3 = OFF_W2 + (size_t)T_HID * KS_L2 * FRAG;
constexpr size_t OFF_C0 = OFF_W3 + (size_t)T_HID * KS_HID * FRAG;
constexpr size_t OFF_C1 = OFF_C0 + (size_t)T_CHID * KS_C0 * FRAG;
constexpr size_t OFF_C2 = OFF_C1 + (size_t)T_CHID * KS_CH * FRAG;
constexpr size_t OFF_F32 = OFF_C2 + (size_t)T_CHID * KS_CH * FRAG;
// fp32 section, "accumulator order" vectors v[t][h][r] = u[32t + (r&3) + 8(r>>2) + 4h]
constexpr size_t F_B0 = 0, F_B1 = 256, F_B2 = 512, F_B3 = 768;      // block biases
constexpr size_t F_CB0 = 1024, F_CB1 = 1152, F_CB2 = 1280;            // colour biases
constexpr size_t F_WA = 1408;                                          // alpha weight [256]
constexpr size_t F_BA = 1664;                                          // alpha bias
constexpr size_t F_WC3 = 1668;                                         // colour out [3][128]
constexpr size_t F_BC3 = 2052;                                         // colour out bias [3]
constexpr size_t N_F32 = 2056;
constexpr size_t BASE_BYTES = OFF_F32 + N_F32 * 4;

// Split block1.0 (inference): its inputs [feat 32 | PE(feat) 192 | PE(dists) 60] are
// per-point for the first 224 channels, so W0a [feat | PE(feat)] + b0 is applied once per
// point and frame (k_point_proj -> P[point], fp16) and the per-row layer 0 only multiplies
// W0b by the 30 PE(dists) channels of each lane-half (4 k-steps), its accumulators starting
// at P[pid].  Same sums, regrouped; the sections are appended after the base blob.
constexpr int KS_L0S = 4;        // per-row k-steps: local channels 112..143 of each lane-half
constexpr int KS_P0 = 14;        // per-point k-steps: local channels 0..111 of each lane-half
constexpr size_t OFF_W0B = BASE_BYTES;                                   // [1 pass][4 ks][8 tiles]
constexpr size_t OFF_W0A = OFF_W0B + (size_t)T_HID * KS_L0S * FRAG;      // [tile][14 ks]
constexpr size_t TOTAL_BYTES = OFF_W0A + (size_t)T_HID * KS_P0 * FRAG;
constexpr size_t PROJ_BYTES_PER_POINT = HID * 2;  // P[point]: 2 lane-halves x 128 fp16, acc order

// SG-NeRF extension (shading_feature_mlp_layer2_bpnet = 1, point_aggregators.py:345-354,
// :629-636): block2_bpnet.0 = Linear(256 + bpnet_dim -> 256) + LReLU between block1 and
// block3, appended after the base blob so the base layout is unchanged.
//   k-steps 0..15: the chained block1 output (perm_acc order); 16..: the gathered per-point
//   BPNet embedding, channel 16 j + 8 h + e at k-step 16 + j, lane-half h, element e
//   (= natural [N, bpnet_dim] order, so the fp16 point table needs no permutation).
constexpr int BP_DIM = 96;                           // predict_semantic = 1 (:346)
__host__ __device__ constexpr int ks_bp(int bpnet_dim) { return KS_HID + (bpnet_dim + 15) / 16; }
constexpr size_t OFF_WB = TOTAL_BYTES;                // block2_bpnet.0 fragments (k-outer stream order)
__host__ __device__ constexpr size_t off_bb(int ksb) { return OFF_WB + (size_t)T_HID * ksb * FRAG; }  // bias, acc order
__host__ __device__ constexpr size_t total_bytes_sg(int ksb) { return ksb ? off_bb(ksb) + HID * 4 : TOTAL_BYTES; }
constexpr size_t F_BB = N_F32;                        // bias slot after the base fp32 section (LDS copy)

// unit of the 32-wide tile held by accumulator register r of lane-half h
__host__ __device__ constexpr int acc_unit(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }
// B-operand position p (0..15, p = 8h + e) of a k-step fed from accumulator registers
// 8s..8s+7 -> input unit offset inside the 16-wide step
__host__ __device__ constexpr int perm_acc(int p) { return 8 * ((p & 7) >> 2) + 4 * (p >> 3) + (p & 3); }

// Layer-0 channel order.  Lane-half h builds local channels c = 8*kstep + e (0..143):
//   c <  16        : feat[16h + c]
//   16 <= c < 112  : PE(feat):  m = c-16, d = m/6, f = (m%6)/2, sc = m%2 -> sin/cos(feat[16h+d]*2^f)
//   112 <= c < 142 : PE(dists): m = c-112, dd = m/10, f = (m%10)/2, sc = m%2 -> sin/cos(dist[3h+dd]*2^f)
//   142, 143       : zero
// Reference column (feat 32 | PE(feat) 192 | PE(dists) 60), networks.py:175-192 order.
__host__ __device__ constexpr int l0_ref_col(int h, int c) {
    return c < 16 ? 16 * h + c
         : c < 112 ? 32 + ((16 * h + (c - 16) / 6) * 3 + ((c - 16) % 6) / 2) * 2 + (c - 16) % 2
         : c < 142 ? 224 + ((3 * h + (c - 112) / 10) * 5 + ((c - 112) % 10) / 2) * 2 + (c - 112) % 2
         : -1;
}

}  // namespace mlp
}  // namespace sgn
