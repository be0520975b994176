"""Hot-path subset of the reference's option namespace.

The reference spreads these over argparse hooks
(models/neural_points/neural_points.py:80-309,
models/aggregators/point_aggregators.py:14-253,
models/neural_points_volumetric_model.py:63-124).  Defaults below are the
ScanNet values of dev_scripts/w_scannet_etf/scene241.sh:11-106 and
pointnerf/run/checkpoints/scannet/scene0710_00640480/opt.txt.
"""
from dataclasses import dataclass, field, fields, replace
from typing import Tuple


@dataclass(frozen=True)
class HotPathOpts:
    # querier (query_point_indices_worldcoords.py)
    vsize: Tuple[float, float, float] = (0.008, 0.008, 0.008)
    vscale: Tuple[int, int, int] = (2, 2, 2)
    kernel_size: Tuple[int, int, int] = (3, 3, 3)
    query_size: Tuple[int, int, int] = (3, 3, 3)
    ranges: Tuple[float, ...] = (-10.0, -10.0, -10.0, 10.0, 10.0, 10.0)
    radius_limit_scale: float = 4.0
    depth_limit_scale: float = 0.0
    z_depth_dim: int = 400
    max_o: int = 610000
    SR: int = 24
    K: int = 8
    P: int = 26
    NN: int = 2
    inverse: int = 0
    wcoord_query: int = 1
    semantic_guidance: int = 0
    predict_semantic: int = 0  # 1: BPNet embedding (96) feeds block2_bpnet (point_aggregators.py:346)
    near_plane: float = 0.1
    far_plane: float = 8.0
    # aggregator (point_aggregators.py)
    point_features_dim: int = 32
    shading_feature_num: int = 256
    shading_feature_mlp_layer1: int = 2
    shading_feature_mlp_layer2: int = 0
    shading_feature_mlp_layer2_bpnet: int = 0
    shading_feature_mlp_layer3: int = 2
    shading_alpha_mlp_layer: int = 1
    shading_color_mlp_layer: int = 4
    shading_color_channel_num: int = 3
    num_feat_freqs: int = 3
    dist_xyz_freq: int = 5
    num_viewdir_freqs: int = 4
    num_pos_freqs: int = 10
    view_ori: int = 0
    agg_dist_pers: int = 20
    agg_distance_kernel: str = "linear"
    agg_intrp_order: int = 2
    agg_weight_norm: int = 1
    agg_axis_weight: Tuple[float, float, float] = (1.0, 1.0, 1.0)
    agg_feat_xyz_mode: str = "None"
    agg_alpha_xyz_mode: str = "None"
    agg_color_xyz_mode: str = "None"
    apply_pnt_mask: int = 1
    act_type: str = "LeakyReLU"
    act_super: int = 1
    dist_xyz_deno: float = 0.0
    point_color_mode: str = "1"
    point_dir_mode: str = "1"
    point_conf_mode: str = "1"
    # ray marching (neural_points_volumetric_model.py)
    raydist_mode_unit: int = 1
    which_tonemap_func: str = "off"
    which_render_func: str = "radiance"
    which_blend_func: str = "alpha"
    bg_color: str = "white"
    # knobs of this implementation (no reference counterpart)
    # aggregator arithmetic: "f32" = the reference's fp32 products, each carried as three fp16 MFMA
    # products with fp32 accumulation (mlp_x3.hip); "f16" = fp16 MFMA operands (mlp.hip, faster)
    precision: str = "f32"
    fix_occ0: int = 0          # 1: do not reproduce the `voxel_idx > 0` bug (worldcoords.py:395)
    reservoir_seed: int = 0    # replaces the reference's wall-clock curand seed (:314, :402)
    is_train: int = 0

    @property
    def bpnet_variant(self):
        """(bpnet_layers, bpnet_dim) of the aggregator (SG block2_bpnet, point_aggregators.py:345-354)."""
        if self.shading_feature_mlp_layer2_bpnet == 0:
            return 0, 0
        return 1, (96 if self.predict_semantic == 1 else 0)

    @classmethod
    def from_opt(cls, opt, **overrides):
        """Take every known field from a reference-style Namespace."""
        kw = {}
        for f in fields(cls):
            if hasattr(opt, f.name):
                v = getattr(opt, f.name)
                if isinstance(v, list):
                    v = tuple(v)
                kw[f.name] = v
        kw.update(overrides)
        o = cls(**kw)
        if o.query_size[0] == 0:  # neural_points.py:425
            o = replace(o, query_size=o.kernel_size)
        return o

    def check_supported(self):
        """The HIP path implements the ScanNet viewmlp layout; refuse others loudly."""
        bad = []
        if self.wcoord_query != 1:
            bad.append("wcoord_query must be 1 (perspective querier is out of scope)")
        if self.agg_dist_pers != 20 or self.agg_distance_kernel != "linear" or self.agg_intrp_order != 2:
            bad.append("aggregator must be agg_dist_pers=20, linear kernel, agg_intrp_order=2")
        if (self.point_features_dim, self.shading_feature_num, self.num_feat_freqs, self.dist_xyz_freq,
                self.num_viewdir_freqs) != (32, 256, 3, 5, 4):
            bad.append("MLP widths/frequencies must match the ScanNet viewmlp (32/256/3/5/4)")
        if (self.shading_feature_mlp_layer1, self.shading_feature_mlp_layer2, self.shading_feature_mlp_layer3,
                self.shading_alpha_mlp_layer, self.shading_color_mlp_layer) != (2, 0, 2, 1, 4):
            bad.append("viewmlp layer counts must be (2, 0, 2, 1, 4)")
        if self.shading_feature_mlp_layer2_bpnet not in (0, 1):
            bad.append("block2_bpnet: at most one layer (shading_feature_mlp_layer2_bpnet 0 or 1)")
        elif self.shading_feature_mlp_layer2_bpnet == 1 and bool(self.predict_semantic) != bool(self.semantic_guidance):
            # the reference concatenates the gathered embedding iff semantic_guidance (neural_points.py:971,
            # point_aggregators.py:631-635) but sizes the layer by predict_semantic (:346): other pairs crash there
            bad.append("block2_bpnet needs predict_semantic == semantic_guidance")
        if self.shading_feature_mlp_layer2_bpnet == 0 and self.predict_semantic not in (0, 1):
            bad.append("predict_semantic must be 0 or 1")
        if self.act_type != "LeakyReLU" or self.act_super != 1 or self.view_ori != 0:
            bad.append("activations must be LeakyReLU + act_super=1, view_ori=0")
        if self.agg_feat_xyz_mode != "None" or self.agg_alpha_xyz_mode != "None" or self.agg_color_xyz_mode != "None":
            bad.append("agg_*_xyz_mode must be None")
        if self.dist_xyz_deno != 0.0 or self.apply_pnt_mask != 1 or self.agg_weight_norm != 1:
            bad.append("dist_xyz_deno=0, apply_pnt_mask=1, agg_weight_norm=1 required")
        if self.which_render_func != "radiance" or self.which_blend_func != "alpha":
            bad.append("radiance render + alpha blend required")
        if self.precision not in ("f32", "f16"):
            bad.append("precision must be 'f32' (reference arithmetic) or 'f16'")
        if self.inverse != 0:
            bad.append("inverse (disparity) ray generation is not implemented")
        if bad:
            raise NotImplementedError("; ".join(bad))
        return self


SCANNET = HotPathOpts()
