"""The reference's operator API for the per-ray hot path, on the HIP kernels.

Mirrors, name for name and output for output:

  NeuralPointsRayMarching.forward(inputs: dict) -> dict
        models/neural_points_volumetric_model.py:435-671 (Point-NeRF path, predict_semantic 0)
  NeuralPointsVolumetricModel.fill_invalid(output, input)  (module function here)
        models/neural_points_volumetric_model.py:158-195
  PointAggregator.forward(15 args) -> (decoded [1,R,SR,4], ray_valid, weight, conf_coefficient)
        models/aggregators/point_aggregators.py:868-959
  ray_march(ray_dist, ray_valid, ray_features, render_func, blend_func, bg_color) -> 7-tuple
        models/rendering/diff_ray_marching.py:509-555
  NeuralPoints (point-parameter holder with the reference attribute names)
        models/neural_points/neural_points.py:321-423

Every computation runs in libsgn_hip.so (query, aggregator MLP, composite); torch
is used here only for allocation, reshaping and the index bookkeeping the
reference itself does in torch (compaction by ray_mask, fill_invalid scatter).
There is no CPU fallback: a missing library raises (_lib.lib()).
"""
import ctypes

import torch

from . import _lib
from .opts import HotPathOpts
from .render import HipRenderer, PointTables
from .weights import mlp_variant, pack_mlp, strip_prefix


def _bg_tuple(bg_color, opts):
    """bg_color input ([1,3] tensor, 3 floats or None) -> host floats (one tiny copy)."""
    if bg_color is None:
        return (1.0, 1.0, 1.0) if opts.bg_color == "white" else (0.0, 0.0, 0.0)
    if torch.is_tensor(bg_color):
        bg_color = bg_color.detach().reshape(-1)[:3].cpu().tolist()
    return tuple(float(x) for x in bg_color)


def _scalar(x):
    if torch.is_tensor(x):
        return float(x.reshape(-1)[0].item())
    try:
        return float(x)
    except TypeError:
        return float(x[0])


# ----------------------------------------------------------------------------------
class NeuralPoints:
    """Neural point parameters under the reference names (neural_points.py:321-423):
    xyz [N,3], points_embeding [1,N,F], points_color [1,N,3], points_dir [1,N,3],
    points_conf [1,N,1].  `tables()` gives the flat fp32 device view the kernels read;
    it is rebuilt only when a tensor changes (torch version counter).

    The semantic attributes ride along: points_feats [N,3] (the init cloud's RGB in 0..255,
    BPNet's input, scannet_ft_dataset.py:482 / neural_points.py:589-590), points_label [N,1]
    and bpnet_points_embedding [1,N,96] (neural_points.py:653-665)."""

    def __init__(self, xyz, points_embeding, points_color, points_dir, points_conf, device="cuda",
                 points_feats=None, points_label=None, bpnet_points_embedding=None):
        dev = torch.device(device)
        f = dict(dtype=torch.float32, device=dev)
        self.xyz = torch.as_tensor(xyz).to(**f).reshape(-1, 3)
        n = self.xyz.shape[0]
        self.points_embeding = torch.as_tensor(points_embeding).to(**f).reshape(1, n, -1)
        self.points_color = torch.as_tensor(points_color).to(**f).reshape(1, n, 3)
        self.points_dir = torch.as_tensor(points_dir).to(**f).reshape(1, n, 3)
        self.points_conf = torch.as_tensor(points_conf).to(**f).reshape(1, n, 1)
        self.Rw2c = torch.eye(3, **f)
        self.device = dev
        # SG-NeRF semantic attributes (neural_points.py:653-665), set by set_bpnet_feats
        self.bpnet_points_embedding = None  # [1,N,96], detached
        self.points_label = None            # [N,1]
        self.points_label_prob = None
        self.points_feats = None if points_feats is None else torch.as_tensor(points_feats).to(**f).reshape(-1, 3)
        if points_label is not None:
            self.points_label = torch.as_tensor(points_label).to(dev).reshape(-1, 1)
        if bpnet_points_embedding is not None:
            self.bpnet_points_embedding = torch.as_tensor(bpnet_points_embedding).detach().to(**f).reshape(1, n, -1)
        self._tables = None
        self._key = None

    def set_bpnet_feats(self, points_label_prob, points_label, bpnet_points_embedding):
        """neural_points.py:653-665: per-point BPNet labels and (first call only) embedding."""
        self.points_label_prob = points_label_prob
        self.points_label = None if points_label is None else torch.as_tensor(points_label).to(self.device).reshape(-1, 1)
        if bpnet_points_embedding is not None and self.bpnet_points_embedding is None:
            self.bpnet_points_embedding = torch.as_tensor(bpnet_points_embedding).detach().to(
                self.device, torch.float32).reshape(1, self.xyz.shape[0], -1)

    @classmethod
    def from_state_dict(cls, sd, device="cuda", prefix="neural_points."):
        """Reference checkpoint layout (`*_net_ray_marching.pth`: neural_points.xyz, ...;
        neural_points.py:321-386).  points_feats / points_label / bpnet_points_embedding are
        read when the file holds them (the reference requires points_feats, :362; the other
        two are optional here as they are there)."""
        g = lambda k: sd[prefix + k]  # noqa: E731
        o = lambda k: sd.get(prefix + k)  # noqa: E731
        p = cls(g("xyz"), g("points_embeding"), g("points_color"), g("points_dir"), g("points_conf"), device,
                points_feats=o("points_feats"), points_label=o("points_label"),
                bpnet_points_embedding=o("bpnet_points_embedding"))
        if o("Rw2c") is not None:
            p.Rw2c = torch.as_tensor(o("Rw2c")).to(p.device, torch.float32)
        return p

    @classmethod
    def from_cloud(cls, pc, device="cuda"):
        return cls(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, device)

    def state_dict(self, prefix="neural_points."):
        """The reference's keys; the semantic ones only when set (a reference loader reads
        points_feats unconditionally, so checkpoints meant for it need set_points(points_feats=...))."""
        sd = {prefix + k: getattr(self, k) for k in
              ("xyz", "points_embeding", "points_color", "points_dir", "points_conf", "Rw2c")}
        for k in ("points_feats", "points_label", "bpnet_points_embedding"):
            if getattr(self, k) is not None:
                sd[prefix + k] = getattr(self, k)
        return sd

    def _version_key(self):
        ts = (self.xyz, self.points_embeding, self.points_color, self.points_dir, self.points_conf)
        if self.bpnet_points_embedding is not None:
            ts = ts + (self.bpnet_points_embedding,)
        return tuple((t.data_ptr(), tuple(t.shape), t._version) for t in ts)

    def tables(self):
        key = self._version_key()
        if self._tables is None or key != self._key:
            if self.points_embeding.shape[-1] != 32:
                raise NotImplementedError("the MFMA aggregator is built for point_features_dim = 32")
            self._tables = PointTables(self.xyz, self.points_embeding, self.points_color, self.points_dir,
                                       self.points_conf, self.device, self.bpnet_points_embedding)
            self._key = key
        return self._tables

    def set_points(self, xyz, points_embeding, points_color=None, points_dir=None, points_conf=None):
        """neural_points.py:520-572 (replace the cloud; grid is rebuilt on next query)."""
        self.__init__(xyz, points_embeding, points_color if points_color is not None else self.points_color,
                      points_dir if points_dir is not None else self.points_dir,
                      points_conf if points_conf is not None else self.points_conf, self.device)


# ----------------------------------------------------------------------------------
def fill_invalid(output, input, bg_color=None):
    """neural_points_volumetric_model.py:158-195: expand the compacted [1,R'',.] outputs
    of forward() to all R rays (bg colour, background 1, opacity 0, queried_shading 1)."""
    ray_mask = output["ray_mask"]
    B, OR = ray_mask.shape
    keep = torch.nonzero(ray_mask.reshape(-1)).reshape(-1)
    dev = ray_mask.device
    bgT = torch.ones(B, OR, 1, dtype=torch.float32, device=dev)
    bgT[0, keep] = output["coarse_is_background"][0]
    output["coarse_is_background"] = bgT
    output["coarse_mask"] = 1 - bgT
    if bg_color is None:
        bg_color = input.get("bg_color") if isinstance(input, dict) else None
    bg = torch.tensor(_bg_tuple(bg_color, HotPathOpts()), dtype=torch.float32, device=dev)
    rgb = torch.ones(B, OR, 3, dtype=torch.float32, device=dev) * bg
    rgb[0, keep] = output["coarse_raycolor"][0]
    output["coarse_raycolor"] = rgb
    op = output["coarse_point_opacity"]
    full = torch.zeros(B, OR, op.shape[2], dtype=op.dtype, device=dev)
    full[0, keep] = op[0]
    output["coarse_point_opacity"] = full
    qs = output["queried_shading"]
    fq = torch.ones(B, OR, qs.shape[2], dtype=qs.dtype, device=dev)
    fq[0, keep] = qs[0]
    output["queried_shading"] = fq
    return output


def _dense_from_samples(q, vals, R, SR, fill):
    """Sample-major values [S, ...] -> ray-slot dense [R, SR, ...] (slot s of ray r is
    sample ray_soff[r] + s when s < ray_ns[r], `fill` elsewhere)."""
    dev = vals.device
    slot = torch.arange(SR, device=dev, dtype=torch.int64)
    ns = q.ray_ns[:R].long()
    sid = q.ray_soff[:R].long()[:, None] + slot[None, :]
    ok = slot[None, :] < ns[:, None]
    sid = torch.where(ok, sid, torch.zeros_like(sid))
    out = vals[sid.reshape(-1)].reshape((R, SR) + vals.shape[1:])
    fillv = torch.full_like(out, fill)
    okx = ok.reshape((R, SR) + (1,) * (vals.dim() - 1))
    return torch.where(okx, out, fillv)


class NeuralPointsRayMarching:
    """neural_points_volumetric_model.py:382-671 on the HIP path.

    forward(inputs) returns the reference's compacted dict (coarse_raycolor,
    coarse_point_opacity, queried_shading, coarse_is_background, ray_mask and, with
    `return_weights`, weight / blend_weight / conf_coefficient).  render(inputs) is the
    production entry: the same values already expanded by fill_invalid, without the
    compaction round trip and without any host synchronisation."""

    def __init__(self, neural_points: NeuralPoints, aggregator_state, opt=None, device="cuda",
                 return_weights=True):
        self.opts = opt if isinstance(opt, HotPathOpts) else (HotPathOpts.from_opt(opt) if opt is not None
                                                               else HotPathOpts())
        self.opt = opt
        self.neural_points = neural_points
        self.device = torch.device(device)
        self.return_weights = return_weights
        self.renderer = HipRenderer(neural_points.tables(), strip_prefix(aggregator_state), self.opts, self.device)

    def set_aggregator_state(self, state):
        self.renderer.set_mlp(strip_prefix(state))

    def _render(self, inputs, want_weights):
        self.renderer.points = self.neural_points.tables()
        campos = inputs["campos"].reshape(3)
        rot = inputs["camrotc2w"].reshape(3, 3)
        raydir = inputs["raydir"].reshape(-1, 3)
        near = _scalar(inputs["near"]) if "near" in inputs else self.opts.near_plane
        far = _scalar(inputs["far"]) if "far" in inputs else self.opts.far_plane
        # a per-ray background (bgmodel '*plane', set_bg) replaces the constant one: the composite runs
        # without background (ray_march with bg_color None, neural_points_volumetric_model.py:311-312)
        bg = (0.0, 0.0, 0.0) if inputs.get("bg_ray") is not None else _bg_tuple(inputs.get("bg_color"), self.opts)
        pl = rl = None
        if self.opts.semantic_guidance == 1:  # neural_points.py:771-785: labels of the points and of the rays
            if self.neural_points.points_label is None or inputs.get("pixel_label") is None:
                raise ValueError("semantic_guidance = 1 needs neural_points.points_label and inputs['pixel_label']")
            pl = self.neural_points.points_label.reshape(-1).to(self.device, torch.int32).contiguous()
            rl = torch.as_tensor(inputs["pixel_label"]).reshape(-1).to(self.device, torch.int32).contiguous()
        return self.renderer.render(campos, rot, raydir, near, far, want_opacity=True, want_blend=False,
                                    bg=bg, want_weights=want_weights, point_labels=pl, ray_labels=rl,
                                    seconds=inputs.get("seconds")), raydir.shape[0]

    def _weights(self, out, R):
        """weight [R,SR,K], blend_weight [R,SR,1], conf_coefficient [R,SR,K] (dense ray slots)."""
        o, q = self.opts, out.query
        SR, K = o.SR, o.K
        weight = _dense_from_samples(q, out.wnorm.view(-1, K), R, SR, 0.0)
        pidx = _dense_from_samples(q, q.pidx.view(-1, K), R, SR, -1)
        conf = self.renderer.points.conf.reshape(-1)
        # point_aggregators.py:951-953: clamp(conf[clamp(pidx, 0)], 1e-4, 1) (forward value)
        conf_coef = torch.clamp(conf[torch.clamp(pidx, min=0).long()], 1e-4, 1.0)
        return weight, out.blendw[:R, :, None], conf_coef

    def render(self, inputs):
        """Expanded outputs (what fill_invalid(forward(inputs)) gives), no host sync.
        Fresh tensors, as the reference returns (the renderer's buffers are reused)."""
        out, R = self._render(inputs, self.return_weights)
        rgb = out.rgb[None].clone()
        if inputs.get("bg_ray") is not None:   # T_bg * bg_ray + colour (neural_points_volumetric_model.py:114-116)
            bg_ray = torch.as_tensor(inputs["bg_ray"]).to(self.device, torch.float32).reshape(1, R, 3)
            rgb.addcmul_(out.bg_transmission[None, :, None], bg_ray)
        res = {
            "coarse_raycolor": rgb,
            "coarse_point_opacity": out.opacity[None].clone(),
            "coarse_is_background": out.bg_transmission[None, :, None].clone(),
            "queried_shading": (1 - out.ray_mask.float())[None, :, None].expand(1, R, 3).contiguous(),
            "ray_mask": out.ray_mask[None].clone(),
        }
        res["coarse_mask"] = 1 - res["coarse_is_background"]
        if self.return_weights:
            w, bw, cc = self._weights(out, R)
            res["weight"], res["blend_weight"], res["conf_coefficient"] = w[None], bw[None].clone(), cc[None]
        return res

    def forward(self, inputs, **kargs):
        """Reference forward: compacted [1,R'',...] outputs + ray_mask [1,R]."""
        out, R = self._render(inputs, self.return_weights)
        keep = torch.nonzero(out.ray_mask).reshape(-1)
        res = {
            "coarse_raycolor": out.rgb[keep][None],
            "coarse_point_opacity": out.opacity[keep][None],
            "queried_shading": torch.zeros(1, keep.numel(), 3, dtype=torch.float32, device=self.device),
            "coarse_is_background": out.bg_transmission[keep][None, :, None],
            "ray_mask": out.ray_mask[None].clone(),
        }
        if self.return_weights:
            w, bw, cc = self._weights(out, R)
            res["weight"], res["blend_weight"], res["conf_coefficient"] = w[keep][None], bw[keep][None], cc[keep][None]
        return res

    __call__ = forward

    def fill_invalid(self, output, input):
        return fill_invalid(output, input)


# ----------------------------------------------------------------------------------
class PointAggregator:
    """point_aggregators.py:868-959 on pre-gathered neighbour tensors (the sub-boundary
    between NeuralPoints.forward and ray_march).  The gathered records are handed to the
    MFMA aggregator as a point table of R*SR*K rows addressed by their own index, so the
    kernels are the same as on the fused path."""

    def __init__(self, aggregator_state, opt=None, device="cuda"):
        self.opts = opt if isinstance(opt, HotPathOpts) else (HotPathOpts.from_opt(opt) if opt is not None
                                                               else HotPathOpts())
        self.device = torch.device(device)
        state = strip_prefix(aggregator_state)
        self.variant = mlp_variant(state)
        # fp32 arithmetic (the reference's) unless opts say f16
        self.f32 = self.opts.precision == "f32"
        self.packed = pack_mlp(state, self.device, self.opts.precision)
        self.state = state              # fp32 weights for the range fallback's plain-fp32 pack
        self.packed_exact = None

    def forward(self, sampled_color, sampled_label_embedding, sampled_Rw2c, sampled_dir, sampled_conf,
                sampled_embedding, sampled_xyz_pers, sampled_xyz, sample_pnt_mask, sample_loc, sample_loc_w,
                sample_ray_dirs, vsize, grid_vox_sz):
        dev = self.device
        shp = sample_loc_w.shape[:-1]  # [1, R, SR]
        K = sample_pnt_mask.shape[-1]
        if not (1 <= K <= 8):
            raise NotImplementedError("the MFMA aggregator takes K = 1 .. 8 neighbours")
        S = int(torch.tensor(shp).prod().item())
        f = lambda t, c: t.reshape(-1, c).to(device=dev, dtype=torch.float32).contiguous()  # noqa: E731
        mask = sample_pnt_mask.reshape(S, K).to(dev).bool()
        ray_valid = mask.any(-1)
        if S == 0:
            return (torch.zeros(shp + (4,), device=dev), ray_valid.view(shp), None, None)
        rows = torch.arange(S * K, device=dev, dtype=torch.int32).view(S, K)
        pidx = torch.where(mask, rows, torch.full_like(rows, -1))
        order = None
        if self.f32:
            # the f32 row kernel reads a sample's valid neighbours as a prefix of its K slots (as the
            # query writes them); a caller's mask may have holes: move each sample's valid slots to
            # the front (stable, so the K-blend sums them in the reference's slot order; the empty
            # slots only added zeros) and scatter the per-slot outputs back afterwards
            order = torch.argsort((~mask).to(torch.int8), dim=1, stable=True)
            pidx = torch.gather(pidx, 1, order)
        pidx = pidx.contiguous()
        # work list: valid samples first, counts on the device (no host sync)
        work = torch.argsort((~ray_valid).to(torch.int8), stable=True).to(torch.int32)
        counters = torch.zeros(4, dtype=torch.int32, device=dev)
        counters[0] = S
        counters[1] = ray_valid.sum().to(torch.int32)
        nnb = mask.sum(-1).to(torch.int32)
        samp_ray = torch.arange(S, device=dev, dtype=torch.int32)
        xyz, pers = f(sampled_xyz, 3), f(sampled_xyz_pers, 3)
        emb = f(sampled_embedding, 32)
        col, pdir, conf = f(sampled_color, 3), f(sampled_dir, 3), f(sampled_conf, 1)
        locw, loc = f(sample_loc_w, 3), f(sample_loc, 3)
        vdir = f(sample_ray_dirs, 3)
        zero3 = torch.zeros(3, device=dev)
        eye = torch.eye(3, device=dev)
        pt = _lib.PointTables()
        pt.xyz, pt.embedding, pt.color = xyz.data_ptr(), emb.data_ptr(), col.data_ptr()
        pt.dir, pt.conf, pt.n_points = pdir.data_ptr(), conf.data_ptr(), S * K
        pt.campos, pt.camrotc2w, pt.raydir = zero3.data_ptr(), eye.data_ptr(), vdir.data_ptr()
        pt.pers, pt.samp_pers = pers.data_ptr(), loc.data_ptr()
        nl, dim = self.variant
        bp = None
        if dim:  # point_aggregators.py:631-635: [h | sampled_label_embedding] into block2_bpnet
            if sampled_label_embedding is None:
                raise ValueError("block2_bpnet with predict_semantic = 1 needs sampled_label_embedding")
            lab = f(sampled_label_embedding, 96)
            if self.f32:
                bp = lab
            else:
                bp = torch.empty(S * K, 96, dtype=torch.float16, device=dev)
                _lib.check(_lib.lib().sgn_bpnet_pack(_lib.ptr(lab), S * K, 96, _lib.ptr(bp), _lib.stream_handle()),
                           "sgn_bpnet_pack")
        qo = _lib.QueryOut()
        qo.ray_ns = qo.ray_soff = qo.samp_d = nnb.data_ptr()
        qo.samp_ray, qo.samp_nnb, qo.pidx = samp_ray.data_ptr(), nnb.data_ptr(), pidx.data_ptr()
        qo.work, qo.counters, qo.samp_locw = work.data_ptr(), counters.data_ptr(), locw.data_ptr()
        feat = torch.zeros(S, 4, dtype=torch.float32, device=dev)
        wnorm = torch.zeros(S, K, dtype=torch.float32, device=dev)
        L = _lib.lib()
        st = _lib.stream_handle()
        if self.f32:
            # block1.0's per-point part over the gathered rows (each row is its own "point")
            proj = torch.empty(int(L.sgn_point_proj_bytes_f32(S * K)), dtype=torch.uint8, device=dev)
            _lib.check(L.sgn_point_project_f32(ctypes.byref(pt), _lib.ptr(self.packed), _lib.ptr(proj), st),
                       "sgn_point_project_f32")
            ws = torch.empty(int(L.sgn_aggregate_workspace_bytes_f32(S)), dtype=torch.uint8, device=dev)
            _lib.check(L.sgn_aggregate_f32(nl, dim, _lib.ptr(bp), _lib.ptr(proj), ctypes.byref(pt), ctypes.byref(qo), S, K,
                                           _lib.ptr(self.packed), _lib.ptr(feat), None, _lib.ptr(wnorm), _lib.ptr(ws),
                                           ws.numel(), 3, st), "sgn_aggregate_f32")
            # an activation outside fp16 range (the split path's limit, mlp_x3.hip): the same operator on the
            # plain-fp32 path instead (sgn_aggregate_exact; the fp32 reference has no such limit)
            off = int(L.sgn_aggregate_flag_offset_f32(ws.numel()))
            if int(ws[off:off + 4].view(torch.int32).item()) != 0:
                if getattr(self, "packed_exact", None) is None:
                    self.packed_exact = pack_mlp(self.state, dev, "exact")
                _lib.check(L.sgn_aggregate_exact(nl, dim, _lib.ptr(bp), ctypes.byref(pt), ctypes.byref(qo), S, K,
                                                 _lib.ptr(self.packed_exact), _lib.ptr(feat), None, _lib.ptr(wnorm),
                                                 _lib.ptr(ws), ws.numel(), st), "sgn_aggregate_exact")
            wnorm = torch.zeros_like(wnorm).scatter_(1, order, wnorm)   # back to the caller's slot order
        else:
            ws = torch.empty(int(L.sgn_aggregate_workspace_bytes(S)), dtype=torch.uint8, device=dev)
            _lib.check(L.sgn_aggregate_sg(nl, dim, _lib.ptr(bp), None, ctypes.byref(pt), ctypes.byref(qo), S, K,
                                          _lib.ptr(self.packed), _lib.ptr(feat), None, _lib.ptr(wnorm), _lib.ptr(ws),
                                          ws.numel(), 3, st), "sgn_aggregate_sg")
        # point_aggregators.py:951-953 (forward value of the straight-through clamp)
        conf_coef = torch.clamp(sampled_conf.to(dev)[..., 0], 1e-4, 1.0)
        return feat.view(shp + (4,)), ray_valid.view(shp), wnorm.view(shp + (K,)), conf_coef

    __call__ = forward


# ----------------------------------------------------------------------------------
def ray_march(ray_dist, ray_valid, ray_features, render_func=None, blend_func=None, bg_color=None):
    """diff_ray_marching.py:509-555 with radiance_render + alpha_blend (the ScanNet pair,
    diff_render_func.py:36-49), on dense [N, R, SR] inputs.  Returns (ray_color,
    point_color, opacity, acc_transmission, blend_weight, background_transmission,
    background_blend_weight)."""
    if ray_features.shape[-1] != 4:
        raise NotImplementedError("ray_march: radiance render expects [alpha, r, g, b] features")
    N, R, SR = ray_dist.shape
    dev = ray_dist.device
    rd = ray_dist.reshape(-1, SR).float().contiguous()
    rv = ray_valid.reshape(-1, SR).to(torch.uint8).contiguous()
    ft = ray_features.reshape(-1, SR, 4).float().contiguous()
    n = rd.shape[0]
    rgb = torch.empty(n, 3, device=dev)
    opacity = torch.empty(n, SR, device=dev)
    acc = torch.empty(n, SR, device=dev)
    bw = torch.empty(n, SR, device=dev)
    bgT = torch.empty(n, device=dev)
    bg = None
    if bg_color is not None:
        bg = (ctypes.c_float * 3)(*_bg_tuple(bg_color, HotPathOpts()))
    _lib.check(_lib.lib().sgn_ray_march_dense(_lib.ptr(rd), _lib.ptr(rv), _lib.ptr(ft), n, SR, bg, _lib.ptr(rgb),
                                              _lib.ptr(opacity), _lib.ptr(acc), _lib.ptr(bw), _lib.ptr(bgT),
                                              _lib.stream_handle()), "sgn_ray_march_dense")
    T = bgT.view(N, R, 1)
    return (rgb.view(N, R, 3), ray_features[..., 1:4], opacity.view(N, R, SR), acc.view(N, R, SR),
            bw.view(N, R, SR, 1), T, T)
