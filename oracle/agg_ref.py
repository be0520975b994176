"""TEST INFRASTRUCTURE ONLY -- torch fp32 restatement of the aggregator,
ray_dist and alpha composite, on the sample-major query output.

Follows, operation for operation:
  NeuralPoints.forward gather / w2pers     models/neural_points/neural_points.py:838-850, :956-967
  querier w2pers of sample positions       models/neural_points/query_point_indices_worldcoords.py:125-132
  PointAggregator.forward (agg_dist_pers=20, linear kernel, weight norm, conf clamp)
                                           models/aggregators/point_aggregators.py:868-959, :494-502, :863-865
  viewmlp (agg_intrp_order=2)              models/aggregators/point_aggregators.py:561-786
    + SG block2_bpnet                        models/aggregators/point_aggregators.py:345-354, :629-636
  positional_encoding                      models/helpers/networks.py:175-192
  ray_dist                                 models/neural_points_volumetric_model.py:569-577
  ray_march + alpha_blend + radiance       models/rendering/diff_ray_marching.py:509-555,
                                           models/rendering/diff_render_func.py:36-49
  fill_invalid (white background)          models/neural_points_volumetric_model.py:158-195

Pinned against tests/golden/reference_aggregator.npz (outputs of the imported
reference PointAggregator / ray_march).  Only tests/, smoke() and bench.py's
cpu_baseline leg use this module.
"""
import torch
import torch.nn.functional as F

LAYERS = ["block1.0", "block1.2", "block3.0", "block3.2", "alpha_branch.0", "color_branch.0",
          "color_branch.2", "color_branch.4", "color_branch.6"]


def positional_encoding(positions, freqs, ori=False):
    freq_bands = (2 ** torch.arange(freqs).float()).to(positions.device)
    ori_c = positions.shape[-1]
    pts = (positions[..., None] * freq_bands).reshape(positions.shape[:-1] + (freqs * positions.shape[-1],))
    if ori:
        pts = torch.cat([positions, torch.sin(pts), torch.cos(pts)], dim=-1).reshape(pts.shape[:-1] + (pts.shape[-1] * 2 + ori_c,))
    else:
        pts = torch.stack([torch.sin(pts), torch.cos(pts)], dim=-1).reshape(pts.shape[:-1] + (pts.shape[-1] * 2,))
    return pts


def w2pers_points(xyz, rot, campos):
    shift = xyz[None, ...] - campos[:, None, :]
    c = torch.sum(rot[:, None, :, :] * shift[:, :, :, None], dim=-2)
    return torch.stack([c[:, :, 0] / c[:, :, 2], c[:, :, 1] / c[:, :, 2], c[:, :, 2]], dim=-1)


def w2pers_samples(loc_w, rot, campos):
    shift = loc_w - campos[:, None, :]
    c = torch.sum(shift[..., None, :] * torch.transpose(rot, 1, 2)[:, None, None, ...], dim=-1)
    return torch.stack([c[..., 0] / c[..., 2], c[..., 1] / c[..., 2], c[..., 2]], dim=-1)


def _lin(mlp, name, x):
    return F.linear(x, mlp[name + ".weight"], mlp[name + ".bias"])


def _lrelu(x):
    return F.leaky_relu(x, 0.01)


def aggregate(points, mlp, campos, rot, raydir, samp_ray, samp_locw, pidx):
    """points: dict xyz[N,3], embedding[N,32], color[N,3], dir[N,3], conf[N,1] (fp32 tensors),
    optional bpnet[N,96] (SG);
    mlp: reference state_dict names (aggregator.* prefix stripped);
    campos [3], rot [3,3], raydir [R,3]; per sample: samp_ray [S], samp_locw [S,3], pidx [S,K].
    Returns feat [S,4] = (alpha, r, g, b) (zeros for samples without neighbours) and
    weight*conf [S,K]."""
    S, K = pidx.shape
    campos = campos.reshape(1, 3)
    rot = rot.reshape(1, 3, 3)
    mask = pidx >= 0
    flat = torch.clamp(pidx, min=0).reshape(-1).long()
    xyz = points["xyz"][flat].view(S, K, 3)
    pers_all = w2pers_points(points["xyz"], rot, campos)[0]
    pers = pers_all[flat].view(S, K, 3)
    emb = points["embedding"][flat].view(S, K, -1)
    color = points["color"][flat].view(S, K, 3)
    pdir = points["dir"][flat].view(S, K, 3)
    conf = points["conf"][flat].view(S, K, 1)
    loc_w = samp_locw.view(S, 3)
    loc = w2pers_samples(loc_w[None, None], rot, campos)[0, 0]
    # point_aggregators.py:917-925
    xd = pers[..., 0] * pers[..., 2] - loc[:, None, 0] * loc[:, None, 2]
    yd = pers[..., 1] * pers[..., 2] - loc[:, None, 1] * loc[:, None, 2]
    zd = pers[..., 2] - loc[:, None, 2]
    dists = torch.cat([xyz - loc_w[:, None, :], torch.stack([xd, yd, zd], dim=-1)], dim=-1)
    # linear kernel :494-502, normalisation :946-947, conf clamp :951-953
    weight = mask / torch.clamp(torch.norm(dists[..., :3], dim=-1), min=1e-6)
    weight = weight / torch.clamp(torch.sum(weight, dim=-1, keepdim=True), min=1e-8)
    conf_coef = torch.clamp(conf[..., 0], 0.0001, 1)
    weight = weight * conf_coef
    ray_valid = torch.any(mask, dim=-1)
    v = raydir.reshape(-1, 3)[samp_ray.long()] @ torch.eye(3, device=raydir.device)
    vpe = positional_encoding(v, 4, ori=True)
    ori_v, vpe = vpe[..., :3], vpe[..., 3:]
    # viewmlp :594-653 on the valid (sample, neighbour) rows
    m = mask.reshape(-1)
    d6 = dists.reshape(-1, 6)[m]
    d6 = positional_encoding(d6, 5)
    f = emb.reshape(S * K, -1)[m]
    f = torch.cat([f, positional_encoding(f, 3)], dim=-1)
    f = torch.cat([f, d6], dim=-1)
    f = _lrelu(_lin(mlp, "block1.2", _lrelu(_lin(mlp, "block1.0", f))))
    if "block2_bpnet.0.weight" in mlp:
        # SG block2_bpnet (point_aggregators.py:629-636): [h | gathered BPNet embedding] when the
        # embedding is given (semantic_guidance, neural_points.py:970-972), then Linear + LReLU
        if points.get("bpnet") is not None:
            f = torch.cat([f, points["bpnet"][flat].view(S * K, -1)[m]], dim=-1)
        f = _lrelu(_lin(mlp, "block2_bpnet.0", f))
    sd = pdir.reshape(-1, 3)[m]
    ov = ori_v[:, None, :].repeat(1, K, 1).reshape(-1, 3)[m]
    f = torch.cat([f, color.reshape(-1, 3)[m], sd - ov, torch.sum(sd * ov, dim=-1, keepdim=True)], dim=-1)
    f = _lrelu(_lin(mlp, "block3.2", _lrelu(_lin(mlp, "block3.0", f))))
    # alpha + K-blend :743-770
    alpha = F.softplus(_lin(mlp, "alpha_branch.0", f) - 1)
    ah = torch.zeros(S * K, 1, device=pidx.device)
    ah[m] = alpha
    alpha = torch.sum(ah.view(S, K, 1) * weight[..., None], dim=-2)[ray_valid]
    fh = torch.zeros(S * K, f.shape[-1], device=pidx.device)
    fh[m] = f
    fs = torch.sum(fh.view(S, K, -1) * weight[..., None], dim=-2)[ray_valid]
    c = torch.cat([fs, vpe[ray_valid]], dim=-1)
    c = _lrelu(_lin(mlp, "color_branch.0", c))
    c = _lrelu(_lin(mlp, "color_branch.2", c))
    c = _lrelu(_lin(mlp, "color_branch.4", c))
    c = torch.sigmoid(_lin(mlp, "color_branch.6", c)) * (1 + 2 * 0.001) - 0.001
    out = torch.zeros(S, 4, device=pidx.device)
    out[ray_valid] = torch.cat([alpha, c], dim=-1)
    return out, weight


def composite(feat_dense, valid_dense, loc_w_dense, rot, campos, vsize_z=0.008, raydist_mode_unit=1,
              bg=(1.0, 1.0, 1.0)):
    """Reference ray_dist + ray_march on dense [R, SR] slots (empty slots: loc_w = 0,
    as sample_loc_tensor's zero fill, worldcoords.py:835).  Returns ray colour [R,3],
    opacity [R,SR], background transmission [R]."""
    loc = w2pers_samples(loc_w_dense[None], rot.reshape(1, 3, 3), campos.reshape(1, 3))
    ray_dist = torch.cummax(loc[..., 2], dim=-1)[0]
    ray_dist = torch.cat([ray_dist[..., 1:] - ray_dist[..., :-1],
                          torch.full((ray_dist.shape[0], ray_dist.shape[1], 1), vsize_z, device=loc.device)], dim=-1)
    m = ray_dist < 1e-8
    if raydist_mode_unit > 0:
        m = torch.logical_or(m, ray_dist > 2 * vsize_z)
    m = m.to(torch.float32)
    ray_dist = ray_dist * (1.0 - m) + m * vsize_z
    ray_dist = ray_dist * valid_dense[None].float()
    feats = feat_dense[None]
    point_color = feats[..., 1:4]
    sigma = feats[..., 0] * valid_dense[None].float()
    opacity = 1 - torch.exp(-sigma * ray_dist)
    acc = torch.cumprod(1. - opacity + 1e-10, dim=-1)
    bg_t = acc[:, :, [-1]]
    acc = torch.cat([torch.ones(opacity.shape[0:2] + (1,), device=acc.device), acc[:, :, :-1]], dim=-1)
    w = (opacity * acc)[..., None]
    color = torch.sum(point_color * w, dim=-2) + torch.as_tensor(bg, dtype=torch.float32, device=bg_t.device).view(1, 1, 3) * bg_t
    return color[0], opacity[0], bg_t[0, :, 0]


def densify(R, SR, ray_ns, samp_ray, samp_locw, feat, nnb):
    """sample-major -> dense [R, SR] (feat, valid, loc_w)."""
    S = samp_ray.shape[0]
    soff = torch.cumsum(ray_ns, 0) - ray_ns
    dev = feat.device
    slot = torch.arange(S, device=dev) - soff[samp_ray.long()]
    fd = torch.zeros(R, SR, 4, device=dev)
    vd = torch.zeros(R, SR, dtype=torch.bool, device=dev)
    ld = torch.zeros(R, SR, 3, device=dev)
    fd[samp_ray.long(), slot] = feat
    vd[samp_ray.long(), slot] = nnb > 0
    ld[samp_ray.long(), slot] = samp_locw
    return fd, vd, ld


def render(points, mlp, campos, rot, raydir, q, SR, vsize_z=0.008, bg=(1.0, 1.0, 1.0)):
    """Full oracle render from an oracle query result dict (oracle_query.OracleGrid.query).
    Returns colour [R,3] (background for invalid rays), ray_mask [R], feat dense [R,SR,4]."""
    import numpy as np
    R = raydir.shape[0]
    ray_ns = torch.from_numpy(q["ray_ns"]).long()
    rr, ss = np.nonzero(np.arange(SR)[None, :] < q["ray_ns"][:, None])
    samp_ray = torch.from_numpy(rr)
    samp_locw = torch.from_numpy(q["loc_w"][rr, ss])
    pidx = torch.from_numpy(q["pidx"][rr, ss])
    feat, weight = aggregate(points, mlp, campos, rot, raydir, samp_ray, samp_locw, pidx)
    nnb = (pidx >= 0).sum(-1)
    fd, vd, ld = densify(R, SR, ray_ns, samp_ray, samp_locw, feat, nnb)
    color, opacity, bg_t = composite(fd, vd, ld, rot, campos, vsize_z=vsize_z, bg=bg)
    ray_mask = vd.any(-1)
    full = torch.as_tensor(bg, dtype=torch.float32).view(1, 3).repeat(R, 1)
    full[ray_mask] = color[ray_mask]
    return full, ray_mask, fd, opacity, bg_t
