"""Training step of the per-ray path, first version.

One step on a batch of rays, as the reference's `optimize_parameters` does it
(models/base_rendering_model.py:534-664, models/mvs_points_volumetric_model.py:47-141):

  query        HIP (`sgn_query`, bit-exact vs the oracle): shading samples + neighbour
               indices; no gradient flows through it (the reference's is pycuda, also
               non-differentiable)
  aggregator   NeuralPoints gather + PointAggregator / viewmlp (point_aggregators.py:868-959,
               :561-786) as differentiable torch ops on the device: the GEMMs run on the ROCm
               BLAS libraries, gradients reach the MLP and the per-point parameters
               (points_embeding, points_color, points_dir, points_conf) through the gather;
               conf goes through the straight-through clamp (:863-865)
  composite    ray_dist + ray_march (neural_points_volumetric_model.py:569-631,
               diff_ray_marching.py:509-555)
  losses       ray-masked colour MSE (`ray_masked_coarse_raycolor`, weight 1) + zero-one on
               `conf_coefficient` (weight 1e-4, zero_epsilon 1e-3), ScanNet opt.txt:33-34,202-204
  update       data-parallel: gradients all-reduced (mean) over ranks in flat buckets
               (RCCL over xGMI; gloo in the CPU tests), then two Adam groups
               (net lr 5e-4, points plr 2e-3, betas (0.9, 0.999)) with the reference's
               iter_exponential_decay schedule (lr * 0.1 ** (step / 1e6))

The forward used for rendering stays the fused HIP kernels; this module is the
differentiable restatement needed for gradients until the HIP backward lands.  `loss_from_query`
takes a query result (sample-major) so the same code runs on CPU with the oracle's query in
the parity tests.
"""
import math
import os

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from .opts import HotPathOpts
from .weights import LAYERS, strip_prefix


def _pe(x, freqs, ori=False):
    """positional_encoding (networks.py:175-192)."""
    bands = (2.0 ** torch.arange(freqs, device=x.device, dtype=x.dtype))
    p = (x[..., None] * bands).reshape(x.shape[:-1] + (freqs * x.shape[-1],))
    if ori:
        return torch.cat([x, torch.sin(p), torch.cos(p)], dim=-1)
    return torch.stack([torch.sin(p), torch.cos(p)], dim=-1).reshape(p.shape[:-1] + (p.shape[-1] * 2,))


class ViewMLP(nn.Module):
    """The ScanNet viewmlp parameters under the reference names (block1.0.weight, ...)."""

    def __init__(self, state):
        super().__init__()
        state = strip_prefix(state)
        self.lin = nn.ModuleDict()
        for name, o, i, _ in LAYERS:
            m = nn.Linear(i, o)
            with torch.no_grad():
                m.weight.copy_(torch.as_tensor(state[name + ".weight"]))
                m.bias.copy_(torch.as_tensor(state[name + ".bias"]))
            self.lin[name.replace(".", "_")] = m

    def f(self, name, x):
        return self.lin[name.replace(".", "_")](x)

    def w(self, name):
        return self.lin[name.replace(".", "_")].weight

    def b(self, name):
        return self.lin[name.replace(".", "_")].bias

    def state(self):
        out = {}
        for name, *_ in LAYERS:
            m = self.lin[name.replace(".", "_")]
            out[name + ".weight"] = m.weight.detach()
            out[name + ".bias"] = m.bias.detach()
        return out


class PointParams(nn.Module):
    """Trainable neural-point parameters (neural_points.py:370-414 names)."""

    def __init__(self, xyz, embedding, color, dir, conf, device):
        super().__init__()
        f = dict(dtype=torch.float32, device=device)
        self.register_buffer("xyz", torch.as_tensor(xyz).to(**f).reshape(-1, 3).contiguous())
        n = self.xyz.shape[0]
        self.points_embeding = nn.Parameter(torch.as_tensor(embedding).to(**f).reshape(n, -1).clone())
        self.points_color = nn.Parameter(torch.as_tensor(color).to(**f).reshape(n, 3).clone())
        self.points_dir = nn.Parameter(torch.as_tensor(dir).to(**f).reshape(n, 3).clone())
        self.points_conf = nn.Parameter(torch.as_tensor(conf).to(**f).reshape(n, 1).clone())


def _w2pers(p, rot, campos):
    c = (p - campos) @ rot  # c_j = sum_i R[i][j] (p_i - campos_i)  (neural_points.py:845-850)
    return torch.stack([c[..., 0] / c[..., 2], c[..., 1] / c[..., 2], c[..., 2]], dim=-1)


class _SavedLinear(torch.autograd.Function):
    """z = x W^T + b whose forward value was computed elsewhere (the HIP fp32-faithful row kernel,
    k_rows16's save mode) and is passed in; the backward is the plain fp32 one: dx = dz W,
    dW = dz^T x, db = sum dz."""

    @staticmethod
    def forward(ctx, x, w, b, z):
        ctx.save_for_backward(x, w)
        return z.clone()

    @staticmethod
    def backward(ctx, gz):
        x, w = ctx.saved_tensors
        return gz @ w, _dw_rows(gz, x), gz.sum(0), None


DW_CHUNK_F32 = int(os.environ.get("SGN_DW_CHUNK_F32", "4096"))  # rows per split-K batch (0: one plain GEMM)


class _LinearRows(torch.autograd.Function):
    """F.linear whose weight gradient is the split-K _dw_rows (same fp32 math, other grid)."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        return F.linear(x, w, b)

    @staticmethod
    def backward(ctx, gz):
        x, w = ctx.saved_tensors
        return gz @ w, _dw_rows(gz, x), gz.sum(0)


class _LinearSink(torch.autograd.Function):
    """z = x W^T + b (or the z computed elsewhere, passed in a one-element list) whose weight and
    bias gradients the backward hands to `sink(gz, x)` -- which adds them into the trainer's flat
    gradient -- instead of returning them through autograd (autograd through views of a flat
    parameter zero-fills a full-size gradient per view, copies the slice in and adds it)."""

    @staticmethod
    def forward(ctx, x, w, b, sink, zbox):
        ctx.save_for_backward(x, w)
        ctx.sink = sink
        return zbox[0] if zbox is not None else F.linear(x, w, b)

    @staticmethod
    def backward(ctx, gz):
        x, w = ctx.saved_tensors
        gz = gz.contiguous()
        ctx.sink(gz, x)
        return (gz @ w if ctx.needs_input_grad[0] else None), None, None, None, None


def _linear(mlp, name, x, z=None, split=False):
    """One aggregator layer: through the mlp's gradient sink when it has one (the HIP trainer's flat
    parameter), else _SavedLinear (z given) / _LinearRows (split-K dW) / nn.Linear."""
    sink = mlp.grad_sink(name) if hasattr(mlp, "grad_sink") else None
    if sink is not None:
        return _LinearSink.apply(x, mlp.w(name).detach(), mlp.b(name).detach(), sink, None if z is None else [z])
    if z is not None:
        return _SavedLinear.apply(x, mlp.w(name), mlp.b(name), z)
    if split:
        return _LinearRows.apply(x, mlp.w(name), mlp.b(name))
    return mlp.f(name, x)


def _dw_rows(gz, x, chunk=DW_CHUNK_F32):
    """gz^T x over the row dimension (fp32): the rows in `chunk`-row batches through one batched
    GEMM, the partials summed (a [256 x C] output of a plain GEMM with K = tens of thousands of rows
    occupies a handful of CUs), a ragged tail of rows as one more GEMM."""
    rows = gz.shape[0]
    nb = rows // chunk if chunk > 0 else 0
    if nb <= 1:
        return gz.t() @ x
    body = nb * chunk
    g = torch.bmm(gz[:body].reshape(nb, chunk, gz.shape[1]).transpose(1, 2),
                  x[:body].reshape(nb, chunk, x.shape[1])).sum(0)
    if body < rows:
        g = g + gz[body:].t() @ x[body:]
    return g


def aggregate(points: PointParams, mlp: ViewMLP, campos, rot, raydir, samp_ray, samp_locw, pidx, saved=None,
              rows=None):
    """Differentiable PointAggregator.forward on sample-major neighbours.
    Returns feat [S,4] (alpha, r, g, b; zeros for samples without neighbours), conf_coefficient
    [S,K] (straight-through clamp) and the neighbour mask [S,K].

    saved = (z1, z2, z3): the pre-activations of block1.0, block1.2 and block3.0 per row s * K + k
    ([>= S K, 256] fp32, from sgn_aggregate_train_fwd_f32): those three layers then take their
    forward values from there (_SavedLinear) instead of recomputing them, with the same fp32
    backward.

    rows: the valid rows s * K + k in order (torch.nonzero of pidx >= 0), when the caller has them
    without a host sync (nonzero_static with a device-side count); else computed here (one sync).
    Every masked selection goes through them (index_select / index_copy, no further syncs)."""
    S, K = pidx.shape
    mask = pidx >= 0
    flat = torch.clamp(pidx, min=0).reshape(-1).long()
    xyz = points.xyz[flat].view(S, K, 3)
    pers = _w2pers(xyz, rot, campos)
    loc = _w2pers(samp_locw, rot, campos)
    dists = torch.cat([xyz - samp_locw[:, None, :],
                       torch.stack([pers[..., 0] * pers[..., 2] - loc[:, None, 0] * loc[:, None, 2],
                                    pers[..., 1] * pers[..., 2] - loc[:, None, 1] * loc[:, None, 2],
                                    pers[..., 2] - loc[:, None, 2]], dim=-1)], dim=-1)
    weight = mask / torch.clamp(torch.norm(dists[..., :3], dim=-1), min=1e-6)        # :494-502
    weight = weight / torch.clamp(torch.sum(weight, dim=-1, keepdim=True), min=1e-8)  # :946-947
    conf = torch.index_select(points.points_conf, 0, flat).view(S, K)
    conf_coef = conf - (conf - torch.clamp(conf, 1e-4, 1.0)).detach()                # :863-865
    w = weight * conf_coef
    valid = mask.any(-1)
    v = raydir[samp_ray.long()]
    vpe = _pe(v, 4, ori=True)
    ori_v, vpe = vpe[..., :3], vpe[..., 3:]
    m = mask.reshape(-1)
    if rows is None:
        rows = torch.nonzero(m).reshape(-1)   # the valid rows s * K + k, in the order of m
    fm = flat.index_select(0, rows)  # index_select: its backward is an index_add (atomics), not a sort-based index_put
    emb = torch.index_select(points.points_embeding, 0, fm)
    x = torch.cat([emb, _pe(emb, 3), _pe(dists.reshape(-1, 6).index_select(0, rows), 5)], dim=-1)
    lr_ = lambda t: F.leaky_relu(t, 0.01)  # noqa: E731
    if saved is not None:
        zs = [z.index_select(0, rows) for z in saved]
        lin = lambda name, t, zi: _linear(mlp, name, t, z=zs[zi])  # noqa: E731
    else:
        lin = lambda name, t, zi: _linear(mlp, name, t)  # noqa: E731
    h = lr_(lin("block1.2", lr_(lin("block1.0", x, 0)), 1))
    sd = torch.index_select(points.points_dir, 0, fm)
    ov = ori_v[:, None, :].expand(S, K, 3).reshape(-1, 3).index_select(0, rows)
    h = torch.cat([h, torch.index_select(points.points_color, 0, fm), sd - ov, torch.sum(sd * ov, dim=-1, keepdim=True)], dim=-1)
    h = lr_(_linear(mlp, "block3.2", lr_(lin("block3.0", h, 2)), split=True))
    alpha = F.softplus(mlp.f("alpha_branch.0", h) - 1)
    hk = torch.zeros(S * K, h.shape[-1], device=h.device, dtype=h.dtype).index_copy(0, rows, h)
    ak = torch.zeros(S * K, 1, device=h.device, dtype=h.dtype).index_copy(0, rows, alpha)
    fs = torch.sum(hk.view(S, K, -1) * w[..., None], dim=1)
    a_s = torch.sum(ak.view(S, K, 1) * w[..., None], dim=1)
    c = torch.cat([fs, vpe], dim=-1)
    lin_r = lambda name, t: _linear(mlp, name, t, split=True)  # noqa: E731  (split-K dW)
    c = lr_(lin_r("color_branch.0", c))
    c = lr_(lin_r("color_branch.2", c))
    c = lr_(lin_r("color_branch.4", c))
    c = torch.sigmoid(lin_r("color_branch.6", c)) * (1 + 2 * 0.001) - 0.001
    feat = torch.cat([a_s, c], dim=-1) * valid[:, None]
    return feat, conf_coef, mask


def loss_from_query(points, mlp, q, campos, rot, raydir, gt, opts: HotPathOpts, bg=(1.0, 1.0, 1.0),
                    zero_one_weight=1e-4, zero_eps=1e-3):
    """Reference losses for one batch given a sample-major query result q (dict of tensors:
    ray_ns [R], ray_soff [R], samp_ray [S], samp_locw [S,3], pidx [S,K]).
    Returns (total loss, dict of parts, rendered colour [R,3], ray_mask [R])."""
    campos = campos.reshape(1, 3)
    rot = rot.reshape(3, 3)
    feat, conf_coef, mask = aggregate(points, mlp, campos, rot, raydir, q["samp_ray"], q["samp_locw"], q["pidx"])
    return composite_losses(points, q, feat, mask.sum(-1) > 0, campos, rot, raydir, gt, opts, bg, zero_one_weight,
                            zero_eps)


class _CumprodPositive(torch.autograd.Function):
    """torch.cumprod along the last dim for strictly positive inputs (the transmittance
    factors 1 - o + 1e-10), with the backward torch itself takes when no input is zero
    (reversed cumsum of grad * out, divided by the input) but without torch's device-to-host
    check for zeros, so the step stays free of syncs and can be captured in a HIP graph."""

    @staticmethod
    def forward(ctx, x):
        out = torch.cumprod(x, dim=-1)
        ctx.save_for_backward(x, out)
        return out

    @staticmethod
    def backward(ctx, grad):
        x, out = ctx.saved_tensors
        return (grad * out).flip(-1).cumsum(-1).flip(-1).div(x)


def composite_losses(points, q, feat, valid, campos, rot, raydir, gt, opts: HotPathOpts, bg=(1.0, 1.0, 1.0),
                     zero_one_weight=1e-4, zero_eps=1e-3, s_count=None):
    """ray_dist + ray_march + the reference losses from per-sample features feat [S,4]
    (alpha, r, g, b) and the per-sample validity (>= 1 neighbour).  bg: a constant colour (3
    floats) or the rays' background [R, 3] (the plane model's bg_ray: T_bg * bg_ray + colour).

    s_count (device scalar, optional): only the first s_count of the S sample entries are
    real; the rest (capacity padding, for a graph-captured step with static shapes) are routed
    to a sentinel ray row that is dropped, so the result equals the unpadded call."""
    R = raydir.shape[0]
    SR = opts.SR
    campos = campos.reshape(1, 3)
    rot = rot.reshape(3, 3)
    S = q["samp_ray"].shape[0]
    dev = raydir.device
    sr = q["samp_ray"]          # int32 or int64 indices
    ar = torch.arange(S, device=dev)
    Rd = R
    if s_count is None:
        slot = ar - q["ray_soff"][sr]
    else:
        ok_s = ar < s_count
        sr_c = torch.where(ok_s, sr, 0)
        slot = torch.where(ok_s, ar - q["ray_soff"][sr_c], 0)
        sr = torch.where(ok_s, sr, R)
        Rd = R + 1
    fd = torch.zeros(Rd, SR, 4, device=dev).index_put((sr, slot), feat)[:R]
    vd = torch.zeros(Rd, SR, dtype=torch.bool, device=dev).index_put((sr, slot), valid)[:R]
    ld = torch.zeros(Rd, SR, 3, device=dev).index_put((sr, slot), q["samp_locw"])[:R]
    z = _w2pers(ld, rot, campos)[..., 2]
    cm = torch.cummax(z, dim=-1)[0]
    rd = torch.cat([cm[:, 1:] - cm[:, :-1], torch.full((R, 1), float(opts.vsize[2]), device=dev)], dim=-1)
    msk = rd < 1e-8
    if opts.raydist_mode_unit:
        msk = msk | (rd > 2 * float(opts.vsize[2]))
    msk = msk.float()
    rd = (rd * (1 - msk) + msk * float(opts.vsize[2])) * vd.float()
    sigma = fd[..., 0] * vd.float()
    o = 1 - torch.exp(-sigma * rd)
    acc = _CumprodPositive.apply(1 - o + 1e-10)
    bg_t = acc[:, -1:]
    acc = torch.cat([torch.ones(R, 1, device=dev), acc[:, :-1]], dim=-1)
    if torch.is_tensor(bg):   # per-ray background [R, 3] (inputs['bg_ray'], neural_points_volumetric_model.py:175-177)
        bgv = bg.reshape(R, 3).to(dev, torch.float32)
    else:
        bgv = torch.cat([torch.full((1,), float(b), device=dev) for b in bg])  # no host copy (graph-safe)
    color = torch.sum(fd[..., 1:4] * (o * acc)[..., None], dim=1) + bgv * bg_t
    ray_mask = vd.any(-1)
    full = torch.where(ray_mask[:, None], color, bgv.expand(R, 3))
    # ray_masked_coarse_raycolor (weight 1), ray_miss / coarse (weight 0): each adds 1e-6 (:560)
    # = F.mse_loss(full[ray_mask], gt[ray_mask]) (0 when no ray is valid), as a masked mean so
    # the step issues no host sync (boolean indexing would wait for the mask's count)
    wm = ray_mask.to(full.dtype)[:, None]
    se = (full - gt) ** 2
    l_col = torch.sum(se * wm) / torch.clamp(wm.sum() * 3, min=1.0)
    # ray_miss_coarse_raycolor (:553-563) = mse over the missed rays x their count = their sum / 3;
    # coarse_raycolor = mse over every ray.  Both carry weight 0: logged, and ranked per frame by
    # the probe (mvs_points_volumetric_model.py:157-176), never differentiated.
    with torch.no_grad():
        l_miss = torch.sum(se * (1 - wm)) / 3
        l_all = se.mean()
    # zero_one_loss on conf_coefficient (:607-614) over the reference's dense [R'', SR, K] tensor
    # (point_aggregators.py:951-958): every (slot, k) of a valid ray, where empty slots and masked
    # neighbours read conf at the clamped index 0 (neural_points.py:956-967)
    K = q["pidx"].shape[1]
    pidx = q["pidx"]
    pd = torch.full((Rd, SR, K), -1, dtype=pidx.dtype, device=dev).index_put((sr, slot), pidx)[:R]
    # Empty entries all read conf[0]: gather them as one scalar (its gradient is a reduction)
    # and spread their gather indices, so the index_select backward does not pile every empty
    # entry's atomic add onto point 0.  Invalid rays are weighted out instead of compacted
    # (no host sync); the value is the mean over the valid rays' entries, as in the reference.
    n_pts = points.points_conf.shape[0]
    ok = pd >= 0
    spread = (torch.arange(pd.numel(), device=dev) % n_pts).view(pd.shape)
    cg = torch.index_select(points.points_conf, 0, torch.where(ok, pd, spread).reshape(-1)).view(pd.shape)
    cd = torch.where(ok, cg, points.points_conf[0, 0])
    cc = cd - (cd - torch.clamp(cd, 1e-4, 1.0)).detach()
    val = torch.clamp(cc, zero_eps, 1 - zero_eps)
    wr = ray_mask.to(val.dtype)[:, None, None]
    n_e = wr.sum() * (SR * K)
    l_zo = torch.sum((torch.log(val) + torch.log(1 - val)) * wr) / torch.clamp(n_e, min=1.0)
    total = l_col + 3e-6 + zero_one_weight * l_zo
    return total, {"ray_masked_coarse_raycolor": l_col.detach(), "ray_miss_coarse_raycolor": l_miss,
                   "coarse_raycolor": l_all, "conf_coefficient": l_zo.detach()}, full, ray_mask


def _allreduce_buckets(grads, bucket_elems):
    """Mean of the gradients over ranks, in flat buckets (one collective per bucket; a single
    tensor larger than a bucket is reduced in place)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    n = dist.get_world_size()
    i = 0
    while i < len(grads):
        if grads[i].numel() >= bucket_elems:
            dist.all_reduce(grads[i])
            grads[i] /= n
            i += 1
            continue
        bucket, size = [], 0
        while i < len(grads) and grads[i].numel() < bucket_elems and (not bucket or size + grads[i].numel() <= bucket_elems):
            bucket.append(grads[i])
            size += grads[i].numel()
            i += 1
        flat = torch.cat([g.reshape(-1) for g in bucket])
        dist.all_reduce(flat)
        flat /= n
        off = 0
        for g in bucket:
            g.copy_(flat[off:off + g.numel()].view_as(g))
            off += g.numel()


def touched_rows(pidx, s_count, K, n_points):
    """Points whose gradient a step can change, on the device and without a host sync: the
    neighbours (pidx >= 0) of the first s_count samples, plus point 0 (the conf read of empty
    neighbour slots, train.composite_losses).  Returns (idx [n_points + 1] int64: the touched
    indices in ascending order, then the sentinel n_points; count: 0-d int64 tensor)."""
    dev = pidx.device
    p = pidx.reshape(-1, K)
    ok = (torch.arange(p.shape[0], device=dev) < s_count)[:, None] & (p >= 0)
    touched = torch.zeros(n_points + 1, dtype=torch.bool, device=dev)
    touched.index_fill_(0, torch.where(ok, p, n_points).reshape(-1).long(), True)
    touched[0] = True
    touched[n_points] = False
    pos = torch.cumsum(touched, 0) - 1
    idx = torch.full((n_points + 1,), n_points, dtype=torch.int64, device=dev)
    idx.scatter_(0, torch.where(touched, pos, n_points), torch.arange(n_points + 1, device=dev))
    idx[n_points] = n_points
    return idx, touched.sum()


def gather_counts(count):
    """All-gather one 0-d count per rank into a device tensor [world] (no host sync: the
    caller reads it together with its other per-step counters)."""
    n = dist.get_world_size()
    out = torch.empty(n, dtype=torch.int64, device=count.device)
    dist.all_gather_into_tensor(out, count.reshape(1).to(torch.int64))
    return out


def _allreduce_point_rows(grads, idx=None, counts=None):
    """Mean over ranks of per-point gradients ([N, C_i] tensors sharing N), sparse: each rank
    sends only the rows its rays touched (a 4096-ray batch touches ~50 k of 1.2 M points), as
    an all-gather of (index, row) padded to the largest count; every rank then adds the ranks'
    slices in rank order (indices unique within a slice), so all ranks get identical sums.
    Equals the dense all-reduce up to the order of the fp32 additions; ~30x fewer bytes than
    all-reducing 187 MB of point gradients per step over xGMI at 8 GPUs.

    idx / counts: the touched rows (touched_rows, device) and every rank's count (host ints,
    read in the step's one sync, gather_counts); without them they are derived from the
    non-zero gradient rows here, at the cost of two host syncs.  Every row outside idx must
    hold a zero gradient (true of both sources)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return None
    n = dist.get_world_size()
    dev = grads[0].device
    N = grads[0].shape[0]
    if idx is None:
        touched = torch.zeros(N, dtype=torch.bool, device=dev)
        for g in grads:
            touched |= (g != 0).reshape(g.shape[0], -1).any(1)
        own = torch.nonzero(touched).reshape(-1)
        idx = torch.full((N + 1,), N, dtype=torch.int64, device=dev)
        idx[:own.numel()] = own
        counts = gather_counts(torch.tensor(own.numel(), device=dev)).tolist()
    m = max(max(counts), 1)
    pidx = idx[:m].contiguous()              # own rows, then the sentinel N
    widths = [g.reshape(g.shape[0], -1).shape[1] for g in grads]
    keep = (pidx < N)[:, None]
    safe = torch.clamp(pidx, max=N - 1)
    rows = torch.cat([g.reshape(N, -1).index_select(0, safe) for g in grads], 1)
    rows = torch.where(keep, rows, torch.zeros((), dtype=rows.dtype, device=dev))
    all_idx = torch.empty(n * m, dtype=torch.int64, device=dev)
    all_rows = torch.empty(n * m, rows.shape[1], dtype=rows.dtype, device=dev)
    dist.all_gather_into_tensor(all_idx, pidx)
    dist.all_gather_into_tensor(all_rows, rows)
    all_rows /= n
    all_idx.clamp_(max=N - 1)                # padding rows are zeros: adding them is a no-op
    # in place: the gradient is non-zero only on this rank's own rows, which were just sent;
    # clear them and add every rank's slice in rank order (no dense accumulator, no full pass)
    off = 0
    for g, wdt in zip(grads, widths):
        assert g.is_contiguous()
        g2 = g.view(N, wdt)
        g2.index_fill_(0, safe, 0.0)
        for r in range(n):
            g2.index_add_(0, all_idx[r * m:(r + 1) * m], all_rows[r * m:(r + 1) * m, off:off + wdt])
        off += wdt
    return all_idx   # every rank's rows (duplicates, and padding clamped to N - 1): the rows the step changed


class Trainer:
    """One data-parallel training step per call (config 5: 4096 random rays per rank)."""

    def __init__(self, points: PointParams, mlp_state, opts: HotPathOpts, device, lr=5e-4, plr=2e-3,
                 lr_decay_exp=0.1, lr_decay_iters=1_000_000, bucket_mb=64, querier=None):
        self.device = torch.device(device)
        self.opts = opts
        self.points = points
        self.mlp = ViewMLP(mlp_state).to(self.device)
        self.net_params = list(self.mlp.parameters())
        self.point_params = [points.points_embeding, points.points_color, points.points_dir, points.points_conf]
        self.opt_net = torch.optim.Adam(self.net_params, lr=lr, betas=(0.9, 0.999))
        self.opt_pts = torch.optim.Adam(self.point_params, lr=plr, betas=(0.9, 0.999))
        self.base_lr = (lr, plr)
        self.decay = (lr_decay_exp, lr_decay_iters)
        self.step_count = 0
        self.bucket_elems = bucket_mb * (1 << 20) // 4
        self.querier = querier

    def _query(self, campos, raydir, near, far):
        """HIP query -> sample-major dict (indices carry no gradient)."""
        if self.querier is None:
            from .querier import LightningFastQuerier
            self.querier = LightningFastQuerier(self.device, self.opts)
        res = self.querier.query_samples(self.points.xyz, campos, raydir, near, far)
        S = res.n_samples()
        return {"ray_ns": res.ray_ns[: raydir.shape[0]].long(), "ray_soff": res.ray_soff[: raydir.shape[0]].long(),
                "samp_ray": res.samp_ray[:S].long(), "samp_locw": res.samp_locw[: S * 3].view(S, 3).clone(),
                "pidx": res.pidx[: S * self.opts.K].view(S, self.opts.K).long()}

    def allreduce_grads(self, params):
        _allreduce_buckets([p.grad for p in params if p.grad is not None], self.bucket_elems)

    def _set_lr(self):
        exp, iters = self.decay
        f = exp ** (self.step_count / iters)  # iter_exponential_decay (helpers/networks.py get_scheduler)
        for opt, base in ((self.opt_net, self.base_lr[0]), (self.opt_pts, self.base_lr[1])):
            for g in opt.param_groups:
                g["lr"] = base * f

    def backward(self, campos, rot, raydir, near, far, gt, q=None, bg_ray=None):
        """Forward + backward + gradient all-reduce (no parameter update).  bg_ray: the rays'
        background [R, 3] (plane model) or None (white)."""
        if q is None:
            q = self._query(campos.reshape(3).contiguous(), raydir.reshape(-1, 3).contiguous(), near, far)
        self.opt_net.zero_grad(set_to_none=True)
        self.opt_pts.zero_grad(set_to_none=True)
        bg = (1.0, 1.0, 1.0) if bg_ray is None else bg_ray
        total, parts, full, ray_mask = loss_from_query(self.points, self.mlp, q, campos, rot, raydir, gt, self.opts,
                                                       bg)
        total.backward()
        for p in self.point_params + self.net_params:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        self.allreduce_grads(self.net_params)
        _allreduce_point_rows([p.grad for p in self.point_params])
        parts["total"] = total.detach()
        return parts, full.detach(), ray_mask

    def apply(self):
        self._set_lr()
        self.opt_net.step()
        self.opt_pts.step()
        self.step_count += 1

    def step(self, campos, rot, raydir, near, far, gt, q=None):
        """One optimisation step; returns the loss parts (detached) and the rendered colour."""
        out = self.backward(campos, rot, raydir, near, far, gt, q)
        self.apply()
        return out

    def mlp_state(self):
        return self.mlp.state()


def psnr(mse):
    return -10.0 * math.log10(max(float(mse), 1e-12))
