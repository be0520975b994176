"""CPU tests of the training step (sgnerf_amd.train):

* loss and gradients of `loss_from_query` equal autograd through the oracle's torch
  restatement (oracle/agg_ref.py, pinned to the reference's PointAggregator/ray_march
  goldens) on the same oracle query;
* a few optimisation steps on a fixed batch lower the loss;
* world-size-2 gloo: the bucketed gradient all-reduce leaves identical parameters on both
  ranks, equal to one Adam step on the mean of the two ranks' gradients."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import agg_ref
import oracle_query as oq
from helpers import hyper_for, make_view, small_room, t_table
from sgnerf_amd.opts import HotPathOpts
from sgnerf_amd.train import PointParams, Trainer, ViewMLP, loss_from_query
from sgnerf_amd.weights import init_mlp

O = HotPathOpts(SR=24)


def _setup(seed=0, h=12, w=16, yaw=30.0):
    pc = small_room(60_000, seed=seed)
    view = make_view(h, w, yaw=yaw, pitch=-8.0)
    hy = hyper_for(pc, O)
    q = oq.OracleGrid(pc.xyz, hy, O).query(view.campos, view.raydir, t_table(O).numpy())
    R = view.raydir.shape[0]
    rr, ss = np.nonzero(np.arange(O.SR)[None, :] < q["ray_ns"][:, None])
    ray_ns = torch.from_numpy(q["ray_ns"]).long()
    qd = {"ray_ns": ray_ns, "ray_soff": torch.cumsum(ray_ns, 0) - ray_ns, "samp_ray": torch.from_numpy(rr).long(),
          "samp_locw": torch.from_numpy(q["loc_w"][rr, ss]), "pidx": torch.from_numpy(q["pidx"][rr, ss]).long()}
    mlp = init_mlp(seed, bias_std=0.01)
    mlp["alpha_branch.0.bias"] = mlp["alpha_branch.0.bias"] + 100.0
    gt = torch.rand(R, 3, generator=torch.Generator().manual_seed(seed))
    return pc, view, qd, mlp, gt


def _oracle_loss(pc, view, qd, mlp, gt):
    """Autograd through oracle/agg_ref.py (+ the same loss formula)."""
    pts = {k: torch.from_numpy(getattr(pc, k)).clone().requires_grad_(k != "xyz")
           for k in ("xyz", "embedding", "color", "dir", "conf")}
    m = {k: v.clone().requires_grad_(True) for k, v in mlp.items()}
    campos, rot, raydir = (torch.from_numpy(view.campos), torch.from_numpy(view.camrotc2w),
                           torch.from_numpy(view.raydir))
    feat, _ = agg_ref.aggregate(pts, m, campos, rot, raydir, qd["samp_ray"], qd["samp_locw"], qd["pidx"])
    nnb = (qd["pidx"] >= 0).sum(-1)
    R = raydir.shape[0]
    fd, vd, ld = agg_ref.densify(R, O.SR, qd["ray_ns"], qd["samp_ray"], qd["samp_locw"], feat, nnb)
    color, _, _ = agg_ref.composite(fd, vd, ld, rot, campos)
    ray_mask = vd.any(-1)
    l_col = torch.mean((color[ray_mask] - gt[ray_mask]) ** 2)
    # zero-one on the dense conf_coefficient of valid rays (clamped index 0 for empty entries)
    S = qd["samp_ray"].shape[0]
    slot = torch.arange(S) - qd["ray_soff"][qd["samp_ray"]]
    pd = torch.full((R, O.SR, O.K), -1, dtype=torch.long)
    pd[qd["samp_ray"], slot] = qd["pidx"]
    cd = pts["conf"][torch.clamp(pd[ray_mask], min=0).reshape(-1), 0]
    val = torch.clamp(torch.clamp(cd, 1e-4, 1.0), 1e-3, 1 - 1e-3)
    l_zo = torch.mean(torch.log(val) + torch.log(1 - val))
    total = l_col + 3e-6 + 1e-4 * l_zo
    total.backward()
    return total, pts, m


def test_loss_and_gradients_match_oracle_autograd():
    pc, view, qd, mlp, gt = _setup()
    ref_total, ref_pts, ref_m = _oracle_loss(pc, view, qd, mlp, gt)
    points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, "cpu")
    net = ViewMLP(mlp)
    total, parts, full, ray_mask = loss_from_query(points, net, qd, torch.from_numpy(view.campos),
                                                   torch.from_numpy(view.camrotc2w), torch.from_numpy(view.raydir),
                                                   gt, O)
    total.backward()
    assert int(ray_mask.sum()) > 0.5 * ray_mask.numel()
    torch.testing.assert_close(total, ref_total, rtol=1e-5, atol=1e-7)
    for name, *_ in [(n,) for n in mlp]:
        g = net.lin[name.rsplit(".", 1)[0].replace(".", "_")]
        g = g.weight.grad if name.endswith("weight") else g.bias.grad
        torch.testing.assert_close(g, ref_m[name].grad, rtol=2e-4, atol=1e-7, msg=name)
    for mine, ref in (("points_embeding", "embedding"), ("points_color", "color"), ("points_dir", "dir"),
                      ("points_conf", "conf")):
        torch.testing.assert_close(getattr(points, mine).grad, ref_pts[ref].grad, rtol=2e-4, atol=1e-7, msg=mine)
    assert float(points.points_embeding.grad.abs().sum()) > 0


def test_steps_lower_the_loss():
    pc, view, qd, mlp, gt = _setup(seed=1)
    points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, "cpu")
    tr = Trainer(points, mlp, O, "cpu", lr=2e-3, plr=5e-3)
    args = (torch.from_numpy(view.campos), torch.from_numpy(view.camrotc2w), torch.from_numpy(view.raydir), 0.1, 8.0,
            gt)
    first = float(tr.step(*args, q=qd)[0]["ray_masked_coarse_raycolor"])
    for _ in range(5):
        last = float(tr.step(*args, q=qd)[0]["ray_masked_coarse_raycolor"])
    assert last < first
    assert tr.step_count == 6


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _dp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        pc, view, qd, mlp, gt = _setup(seed=2, yaw=30.0 + 40.0 * rank)
        points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, "cpu")
        tr = Trainer(points, mlp, O, "cpu", bucket_mb=1)
        tr.step(torch.from_numpy(view.campos), torch.from_numpy(view.camrotc2w), torch.from_numpy(view.raydir),
                0.1, 8.0, gt, q=qd)
        # numpy (pickled by value): shared-memory tensors die with the worker
        q.put((rank, {k: v.detach().numpy().copy() for k, v in tr.mlp_state().items()},
               points.points_embeding.detach().numpy().copy()))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, repr(e), None))
    finally:
        torch.distributed.destroy_process_group()


def test_data_parallel_step_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (a, b)) for r, a, b in [q.get(timeout=300) for _ in range(world)])
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert isinstance(res[r][0], dict), res[r][0]
    # identical parameters on both ranks
    for k in res[0][0]:
        assert np.array_equal(res[0][0][k], res[1][0][k]), k
    assert np.array_equal(res[0][1], res[1][1])
    # == one Adam step on the mean of the two ranks' gradients, computed here
    grads, pgrads = [], []
    for rank in range(world):
        pc, view, qd, mlp, gt = _setup(seed=2, yaw=30.0 + 40.0 * rank)
        points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, "cpu")
        net = ViewMLP(mlp)
        total, *_ = loss_from_query(points, net, qd, torch.from_numpy(view.campos), torch.from_numpy(view.camrotc2w),
                                    torch.from_numpy(view.raydir), gt, O)
        total.backward()
        grads.append([p.grad.clone() for p in net.parameters()])
        pgrads.append(points.points_embeding.grad.clone())
    # the point embedding: one Adam step (plr 2e-3) on the mean of the ranks' dense gradients
    # (the trainer all-gathers only the touched rows)
    pts0 = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, "cpu")
    popt = torch.optim.Adam([pts0.points_embeding], lr=2e-3, betas=(0.9, 0.999))
    pts0.points_embeding.grad = (pgrads[0] + pgrads[1]) / 2
    popt.step()
    assert int((pgrads[0] != 0).any(1).sum()) < pgrads[0].shape[0] // 2  # the exchange really is sparse
    torch.testing.assert_close(torch.from_numpy(res[0][1]), pts0.points_embeding.detach(), rtol=1e-5, atol=1e-7)
    net0 = ViewMLP(init_mlp(2, bias_std=0.01) | {"alpha_branch.0.bias": init_mlp(2, bias_std=0.01)["alpha_branch.0.bias"] + 100.0})
    opt = torch.optim.Adam(net0.parameters(), lr=5e-4, betas=(0.9, 0.999))
    for p, g0, g1 in zip(net0.parameters(), *grads):
        p.grad = (g0 + g1) / 2
    opt.step()
    ref = net0.state()
    for k in ref:
        torch.testing.assert_close(torch.from_numpy(res[0][0][k]), ref[k], rtol=1e-5, atol=1e-7, msg=k)


@pytest.mark.gpu
def test_gpu_training_gradients_match_cpu():
    """The device backward (HIP query + device autograd) == the CPU backward on the oracle query."""
    pc, view, qd, mlp, gt = _setup(seed=3)
    dev = "cuda:0"
    points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, dev)
    tr = Trainer(points, mlp, O, dev)
    d = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    parts, full, ray_mask = tr.backward(d(view.campos), d(view.camrotc2w), d(view.raydir), 0.1, 8.0, gt.to(dev))
    pc_points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, "cpu")
    tr_cpu = Trainer(pc_points, mlp, O, "cpu")
    parts_c, full_c, mask_c = tr_cpu.backward(torch.from_numpy(view.campos), torch.from_numpy(view.camrotc2w),
                                              torch.from_numpy(view.raydir), 0.1, 8.0, gt, q=qd)
    assert torch.equal(ray_mask.cpu(), mask_c)
    torch.testing.assert_close(parts["total"].cpu(), parts_c["total"], rtol=1e-5, atol=1e-7)
    for a, b in zip(tr.net_params + tr.point_params, tr_cpu.net_params + tr_cpu.point_params):
        torch.testing.assert_close(a.grad.cpu(), b.grad, rtol=1e-3, atol=1e-7)
    tr.apply()
    assert tr.step_count == 1


@pytest.mark.parametrize("seed", [4, 9])
def test_flat_pack_f32_codes_match_host_pack(seed):
    """train_hip._PackerF32's per-element codes (what sgn_pack_scaled_f32 decodes on the device),
    decoded here on the CPU with the kernel's rules, against the C packer (pack_blob_x3 into host
    memory), byte for byte; the layers' weights span several binades so every layer gets its own
    shift.  The device kernel itself: tests/test_train_gpu.py::test_device_pack_f32_matches_host_pack."""
    from sgnerf_amd.train_hip import FlatMLP, _PackerF32
    from sgnerf_amd.weights import LAYERS, init_mlp, pack_mlp
    mlp = init_mlp(seed, bias_std=0.05)
    for i, (n, *_) in enumerate(LAYERS):
        mlp[n + ".weight"] = mlp[n + ".weight"] * 2.0 ** (3 - i)
    flat = FlatMLP(mlp, "cpu")
    pk = _PackerF32("cpu", flat)
    f = flat.flat.detach()
    sh = torch.zeros(16)
    for li, (a, b) in enumerate(pk.wspan):
        m = f[a:b].abs().max()
        sh[li] = float(14 - int(torch.frexp(m)[1])) if bool(m > 0) and bool(torch.isfinite(m)) else 0.0
    c = pk.code16.long()
    ok = c >= 0
    v = torch.where(ok, f[torch.where(ok, c & 0x3FFFFF, 0)] * torch.exp2(sh[(c >> 22) & 15]), 0.0)
    hi = v.half()
    out16 = torch.where(ok & ((c >> 26) & 1 == 1), (v - hi.float()).half(), hi)
    c = pk.code32.long()
    idx, l, k = c & 0x3FFFFF, (c >> 22) & 15, c >> 26
    y = torch.zeros(c.shape)
    y = torch.where((k == pk.YK_W) | (k == pk.YK_B), f[idx], y)
    y = torch.where(k == pk.YK_BS, f[idx] * torch.exp2(sh[l]), y)
    y = torch.where(k == pk.YK_INV, torch.exp2(-sh[l]), y)
    y = torch.where(k == pk.YK_ONE, torch.ones_like(y), y)
    y = torch.where(k == pk.YK_WINV, f[idx] * torch.exp2(-sh[3]), y)
    blob = torch.zeros(pk.total, dtype=torch.uint8)
    blob[:pk.n16b].view(torch.float16).copy_(out16)
    blob[pk.n16b:pk.n16b + 4 * y.numel()].view(torch.float32).copy_(y)
    host = pack_mlp(mlp, "cpu", precision="f32")
    assert blob.numel() == host.numel()
    bad = torch.nonzero(blob != host).reshape(-1)
    assert bad.numel() == 0, bad[:20]
