"""GPU tests of the HIP training path (sgnerf_amd.train_hip).

Gradient parity bar: the forward runs fp16-in / fp32-accumulate MFMA and the backward keeps
fp16 deltas under a power-of-two loss scale, so each gradient tensor must match the fp32
autograd of the torch restatement (train.Trainer on CPU, itself pinned to oracle/agg_ref.py)
within a relative L2 error of 2e-2 for the MLP weights/biases (sums over all rows) and 6e-2
for the per-point parameters (each a sum over the few rows that gather the point, so fp16
rounding and LReLU-mask flips near zero do not average out; measured 2.7-3.6e-2); the loss
within 1e-3 relative and the rendered colour within the north-star 1e-3."""
import ctypes
from dataclasses import replace as dataclasses_replace

import numpy as np
import pytest
import torch

from sgnerf_amd import _lib
from sgnerf_amd.train import PointParams, Trainer
from sgnerf_amd.train_hip import FlatMLP, HipTrainer, _Packer, _PackerF32, grads_named
from sgnerf_amd.weights import LAYERS, init_mlp, pack_mlp
import oracle_query as oq
from helpers import hyper_for, t_table
from test_train_cpu import O, _setup

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
GRAD_TOL_MLP = 2e-2
GRAD_TOL_POINTS = 6e-2
# graph vs eager Adam updates after 3 steps, relative L2 per tensor.  Measured 2e-3..7.3e-2 (the
# eager path against itself: 1e-6..5e-3 across runs, atomic accumulation order).  The padded loss stage sums
# in another order (fp32, ~1e-7), the fp16 deltas of the HIP backward round a few elements the
# other way (gradients then differ by <= 8.5e-5 relative L2), and Adam's m / sqrt(v) turns the
# sign of near-zero gradient components into lr-sized steps.
UPDATE_TOL = 0.1
GRAD_TOL_F32 = 1e-4     # precision "f32": every gradient, relative L2 vs fp32 autograd
# precision "f32" point gradients against the CPU restatement on the ORACLE's query: the near-opaque
# config-5 batch is ill-conditioned -- two fp32 autograd runs of the same restatement on the same query
# (torch GPU vs torch CPU) already differ by 1.1e-3..1.5e-3 in the point gradients (measured), and the
# HIP f32 path measured 1.8e-3 here, 1.1e-3 against torch on the GPU (MLP gradients <= 6.4e-5).
GRAD_TOL_F32_ORACLE_Q = 5e-3
LOSS_CURVE_TOL = 0.05   # HIP vs fp32 torch colour loss, 200 steps, 20-step window means (measured max 0.0064 and 0.023 in two runs: the atomic accumulation order of the point gradients makes runs differ)


def test_device_pack_matches_host_pack():
    mlp = init_mlp(4, bias_std=0.05)
    flat = FlatMLP(mlp, DEV)
    pk = _Packer(DEV)
    blob, tblob = pk.pack(flat.flat)
    host = pack_mlp(mlp, DEV)
    assert torch.equal(blob.cpu(), host.cpu())
    L = _lib.lib()
    ref_t = torch.empty(int(L.sgn_train_tblob_bytes()), dtype=torch.uint8, device=DEV)
    ws = [np.ascontiguousarray(mlp[n + ".weight"].numpy()) for n, *_ in LAYERS[:4]]
    wp = (ctypes.c_void_p * 4)(*[w.ctypes.data for w in ws])
    _lib.check(L.sgn_train_pack_t(wp, _lib.ptr(ref_t), _lib.stream_handle()), "sgn_train_pack_t")
    assert torch.equal(tblob.cpu(), ref_t.cpu())


@pytest.mark.parametrize("seed", [4, 9])
def test_device_pack_f32_matches_host_pack(seed):
    """_PackerF32 (index gathers from the flat parameter, per-layer shifts on the device) against
    sgn_mlp_pack_f32 (pack_blob_x3 on the host), byte for byte; the weights span several binades
    so the shifts differ per layer."""
    mlp = init_mlp(seed, bias_std=0.05)
    for i, (n, *_) in enumerate(LAYERS):
        mlp[n + ".weight"] = mlp[n + ".weight"] * 2.0 ** (3 - i)
    flat = FlatMLP(mlp, DEV)
    blob = _PackerF32(DEV, flat).pack(flat.flat)
    host = pack_mlp(mlp, DEV, precision="f32")
    assert blob.numel() == host.numel()
    assert torch.equal(blob.cpu(), host.cpu())


def _rel(a, b):
    return float(torch.linalg.vector_norm(a.double() - b.double()) / max(torch.linalg.vector_norm(b.double()), 1e-30))


def _grads_vs_fp32(pc, campos, rot, raydir, qd, mlp, gt, precision="f16"):
    """One HIP backward (GPU) and one fp32 torch-autograd backward (train.Trainer on the CPU, on
    the oracle's query of the same rays): the loss, colour and every gradient compared at the
    module's bars (precision "f32": GRAD_TOL_F32 for every tensor).  Returns the per-tensor
    relative L2 errors."""
    points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, DEV)
    tr = HipTrainer(points, mlp, O, DEV, precision=precision)
    d = lambda a: torch.from_numpy(a).to(DEV)  # noqa: E731
    parts, full, ray_mask = tr.backward(d(campos), d(rot), d(raydir), 0.1, 8.0, gt.to(DEV))
    torch.cuda.synchronize()
    pc_points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, "cpu")
    ref = Trainer(pc_points, mlp, O, "cpu")
    parts_c, full_c, mask_c = ref.backward(torch.from_numpy(campos), torch.from_numpy(rot),
                                           torch.from_numpy(raydir), 0.1, 8.0, gt, q=qd)
    assert torch.equal(ray_mask.cpu(), mask_c)
    assert abs(float(parts["total"]) - float(parts_c["total"])) <= 1e-3 * abs(float(parts_c["total"]))
    assert float((full.cpu() - full_c).abs().max()) <= 1e-3  # north-star RGB bound
    g = grads_named(tr)
    ref_g = {}
    for name, *_ in LAYERS:
        m = ref.mlp.lin[name.replace(".", "_")]
        ref_g[name + ".weight"], ref_g[name + ".bias"] = m.weight.grad, m.bias.grad
    for k in ("points_embeding", "points_color", "points_dir", "points_conf"):
        ref_g[k] = getattr(pc_points, k).grad
    worst = {}
    for k, b in ref_g.items():
        e = _rel(g[k].cpu().reshape(b.shape), b)
        worst[k] = e
    print("relative L2 gradient errors:", {k: f"{v:.2e}" for k, v in worst.items()})
    if precision == "f32":
        bad = {k: v for k, v in worst.items() if v > (GRAD_TOL_F32_ORACLE_Q if k.startswith("points_") else GRAD_TOL_F32)}
    else:
        bad = {k: v for k, v in worst.items() if v > (GRAD_TOL_POINTS if k.startswith("points_") else GRAD_TOL_MLP)}
    assert not bad, bad
    return worst, int(ray_mask.sum())


@pytest.mark.parametrize("seed", [3, 5])
def test_hip_training_gradients_match_torch_fp32(seed):
    pc, view, qd, mlp, gt = _setup(seed=seed)
    _grads_vs_fp32(pc, view.campos, view.camrotc2w, view.raydir, qd, mlp, gt)


@pytest.mark.parametrize("seed", [3, 5])
def test_hip_f32_training_gradients_match_torch_fp32(seed):
    """precision "f32": the fp32-faithful HIP forward (k_rows16 save mode) + fp32 backward through
    the saved pre-activations, every gradient within GRAD_TOL_F32 of fp32 autograd."""
    pc, view, qd, mlp, gt = _setup(seed=seed)
    _grads_vs_fp32(pc, view.campos, view.camrotc2w, view.raydir, qd, mlp, gt, precision="f32")


@pytest.mark.parametrize("cfg", ["small", "config5"])
def test_f32_training_matches_fp32_autograd_on_same_query(cfg):
    """precision "f32" against train.Trainer (fp32 torch autograd) on the GPU over the very samples
    the HIP query produced (HipTrainer.last_query): isolates the aggregator's arithmetic from the
    query's (whose sample positions differ from the CPU oracle's in the last bits, which the
    near-opaque config-5 batch amplifies in the point gradients).  The loss and colour within
    GRAD_TOL_F32; every gradient within GRAD_TOL_F32 or, where the batch is ill-conditioned, within
    twice the spread of two fp32 autograd runs (torch on the GPU vs torch on the CPU, same query)."""
    if cfg == "small":
        pc, view, _, mlp, gt = _setup(seed=3)
        raydir = view.raydir
    else:
        pc, view, raydir, _, mlp, gt, _ = _config5()
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(DEV)  # noqa: E731
    points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, DEV)
    tr = HipTrainer(points, mlp, O, DEV, precision="f32")
    parts, full, ray_mask = tr.backward(d(view.campos), d(view.camrotc2w), d(raydir), 0.1, 8.0, gt.to(DEV))
    qd = {k: v.long() if v.dtype == torch.int32 else v for k, v in tr.last_query.items()}
    ref_points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, DEV)
    ref = Trainer(ref_points, mlp, O, DEV)
    parts_c, full_c, mask_c = ref.backward(d(view.campos), d(view.camrotc2w), d(raydir), 0.1, 8.0, gt.to(DEV), q=qd)
    torch.cuda.synchronize()
    assert torch.equal(ray_mask, mask_c)
    assert _rel(full, full_c) <= GRAD_TOL_F32
    assert abs(float(parts["total"]) - float(parts_c["total"])) <= GRAD_TOL_F32 * abs(float(parts_c["total"]))
    # the fp32 noise floor of this batch: the same autograd on the CPU, same query
    cpu_points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, "cpu")
    cpu = Trainer(cpu_points, mlp, O, "cpu")
    cpu.backward(torch.from_numpy(view.campos), torch.from_numpy(view.camrotc2w), torch.from_numpy(raydir),
                 0.1, 8.0, gt, q={k: v.cpu() for k, v in qd.items()})

    def named(trainer, pts):
        out = {}
        for name, *_ in LAYERS:
            m = trainer.mlp.lin[name.replace(".", "_")]
            out[name + ".weight"], out[name + ".bias"] = m.weight.grad, m.bias.grad
        for k in ("points_embeding", "points_color", "points_dir", "points_conf"):
            out[k] = getattr(pts, k).grad
        return out
    ref_g, cpu_g, g = named(ref, ref_points), named(cpu, cpu_points), grads_named(tr)
    worst = {k: _rel(g[k].reshape(b.shape), b) for k, b in ref_g.items()}
    floor = {k: _rel(cpu_g[k], b.cpu()) for k, b in ref_g.items()}
    print(f"{cfg}: relative L2 gradient errors (same query):", {k: f"{v:.2e}" for k, v in worst.items()})
    print(f"{cfg}: fp32 floor, torch GPU vs torch CPU:", {k: f"{v:.2e}" for k, v in floor.items()})
    bad = {k: (v, floor[k]) for k, v in worst.items() if v > max(GRAD_TOL_F32, 2 * floor[k])}
    assert not bad, bad


@pytest.mark.parametrize("K", [4, 1])
def test_f16_training_small_k_matches_fp32_autograd(K):
    """precision "f16" with K < 8 neighbours per sample (rows k < K of a sample read pidx index
    s * K + k, rows k >= K are empty in the forward and the backward): every gradient within the
    f16 bars (GRAD_TOL_MLP / GRAD_TOL_POINTS) of train.Trainer's fp32 autograd on the very samples
    the HIP query produced; colour within the north-star 1e-3."""
    o = dataclasses_replace(O, K=K)
    pc, view, _, mlp, gt = _setup(seed=5)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(DEV)  # noqa: E731
    points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, DEV)
    tr = HipTrainer(points, mlp, o, DEV, precision="f16")
    parts, full, ray_mask = tr.backward(d(view.campos), d(view.camrotc2w), d(view.raydir), 0.1, 8.0, gt.to(DEV))
    qd = {k: v.long() if v.dtype == torch.int32 else v for k, v in tr.last_query.items()}
    assert qd["pidx"].shape[1] == K
    ref_points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, DEV)
    ref = Trainer(ref_points, mlp, o, DEV)
    parts_c, full_c, mask_c = ref.backward(d(view.campos), d(view.camrotc2w), d(view.raydir), 0.1, 8.0, gt.to(DEV),
                                           q=qd)
    torch.cuda.synchronize()
    assert torch.equal(ray_mask, mask_c)
    assert float((full - full_c).abs().max()) <= 1e-3
    assert abs(float(parts["total"]) - float(parts_c["total"])) <= 1e-3 * abs(float(parts_c["total"]))
    g = grads_named(tr)
    worst = {}
    for name, *_ in LAYERS:
        m = ref.mlp.lin[name.replace(".", "_")]
        worst[name + ".weight"] = _rel(g[name + ".weight"], m.weight.grad)
        worst[name + ".bias"] = _rel(g[name + ".bias"], m.bias.grad)
    for k in ("points_embeding", "points_color", "points_dir", "points_conf"):
        worst[k] = _rel(g[k].reshape(getattr(ref_points, k).grad.shape), getattr(ref_points, k).grad)
    print(f"K={K} [f16]: relative L2 gradient errors (same query):", {k: f"{v:.2e}" for k, v in worst.items()})
    bad = {k: v for k, v in worst.items() if v > (GRAD_TOL_POINTS if k.startswith("points_") else GRAD_TOL_MLP)}
    assert not bad, bad


@pytest.mark.parametrize("K", [4, 1])
def test_f32_training_small_k_matches_fp32_autograd(K):
    """precision "f32" with K < 8 neighbours per sample (saved pre-activations at pidx index
    s * K + k): every gradient within GRAD_TOL_F32 of train.Trainer's fp32 autograd on the very
    samples the HIP query produced."""
    o = dataclasses_replace(O, K=K)
    pc, view, _, mlp, gt = _setup(seed=5)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(DEV)  # noqa: E731
    points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, DEV)
    tr = HipTrainer(points, mlp, o, DEV, precision="f32")
    parts, full, ray_mask = tr.backward(d(view.campos), d(view.camrotc2w), d(view.raydir), 0.1, 8.0, gt.to(DEV))
    qd = {k: v.long() if v.dtype == torch.int32 else v for k, v in tr.last_query.items()}
    assert qd["pidx"].shape[1] == K
    ref_points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, DEV)
    ref = Trainer(ref_points, mlp, o, DEV)
    parts_c, full_c, mask_c = ref.backward(d(view.campos), d(view.camrotc2w), d(view.raydir), 0.1, 8.0, gt.to(DEV),
                                           q=qd)
    torch.cuda.synchronize()
    assert torch.equal(ray_mask, mask_c)
    assert _rel(full, full_c) <= GRAD_TOL_F32
    g = grads_named(tr)
    worst = {}
    for name, *_ in LAYERS:
        m = ref.mlp.lin[name.replace(".", "_")]
        worst[name + ".weight"] = _rel(g[name + ".weight"], m.weight.grad)
        worst[name + ".bias"] = _rel(g[name + ".bias"], m.bias.grad)
    for k in ("points_embeding", "points_color", "points_dir", "points_conf"):
        worst[k] = _rel(g[k].reshape(getattr(ref_points, k).grad.shape), getattr(ref_points, k).grad)
    print(f"K={K}: relative L2 gradient errors (same query):", {k: f"{v:.2e}" for k, v in worst.items()})
    bad = {k: v for k, v in worst.items() if v > GRAD_TOL_F32}
    assert not bad, bad


@pytest.mark.parametrize("precision,graph", [("f32", False), ("f16", True), ("f16", False)])
def test_training_with_plane_background_matches_fp32_autograd(precision, graph):
    """A step whose rays carry the plane background model's per-ray colour (inputs['bg_ray'] from
    set_bg, run/train_ft.py:209-218): the loss composites T_bg * bg_ray + colour and its gradient
    flows through T_bg (neural_points_volumetric_model.py:175-177).  Against train.Trainer's fp32
    autograd with the same bg_ray on the very samples the HIP query produced: f32 within
    GRAD_TOL_F32, f16 (captured loss graph and eager) within the f16 bars."""
    pc, view, _, mlp, gt = _setup(seed=3)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(DEV)  # noqa: E731
    R = view.raydir.shape[0]
    bg_ray = torch.rand(1, R, 3, generator=torch.Generator().manual_seed(21)).to(DEV)
    points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, DEV)
    tr = HipTrainer(points, mlp, O, DEV, precision=precision)
    tr.use_graph = graph
    parts, full, ray_mask = tr.backward(d(view.campos), d(view.camrotc2w), d(view.raydir), 0.1, 8.0, gt.to(DEV),
                                        bg_ray=bg_ray)
    qd = {k: v.long() if v.dtype == torch.int32 else v for k, v in tr.last_query.items()}
    ref_points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, DEV)
    ref = Trainer(ref_points, mlp, O, DEV)
    parts_c, full_c, mask_c = ref.backward(d(view.campos), d(view.camrotc2w), d(view.raydir), 0.1, 8.0, gt.to(DEV),
                                           q=qd, bg_ray=bg_ray[0])
    # the white-background loss differs: the plane colour reached the loss
    ref_w = Trainer(PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, DEV), mlp, O, DEV)
    parts_w, _, _ = ref_w.backward(d(view.campos), d(view.camrotc2w), d(view.raydir), 0.1, 8.0, gt.to(DEV), q=qd)
    torch.cuda.synchronize()
    assert torch.equal(ray_mask, mask_c)
    assert torch.equal(full[~ray_mask], bg_ray[0][~ray_mask])
    assert abs(float(parts_w["total"]) - float(parts_c["total"])) > 1e-3 * abs(float(parts_c["total"]))
    tol_c = GRAD_TOL_F32 if precision == "f32" else 1e-3
    assert float((full - full_c).abs().max()) <= tol_c
    assert abs(float(parts["total"]) - float(parts_c["total"])) <= tol_c * abs(float(parts_c["total"]))
    g = grads_named(tr)
    worst = {}
    for name, *_ in LAYERS:
        m = ref.mlp.lin[name.replace(".", "_")]
        worst[name + ".weight"] = _rel(g[name + ".weight"], m.weight.grad)
        worst[name + ".bias"] = _rel(g[name + ".bias"], m.bias.grad)
    for k in ("points_embeding", "points_color", "points_dir", "points_conf"):
        worst[k] = _rel(g[k].reshape(getattr(ref_points, k).grad.shape), getattr(ref_points, k).grad)
    print(f"bg_ray [{precision}, graph {graph}]: relative L2 gradient errors:", {k: f"{v:.2e}" for k, v in worst.items()})
    if precision == "f32":
        bad = {k: v for k, v in worst.items() if v > GRAD_TOL_F32}
    else:
        bad = {k: v for k, v in worst.items() if v > (GRAD_TOL_POINTS if k.startswith("points_") else GRAD_TOL_MLP)}
    assert not bad, bad


def _config5():
    from sgnerf_amd import scene
    pc = scene.synth_room(1_200_000, seed=0)
    yaw, pitch = scene.spiral_yaw_pitch(37, 120)
    view = scene.room_view(800, 800, yaw=yaw + 15.0, pitch=pitch - 5.0)
    g = torch.Generator().manual_seed(2)
    idx = torch.randint(0, 800 * 800, (4096,), generator=g).numpy()
    raydir = np.ascontiguousarray(view.raydir[idx])
    gt = torch.rand(4096, 3, generator=g)
    q = oq.OracleGrid(pc.xyz, hyper_for(pc, O), O).query(view.campos, raydir, t_table(O).numpy())
    rr, ss = np.nonzero(np.arange(O.SR)[None, :] < q["ray_ns"][:, None])
    ray_ns = torch.from_numpy(q["ray_ns"]).long()
    qd = {"ray_ns": ray_ns, "ray_soff": torch.cumsum(ray_ns, 0) - ray_ns, "samp_ray": torch.from_numpy(rr).long(),
          "samp_locw": torch.from_numpy(q["loc_w"][rr, ss]), "pidx": torch.from_numpy(q["pidx"][rr, ss]).long()}
    mlp = init_mlp(0, bias_std=0.01)
    mlp["alpha_branch.0.bias"] = mlp["alpha_branch.0.bias"] + 50.0
    return pc, view, raydir, qd, mlp, gt, len(rr)


@pytest.mark.parametrize("precision", ["f16", "f32"])
def test_config5_batch_gradients_match_torch_fp32(precision):
    """BASELINE config 5 at its workload: one 4096-ray batch (random pixels of a spiral pose of the
    800x800 frame, as bench.py's training key draws them) over the 1.2 M-point synth-room, SR 24,
    the opaque aggregator; HIP backward against fp32 autograd of the torch restatement on the
    oracle's query of the same rays, at the module's gradient bars."""
    pc, view, raydir, qd, mlp, gt, ns = _config5()
    worst, n_valid = _grads_vs_fp32(pc, view.campos, view.camrotc2w, raydir, qd, mlp, gt, precision)
    print(f"config 5 ({precision}): 4096 rays, {n_valid} valid, {ns} samples")
    assert n_valid > 3000


def test_hip_training_steps_lower_loss():
    pc, view, qd, mlp, gt = _setup(seed=1)
    points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, DEV)
    tr = HipTrainer(points, mlp, O, DEV, lr=2e-3, plr=5e-3)
    d = lambda a: torch.from_numpy(a).to(DEV)  # noqa: E731
    losses = []
    for _ in range(8):
        parts, _, _ = tr.step(d(view.campos), d(view.camrotc2w), d(view.raydir), 0.1, 8.0, gt.to(DEV))
        losses.append(float(parts["total"]))
    print("losses", losses)
    assert losses[-1] < losses[0]
    assert tr.step_count == 8


def test_model_plugin_training_surface(tmp_path):
    """The plugin's training surface as run/train_ft.py drives it (setup / set_points ->
    optimize_parameters(total_steps) -> get_current_losses -> update_learning_rate, prune /
    grow with optimizer rebuilds, test() and checkpoints of the trained state): the first
    step equals a HipTrainer step on the same batch and jitter seed, the loss falls over a
    fixed batch, and a checkpoint reloaded into an inference model renders identically."""
    import argparse
    import dataclasses

    from sgnerf_amd.model import LOSS_NAMES, HipPointsVolumetricModel
    pc, view, qd, mlp, gt = _setup(seed=3)
    d = lambda a: torch.from_numpy(a).to(DEV)  # noqa: E731
    opt = argparse.Namespace(SR=24, K=8, gpu_ids=[0], is_train=True, checkpoints_dir=str(tmp_path), name="scene",
                             lr=5e-4, plr=2e-3, lr_decay_exp=0.1, lr_decay_iters=1_000_000, bg_color="white")
    m = HipPointsVolumetricModel()
    m.initialize(opt)
    m.set_points(points_xyz=pc.xyz, points_feats=pc.color * 255.0, points_embedding=pc.embedding,
                 points_color=pc.color, points_dir=pc.dir, points_conf=pc.conf, aggregator_state=mlp)
    m.setup(opt)
    inputs = {"campos": d(view.campos)[None], "raydir": d(view.raydir)[None], "camrotc2w": d(view.camrotc2w)[None],
              "near": torch.tensor([[[0.1]]]), "far": torch.tensor([[[8.0]]]), "gt_image": gt[None].to(DEV)}
    m.set_input(inputs)
    before = m.test()["coarse_raycolor"].clone()
    # reference step: HipTrainer on the same batch, same jitter seed
    tr = HipTrainer(PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, DEV), mlp,
                    dataclasses.replace(O, is_train=1), DEV, precision="f32")   # the plugin's default arithmetic
    assert m.trainer.precision == "f32"
    torch.manual_seed(11)
    parts_ref, _, _ = tr.step(d(view.campos), d(view.camrotc2w), d(view.raydir), 0.1, 8.0, gt.to(DEV))
    torch.manual_seed(11)
    m.optimize_parameters(total_steps=0)
    losses = m.get_current_losses()
    assert set(losses) == set(LOSS_NAMES)
    assert float(losses["total"]) == float(parts_ref["total"])
    lrs = m.update_learning_rate(opt=opt, total_steps=0)
    assert len(lrs) == 2 and abs(lrs[0] - 5e-4 * 0.1 ** (1 / 1_000_000)) < 1e-12
    hist = [float(losses["total"])]
    for step in range(1, 6):
        m.optimize_parameters(total_steps=step)
        hist.append(float(m.get_current_losses()["total"]))
    assert hist[-1] < hist[0], hist
    # test() renders the trained state, and so does a checkpoint reloaded for inference
    after = m.test()["coarse_raycolor"].clone()
    assert not torch.equal(after, before)
    m.save_networks("latest")
    opt_test = argparse.Namespace(**{**vars(opt), "is_train": False, "resume_dir": str(tmp_path / "scene")})
    m2 = HipPointsVolumetricModel()
    m2.initialize(opt_test)
    m2.load_networks("latest")
    m2.set_input(inputs)
    assert torch.equal(m2.test()["coarse_raycolor"], after)
    # prune (run/train_ft.py:878-884) and grow (:916-917), each followed by a training step
    n0 = m.neural_points.xyz.shape[0]
    thresh = float(torch.quantile(m.neural_points.points_conf.reshape(-1), 0.25))
    m.clean_optimizer()
    m.clean_scheduler()
    n_pruned = m.prune_points(thresh)
    m.setup_optimizer(opt)
    m.init_scheduler(6, opt)
    assert n_pruned > 0 and m.neural_points.xyz.shape[0] == n0 - n_pruned
    assert bool((m.neural_points.points_conf >= thresh).all())
    m.optimize_parameters(total_steps=6)
    assert np.isfinite(float(m.get_current_losses()["total"]))
    k = 64
    g = torch.Generator().manual_seed(0)
    add = [torch.rand(k, c, generator=g) for c in (3, 32, 3, 3, 1)]
    add[0] = add[0] * 0.1 + torch.from_numpy(pc.xyz[:1])
    m.clean_optimizer_scheduler()
    m.grow_points(*add, add_label=None)
    assert m.neural_points.xyz.shape[0] == n0 - n_pruned + k
    m.optimize_parameters(total_steps=7)
    assert np.isfinite(float(m.get_current_losses()["total"]))
    assert m.test()["coarse_raycolor"].shape == before.shape


@pytest.mark.parametrize("sizes", [(4096,), (1003,), (3,), (38_401, 3_601, 7, 1_200)])
def test_point_adam_matches_torch_adam(sizes):
    """PointAdam (sgn_adam_step_multi: one launch per group) against torch.optim.Adam (fp32,
    single-tensor) over three steps with changing gradients and a decayed lr: parameters and
    both moments within fp32 rounding, for one tensor and for a group of ragged tensors (n % 4
    tails, float4 ranges crossing tensors); the gradient is cleared by the step when zero_grad
    is on."""
    from sgnerf_amd.train_hip import PointAdam
    g = torch.Generator().manual_seed(sum(sizes))
    p0 = [torch.randn(n, generator=g) for n in sizes]
    a = [torch.nn.Parameter(x.clone().to(DEV)) for x in p0]
    b = [torch.nn.Parameter(x.clone().to(DEV)) for x in p0]
    oa = PointAdam(a, lr=2e-3, betas=(0.9, 0.999))
    ob = torch.optim.Adam(b, lr=2e-3, betas=(0.9, 0.999), foreach=False)
    for it in range(3):
        for x, y, n in zip(a, b, sizes):
            gr = (torch.randn(n, generator=g) * 10 ** (it - 1)).to(DEV)
            gr[::7] = 0.0                                    # untouched points still decay
            x.grad = gr.clone()
            y.grad = gr.clone()
        for o in (oa, ob):
            o.param_groups[0]["lr"] = 2e-3 * 0.9 ** it
        oa.step()
        ob.step()
        for x, y in zip(a, b):
            assert torch.count_nonzero(x.grad) == 0
            torch.testing.assert_close(x, y, rtol=1e-6, atol=1e-7)
            for k in ("exp_avg", "exp_avg_sq"):
                ref = ob.state[y][k]   # atol: fp32 rounding at the tensor's scale (m cancels to ~0)
                torch.testing.assert_close(oa.state[x][k], ref, rtol=1e-6, atol=1e-6 * float(ref.abs().max()))
    assert all(float(oa.state[x]["step"]) == 3.0 for x in a)


@pytest.mark.parametrize("n_rows,steps,flush_every,dp", [(5_003, 12, 256, False), (20_000, 9, 4, False),
                                                         (7, 5, 256, False), (5_003, 12, 256, True),
                                                         (20_000, 9, 4, True)])
def test_row_sparse_adam_matches_dense_bit_for_bit(n_rows, steps, flush_every, dp):
    """PointAdam(rows=True) (sgn_adam_rows: a step's update deferred to the next step's launch, which
    brings the rows it lists forward, each first replaying the zero-gradient steps it missed) against
    the dense PointAdam on the point group's
    shapes [N, 32] [N, 3] [N, 3] [N, 1]: every step's gradient lives on a random row subset plus
    row 0 (the loss stage's conf read), the list holds those rows as a neighbour table would (-1
    slots, duplicates, a device int32 count times K), lr decays per step.  Rows a step reads equal
    the dense state at its start, and after flush() every parameter and moment equals the dense
    one exactly (the same fp32 operations in the same order); state_dict() flushes, and so does
    zero_grad() while a step is pending.  dp: the data-parallel sequence of HipTrainer (the exchanged
    gradient also holds other ranks' rows, which this rank's step never read; set_update_rows gets
    every rank's list as _allreduce_point_rows returns it: padded slices, duplicates, pad row N-1)."""
    from sgnerf_amd.train_hip import PointAdam
    g = torch.Generator().manual_seed(n_rows + steps)
    widths = (32, 3, 3, 1)
    p0 = [torch.randn(n_rows, w, generator=g) for w in widths]
    a = [torch.nn.Parameter(x.clone().to(DEV)) for x in p0]
    b = [torch.nn.Parameter(x.clone().to(DEV)) for x in p0]
    od = PointAdam(a, lr=2e-3)
    orow = PointAdam(b, lr=2e-3, rows=True, flush_every=flush_every)
    K = 8
    for it in range(steps):
        n_s = max(1, n_rows // 40)
        table = torch.randint(0, n_rows, (n_s, K), generator=g, dtype=torch.int32)
        table[torch.rand(n_s, K, generator=g) < 0.3] = -1          # empty neighbour slots
        table[: n_s // 4, 1] = table[: n_s // 4, 0]                  # duplicates
        used = torch.unique(table[table >= 0].long())
        cap = torch.full((n_s + 5, K), n_rows - 1, dtype=torch.int32)   # entries past the count: ignored
        cap[:n_s] = table
        rows = cap.reshape(-1).to(DEV)
        count = torch.tensor([n_s, 0], dtype=torch.int32, device=DEV)
        pb = orow.set_rows(rows, count, False, K)   # applies the previous step, brings these rows forward
        read = torch.cat([used, torch.zeros(1, dtype=torch.long)]).to(DEV)   # the rows the step may read
        for x, y in zip(a, b):                                       # caught up: the dense state
            assert torch.equal(x.detach()[read], y.detach()[read])
        n_pb = int(pb[:8].view(torch.int64).item())                  # the step's distinct rows, row 0 too
        assert n_pb == torch.unique(read).numel() and int(pb[8:16].view(torch.int64).item()) == 0
        assert torch.equal(torch.sort(pb[16:].view(torch.int32)[:n_pb].long()).values, torch.unique(read))
        upd = read
        if dp:   # two other ranks' rows (most of them never read here), as all_gather lays them out
            other = [torch.unique(torch.randint(0, n_rows, (n_s * 3,), generator=g)) for _ in range(2)]
            slices = [read.cpu()] + [torch.cat([o, torch.zeros(1, dtype=torch.long)]) for o in other]
            m = max(s.numel() for s in slices)
            all_idx = torch.full((3, m), n_rows - 1, dtype=torch.long)
            for r, s in enumerate(slices):
                all_idx[r, :s.numel()] = s
            upd = torch.unique(all_idx).to(DEV)
        for x, y, w in zip(a, b, widths):
            gr = torch.zeros(n_rows, w)
            gr[upd.cpu()] = torch.randn(upd.numel(), w, generator=g) * 10 ** (it % 3 - 1)
            gr[0] = torch.randn(w, generator=g)
            x.grad = gr.to(DEV)
            y.grad = gr.to(DEV)
        if dp:
            orow.set_update_rows(all_idx.reshape(-1).to(DEV).to(torch.int32))
        for o in (od, orow):
            o.param_groups[0]["lr"] = 2e-3 * 0.97 ** it
        od.step()
        orow.step()                                                  # deferred to the next set_rows
        if it == 1:
            orow.zero_grad(set_to_none=False)                        # applies the pending step first
            assert all(torch.count_nonzero(y.grad) == 0 for y in b)
    sd = orow.state_dict()                                           # flushes: the last step applied
    for x, y in zip(a, b):
        assert torch.count_nonzero(y.grad) == 0
        assert torch.equal(x.detach(), y.detach())
        for k in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(od.state[x][k], orow.state[y][k])
    assert all(float(v["step"]) == steps for v in sd["state"].values())
    # a fresh optimizer loads the state (the narrow tensors' moments back into its packed buffer) and
    # steps on as the dense one does
    o2 = PointAdam(b, lr=2e-3, rows=True, flush_every=flush_every)
    o2.load_state_dict(sd)
    assert o2._mv is not None and o2.state[b[1]]["exp_avg"].data_ptr() == o2._mv.data_ptr() + 4 * o2._narrow[1][0]
    for x, y, w in zip(a, b, widths):
        gr = torch.randn(n_rows, w, generator=g)
        x.grad = gr.to(DEV)
        y.grad = gr.to(DEV)
    od.step()
    o2.step()                                                        # no row list: every row at once
    for x, y in zip(a, b):
        assert torch.equal(x.detach(), y.detach())
        for k in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(od.state[x][k], o2.state[y][k])


def _fake_two_ranks(monkeypatch):
    """torch.distributed as two ranks holding the same batch: all_reduce sums two equal copies,
    all_gather_into_tensor lays out two equal slices (the driver's multi-GPU runs are the only real
    N > 1 runs; this drives HipTrainer's data-parallel branches on one GPU)."""
    import torch.distributed as dist
    monkeypatch.setattr(dist, "is_available", lambda: True)
    monkeypatch.setattr(dist, "is_initialized", lambda: True)
    monkeypatch.setattr(dist, "get_world_size", lambda group=None: 2)
    monkeypatch.setattr(dist, "all_reduce", lambda t, *a, **k: t.mul_(2))

    def gather(out, inp, *a, **k):
        assert out.numel() == 2 * inp.numel()
        out.view(2, -1).copy_(inp.reshape(1, -1).expand(2, -1))
    monkeypatch.setattr(dist, "all_gather_into_tensor", gather)


@pytest.mark.parametrize("precision", ["f16", "f32"])
def test_data_parallel_step_matches_single_rank(precision, monkeypatch):
    """HipTrainer's data-parallel step (touched rows and counts gathered, the sparse point-row
    exchange, the row-sparse Adam over every rank's rows: _adam_union / set_update_rows) with two
    ranks holding the same batch equals the one-rank step: the exchanged means are exact (x/2 + x/2),
    so the parameters after three steps differ only by the atomic accumulation order of the point
    gradients, bounded here by the one-rank run's own spread."""
    pc, view, qd, mlp, gt = _setup(seed=7)
    d = lambda a: torch.from_numpy(a).to(DEV)  # noqa: E731
    names = ("points_embeding", "points_color", "points_dir", "points_conf")
    runs = {}
    for mode in ("one", "one_again", "dp"):
        if mode == "dp":
            _fake_two_ranks(monkeypatch)
        points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, DEV)
        tr = HipTrainer(points, mlp, dataclasses_replace(O), DEV, precision=precision)
        p0 = {k: getattr(points, k).detach().clone() for k in names}
        p0["mlp"] = tr.mlp.flat.detach().clone()
        losses = []
        for it in range(3):
            torch.manual_seed(100 + it)
            gti = torch.rand(gt.shape, generator=torch.Generator().manual_seed(it)).to(DEV)
            parts, _, _ = tr.step(d(view.campos), d(view.camrotc2w), d(view.raydir), 0.1, 8.0, gti)
            losses.append(float(parts["total"]))
        tr.sync_points()
        upd = {k: getattr(points, k).detach() - p0[k] for k in names}
        upd["mlp"] = tr.mlp.flat.detach() - p0["mlp"]
        runs[mode] = (losses, upd)
        monkeypatch.undo()
    rel = lambda x, y: {k: float(torch.linalg.vector_norm((x[k] - y[k]).double())  # noqa: E731
                                 / torch.linalg.vector_norm(y[k].double())) for k in y}
    spread = rel(runs["one_again"][1], runs["one"][1])
    err = rel(runs["dp"][1], runs["one"][1])
    print("one-rank spread", {k: f"{v:.1e}" for k, v in spread.items()})
    print("dp vs one-rank", {k: f"{v:.1e}" for k, v in err.items()})
    assert abs(runs["dp"][0][0] - runs["one"][0][0]) <= 1e-5 * abs(runs["one"][0][0])
    for a, b in zip(runs["dp"][0], runs["one"][0]):
        assert abs(a - b) <= 1e-3 * abs(b)
    for k in err:   # every point and MLP tensor moved, by the one-rank update
        assert float(torch.linalg.vector_norm(runs["dp"][1][k])) > 0
        assert err[k] <= max(UPDATE_TOL if precision == "f16" else 1e-2, 3 * spread[k]), (k, err, spread)


@pytest.mark.parametrize("rows", [0, 1, 777, 165_000])
def test_colsum_matches_torch_sum(rows):
    """sgn_colsum_f16 (bias gradients) against a float64 column sum of the same fp16 tiles,
    and bit-identical across two calls (fixed summation order)."""
    L = _lib.lib()
    g = torch.Generator().manual_seed(rows)
    xs = [torch.randn(max(rows, 1), 256, generator=g).half().to(DEV) for _ in range(4)]
    ws = torch.empty(int(L.sgn_colsum_workspace_bytes(4)) // 4, device=DEV)
    outs = []
    for _ in range(2):
        out = torch.full((4, 256), float("nan"), device=DEV)
        ptrs = (ctypes.c_void_p * 4)(*(x.data_ptr() for x in xs))
        _lib.check(L.sgn_colsum_f16(4, ptrs, rows, 256, _lib.ptr(ws), _lib.ptr(out), _lib.stream_handle()),
                   "sgn_colsum_f16")
        outs.append(out.cpu())
    assert torch.equal(outs[0], outs[1])
    ref = torch.stack([x[:rows].double().sum(0) for x in xs]).float().cpu()
    torch.testing.assert_close(outs[0], ref, rtol=1e-5, atol=1e-5 * max(rows, 1) ** 0.5)


@pytest.mark.parametrize("rows", [0, 1, 777, 165_000])
def test_colsum_weighted_parts(rows):
    """sgn_colsum_f16_weighted_parts (the alpha branch's dza^T h4 and sum(dza) as row-slab partials):
    the slabs summed equal a float64 weighted column sum / weight sum, and the weighted launch with a
    final pass (sgn_colsum_f16_weighted) agrees with the slab sums; rows past `rows` (NaN here) are never
    read."""
    L = _lib.lib()
    ns = _lib.COLSUM_SLABS
    g = torch.Generator().manual_seed(rows + 5)
    n = max(rows, 1) + 64
    xs = [torch.randn(n, 256, generator=g).half() for _ in range(2)]
    rws = [torch.randn(n, generator=g) for _ in range(2)]
    for x, w in zip(xs, rws):
        x[rows:] = float("nan")
        w[rows:] = float("nan")
    xd, wd = [x.to(DEV) for x in xs], [w.to(DEV) for w in rws]
    ws = torch.full((int(L.sgn_colsum_workspace_bytes(2)) // 4,), float("nan"), device=DEV)
    assert ws.numel() == 2 * ns * 257
    xp = (ctypes.c_void_p * 2)(*(x.data_ptr() for x in xd))
    wp = (ctypes.c_void_p * 2)(wd[0].data_ptr(), None)   # the second matrix unweighted
    _lib.check(L.sgn_colsum_f16_weighted_parts(2, xp, wp, rows, 256, _lib.ptr(ws), _lib.stream_handle()),
               "sgn_colsum_f16_weighted_parts")
    cols = ws[:2 * ns * 256].view(2, ns, 256).double().sum(1).cpu()
    wsum = ws[2 * ns * 256:2 * ns * 256 + ns].double().sum().cpu()
    r0 = (xs[0][:rows].double() * rws[0][:rows].double()[:, None]).sum(0)
    r1 = xs[1][:rows].double().sum(0)
    tol = 1e-5 * max(rows, 1) ** 0.5
    torch.testing.assert_close(cols[0], r0, rtol=1e-5, atol=tol)
    torch.testing.assert_close(cols[1], r1, rtol=1e-5, atol=tol)
    torch.testing.assert_close(wsum, rws[0][:rows].double().sum(), rtol=1e-5, atol=tol)
    out = torch.empty(2, 256, device=DEV)
    _lib.check(L.sgn_colsum_f16_weighted(2, xp, wp, rows, 256, _lib.ptr(ws), _lib.ptr(out), _lib.stream_handle()),
               "sgn_colsum_f16_weighted")
    torch.testing.assert_close(out.double().cpu(), cols, rtol=1e-5, atol=tol)   # fp32 vs float64 slab sums


def test_graph_captured_step_matches_eager_step():
    """The loss stage replayed as a HIP graph over padded capacity (HipTrainer.use_graph) gives
    the eager step's loss, gradients and, over three steps with Adam, parameters: padding items
    and samples contribute nothing (bar fp32 summation order in differently shaped GEMMs)."""
    pc, view, qd, mlp, gt = _setup(seed=7)
    d = lambda a: torch.from_numpy(a).to(DEV)  # noqa: E731
    runs = {}
    for use_graph in (False, True, "eager2"):
        points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, DEV)
        tr = HipTrainer(points, mlp, O, DEV)
        tr.use_graph = use_graph is True
        p0 = {k: getattr(points, k).detach().cpu().clone()
              for k in ("points_embeding", "points_color", "points_dir", "points_conf")}
        p0["mlp"] = tr.mlp.flat.detach().cpu().clone()
        losses, grads = [], None
        for it in range(3):
            torch.manual_seed(100 + it)                   # same jittered depth table in both runs
            gti = torch.rand(gt.shape, generator=torch.Generator().manual_seed(it)).to(DEV)
            parts, full, mask = tr.backward(d(view.campos), d(view.camrotc2w), d(view.raydir), 0.1, 8.0, gti)
            if it == 0:
                grads = {k: v.cpu() for k, v in grads_named(tr).items()}
                first = (full.cpu(), mask.cpu())
            tr.apply()
            losses.append(float(parts["total"]))
        torch.cuda.synchronize()
        params = {k: getattr(points, k).detach().cpu().clone() - p0[k]
                  for k in ("points_embeding", "points_color", "points_dir", "points_conf")}
        params["mlp"] = tr.mlp.flat.detach().cpu().clone() - p0["mlp"]
        runs[use_graph] = (losses, grads, params, first)
        if use_graph is True:
            assert tr._graphs, "the graph path did not run"
    (le, ge, pe, fe), (lg, gg, pg, fg) = runs[False], runs[True]
    # run-to-run spread of the eager path itself (atomic accumulation order in the backward)
    pe2 = runs["eager2"][2]
    ee_err = {k: float(torch.linalg.vector_norm((pe2[k] - pe[k]).double())
                       / torch.linalg.vector_norm(pe[k].double())) for k in pe}
    print("eager-vs-eager update rel L2", {k: f"{v:.1e}" for k, v in ee_err.items()})
    assert torch.equal(fe[1], fg[1])
    assert float((fe[0] - fg[0]).abs().max()) <= 1e-5
    ge_err = {k: _rel(gg[k], ge[k]) for k in ge}
    # the three Adam updates (p_3 - p_0), graph vs eager, relative L2 per tensor: m / sqrt(v)
    # normalises near-zero gradients, so rounding differences become lr-sized on a few elements
    pe_err = {k: float(torch.linalg.vector_norm((pg[k] - pe[k]).double())
                       / torch.linalg.vector_norm(pe[k].double())) for k in pe}
    print("losses eager", le, "graph", lg)
    print("grad rel L2", {k: f"{v:.1e}" for k, v in ge_err.items()})
    print("param rel L2", {k: f"{v:.1e}" for k, v in pe_err.items()})
    assert abs(le[0] - lg[0]) <= 1e-5 * abs(le[0])
    for a, b in zip(le, lg):
        assert abs(a - b) <= 1e-3 * abs(a)
    # the graph path's colour backward multiplies in fp16 (ColourStep products=1, the step's delta
    # precision) where the eager path's torch autograd runs fp32: measured 7.2e-4 (block3.2), every
    # tensor far inside the f16 step's bars against fp32 autograd (GRAD_TOL_MLP / GRAD_TOL_POINTS)
    assert max(ge_err.values()) <= 2e-3, ge_err
    assert max(pe_err.values()) <= UPDATE_TOL, (pe_err, ee_err)


def test_graph_step_without_hits():
    """A batch whose rays all miss the cloud (the graph loss stage read sample 0's ray
    when the step had no samples): eager and graph steps both run, render the background,
    report a zero masked loss and leave every gradient at zero."""
    pc, view, qd, mlp, gt = _setup(seed=3)
    d = lambda a: torch.from_numpy(a).to(DEV)  # noqa: E731
    campos = d(view.campos) + 100.0
    for use_graph in (False, True):
        points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, DEV)
        tr = HipTrainer(points, mlp, O, DEV)
        tr.use_graph = use_graph
        for _ in range(2):   # the second step replays the captured graph
            parts, full, mask = tr.backward(campos, d(view.camrotc2w), d(view.raydir), 0.1, 8.0, gt.to(DEV))
        torch.cuda.synchronize()
        assert not bool(mask.any())
        assert torch.equal(full.cpu(), torch.ones_like(full.cpu()))
        assert float(parts["ray_masked_coarse_raycolor"]) == 0.0
        assert abs(float(parts["ray_miss_coarse_raycolor"]) - float(((1 - gt) ** 2).sum() / 3)) <= 1e-4 * float(
            ((1 - gt) ** 2).sum())
        for k, g in grads_named(tr).items():
            assert float(g.abs().max()) == 0.0, k
        tr.apply()
        assert all(torch.isfinite(getattr(points, k)).all() for k in ("points_embeding", "points_conf"))
    assert tr._graphs, "the graph path did not run"


def test_f32_step_without_hits():
    """The fp32 step (every count on the device) on a batch whose rays all miss: background colour,
    zero masked loss, every gradient exactly zero, finite parameters after the update."""
    pc, view, qd, mlp, gt = _setup(seed=3)
    d = lambda a: torch.from_numpy(a).to(DEV)  # noqa: E731
    campos = d(view.campos) + 100.0
    points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, DEV)
    tr = HipTrainer(points, mlp, O, DEV, precision="f32")
    for _ in range(2):
        parts, full, mask = tr.backward(campos, d(view.camrotc2w), d(view.raydir), 0.1, 8.0, gt.to(DEV))
        torch.cuda.synchronize()
        assert not bool(mask.any())
        assert torch.equal(full.cpu(), torch.ones_like(full.cpu()))
        assert float(parts["ray_masked_coarse_raycolor"]) == 0.0
        for k, g in grads_named(tr).items():
            assert float(g.abs().max()) == 0.0, k
        tr.apply()
        assert all(torch.isfinite(getattr(points, k)).all() for k in ("points_embeding", "points_conf"))


def test_colour_inputs_kernel_matches_torch():
    """sgn_colour_inputs (the f16 step's captured colour-stage inputs) element by element against the
    torch construction it replaced: items < counters[1] get fp32 f_s, the sample's alpha, its ray's
    direction and the sample id; padding items zeros, ray 0's direction and the sentinel s_cap."""
    from sgnerf_amd import _lib
    g = torch.Generator().manual_seed(7)
    n_cap, s_cap, n, R = 300, 500, 217, 64
    work = torch.randperm(s_cap, generator=g)[:n_cap].to(torch.int32)
    samp_ray = torch.randint(0, R, (s_cap,), generator=g, dtype=torch.int32)
    fs16 = torch.randn(n_cap, 256, generator=g).half()
    feat = torch.randn(s_cap, 4, generator=g)
    raydir = torch.randn(R, 3, generator=g)
    counters = torch.tensor([s_cap, n, 0, 0], dtype=torch.int32)
    dv = {k: v.to(DEV) for k, v in dict(work=work, samp_ray=samp_ray, fs16=fs16, feat=feat, raydir=raydir,
                                         counters=counters).items()}
    fs32 = torch.full((n_cap, 256), float("nan"), device=DEV)
    al32 = torch.full((n_cap,), float("nan"), device=DEV)
    v = torch.full((n_cap, 3), float("nan"), device=DEV)
    samp = torch.full((n_cap,), -7, dtype=torch.int32, device=DEV)
    vpe = torch.full((n_cap, 32), float("nan"), device=DEV)
    p = _lib.ptr
    _lib.check(_lib.lib().sgn_colour_inputs(p(dv["counters"]), p(dv["work"]), p(dv["samp_ray"]), n_cap, s_cap,
                                            p(dv["fs16"]), p(dv["feat"]), p(dv["raydir"]), p(fs32), p(al32), p(v),
                                            p(samp), p(vpe), _lib.stream_handle()), "sgn_colour_inputs")
    torch.cuda.synchronize()
    ok = torch.arange(n_cap) < n
    wk = work.long()
    exp_fs = torch.where(ok[:, None], fs16.float(), torch.zeros(()))
    exp_al = torch.where(ok, feat[wk, 0], torch.zeros(()))
    exp_v = torch.where(ok[:, None], raydir[samp_ray[wk].long()], raydir[0].expand(n_cap, 3))
    exp_samp = torch.where(ok, work, torch.full((), s_cap, dtype=torch.int32))
    assert torch.equal(fs32.cpu(), exp_fs)
    assert torch.equal(al32.cpu(), exp_al)
    assert torch.equal(v.cpu(), exp_v)
    assert torch.equal(samp.cpu(), exp_samp)
    # PE(viewdir) as the torch construction it replaced (sin | cos of v 2^f), the ones column, zeros
    x = (exp_v[:, :, None] * torch.tensor([1.0, 2.0, 4.0, 8.0])).reshape(-1, 12)
    exp_vpe = torch.cat([torch.sin(x), torch.cos(x), torch.ones(n_cap, 1), torch.zeros(n_cap, 7)], dim=1)
    torch.testing.assert_close(vpe.cpu(), exp_vpe, rtol=0, atol=2e-6)


def test_copy_segments_kernel():
    """sgn_copy_segments: 16-B, 4-B and byte-granular segments (odd offsets and lengths) and a
    clear (null source) in one launch; bytes outside each destination untouched."""
    g = torch.Generator().manual_seed(5)
    src = torch.randint(0, 255, (4096,), generator=g, dtype=torch.uint8).to(DEV)
    dst = torch.full((4096,), 7, dtype=torch.uint8, device=DEV)
    spans = [(0, 64, 1024), (4, 1200, 36), (3, 2001, 13), (None, 3000, 100)]   # (src off, dst off, bytes)
    _lib.copy_segments([(None if so is None else src[so:so + n], dst[do:do + n]) for so, do, n in spans])
    torch.cuda.synchronize()
    exp = torch.full((4096,), 7, dtype=torch.uint8)
    s = src.cpu()
    for so, do, n in spans:
        exp[do:do + n] = 0 if so is None else s[so:so + n]
    assert torch.equal(dst.cpu(), exp)


def test_touched_points_kernel_matches_torch():
    """sgn_touched_points (the single-GPU fp32 step's projection subset) against train.touched_rows
    over consecutive steps on one stamp table: the same set of points (point 0 always, -1 slots
    and samples >= S skipped, duplicates listed once), each step's count in its parity slot and
    the other slot cleared; S = 0 lists point 0 alone.  Neighbour ids >= n_points are never
    listed and are counted in the third word (a query / point-table mismatch must not pass silently)."""
    from sgnerf_amd.train import touched_rows
    g = torch.Generator().manual_seed(11)
    n_points, K, s_cap = 5000, 8, 3000
    stamp = torch.full((n_points,), -1, dtype=torch.int32, device=DEV)
    lst = torch.full((n_points,), -9, dtype=torch.int32, device=DEV)
    cnt = torch.full((3,), 0, dtype=torch.int64, device=DEV)
    p = _lib.ptr
    for step, S in enumerate([2500, 3000, 0, 1777]):
        pidx = torch.randint(-1, n_points, (s_cap * K,), generator=g, dtype=torch.int32)
        pidx[::5] = -1
        pidx[7] = n_points - 1
        counters = torch.tensor([S, 0, 0, 0], dtype=torch.int32)
        dp_, dc = pidx.to(DEV), counters.to(DEV)
        cnt[(step + 1) & 1] = 12345   # the kernel clears the next step's slot
        _lib.check(_lib.lib().sgn_touched_points(p(dp_), p(dc), s_cap, K, n_points, step, p(stamp), p(lst), p(cnt),
                                                 _lib.stream_handle()), "sgn_touched_points")
        torch.cuda.synchronize()
        idx, c = touched_rows(pidx, counters[0], K, n_points)
        c = int(c)
        assert int(cnt[step & 1]) == c
        assert int(cnt[(step + 1) & 1]) == 0
        assert int(cnt[2]) == 0
        got = torch.sort(lst[:c].cpu().long()).values
        assert torch.equal(got, idx[:c])
        if S == 0:
            assert c == 1 and int(lst[0]) == 0
    # a planted out-of-range id (inside the S samples) is counted, never listed
    pidx = torch.zeros(s_cap * K, dtype=torch.int32)
    pidx[3] = n_points + 5
    counters = torch.tensor([10, 0, 0, 0], dtype=torch.int32)
    dp_, dc = pidx.to(DEV), counters.to(DEV)
    _lib.check(_lib.lib().sgn_touched_points(p(dp_), p(dc), s_cap, K, n_points, 4, p(stamp), p(lst), p(cnt),
                                             _lib.stream_handle()), "sgn_touched_points")
    torch.cuda.synchronize()
    assert int(cnt[2]) == 1 and int(cnt[0]) == 1 and int(lst[0]) == 0


def test_model_ranks_frames_by_ray_miss_loss(tmp_path):
    """optimize_parameters -> update_rank_ray_miss (neural_points_volumetric_model.py:328-330,
    mvs_points_volumetric_model.py:157-176) on real steps: the logged ray-miss loss is the
    missed rays' squared error summed / 3, and the ranking keeps the worst frames first."""
    import argparse

    from sgnerf_amd.model import HipPointsVolumetricModel
    pc, view, qd, mlp, gt = _setup(seed=3)
    d = lambda a: torch.from_numpy(a).to(DEV)  # noqa: E731
    opt = argparse.Namespace(SR=24, K=8, gpu_ids=[0], is_train=True, checkpoints_dir=str(tmp_path), name="scene",
                             bg_color="white", prob_freq=100, prob_num_step=2, prob_kernel_size=None)
    m = HipPointsVolumetricModel()
    m.initialize(opt)
    m.set_points(points_xyz=pc.xyz, points_feats=pc.color * 255.0, points_embedding=pc.embedding,
                 points_color=pc.color, points_dir=pc.dir, points_conf=pc.conf, aggregator_state=mlp)
    m.setup(opt, train_len=6)
    assert m.top_ray_miss_loss.shape == (4,)
    seen = {}
    for step, fid in enumerate((4, 1, 4, 0)):
        gti = torch.rand(gt.shape, generator=torch.Generator().manual_seed(step))
        m.set_input({"campos": d(view.campos)[None], "raydir": d(view.raydir)[None],
                     "camrotc2w": d(view.camrotc2w)[None], "near": torch.tensor([[[0.1]]]),
                     "far": torch.tensor([[[8.0]]]), "gt_image": gti[None], "id": torch.tensor([fid])})
        m.optimize_parameters(total_steps=step)
        miss = ~m.ray_mask[0].bool().cpu()
        want = float(((m.coarse_raycolor[0].cpu() - gti) ** 2)[miss].sum() / 3)
        got = float(m.get_current_losses()["ray_miss_coarse_raycolor"])
        assert abs(got - want) <= 1e-5 * max(want, 1e-6), (got, want)
        seen[fid] = max(seen.get(fid, 0.0), got)
    ids = m.top_ray_miss_ids.cpu().tolist()
    losses = m.top_ray_miss_loss.cpu().tolist()
    assert losses == sorted(losses, reverse=True)
    for fid, l in seen.items():
        if l > 0:
            assert fid in ids and abs(losses[ids.index(fid)] - l) <= 1e-6 * l


def test_graph_cache_buckets_and_lru(monkeypatch):
    """Loss-stage graphs per capacity bucket: a batch of another size captures a second graph,
    returning to the first size replays the first (LRU hit, no capture); with room for one
    graph every change recaptures.  Each replayed step equals the eager step's loss."""
    import sgnerf_amd.train_hip as th
    pc, view, qd, mlp, gt = _setup(seed=7)
    d = lambda a: torch.from_numpy(a).to(DEV)  # noqa: E731
    sizes = [view.raydir.shape[0], view.raydir.shape[0] // 3, view.raydir.shape[0]]
    monkeypatch.setattr(th, "GRAPH_BUCKET", 64)

    def run(use_graph, cache):
        monkeypatch.setattr(th, "GRAPH_CACHE", cache)
        points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, DEV)
        tr = HipTrainer(points, mlp, O, DEV)
        tr.use_graph = use_graph
        out = []
        for i, R in enumerate(sizes):
            torch.manual_seed(300 + i)
            parts, full, mask = tr.backward(d(view.campos), d(view.camrotc2w), d(view.raydir[:R]), 0.1, 8.0,
                                            gt[:R].to(DEV))
            out.append(float(parts["total"]))
        return tr, out
    _, eager = run(False, 8)
    tr, graph = run(True, 8)
    assert tr.graph_captures == 2 and len(tr._graphs) == 2
    for a, b in zip(eager, graph):
        assert abs(a - b) <= 1e-5 * abs(a), (eager, graph)
    tr1, _ = run(True, 1)
    assert tr1.graph_captures == 3 and len(tr1._graphs) == 1


def test_200_step_training_tracks_fp32_torch():
    """200 training steps of the HIP path (fp16-in MFMA forward, fp16-delta backward) against
    the fp32 torch-autograd restatement (train.Trainer on the same device, same HIP query and
    jitter, same batches) fitting a teacher aggregator's renders: both loss curves fall, and
    the HIP curve stays within LOSS_CURVE_TOL (relative, mean over 20-step windows) of the
    fp32 one."""
    from sgnerf_amd.render import HipRenderer, PointTables
    from sgnerf_amd.scene import synth_room, room_view
    pc = synth_room(150_000, seed=8)
    teacher = init_mlp(9, bias_std=0.01)
    teacher["alpha_branch.0.bias"] = teacher["alpha_branch.0.bias"] + 50.0
    student = init_mlp(8, bias_std=0.01)
    student["alpha_branch.0.bias"] = student["alpha_branch.0.bias"] + 50.0
    r = HipRenderer(PointTables.from_cloud(pc, DEV), teacher, O, DEV)
    views = [room_view(64, 64, yaw=30.0 * i, pitch=-8.0) for i in range(12)]
    gts = []
    for v in views:
        out = r.render(torch.from_numpy(v.campos), torch.from_numpy(v.camrotc2w), torch.from_numpy(v.raydir),
                       v.near, v.far)
        gts.append(out.rgb.clone())
    del r
    g = torch.Generator().manual_seed(0)
    batches = []
    for i in range(200):
        v = views[i % len(views)]
        idx = torch.randperm(64 * 64, generator=g)[:2048]
        batches.append((torch.from_numpy(v.campos).to(DEV), torch.from_numpy(v.camrotc2w).to(DEV),
                        torch.from_numpy(v.raydir)[idx].to(DEV), gts[i % len(views)][idx.to(DEV)]))
    curves = {}
    for name, cls in (("hip", HipTrainer), ("torch", Trainer)):
        points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, DEV)
        tr = cls(points, student, dataclasses_replace(O, is_train=1), DEV, lr=1e-3, plr=2e-3)
        ls = []
        for i, (c, rot, rd, gt) in enumerate(batches):
            torch.manual_seed(5000 + i)          # same depth jitter in both runs
            parts, _, _ = tr.step(c, rot, rd, 0.1, 8.0, gt)
            ls.append(float(parts["ray_masked_coarse_raycolor"]))
        curves[name] = np.array(ls)
    h, t = curves["hip"], curves["torch"]
    wh, wt = h.reshape(10, 20).mean(1), t.reshape(10, 20).mean(1)
    rel = np.abs(wh - wt) / wt
    print("colour loss per 20-step window: hip", np.round(wh, 5).tolist(), "torch", np.round(wt, 5).tolist(),
          "rel", np.round(rel, 4).tolist())
    assert wh[-1] < 0.7 * wh[0] and wt[-1] < 0.7 * wt[0]
    assert rel.max() <= LOSS_CURVE_TOL, rel


@pytest.mark.parametrize("dim,seed", [(96, 3), (96, 5), (0, 3)])
def test_hip_sg_training_gradients_match_oracle(dim, seed):
    """SG-NeRF's block2_bpnet (point_aggregators.py:345-354, :629-636) on the HIP training path:
    one backward against fp32 autograd through oracle/agg_ref.py's SG aggregator on the same
    neighbours (dim 96: the semantic-guided query with a `seconds` that passes every label, so
    it equals the plain query), with the base bars: MLP gradients (block2_bpnet.0 included)
    within 2e-2 relative L2, point gradients within 6e-2, colour within 1e-3.  Seeds 3 and 5
    are the base test's; measured worst MLP errors 1.0-1.3e-2 (block1.0, two fp16 layers
    further from the loss than in the base net).  Seed 4 lands at 2.2e-2 on block1.0 with
    every layer ~2.5x noisier than seeds 3/5, colour_branch.0 included, which block2_bpnet's
    backward does not touch: an fp16-rounding outlier of that scene, not an SG term."""
    import math

    import agg_ref
    from test_train_cpu import O as O_BASE
    pc, view, qd, mlp, gt = _setup(seed=seed)
    n = pc.xyz.shape[0]
    g = torch.Generator().manual_seed(11)
    bound = math.sqrt(6.0 / (256 + dim + 256)) * 0.5
    mlp = dict(mlp)
    mlp["block2_bpnet.0.weight"] = (torch.rand(256, 256 + dim, generator=g) * 2 - 1) * bound
    mlp["block2_bpnet.0.bias"] = torch.randn(256, generator=g) * 0.01
    bp = (torch.rand(n, dim, generator=g) - 0.5) if dim else None
    o = dataclasses_replace(O_BASE, shading_feature_mlp_layer2_bpnet=1, predict_semantic=1 if dim else 0,
                            semantic_guidance=1 if dim else 0)
    d = lambda a: torch.from_numpy(a).to(DEV)  # noqa: E731
    points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, DEV)
    tr = HipTrainer(points, mlp, o, DEV, bpnet=bp)
    R = view.raydir.shape[0]
    labels = (torch.zeros(n, dtype=torch.int32), torch.ones(R, dtype=torch.int32), 10) if dim else None
    parts, full, mask = tr.backward(d(view.campos), d(view.camrotc2w), d(view.raydir), 0.1, 8.0, gt.to(DEV), labels)
    torch.cuda.synchronize()
    hg = grads_named(tr)
    # oracle: fp32 autograd of the same loss (test_train_cpu._oracle_loss with the SG aggregator)
    pts = {k: torch.from_numpy(getattr(pc, k)).clone().requires_grad_(k != "xyz")
           for k in ("xyz", "embedding", "color", "dir", "conf")}
    if dim:
        pts["bpnet"] = bp
    m = {k: v.clone().requires_grad_(True) for k, v in mlp.items()}
    campos, rot, raydir = (torch.from_numpy(view.campos), torch.from_numpy(view.camrotc2w), torch.from_numpy(view.raydir))
    feat, _ = agg_ref.aggregate(pts, m, campos, rot, raydir, qd["samp_ray"], qd["samp_locw"], qd["pidx"])
    nnb = (qd["pidx"] >= 0).sum(-1)
    fd, vd, ld = agg_ref.densify(R, O_BASE.SR, qd["ray_ns"], qd["samp_ray"], qd["samp_locw"], feat, nnb)
    color, _, _ = agg_ref.composite(fd, vd, ld, rot, campos)
    ray_mask = vd.any(-1)
    l_col = torch.mean((color[ray_mask] - gt[ray_mask]) ** 2)
    S = qd["samp_ray"].shape[0]
    slot = torch.arange(S) - qd["ray_soff"][qd["samp_ray"]]
    pd = torch.full((R, O_BASE.SR, O_BASE.K), -1, dtype=torch.long)
    pd[qd["samp_ray"], slot] = qd["pidx"]
    cd = pts["conf"][torch.clamp(pd[ray_mask], min=0).reshape(-1), 0]
    val = torch.clamp(torch.clamp(cd, 1e-4, 1.0), 1e-3, 1 - 1e-3)
    l_zo = torch.mean(torch.log(val) + torch.log(1 - val))
    (l_col + 3e-6 + 1e-4 * l_zo).backward()
    assert torch.equal(mask.cpu(), ray_mask)
    assert float((full.cpu()[ray_mask] - color[ray_mask].detach()).abs().max()) <= 1e-3
    names = {"points_embeding": "embedding", "points_color": "color", "points_dir": "dir", "points_conf": "conf"}
    worst = {}
    for k, v in hg.items():
        ref = pts[names[k]].grad if k in names else m[k].grad
        worst[k] = _rel(v.cpu().reshape(ref.shape), ref)
    print(f"SG dim {dim} relative L2 gradient errors:", {k: f"{v:.2e}" for k, v in worst.items()})
    assert "block2_bpnet.0.weight" in worst
    # precision "f16" (the default): the f16 bars; "f32": test_hip_sg_f32_training_gradients_match_fp32_autograd
    bad = {k: v for k, v in worst.items() if v > (GRAD_TOL_POINTS if k.startswith("points_") else GRAD_TOL_MLP)}
    assert not bad, bad


@pytest.mark.parametrize("precision,dim,seed,K", [("f32", 96, 3, 8), ("f32", 0, 5, 8), ("f16", 96, 3, 4),
                                                  ("f32", 96, 3, 4)])
def test_hip_sg_f32_training_gradients_match_fp32_autograd(precision, dim, seed, K):
    """SG-NeRF's block2_bpnet at precision "f32" (train_f32.F32Step with block2_bpnet.0 between
    block1.2 and block3.0): one backward against fp32 autograd through oracle/agg_ref.py's SG
    aggregator, on the GPU, over the very samples the HIP query produced (last_query): the
    colour, the loss and every gradient (block2_bpnet.0 and the points included) within
    GRAD_TOL_F32.  K = 4 (rows k >= K of a sample empty): also at precision "f16", whose
    block2_bpnet.0 weight gradient gathers each row's BPNet embedding at pidx index s * K + k
    (ADVICE r5), held to the f16 bars (GRAD_TOL_MLP / GRAD_TOL_POINTS, colour 1e-3)."""
    import math

    import agg_ref
    from test_train_cpu import O as O_BASE
    pc, view, _, mlp, gt = _setup(seed=seed)
    n = pc.xyz.shape[0]
    g = torch.Generator().manual_seed(11)
    bound = math.sqrt(6.0 / (256 + dim + 256)) * 0.5
    mlp = dict(mlp)
    mlp["block2_bpnet.0.weight"] = (torch.rand(256, 256 + dim, generator=g) * 2 - 1) * bound
    mlp["block2_bpnet.0.bias"] = torch.randn(256, generator=g) * 0.01
    bp = (torch.rand(n, dim, generator=g) - 0.5) if dim else None
    o = dataclasses_replace(O_BASE, shading_feature_mlp_layer2_bpnet=1, predict_semantic=1 if dim else 0,
                            semantic_guidance=1 if dim else 0, K=K)
    d = lambda a: torch.from_numpy(a).to(DEV)  # noqa: E731
    points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, DEV)
    tr = HipTrainer(points, mlp, o, DEV, bpnet=bp, precision=precision)
    R = view.raydir.shape[0]
    labels = (torch.zeros(n, dtype=torch.int32), torch.ones(R, dtype=torch.int32), 10) if dim else None
    parts, full, mask = tr.backward(d(view.campos), d(view.camrotc2w), d(view.raydir), 0.1, 8.0, gt.to(DEV), labels)
    torch.cuda.synchronize()
    hg = grads_named(tr)
    qd = {k: v.long() if v.dtype == torch.int32 else v for k, v in tr.last_query.items()}
    pts = {k: torch.from_numpy(getattr(pc, k)).to(DEV).requires_grad_(k != "xyz")
           for k in ("xyz", "embedding", "color", "dir", "conf")}
    if dim:
        pts["bpnet"] = bp.to(DEV)
    m = {k: v.to(DEV).requires_grad_(True) for k, v in mlp.items()}
    campos, rot, raydir = d(view.campos), d(view.camrotc2w), d(view.raydir)
    feat, _ = agg_ref.aggregate(pts, m, campos, rot, raydir, qd["samp_ray"], qd["samp_locw"], qd["pidx"])
    nnb = (qd["pidx"] >= 0).sum(-1)
    fd, vd, ld = agg_ref.densify(R, O_BASE.SR, qd["ray_ns"], qd["samp_ray"], qd["samp_locw"], feat, nnb)
    color, _, _ = agg_ref.composite(fd, vd, ld, rot, campos)
    ray_mask = vd.any(-1)
    gtd = gt.to(DEV)
    l_col = torch.mean((color[ray_mask] - gtd[ray_mask]) ** 2)
    S = qd["samp_ray"].shape[0]
    slot = torch.arange(S, device=DEV) - qd["ray_soff"][qd["samp_ray"]]
    pd = torch.full((R, O_BASE.SR, K), -1, dtype=torch.long, device=DEV)
    pd[qd["samp_ray"], slot] = qd["pidx"]
    assert qd["pidx"].shape[1] == K
    cd = pts["conf"][torch.clamp(pd[ray_mask], min=0).reshape(-1), 0]
    val = torch.clamp(torch.clamp(cd, 1e-4, 1.0), 1e-3, 1 - 1e-3)
    l_zo = torch.mean(torch.log(val) + torch.log(1 - val))
    total = l_col + 3e-6 + 1e-4 * l_zo
    total.backward()
    torch.cuda.synchronize()
    assert torch.equal(mask, ray_mask)
    if precision == "f32":
        assert _rel(full[ray_mask], color[ray_mask].detach()) <= GRAD_TOL_F32
        assert abs(float(parts["total"]) - float(total)) <= GRAD_TOL_F32 * abs(float(total))
    else:
        assert float((full[ray_mask] - color[ray_mask].detach()).abs().max()) <= 1e-3
        assert abs(float(parts["total"]) - float(total)) <= 1e-3 * abs(float(total))
    names = {"points_embeding": "embedding", "points_color": "color", "points_dir": "dir", "points_conf": "conf"}
    worst = {}
    for k, v in hg.items():
        ref = pts[names[k]].grad if k in names else m[k].grad
        worst[k] = _rel(v.reshape(ref.shape), ref)
    print(f"SG {precision} dim {dim} K {K} relative L2 gradient errors (same query):",
          {k: f"{v:.2e}" for k, v in worst.items()})
    assert "block2_bpnet.0.weight" in worst
    if precision == "f32":
        bad = {k: v for k, v in worst.items() if v > GRAD_TOL_F32}
    else:
        bad = {k: v for k, v in worst.items() if v > (GRAD_TOL_POINTS if k.startswith("points_") else GRAD_TOL_MLP)}
    assert not bad, bad


def test_model_plugin_sg_training(tmp_path):
    """The plugin trains the SG-NeRF variant (block2_bpnet + semantic-guided query) on the HIP
    path as run/train_ft.py drives it: the first optimize_parameters equals a HipTrainer step
    with the same BPNet embedding and labels, the loss falls, block2_bpnet.0 moves, test()
    renders the trained state, and grow_points keeps the BPNet table aligned with the points."""
    import argparse
    import dataclasses
    import math

    from sgnerf_amd.model import HipPointsVolumetricModel
    pc, view, qd, mlp, gt = _setup(seed=3)
    n = pc.xyz.shape[0]
    g = torch.Generator().manual_seed(5)
    bound = math.sqrt(6.0 / (256 + 96 + 256)) * 0.5
    mlp = dict(mlp)
    mlp["block2_bpnet.0.weight"] = (torch.rand(256, 352, generator=g) * 2 - 1) * bound
    mlp["block2_bpnet.0.bias"] = torch.randn(256, generator=g) * 0.01
    bp = torch.rand(n, 96, generator=g) - 0.5
    lab = torch.zeros(n, dtype=torch.int32)
    d = lambda a: torch.from_numpy(a).to(DEV)  # noqa: E731
    R = view.raydir.shape[0]
    sg = dict(shading_feature_mlp_layer2_bpnet=1, predict_semantic=1, semantic_guidance=1)
    opt = argparse.Namespace(SR=24, K=8, gpu_ids=[0], is_train=True, checkpoints_dir=str(tmp_path), name="scene",
                             lr=5e-4, plr=2e-3, lr_decay_exp=0.1, lr_decay_iters=1_000_000, bg_color="white", **sg)
    m = HipPointsVolumetricModel()
    m.initialize(opt)
    m.set_points(points_xyz=pc.xyz, points_feats=pc.color * 255.0, points_embedding=pc.embedding, points_label=lab,
                 points_color=pc.color, points_dir=pc.dir, points_conf=pc.conf, aggregator_state=mlp)
    m.neural_points.set_bpnet_feats(None, lab, bp)
    m.setup(opt)
    inputs = {"campos": d(view.campos)[None], "raydir": d(view.raydir)[None], "camrotc2w": d(view.camrotc2w)[None],
              "near": torch.tensor([[[0.1]]]), "far": torch.tensor([[[8.0]]]), "gt_image": gt[None].to(DEV),
              "pixel_label": torch.zeros(1, R, 1, dtype=torch.int32, device=DEV)}
    m.set_input(inputs)
    before = m.test()["coarse_raycolor"].clone()
    tr = HipTrainer(PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, DEV), mlp,
                    dataclasses.replace(O, is_train=1, **sg), DEV, bpnet=bp, precision=m.trainer.precision)
    torch.manual_seed(11)
    parts_ref, _, _ = tr.step(d(view.campos), d(view.camrotc2w), d(view.raydir), 0.1, 8.0, gt.to(DEV),
                              labels=(lab, torch.zeros(R, dtype=torch.int32), None))
    torch.manual_seed(11)
    m.optimize_parameters(total_steps=0)
    hist = [float(m.get_current_losses()["total"])]
    assert hist[0] == float(parts_ref["total"])
    w0 = mlp["block2_bpnet.0.weight"].clone()
    for step in range(1, 6):
        m.optimize_parameters(total_steps=step)
        hist.append(float(m.get_current_losses()["total"]))
    print("SG plugin losses", hist)
    assert hist[-1] < hist[0], hist
    w = m.trainer.mlp_state()["block2_bpnet.0.weight"].cpu()
    assert not torch.equal(w, w0)
    after = m.test()["coarse_raycolor"].clone()
    assert not torch.equal(after, before)
    k = 64
    add = [torch.rand(k, c, generator=g) for c in (3, 32, 3, 3, 1)]
    add[0] = add[0] * 0.1 + torch.from_numpy(pc.xyz[:1])
    m.clean_optimizer_scheduler()
    m.grow_points(*add, add_label=torch.zeros(k, dtype=torch.int32))
    assert m.neural_points.bpnet_points_embedding.shape == (1, n + k, 96)
    m.optimize_parameters(total_steps=6)
    assert np.isfinite(float(m.get_current_losses()["total"]))
