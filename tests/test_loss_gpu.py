"""GPU tests of the HIP loss stage (csrc/loss.hip via sgnerf_amd.loss_hip.LossStage) against the
torch autograd of train.composite_losses -- the restatement of ray_dist / ray_march /
fill_invalid and the training losses (neural_points_volumetric_model.py:569-631,
diff_ray_marching.py:509-555, base_rendering_model.py:534-664, mvs_points_volumetric_model.py:607-614)
that the CPU tests pin to oracle/agg_ref.py.  Same query, features and conf on both sides.

Bars (fp32 on both sides, different summation orders): loss parts 1e-5 relative, rendered colour
1e-5 absolute (the f32 bar; measured 3.9e-6 on near-opaque rays, where torch's tree-ordered slot sum
and scan cumprod round differently from the per-ray sequential pass), ray mask equal, gradients
w.r.t. the features and conf 1e-4 relative L2."""
import pytest
import torch

from sgnerf_amd.loss_hip import LossStage
from sgnerf_amd.opts import HotPathOpts
from sgnerf_amd.querier import LightningFastQuerier
from sgnerf_amd.train import PointParams, composite_losses
from helpers import make_view, small_room

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _rel(a, b):
    return float(torch.linalg.vector_norm(a.double() - b.double()) / max(torch.linalg.vector_norm(b.double()), 1e-30))


def _case(seed, SR, alpha_scale, conf_lo, conf_hi, h=24, w=32, n=60_000, unit=0):
    o = HotPathOpts(SR=SR, raydist_mode_unit=unit)
    pc = small_room(n, seed=seed)
    view = make_view(h, w, yaw=30.0, pitch=-8.0)
    g = torch.Generator().manual_seed(seed)
    conf = conf_lo + (conf_hi - conf_lo) * torch.rand(n, 1, generator=g)   # spans both clamps
    points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, conf.numpy(), DEV)
    qr = LightningFastQuerier(DEV, o)
    campos = torch.from_numpy(view.campos).to(DEV)
    rot = torch.from_numpy(view.camrotc2w).to(DEV)
    raydir = torch.from_numpy(view.raydir).to(DEV)
    q = qr.query_samples(points.xyz, campos, raydir, 0.1, 8.0)
    S = q.n_samples()
    R = raydir.shape[0]
    valid = q.samp_nnb[:S] > 0
    feat = torch.rand(S, 4, generator=g).to(DEV)
    feat[:, 0] *= alpha_scale
    feat = torch.where(valid[:, None], feat, torch.zeros_like(feat))
    gt = torch.rand(R, 3, generator=g).to(DEV)
    qd = {"ray_ns": q.ray_ns[:R], "ray_soff": q.ray_soff[:R], "samp_ray": q.samp_ray[:S],
          "samp_locw": q.samp_locw[:S * 3].view(S, 3), "pidx": q.pidx[:S * o.K].view(S, o.K)}
    return o, points, q, qd, feat, valid, campos, rot, raydir, gt, R


@pytest.mark.parametrize("seed,SR,alpha_scale,conf_lo,conf_hi,unit,bgr", [
    (0, 24, 100.0, -0.1, 1.2, 0, False),    # config-5 shape, near-opaque samples, conf outside both clamps
    (1, 24, 2.0, 0.0, 1.0, 0, False),       # translucent
    (2, 64, 20.0, 0.0005, 0.9995, 1, False),  # SR 64, raydist_mode_unit, conf around the zero-one eps
    (1, 24, 2.0, 0.0, 1.0, 0, True),        # translucent, per-ray background (the plane model's bg_ray)
    (0, 24, 100.0, -0.1, 1.2, 0, True),
])
def test_loss_stage_matches_torch_autograd(seed, SR, alpha_scale, conf_lo, conf_hi, unit, bgr):
    """bgr: the rays' background is inputs['bg_ray'] [R, 3] (set_bg), composited as T_bg * bg_ray
    and taken by the rays without a valid sample (neural_points_volumetric_model.py:175-177)."""
    o, points, q, qd, feat, valid, campos, rot, raydir, gt, R = _case(seed, SR, alpha_scale, conf_lo, conf_hi,
                                                                     unit=unit)
    bg_ray = torch.rand(R, 3, generator=torch.Generator().manual_seed(seed + 40)).to(DEV) if bgr else None
    # torch restatement
    f_t = feat.clone().requires_grad_(True)
    points.points_conf.grad = None
    tot_t, parts_t, full_t, mask_t = composite_losses(points, qd, f_t, valid, campos, rot, raydir, gt, o,
                                                      bg=bg_ray if bgr else (1.0, 1.0, 1.0))
    tot_t.backward()
    dconf_t = points.points_conf.grad.clone()
    # HIP loss stage
    f_h = feat.clone().requires_grad_(True)
    points.points_conf.grad = None
    tot_h, parts_h, full_h, mask_h = LossStage(DEV)(points, q.abi(), f_h, campos, rot, gt, o, R, bg_ray=bg_ray)
    tot_h.backward()
    dconf_h = points.points_conf.grad.clone()
    torch.cuda.synchronize()
    assert int(mask_h.sum()) > 10 and int((~mask_h).sum()) > 0
    assert torch.equal(mask_h, mask_t)
    if bgr:   # the rays without a valid sample take their own background
        assert torch.equal(full_h[~mask_h], bg_ray[~mask_h])
    assert float((full_h - full_t.detach()).abs().max()) <= 1e-5
    assert abs(float(tot_h) - float(tot_t)) <= 1e-5 * abs(float(tot_t))
    for k in parts_t:
        a, b = float(parts_h[k]), float(parts_t[k])
        assert abs(a - b) <= 1e-5 * max(abs(b), 1e-12), (k, a, b)
    e_feat = _rel(f_h.grad, f_t.grad)
    e_conf = _rel(dconf_h, dconf_t)
    print(f"SR {SR}: d feat rel L2 {e_feat:.2e}, d conf rel L2 {e_conf:.2e}, valid rays {int(mask_h.sum())}/{R}")
    assert e_feat <= 1e-4 and e_conf <= 1e-4


def test_loss_stage_no_valid_ray():
    """A batch whose rays all miss: zero colour loss and gradients, the background colour, and the
    losses logged as the reference does (coarse colour over every ray)."""
    o = HotPathOpts(SR=24)
    pc = small_room(20_000, seed=3)
    points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, DEV)
    view = make_view(8, 8, yaw=210.0, pitch=80.0)    # looking away from the room
    campos = torch.from_numpy(view.campos).to(DEV) + torch.tensor([0.0, 0.0, 50.0], device=DEV)
    rot = torch.from_numpy(view.camrotc2w).to(DEV)
    raydir = torch.from_numpy(view.raydir).to(DEV)
    q = LightningFastQuerier(DEV, o).query_samples(points.xyz, campos, raydir, 0.1, 8.0)
    R = raydir.shape[0]
    feat = torch.zeros(max(q.n_samples(), 1), 4, device=DEV, requires_grad=True)
    gt = torch.rand(R, 3, device=DEV)
    tot, parts, full, mask = LossStage(DEV)(points, q.abi(), feat, campos, rot, gt, o, R)
    tot.backward()
    assert not bool(mask.any())
    assert torch.equal(full, torch.ones(R, 3, device=DEV))
    assert abs(float(parts["ray_masked_coarse_raycolor"])) == 0.0
    assert abs(float(parts["coarse_raycolor"]) - float(((1 - gt) ** 2).mean())) <= 1e-6
    assert float(feat.grad.abs().max()) == 0.0
