"""The model plugin's host-side surface on the CPU (no kernels run): checkpoint keys the
reference's NeuralPoints reads, the train_ft.py save block and probe guard, the ray-miss
ranking, the semantic point dumps and set_bg's plane background.

  run/train_ft.py:1006-1020   save block (saveSemanticEmbedding + save_networks in try/except)
  run/train_ft.py:888-891     probe guard (top_ray_miss_loss[0] > 1e-5 ...)
  models/neural_points/neural_points.py:321-386   checkpoint key reads
  models/mvs_points_volumetric_model.py:157-189   update_rank_ray_miss / rank_ray_miss / reset
  models/neural_points_volumetric_model.py:674-720 saveSemanticPoints(_test) text format
"""
import argparse
import os
import types

import numpy as np
import pytest
import torch

from sgnerf_amd.model import LABEL_RGB, HipPointsVolumetricModel, label_colours
from sgnerf_amd.ray_marching import NeuralPoints

N = 50


def _points(seed=0, labels=True, bpnet=True):
    g = torch.Generator().manual_seed(seed)
    r = lambda *s: torch.rand(*s, generator=g)  # noqa: E731
    lab = torch.randint(0, 20, (N,), generator=g)
    lab[:3] = 255
    return NeuralPoints(r(N, 3), r(1, N, 32), r(1, N, 3), r(1, N, 3), r(1, N, 1), "cpu",
                        points_feats=r(N, 3) * 255, points_label=lab if labels else None,
                        bpnet_points_embedding=r(N, 96) if bpnet else None)


def _model(tmp_path, **extra):
    opt = argparse.Namespace(SR=24, K=8, gpu_ids=[0], is_train=True, checkpoints_dir=str(tmp_path), name="scene",
                             bg_color="white", **extra)
    m = HipPointsVolumetricModel()
    m.initialize(opt)
    m.device = torch.device("cpu")     # host-only: no renderer, no kernels
    m.is_train = False                 # no HipTrainer (setup() would build one)
    m.neural_points = _points()
    mlp = {"block1.0.weight": torch.ones(2, 2)}
    m.net_ray_marching = types.SimpleNamespace(renderer=types.SimpleNamespace(mlp_state=mlp))
    return m


def _reference_key_reads(sd):
    """What NeuralPoints.__init__ reads from a checkpoint (neural_points.py:332-386): xyz and
    points_feats unconditionally, the rest when present."""
    got = {"xyz": sd["neural_points.xyz"], "points_feats": sd["neural_points.points_feats"]}
    for k in ("points_embeding", "points_conf", "points_dir", "points_color", "eulers", "Rw2c"):
        if "neural_points." + k in sd:
            got[k] = sd["neural_points." + k]
    return got


def test_checkpoint_keys_round_trip(tmp_path):
    m = _model(tmp_path)
    m.save_networks(7, {"total_steps": 7})
    sd = torch.load(tmp_path / "scene" / "7_net_ray_marching.pth", map_location="cpu", weights_only=True)
    got = _reference_key_reads(sd)
    p = m.neural_points
    assert got["points_feats"].shape == (N, 3) and torch.equal(got["points_feats"], p.points_feats)
    assert got["points_embeding"].shape == (1, N, 32)
    assert torch.equal(sd["neural_points.points_label"].reshape(-1), p.points_label.reshape(-1))
    assert sd["neural_points.bpnet_points_embedding"].shape == (1, N, 96)
    assert "aggregator.block1.0.weight" in sd
    q = NeuralPoints.from_state_dict(sd, "cpu")
    for k in ("xyz", "points_embeding", "points_color", "points_dir", "points_conf", "points_feats", "points_label",
              "bpnet_points_embedding"):
        assert torch.equal(getattr(q, k), getattr(p, k)), k
    # without the optional semantic keys the file still loads (labels / embedding stay unset)
    for k in ("neural_points.points_label", "neural_points.bpnet_points_embedding"):
        del sd[k]
    q = NeuralPoints.from_state_dict(sd, "cpu")
    assert q.points_label is None and q.bpnet_points_embedding is None
    assert torch.load(tmp_path / "scene" / "7_states.pth", weights_only=True) == {"total_steps": 7}


def test_save_block_replay(tmp_path):
    """train_ft.py:1006-1020 with total_steps == 1: embedding dump, then the checkpoint."""
    m = _model(tmp_path)
    total_steps, best_PSNR, best_iter, epoch = 1, 0.0, 0, 0
    errors = []
    try:
        if total_steps == 1 or (total_steps % 1000 == 0 and total_steps > 0):
            m.saveSemanticEmbedding(total_steps)
            other_states = {"best_PSNR": best_PSNR, "best_iter": best_iter, "epoch_count": epoch,
                            "total_steps": total_steps}
            m.save_networks(total_steps, other_states)
    except Exception as e:  # the reference prints and carries on
        errors.append(e)
    assert not errors
    emb = torch.load(tmp_path / "scene" / "1_semanticEmbedding.pth", weights_only=True)
    assert emb.shape == (N, 96) and torch.equal(emb, m.neural_points.bpnet_points_embedding[0])
    assert (tmp_path / "scene" / "1_net_ray_marching.pth").is_file()
    # before BPNet ran the reference saves None
    m.neural_points.bpnet_points_embedding = None
    m.saveSemanticEmbedding(2)
    assert torch.load(tmp_path / "scene" / "2_semanticEmbedding.pth", weights_only=True) is None


def _rank_ref(new_id, newloss, inds, losses):
    """Plain restatement of mvs_points_volumetric_model.py:166-176 on lists."""
    inds, losses = list(inds), list(losses)
    hit = [i for i, x in enumerate(inds) if x == new_id]
    if hit:
        for i in hit:
            losses[i] = max(newloss, losses[i])
    else:
        inds[-1], losses[-1] = new_id, newloss
    order = sorted(range(len(losses)), key=lambda i: -losses[i])
    return [losses[i] for i in order], [inds[i] for i in order]


def test_ray_miss_ranking_and_probe_guard(tmp_path):
    m = _model(tmp_path, prob_freq=10, prob_num_step=4, prob_kernel_size=None, prob_mode=0, far_thresh=-1.0)
    m.setup(m.opt, train_len=20)
    assert m.num_probe == 5
    assert m.top_ray_miss_loss.tolist() == [0.0] * 6 and m.top_ray_miss_ids.tolist() == list(range(6))
    assert m.top_ray_miss_ids.dtype == torch.int32
    rng = np.random.default_rng(0)
    ref_l, ref_i = [0.0] * 6, list(range(6))
    for step in range(40):
        fid = int(rng.integers(0, 20))
        loss = float(rng.random()) * 1e-3      # distinct losses: the sort has no ties
        m.input = {"id": torch.tensor([fid])}
        m.loss_ray_miss_coarse_raycolor = torch.tensor(loss)
        m.update_rank_ray_miss(step)
        ref_l, ref_i = _rank_ref(fid, loss, ref_i, ref_l)
        np.testing.assert_allclose(m.top_ray_miss_loss.numpy(), np.float32(ref_l), rtol=0, atol=0)
        assert m.top_ray_miss_ids.tolist() == ref_i
    # train_ft.py:888-891 probe guard reads the ranking's head
    opt = m.opt
    assert (m.top_ray_miss_loss[0] > 1e-5 or opt.prob_mode != 0 or opt.far_thresh > 0)
    # the probe resets the ranking afterwards (train_ft.py:532-533)
    m.reset_ray_miss_ranking()
    assert not (m.top_ray_miss_loss[0] > 1e-5 or opt.prob_mode != 0 or opt.far_thresh > 0)
    # prob_num_step == 1: a running maximum in one slot
    m1 = _model(tmp_path, prob_freq=10, prob_num_step=1, prob_kernel_size=None)
    m1.setup(m1.opt, train_len=20)
    for loss in (0.3, 0.7, 0.5):
        m1.input = {"id": torch.tensor([0])}
        m1.loss_ray_miss_coarse_raycolor = torch.tensor(loss)
        m1.update_rank_ray_miss(1)
    assert m1.top_ray_miss_loss.tolist() == [pytest.approx(0.7)]
    # past the last probe tier nothing is ranked (mvs_points_volumetric_model.py:158)
    m2 = _model(tmp_path, prob_freq=10, prob_num_step=4, prob_kernel_size=[1.0, 1.0, 1.0], prob_tiers=[5])
    m2.setup(m2.opt, train_len=20)
    m2.input = {"id": torch.tensor([3])}
    m2.loss_ray_miss_coarse_raycolor = torch.tensor(0.5)
    m2.update_rank_ray_miss(100)
    assert float(m2.top_ray_miss_loss.max()) == 0.0
    m2.update_rank_ray_miss(2)
    assert float(m2.top_ray_miss_loss[0]) == 0.5


def test_semantic_point_dumps(tmp_path):
    m = _model(tmp_path)
    p = m.neural_points
    f = m.saveSemanticPoints(1000)
    assert f == os.path.join(str(tmp_path), "scene", "predict_points_1000.txt")
    a = np.loadtxt(f)
    assert a.shape == (N, 6)
    np.testing.assert_allclose(a[:, :3], p.xyz.numpy(), atol=5e-7)
    want = np.array([LABEL_RGB[int(x)] for x in p.points_label.reshape(-1)], np.float64)
    np.testing.assert_array_equal(a[:, 3:], want)
    with open(f) as fh:
        assert fh.readline().split()[3] == "255.000000"      # np.savetxt fmt="%f" as the reference
    g = m.saveSemanticPoints_test(300, 2)
    assert g.endswith(os.path.join("test_300", "test_predict_points_iter300_imgNum2.txt"))
    np.testing.assert_array_equal(np.loadtxt(g), a)
    with pytest.raises(KeyError):
        label_colours([21])
    m.neural_points.points_label = None
    with pytest.raises(RuntimeError):
        m.saveSemanticPoints(1)


def _plane_bg_loops(campos, raydir, pnt, nrm, imgs, w2cs, Ks, plane_color, pts, thresh=0.03):
    """Independent float64 restatement of set_bg (mvs_points_volumetric_model.py:276-315 over
    mvs_utils.py:299-420) with explicit loops: per ray and view the plane point's projection, the
    foreground test at its ceil'd pixel, a hand-written bilinear tap (align_corners, zero padding).
    Returns bg [R,3] and, per (ray, view), the sampled colour's distance to the fit boundary."""
    R, V = raydir.shape[0], len(imgs)
    bg = np.zeros((R, 3))
    margin = np.full((R, V), np.inf)
    for v in range(V):
        _, C, H, W = imgs[v].shape
        w2c, K = w2cs[v][0, 0], Ks[v][0]

        def proj(x):
            c = w2c @ np.append(x, 1.0)
            with np.errstate(divide="ignore", invalid="ignore"):   # z = 0: nan / inf, outside the image
                return (K @ (c[:3] / c[2]))[:2]
        fg = np.zeros((H, W), bool)
        for x in pts:
            u = proj(x)
            if 0 <= u[0] <= W - 1 and 0 <= u[1] <= H - 1:
                fg[int(np.ceil(u[1])), int(np.ceil(u[0]))] = True
        for r in range(R):
            d = raydir[r]
            dot = nrm @ d
            hit = campos + d * (-(nrm @ (campos - pnt)) / dot) if dot >= 1e-3 else np.zeros(3)
            u = proj(hit)
            if not (0 <= u[0] <= W - 1 and 0 <= u[1] <= H - 1) or fg[int(np.ceil(u[1])), int(np.ceil(u[0]))]:
                s = np.zeros(3)
            else:
                x0, y0 = int(np.floor(u[0])), int(np.floor(u[1]))
                fx, fy = u[0] - x0, u[1] - y0
                s = np.zeros(3)
                for (yy, xx, wt) in ((y0, x0, (1 - fx) * (1 - fy)), (y0, x0 + 1, fx * (1 - fy)),
                                     (y0 + 1, x0, (1 - fx) * fy), (y0 + 1, x0 + 1, fx * fy)):
                    if 0 <= yy < H and 0 <= xx < W:
                        s = s + wt * imgs[v][0, :, yy, xx]
            dist = np.abs(np.abs(s - plane_color) - thresh).min()
            margin[r, v] = dist
            if np.all(np.abs(s - plane_color) <= thresh):
                bg[r] = np.maximum(bg[r], s)
    return bg, margin


def test_set_bg_plane_background_matches_loops(tmp_path):
    """set_bg (bgmodel '*plane'): the rays' plane points warped into two source views, foreground
    pixels (where neural points project) excluded, colours within 0.03 of the plane colour kept, max
    over views -- against the explicit-loop restatement above (rays whose sampled colour sits within
    1e-4 of the fit boundary are skipped: float32 vs float64 may decide them either way)."""
    from sgnerf_amd.plane_bg import gen_bg_points
    m = _model(tmp_path)
    g = np.random.default_rng(3)
    H, W, pc = 12, 16, np.array([0.5, 0.4, 0.3])
    imgs = []
    for v in range(2):
        im = pc[None, :, None, None] + g.uniform(-0.02, 0.02, (1, 3, H, W))
        far = g.random((H, W)) < 0.3
        im[0][:, far] = g.uniform(0, 1, (3, int(far.sum())))
        imgs.append(im.astype(np.float32))
    Ks = [np.array([[[8.0, 0, 7.5], [0, 8.0, 5.5], [0, 0, 1]]], np.float32)] * 2
    w2cs = []
    for t in ([0.1, -0.05, 0.0], [-0.15, 0.1, 0.2]):
        e = np.eye(4, dtype=np.float32)
        e[:3, 3] = -np.array(t, np.float32)
        w2cs.append(e[None, None])
    campos = np.zeros(3, np.float32)
    d = np.stack([g.uniform(-0.8, 0.8, 60), g.uniform(-0.6, 0.6, 60), np.ones(60)], -1).astype(np.float32)
    d[:3] = [[0.2, 0.1, -1.0], [0.0, 0.0, 1e-4], [1.5, 0.0, 1.0]]   # away from the plane, parallel, off-image
    pnt, nrm = np.array([0.0, 0.0, 2.0], np.float32), np.array([0.0, 0.0, 1.0], np.float32)
    pts = np.concatenate([g.uniform(-0.5, 0.5, (12, 2)), np.full((12, 1), 2.0)], -1).astype(np.float32)
    m.neural_points.xyz = torch.from_numpy(pts)
    batch = {"campos": torch.from_numpy(campos)[None], "raydir": torch.from_numpy(d)[None],
             "plane_pnt": torch.from_numpy(pnt)[None], "plane_normal": torch.from_numpy(nrm)[None]}
    xyz = gen_bg_points(batch)
    bg, fgm = m.set_bg(xyz, [torch.from_numpy(i) for i in imgs], None, [torch.from_numpy(w) for w in w2cs],
                       [torch.from_numpy(k) for k in Ks], [(H, W)] * 2, torch.from_numpy(pc.astype(np.float32)))
    assert bg.shape == (1, 60, 3) and fgm is None
    ref, margin = _plane_bg_loops(campos.astype(np.float64), d.astype(np.float64), pnt, nrm, imgs, w2cs, Ks, pc,
                                  pts.astype(np.float64))
    ok = margin.min(1) > 1e-4
    assert ok.sum() >= 40 and (ref[ok].sum(1) > 0).sum() >= 10   # enough rays decided, some with a background
    np.testing.assert_allclose(bg[0].numpy()[ok], ref[ok], atol=1e-5)
    np.testing.assert_array_equal(bg[0, :3].numpy(), 0.0)   # behind the camera, parallel, off both images


def test_set_points_reference_signature(tmp_path):
    """mvs_points_volumetric_model.py:191 argument names, as run/train_ft.py:797 passes them."""
    m = _model(tmp_path)
    p = _points(1)
    kw = dict(points_xyz=p.xyz, points_feats=p.points_feats, points_embedding=p.points_embeding,
              points_color=p.points_color, points_dir=p.points_dir, points_conf=p.points_conf, Rw2c=None)
    # a renderer already exists: the new points are bound to it without repacking weights
    m._sync_weights = lambda: None
    m.set_points(**kw)
    assert torch.equal(m.neural_points.points_feats, p.points_feats)
    assert m.net_ray_marching.neural_points is m.neural_points
    with pytest.raises(NotImplementedError):
        m.set_points(**kw, editing=True)


def test_sg_optimize_without_bpnet_embedding_raises(tmp_path):
    """SG with predict_semantic = 1: setup_optimizer leaves the trainer unset until the BPNet
    embedding exists (neural_points.py:653-665); optimize_parameters then says so instead of
    failing on a None trainer."""
    m = _model(tmp_path, shading_feature_mlp_layer2_bpnet=1, predict_semantic=1, semantic_guidance=1)
    m.neural_points = _points(bpnet=False)
    m.input = {}
    with pytest.raises(ValueError, match="BPNet embedding"):
        m.optimize_parameters(total_steps=1)
