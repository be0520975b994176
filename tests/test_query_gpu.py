"""GPU parity of the HIP grid build + march + layered kNN against the C
restatement (oracle/query_ref.c).  Bit-exact: integer indices and the fp32
sample positions must match exactly."""
import numpy as np
import pytest
import torch

from helpers import assert_equal_arrays, hyper_for, make_view, opts as mkopts, small_room, t_table
import oracle_query as oq

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _run(pc, o, view, per_ray_t=None, labels=None, seconds=0):
    from sgnerf_amd.querier import HipGrid, QueryWorkspace, run_query
    hy = hyper_for(pc, o)
    og = oq.OracleGrid(pc.xyz, hy, o)
    xyz = torch.from_numpy(pc.xyz).to(DEV)
    g = HipGrid(xyz, o, hyper=hy)
    if per_ray_t is None:
        t = t_table(o)
        per = 0
    else:
        t = per_ray_t
        per = 1
    R = view.raydir.shape[0]
    pl = rl = None
    if labels is not None:
        pl = torch.from_numpy(labels[0]).to(DEV)
        rl = torch.from_numpy(labels[1]).to(DEV)
    ws = QueryWorkspace(R, o.SR, o.K, DEV, dense=True)
    res = run_query(g, o, torch.from_numpy(view.campos).to(DEV), torch.from_numpy(view.raydir).to(DEV),
                    t.to(DEV), per, ws, dense=True, point_labels=pl, ray_labels=rl, seconds=seconds)
    torch.cuda.synchronize()
    ref = og.query(view.campos, view.raydir, t.numpy(), per_ray_t=bool(per),
                   point_labels=None if labels is None else labels[0],
                   ray_labels=None if labels is None else labels[1], seconds=seconds)
    return og, g, res, ref


def _check(og, g, res, ref, o):
    R = res.R
    coor_occ, coor_2_occ, numpnts, lists = g.export()
    assert_equal_arrays(coor_occ.cpu().numpy(), og.coor_occ, "coor_occ")
    assert_equal_arrays(coor_2_occ.cpu().numpy(), og.coor_2_occ, "coor_2_occ")
    assert_equal_arrays(numpnts.cpu().numpy(), og.occ_numpnts, "occ_numpnts")
    assert_equal_arrays(lists.cpu().numpy(), og.occ_2_pnts, "occ_2_pnts")
    assert g.info()["n_claimed"] == og.occ_idx
    assert_equal_arrays(res.ray_ns[:R].cpu().numpy(), ref["ray_ns"], "ray_ns")
    pidx = res.pidx[: R * o.SR * o.K].view(R, o.SR, o.K).cpu().numpy()
    assert_equal_arrays(pidx, ref["pidx"], "sample_pidx")
    S = res.n_samples()
    assert S == int(ref["ray_ns"].sum())
    sr = res.samp_ray[:S].cpu().numpy()
    slot = np.arange(S) - res.ray_soff[:R].cpu().numpy()[sr]
    assert_equal_arrays(res.samp_d[:S].cpu().numpy(), ref["ray_d"][sr, slot], "samp_d")
    assert_equal_arrays(res.samp_locw[: S * 3].view(S, 3).cpu().numpy(), ref["loc_w"][sr, slot], "sample_loc_w")
    nnb = (ref["pidx"][sr, slot] >= 0).sum(-1)
    assert_equal_arrays(res.samp_nnb[:S].cpu().numpy(), nnb, "samp_nnb")
    nwork = int(res.counters[1].item())
    work = np.sort(res.work[:nwork].cpu().numpy())
    assert_equal_arrays(work, np.nonzero(nnb > 0)[0], "worklist")


@pytest.fixture(scope="module")
def room():
    return small_room(200_000)


@pytest.mark.parametrize("kw", [
    dict(),                                  # ScanNet defaults (SR 24, K 8, P 26)
    dict(SR=64, K=16),
    dict(SR=1, K=4),
    dict(fix_occ0=1),
    dict(max_o=20_000, reservoir_seed=7),    # voxel reservoir (claim_occ :312-321)
    dict(P=2, reservoir_seed=3),             # point reservoir (fill_occ2pnts :400-407)
    dict(kernel_size=(5, 5, 5), query_size=(5, 5, 5)),
])
def test_query_parity(room, kw):
    o = mkopts(**kw)
    og, g, res, ref = _run(room, o, make_view(40, 56, yaw=35.0, pitch=-12.0))
    _check(og, g, res, ref, o)
    assert res.n_samples() > 0


@pytest.mark.parametrize("march", ["wave", "thread"])
def test_query_parity_both_march_kernels(room, march, monkeypatch):
    """Small batches march one wave per ray (k_march_wave), large ones a thread per ray
    (k_march): both give the oracle's slots (the threshold forced to 0 selects k_march)."""
    monkeypatch.setenv("SGN_MARCH_WAVE_MAX_RAYS", "1000000000" if march == "wave" else "0")
    for kw in (dict(), dict(SR=64, K=16), dict(SR=1, K=4)):
        o = mkopts(**kw)
        og, g, res, ref = _run(room, o, make_view(40, 56, yaw=35.0, pitch=-12.0))
        _check(og, g, res, ref, o)


@pytest.mark.parametrize("march", ["wave", "thread"])
def test_query_parity_jittered_rays(room, march, monkeypatch):
    monkeypatch.setenv("SGN_MARCH_WAVE_MAX_RAYS", "1000000000" if march == "wave" else "0")
    o = mkopts(SR=32)
    view = make_view(24, 24, yaw=200.0, pitch=5.0)
    R = view.raydir.shape[0]
    from sgnerf_amd.raygen import depth_table
    t = depth_table(0.1, 8.0, o.z_depth_dim, jitter=0.3, R=R, generator=torch.Generator().manual_seed(0))
    og, g, res, ref = _run(room, o, view, per_ray_t=t)
    _check(og, g, res, ref, o)


@pytest.mark.parametrize("R,D", [(1, 1), (3, 64), (257, 400), (4096, 400)])
def test_depth_table_jitter_hip_matches_torch(R, D):
    """sgn_depth_table_jitter against raygen.depth_table (the torch restatement of
    near_far_linear_ray_generation) on the same torch.rand draw: the cumsum's order differs (wave
    scan vs torch's scan), so within 4 ulp of far (4.8e-6 at 8.0); strictly increasing per ray."""
    from sgnerf_amd.querier import depth_table_jitter_hip
    from sgnerf_amd.raygen import depth_table
    t = depth_table_jitter_hip(0.1, 8.0, D, 0.3, R, DEV, generator=torch.Generator(DEV).manual_seed(7))
    ref = depth_table(0.1, 8.0, D, jitter=0.3, R=R, device=DEV, generator=torch.Generator(DEV).manual_seed(7))
    assert t.shape == ref.shape == (R, D)
    assert float((t - ref).abs().max()) <= 4.8e-6
    if D > 1:
        assert bool((t[:, 1:] > t[:, :-1]).all())
    assert float(t.min()) > 0.1


@pytest.mark.parametrize("seconds", [3, 11])
def test_query_parity_semantic(room, seconds):
    o = mkopts(semantic_guidance=1)
    view = make_view(24, 32, yaw=120.0)
    rng = np.random.default_rng(5)
    labels = (rng.integers(0, 4, room.n).astype(np.int32), rng.integers(0, 4, view.raydir.shape[0]).astype(np.int32))
    og, g, res, ref = _run(room, o, view, labels=labels, seconds=seconds)
    _check(og, g, res, ref, o)


def test_query_edge_cases():
    # single point: it owns occupancy id 0, so the `> 0` bug leaves its list empty
    pc = small_room(1)
    o = mkopts()
    view = make_view(8, 8)
    og, g, res, ref = _run(pc, o, view)
    _check(og, g, res, ref, o)
    assert int(res.counters[1].item()) == 0
    # camera outside the scene looking away: no flagged candidate at all
    pc = small_room(50_000)
    view = make_view(8, 8, yaw=0.0, pitch=0.0, campos=(-5.0, 2.0, 1.5))
    view.raydir[:] = -view.raydir
    og, g, res, ref = _run(pc, o, view)
    _check(og, g, res, ref, o)
    assert res.n_samples() == 0


def test_query_points_reference_layout(room):
    """LightningFastQuerier.query_points returns the reference's 7-tuple layout."""
    from sgnerf_amd.querier import LightningFastQuerier
    o = mkopts()
    view = make_view(32, 40, yaw=60.0)
    q = LightningFastQuerier(DEV, o)
    xyz = torch.from_numpy(room.xyz).to(DEV)
    campos = torch.from_numpy(view.campos).to(DEV)[None]
    rot = torch.from_numpy(view.camrotc2w).to(DEV)[None]
    raydir = torch.from_numpy(view.raydir).to(DEV)[None]
    out = q.query_points(None, None, xyz[None], None, view.h, view.w, view.intrinsic, 0.1, 8.0, raydir, campos, rot)
    sample_pidx, sample_loc, sample_loc_w, sample_ray_dirs, ray_mask, vsize, ranges = out
    hy = hyper_for(room, o)
    og = oq.OracleGrid(room.xyz, hy, o)
    ref = og.query(view.campos, view.raydir, t_table(o).numpy())
    rp, rl, rm = oq.reference_layout(ref)
    assert_equal_arrays(ray_mask[0].cpu().numpy(), rm, "ray_mask")
    assert_equal_arrays(sample_pidx[0].cpu().numpy(), rp, "sample_pidx")
    assert_equal_arrays(sample_loc_w[0].cpu().numpy(), rl, "sample_loc_w")
    assert sample_ray_dirs.shape == (1, rp.shape[0], o.SR, 3)
    assert sample_loc.shape == sample_loc_w.shape
    np.testing.assert_array_equal(ranges, hy.ranges)
