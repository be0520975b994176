"""Shared test helpers: seeded scenes, options, hyper-parameters, golden files."""
import os

import numpy as np
import torch

import sgnerf_amd  # noqa: F401
from sgnerf_amd import raygen, scene
from sgnerf_amd.hyper import grid_hyperparameters
from sgnerf_amd.opts import HotPathOpts


def small_room(n=200_000, seed=0):
    return scene.synth_room(n, seed=seed)


def hyper_for(pc, opts):
    return grid_hyperparameters(opts, torch.from_numpy(pc.xyz.min(0)), torch.from_numpy(pc.xyz.max(0)))


def make_view(h=48, w=64, yaw=30.0, pitch=-10.0, **kw):
    return scene.room_view(h, w, yaw=yaw, pitch=pitch, **kw)


def t_table(opts, near=0.1, far=8.0):
    return raygen.depth_table(near, far, opts.z_depth_dim)


def opts(**kw):
    return HotPathOpts(**kw)


def assert_equal_arrays(a, b, what):
    a = np.asarray(a)
    b = np.asarray(b)
    assert a.shape == b.shape, f"{what}: shape {a.shape} vs {b.shape}"
    if a.dtype.kind == "f":
        ok = np.array_equal(a.view(np.int32), b.astype(a.dtype).view(np.int32))
    else:
        ok = np.array_equal(a, b)
    if not ok:
        diff = np.nonzero((a != b).reshape(-1))[0]
        raise AssertionError(f"{what}: {diff.size} mismatches, first at {diff[:10]}: "
                             f"{a.reshape(-1)[diff[:5]]} vs {b.reshape(-1)[diff[:5]]}")


GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden_points(g, pcn):
    """A golden file's point cloud: stored arrays, or (`{pcn}/gen`) the seeded scene generator
    call the reference was run on, checked against the stored float64 checksums."""
    keys = ("xyz", "embedding", "color", "dir", "conf")
    if f"{pcn}/gen" not in g.files:
        return {k: g[f"{pcn}/{k}"] for k in keys}
    fn, n, seed = str(g[f"{pcn}/gen"]).split(":")
    pc = getattr(scene, fn)(int(n), int(seed))
    pts = dict(zip(keys, (pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf)))
    got = np.array([np.float64(pts[k]).sum() for k in keys])
    np.testing.assert_array_equal(got, g[f"{pcn}/checksum"], err_msg=f"regenerated cloud {pcn} differs")
    return pts


def load_golden(file, name):
    """(points, aggregator state, case arrays) of one golden case."""
    g = np.load(os.path.join(GOLDEN_DIR, file), allow_pickle=False)
    pts = golden_points(g, str(g[f"{name}/points"]))
    mlp = {k[4:]: torch.from_numpy(g[k]) for k in g.files if k.startswith("mlp/")}
    case = {k.split("/", 1)[1]: g[k] for k in g.files if k.startswith(name + "/")}
    return pts, mlp, case


def check_query_sample_major(q, ref, R, K):
    """A renderer's sample-major query (querier.QueryResult) against an oracle query of the same
    rays (OracleGrid.query, dense [R, SR, ...]): ray_ns, every sample's K neighbour indices,
    depth index and position, neighbour count and the work list, all bit-exact."""
    assert_equal_arrays(q.ray_ns[:R].cpu().numpy(), ref["ray_ns"], "ray_ns")
    S = q.n_samples()
    assert S == int(ref["ray_ns"].sum())
    sr = q.samp_ray[:S].cpu().numpy()
    slot = np.arange(S) - q.ray_soff[:R].cpu().numpy()[sr]
    assert_equal_arrays(q.pidx[:S * K].view(S, K).cpu().numpy(), ref["pidx"][sr, slot], "sample_pidx")
    assert_equal_arrays(q.samp_d[:S].cpu().numpy(), ref["ray_d"][sr, slot], "samp_d")
    assert_equal_arrays(q.samp_locw[:S * 3].view(S, 3).cpu().numpy(), ref["loc_w"][sr, slot], "sample_loc_w")
    nnb = (ref["pidx"][sr, slot] >= 0).sum(-1)
    assert_equal_arrays(q.samp_nnb[:S].cpu().numpy(), nnb, "samp_nnb")
    nwork = int(q.counters[1].item())
    assert_equal_arrays(np.sort(q.work[:nwork].cpu().numpy()), np.nonzero(nnb > 0)[0], "worklist")
    return S


def check_grid(g, og):
    """HipGrid.export() against the oracle's reference-format grid tensors, bit-exact."""
    coor_occ, coor_2_occ, numpnts, lists = g.export()
    assert_equal_arrays(coor_occ.cpu().numpy(), og.coor_occ, "coor_occ")
    assert_equal_arrays(coor_2_occ.cpu().numpy(), og.coor_2_occ, "coor_2_occ")
    assert_equal_arrays(numpnts.cpu().numpy(), og.occ_numpnts, "occ_numpnts")
    assert_equal_arrays(lists.cpu().numpy(), og.occ_2_pnts, "occ_2_pnts")
    assert g.info()["n_claimed"] == og.occ_idx
