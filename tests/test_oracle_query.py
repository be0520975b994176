"""Known-answer tests of the query restatement (oracle/query_ref.c) on a hand-built
6x6x6 grid of unit voxels, with the expected values worked out by hand from the
reference kernels (models/neural_points/query_point_indices_worldcoords.py):

  claim_occ :265-326        occupancy ids in point order (parity mode)
  map_coor2occ :328-363     coor_occ = 1 on the query_size neighbourhood of claimed voxels
  fill_occ2pnts :365-410    lists in point order, `voxel_idx > 0` drops occ id 0,
                            reservoir above P (counter keeps counting)
  mask_raypos + compaction  first SR flagged candidates become the shading samples
  layered kNN :594-681      Chebyshev layers, x/y/z loop order, fill then replace-farthest

The same cases run on the GPU path (bit-exact) in the `gpu`-marked tests below."""
import types

import numpy as np
import pytest
import torch

import oracle_query as oq
from sgnerf_amd.opts import HotPathOpts

PTS = np.array([[0.5, 0.5, 0.5],    # 0 -> voxel (0,0,0), occ id 0 (dropped by the >0 bug)
                [2.5, 2.5, 2.5],    # 1 -> (2,2,2), occ id 1
                [2.2, 2.6, 2.4],    # 2 -> (2,2,2)
                [2.9, 2.1, 2.8],    # 3 -> (2,2,2): third point with P = 2 -> reservoir
                [3.5, 2.5, 2.5],    # 4 -> (3,2,2), occ id 2
                [-1.0, 0.0, 0.0]],  # 5 -> outside the grid, ignored
               np.float32)


def _hyper(r2=0.0):
    return types.SimpleNamespace(shift=np.zeros(3, np.float32), scaled_vsize=np.ones(3, np.float32),
                                 scaled_vdim=np.array([6, 6, 6], np.int32), r2=np.float32(r2))


def _opts(**kw):
    base = dict(max_o=100, P=2, K=2, SR=3, reservoir_seed=7, fix_occ0=0)
    base.update(kw)
    return HotPathOpts(**base)


def _reservoir_slot(seed, i_pt=3, tmp=2, P=2):
    """fill_occ2pnts :399-407: insrtidx = ceilf(u * (tmp + 1)) - 1, u from the parity-mode draw."""
    u = oq.lib().sgnref_uniform(seed, 2, i_pt)  # stream 2 = fill_occ2pnts draws
    j = int(np.ceil(np.float32(u) * np.float32(tmp + 1))) - 1
    return j if j < P else None


@pytest.mark.parametrize("fix", [0, 1])
def test_grid_structures(fix):
    o = _opts(fix_occ0=fix)
    g = oq.OracleGrid(PTS, _hyper(), o)
    assert g.occ_idx == 3
    c2o = g.coor_2_occ
    assert c2o[0, 0, 0] == 0 and c2o[2, 2, 2] == 1 and c2o[3, 2, 2] == 2
    assert (c2o >= 0).sum() == 3
    # coor_occ: 3x3x3 neighbourhoods of (0,0,0), (2,2,2), (3,2,2)
    want = np.zeros((6, 6, 6), bool)
    for c in [(0, 0, 0), (2, 2, 2), (3, 2, 2)]:
        lo = [max(0, x - 1) for x in c]
        hi = [min(6, x + 2) for x in c]
        want[lo[0]:hi[0], lo[1]:hi[1], lo[2]:hi[2]] = True
    np.testing.assert_array_equal(g.coor_occ.astype(bool), want)
    # lists
    assert g.occ_numpnts[0] == (1 if fix else 0)
    if fix:
        assert g.occ_2_pnts[0, 0] == 0
    assert g.occ_numpnts[1] == 3            # the counter keeps counting past P
    lst = [1, 2]
    j = _reservoir_slot(o.reservoir_seed)
    if j is not None:
        lst[j] = 3
    assert list(g.occ_2_pnts[1, :2]) == lst
    assert g.occ_numpnts[2] == 1 and g.occ_2_pnts[2, 0] == 4


def _knn(g, center, o):
    out = np.full(o.K, -1, np.int32)
    p = g.params
    oq.lib().sgnref_knn_one(p, oq._p(g.xyz), oq._p(g.coor_2_occ.reshape(-1)), oq._p(g.occ_numpnts),
                            oq._p(g.occ_2_pnts.reshape(-1)), oq._p(np.asarray(center, np.float32)), oq._p(out),
                            None, 0, 0)
    return list(out)


def test_knn_layers_fill_and_replace():
    o = _opts(reservoir_seed=1)
    g = oq.OracleGrid(PTS, _hyper(), o)
    lst = [int(x) for x in g.occ_2_pnts[1, :2]]
    # centre voxel (2,2,2): layer 0 fills the first K list entries in list order, then stops
    assert _knn(g, [2.5, 2.5, 2.5], o) == lst
    # centre voxel (3,3,2): layer 1 visits (2,2,2) (x=-1 first), then (3,2,2); point 4
    # (d2 = 1.0) replaces the farthest of the filled pair
    got = _knn(g, [3.5, 3.5, 2.5], o)
    d2 = {i: float(((PTS[i] - np.float32([3.5, 3.5, 2.5])) ** 2).sum()) for i in range(5)}
    far = int(np.argmax([d2[lst[0]], d2[lst[1]]]))
    want = list(lst)
    if d2[4] < d2[lst[far]]:
        want[far] = 4
    assert got == want


def test_knn_radius_and_occ0_bug():
    g = oq.OracleGrid(PTS, _hyper(r2=1.5), _opts())
    assert _knn(g, [3.5, 3.5, 2.5], _opts()) == [4, -1]        # 2.0 and 2.51 are outside r2
    assert _knn(g, [0.5, 0.5, 0.5], _opts()) == [-1, -1]       # occ id 0 has an empty list (bug)
    gf = oq.OracleGrid(PTS, _hyper(r2=1.5), _opts(fix_occ0=1))
    assert _knn(gf, [0.5, 0.5, 0.5], _opts(fix_occ0=1)) == [0, -1]


def test_march_first_sr_flagged_candidates():
    o = _opts(reservoir_seed=1)
    g = oq.OracleGrid(PTS, _hyper(), o)
    campos = np.array([0.1, 2.5, 2.5], np.float32)
    raydir = np.array([[1.0, 0.0, 0.0], [0.0, 0.0, 1.0]], np.float32)
    t = np.array([0.5, 1.5, 2.5, 3.5, 4.5, 5.5], np.float32)
    q = g.query(campos, raydir, t)
    # ray 0: x = 0.6 .. 5.6 along y = z = 2.5: flagged voxels x = 1..4, first SR = 3 kept
    assert q["ray_ns"][0] == 3
    np.testing.assert_array_equal(q["ray_d"][0], [1, 2, 3])
    np.testing.assert_allclose(q["loc_w"][0, :, 0], campos[0] + t[1:4], rtol=0, atol=1e-6)
    # ray 1: (0.1, 2.5, 3.0..8.0) -> voxels (0, 2, 3..5): none flagged
    assert q["ray_ns"][1] == 0
    assert np.all(q["pidx"][1] == -1)
    # sample (1.6, 2.5, 2.5): layer 1 reaches (2,2,2) only
    lst = [int(x) for x in g.occ_2_pnts[1, :2]]
    assert list(q["pidx"][0, 0]) == lst


# ---- the same known answers on the GPU path -----------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("fix", [0, 1])
def test_gpu_matches_known_answers(fix):
    from sgnerf_amd.querier import HipGrid, QueryWorkspace, run_query
    dev = "cuda:0"
    o = _opts(fix_occ0=fix, reservoir_seed=1, K=4)  # the GPU kNN is instantiated for K = 1, 4, 8, 16
    hy = types.SimpleNamespace(shift=np.zeros(3, np.float32), scaled_vsize=np.ones(3, np.float32),
                               scaled_vdim=np.array([6, 6, 6], np.int32), r2=np.float32(0.0), volume=216)
    g = HipGrid(torch.from_numpy(PTS).to(dev), o, hyper=hy)
    coor_occ, coor_2_occ, numpnts, o2p = g.export()
    ref = oq.OracleGrid(PTS, _hyper(), o)
    np.testing.assert_array_equal(coor_2_occ.cpu().numpy().reshape(6, 6, 6), ref.coor_2_occ)
    np.testing.assert_array_equal(numpnts.cpu().numpy()[:3], ref.occ_numpnts[:3])
    campos = np.array([0.1, 2.5, 2.5], np.float32)
    raydir = np.array([[1.0, 0.0, 0.0], [0.0, 0.0, 1.0]], np.float32)
    t = np.array([0.5, 1.5, 2.5, 3.5, 4.5, 5.5], np.float32)
    ws = QueryWorkspace(2, o.SR, o.K, dev, dense=True)
    res = run_query(g, o, torch.from_numpy(campos).to(dev), torch.from_numpy(raydir).to(dev),
                    torch.from_numpy(t).to(dev), 0, ws, dense=True)
    q = ref.query(campos, raydir, t)
    np.testing.assert_array_equal(res.ray_ns[:2].cpu().numpy(), q["ray_ns"])
    np.testing.assert_array_equal(res.pidx[: 2 * o.SR * o.K].view(2, o.SR, o.K).cpu().numpy(), q["pidx"])
