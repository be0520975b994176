"""CPU: the oracle (and the host-side restatements) against the golden vectors
produced by the imported reference code (tests/golden/make_golden.py)."""
import os

import numpy as np
import pytest
import torch

import agg_ref
import oracle_query as oq
from helpers import assert_equal_arrays, load_golden
from sgnerf_amd import raygen
from sgnerf_amd.hyper import grid_hyperparameters
from sgnerf_amd.opts import HotPathOpts

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_aggregator.npz")
OPAQUE = ["opq_patch", "corner64", "sparse32"]   # reference_opaque.npz (alpha bias +50)
CASES = ["patch", "patch64", "dense"] + OPAQUE


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD, allow_pickle=False)


class _Gold:
    """One golden case under the flat `{name}/...` keys, its cloud regenerated when stored as
    a generator call."""

    def __init__(self, name):
        pts, mlp, c = load_golden("reference_opaque.npz" if name in OPAQUE else "reference_aggregator.npz", name)
        self.pts, self.mlp = pts, mlp
        self.d = {f"{name}/{k}": v for k, v in c.items()}
        self.d[f"{name}/points"] = np.array(name)
        for k, v in pts.items():
            self.d[f"{name}/{k}"] = v

    def __getitem__(self, k):
        return self.d[k]


def case(gold, name):
    if not isinstance(gold, _Gold):
        gold = _Gold(name)
    return {k: torch.from_numpy(v) for k, v in gold.pts.items()}, gold.mlp


def test_positional_encoding_golden(gold):
    x = torch.from_numpy(gold["pe/x"])
    assert_equal_arrays(agg_ref.positional_encoding(x, 3).numpy(), gold["pe/f3"], "PE f=3")
    assert_equal_arrays(agg_ref.positional_encoding(x[:, :3], 4, ori=True).numpy(), gold["pe/f4_ori"], "PE ori f=4")


@pytest.mark.parametrize("name", CASES)
def test_depth_table_and_raypos_golden(name):
    gold = _Gold(name)
    near, far = gold[f"{name}/near_far"]
    t = raygen.depth_table(float(near), float(far), 400)
    assert_equal_arrays(t.numpy(), gold[f"{name}/t_table"], "depth table")
    campos = gold[f"{name}/campos"]
    raydir = gold[f"{name}/raydir"]
    # raypos = campos + raydir * t with two fp32 roundings (diff_ray_marching.py:387)
    pos = campos[None, None, :] + (raydir[:4, None, :] * t.numpy()[None, :, None]).astype(np.float32)
    assert_equal_arrays(pos.astype(np.float32), gold[f"{name}/raypos_rays0_3"], "raypos")


@pytest.mark.parametrize("name", CASES)
def test_oracle_render_matches_reference(name):
    gold = _Gold(name)
    pts, mlp = case(gold, name)
    SR, K = int(gold[f"{name}/SR"]), int(gold[f"{name}/K"])
    o = HotPathOpts(SR=SR, K=K)
    xyz = gold[f"{str(gold[f'{name}/points'])}/xyz"]
    hy = grid_hyperparameters(o, torch.from_numpy(xyz.min(0)), torch.from_numpy(xyz.max(0)))
    og = oq.OracleGrid(xyz, hy, o)
    campos, rot, raydir = (torch.from_numpy(gold[f"{name}/{k}"]) for k in ("campos", "camrotc2w", "raydir"))
    q = og.query(gold[f"{name}/campos"], gold[f"{name}/raydir"], gold[f"{name}/t_table"])
    sp, sl, rm = oq.reference_layout(q)
    assert_equal_arrays(sp, gold[f"{name}/sample_pidx"], "sample_pidx (oracle determinism)")
    assert_equal_arrays(rm, gold[f"{name}/ray_mask"], "ray_mask")
    with torch.no_grad():
        full, ray_mask, fd, opacity, bg_t = agg_ref.render(pts, mlp, campos, rot, raydir, q, SR)
    keep = ray_mask.numpy()
    dec = gold[f"{name}/decoded"]
    np.testing.assert_allclose(fd[keep].numpy(), dec, atol=2e-6, rtol=1e-5)
    np.testing.assert_allclose(opacity[keep].numpy(), gold[f"{name}/opacity"], atol=2e-6, rtol=1e-5)
    np.testing.assert_allclose(bg_t[keep].numpy(), gold[f"{name}/bg_transmission"], atol=2e-6, rtol=1e-5)
    np.testing.assert_allclose(full.numpy(), gold[f"{name}/full_color"], atol=2e-6, rtol=1e-5)


# ---- SG-NeRF block2_bpnet variant (tests/golden/reference_sg.npz) -------------------
GOLD_SG = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_sg.npz")


def sg_case(g, name):
    pts = {k: torch.from_numpy(g[f"sgpatch/{k}"]) for k in ("xyz", "embedding", "color", "dir", "conf")}
    if name == "sg96":
        pts["bpnet"] = torch.from_numpy(g["sgpatch/bpnet"])
    pre = f"mlp_{name}/"
    mlp = {k[len(pre):]: torch.from_numpy(g[k]) for k in g.files if k.startswith(pre)}
    return pts, mlp


@pytest.mark.parametrize("name", ["sg96", "sg0"])
def test_oracle_sg_block2_bpnet_matches_reference(name):
    g = np.load(GOLD_SG, allow_pickle=False)
    pts, mlp = sg_case(g, name)
    assert mlp["block2_bpnet.0.weight"].shape[1] == (352 if name == "sg96" else 256)
    o = HotPathOpts(SR=int(g[f"{name}/SR"]))
    xyz = g["sgpatch/xyz"]
    hy = grid_hyperparameters(o, torch.from_numpy(xyz.min(0)), torch.from_numpy(xyz.max(0)))
    q = oq.OracleGrid(xyz, hy, o).query(g[f"{name}/campos"], g[f"{name}/raydir"], g[f"{name}/t_table"])
    sp, _, rm = oq.reference_layout(q)
    assert_equal_arrays(sp, g[f"{name}/sample_pidx"], "sample_pidx")
    campos, rot, raydir = (torch.from_numpy(g[f"{name}/{k}"]) for k in ("campos", "camrotc2w", "raydir"))
    with torch.no_grad():
        full, ray_mask, fd, opacity, bg_t = agg_ref.render(pts, mlp, campos, rot, raydir, q, o.SR)
    keep = ray_mask.numpy()
    np.testing.assert_allclose(fd[keep].numpy(), g[f"{name}/decoded"], atol=2e-6, rtol=1e-5)
    np.testing.assert_allclose(full.numpy(), g[f"{name}/full_color"], atol=2e-6, rtol=1e-5)
