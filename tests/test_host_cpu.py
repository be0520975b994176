"""CPU tests of the host side: the C ABI surface (library loads, exports every symbol
include/sgn_hip.h declares, validates its arguments before touching the GPU), the
option/hyper-parameter logic, weight handling and the reference bookkeeping
(fill_invalid, ray-slot densification) that runs in torch around the kernels."""
import argparse
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from sgnerf_amd import _lib, raygen
from sgnerf_amd.hyper import grid_hyperparameters
from sgnerf_amd.opts import HotPathOpts
from sgnerf_amd.ray_marching import _dense_from_samples, fill_invalid
from sgnerf_amd.weights import LAYERS, N_PARAMS, check_shapes, init_mlp, strip_prefix

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "sgn_hip.h")


def _header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"^[A-Za-z_][\w \t\*]*?\b(sgn_\w+)\s*\(", txt, flags=re.M)))


def test_header_declares_the_boundary():
    names = _header_functions()
    for n in ("sgn_grid_build", "sgn_grid_free", "sgn_query", "sgn_aggregate", "sgn_composite",
              "sgn_ray_march_dense", "sgn_mlp_pack", "sgn_abi_version", "sgn_last_error"):
        assert n in names
    assert set(names) == set(_lib.SIGNATURES), "ctypes SIGNATURES must bind exactly what the header declares"


def test_library_loads_and_exports_every_symbol():
    L = _lib.lib()
    raw = ctypes.CDLL(_lib.LIB_PATH)
    for n in _header_functions():
        assert hasattr(raw, n), f"libsgn_hip.so does not export {n}"
    v = int(re.search(r"#define SGN_ABI_VERSION (\d+)", open(HEADER).read()).group(1))
    assert L.sgn_abi_version() == v == _lib.ABI_VERSION


def test_integration_snippet_matches_binding():
    """INTEGRATION.md §3's reference-side ctypes binding: its ABI constant and struct definitions,
    executed, must equal sgnerf_amd._lib's (sizeof, field names, offsets, types) and the header's
    SGN_ABI_VERSION -- a snippet a maintainer copies must not pass a struct of the wrong size."""
    import ast
    txt = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = txt[txt.index("## 3. ctypes binding"):txt.index("## 4.")]
    code = re.search(r"```python\n(.*?)```", sec, flags=re.S).group(1)
    tree = ast.parse(code)
    keep = [n for n in tree.body if isinstance(n, ast.ClassDef) or
            (isinstance(n, ast.Assign) and any(getattr(t, "id", "") == "SGN_ABI_VERSION" for t in n.targets))]
    ns = {"ctypes": ctypes}
    exec(compile(ast.Module(body=keep, type_ignores=[]), "INTEGRATION.md", "exec"), ns)
    hdr = int(re.search(r"#define SGN_ABI_VERSION (\d+)", open(HEADER).read()).group(1))
    assert ns["SGN_ABI_VERSION"] == _lib.ABI_VERSION == hdr
    classes = [n.name for n in keep if isinstance(n, ast.ClassDef)]
    assert {"QueryParams", "LossParams"} <= set(classes)
    for name in classes:
        mine, ref = ns[name], getattr(_lib, name)
        assert ctypes.sizeof(mine) == ctypes.sizeof(ref), name
        fm = [(f[0], getattr(mine, f[0]).offset, ctypes.sizeof(f[1])) for f in mine._fields_]
        fr = [(f[0], getattr(ref, f[0]).offset, ctypes.sizeof(f[1])) for f in ref._fields_]
        assert fm == fr, name


def test_sizing_functions():
    L = _lib.lib()
    assert L.sgn_mlp_packed_bytes() > 2 * N_PARAMS  # fp16 fragments (+ padding) + fp32 params
    assert L.sgn_query_workspace_bytes(2000) >= L.sgn_query_workspace_bytes(1000) > 0
    assert L.sgn_aggregate_workspace_bytes(10_000) >= 10_000 * 256 * 2


def test_argument_errors_are_reported_without_gpu():
    """Parameter validation runs before any HIP call: bad arguments give rc < 0 and a message."""
    L = _lib.lib()
    fake = ctypes.c_void_p(16)
    pt, qo = _lib.PointTables(), _lib.QueryOut()
    for f in ("xyz", "embedding", "color", "dir", "conf", "campos", "camrotc2w", "raydir"):
        setattr(pt, f, 16)
    rc = L.sgn_aggregate(ctypes.byref(pt), ctypes.byref(qo), 64, 9, fake, fake, None, None, fake, 1 << 20, 3, None)
    assert rc != 0 and b"K = 1 .. 8" in L.sgn_last_error()
    with pytest.raises(_lib.SgnError, match="K = 1 .. 8"):
        _lib.check(rc, "sgn_aggregate")
    cp = _lib.CompositeParams()
    cp.SR = 0
    rc = L.sgn_composite(ctypes.byref(cp), fake, fake, fake, 4, fake, 0, 400, ctypes.byref(qo), fake, fake, fake,
                         fake, None, None, None)
    assert rc != 0 and b"SR" in L.sgn_last_error()
    rc = L.sgn_ray_march_dense(None, None, None, 4, 8, None, None, None, None, None, None, None)
    assert rc != 0 and b"null" in L.sgn_last_error()
    rc = L.sgn_grid_build(None, 10, None, None, ctypes.byref(ctypes.c_void_p()))
    assert rc != 0
    rc = L.sgn_adam_step(fake, fake, fake, fake, 64, 1e-3, 0.9, 0.999, 1e-8, 0, 1, None)
    assert rc != 0 and b"step >= 1" in L.sgn_last_error()
    rc = L.sgn_adam_step(ctypes.c_void_p(20), fake, fake, fake, 64, 1e-3, 0.9, 0.999, 1e-8, 1, 1, None)
    assert rc != 0 and b"aligned" in L.sgn_last_error()
    xs = (ctypes.c_void_p * 1)(16)
    rc = L.sgn_colsum_f16(1, xs, 100, 128, fake, fake, None)
    assert rc != 0 and b"256" in L.sgn_last_error()
    rc = L.sgn_colsum_f16(9, xs, 100, 256, fake, fake, None)
    assert rc != 0 and b"count" in L.sgn_last_error()
    # fp32 aggregator: K = 1 .. 8 (the row table names pidx index s * K + k)
    rc = L.sgn_aggregate_f32(0, 0, None, fake, ctypes.byref(pt), ctypes.byref(qo), 64, 16, fake, fake, None, None,
                             fake, 1 << 20, 3, None)
    assert rc != 0 and b"K = 1 .. 8" in L.sgn_last_error()
    rc = L.sgn_point_project_f32_subset(ctypes.byref(pt), fake, None, fake, fake, None)
    assert rc != 0 and b"null" in L.sgn_last_error()
    # plain-fp32 range fallback: K, the SG variant, the workspace
    rc = L.sgn_aggregate_exact(0, 0, None, ctypes.byref(pt), ctypes.byref(qo), 64, 9, fake, fake, None, None, fake,
                               1 << 20, None)
    assert rc != 0 and b"K = 1 .. 8" in L.sgn_last_error()
    rc = L.sgn_aggregate_exact(1, 64, None, ctypes.byref(pt), ctypes.byref(qo), 64, 8, fake, fake, None, None, fake,
                               1 << 20, None)
    assert rc != 0 and b"block2_bpnet" in L.sgn_last_error()
    rc = L.sgn_aggregate_exact(0, 0, None, ctypes.byref(pt), ctypes.byref(qo), 64, 8, fake, fake, None, None, fake,
                               512, None)
    assert rc != 0 and b"workspace" in L.sgn_last_error()
    assert L.sgn_mlp_packed_bytes_exact(0, 0) >= 4 * N_PARAMS and L.sgn_mlp_packed_bytes_exact(2, 0) == 0
    assert L.sgn_mlp_packed_bytes_exact(1, 96) > L.sgn_mlp_packed_bytes_exact(1, 0) > L.sgn_mlp_packed_bytes_exact(0, 0)
    # training loss stage: null pointers, SR / K, the workspace size
    lp = _lib.LossParams()
    lp.SR, lp.K = 24, 8
    args = (fake, fake, 64, ctypes.byref(qo), fake, fake, fake, fake, fake, fake, fake, fake)
    rc = L.sgn_loss_train(ctypes.byref(lp), *args, fake, 16, None)
    assert rc != 0 and b"workspace" in L.sgn_last_error()
    assert L.sgn_loss_workspace_bytes(64, 24) >= 64 * 24 * 12
    rc = L.sgn_loss_train(ctypes.byref(lp), *args, None, 1 << 20, None)
    assert rc != 0 and b"null" in L.sgn_last_error()
    lp.K = 0
    rc = L.sgn_loss_train(ctypes.byref(lp), *args, fake, 1 << 20, None)
    assert rc != 0 and b"positive" in L.sgn_last_error()
    # training segment kernels: segment count, per-segment shapes, alignment
    gs = (_lib.GradSegment * 17)()
    rc = L.sgn_grad_accumulate(17, gs, None, fake, None)
    assert rc != 0 and b"n_seg" in L.sgn_last_error()
    gs[0] = _lib.GradSegment(16, None, 16, 256, 128, 1, 0)
    rc = L.sgn_grad_accumulate(1, gs, None, fake, None)
    assert rc != 0 and b"stride >= n" in L.sgn_last_error()
    gs[0] = _lib.GradSegment(None, None, 16, 256, 256, 1, 0)
    rc = L.sgn_grad_accumulate(1, gs, None, fake, None)
    assert rc != 0 and b"null" in L.sgn_last_error()
    rc = L.sgn_zero_segments(1, (ctypes.c_void_p * 1)(20), (ctypes.c_int64 * 1)(64), None)
    assert rc != 0 and b"aligned" in L.sgn_last_error()
    rc = L.sgn_zero_segments(1, (ctypes.c_void_p * 1)(16), (ctypes.c_int64 * 1)(60), None)
    assert rc != 0 and b"multiples of 16" in L.sgn_last_error()
    gt = (_lib.GatherSegment * 1)(_lib.GatherSegment(None, 16, 8, 1, 0))
    rc = L.sgn_gather_segments(1, gt, fake, 8, None)
    assert rc != 0 and b"bad segment" in L.sgn_last_error()
    assert L.sgn_grad_accumulate(0, None, None, None, None) == 0   # nothing to do: no launch
    rc = L.sgn_colour_inputs(fake, fake, fake, 16, 64, ctypes.c_void_p(24), fake, fake, fake, fake, fake, fake, None, None)
    assert rc != 0 and b"aligned" in L.sgn_last_error()
    rc = L.sgn_pack_scaled_f32(fake, 100, 17, None, None, fake, 8, fake, 8, fake, fake, fake, None)
    assert rc != 0 and b"n_layers" in L.sgn_last_error()
    rc = L.sgn_pow2_scale(fake, 0, fake, 0, fake, fake, None)
    assert rc != 0 and b"at least one" in L.sgn_last_error()
    rc = L.sgn_depth_table_jitter(0.1, 8.0, 0, 0.3, 4, fake, fake, None)
    assert rc != 0 and b"D >= 1" in L.sgn_last_error()


# ---- options ------------------------------------------------------------------------
def test_opts_from_reference_namespace():
    ns = argparse.Namespace(SR=24, K=8, vsize=[0.008, 0.008, 0.008], kernel_size=[3, 3, 3], query_size=[0, 0, 0],
                            z_depth_dim=400, bg_color="white", unrelated_flag=7)
    o = HotPathOpts.from_opt(ns)
    assert o.vsize == (0.008, 0.008, 0.008) and o.query_size == (3, 3, 3)  # neural_points.py:425
    assert o.check_supported() is o
    with pytest.raises(NotImplementedError, match="block2_bpnet"):
        HotPathOpts(shading_feature_mlp_layer2_bpnet=3).check_supported()
    with pytest.raises(NotImplementedError, match="agg_dist_pers"):
        HotPathOpts(agg_dist_pers=10).check_supported()


def test_grid_hyperparameters_scannet():
    o = HotPathOpts()
    mn = torch.tensor([0.0, 0.0, 0.0])
    mx = torch.tensor([4.0, 4.0, 3.0])
    h = grid_hyperparameters(o, mn, mx)
    assert h.scaled_vsize.dtype == np.float32 and np.all(h.scaled_vsize == np.float32(0.016))
    assert h.radius_limit == np.float32(0.032) and h.r2 == np.float32(np.float32(0.032) ** 2)
    pad = np.float32(0.016 * 3 / 2)
    np.testing.assert_array_equal(h.shift, (mn.numpy() - pad).astype(np.float32))
    # ceil((max - min) / vsize / vscale) in float64 (worldcoords.py:85-86)
    ext = (mx + float(pad)) - (mn - float(pad))
    want = np.ceil(ext.numpy() / np.array(o.vsize) / np.array(o.vscale)).astype(np.int32)
    np.testing.assert_array_equal(h.scaled_vdim, want)
    assert h.volume == int(np.prod(want.astype(np.int64)))


def test_depth_table_linear_and_jittered():
    t = raygen.depth_table(0.1, 8.0, 400)
    assert t.shape == (400,) and t.dtype == torch.float32
    assert torch.all(t[1:] > t[:-1]) and 0.1 < float(t[0]) < float(t[-1]) < 8.0
    g = torch.Generator().manual_seed(3)
    tj = raygen.depth_table(0.1, 8.0, 400, jitter=0.3, R=5, generator=g)
    assert tj.shape == (5, 400)
    assert torch.all(tj[:, 1:] > tj[:, :-1])


# ---- weights -------------------------------------------------------------------------
def test_init_mlp_matches_reference_architecture():
    st = init_mlp(0, bias_std=0.01)
    assert sum(v.numel() for v in st.values()) == N_PARAMS == 341_764
    check_shapes(st)
    assert len(LAYERS) == 9
    full = {"module.aggregator." + k: v for k, v in st.items()}
    full["neural_points.xyz"] = torch.zeros(3, 3)
    assert set(strip_prefix(full)) == set(st)
    bad = dict(st)
    bad["block1.0.weight"] = torch.zeros(256, 283)
    with pytest.raises(ValueError):
        check_shapes(bad)


# ---- reference bookkeeping around the kernels ------------------------------------------
def test_fill_invalid_expands_compacted_outputs():
    R, SR = 6, 4
    ray_mask = torch.tensor([[0, 1, 1, 0, 1, 0]], dtype=torch.int8)
    n = 3
    out = {"ray_mask": ray_mask,
           "coarse_is_background": torch.full((1, n, 1), 0.25),
           "coarse_raycolor": torch.arange(n * 3, dtype=torch.float32).view(1, n, 3),
           "coarse_point_opacity": torch.full((1, n, SR), 0.5),
           "queried_shading": torch.zeros(1, n, 3)}
    res = fill_invalid(out, {"bg_color": torch.tensor([[0.2, 0.3, 0.4]])})
    keep = ray_mask[0].bool()
    assert res["coarse_raycolor"].shape == (1, R, 3)
    torch.testing.assert_close(res["coarse_raycolor"][0, keep], torch.arange(9, dtype=torch.float32).view(3, 3))
    torch.testing.assert_close(res["coarse_raycolor"][0, ~keep], torch.tensor([[0.2, 0.3, 0.4]] * 3))
    assert torch.all(res["coarse_is_background"][0, ~keep] == 1) and torch.all(res["coarse_is_background"][0, keep] == 0.25)
    torch.testing.assert_close(res["coarse_mask"], 1 - res["coarse_is_background"])
    assert torch.all(res["coarse_point_opacity"][0, ~keep] == 0)
    assert torch.all(res["queried_shading"][0, ~keep] == 1) and torch.all(res["queried_shading"][0, keep] == 0)


def test_dense_from_samples():
    class Q:
        ray_ns = torch.tensor([2, 0, 3], dtype=torch.int32)
        ray_soff = torch.tensor([0, 2, 2], dtype=torch.int32)
    vals = torch.arange(5 * 2, dtype=torch.float32).view(5, 2)
    d = _dense_from_samples(Q, vals, 3, 4, -1.0)
    assert d.shape == (3, 4, 2)
    torch.testing.assert_close(d[0, :2], vals[0:2])
    assert torch.all(d[0, 2:] == -1) and torch.all(d[1] == -1)
    torch.testing.assert_close(d[2, :3], vals[2:5])
    assert torch.all(d[2, 3] == -1)


def test_sg_variant_options_and_weights():
    import pytest as _pt
    from sgnerf_amd.opts import HotPathOpts
    from sgnerf_amd.weights import init_mlp, mlp_variant, layers_for
    assert HotPathOpts().bpnet_variant == (0, 0)
    o = HotPathOpts(shading_feature_mlp_layer2_bpnet=1, predict_semantic=1, semantic_guidance=1).check_supported()
    assert o.bpnet_variant == (1, 96)
    assert HotPathOpts(shading_feature_mlp_layer2_bpnet=1).check_supported().bpnet_variant == (1, 0)
    with _pt.raises(NotImplementedError):
        HotPathOpts(shading_feature_mlp_layer2_bpnet=2).check_supported()
    with _pt.raises(NotImplementedError):  # reference would crash (352-wide layer fed 256)
        HotPathOpts(shading_feature_mlp_layer2_bpnet=1, predict_semantic=1, semantic_guidance=0).check_supported()
    s = init_mlp(0, bpnet_layers=1, bpnet_dim=96)
    assert tuple(s["block2_bpnet.0.weight"].shape) == (256, 352)
    assert mlp_variant(s) == (1, 96) and mlp_variant(init_mlp(0)) == (0, 0)
    # base draws unchanged by the extra layer
    b = init_mlp(0)
    assert all(torch.equal(b[k], s[k]) for k in b)
    assert len(layers_for(1, 0)) == 10


def test_sg_abi_sizes():
    from sgnerf_amd import _lib
    L = _lib.lib()
    base = int(L.sgn_mlp_packed_bytes())
    assert int(L.sgn_mlp_packed_bytes_sg(0, 0)) == base
    assert int(L.sgn_mlp_packed_bytes_sg(1, 96)) == base + 8 * 22 * 1024 + 1024
    assert int(L.sgn_mlp_packed_bytes_sg(1, 0)) == base + 8 * 16 * 1024 + 1024
    assert int(L.sgn_mlp_packed_bytes_sg(2, 96)) == 0
    assert int(L.sgn_mlp_packed_bytes_sg(1, 32)) == 0


def test_training_pack_index_maps():
    """Index maps of the device-side re-packing cover every packed parameter exactly as the
    host packers do (flat LAYERS order)."""
    from sgnerf_amd.weights import N_PARAMS
    L = _lib.lib()
    total = int(L.sgn_mlp_packed_bytes())
    n16, n32 = int(L.sgn_mlp_section(0)) // 2, 2056
    a16, a32 = (ctypes.c_int32 * n16)(), (ctypes.c_int32 * n32)()
    assert L.sgn_mlp_pack_index(0, a16, n16) == 0 and L.sgn_mlp_pack_index(1, a32, n32) == 0
    m16, m32 = np.frombuffer(a16, np.int32), np.frombuffer(a32, np.int32)
    # block1/3 + colour hidden weights live in fragments: each exactly once
    used16 = np.bincount(m16[m16 > 0], minlength=N_PARAMS + 1)
    assert used16.max() == 1
    # biases, alpha weights and colour output layer live in the fp32 section
    used32 = np.bincount(m32[m32 > 0], minlength=N_PARAMS + 1)
    assert used32.max() == 1
    assert int((used16 + used32 > 0).sum()) == N_PARAMS  # every parameter packed somewhere
    # split block1.0 sections: block1.0's weights once each (W0b: PE(dists) columns, W0a: the rest)
    nsp = (total - int(L.sgn_mlp_section(1))) // 2
    asp = (ctypes.c_int32 * nsp)()
    assert L.sgn_mlp_pack_index(2, asp, nsp) == 0
    msp = np.frombuffer(asp, np.int32)
    usp = np.bincount(msp[msp > 0], minlength=N_PARAMS + 1)
    assert usp.max() == 1 and int((usp > 0).sum()) == 256 * 284 and int(usp[1:256 * 284 + 1].sum()) == 256 * 284
    nt = int(L.sgn_train_tblob_bytes()) // 2
    at = (ctypes.c_int32 * nt)()
    assert L.sgn_train_pack_index(at, nt) == 0
    mt = np.frombuffer(at, np.int32)
    ut = np.bincount(mt[mt > 0], minlength=N_PARAMS + 1)
    assert ut.max() == 1 and int((ut > 0).sum()) == 256 * (284 + 256 + 263 + 256)
    cm = (ctypes.c_int32 * 256)()
    assert L.sgn_train_colmap(0, cm, 256) == 0
    assert sorted(np.frombuffer(cm, np.int32).tolist()) == list(range(256))
    c1 = (ctypes.c_int32 * 288)()
    assert L.sgn_train_colmap(1, c1, 288) == 0
    v1 = np.frombuffer(c1, np.int32)
    assert sorted(v1[v1 >= 0].tolist()) == list(range(284))
