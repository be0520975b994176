"""Timing probe (not product): config-2 frames (tools/agg_time.py's setup, f32); for each frame the
fraction of the 1.2 M points its samples touch, and HIP-event times of the full block1.0 point
projection (sgn_point_project_f32) against the frame's point list (sgn_frame_points, the renderer's
path) + the subset projection (sgn_point_project_f32_subset).   python tools/proj_touched.py [frames]"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import sgnerf_amd  # noqa: E402,F401
from sgnerf_amd import _lib, scene  # noqa: E402
from sgnerf_amd.opts import HotPathOpts  # noqa: E402
from sgnerf_amd.render import HipRenderer, PointTables  # noqa: E402
from sgnerf_amd.weights import init_mlp  # noqa: E402

nf = int(sys.argv[1]) if len(sys.argv) > 1 else 6
dev = "cuda:0"
pc = scene.synth_room(1_200_000, seed=0)
mlp = init_mlp(0, bias_std=0.01)
mlp["alpha_branch.0.bias"] = mlp["alpha_branch.0.bias"] + 50.0
r = HipRenderer(PointTables.from_cloud(pc, dev), mlp, HotPathOpts(SR=64, precision="f32"), dev)
L = _lib.lib()
N = r.points.n
marks = torch.zeros(int(L.sgn_frame_points_mark_bytes(N)), dtype=torch.uint8, device=dev)
idx = torch.empty(N, dtype=torch.int32, device=dev)
cnt = torch.zeros(2, dtype=torch.int64, device=dev)
out = []
for i in range(2 + nf):
    yaw, pitch = scene.spiral_yaw_pitch(i % 120, 120)
    v = scene.room_view(800, 800, yaw=yaw + 15.0, pitch=pitch - 5.0)
    res = r.render(torch.from_numpy(v.campos).to(dev), torch.from_numpy(v.camrotc2w).to(dev),
                   torch.from_numpy(v.raydir).to(dev), v.near, v.far, check_range=False)
    q = res.query if hasattr(res, "query") else res[4]
    S = int(q.counters[0].item())
    pk = q.pidx[:S * 8]
    frac = torch.unique(pk[pk >= 0]).numel() / N
    st = _lib.stream_handle()
    pt = _lib.PointTables()
    pt.xyz, pt.embedding, pt.color = r.points.xyz.data_ptr(), r.points.embedding.data_ptr(), r.points.color.data_ptr()
    pt.dir, pt.conf, pt.n_points = r.points.dir.data_ptr(), r.points.conf.data_ptr(), N
    c, rot = torch.from_numpy(v.campos).to(dev), torch.from_numpy(v.camrotc2w).to(dev)
    rd = torch.from_numpy(v.raydir).to(dev)
    pt.campos, pt.camrotc2w, pt.raydir = c.data_ptr(), rot.data_ptr(), rd.data_ptr()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    e[0].record()
    _lib.check(L.sgn_point_project_f32(ctypes.byref(pt), _lib.ptr(r.packed), _lib.ptr(r._proj), st), "full")
    e[1].record()
    _lib.check(L.sgn_frame_points(_lib.ptr(q.pidx), _lib.ptr(q.counters), q.pidx.numel() // 8, 8, N,
                                  _lib.ptr(marks), _lib.ptr(idx), _lib.ptr(cnt), st), "frame points")
    e[2].record()
    _lib.check(L.sgn_point_project_f32_subset(ctypes.byref(pt), _lib.ptr(r.packed), _lib.ptr(idx),
                                              _lib.ptr(cnt), _lib.ptr(r._proj), st), "subset")
    e[3].record()
    torch.cuda.synchronize()
    if i >= 2:
        out.append({"touched_frac": frac, "full_ms": e[0].elapsed_time(e[1]), "list_ms": e[1].elapsed_time(e[2]),
                    "subset_ms": e[2].elapsed_time(e[3]), "list_n": int(cnt[0].item())})
print(json.dumps({"lib": os.path.basename(os.environ.get("SGN_HIP_LIB", "intree")), **{k: float(np.median([o[k] for o in out])) for k in out[0]}}))
