"""Timing probe (not product): config-2 frames (synth-room 1.2 M points, 800x800, SR 64) at one
precision; prints one JSON line with per-stage HIP-event medians.  Usage:
    python tools/agg_time.py [f32|f16] [frames]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import sgnerf_amd  # noqa: E402,F401
from sgnerf_amd import scene  # noqa: E402
from sgnerf_amd.opts import HotPathOpts  # noqa: E402
from sgnerf_amd.render import HipRenderer, PointTables  # noqa: E402
from sgnerf_amd.weights import init_mlp  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "f32"
nf = int(sys.argv[2]) if len(sys.argv) > 2 else 8
dev = "cuda:0"
pc = scene.synth_room(1_200_000, seed=0)
mlp = init_mlp(0, bias_std=0.01)
mlp["alpha_branch.0.bias"] = mlp["alpha_branch.0.bias"] + 50.0
r = HipRenderer(PointTables.from_cloud(pc, dev), mlp, HotPathOpts(SR=64, precision=prec), dev)
# SGN_RAY_ORDER=B (B > 0): rays fed in B x B pixel blocks (block-major) instead of row-major
blk = int(os.environ.get("SGN_RAY_ORDER", "0"))
perm = None
if blk > 0:
    yy, xx = np.meshgrid(np.arange(800), np.arange(800), indexing="ij")
    key = ((yy // blk) * (800 // blk) + (xx // blk)) * (blk * blk) + (yy % blk) * blk + (xx % blk)
    perm = torch.from_numpy(np.argsort(key.reshape(-1), kind="stable"))
views = []
for i in range(3 + nf):
    yaw, pitch = scene.spiral_yaw_pitch(i % 120, 120)
    v = scene.room_view(800, 800, yaw=yaw + 15.0, pitch=pitch - 5.0)
    rd = torch.from_numpy(v.raydir)
    if perm is not None:
        rd = rd[perm].contiguous()
    views.append((torch.from_numpy(v.campos).to(dev), torch.from_numpy(v.camrotc2w).to(dev),
                  rd.to(dev), v.near, v.far))
ev = []


def mark(n):
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    ev[-1][n] = e


for i, (c, rot, rd, ne, fa) in enumerate(views):
    if i >= 3:
        ev.append({})
    r.render(c, rot, rd, ne, fa, marks=mark if i >= 3 else None, check_range=False)
torch.cuda.synchronize()
names = ["query", "proj", "agg_rows", "agg_color", "composite", "end"]
res = {n: float(np.median([e[n].elapsed_time(e[names[j + 1]]) for e in ev])) for j, n in enumerate(names[:-1])}
res["frame"] = float(np.median([e["query"].elapsed_time(e["end"]) for e in ev]))
res["prec"] = prec
res["lib"] = os.environ.get("SGN_VARIANT", "base")
res["ray_block"] = blk
print(json.dumps(res), flush=True)
