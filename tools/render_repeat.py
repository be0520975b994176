"""Debug probe (not product): render one config-2 frame (f32 mode) repeatedly and count pixels that
differ bitwise from the first render.  Usage (GPU box): python tools/render_repeat.py [n] [precision]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import sgnerf_amd  # noqa: E402,F401
from sgnerf_amd import scene  # noqa: E402
from sgnerf_amd.opts import HotPathOpts  # noqa: E402
from sgnerf_amd.render import HipRenderer, PointTables  # noqa: E402
from sgnerf_amd.weights import init_mlp  # noqa: E402

DEV = torch.device("cuda", 0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
prec = sys.argv[2] if len(sys.argv) > 2 else "f32"
o = HotPathOpts(SR=64, precision=prec)
pc = scene.synth_room(1_200_000, seed=0)
mlp = init_mlp(0, bias_std=0.01)
mlp["alpha_branch.0.bias"] = mlp["alpha_branch.0.bias"] + 50.0
r = HipRenderer(PointTables.from_cloud(pc, DEV), mlp, o, DEV)
yaw, pitch = scene.spiral_yaw_pitch(5, 120)
v = scene.room_view(800, 800, yaw=yaw + 15.0, pitch=pitch - 5.0)
rd = torch.from_numpy(v.raydir).to(DEV)
cp, rot = torch.from_numpy(v.campos).to(DEV), torch.from_numpy(v.camrotc2w).to(DEV)
first = None
bad_runs = 0
for i in range(n):
    out = r.render(cp, rot, rd, v.near, v.far)
    torch.cuda.synchronize()
    rgb = out.rgb.clone()
    if first is None:
        first = rgb
        continue
    d = (rgb - first).abs().max(1).values
    nb = int((d > 0).sum())
    bad_runs += nb > 0
    print(f"render {i}: {nb} pixels differ, max {float(d.max()):.3e}", flush=True)
print(f"{prec}: {bad_runs} of {n - 1} renders differ from the first")
