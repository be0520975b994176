"""Debug probe (not product): full-frame vs subset render consistency per precision, and where
the mismatching rays' work items sit in the work list (chunk boundaries)."""
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

DEV = "cuda:0"
pc = scene.synth_room(1_200_000, seed=0)
mlp = init_mlp(0, bias_std=0.01)
mlp["alpha_branch.0.bias"] = mlp["alpha_branch.0.bias"] + 50.0
view = scene.room_view(800, 800, yaw=15.0, pitch=-5.0)
idx = np.arange(800 * 800).reshape(800, 800)[::8, ::8].reshape(-1)
for prec in ("f16", "f32"):
    o = HotPathOpts(SR=64, precision=prec)
    r = HipRenderer(PointTables.from_cloud(pc, DEV), mlp, o, DEV)
    cam = (torch.from_numpy(view.campos), torch.from_numpy(view.camrotc2w))
    full = r.render(*cam, torch.from_numpy(view.raydir), view.near, view.far)
    rgb_full = full.rgb.clone()
    q = full.query
    W = int(q.counters[1])
    work = q.work[:W].cpu().numpy()
    samp_ray = q.samp_ray[:int(q.counters[0])].cpu().numpy()
    pos = np.full(800 * 800, -1)
    pos[samp_ray[work]] = np.arange(W)  # a work position of each ray (last one)
    sub = r.render(*cam, torch.from_numpy(view.raydir[idx]), view.near, view.far)
    d = (sub.rgb - rgb_full[torch.from_numpy(idx).to(DEV)]).abs().max(1).values.cpu().numpy()
    bad = np.nonzero(d > 0)[0]
    print(f"[{prec}] work items {W}; mismatching subset rays {len(bad)}/{len(idx)}, max diff {d.max():.3e}")
    if len(bad):
        p = pos[idx[bad]]
        print(f"   work positions of mismatching rays: min {p.min()} max {p.max()}; of matching rays: max "
              f"{pos[idx[d == 0]].max()}")
        # alpha of those rays' samples: full frame vs subset
        print("   first mismatches (ray, full rgb, subset rgb):")
        for b in bad[:3]:
            print("   ", idx[b], rgb_full[idx[b]].tolist(), sub.rgb[b].tolist())
    del r
    torch.cuda.empty_cache()
