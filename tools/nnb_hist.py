"""Probe (not product): histogram of valid neighbours per work item (sample with >= 1 neighbour)
on config-2 frames, i.e. how many of k_rows16's 8-row sample slots are padding.
Usage: python tools/nnb_hist.py [frames]"""
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

nf = int(sys.argv[1]) if len(sys.argv) > 1 else 3
dev = "cuda:0"
pc = scene.synth_room(1_200_000, seed=0)
mlp = init_mlp(0, bias_std=0.01)
r = HipRenderer(PointTables.from_cloud(pc, dev), mlp, HotPathOpts(SR=64, precision="f32"), dev)
hist = np.zeros(9, np.int64)
for i in range(nf):
    yaw, pitch = scene.spiral_yaw_pitch(i * 40 % 120, 120)
    v = scene.room_view(800, 800, yaw=yaw + 15.0, pitch=pitch - 5.0)
    o = r.render(torch.from_numpy(v.campos).to(dev), torch.from_numpy(v.camrotc2w).to(dev),
                 torch.from_numpy(v.raydir).to(dev), v.near, v.far)
    q = o.query
    nw = int(q.counters[1].item())
    nnb = q.samp_nnb[q.work[:nw].long()].cpu().numpy()
    hist += np.bincount(nnb, minlength=9)[:9]
tot = hist.sum()
rows = (hist * np.arange(9)).sum()
print(json.dumps({"hist": hist.tolist(), "items": int(tot), "rows": int(rows), "pad_frac": float(1 - rows / (8 * tot)),
                  "share": (hist / tot).round(4).tolist()}))
