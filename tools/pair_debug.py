"""Debug probe (not product): per-sample decoded-feature error of the f32 renderer on a golden case,
split by the sample's role in its paired k_rows16 half (A, B).  Usage: python tools/pair_debug.py [case]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import sgnerf_amd  # noqa: E402,F401
from helpers import load_golden  # noqa: E402
from sgnerf_amd import scene  # noqa: E402
from sgnerf_amd.opts import HotPathOpts  # noqa: E402
from sgnerf_amd.render import HipRenderer, PointTables  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "patch"
DEV = "cuda:0"
pts, mlp, case = load_golden("reference_aggregator.npz", name)
g = {f"{name}/{k}": v for k, v in case.items()}
near, far = (float(x) for x in g[f"{name}/near_far"])
view = scene.View(g[f"{name}/campos"], g[f"{name}/camrotc2w"], g[f"{name}/raydir"], None, None, 0, 0, near, far)
o = HotPathOpts(SR=int(g[f"{name}/SR"]), K=int(g[f"{name}/K"]), precision="f32")
r = HipRenderer(PointTables(pts["xyz"], pts["embedding"], pts["color"], pts["dir"], pts["conf"], DEV), mlp, o, DEV)
out = r.render(torch.from_numpy(view.campos), torch.from_numpy(view.camrotc2w), torch.from_numpy(view.raydir),
               view.near, view.far, want_blend=True)
torch.cuda.synchronize()
q = out.query
R, SR = view.raydir.shape[0], o.SR
S = q.n_samples()
nw = int(q.counters[1].item())
sr = q.samp_ray[:S].cpu().numpy()
slot = np.arange(S) - q.ray_soff[:R].cpu().numpy()[sr]
nnb = q.samp_nnb[:S].cpu().numpy()
feat = out.feat[:S].cpu().numpy()
dec = g[f"{name}/decoded"] if f"{name}/decoded" in g else None
print("keys", sorted(k.split("/", 1)[1] for k in g)[:40])
ws = r.agg_ws
cap = r._cap[1]
L = sgnerf_amd._lib.lib()
wsi = (ws.numel() - 2048) // (1024 + 48)
rows = ws[wsi * 1024: wsi * 1024 + wsi * 32].view(torch.int32).cpu().numpy()
ent = ws[wsi * 1056: wsi * 1056 + wsi * 16].view(torch.int32).cpu().numpy().reshape(-1, 4)
ns = int(ws[-2048:-2044].view(torch.int32).item())
print("work", nw, "slots", ns)
role = np.full(S, -1)
for j in range(ns):
    a, b, sa, sb = ent[j]
    role[sa] = 0
    if (b >> 28) & 15:
        role[sb] = 1
if dec is not None:
    keep = g[f"{name}/ray_mask"].astype(bool)
    dref = np.zeros((R, SR, dec.shape[-1]), np.float32)
    dref[keep] = dec
    ref = dref[sr, slot]
    err = np.abs(feat - ref[:, :feat.shape[1]]).max(1)
    for rl, nm in ((0, "A"), (1, "B")):
        m = (role == rl) & (nnb > 0)
        if m.any():
            print(nm, int(m.sum()), "max err", float(err[m].max()), "by nnb",
                  {int(k): float(err[m & (nnb == k)].max()) for k in np.unique(nnb[m])})
print("alpha range", feat[nnb > 0, 0].min(), feat[nnb > 0, 0].max())
