"""Debug aid (GPU box): per-sample alpha and blended-feature errors of the MFMA aggregator
against a torch fp32 restatement, on the golden 'patch' case.  Not part of the product."""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import sgnerf_amd  # noqa: E402,F401
import agg_ref  # noqa: E402
from sgnerf_amd import scene  # noqa: E402
from sgnerf_amd.opts import HotPathOpts  # noqa: E402
from sgnerf_amd.render import HipRenderer, PointTables  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "patch"
g = np.load(os.path.join(ROOT, "tests", "golden", "reference_aggregator.npz"))
pcn = str(g[f"{name}/points"])
pts = {k: g[f"{pcn}/{k}"] for k in ("xyz", "embedding", "color", "dir", "conf")}
mlp = {k[4:]: torch.from_numpy(g[k]) for k in g.files if k.startswith("mlp/")}
near, far = (float(x) for x in g[f"{name}/near_far"])
view = scene.View(g[f"{name}/campos"], g[f"{name}/camrotc2w"], g[f"{name}/raydir"], None, None, 0, 0, near, far)
o = HotPathOpts(SR=int(g[f"{name}/SR"]))
dev = "cuda:0"
r = HipRenderer(PointTables(pts["xyz"], pts["embedding"], pts["color"], pts["dir"], pts["conf"], dev), mlp, o, dev)
out = r.render(torch.from_numpy(view.campos), torch.from_numpy(view.camrotc2w), torch.from_numpy(view.raydir),
               near, far, want_blend=True)
torch.cuda.synchronize()
q = out.query
S = q.n_samples()
W = int(q.counters[1].item())
work = q.work[:W].long().cpu()
feat = out.feat[:S].cpu()
fs_gpu = r.agg_ws[: W * 512].view(torch.float16).view(W, 256).float().cpu()

# torch restatement with the blended features exposed
tp = {k: torch.from_numpy(v) for k, v in pts.items()}
samp_ray = q.samp_ray[:S].cpu()
locw = q.samp_locw[: S * 3].view(S, 3).cpu()
pidx = q.pidx[: S * 8].view(S, 8).cpu()
ref_feat, ref_w = agg_ref.aggregate(tp, mlp, torch.from_numpy(view.campos), torch.from_numpy(view.camrotc2w),
                                    torch.from_numpy(view.raydir), samp_ray, locw, pidx)
ea = (feat[work, 0] - ref_feat[work, 0]).abs()
ec = (feat[work, 1:] - ref_feat[work, 1:]).abs()
print(f"W={W} S={S}: alpha err max {ea.max():.3e} mean {ea.mean():.3e} (alpha mean {ref_feat[work, 0].abs().mean():.3e});"
      f" rgb err max {ec.max():.3e}")
bad = torch.nonzero(ea > 1e-2 * (1 + ref_feat[work, 0].abs())).view(-1)
print("bad alpha items (first 20):", bad[:20].tolist(), "item%4:", (bad % 4).bincount(minlength=4).tolist(),
      "item%32:", (bad % 32)[:20].tolist())
print("gpu alpha", feat[work[:8], 0].tolist())
print("ref alpha", ref_feat[work[:8], 0].tolist())

# blended features: recompute f_s in fp32
mask = pidx >= 0
w = ref_w  # weight * conf [S,8]
flat = torch.clamp(pidx, min=0).reshape(-1).long()
emb = tp["embedding"][flat].view(S, 8, -1)
# reuse agg_ref internals by monkeypatching: compute fs via a small copy of its chain
sys.setrecursionlimit(10000)
src = open(agg_ref.__file__).read()
ns = {}
code = src.replace("    c = torch.cat([fs, vpe[ray_valid]], dim=-1)", "    return fs, ray_valid")
exec(compile(code, "agg_ref_fs", "exec"), ns)
fs_ref, rv = ns["aggregate"](tp, mlp, torch.from_numpy(view.campos), torch.from_numpy(view.camrotc2w),
                             torch.from_numpy(view.raydir), samp_ray, locw, pidx)
full = torch.zeros(S, 256)
full[rv] = fs_ref
ef = (fs_gpu - full[work]).abs()
print(f"fs err max {ef.max():.3e} mean {ef.mean():.3e} (|fs| mean {full[work].abs().mean():.3e})")
per_unit = ef.max(0)[0]
per_item = ef.max(1)[0]
print("fs err by unit%32 (max):", [round(float(x), 4) for x in per_unit.view(8, 32).max(0)[0]])
print("fs err by tile (max):", [round(float(x), 4) for x in per_unit.view(8, 32).max(1)[0]])
print("fs err by item%4:", [round(float(per_item[i::4].max()), 4) for i in range(4)])

# effective blend weights: solve fs_gpu[item] = sum_k c_k h_ref[item, k] per item
code2 = src.replace("    # alpha + K-blend :743-770", "    return f, m, weight")
ns2 = {}
exec(compile(code2, "agg_ref_h", "exec"), ns2)
f_rows, m_rows, wref = ns2["aggregate"](tp, mlp, torch.from_numpy(view.campos), torch.from_numpy(view.camrotc2w),
                                        torch.from_numpy(view.raydir), samp_ray, locw, pidx)
hfull = torch.zeros(S * 8, 256)
hfull[m_rows] = f_rows
hfull = hfull.view(S, 8, 256)
for it in range(3):
    s_ = int(work[it])
    Hm = hfull[s_].T  # [256, 8]
    c, res, *_ = torch.linalg.lstsq(Hm.double(), fs_gpu[it].double()[:, None])
    print(f"item {it} sample {s_}: eff w {[round(float(x), 4) for x in c[:, 0]]}")
    print(f"            ref w {[round(float(x), 4) for x in wref[s_]]}  resid {float((Hm.double() @ c - fs_gpu[it].double()[:, None]).abs().max()):.3e}")
