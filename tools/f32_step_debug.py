"""Debug probe (not product): the fp32 training step's forward (per-sample alpha / rgb of F32Step,
the rendered colour) against torch fp32 (train.aggregate + composite_losses) on the very query of
the step, config-5 batch.  Prints the worst samples and rays.  Usage (GPU box):
    python tools/f32_step_debug.py [seed]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import sgnerf_amd  # noqa: E402,F401
from sgnerf_amd import scene  # noqa: E402
from sgnerf_amd.opts import HotPathOpts  # noqa: E402
from sgnerf_amd.train import PointParams, ViewMLP, aggregate, composite_losses  # noqa: E402
from sgnerf_amd.train_hip import HipTrainer  # noqa: E402
from sgnerf_amd.weights import init_mlp  # noqa: E402

DEV = torch.device("cuda", 0)
seed = int(sys.argv[1]) if len(sys.argv) > 1 else 0
torch.manual_seed(seed)
O = HotPathOpts(SR=24, is_train=int(os.environ.get("TRAIN", "1")))
pc = scene.synth_room(1_200_000, seed=0)
yaw, pitch = scene.spiral_yaw_pitch(37, 120)
view = scene.room_view(800, 800, yaw=yaw + 15.0, pitch=pitch - 5.0)
g = torch.Generator().manual_seed(2)
idx = torch.randint(0, 800 * 800, (4096,), generator=g).numpy()
raydir = torch.from_numpy(np.ascontiguousarray(view.raydir[idx])).to(DEV)
gt = torch.rand(4096, 3, generator=g).to(DEV)
mlp = init_mlp(0, bias_std=0.01)
mlp["alpha_branch.0.bias"] = mlp["alpha_branch.0.bias"] + 50.0
campos, rot = torch.from_numpy(view.campos).to(DEV), torch.from_numpy(view.camrotc2w).to(DEV)
points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, DEV)
tr = HipTrainer(points, mlp, O, DEV, precision="f32")
parts, full, mask = tr.backward(campos, rot, raydir, 0.1, 8.0, gt)
torch.cuda.synchronize()
qd = {k: v.long() if v.dtype == torch.int32 else v for k, v in tr.last_query.items()}
S = qd["samp_ray"].shape[0]
st = tr._f32step
feat_h = st.feat[:S].clone()
with torch.no_grad():
    ref_pts = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, DEV)
    vm = ViewMLP(mlp).to(DEV)
    feat_t, _, m = aggregate(ref_pts, vm, campos.reshape(1, 3), rot, raydir, qd["samp_ray"], qd["samp_locw"], qd["pidx"])
    tot, _, full_t, mask_t = composite_losses(ref_pts, qd, feat_t, m.sum(-1) > 0, campos, rot, raydir, gt, O)
nnb = (qd["pidx"] >= 0).sum(1)
da = (feat_h[:, 0] - feat_t[:, 0]).abs() / feat_t[:, 0].abs().clamp(min=1e-6)
dc = (feat_h[:, 1:] - feat_t[:, 1:]).abs().max(1).values
print("samples", S, "items", int((nnb > 0).sum()), "counts", st.counts.tolist())
print("alpha rel err: max %.3e  median %.3e" % (float(da.max()), float(da.median())))
print("rgb abs err:   max %.3e  median %.3e" % (float(dc.max()), float(dc.median())))
for name, d in (("alpha", da), ("rgb", dc)):
    top = torch.topk(d, 8).indices
    for s in top.tolist():
        print(f"  worst {name}: s={s} nnb={int(nnb[s])} ray={int(qd['samp_ray'][s])} hip={feat_h[s].tolist()} "
              f"torch={feat_t[s].tolist()}")
dr = (full - full_t).abs().max(1).values
print("full rel L2 %.3e, ray max abs err %.3e" % (float((full - full_t).norm() / full_t.norm()), float(dr.max())))
for r in torch.topk(dr, 8).indices.tolist():
    ss = torch.nonzero(qd["samp_ray"] == r).reshape(-1)
    print(f"  ray {r}: hip={full[r].tolist()} torch={full_t[r].tolist()} samples={ss.tolist()[:6]} "
          f"alpha_h={[round(float(feat_h[s, 0]), 5) for s in ss[:6]]} alpha_t={[round(float(feat_t[s, 0]), 5) for s in ss[:6]]}")
