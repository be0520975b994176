"""Debug probe (not product): decoded-feature / RGB errors of the f16 and f32 aggregator
modes against the reference goldens and against the torch fp32 oracle on a room.
Usage (GPU box): python tools/x3_check.py"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import agg_ref  # noqa: E402
import oracle_query as oq  # noqa: E402
from helpers import hyper_for, make_view, small_room  # noqa: E402
import sgnerf_amd  # noqa: E402,F401
from sgnerf_amd import scene  # noqa: E402
from sgnerf_amd.opts import HotPathOpts  # noqa: E402
from sgnerf_amd.render import HipRenderer, PointTables  # noqa: E402
from sgnerf_amd.weights import init_mlp  # noqa: E402

DEV = "cuda:0"
GOLD = os.path.join(ROOT, "tests", "golden", "reference_aggregator.npz")


def dense_feat(out, R, SR):
    q = out.query
    S = q.n_samples()
    sr = q.samp_ray[:S].cpu().numpy()
    slot = np.arange(S) - q.ray_soff[:R].cpu().numpy()[sr]
    dense = np.zeros((R, SR, 4), np.float32)
    valid = q.samp_nnb[:S].cpu().numpy() > 0
    dense[sr[valid], slot[valid]] = out.feat[:S].cpu().numpy()[valid]
    return dense


def golden(prec):
    g = np.load(GOLD, allow_pickle=False)
    for name in ("patch", "patch64", "dense"):
        pcn = str(g[f"{name}/points"])
        pts = PointTables(*(g[f"{pcn}/{k}"] for k in ("xyz", "embedding", "color", "dir", "conf")), DEV)
        mlp = {k[4:]: torch.from_numpy(g[k]) for k in g.files if k.startswith("mlp/")}
        near, far = (float(x) for x in g[f"{name}/near_far"])
        o = HotPathOpts(SR=int(g[f"{name}/SR"]), K=int(g[f"{name}/K"]), precision=prec)
        r = HipRenderer(pts, mlp, o, DEV)
        out = r.render(torch.from_numpy(g[f"{name}/campos"]), torch.from_numpy(g[f"{name}/camrotc2w"]),
                       torch.from_numpy(g[f"{name}/raydir"]), near, far)
        torch.cuda.synchronize()
        R = g[f"{name}/raydir"].shape[0]
        keep = g[f"{name}/ray_mask"].astype(bool)
        d = dense_feat(out, R, o.SR)[keep]
        ref = g[f"{name}/decoded"]
        err = np.abs(d - ref)
        rel = err / (np.abs(ref) + 1e-3)
        rgb = np.abs(out.rgb.cpu().numpy() - g[f"{name}/full_color"]).max()
        print(f"[{prec}] golden {name}: decoded max abs {err.max():.3e} (alpha {err[..., 0].max():.3e}, rgb "
              f"{err[..., 1:].max():.3e}), max rel {rel.max():.3e}; ray rgb {rgb:.3e}", flush=True)


def room(prec, alpha_bias=150.0):
    pc = small_room(300_000, seed=2)
    o = HotPathOpts(SR=32, precision=prec)
    mlp = init_mlp(2, bias_std=0.01)
    mlp["alpha_branch.0.bias"] = mlp["alpha_branch.0.bias"] + alpha_bias
    view = make_view(48, 64, yaw=120.0, pitch=-8.0)
    pts = dict(xyz=pc.xyz, embedding=pc.embedding, color=pc.color, dir=pc.dir, conf=pc.conf)
    r = HipRenderer(PointTables(pts["xyz"], pts["embedding"], pts["color"], pts["dir"], pts["conf"], DEV), mlp, o, DEV)
    out = r.render(torch.from_numpy(view.campos), torch.from_numpy(view.camrotc2w), torch.from_numpy(view.raydir),
                   view.near, view.far)
    torch.cuda.synchronize()
    hy = hyper_for(pc, o)
    q = oq.OracleGrid(pc.xyz, hy, o).query(view.campos, view.raydir, r.querier.depth_table(0.1, 8.0, 0)[0].cpu().numpy())
    tp = {k: torch.from_numpy(v) for k, v in pts.items()}
    with torch.no_grad():
        full, mask, fd, opacity, bg_t = agg_ref.render(tp, mlp, torch.from_numpy(view.campos),
                                                       torch.from_numpy(view.camrotc2w), torch.from_numpy(view.raydir), q, o.SR)
    R = view.raydir.shape[0]
    d = dense_feat(out, R, o.SR)
    m = mask.numpy()
    fdn = fd.numpy() if fd is not None else None
    err = np.abs(out.rgb.cpu().numpy() - full.numpy()).max()
    msg = f"[{prec}] room: rgb max {err:.3e}"
    if fdn is not None and fdn.shape == d.shape:
        e = np.abs(d - fdn)
        msg += f", decoded max abs {e.max():.3e} (alpha {e[..., 0].max():.3e} of |alpha| max {np.abs(fdn[..., 0]).max():.1f})"
    print(msg, flush=True)


def speed(prec):
    pc = scene.synth_room(1_200_000, seed=0)
    o = HotPathOpts(SR=64, precision=prec)
    mlp = init_mlp(0, bias_std=0.01)
    mlp["alpha_branch.0.bias"] = mlp["alpha_branch.0.bias"] + 50.0
    view = scene.room_view(800, 800, yaw=15.0, pitch=-5.0)
    r = HipRenderer(PointTables.from_cloud(pc, DEV), mlp, o, DEV)
    cam = (torch.from_numpy(view.campos), torch.from_numpy(view.camrotc2w), torch.from_numpy(view.raydir))
    ev = {}

    def mark(n):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        ev.setdefault(n, []).append(e)
    for i in range(6):
        r.render(*cam, view.near, view.far, marks=mark if i >= 3 else None)
    torch.cuda.synchronize()
    names = ["query", "proj", "agg_rows", "agg_color", "composite", "end"]
    st = {names[i]: np.mean([ev[names[i]][k].elapsed_time(ev[names[i + 1]][k]) for k in range(3)]) for i in range(5)}
    print(f"[{prec}] config-2 frame stages ms: " + ", ".join(f"{k} {v:.3f}" for k, v in st.items()) +
          f"; total {sum(st.values()):.3f}", flush=True)


if __name__ == "__main__":
    for prec in ("f16", "f32"):
        golden(prec)
    for prec in ("f16", "f32"):
        room(prec)
    for prec in ("f16", "f32"):
        speed(prec)
