"""Spiral video renderer (BASELINE config 3), frame-sharded over ranks.

Replaces the loop of run/render_vid.py:26-82 (per pose: chunks of rays through
model.set_input/test, frames collected, written as a video) for the HIP path: every rank
renders whole frames (frame i on rank i % N, `dist.render_frames`), the finished frames are
all-gathered over RCCL, and rank 0 writes them.  The reference's ScanNet dataset has no
`render_poses`, so poses come from the spiral of config 3 (yaw 0->360 deg,
pitch 10 sin(2 pi i / n) deg, camera at the room centre) or from a caller-supplied list.

    python -m torch.distributed.run --nproc-per-node N -m sgnerf_amd.render_vid --frames 120 --out vid/
"""
import argparse
import os

import numpy as np
import torch

from . import dist as sd
from . import scene
from .opts import HotPathOpts
from .render import HipRenderer, PointTables
from .weights import init_mlp


def spiral_views(n_frames, h, w, campos=(2.0, 2.0, 1.5)):
    out = []
    for i in range(n_frames):
        yaw, pitch = scene.spiral_yaw_pitch(i, n_frames)
        out.append(scene.room_view(h, w, yaw=yaw, pitch=pitch, campos=campos))
    return out


def default_scene(n_points=1_200_000):
    """Config 3's synthetic stand-in: synth-room cloud and a random aggregator whose alpha
    bias (+50) makes the volume opaque (median background transmission ~0.4 at SR 24)."""
    pc = scene.synth_room(n_points, seed=0)
    mlp = init_mlp(0, bias_std=0.01)
    mlp["alpha_branch.0.bias"] = mlp["alpha_branch.0.bias"] + 50.0
    return pc, mlp


def render_views(renderer: HipRenderer, views, device):
    """All views -> [n, h*w, 3] on every rank (frame i rendered by rank i % N)."""
    h, w = views[0].h, views[0].w
    cache = {}

    def one(i):
        v = views[i]
        if i not in cache:
            cache.clear()
            cache[i] = (torch.from_numpy(v.campos).to(device), torch.from_numpy(v.camrotc2w).to(device),
                        torch.from_numpy(v.raydir).to(device))
        cp, rot, rd = cache[i]
        return renderer.render(cp, rot, rd, v.near, v.far, want_opacity=False).rgb

    return sd.render_frames(one, len(views), h, w, device)


def write_frames(frames, h, w, out_dir, prefix="frame"):
    """frames [n, h*w, 3] in [0, 1] -> PNG files (8-bit) + one .npy stack."""
    from PIL import Image
    os.makedirs(out_dir, exist_ok=True)
    arr = frames.detach().cpu().numpy().reshape(-1, h, w, 3)
    np.save(os.path.join(out_dir, f"{prefix}s.npy"), arr.astype(np.float16))
    for i, f in enumerate(arr):
        Image.fromarray((np.clip(f, 0, 1) * 255 + 0.5).astype(np.uint8)).save(
            os.path.join(out_dir, f"{prefix}_{i:04d}.png"))
    return arr.shape[0]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=120)
    ap.add_argument("--h", type=int, default=800)
    ap.add_argument("--w", type=int, default=800)
    ap.add_argument("--sr", type=int, default=24)
    ap.add_argument("--points", type=int, default=1_200_000)
    ap.add_argument("--checkpoint", default=None, help="reference *_net_ray_marching.pth (weights_only load)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--precision", default="f32", choices=["f32", "f16"])
    args = ap.parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.distributed.init_process_group("nccl", device_id=dev)
    o = HotPathOpts(SR=args.sr, precision=args.precision)
    if args.checkpoint:
        from .ray_marching import NeuralPoints
        from .weights import strip_prefix
        sd_ = torch.load(args.checkpoint, map_location="cpu", weights_only=True)
        npnts = NeuralPoints.from_state_dict(sd_, dev)
        r = HipRenderer(npnts.tables(), strip_prefix(sd_), o, dev)
    else:
        pc, mlp = default_scene(args.points)
        r = HipRenderer(PointTables.from_cloud(pc, dev), mlp, o, dev)
    views = spiral_views(args.frames, args.h, args.w)
    torch.cuda.synchronize()
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    t0.record()
    frames = render_views(r, views, dev)
    t1.record()
    torch.cuda.synchronize()
    ms = sd.max_over_ranks(t0.elapsed_time(t1), dev)
    _, rank = sd.world()
    if rank == 0:
        print(f"rendered {args.frames} frames {args.h}x{args.w} on {world} GPU(s) in {ms:.1f} ms "
              f"({args.frames * args.h * args.w / ms * 1e3:.3e} rays/s)")
        if args.out:
            write_frames(frames, args.h, args.w, args.out)
    if world > 1:
        torch.distributed.destroy_process_group()
    return frames, ms


if __name__ == "__main__":
    main()
