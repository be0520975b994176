"""Benchmark of the per-ray rendering hot path (BASELINE.json metric: rays/sec + ms/frame,
800x800 rays x 64 shading samples, ScanNet-like scene, 1/2/4/8 GPUs).

One step = one 800x800 frame through the whole hot path on each rank:
  query (march + shading-sample selection + layered kNN over the cached grid)
  -> MFMA aggregator (per-neighbour MLP + K-blend) -> colour MLP -> alpha composite
  [-> RCCL all-gather of the rendered frames when N > 1]
Inputs (point cloud, weights, ray directions of every pose) are resident in HBM before
the timed region; the voxel grid is built once per point cloud (timed separately).
Scene: synthetic "synth-room" (no dataset/checkpoint exists offline),
random-init aggregator weights of the reference architecture.
Multi-GPU: frame sharding (weak scaling), rank r renders spiral pose (step*N + r) % 120.
Precision: the headline runs the aggregator at the reference's fp32 arithmetic (mlp_x3.hip,
every fp32 product as three fp16 MFMA products); the fp16-operand mode is an extra key.

    python bench.py [--gpus N --steps K --warmup W]      (N > 1: launches N ranks itself)
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import gc
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import sgnerf_amd  # noqa: E402
from sgnerf_amd import scene  # noqa: E402
from sgnerf_amd.opts import HotPathOpts  # noqa: E402
from sgnerf_amd.render import HipRenderer, PointTables  # noqa: E402
from sgnerf_amd.weights import init_mlp  # noqa: E402

METRIC = "rays/sec + ms/frame, 800×800×64 samples, ScanNet scene, 1/2/4/8 GPU"
FLOP_PER_NB = 2 * (284 * 256 + 256 * 256 + 263 * 256 + 256 * 256 + 256)  # 542,720
# split block1.0: per row only the 60 PE(dists) inputs of block1.0 remain; the
# 224 per-point inputs are multiplied once per point and frame by k_point_proj
FLOP_PER_ROW_SPLIT = FLOP_PER_NB - 2 * 224 * 256                          # 428,032
FLOP_PER_POINT_PROJ = 2 * 224 * 256                                         # 114,688
FLOP_PER_SMP = 2 * (280 * 128 + 128 * 128 * 2 + 128 * 3)                 # 137,984
PEAK_F16_TFLOPS = 256 * 4 * 1024 * 2.4e9 / 1e12  # dense fp16 MFMA, MI355X_MICROARCH.md (~2.5 PF)
# fp32 mode: each fp32 product is three fp16 MFMA products, so its MFMA ceiling is a third of the
# fp16 peak (the native f32-input MFMA peak, 157.3 TF, is reported beside it)
PEAK_X3_TFLOPS = PEAK_F16_TFLOPS / 3
PEAK_F32_NATIVE_TFLOPS = 157.3
PEAK_HBM_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--h", type=int, default=800)
    ap.add_argument("--w", type=int, default=800)
    ap.add_argument("--sr", type=int, default=None, help="samples per ray (default 64 room, 128 lego)")
    ap.add_argument("--points", type=int, default=None, help="neural points (default 1.2M room, 300k lego)")
    ap.add_argument("--scene", choices=["room", "lego", "dense", "spiral"], default="room",
                    help="room: BASELINE config 2 (headline); lego: config 4 (NeRF-synthetic camera, SR 128)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_latest.json"))
    ap.add_argument("--train", action="store_true",
                    help="BASELINE config 5: training steps on 4096 random rays per rank (backward + DP all-reduce)")
    ap.add_argument("--train-rays", type=int, default=4096)
    ap.add_argument("--train-precision", choices=["f32", "f16"], default="f32",
                    help="config 5 arithmetic (f32: the reference's; f16: fp16-operand row MLP forward/backward)")
    ap.add_argument("--train-torch", action="store_true",
                    help="config 5 on the torch-autograd restatement (train.Trainer) instead of the HIP backward")
    ap.add_argument("--sg", action="store_true",
                    help="SG-NeRF variant: semantic-guided kNN + block2_bpnet (352->256) on the config-2 frame")
    ap.add_argument("--precision", choices=["f32", "f16"], default="f32",
                    help="aggregator arithmetic of the headline (f32: the reference's; f16: fp16 MFMA operands)")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the extra keys (f16-mode frame rate, config-5 training rate)")
    return ap.parse_args()


def self_launch(args):
    """`--gpus N` (N > 1) without a launcher: run this script as N ranks under
    torch.distributed.run (sgnerf_amd.dist.launch_ranks) and return the exit code."""
    from sgnerf_amd import dist as sd
    return sd.launch_ranks(__file__, args.gpus, sys.argv[1:]).returncode


def train_main(args, world, rank, dev, dist, steps=None, warmup=None, precision=None):
    """Config 5: one training step = 4096 random rays of a random spiral pose per rank, HIP query,
    device autograd through aggregator + composite, bucketed RCCL all-reduce, two Adam groups.
    Returns the result dict (rank 0 prints it when run as the headline)."""
    steps = args.steps if steps is None else steps
    warmup = args.warmup if warmup is None else warmup
    precision = args.train_precision if precision is None else precision
    from sgnerf_amd.train import PointParams, Trainer
    from sgnerf_amd.train_hip import HipTrainer
    sg = dict(shading_feature_mlp_layer2_bpnet=1, predict_semantic=1, semantic_guidance=1) if args.sg else {}
    if args.sg and args.train_torch:
        raise SystemExit("--train-torch covers the base viewmlp only")
    o = HotPathOpts(SR=24, is_train=1, **sg)
    pc = scene.synth_room(args.points, seed=0)
    if args.sg:
        pc = scene.with_semantics(pc, seed=1, n_classes=20, cell=0.5)
    mlp = init_mlp(0, bias_std=0.01, bpnet_layers=1 if args.sg else 0, bpnet_dim=96 if args.sg else 0)
    mlp["alpha_branch.0.bias"] = mlp["alpha_branch.0.bias"] + 50.0
    points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, dev)
    tr = Trainer(points, mlp, o, dev) if args.train_torch else HipTrainer(points, mlp, o, dev, bpnet=pc.bpnet,
                                                                                 precision=precision)
    g = torch.Generator().manual_seed(1 + rank)
    n_steps = warmup + steps
    batches = []
    labels = [None] * n_steps
    for i in range(n_steps):
        v = pose_view(int(torch.randint(0, 120, (1,), generator=g)), args.h, args.w)
        idx = torch.randint(0, args.h * args.w, (args.train_rays,), generator=g)
        gt = torch.rand(args.train_rays, 3, generator=g)
        batches.append(tuple(x.to(dev) for x in (torch.from_numpy(v.campos), torch.from_numpy(v.camrotc2w),
                                                   torch.from_numpy(v.raydir)[idx], gt)))
        if args.sg:   # ray labels: the first neighbour's label of each ray (as render_run), untimed
            labels[i] = _ray_labels(dev, o, pc, batches[i][0], batches[i][2], 0.1, 8.0)
    tr.querier = None
    for i in range(warmup):
        c, r_, d, gt = batches[i]
        tr.step(c, r_, d, 0.1, 8.0, gt, **_lab(labels[i]))
    torch.cuda.synchronize()
    # the garbage of the runs before this one (the render extras' renderers and tables) is collected here,
    # untimed, not by an automatic full collection somewhere inside the timed steps
    gc.collect()
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    losses = []
    for i in range(warmup, n_steps):
        c, r_, d, gt = batches[i]
        parts, _, _ = tr.step(c, r_, d, 0.1, 8.0, gt, **_lab(labels[i]))
        losses.append(parts["total"])
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if dist:
        torch.distributed.all_reduce(el, op=torch.distributed.ReduceOp.MAX)
    elapsed = float(el.item())
    rays = args.train_rays * steps * world
    res = {"metric": "training rays/sec, 4096-ray batches with backward, DP (BASELINE config 5)",
           "value": rays / elapsed, "unit": "rays/s", "n_gpus": world, "steps": steps, "warmup": warmup,
           "ms_per_step": elapsed / steps * 1e3, "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "f32" if (args.train_torch or precision == "f32") else "f16",
           "data": "synthetic",
           "config": {"workload": f"synth-room, {args.train_rays} random rays per rank per step, SR=24, K=8, "
                                  f"{args.points} neural points, HIP query + "
                                  + ("torch autograd" if args.train_torch else
                                     "fp32 forward + backward on hand-written HIP kernels (k_rows16 save mode, split-fp16 "
                                     "MFMA GEMMs k_x3rows / k_x3tn, HIP loss stage), HIP Adam"
                                     if precision == "f32"
                                     else "HIP MFMA row-MLP forward/backward (fp16 operands) + colour MLP and losses "
                                          "on the split-fp16 GEMMs and HIP loss stage in one captured graph, HIP Adam")
                                  + (" (SG-NeRF variant: semantic-guided kNN, block2_bpnet 352->256)" if args.sg else "")
                                  + (" + RCCL all-reduce of the gradients" if world > 1 else
                                     ", one GPU (no gradient exchange)"),
                      "parallelism": f"dp{world}"},
           "final_loss": float(torch.stack(losses).mean().item()),
           "graph_captures": int(getattr(tr, "graph_captures", 0))}   # loss-stage captures, warm-up included
    return res


def _lab(labels):
    return {} if labels is None else {"labels": labels}


def _ray_labels(dev, o, pc, campos, raydir, near, far):
    """SG stand-in for BPNet's per-pixel labels: the label of the first neighbour of each ray's
    first occupied sample under the plain query; (point_labels, ray_labels, seconds)."""
    from sgnerf_amd.querier import LightningFastQuerier
    import dataclasses
    qr = LightningFastQuerier(dev, dataclasses.replace(o, semantic_guidance=0))
    xyz = torch.from_numpy(pc.xyz).to(dev)
    q = qr.query_samples(xyz, campos, raydir, near, far)
    S, R, K = q.n_samples(), raydir.shape[0], o.K
    pl = torch.from_numpy(pc.labels).to(dev)
    sr = q.samp_ray[:S].long()
    ok = q.samp_nnb[:S] > 0
    first = torch.full((R,), S, dtype=torch.int64, device=dev)
    first.scatter_reduce_(0, sr[ok], torch.arange(S, device=dev)[ok], reduce="amin")
    has = first < S
    rl = torch.zeros(R, dtype=torch.int32, device=dev)
    rl[has] = pl[q.pidx[first[has] * K].long()]
    return pl, rl.contiguous(), 12


def lego_pose_view(i, h, w, n_poses=120):
    """Config 4: the render_vid-style orbit of load_blender.py:51-56 (theta 0..360, phi -30, r 4)."""
    return scene.lego_view(360.0 * (i % n_poses) / n_poses, h, w, focal=1111.1111 * w / 800)


def spiral_pose_view(i, h, w, n_poses=120):
    """Config 3: the render_vid spiral (sgnerf_amd.render_vid.spiral_views: yaw 0->360 deg, pitch
    10 sin(2 pi i / n) deg, camera at the room centre)."""
    yaw, pitch = scene.spiral_yaw_pitch(i % n_poses, n_poses)
    return scene.room_view(h, w, yaw=yaw, pitch=pitch, campos=(2.0, 2.0, 1.5))


def pose_view(i, h, w, n_poses=120):
    yaw, pitch = scene.spiral_yaw_pitch(i % n_poses, n_poses)
    return scene.room_view(h, w, yaw=yaw + 15.0, pitch=pitch - 5.0)


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(pc, mlp, o, view, stride=4):
    """Oracle ('port'): C restatement of the query + torch-CPU fp32 aggregator/composite on the GPU
    box's host cores.  Main number: BASELINE config 1 (one 200x200 view at 32 samples per ray, the
    reference's CPU case) of the benched scene and pose; beside it a bounded sample of the
    headline workload itself (every `stride`-th pixel of the 800x800 SR-64 frame) and a
    1-thread rate."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import agg_ref
    import oracle_query as oq
    from dataclasses import replace
    from sgnerf_amd.hyper import grid_hyperparameters
    from sgnerf_amd.raygen import depth_table
    pts = {k: torch.from_numpy(getattr(pc, k)) for k in ("xyz", "embedding", "color", "dir", "conf")}

    def runner(oo):
        hy = grid_hyperparameters(oo, torch.from_numpy(pc.xyz.min(0)), torch.from_numpy(pc.xyz.max(0)))
        og = oq.OracleGrid(pc.xyz, hy, oo)

        def run(v, rd):
            t = depth_table(v.near, v.far, oo.z_depth_dim).numpy()
            t0 = time.perf_counter()
            q = og.query(v.campos, rd, t)
            with torch.no_grad():
                agg_ref.render(pts, mlp, torch.from_numpy(v.campos), torch.from_numpy(v.camrotc2w),
                               torch.from_numpy(rd), q, oo.SR)
            return time.perf_counter() - t0
        return run

    threads = torch.get_num_threads()
    # config 1: 200x200 view of the same pose (focal scaled with the image), SR 32
    yaw, pitch = scene.spiral_yaw_pitch(0, 120)
    v1 = scene.room_view(200, 200, yaw=yaw + 15.0, pitch=pitch - 5.0)
    run1 = runner(replace(o, SR=32))
    dt_c1 = run1(v1, v1.raydir)
    # sample of the headline workload (SR 64)
    idx = np.arange(view.h * view.w).reshape(view.h, view.w)[::stride, ::stride].reshape(-1)
    run2 = runner(o)
    dt2 = run2(view, view.raydir[idx])
    sub = view.raydir[idx][::4]
    torch.set_num_threads(1)
    oq.lib().sgnref_set_threads(1)
    dt1 = run2(view, sub)
    torch.set_num_threads(threads)
    oq.lib().sgnref_set_threads(threads)
    n1 = v1.raydir.shape[0]
    return {"value": n1 / dt_c1, "unit": "rays/s", "cores": threads, "kind": "port",
            "ms_per_frame": dt_c1 * 1e3,
            "sample": f"BASELINE config 1: one 200x200 view (focal 100) of the benched scene at SR=32, {n1} rays in "
                      f"{dt_c1:.2f} s on {threads} threads; C query (OpenMP) + torch-CPU fp32 aggregator/composite",
            "config2_sample": {"value": len(idx) / dt2, "unit": "rays/s", "cores": threads,
                               "sample": f"{len(idx)} rays ({view.h // stride}x{view.w // stride} strided subset of "
                                         f"the 800x800 SR={o.SR} frame 0) in {dt2:.2f} s"},
            "value_1thread": len(sub) / dt1,
            "sample_1thread": f"{len(sub)} rays of the config-2 sample in {dt1:.2f} s on 1 thread",
            "cpu_model": _cpu_model()}


def dense_pose_view(i, h, w):
    """SURVEY §8d dense stress variant: the cube face-on, the camera sliding by 2 cm per frame."""
    return scene.dense_stress_view(h, w, shift=0.02 * ((i % 5) - 2))


def render_run(args, precision, world, rank, dev, dist, steps, warmup, lego, want_stats=True):
    """Headline-shaped frame loop at `precision`; returns the result fields (no cpu baseline)."""
    sg = dict(shading_feature_mlp_layer2_bpnet=1, predict_semantic=1, semantic_guidance=1) if args.sg else {}
    o = HotPathOpts(SR=args.sr, precision=precision, **sg)
    dense = args.scene == "dense"
    spiral = args.scene == "spiral"
    pc = (scene.lego_standin(args.points, seed=0) if lego else
          scene.dense_cube(args.points, seed=0) if dense else scene.synth_room(args.points, seed=0))
    if args.sg:
        pc = scene.with_semantics(pc, seed=1, n_classes=20, cell=0.5)
    mlp = init_mlp(0, bias_std=0.01, bpnet_layers=1 if args.sg else 0, bpnet_dim=96 if args.sg else 0)
    mlp["alpha_branch.0.bias"] = mlp["alpha_branch.0.bias"] + 50.0  # opaque surfaces, as a trained scene
    r = HipRenderer(PointTables.from_cloud(pc, dev), mlp, o, dev)
    n_frames = warmup + steps
    # timed frame j renders pose j * N + rank whatever --warmup is (the warm-up frames take poses from
    # the other end of the spiral), so runs with different warm-up counts time the same frames
    poses = [(-1 - s * world - rank) % 120 for s in range(warmup)] + [(s * world + rank) for s in range(steps)]
    views = [(lego_pose_view if lego else dense_pose_view if dense else spiral_pose_view if spiral else pose_view)(
        p, args.h, args.w) for p in poses]
    rays = [torch.from_numpy(v.raydir).to(dev) for v in views]
    cams = [(torch.from_numpy(v.campos).to(dev), torch.from_numpy(v.camrotc2w).to(dev)) for v in views]
    R = args.h * args.w
    # grid build (once per point cloud), timed separately: host-synchronous wall time of the first
    # build (two size read-backs inside) and the HIP-event time of a rebuild
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r.querier.grid_for(r.points.xyz)
    torch.cuda.synchronize()
    grid_ms = (time.perf_counter() - t0) * 1e3
    gathered = [torch.empty(world * R, 3, dtype=torch.float32, device=dev) for _ in range(2)] \
        if dist and not args.no_gather else None

    sem = [{} for _ in range(n_frames)]
    if args.sg:
        # ray labels = a per-frame label image stand-in (BPNet's 2D prediction): the label of the
        # first neighbour of each ray's first occupied sample (plain query, untimed); seconds fixed
        pl = torch.from_numpy(pc.labels).to(dev)
        for i in range(n_frames):
            q = r.querier.query_samples(r.points.xyz, cams[i][0], rays[i], views[i].near, views[i].far)
            S = q.n_samples()
            sr = q.samp_ray[:S].long()
            ok = q.samp_nnb[:S] > 0
            first = torch.full((R,), S, dtype=torch.int64, device=dev)
            sid = torch.arange(S, device=dev)
            first.scatter_reduce_(0, sr[ok], sid[ok], reduce="amin")
            has = first < S
            rl = torch.zeros(R, dtype=torch.int32, device=dev)
            rl[has] = pl[q.pidx[first[has] * 8].long()]
            sem[i] = dict(point_labels=pl, ray_labels=rl.contiguous(), seconds=12)

    # N > 1: the finished frame is all-gathered on a side stream while the next frame renders;
    # frames alternate between two colour buffers so the collective never reads a buffer the
    # renderer is writing
    comm = torch.cuda.Stream(dev) if gathered is not None else None
    rgb_bufs = [None, None]
    gather_done = [None, None]

    def frame(i, marks=None, count=False):
        out = r.render(cams[i][0], cams[i][1], rays[i], views[i].near, views[i].far, want_opacity=True, marks=marks,
                       count_traffic=count, check_range="deferred", **sem[i])
        if gathered is not None:
            b = i & 1
            if rgb_bufs[b] is None:
                rgb_bufs[b] = torch.empty_like(out.rgb)
            if gather_done[b] is not None:  # the gather of frame i - 2 still reads this buffer
                torch.cuda.current_stream().wait_event(gather_done[b])
            rgb_bufs[b].copy_(out.rgb)
            ready = torch.cuda.Event()
            ready.record()
            with torch.cuda.stream(comm):
                comm.wait_event(ready)
                torch.distributed.all_gather_into_tensor(gathered[b], rgb_bufs[b])
                gather_done[b] = torch.cuda.Event()
                gather_done[b].record(comm)
        return out

    def drain():
        if comm is not None:
            torch.cuda.current_stream().wait_stream(comm)
        r.finish()   # the fp16-range guard of the frames rendered so far (raises if one failed)

    for i in range(warmup):
        frame(i)
        drain()
    torch.cuda.synchronize()
    events = []

    def marks(name):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        events[-1][name] = e

    gc.collect()   # untimed (see train_main)
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(warmup, n_frames):
        events.append({})
        frame(i, marks)
    drain()
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if dist:
        torch.distributed.all_reduce(el, op=torch.distributed.ReduceOp.MAX)
    elapsed = float(el.item())
    stage_names = ["query", "proj", "agg_rows", "agg_color", "composite"]
    order = stage_names + ["end"]
    stage_ms = {n: float(np.mean([ev[n].elapsed_time(ev[order[j + 1]]) for ev in events]))
                for j, n in enumerate(stage_names)}
    total_rays = R * steps * world
    res = {"value": total_rays / elapsed, "ms_per_frame": elapsed / steps * 1e3, "stages_ms": stage_ms,
           "grid_build_ms": grid_ms, "o": o, "r": r, "pc": pc, "mlp": mlp, "views": views}
    if not want_stats:
        return res
    # grid rebuild on the device clock (no host read-back inside the timed span: the build's two
    # size read-backs synchronise, so this is wall time of the stream with those syncs)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    e0.record()
    from sgnerf_amd.querier import HipGrid
    g2 = HipGrid(r.points.xyz, o)
    e1.record()
    torch.cuda.synchronize()
    g2.close()
    res["grid_rebuild_ms"] = {"hip_events": e0.elapsed_time(e1), "wall": (time.perf_counter() - t1) * 1e3}
    # occupancy / algorithmic work of the timed frames (deterministic re-render, untimed)
    n_nb, n_smp, n_samples, q_bytes, n_proj = [], [], [], [], []
    for i in range(warmup, n_frames):
        out = frame(i, count=True)
        drain()
        q = out.query
        S = q.n_samples()
        pp = r.points_projected()   # the f32 mode projects the frame's points only (sgn_frame_points)
        n_proj.append(pp[0] if pp is not None else r.points.n)
        cnt = [c & 0xFFFFFFFF for c in q.counters.tolist()]  # [3] is uint32
        W = cnt[1]
        n_samples.append(S)
        n_smp.append(W)
        n_nb.append(int(q.samp_nnb[:S].sum().item()))
        # query-stage algorithmic bytes (no reuse credit): march: ray direction + per-ray
        # outputs; kNN: voxel words + 16-B candidate records read, per-sample inputs and outputs
        q_bytes.append(R * (12 + 4 + 4 + 2 * args.sr) + 4 * cnt[2] + 16 * cnt[3] + S * (4 + 4 + 12 + 12 + 4 + 4 * 8)
                       + 4 * W)
    torch.cuda.synchronize()
    res.update(n_nb=float(np.mean(n_nb)), n_smp=float(np.mean(n_smp)), n_samples=float(np.mean(n_samples)),
               q_bytes=float(np.mean(q_bytes)), n_proj=float(np.mean(n_proj)))
    return res


def extra_render(args, world, rank, dev, dist, scene_name, sr, points, steps, warmup, label, sg=False):
    """One more frame workload at the headline's arithmetic, as an extra key of the bench line:
    rate, stage times, the row kernel's MFMA roofline fraction and the occupancy."""
    x3 = args.precision == "f32"
    a = argparse.Namespace(**{**vars(args), "scene": scene_name, "sr": sr, "points": points, "sg": sg})
    e = render_run(a, args.precision, world, rank, dev, dist, steps, warmup, scene_name == "lego")
    R = args.h * args.w
    flop_nb = FLOP_PER_ROW_SPLIT + (2 * 352 * 256 if sg else 0)
    peak = PEAK_X3_TFLOPS if x3 else PEAK_F16_TFLOPS
    st = e["stages_ms"]
    achieved = flop_nb * e["n_nb"] / (st["agg_rows"] * 1e-3) / 1e12
    out = {"value": e["value"], "unit": "rays/s", "ms_per_frame": e["ms_per_frame"], "steps": steps,
           "warmup": warmup, "n_gpus": world, "dtype": "f32 (3xf16 split MFMA, fp32 accumulate)" if x3 else "f16",
           "workload": f"{label}; {args.h}x{args.w} rays x SR={sr}, K=8",
           "stages_ms": st,
           "roofline": {"kernel": ("k_rows16" if x3 else "k_agg_rows") + (" (SG, + block2_bpnet.0)" if sg else ""),
                        "bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                        "frac": achieved / peak, "flop_per_valid_row": flop_nb, "avg_launch_ms": st["agg_rows"]},
           "occupancy": {"samples_per_ray": e["n_samples"] / R, "valid_samples_per_ray": e["n_smp"] / R,
                         "valid_neighbours_per_ray": e["n_nb"] / R}}
    del e
    torch.cuda.empty_cache()
    return out


def _query_counter(query_ms, key, path=os.path.join(ROOT, "profiles", "traffic_query_latest.json")):
    """Counter bytes per launch of k_knn27 / k_march (profiles/traffic_query_latest.json, written from
    the PMC summary of the same workload) and their rate over this run's query-stage time."""
    try:
        tj = json.load(open(path))
    except (OSError, ValueError):
        return None
    if tj.get("workload_key") != key:
        return None
    ks = tj.get("kernels", {})
    b = sum(v["bytes_per_launch"] for v in ks.values())
    return {"bytes_per_frame": b, "GBps_over_query_stage": b / (query_ms * 1e-3) / 1e9,
            "frac_of_hbm_peak": b / (query_ms * 1e-3) / 1e9 / PEAK_HBM_GBS,
            "per_kernel": {k: {"bytes_per_launch": v["bytes_per_launch"], "l2_hit_rate": v.get("l2_hit_rate"),
                               "counter_GBps_at_profiled_duration": v.get("counter_GBps")} for k, v in ks.items()},
            "source": tj.get("source")}


def main():
    args = parse()
    lego = args.scene == "lego"
    if args.sr is None:
        args.sr = 128 if lego else 64
    if args.points is None:
        args.points = 300_000 if lego else 3_900_000 if args.scene == "dense" else 1_200_000
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(self_launch(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} (launch with matching counts)")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    # SGN_BENCH_BACKEND=gloo: rehearsal of the N > 1 code path with every rank on the visible
    # GPU(s) (RCCL refuses two ranks on one device); frames are then not all-gathered
    backend = os.environ.get("SGN_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(torch.cuda.device_count(), 1)
        args.no_gather = True
    if dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if backend == "nccl":
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            torch.distributed.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if args.train:
        res = train_main(args, world, rank, dev, dist)
        if rank == 0:
            print(json.dumps(res))
        if dist:
            torch.distributed.destroy_process_group()
        return
    x3 = args.precision == "f32"
    h = render_run(args, args.precision, world, rank, dev, dist, args.steps, args.warmup, lego)
    R = args.h * args.w
    stage_ms = h["stages_ms"]
    flop_nb = FLOP_PER_ROW_SPLIT + (2 * 352 * 256 if args.sg else 0)  # + block2_bpnet.0 (SG)
    rows_flop = flop_nb * h["n_nb"]
    ref_flop = (FLOP_PER_NB + (2 * 352 * 256 if args.sg else 0)) * h["n_nb"]
    achieved = rows_flop / (stage_ms["agg_rows"] * 1e-3) / 1e12
    peak = PEAK_X3_TFLOPS if x3 else PEAK_F16_TFLOPS
    kname = "k_rows16" if x3 else "k_agg_rows"
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            if tj.get("kernel") == kname and tj.get("workload_key") == f"{args.h}x{args.w}x{args.sr}":
                traffic = tj.get("bytes_per_launch")
        except Exception:
            traffic = None
    res = {
        "metric": METRIC,
        "value": h["value"],
        "unit": "rays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": h["ms_per_frame"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32 (3xf16 split MFMA, fp32 accumulate)" if x3 else "f16",
        "data": "synthetic",
        "config": {
            "workload": (f"synth-lego stand-in {args.h}x{args.w} rays x SR={args.sr} samples, D=400, K=8, P=26, "
                         f"{args.points} neural points, Blender camera orbit, near 2 far 6 (BASELINE config 4, "
                         f"1 frame per rank per step)") if lego else
                        (f"synth-room {args.h}x{args.w} rays x SR={args.sr} samples, D=400, K=8, P=26, "
                         f"{args.points} neural points (BASELINE config 2, 1 frame per rank per step)")
                        + (" + SG-NeRF variant: semantic-guided kNN (20 labels), block2_bpnet 352->256" if args.sg else ""),
            "rays_per_frame": R, "SR": args.sr, "K": 8, "D": 400, "points": args.points,
            "parallelism": f"frame-sharded x{world}" + ("" if (not dist or args.no_gather)
                                                         else " + all-gather of frames (side stream, double-buffered)"),
            "mlp": "viewmlp 284-256-256 / 263-256-256 / alpha / colour 280-128x3-3 (341,764 params, random init)",
            "outputs": "rgb, ray mask, background transmission, coarse_point_opacity [R, SR]",
        },
        "roofline": {
            "kernel": kname + " (per-neighbour MLP 284->256->256->" + ("352->256->" if args.sg else "")
                      + "263->256->256 + alpha + K-blend)",
            "bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
            "frac": achieved / peak, "traffic": traffic,
            "peak_note": ("fp16 dense MFMA peak / 3 (each fp32 product = 3 fp16 MFMA products); native f32-input "
                          f"MFMA peak {PEAK_F32_NATIVE_TFLOPS} TF/s") if x3 else "fp16 dense MFMA peak",
            "flop_per_launch": rows_flop, "flop_per_valid_row": flop_nb, "avg_launch_ms": stage_ms["agg_rows"],
            "reference_formulation_TFLOPs": ref_flop / (stage_ms["agg_rows"] * 1e-3) / 1e12,
        },
        "roofline_query": {
            "kernel": "query stage (k_march + scan + k_emit_samples + k_knn)", "bound": "hbm/l2 gather",
            # SURVEY §8d byte model with NO reuse credit: every voxel word and 16-B candidate record
            # counted each time a sample reads it.  Most of those re-reads hit L2/MALL, so this
            # effective rate can exceed the HBM peak; HBM bytes proper come from the PMC passes
            # (profiles/, FETCH_SIZE + WRITE_SIZE of k_knn / k_march).
            "effective_GBps_no_reuse_credit": h["q_bytes"] / (stage_ms["query"] * 1e-3) / 1e9,
            "hbm_peak_GBps": PEAK_HBM_GBS,
            "bytes_per_frame_no_reuse_credit": h["q_bytes"],
            # HBM bytes of the query kernels from the PMC passes of the same workload (traffic file),
            # over this run's query-stage time, beside the no-reuse model
            "counter": _query_counter(stage_ms["query"], f"{args.h}x{args.w}x{args.sr}"),
        },
        "roofline_proj": {
            "kernel": ("k_point_proj16" if x3 else "k_point_proj") + (
                " (block1.0 point inputs of the points the frame's samples name, sgn_frame_points + subset "
                "projection, once per frame)"),
            "bound": "mfma", "achieved": FLOP_PER_POINT_PROJ * h["n_proj"] / (stage_ms["proj"] * 1e-3) / 1e12,
            "peak": peak, "unit": "TFLOP/s", "avg_launch_ms": stage_ms["proj"], "points_projected": h["n_proj"],
        },
        "stages_ms": stage_ms,
        "grid_build_ms": h["grid_build_ms"],
        "grid_rebuild_ms": h["grid_rebuild_ms"],
        "occupancy": {
            "samples_per_ray": h["n_samples"] / R,
            "valid_samples_per_ray": h["n_smp"] / R,
            "valid_neighbours_per_ray": h["n_nb"] / R,
        },
        "ms_per_frame": h["ms_per_frame"],
    }
    if not args.no_extras:
        # the other arithmetic mode on the same frames (extra key; the headline stays the reference's fp32)
        other = "f16" if x3 else "f32"
        e = render_run(args, other, world, rank, dev, dist, args.steps, args.warmup, lego, want_stats=False)
        peak_o = PEAK_F16_TFLOPS if x3 else PEAK_X3_TFLOPS
        res[f"{other}_mode"] = {"value": e["value"], "unit": "rays/s", "ms_per_frame": e["ms_per_frame"],
                                "dtype": "f16" if x3 else "f32 (3xf16 split MFMA)", "stages_ms": e["stages_ms"],
                                "roofline_frac": rows_flop / (e["stages_ms"]["agg_rows"] * 1e-3) / 1e12 / peak_o}
        del e
        torch.cuda.empty_cache()
        # BASELINE config 5 (training step, 4096-ray batches, DP over the ranks)
        tr = train_main(args, world, rank, dev, dist, steps=max(args.steps, 20), warmup=5)
        torch.cuda.empty_cache()
        tr16 = None
        if tr["dtype"] == "f32":
            tr16 = train_main(args, world, rank, dev, dist, steps=max(args.steps, 20), warmup=5, precision="f16")
            torch.cuda.empty_cache()
        # SURVEY §8d dense stress variant (3.9 M points in a 1 m cube, every candidate occupied)
        sa = argparse.Namespace(**{**vars(args), "scene": "dense", "points": 3_900_000})
        e = render_run(sa, args.precision, world, rank, dev, dist, 2, 1, False)
        Rd = args.h * args.w
        res["stress_dense"] = {
            "value": e["value"], "unit": "rays/s", "ms_per_frame": e["ms_per_frame"], "steps": 2, "warmup": 1,
            "dtype": res["dtype"], "stages_ms": e["stages_ms"],
            "workload": f"dense cube 3.9 M points, {args.h}x{args.w} rays x SR={args.sr}, face-on (SURVEY §8d)",
            "occupancy": {"samples_per_ray": e["n_samples"] / Rd, "valid_samples_per_ray": e["n_smp"] / Rd,
                          "valid_neighbours_per_ray": e["n_nb"] / Rd},
            "roofline_frac": flop_nb * e["n_nb"] / (e["stages_ms"]["agg_rows"] * 1e-3) / 1e12 / peak}
        del e
        torch.cuda.empty_cache()
        # BASELINE config 4 (lego stand-in, SR 128), the SG-NeRF variant on the config-2 frame and
        # config 3 (the 120-frame render_vid spiral, SR 24) on this job's GPUs, at the headline's arithmetic
        res["lego"] = extra_render(args, world, rank, dev, dist, scene_name="lego", sr=128, points=300_000, steps=4,
                                   warmup=1, label="BASELINE config 4: synth-lego stand-in, Blender orbit, "
                                                   "near 2 far 6, 300k points")
        res["sg"] = extra_render(args, world, rank, dev, dist, scene_name="room", sr=args.sr, points=args.points,
                                 steps=4, warmup=1, sg=True,
                                 label="config-2 frame with the SG-NeRF variant: semantic-guided kNN (20 labels), "
                                       "block2_bpnet 352->256")
        n3 = -(-120 // world)
        res[f"config3_{world}gpu"] = extra_render(
            args, world, rank, dev, dist, scene_name="spiral", sr=24, points=1_200_000, steps=n3, warmup=1,
            label=f"BASELINE config 3: 120-frame render_vid spiral (camera at the room centre, SR 24), "
                  f"frame-sharded over {world} GPU(s), {n3} frames per rank")
        keys = ("value", "unit", "ms_per_step", "steps", "warmup", "dtype", "final_loss", "graph_captures", "config")
        res["train_config5"] = {k: tr[k] for k in keys}
        if tr16 is not None:
            res["train_config5_f16"] = {k: tr16[k] for k in keys}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(h["pc"], h["mlp"], h["o"], h["views"][0])
    if rank == 0:
        print(json.dumps(res))
    if dist:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
