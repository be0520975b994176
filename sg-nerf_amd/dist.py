"""Multi-GPU sharding of the per-ray path.

Rays are independent given the read-only point cloud and MLP weights, so the path
shards with no data-path collective: every rank holds a replica of the points and
builds its own grid.  Two partitions:

  frames     round-robin over ranks (config 3 spiral): rank r renders frames
             r, r+N, r+2N, ...; one all-gather per step assembles the N frames.
  row bands  one frame split into N contiguous row bands (balanced to one row);
             one all-gather of the (padded) bands assembles the frame.

The collective is torch.distributed all_gather_into_tensor: RCCL over xGMI on the
GPU box (backend "nccl"), gloo on CPU in the tests.  Rendering itself is passed in
as a callable, so these functions are the same for the HIP renderer and the tests.
"""
import os
import socket
import subprocess
import sys

import torch
import torch.distributed as dist


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def frame_assignment(n_frames, world_size, rank):
    """Frames rendered by `rank` (round-robin)."""
    return list(range(rank, n_frames, world_size))


def row_bands(h, world_size):
    """[(r0, r1)] per rank, contiguous, sizes differ by at most one row."""
    base, extra = divmod(h, world_size)
    out, r0 = [], 0
    for r in range(world_size):
        r1 = r0 + base + (1 if r < extra else 0)
        out.append((r0, r1))
        r0 = r1
    return out


def gather_step(local, group=None):
    """All-gather one tensor per rank (same shape) -> [N, *shape] on every rank."""
    n, _ = world()
    if n == 1:
        return local[None]
    local = local.contiguous().reshape((-1,) + tuple(local.shape[1:])) if local.dim() else local.reshape(1)
    out = torch.empty((n * local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, local, group=group)  # concatenated along dim 0 (gloo and RCCL)
    return out.view((n,) + tuple(local.shape))


def render_frames(render_frame, n_frames, h, w, device, channels=3, group=None):
    """Render frames 0..n_frames-1 across ranks; returns [n_frames, h*w, channels] on
    every rank.  render_frame(i) -> [h*w, channels] tensor on `device`.  Ranks with no
    frame left in the last step contribute a zero tile that is dropped."""
    n, rank = world()
    steps = (n_frames + n - 1) // n
    frames = torch.empty(steps * n, h * w, channels, dtype=torch.float32, device=device)
    for s in range(steps):
        i = s * n + rank
        tile = render_frame(i) if i < n_frames else torch.zeros(h * w, channels, dtype=torch.float32, device=device)
        frames[s * n:(s + 1) * n] = gather_step(tile.reshape(h * w, channels).float(), group)
    return frames[:n_frames]


def render_frame_bands(render_rows, h, w, device, channels=3, group=None):
    """One frame split in row bands.  render_rows(r0, r1) -> [(r1-r0)*w, channels].
    Returns the full [h*w, channels] frame on every rank."""
    n, rank = world()
    bands = row_bands(h, n)
    r0, r1 = bands[rank]
    max_rows = max(b - a for a, b in bands)
    tile = torch.zeros(max_rows * w, channels, dtype=torch.float32, device=device)
    if r1 > r0:
        tile[: (r1 - r0) * w] = render_rows(r0, r1).reshape(-1, channels).float()
    allt = gather_step(tile, group)
    return torch.cat([allt[r, : (b - a) * w] for r, (a, b) in enumerate(bands)], dim=0)


def max_over_ranks(x, device):
    """Scalar max over ranks (bench timing)."""
    n, _ = world()
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    if n > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def launch_ranks(script, nproc, argv, env=None, capture=False):
    """Run `script argv` as nproc ranks under torch.distributed.run (one node, rendezvous on
    127.0.0.1, a free port) in a child process; returns its CompletedProcess.  Nothing here
    touches the GPU, so each rank initialises its own device (bench.py --gpus N)."""
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(script)] + list(argv)
    return subprocess.run(cmd, env=dict(os.environ if env is None else env), capture_output=capture, text=True)
