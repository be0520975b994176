"""world_size-2 gloo tests of the frame / row-band sharding (sgnerf_amd.dist), the
same functions bench.py and render_vid use over RCCL on the GPU box.  The renderer
is replaced by a deterministic function of (frame, pixel), so the assembled frames
can be checked exactly."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from sgnerf_amd import dist as sd


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _fake_frame(i, h, w):
    pix = torch.arange(h * w, dtype=torch.float32)
    return torch.stack([pix + 1000 * i, -pix, torch.full_like(pix, float(i))], dim=-1)


def _worker(rank, world, port, h, w, n_frames, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rendered = []
        frames = sd.render_frames(lambda i: (rendered.append(i), _fake_frame(i, h, w))[1], n_frames, h, w, "cpu")
        ref = torch.stack([_fake_frame(i, h, w) for i in range(n_frames)])
        ok_frames = torch.equal(frames, ref) and rendered == sd.frame_assignment(n_frames, world, rank)
        full = _fake_frame(7, h, w).view(h, w, 3)
        band = sd.render_frame_bands(lambda r0, r1: full[r0:r1].reshape(-1, 3), h, w, "cpu")
        ok_bands = torch.equal(band, full.reshape(-1, 3))
        m = sd.max_over_ranks(float(rank) + 0.5, "cpu")
        q.put((rank, ok_frames, ok_bands, m))
    except Exception as e:  # report instead of hanging the parent on q.get
        q.put((rank, repr(e), None, None))
    finally:
        torch.distributed.destroy_process_group()


@pytest.mark.parametrize("n_frames,h", [(5, 7), (4, 6), (1, 3)])
def test_sharded_rendering_world2(n_frames, h):
    world, w = 2, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, h, w, n_frames, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok_frames, ok_bands, m in res:
        assert ok_frames is True, f"rank {rank}: {ok_frames}"
        assert ok_frames, f"rank {rank}: frame sharding"
        assert ok_bands, f"rank {rank}: row bands"
        assert m == world - 0.5


def test_row_bands_and_assignment():
    assert sd.row_bands(800, 8) == [(100 * i, 100 * (i + 1)) for i in range(8)]
    b = sd.row_bands(10, 4)
    assert b == [(0, 3), (3, 6), (6, 8), (8, 10)]
    assert sd.row_bands(1, 2) == [(0, 1), (1, 1)]
    assert sd.frame_assignment(120, 8, 3) == list(range(3, 120, 8))
