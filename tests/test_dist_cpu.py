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


def test_launch_ranks_gloo():
    """bench.py --gpus N's launcher (dist.launch_ranks) on CPU: N gloo ranks rendezvous on
    127.0.0.1 and see the forwarded arguments."""
    import json
    probe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dist_probe.py")
    env = dict(os.environ, OMP_NUM_THREADS="1")
    res = sd.launch_ranks(probe, 3, ["--steps", "2"], env=env, capture=True)
    assert res.returncode == 0, res.stderr[-2000:]
    line = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1, res.stdout
    out = json.loads(line[0])
    assert out == {"world": 3, "sum": 6.0, "argv": ["--steps", "2"], "master": "127.0.0.1"}


def test_touched_rows():
    from sgnerf_amd.train import touched_rows
    g = torch.Generator().manual_seed(0)
    N, K, cap = 40, 4, 30
    pidx = torch.randint(-1, N, (cap * K,), generator=g, dtype=torch.int32)
    S = 17
    idx, cnt = touched_rows(pidx, torch.tensor(S), K, N)
    p = pidx.view(cap, K)[:S]
    want = sorted(set(p[p >= 0].tolist()) | {0})
    assert int(cnt) == len(want)
    assert idx[:len(want)].tolist() == want
    assert bool((idx[len(want):] == N).all()) and idx.shape == (N + 1,)


def _rows_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from sgnerf_amd.train import _allreduce_point_rows, gather_counts, touched_rows
        N, K, cap = 60, 4, 25
        g = torch.Generator().manual_seed(10 + rank)
        pidx = torch.randint(-1, N, (cap * K,), generator=g, dtype=torch.int32)
        S = 20 - 3 * rank
        p = pidx.view(cap, K)[:S]
        rows = sorted(set(p[p >= 0].tolist()) | {0})
        grads = [torch.zeros(N, c) for c in (5, 3, 1)]
        for t in grads:    # non-zero only on rows this rank's samples reach
            t[rows] = torch.randn(len(rows), t.shape[1], generator=g)
        dense = [t.clone() for t in grads]
        for t in dense:
            torch.distributed.all_reduce(t)
            t /= world
        derived = [t.clone() for t in grads]
        _allreduce_point_rows(derived)
        idx, cnt = touched_rows(pidx, torch.tensor(S), K, N)
        counts = gather_counts(cnt).tolist()
        _allreduce_point_rows(grads, idx, counts)
        ok = all(torch.allclose(a, b, rtol=1e-6, atol=1e-7) for a, b in zip(grads, dense))
        same = all(torch.equal(a, b) for a, b in zip(grads, derived))
        q.put((rank, ok, same, torch.cat([t.reshape(-1) for t in grads])))
    except Exception as e:
        q.put((rank, repr(e), None, None))
    finally:
        torch.distributed.destroy_process_group()


def test_sparse_point_row_allreduce_world2():
    """_allreduce_point_rows with device-built touched rows (the HipTrainer path, no host sync
    beyond the step's own) equals the dense mean all-reduce and the gradient-derived variant,
    and every rank ends with bit-identical gradients."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rows_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=120) for _ in range(world)), key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok, same, _ in res:
        assert ok is True, f"rank {rank}: {ok}"
        assert same, f"rank {rank}: explicit and derived index paths differ"
    assert torch.equal(res[0][3], res[1][3])
