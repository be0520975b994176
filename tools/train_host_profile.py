"""Host-side (CPU) time of the HIP training step by torch op, and the step's wall time with
the GPU synchronised per phase.  Run on the GPU box: python tools/train_host_profile.py"""
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from sgnerf_amd import scene  # noqa: E402
from sgnerf_amd.opts import HotPathOpts  # noqa: E402
from sgnerf_amd.train import PointParams  # noqa: E402
from sgnerf_amd.train_hip import HipTrainer  # noqa: E402
from sgnerf_amd.weights import init_mlp  # noqa: E402

dev = "cuda:0"
o = HotPathOpts(SR=24, is_train=1)
pc = scene.synth_room(1_200_000, seed=0)
mlp = init_mlp(0, bias_std=0.01)
mlp["alpha_branch.0.bias"] = mlp["alpha_branch.0.bias"] + 50.0
points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, dev)
tr = HipTrainer(points, mlp, o, dev)
g = torch.Generator().manual_seed(1)
batches = []
for i in range(25):
    v = bench.pose_view(int(torch.randint(0, 120, (1,), generator=g)), 800, 800)
    idx = torch.randint(0, 800 * 800, (4096,), generator=g)
    gt = torch.rand(4096, 3, generator=g)
    batches.append(tuple(x.to(dev) for x in (torch.from_numpy(v.campos), torch.from_numpy(v.camrotc2w),
                                               torch.from_numpy(v.raydir)[idx], gt)))
for b in batches[:5]:
    tr.step(*b[:3], 0.1, 8.0, b[3])
torch.cuda.synchronize()
# host time per step with no GPU sync inside (the GPU runs behind)
t0 = time.perf_counter()
for b in batches[5:15]:
    tr.step(*b[:3], 0.1, 8.0, b[3])
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"host issue {1e3 * (t1 - t0) / 10:.3f} ms/step, drain after {1e3 * (t2 - t1):.3f} ms")
# in-process A/B of the graph-captured loss stage: blocks of 10 steps, alternated
res = {False: [], True: []}
for rep in range(4):
    for ug in (False, True):
        tr.use_graph = ug
        for b in batches[:2]:
            tr.step(*b[:3], 0.1, 8.0, b[3])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for b in batches[5:15]:
            tr.step(*b[:3], 0.1, 8.0, b[3])
        torch.cuda.synchronize()
        res[ug].append(1e3 * (time.perf_counter() - t0) / 10)
for ug in (False, True):
    print(f"use_graph={ug}: ms/step " + " ".join(f"{x:.3f}" for x in res[ug]))
tr.use_graph = True
t0 = time.perf_counter()
for b in batches[5:15]:
    tr.step(*b[:3], 0.1, 8.0, b[3])
t1 = time.perf_counter()
torch.cuda.synchronize()
print(f"graph: host issue {1e3 * (t1 - t0) / 10:.3f} ms/step, drain after {1e3 * (time.perf_counter() - t1):.3f} ms")
from torch.profiler import ProfilerActivity, profile  # noqa: E402
with profile(activities=[ProfilerActivity.CPU]) as prof:
    for b in batches[15:20]:
        tr.step(*b[:3], 0.1, 8.0, b[3])
    torch.cuda.synchronize()
ev = prof.key_averages()
print(f"ops/step {sum(e.count for e in ev if e.key.startswith('aten::')) / 5:.0f}")
print(ev.table(sort_by="self_cpu_time_total", row_limit=40))
