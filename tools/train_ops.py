"""Which host calls launch the training step's fill / copy kernels: torch.profiler over a few
config-5 steps, every aten op that issued a fill or copy (or hipMemcpy / hipMemset), with the
innermost sg-nerf_amd frame of its Python stack.  Run on the GPU box:
    python tools/train_ops.py [f32|f16]"""
import collections
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, ".")
import bench  # noqa: E402
from sgnerf_amd import scene  # noqa: E402
from sgnerf_amd.opts import HotPathOpts  # noqa: E402
from sgnerf_amd.train import PointParams  # noqa: E402
from sgnerf_amd.train_hip import HipTrainer  # noqa: E402
from sgnerf_amd.weights import init_mlp  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "f32"
dev = "cuda:0"
o = HotPathOpts(SR=24, is_train=1)
pc = scene.synth_room(1_200_000, seed=0)
mlp = init_mlp(0, bias_std=0.01)
mlp["alpha_branch.0.bias"] = mlp["alpha_branch.0.bias"] + 50.0
points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, dev)
tr = HipTrainer(points, mlp, o, dev, precision=prec)
g = torch.Generator().manual_seed(1)
batches = []
for i in range(10):
    v = bench.pose_view(int(torch.randint(0, 120, (1,), generator=g)), 800, 800)
    idx = torch.randint(0, 800 * 800, (4096,), generator=g)
    gt = torch.rand(4096, 3, generator=g)
    batches.append(tuple(x.to(dev) for x in (torch.from_numpy(v.campos), torch.from_numpy(v.camrotc2w),
                                               torch.from_numpy(v.raydir)[idx], gt)))
for b in batches[:5]:
    tr.step(*b[:3], 0.1, 8.0, b[3])
torch.cuda.synchronize()
steps = 5
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    for b in batches[5:5 + steps]:
        tr.step(*b[:3], 0.1, 8.0, b[3])
    torch.cuda.synchronize()

GLUE = ("Fill", "fill", "copy", "Copy", "Memcpy", "Memset", "memcpy", "memset")
cnt = collections.Counter()
for e in prof.events():
    kids = [k for k in getattr(e, "cpu_children", [])]
    names = [k.name for k in getattr(e, "kernels", [])]
    if not any(any(t in n for t in GLUE) for n in names):
        continue
    stack = [s for s in (e.stack or []) if "sg-nerf_amd" in s or "bench" in s]
    where = stack[0] if stack else "?"
    cnt[(e.name, where, ",".join(sorted(set(n[:40] for n in names))))] += 1
for (name, where, ks), c in sorted(cnt.items(), key=lambda x: -x[1]):
    print(f"{c / steps:5.2f}/step  {name:32s} {where}  [{ks}]")
