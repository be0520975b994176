"""Host-side (Python) time of the training step by function (cProfile), with the step's wall time and
the host issue time beside it.  Run on the GPU box: python tools/train_host_cprofile.py [f16|f32]"""
import cProfile
import pstats
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

prec = sys.argv[1] if len(sys.argv) > 1 else "f16"
dev = "cuda:0"
o = HotPathOpts(SR=24, is_train=1)
pc = scene.synth_room(1_200_000, seed=0)
mlp = init_mlp(0, bias_std=0.01)
mlp["alpha_branch.0.bias"] = mlp["alpha_branch.0.bias"] + 50.0
points = PointParams(pc.xyz, pc.embedding, pc.color, pc.dir, pc.conf, dev)
tr = HipTrainer(points, mlp, o, dev, precision=prec)
g = torch.Generator().manual_seed(1)
batches = []
for i in range(45):
    v = bench.pose_view(int(torch.randint(0, 120, (1,), generator=g)), 800, 800)
    idx = torch.randint(0, 800 * 800, (4096,), generator=g)
    gt = torch.rand(4096, 3, generator=g)
    batches.append(tuple(x.to(dev) for x in (torch.from_numpy(v.campos), torch.from_numpy(v.camrotc2w),
                                               torch.from_numpy(v.raydir)[idx], gt)))
for b in batches[:5]:
    tr.step(*b[:3], 0.1, 8.0, b[3])
torch.cuda.synchronize()
t0 = time.perf_counter()
for b in batches[5:25]:
    tr.step(*b[:3], 0.1, 8.0, b[3])
torch.cuda.synchronize()
print(f"{prec}: wall {1e3 * (time.perf_counter() - t0) / 20:.3f} ms/step")
pr = cProfile.Profile()
pr.enable()
for b in batches[25:45]:
    tr.step(*b[:3], 0.1, 8.0, b[3])
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(30)
st.sort_stats("cumulative").print_stats(40)
