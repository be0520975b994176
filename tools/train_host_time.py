"""Host issue time vs GPU-bound wall of config-5 training steps (NOT product): bench.py's train_main
with HipTrainer.step timed per call without synchronising (the launches queue; the call returns once
issued), so host ms/step is the Python + launch overhead the GPU must stay ahead of.
    python tools/train_host_time.py [f32|f16]"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import bench  # noqa: E402
import sgnerf_amd.train_hip as th  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "f32"
host = []
_step = th.HipTrainer.step


def step(self, *a, **k):
    t0 = time.perf_counter()
    out = _step(self, *a, **k)
    host.append(time.perf_counter() - t0)
    return out


th.HipTrainer.step = step
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
sys.argv = ["bench.py", "--train", "--train-precision", prec, "--steps", "30", "--warmup", "5", "--no-cpu-baseline",
            "--points", "1200000"]
res = bench.train_main(bench.parse(), 1, 0, dev, None)
h = sorted(host[5:])
print(json.dumps({"precision": prec, "wall_ms_per_step": res["ms_per_step"], "host_ms_per_step_median": h[len(h) // 2] * 1e3,
                  "host_ms_per_step_mean": sum(h) / len(h) * 1e3}))
