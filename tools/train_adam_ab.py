"""Same-box A/B (NOT product): config-5 training steps (bench.py train_main) with the point group on
the row-sparse Adam (the trainer's default) and on the dense PointAdam, interleaved, both precisions.
Prints one JSON line per run.   python tools/train_adam_ab.py [reps=2]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import bench  # noqa: E402
import sgnerf_amd.train_hip as th  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
_init = th.HipTrainer.__init__
mode = {"adam": "rows"}


def init(self, *a, **k):
    _init(self, *a, **k)
    if mode["adam"] == "dense":
        self.opt_pts = th.PointAdam(self.point_params, lr=self.base_lr[1], betas=(0.9, 0.999))


th.HipTrainer.__init__ = init
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
for prec in ("f32", "f16"):
    for r in range(reps):
        for m in ("dense", "rows"):
            mode["adam"] = m
            sys.argv = ["bench.py", "--train", "--train-precision", prec, "--steps", "30", "--warmup", "5",
                        "--no-cpu-baseline", "--points", "1200000"]
            res = bench.train_main(bench.parse(), 1, 0, dev, None)
            print(json.dumps({"precision": prec, "adam": m, "rep": r, "ms_per_step": res["ms_per_step"],
                              "final_loss": res["final_loss"]}), flush=True)
