"""Row-sparse point Adam workload of config-5 training steps (NOT product): bench.py's train_main with
every sgn_adam_rows launch followed by a read-back of its compact (row, step held) list -- rows per
launch, zero-gradient replays per row (mean / p50 / p90 / max), rows per 64-lane wave spread.
    python tools/adam_rows_stats.py [f32|f16]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import bench  # noqa: E402
import sgnerf_amd.train_hip as th  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "f16"
stats = []
_launch = th.PointAdam._launch


def launch(self, step, apply, rows=None, *a, **k):
    pb = _launch(self, step, apply, rows, *a, **k)
    if rows is not None:
        ws = self._ws.view(torch.int32)
        n = int(ws[0].item())
        cap = (self._ws.numel() // 4 - 4) // 2
        r = ws[4:4 + n].cpu().numpy()
        fr = ws[4 + cap:4 + cap + n].cpu().numpy()
        upto = step - 1 if apply else step
        rep = np.maximum(upto - fr, 0)
        stats.append({"step": step, "apply": apply, "rows": n, "replay_mean": float(rep.mean()) if n else 0,
                      "replay_p50": float(np.percentile(rep, 50)) if n else 0,
                      "replay_p90": float(np.percentile(rep, 90)) if n else 0, "replay_max": int(rep.max()) if n else 0,
                      "row_min": int(r.min()) if n else -1})
    return pb


th.PointAdam._launch = launch
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
sys.argv = ["bench.py", "--train", "--train-precision", prec, "--steps", "40", "--warmup", "5", "--no-cpu-baseline",
            "--points", "1200000"]
bench.train_main(bench.parse(), 1, 0, dev, None)
for s in stats[::4] + stats[-2:]:
    print(json.dumps(s))
