"""Timing experiment (NOT product): config-5 f16 training steps in which every sgn_aggregate_backward
call is issued twice back to back (the second call's gradients are garbage: timing only), so a kernel
trace shows the in-step launch next to a warm re-launch on the same inputs.
    rocprofv3 --kernel-trace -d <dir> -o run --output-format csv -- python tools/agg_bwd_twice.py
then: python tools/agg_bwd_twice.py --report <run_kernel_trace.csv>"""
import csv
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]

if len(sys.argv) > 2 and sys.argv[1] == "--report":
    kt = sorted(csv.DictReader(open(sys.argv[2])), key=lambda r: int(r["Start_Timestamp"]))
    d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in kt if re.search("k_agg_bwd", r["Kernel_Name"])]
    first, second = d[0::2][-20:], d[1::2][-20:]
    print("in-step launch %.1f us, warm re-launch %.1f us (last 20 steps)" % (sum(first) / len(first) / 1e3,
                                                                              sum(second) / len(second) / 1e3))
    sys.exit(0)

import torch  # noqa: E402
import bench  # noqa: E402
from sgnerf_amd import _lib  # noqa: E402

L0 = _lib.lib()


class Proxy:
    def __getattr__(self, k):
        f = getattr(L0, k)
        if k != "sgn_aggregate_backward":
            return f

        def w(*a):
            rc = f(*a)
            f(*a)
            return rc
        return w


_lib.lib = lambda: Proxy()
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
sys.argv = ["bench.py", "--train", "--train-precision", "f16", "--steps", "30", "--warmup", "5", "--no-cpu-baseline",
            "--points", "1200000"]
bench.train_main(bench.parse(), 1, 0, dev, None)
