"""Same-box A/B of k_agg_bwd builds (NOT product).  A few config-5 training steps (bench.py's
train_main, f16) on the in-tree library record the last sgn_aggregate_backward[_sg] call; every
library named on the command line (tools/src_variant.sh builds) then replays that call between
HIP events on the same stream, interleaved over rounds.  Before timing, each library's outputs of
one replay (deltas, h4, dza bit for bit; point gradients to 1e-5 relative, atomics reorder) are
compared with the in-tree library's.  Prints one JSON line per library.
    python tools/agg_bwd_ab.py [--sg] lib.so ..."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import bench  # noqa: E402
import sgnerf_amd.train_hip as th  # noqa: E402
from sgnerf_amd import _lib  # noqa: E402

sg = "--sg" in sys.argv
libs = [a for a in sys.argv[1:] if not a.startswith("--")]
NAME = "sgn_aggregate_backward_sg" if sg else "sgn_aggregate_backward"
rec = {}
L0 = _lib.lib()


class Proxy:
    def __getattr__(self, k):
        f = getattr(L0, k)
        if k != NAME:
            return f

        def w(*a):
            rec["args"] = a
            return f(*a)
        return w


_lib.lib = lambda: Proxy()
_init = th.HipTrainer.__init__


def init(self, *a, **k):
    _init(self, *a, **k)
    rec["tr"] = self


th.HipTrainer.__init__ = init
_step = th.HipTrainer.step


def step(self, *a, **k):   # the replayed call reads the batch's camera / ray tensors: keep them alive
    rec["batch"] = (a, k)
    return _step(self, *a, **k)


th.HipTrainer.step = step
sys.argv = ["bench.py", "--train", "--train-precision", "f16", "--steps", "2", "--warmup", "2",
            "--no-cpu-baseline", "--points", "1200000"] + (["--sg"] if sg else [])
args = bench.parse()
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
bench.train_main(args, 1, 0, dev, None)
torch.cuda.synchronize()
tr, a = rec["tr"], rec["args"]
n = int(a[4 if sg else 2])
P = tr.points
outs = [tr.d[0], tr.d[1], tr.d[2], tr.d[3], tr.h4, tr.dza] + ([tr.db] if sg else [])
grads = [P.points_embeding.grad, P.points_color.grad, P.points_dir.grad, P.points_conf.grad]


def fn_of(path):
    if path == "intree":
        return getattr(L0, NAME)
    h = ctypes.CDLL(path)
    f = getattr(h, NAME)
    f.restype, f.argtypes = _lib.SIGNATURES[NAME]
    return f


def snapshot(f):
    for t in outs:
        t.zero_()
    for g in grads:
        g.zero_()
    assert f(*a) == 0
    torch.cuda.synchronize()
    return [t.clone() for t in outs], [g.clone() for g in grads]


fns = {p: fn_of(p) for p in ["intree"] + libs}
ref_o, ref_g = snapshot(fns["intree"])
rows = n * 8
check = {}
for p in libs:
    o, g = snapshot(fns[p])
    same = all(torch.equal(x.view(-1)[: rows * (x.numel() // x.shape[0])], y.view(-1)[: rows * (x.numel() // x.shape[0])])
               for x, y in zip(o, ref_o))
    gerr = max(float((x - y).abs().max() / (y.abs().max() + 1e-30)) for x, y in zip(g, ref_g))
    check[p] = {"deltas_bitexact": bool(same), "grad_rel_err": gerr}
st = torch.cuda.current_stream()
times = {p: [] for p in fns}
for rnd in range(6):
    for p, f in fns.items():
        for _ in range(2):
            f(*a)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(10):
            f(*a)
        e1.record(st)
        torch.cuda.synchronize()
        times[p].append(e0.elapsed_time(e1) / 10)
for p in fns:
    print(json.dumps({"lib": os.path.basename(p), "n_items": n, "sg": sg, "ms_median": float(np.median(times[p])),
                      "ms_min": float(np.min(times[p])), **check.get(p, {})}), flush=True)
