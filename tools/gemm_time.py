"""Launch timing of the fp32 training step's row GEMMs in isolation (not product): the backward-data
product d1 = (d2 W) * LReLU'(z1) (k_x3rows<16, 4>, mask + amax), the forward z4 = LReLU(z3) W^T + b,
and the weight gradient d2^T [LReLU(z1) | 1] (k_x3dw), at config 5's row count, on synthetic
operands.  HIP events on torch's current stream (the launches go on it); the library from
SGN_HIP_LIB= if set.  Prints one JSON line.  Usage (GPU box): python tools/gemm_time.py [rows]"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import sgnerf_amd  # noqa: E402,F401
from sgnerf_amd import _lib  # noqa: E402
from sgnerf_amd.train_f32 import _addr, _operand, _rows_gemm, _splitk_gemm, SPLITS_ROWS  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 147_000
cap = (rows + 127) // 128 * 128
dev = "cuda:0"
g = torch.Generator(device=dev).manual_seed(0)
f32 = dict(device=dev, dtype=torch.float32)
d2 = torch.randn(cap, 256, generator=g, **f32)
z1 = torch.randn(cap, 256, generator=g, **f32)
z3 = torch.randn(cap, 256, generator=g, **f32)
w = torch.randn(256, 256, generator=g, **f32) * 0.05
bias = torch.randn(256, generator=g, **f32) * 0.01
out = torch.empty(cap, 256, **f32)
part = torch.empty(SPLITS_ROWS, 256, 257, **f32)
cnt = torch.tensor([rows], dtype=torch.int32, device=dev)
shift = torch.tensor([5], dtype=torch.int32, device=dev)
amax = torch.zeros(4, dtype=torch.int32, device=dev)
amax[0] = torch.tensor(4.5, dtype=torch.float32).view(torch.int32)
A = lambda t, i=0: _addr(t, i)  # noqa: E731
gs = {
    "bwd_data_16x4": _rows_gemm(_operand(A(d2), 256, 256, 0, amax=A(amax, 0)), _operand(A(w), 256, 256, 1, shift=A(shift)),
                                cap, 256, 256, A(cnt), A(out), 256, mask=A(z1), ldm=256, amax_out=A(amax, 1)),
    "fwd_16x4": _rows_gemm(_operand(A(z3), 256, 256, 0, act=1), _operand(A(w), 256, 256, 0, shift=A(shift)), cap, 256, 256,
                           A(cnt), A(out), 256, bias=A(bias)),
    "dw": _splitk_gemm(_operand(A(d2), 256, 256, 1, amax=A(amax, 0)), _operand(A(z1), 256, 256, 1, ones_col=256, act=1),
                       256, 257, cap, A(cnt), A(part), SPLITS_ROWS),
}
L = _lib.lib()
st = _lib.stream_handle()
bp = torch.empty(1 << 20, dtype=torch.uint8, device=dev)
for k in list(gs):   # the same rows launches with the weight images (bpack)
    if gs[k].mode == 0:
        g2 = type(gs[k]).from_buffer_copy(gs[k])
        g2.bpack = bp.data_ptr()
        gs[k + "_bpack"] = g2
res = {"rows": rows, "lib": os.path.basename(os.environ.get("SGN_HIP_LIB", "in-tree"))}
for name, ga in gs.items():
    def run():
        _lib.check(L.sgn_x3_gemm(ctypes.byref(ga), st), name)
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    n = 20
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        run()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / n * 1e3
    mb = rows * 256 * 4 * (3 if name.startswith("bwd") else 2 if name.startswith("fwd") else 2) / 1e6
    res[name] = {"us": round(us, 1), "GB/s": round(mb / us * 1e3, 0)}
print(json.dumps(res))
