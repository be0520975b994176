"""Probe (not product): which d column / x column each output element of sgn_f16_weight_grad picks up."""
import sys
import torch
sys.path.insert(0, ".")
import sgnerf_amd  # noqa
from sgnerf_amd import _lib
dev = "cuda:0"
rows, ncols = 32, 256
# d[r][m] = 1 if r == m % 32 (one row per column group), x[r][n] = n + 1000 r: dW[m][n] = x[m % 32][n]
d = torch.zeros(rows, 256, dtype=torch.float16, device=dev)
for m in range(256):
    d[m % 32, m] = 1.0 + m // 32   # weight encodes the column block
x = torch.zeros(rows, ncols, dtype=torch.float16, device=dev)
for r in range(rows):
    x[r] = torch.arange(ncols, device=dev) % 64 + 64 * (r % 16)  # exact in fp16 (< 2048)
part = torch.zeros(1, 256, ncols, device=dev)
_lib.check(_lib.lib().sgn_f16_weight_grad(_lib.ptr(d), 256, _lib.ptr(x), ncols, ncols, rows, 1, _lib.ptr(part),
                                          _lib.stream_handle()), "f16dw")
torch.cuda.synchronize()
ref = d.double().t() @ x.double()
got = part[0].double()
bad = (got - ref).abs() > 1e-3
print("bad elements", int(bad.sum()), "of", bad.numel())
for m in [0, 1, 2, 3, 4, 5, 16, 17, 31, 32, 33]:
    print("m", m, "got", got[m, :6].tolist(), "ref", ref[m, :6].tolist())
