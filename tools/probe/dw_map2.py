"""Probe (not product): sgn_f16_weight_grad with one operand all ones: which rows of the other it sums."""
import sys
import torch
sys.path.insert(0, ".")
import sgnerf_amd  # noqa
from sgnerf_amd import _lib
dev = "cuda:0"
rows, ncols = 32, 256


def run(d, x):
    part = torch.zeros(1, 256, ncols, device=dev)
    _lib.check(_lib.lib().sgn_f16_weight_grad(_lib.ptr(d), 256, _lib.ptr(x), ncols, ncols, rows, 1, _lib.ptr(part),
                                              _lib.stream_handle()), "f16dw")
    torch.cuda.synchronize()
    return part[0].double()


# A = ones: got[m][n] = sum_k x[k][n]; x[k][n] = 2^(k % 11) exact-ish -> decode which k were summed
ones_d = torch.ones(rows, 256, dtype=torch.float16, device=dev)
x = torch.zeros(rows, ncols, dtype=torch.float16, device=dev)
x[:, 0] = torch.arange(rows, device=dev).to(torch.float16)          # column 0: k
x[:, 1] = 1.0
got = run(ones_d, x)
print("B test: sum_k k =", got[0, 0].item(), "(ref", sum(range(rows)), ") count", got[0, 1].item(), "m=5:", got[5, :2].tolist())
# B = ones: got[m][n] = sum_k d[k][m]
ones_x = torch.ones(rows, ncols, dtype=torch.float16, device=dev)
d = torch.zeros(rows, 256, dtype=torch.float16, device=dev)
d[:, 0] = torch.arange(rows, device=dev).to(torch.float16)
d[:, 1] = 1.0
got = run(d, ones_x)
print("A test: sum_k k =", got[0, 0].item(), "count", got[1, 0].item(), "n=7:", got[0, 7].item(), got[1, 7].item())
