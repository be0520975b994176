# the same check against the product library (sgn_f16_weight_grad)
import sys, torch
sys.path.insert(0, ".")
import sgnerf_amd  # noqa
from sgnerf_amd import _lib
dev = "cuda:0"
rows, ncols = 32, 256
d = torch.zeros(rows, 256, dtype=torch.float16, device=dev)
for r in range(rows):
    d[r] = torch.arange(256, device=dev).to(torch.float32).remainder(64).to(torch.float16) + 64 * (r % 16)
x = torch.ones(rows, ncols, dtype=torch.float16, device=dev)
part = torch.zeros(256 * ncols, device=dev)
_lib.check(_lib.lib().sgn_f16_weight_grad(_lib.ptr(d), 256, _lib.ptr(x), ncols, ncols, rows, 1, _lib.ptr(part), _lib.stream_handle()), "x")
torch.cuda.synchronize()
got = part.view(256, ncols).cpu().double()
ref = (d.double().t() @ x.double()).cpu()
print("product lib: max err", float((got - ref).abs().max()), "got[0:4,0]", got[0:4, 0].tolist(), "ref", ref[0:4, 0].tolist())
