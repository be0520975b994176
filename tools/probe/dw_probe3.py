import ctypes, torch
lib = ctypes.CDLL("./tools/probe/dw_probe.so")
dev = "cuda:0"
rows, ncols = 32, 256
d = torch.zeros(rows, 256, dtype=torch.float16, device=dev)
for r in range(rows):
    d[r] = torch.arange(256, device=dev).to(torch.float32).remainder(64).to(torch.float16) + 64 * (r % 16)
x = torch.ones(rows, ncols, dtype=torch.float16, device=dev)
part = torch.zeros(256 * ncols + 4096, device=dev)
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
lib.probe_f16_weight_grad.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                      ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]
lib.probe_f16_weight_grad(d.data_ptr(), 256, x.data_ptr(), ncols, ncols, rows, 1, part.data_ptr(), st)
torch.cuda.synchronize()
base = 256 * ncols
af = part[base:base + 512].view(64, 8).cpu()
bf = part[base + 512:base + 1024].view(64, 8).cpu()
acc = part[base + 1024:base + 2048].view(64, 16).cpu()
print("bf all ones:", bool((bf == 1).all()))
A = torch.zeros(32, 16); 
for l in range(64):
    for e in range(8):
        A[l % 32, 8 * (l // 32) + e] = af[l, e]
D = A @ torch.ones(16, 32)
for l in [0, 1, 33]:
    print("lane", l, "acc r0..3", acc[l, :4].tolist(), "expect", [D[(r & 3) + 8 * (r >> 2) + 4 * (l // 32), l % 32].item() for r in range(4)])
