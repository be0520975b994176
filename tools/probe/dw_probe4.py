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
acc = part[base:base + 1024].view(64, 16).cpu()
got = part[:base].view(256, ncols).cpu()
for l in [0, 1, 33]:
    print("lane", l, "final acc r0..3", acc[l, :4].tolist(), "stored", [got[(r & 3) + 4 * (l // 32), l % 32].item() for r in range(4)])
