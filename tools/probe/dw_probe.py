import ctypes, torch
lib = ctypes.CDLL("./tools/probe/dw_probe.so")
dev = "cuda:0"
rows, ncols = 32, 256
d = torch.zeros(rows, 256, dtype=torch.float16, device=dev)
for r in range(rows):
    d[r] = torch.arange(256, device=dev).to(torch.float32).remainder(64).to(torch.float16) + 64 * (r % 16)  # d[r][m] = m%64 + 64 (r%16)
x = torch.ones(rows, ncols, dtype=torch.float16, device=dev)
part = torch.zeros(256 * ncols + 4096, device=dev)
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
lib.probe_f16_weight_grad.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                      ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]
print(lib.probe_f16_weight_grad(d.data_ptr(), 256, x.data_ptr(), ncols, ncols, rows, 1, part.data_ptr(), st))
torch.cuda.synchronize()
f = part[256 * ncols:256 * ncols + 512].view(64, 8).cpu()
a0 = part[256 * ncols + 512:256 * ncols + 768].view(64, 4).cpu()
for l in [0, 1, 2, 3, 4, 5, 15, 16, 17, 31, 32, 33]:
    print(l, "af (col, row):", [(int(v) % 64, int(v) // 64) for v in f[l].tolist()], "a0", [(int(v) % 64, int(v) // 64) for v in a0[l].tolist()])
got = part[:256 * ncols].view(256, ncols).cpu().double()
ref = (d.double().t() @ x.double()).cpu()
print("max err", float((got - ref).abs().max()), "got[0:4,0]", got[0:4, 0].tolist(), "ref", ref[0:4, 0].tolist())
