"""Chunk-boundary timing trace of a SGN_TIMING build (mlp.hip tmark): median cycles per stream
chunk per work tile.  Usage: python tools/tdbg.py gpurun_out/tdbg.bin [chunks_per_tile]"""
import sys

import numpy as np

t = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(4, 8, 512).astype(np.int64)
NC = int(sys.argv[2]) if len(sys.argv) > 2 else 15
for b in range(2):
    w0 = t[b, 0]
    n = int((w0 > 0).sum())
    d = np.diff(w0[:n])
    items = (n - 1) // NC
    arr = d[:items * NC].reshape(items, NC)
    print(f"block {b}: {items} tiles, median cycles per chunk:", np.median(arr, axis=0).astype(int).tolist(),
          "tile total", int(np.median(arr.sum(1))))
n = int((t[0, 0] > 0).sum())
sk = t[0, :, :n].max(0) - t[0, :, :n].min(0)
print("barrier exit skew across waves: median", float(np.median(sk)), "max", int(sk.max()))
