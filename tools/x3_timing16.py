"""SGN_X3_TIMING dump of k_rows16 (8 waves): median cycles per phase of a work tile.
Usage: python tools/x3_timing16.py <dump> [waves per workgroup: 4 (default) or 8]"""
import sys

import numpy as np

EV = 2048
RW = int(sys.argv[2]) if len(sys.argv) > 2 else 4
RING = len(sys.argv) > 3 and sys.argv[3] == "ring"   # SGN_X3_RING: 8 waves, 16-pair chunks
TB, NW = (8, 8) if RW == 8 else (16, 4)   # the stamp buffer holds 64 waves (mlp_x3.hip TD_BLOCKS x NW16)
d = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(TB, NW, EV).astype(np.int64)
if RW == 8 and not RING:   # 32-pair chunks: L0 1, L1 4, L2 4 + 1 of 16, L3 4
    ch = [("L0", 32)] + [(f"L1C{c}", 32) for c in range(4)] + [(f"L2C{c}", 32 if c < 4 else 16) for c in range(5)] + \
         [(f"L3C{c}", 32) for c in range(4)]
else:         # 16-pair chunks: L0 2, L1 8, L2 9, L3 2 passes x 4
    ch = [(f"L0C{c}", 16) for c in range(2)] + [(f"L1C{c}", 16) for c in range(8)] + [(f"L2C{c}", 16) for c in range(9)] + \
         [(f"L3P{c // 4}C{c % 4}", 16) for c in range(8)]
labels = ["tile start -> gather + PE", "-> L0 chunk entered"] + [n for n, _ in ch[:-1]] + \
         [ch[-1][0] + " -> MFMAs issued", "-> block3.2 epilogue done", "f_s + alpha -> tile end",
                                 "loop back -> tile start"]
pairs = [0, 0] + [p for _, p in ch] + [0, 0, 0]
M = len(labels)
rows = []
clocks = []
for b in range(TB):
    for w in range(NW):
        s = d[b, w][:EV - 4]
        s = s[:int(np.count_nonzero(s))]
        t0, r0, t1, r1 = d[b, w][EV - 4:]
        if r1 > r0:
            clocks.append((t1 - t0) / (r1 - r0) * 100.0)  # MHz (s_memrealtime ticks at 100 MHz)
        nt = (len(s) - 1) // M
        if nt < 3:
            continue
        rows.append(np.diff(s[: nt * M + 1])[: nt * M].reshape(nt, M)[1:])
a = np.concatenate(rows)
med = np.median(a, axis=0)
labels = labels[:len(pairs)]
ideal = sum(pairs) * 48 * 2  # 3 MFMAs x 16 cycles per pair, two waves share a SIMD
print(f"tiles {a.shape[0]}; median cycles per tile {med.sum():.0f} (MFMA-only ideal per SIMD {ideal}, {ideal / med.sum():.1%})")
for i in range(M):
    print(f"  {i:2d} {labels[i]:34s} {med[i]:8.0f}   SIMD-ideal {pairs[i] * 96:5d}")
if clocks:
    print(f"in-kernel clock (s_memtime / s_memrealtime, median over {len(clocks)} waves): {np.median(clocks):.0f} MHz")
