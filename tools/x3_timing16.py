"""SGN_X3_TIMING dump of k_rows16 (8 waves): median cycles per phase of a work tile.
Usage: python tools/x3_timing16.py <dump>"""
import sys

import numpy as np

TB, NW, EV = 8, 8, 2048
d = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(TB, NW, EV).astype(np.int64)
labels = ["tile start -> gather + PE", "-> L0 chunk entered", "L0 (32 pairs) + P add", "L1C0 (32)", "L1C1", "L1C2",
          "L1C3", "L2C0 (32)", "L2C1", "L2C2", "L2C3", "L2C4 (16)", "L3C0 (32)", "L3C1", "L3C2", "L3C3 -> MFMAs issued",
          "-> block3.2 epilogue done", "f_s + alpha -> tile end", "loop back -> tile start"]
pairs = [0, 0, 32, 32, 32, 32, 32, 32, 32, 32, 32, 16, 32, 32, 32, 32, 0, 0, 0]
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
ideal = sum(pairs) * 48 * 2  # 3 MFMAs x 16 cycles per pair, two waves share a SIMD
print(f"tiles {a.shape[0]}; median cycles per tile {med.sum():.0f} (MFMA-only ideal per SIMD {ideal}, {ideal / med.sum():.1%})")
for i in range(M):
    print(f"  {i:2d} {labels[i]:34s} {med[i]:8.0f}   SIMD-ideal {pairs[i] * 96:5d}")
if clocks:
    print(f"in-kernel clock (s_memtime / s_memrealtime, median over {len(clocks)} waves): {np.median(clocks):.0f} MHz")
