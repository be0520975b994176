"""Reads the stamp dump of a tools/x3_variant.py 'timing' build (k_rows16, NS = 2, 4 waves): median
cycles per phase of a tile and the in-kernel clock.  Usage: python tools/x3_timing_ns2.py <dump>"""
import sys

import numpy as np

TB, NW, EV, PER = 8, 4, 2048, 32
d = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(TB, NW, EV).astype(np.int64)
# 16-pair chunks: block1.0 2, block1.2 8, block3.0 9, block3.2 2 passes x 4
ch = [f"L0C{c}" for c in range(2)] + [f"L1C{c}" for c in range(8)] + [f"L2C{c}" for c in range(9)] + \
     [f"L3P{c // 4}C{c % 4}" for c in range(8)]
# per tile: 29 start, 0..26 chunk entries, 27 block3.2 MFMAs done, 28 tile end, then the next 29
order = [29] + list(range(27)) + [27, 28]
labels = ["tile start -> L0C0 entered"] + [f"{c} (16 pairs)" for c in ch[:-1]] + \
         [ch[-1] + " -> MFMAs done (16 pairs)", "epilogue rest + epi_end", "loop back -> tile start"]
ideal = [0] + [16 * 3 * 2 * 16] * 26 + [16 * 3 * 2 * 16, 0, 0]   # 3 MFMAs x 2 row sets x 16 cycles per pair
rows, clocks = [], []
for b in range(TB):
    for w in range(NW):
        s = d[b, w]
        t0, r0, t1, r1 = s[EV - 4:]
        if r1 > r0:
            clocks.append((t1 - t0) / (r1 - r0) * 100.0)
        nt = (EV - 4) // PER
        for it in range(nt - 1):
            a = s[it * PER:(it + 1) * PER]
            nxt = s[(it + 1) * PER + 29]
            if not (a[order] > 0).all() or nxt == 0:
                continue
            seq = list(a[order]) + [nxt]
            rows.append(np.diff(seq))
a = np.array(rows)
if len(a) == 0:
    raise SystemExit("no complete tiles in the dump")
med = np.median(a, axis=0)
print(f"tiles {a.shape[0]}; median cycles per tile {med.sum():.0f}; MFMA-only ideal {sum(ideal)} "
      f"({sum(ideal) / med.sum():.1%})")
for i, lab in enumerate(labels):
    print(f"  {i:2d} {lab:34s} {med[i]:8.0f}   ideal {ideal[i]:5d}")
if clocks:
    print(f"in-kernel clock (s_memtime / s_memrealtime, median over {len(clocks)} waves): {np.median(clocks):.0f} MHz")
