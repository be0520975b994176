"""Reads the stamp dump of a tools/x3_variant.py 'timing2' build (k_rows16 NS = 2: 8 stamps per tile at
the layer boundaries): median cycles per layer of a tile against the MFMA-only time, and the in-kernel
clock.  Usage: python tools/x3_timing2.py <dump>"""
import sys

import numpy as np

TB, NW, EV, PER = 8, 4, 2048, 8
d = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(TB, NW, EV).astype(np.int64)
labels = ["tile start: indices, records, row math", "block1.0 (2 chunks, PE(dists))", "block1.2 (8 chunks)",
          "block3.0 (9 chunks)", "block3.2 pass 0 (4 chunks)", "block3.2 pass 1 (4 chunks, epilogue half)",
          "epilogue rest, P loads, f_s, alpha", "loop back"]
ideal = [0, 2 * 1536, 8 * 1536, 9 * 1536, 4 * 1536, 4 * 1536, 0, 0]
rows, clocks = [], []
for b in range(TB):
    for w in range(NW):
        s = d[b, w]
        t0, r0, t1, r1 = s[EV - 4:]
        if r1 > r0:
            clocks.append((t1 - t0) / (r1 - r0) * 100.0)
        nt = (EV - 4) // PER
        for it in range(nt - 1):
            a = list(s[it * PER:(it + 1) * PER]) + [s[(it + 1) * PER]]
            if min(a) <= 0:
                continue
            rows.append(np.diff(a))
a = np.array(rows)
med = np.median(a, axis=0)
print(f"tiles {a.shape[0]}; median cycles per tile {med.sum():.0f}; MFMA-only {sum(ideal)} ({sum(ideal) / med.sum():.1%})")
for i, lab in enumerate(labels):
    print(f"  {lab:44s} {med[i]:8.0f}   MFMA-only {ideal[i]:6d}" + (f"  ({ideal[i] / med[i]:.0%})" if ideal[i] else ""))
if clocks:
    print(f"in-kernel clock (median over {len(clocks)} waves): {np.median(clocks):.0f} MHz")
