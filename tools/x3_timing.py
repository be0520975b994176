"""Reads the SGN_X3_TIMING stamp dump of k_agg_rows_x3 (SGN_X3_TDBG=<file>) and prints the
median cycles of each phase of a work tile beside its MFMA-only ideal (3 x 32 cycles per
fragment pair).  Usage: python tools/x3_timing.py <dump> [TD_BLOCKS NW TD_EV]"""
import sys

import numpy as np

path = sys.argv[1]
TB, NW, EV = (int(x) for x in sys.argv[2:5]) if len(sys.argv) > 4 else (8, 4, 2048)
d = np.fromfile(path, dtype=np.uint64).reshape(TB, NW, EV).astype(np.int64)
# stamps per tile (base viewmlp): see k_agg_rows_x3
labels = ["tile start -> gather+PE issued", "gather -> L0 chunk entered (vmcnt + barrier)",
          "L0 chunk (32 pairs) + L0 epilogue (8 tiles)", "L0 epi -> L1P0C0 entered",
          "L1P0C0 (32 pairs)", "L1P0C1 (32) + epi", "-> L1P1C0 entered", "L1P1C0 (32)", "L1P1C1 (32) + epi",
          "-> L2P0C0 entered", "L2P0C0 (24)", "L2P0C1 (24)", "L2P0C2 (20) + epi", "-> L2P1C0 entered",
          "L2P1C0 (24)", "L2P1C1 (24)", "L2P1C2 (20) + epi", "-> L3P0C0 entered", "L3P0C0 (32)",
          "L3P0C1 (32) + l3 epilogue 0", "-> L3P1C0 entered (+fs flush 0 after)", "L3P1C0 (32)",
          "L3P1C1 (32) + l3 epilogue 1 + flush", "alpha reduction + feat write", "loop back -> next tile start"]
pairs = [0, 0, 32, 0, 32, 32, 0, 32, 32, 0, 24, 24, 20, 0, 24, 24, 20, 0, 32, 32, 0, 32, 32, 0, 0]
M = len(labels)
rows = []
for b in range(TB):
    for w in range(NW):
        s = d[b, w]
        n = int(np.count_nonzero(s))
        s = s[:n]
        nt = (n - 1) // M
        if nt < 2:
            continue
        t = s[: nt * M + 1]
        dif = np.diff(t)[: nt * M].reshape(nt, M)
        rows.append(dif[1:])  # drop the first tile (cold)
if not rows:
    sys.exit("no stamps")
a = np.concatenate(rows)
med = np.median(a, axis=0)
tot = med.sum()
ideal = sum(pairs) * 96
print(f"tiles {a.shape[0]}; median cycles per tile {tot:.0f} (MFMA-only ideal {ideal}, {ideal / tot:.1%})")
for i in range(M):
    ide = pairs[i] * 96
    print(f"  {i:2d} {labels[i]:48s} {med[i]:8.0f}   ideal {ide:5d}   over {med[i] - ide:7.0f}")
