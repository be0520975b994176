"""Steady-state per-step view of a training kernel trace (rocprofv3 --kernel-trace, csv): the steps
are cut at their first launch (k_depth_jitter, the query's jittered depth table: one per step), the
last `n` complete steps averaged -- no setup, grid build or graph capture in the numbers.
Usage: python tools/step_window.py <run_kernel_trace.csv> [n=20] [top=30]"""
import collections
import csv
import re
import sys

kt = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
starts = [i for i, r in enumerate(kt) if "k_depth_jitter" in r["Kernel_Name"]]
last = max(i for i, r in enumerate(kt) if "k_adam" in r["Kernel_Name"])
cuts = [i - 1 for i in starts] + [last]   # window (a, b]: from a step's first launch to the next's
pairs = list(zip(cuts[:-1], cuts[1:]))[-n:]
tot = collections.Counter()
calls = collections.Counter()
wall = busy = hip = 0
glue = 0
for a, b in pairs:
    wall += int(kt[b]["End_Timestamp"]) - int(kt[a]["End_Timestamp"])
    for r in kt[a + 1:b + 1]:
        nm = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", ""))
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        busy += d
        hip += d if "sgn::" in r["Kernel_Name"] else 0
        glue += bool(re.search(r"FillFunctor|copyBuffer|fillBuffer|direct_copy|_copy_kernel", nm))
        tot[nm[:90]] += d
        calls[nm[:90]] += 1
k = len(pairs)
print(f"{k} steps: wall {wall / k / 1e6:.3f} ms/step, kernels {busy / k / 1e6:.3f} ms, "
      f"{sum(calls.values()) / k:.1f} launches, HIP-authored {hip / busy:.3f}, fills+copies {glue / k:.1f}")
for nm, t in tot.most_common(top):
    print(f"{calls[nm] / k:6.2f} {t / k / 1e3:8.1f}us  {nm}")
