"""Per-step summary of a training kernel-stats CSV (rocprofv3 --stats): launches and time per step,
HIP-authored share, small-kernel glue.  Usage: python tools/train_stats.py <kernel_stats.csv> [steps]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 25
tot = sum(float(r["TotalDurationNs"]) for r in rows)
hip = sum(float(r["TotalDurationNs"]) for r in rows if "sgn::" in r["Name"])
glue = [r for r in rows if re.search(r"FillFunctor|copyBuffer|fillBuffer|direct_copy|_copy_kernel", r["Name"])]
print(f"per step: {tot / steps / 1e6:.3f} ms kernel time, {sum(int(r['Calls']) for r in rows) / steps:.1f} launches, "
      f"HIP-authored {hip / tot:.3f}, fills+copies {sum(int(r['Calls']) for r in glue) / steps:.1f} "
      f"({sum(float(r['TotalDurationNs']) for r in glue) / steps / 1e3:.1f} us)")
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:int(sys.argv[3]) if len(sys.argv) > 3 else 40]:
    n = re.sub(r"\(.*", "", r["Name"])
    n = n[:60] if n.startswith("Cijk") else n[:100]
    print(f'{int(r["Calls"]) / steps:6.2f} {float(r["TotalDurationNs"]) / steps / 1e3:8.1f}us {float(r["AverageNs"]) / 1e3:7.1f}  {n}')
