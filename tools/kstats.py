"""Per-step kernel table of a rocprofv3 kernel-stats CSV with short kernel names (template args kept).
Usage: python tools/kstats.py <kernel_stats.csv> [steps] [top]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 25
top = int(sys.argv[3]) if len(sys.argv) > 3 else 20
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:top]:
    n = r["Name"]
    m = re.search(r"(k_\w+)(<[^(]*?>)?\(", n)
    name = m.group(1) + (m.group(2) or "") if m else re.sub(r"\(.*", "", n)[:70]
    print(f"{int(r['Calls']) / steps:6.2f} {float(r['TotalDurationNs']) / steps / 1e3:8.1f}us "
          f"{float(r['AverageNs']) / 1e3:8.1f}  {name}")
