"""Write profiles/traffic_latest.json (k_rows16) and profiles/traffic_query_latest.json (k_knn27,
k_march) from a PMC summary of the headline workload (tools/pmc_summary.py output) and the kernel
stats of the same tree (rocprofv3 --kernel-trace --stats).  bench.py reads them into
roofline.traffic and roofline_query.counter.
Usage: python tools/traffic_json.py <pmc_summary.json> <kernel_stats.csv> <tag>"""
import csv
import json
import os
import re
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
pmc = json.load(open(sys.argv[1]))
avg = {}
for row in csv.DictReader(open(sys.argv[2])):
    m = re.search(r"(k_[a-z0-9_]+)", row["Name"])
    if m:
        k = m.group(1)
        avg[k] = avg.get(k, 0.0) + float(row["TotalDurationNs"]) / max(float(row["Calls"]), 1.0) / 1e6
tag = sys.argv[3]
src = f"profiles/{tag}_pmc_summary.json (tools/profile_pmc.sh: FETCH_SIZE x2 per the gfx950 note + WRITE_SIZE, per launch)"
r = pmc["k_rows16"]["derived"]
rows = {"kernel": "k_rows16", "workload_key": "800x800x64",
        "bytes_per_launch": r["hbm_read_bytes_corrected"] + r["hbm_write_bytes"],
        "read_bytes_corrected": r["hbm_read_bytes_corrected"], "write_bytes": r["hbm_write_bytes"],
        "source": src,
        "note": "reads: the per-row P gathers (1 KiB fp32 per (sample, neighbour) row) and the packed point "
                "records; writes: the fp32 blended features (1 KiB per valid sample) read by k_color16"}
json.dump(rows, open(os.path.join(ROOT, "profiles", "traffic_latest.json"), "w"), indent=1)
ks = {}
for k in ("k_knn27", "k_march"):
    if k in pmc:
        d = pmc[k]["derived"]
        b = d["hbm_read_bytes_corrected"] + d["hbm_write_bytes"]
        ks[k] = {"bytes_per_launch": b, "l2_hit_rate": d.get("l2_hit_rate"), "avg_launch_ms": avg.get(k),
                 "counter_GBps": b / (avg[k] * 1e-3) / 1e9 if avg.get(k) else None}
q = {"workload_key": "800x800x64", "source": src + f" and profiles/{tag}_kernel_stats.csv (average durations)",
     "kernels": ks}
json.dump(q, open(os.path.join(ROOT, "profiles", "traffic_query_latest.json"), "w"), indent=1)
print(json.dumps(rows, indent=1))
print(json.dumps(q, indent=1))
