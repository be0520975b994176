"""Summarise rocprofv3 --pmc CSVs (tools/profile_pmc.sh) per kernel: mean counter value per
dispatch, plus derived MFMA utilisation and HBM bytes (FETCH_SIZE doubled for the gfx950
wide-read under-count, MI355X_MICROARCH.md §HBM)."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def load(outdir):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(outdir, "p*", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            m = re.search(r"(k_[a-z0-9_]+)", row["Kernel_Name"])
            k = m.group(1) if m else row["Kernel_Name"][:40]
            acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def derive(c):
    d = {}
    if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "GRBM_GUI_ACTIVE" in c:
        # MFMA busy cycles are summed over all SIMDs (1024); GUI_ACTIVE over 8 XCDs
        simd_cycles = c["GRBM_GUI_ACTIVE"] / 8 * 1024
        d["mfma_busy_frac"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cycles if simd_cycles else None
    if "FETCH_SIZE" in c:
        d["hbm_read_bytes_corrected"] = c["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in c:
        d["hbm_write_bytes"] = c["WRITE_SIZE"] * 1024
    if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c and (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]) > 0:
        d["l2_hit_rate"] = c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"]:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in c:
                d[k.lower() + "_frac"] = c[k] / c["SQ_WAVE_CYCLES"]
    return d


if __name__ == "__main__":
    res = load(sys.argv[1])
    out = {k: {"counters": v, "derived": derive(v)} for k, v in res.items()}
    print(json.dumps(out, indent=1))
