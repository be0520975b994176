#!/bin/bash
# PMC passes of k_rows16 for the row-set variants (SGN_ROWS_NS 1 / 2), summarised per variant.
# Usage (GPU box): bash tools/pmc_ns.sh <tag> [ns list]
set -e
TAG=$1
for ns in ${2:-1 2}; do
    SGN_ROWS_NS=$ns KREGEX=k_rows16 bash tools/profile_pmc.sh gpurun_out/pmc_${TAG}_ns$ns > /dev/null
    python tools/pmc_summary.py gpurun_out/pmc_${TAG}_ns$ns > gpurun_out/pmc_${TAG}_ns$ns.json
    python - <<PY
import json
d = json.load(open("gpurun_out/pmc_${TAG}_ns$ns.json"))
for k, v in d.items():
    c, dv = v["counters"], v["derived"]
    w = c["SQ_WAVE_CYCLES"]
    print("NS=$ns", k, "mfma_busy %.3f" % dv["mfma_busy_frac"], "wait_any %.3f" % (c["SQ_WAIT_ANY"] / w),
          "wait_inst %.3f" % (c["SQ_WAIT_INST_ANY"] / w), "active %.3f" % (c["SQ_ACTIVE_INST_ANY"] / w),
          "valu/mfma %.2f" % (c["SQ_INSTS_VALU"] / c["SQ_INSTS_MFMA"]), "lds/mfma %.2f" % (c["SQ_INSTS_LDS"] / c["SQ_INSTS_MFMA"]),
          "lds_conf %.3g" % c["SQ_LDS_BANK_CONFLICT"], "wait_lds %.3f" % (c["SQ_WAIT_INST_LDS"] / w),
          "hbm_rd %.3g" % dv["hbm_read_bytes_corrected"])
PY
done
