#!/bin/bash
# The final tree's PMC passes of the headline bench (one rocprofv3 --pmc run per counter group,
# tools/profile_pmc.sh), their per-kernel summary, and the kernel stats of the same tree, so
# profiles/traffic_*.json can be regenerated from them (tools/traffic_json.py).
# Usage (GPU box): bash tools/gpu_pmc_final.sh <tag>
set -eu
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/profile_pmc.sh gpurun_out/pmc_$TAG > gpurun_out/pmc_$TAG.log 2>&1
python tools/pmc_summary.py gpurun_out/pmc_$TAG > gpurun_out/pmc_summary_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kst_$TAG -o run --output-format csv -- \
    python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras > gpurun_out/kst_$TAG.json 2> gpurun_out/kst_$TAG.err
echo PMC_FINAL_DONE
