#!/bin/bash
# PMC passes (tools/profile_pmc.sh: one rocprofv3 --pmc run per counter group) of the config-5 training
# steps' largest kernels at both precisions, and their per-kernel summaries (tools/pmc_summary.py).
# Usage (GPU box): bash tools/gpu_pmc_train.sh <tag>
set -eu
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export KREGEX="k_agg_bwd|k_f16dw|k_x3rows|k_x3dw|k_x3tn|k_adam|k_rows_update|k_rows_claim|k_rows16|k_agg_rows|k_row_inputs|k_row_head|k_row_tail"
for P in f16 f32; do
  bash tools/profile_pmc.sh gpurun_out/pmctr_${P}_$TAG --train --train-precision $P --steps 4 --warmup 2 --no-cpu-baseline \
      > gpurun_out/pmctr_${P}_$TAG.log 2>&1
  python tools/pmc_summary.py gpurun_out/pmctr_${P}_$TAG > gpurun_out/pmc_summary_train_${P}_$TAG.json
done
echo PMC_TRAIN_DONE
