#!/bin/bash
# PMC passes (one rocprofv3 run per counter group, no tracing domains mixed in) for the
# dominant kernels of bench.py.  Usage (on the GPU box):  bash tools/profile_pmc.sh <outdir> [bench args]
set -e
OUT=${1:-gpurun_out/pmc}
shift || true
ARGS=${@:---steps 2 --warmup 1 --no-cpu-baseline --no-extras}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
i=0
for grp in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
  "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES SQ_IFETCH" \
  "FETCH_SIZE TCC_HIT_sum" \
  "WRITE_SIZE TCC_MISS_sum" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "${KREGEX:-k_agg_rows|k_rows16|k_point_proj|k_knn|k_march|k_color|k_composite}" \
      -d "$OUT/p$i" -o pmc --output-format csv -- python bench.py $ARGS > "$OUT/p$i.log" 2>&1
done
echo PMC_DONE
