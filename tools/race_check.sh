#!/bin/bash
# Determinism / parity probe of k_rows16 builds (GPU box): per library, the golden patch test and
# 20 repeated config-2 renders (bitwise comparison).  Usage: bash tools/race_check.sh lib...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for lib in "$@"; do
  for ns in 1 2; do
    echo "== $lib NS=$ns"
    SGN_ROWS_NS=$ns SGN_HIP_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 200 python -u -m pytest tests/test_render_gpu.py -q --timeout 200 \
        -k "golden and f32 and not sg" 2>&1 | grep -E "passed|failed|max \|rgb" | tail -3
    SGN_ROWS_NS=$ns SGN_HIP_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 200 python -u tools/render_repeat.py 12 2>&1 | tail -1 || exit 1
  done
done
