#!/bin/bash
# Row-kernel change check (GPU box): render + API parity (product NS), the fp32 training
# gradients (save mode), then the NS A/B of tools/gpu_ns.sh.  Usage: bash tools/gpu_rows.sh <tag>
set -u
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_render_gpu.py tests/test_api_gpu.py tests/test_train_gpu.py -x -v --timeout 200 \
    --timeout-method thread -k "not (200_step or lower_loss or plugin or ranks_frames or graph or colsum or adam or pack)" \
    > gpurun_out/pytest_rows_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_rows_$TAG.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_ns.sh $TAG
