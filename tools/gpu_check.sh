#!/bin/bash
# One GPU call: the GPU test suite (one process), then the training bench and its kernel trace.
# Usage (GPU box): bash tools/gpu_check.sh <tag> [pytest -k expression]
set -u
TAG=$1
K=${2:-}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ -n "$K" ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "$K" > gpurun_out/pytest_$TAG.log 2>&1
else
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
fi
rc=$?
tail -5 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --train --steps 20 --warmup 5 > gpurun_out/train_$TAG.json 2> gpurun_out/train_$TAG.err || { tail -20 gpurun_out/train_$TAG.err; exit 1; }
cat gpurun_out/train_$TAG.json
bash tools/prof_train.sh $TAG --steps 20 --warmup 5 > /dev/null
