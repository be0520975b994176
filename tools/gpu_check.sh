#!/bin/bash
# One GPU call: GPU tests, smoke, bench (config 2) and the training bench (config 5).
# Usage (GPU box): bash tools/gpu_check.sh <tag>
set -u
TAG=${1:-chk}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_$TAG.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke_$TAG.log; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 300 python bench.py --train > gpurun_out/train_$TAG.json 2> gpurun_out/train_$TAG.err || { echo TRAIN_FAIL; tail -30 gpurun_out/train_$TAG.err; exit 1; }
cat gpurun_out/train_$TAG.json
echo GPU_CHECK_DONE
