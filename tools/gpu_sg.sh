#!/bin/bash
# GPU call: full GPU test suite, base bench, SG bench.
set -u
TAG=${1:-sg}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_$TAG.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error|error|assert" gpurun_out/pytest_$TAG.log | head -30; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_$TAG.log
grep -E "max \|" gpurun_out/pytest_$TAG.log | head -40
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 300 python bench.py --no-cpu-baseline --sg > gpurun_out/benchsg_$TAG.json 2> gpurun_out/benchsg_$TAG.err || { echo BENCHSG_FAIL; tail -30 gpurun_out/benchsg_$TAG.err; exit 1; }
cat gpurun_out/benchsg_$TAG.json
echo GPU_SG_DONE
