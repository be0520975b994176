#!/bin/bash
# One GPU call: GPU tests (all, not stopping at the first failure), smoke, and a short headline
# bench.  Usage (GPU box): bash tools/gpu_r03.sh <tag> [pytest -k expr]
set -u
TAG=${1:-chk}
K=${2:-}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
KARG=()
[ -n "$K" ] && KARG=(-k "$K")
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread "${KARG[@]}" \
    > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_$TAG.log | grep -v PASSED | head -40
tail -3 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo PYTEST_ABORT rc=$rc; exit 1; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke_$TAG.log; exit 1; }
tail -2 gpurun_out/smoke_$TAG.log
timeout -k 10 300 python bench.py --no-extras --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
echo GPU_R03_DONE pytest_rc=$rc
