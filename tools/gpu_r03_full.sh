#!/bin/bash
# One GPU call for the round's evidence: all GPU tests, smoke, the default bench line, kernel-trace
# stats + PMC passes of the f32 headline, lego / SG lines, training kernel traces (f32 and f16).
# Usage (GPU box): bash tools/gpu_r03_full.sh <tag>
set -u
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
grep -E "FAILED|ERROR" gpurun_out/pytest_$TAG.log | head -20; tail -1 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo PYTEST_ABORT rc=$rc; exit 1; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke_$TAG.log; exit 1; }
tail -2 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
echo BENCH_OK
bash tools/prof_x3.sh $TAG || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --scene lego > gpurun_out/benchlego_$TAG.json 2> gpurun_out/benchlego_$TAG.err || { echo LEGO_FAIL; tail gpurun_out/benchlego_$TAG.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --sg > gpurun_out/benchsg_$TAG.json 2> gpurun_out/benchsg_$TAG.err || { echo SG_FAIL; tail gpurun_out/benchsg_$TAG.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/proftrain_$TAG -o run --output-format csv -- \
    python bench.py --train --steps 20 --warmup 5 > gpurun_out/proftrain_$TAG.json 2> gpurun_out/proftrain_$TAG.err || { echo TRAINPROF_FAIL; tail gpurun_out/proftrain_$TAG.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/proftrain16_$TAG -o run --output-format csv -- \
    python bench.py --train --train-precision f16 --steps 20 --warmup 5 > gpurun_out/proftrain16_$TAG.json 2> gpurun_out/proftrain16_$TAG.err || { echo TRAIN16PROF_FAIL; tail gpurun_out/proftrain16_$TAG.err; exit 1; }
echo GPU_R03_FULL_DONE pytest_rc=$rc
