#!/bin/bash
# Training-glue check 2: query / training / loss GPU tests, f16 + f32 training lines, f16 training kernel trace.
set -u
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_query_gpu.py tests/test_train_gpu.py tests/test_loss_gpu.py -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
grep -E "FAILED|ERROR" gpurun_out/pytest_$TAG.log | head -20; tail -1 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ]; then echo PYTEST_FAIL rc=$rc; exit 1; fi
for p in f16 f32; do
  timeout -k 10 300 python bench.py --train --train-precision $p --steps 30 --warmup 5 > gpurun_out/train${p}_$TAG.json 2> gpurun_out/train${p}_$TAG.err || { echo TRAIN_FAIL $p; tail -30 gpurun_out/train${p}_$TAG.err; exit 1; }
  cut -c1-250 gpurun_out/train${p}_$TAG.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/proftrain16_$TAG -o run --output-format csv -- \
    python bench.py --train --train-precision f16 --steps 20 --warmup 5 > gpurun_out/proftrain16_$TAG.json 2> gpurun_out/proftrain16_$TAG.err || { echo TRAIN16PROF_FAIL; tail gpurun_out/proftrain16_$TAG.err; exit 1; }
echo GPU_R03H_DONE
