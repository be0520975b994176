#!/bin/bash
# One GPU call: the training GPU tests, then config-5 training steps at both precisions (bench.py
# --train).  Usage (GPU box): bash tools/gpu_train_check.sh <tag> [pytest -k expr]
set -u
TAG=$1; KEXPR=${2:-}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_train_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread \
    ${KEXPR:+-k "$KEXPR"} > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
for P in f32 f16; do
  timeout -k 10 300 python bench.py --train --train-precision $P --steps 30 --warmup 5 --no-cpu-baseline \
      > gpurun_out/train_${P}_$TAG.json 2> gpurun_out/train_${P}_$TAG.err || { tail -5 gpurun_out/train_${P}_$TAG.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/train_${P}_$TAG.json')); print('$P', round(d['ms_per_step'],3), d['final_loss'])"
done
