#!/bin/bash
# One GPU call (NOT product): the training GPU tests on the in-tree library, then config-5 steps of
# the in-tree library and of a variant build (SGN_HIP_LIB), interleaved, at the given precisions.
# Usage (GPU box): bash tools/gpu_train_ab.sh <tag> "<variant.so ...>" [precisions="f32 f16"] [reps=2]
set -u
TAG=$1; VARS=$2; PRECS=${3:-f32 f16}; REPS=${4:-2}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_train_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -2 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
for P in $PRECS; do
  for i in $(seq 1 $REPS); do
    for v in intree $VARS; do
      lib=$GRAFT_REPO_ROOT/sg-nerf_amd/libsgn_hip.so; [ $v != intree ] && lib=$GRAFT_REPO_ROOT/$v
      b=$(basename $v .so)
      SGN_HIP_LIB=$lib timeout -k 10 300 python bench.py --train --train-precision $P --steps 30 --warmup 5 \
          --no-cpu-baseline > gpurun_out/tab_${TAG}_$P${b}_$i.json 2> gpurun_out/tab_$TAG.err || { tail -5 gpurun_out/tab_$TAG.err; exit 1; }
      python -c "import json; d=json.load(open('gpurun_out/tab_${TAG}_$P${b}_$i.json')); print('$P $b', round(d['ms_per_step'],3))"
    done
  done
done
