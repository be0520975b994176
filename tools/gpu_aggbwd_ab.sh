#!/bin/bash
# One GPU call (NOT product): the training GPU tests on the in-tree library, then the k_agg_bwd
# replay A/B (tools/agg_bwd_ab.py) against the given variant builds, base and SG, then the f16
# training step of the in-tree library and of the first variant.
# Usage (GPU box): bash tools/gpu_aggbwd_ab.sh <tag> variant.so ...
set -u
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/agg_bwd_ab.py "$@" > gpurun_out/aggab_$TAG.jsonl 2> gpurun_out/aggab_$TAG.err || { tail -5 gpurun_out/aggab_$TAG.err; exit 1; }
cat gpurun_out/aggab_$TAG.jsonl
timeout -k 10 300 python -u tools/agg_bwd_ab.py --sg "$@" > gpurun_out/aggab_sg_$TAG.jsonl 2> gpurun_out/aggab_sg_$TAG.err || { tail -5 gpurun_out/aggab_sg_$TAG.err; exit 1; }
cat gpurun_out/aggab_sg_$TAG.jsonl
for v in intree "$1"; do
  lib=sg-nerf_amd/libsgn_hip.so; [ $v != intree ] && lib=$v
  SGN_HIP_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 200 python bench.py --train --train-precision f16 --steps 30 --warmup 5 \
      --no-cpu-baseline > gpurun_out/abt_${TAG}_$(basename $v).json 2> gpurun_out/abt_$TAG.err || { tail -5 gpurun_out/abt_$TAG.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/abt_${TAG}_$(basename $v).json')); print('$v', round(d['ms_per_step'],3))"
done
