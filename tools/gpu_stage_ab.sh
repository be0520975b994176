#!/bin/bash
# One GPU call (NOT product): a subset of the -m gpu suite on the in-tree library, then the config-2
# per-stage timing (tools/agg_time.py) of the in-tree library and of variant builds, interleaved.
# Usage (GPU box): bash tools/gpu_stage_ab.sh <tag> "<pytest -k expr>" "<variant.so ...>" [prec=f32] [reps=3]
set -u
TAG=$1; KEXPR=$2; VARS=$3; PREC=${4:-f32}; REPS=${5:-3}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$KEXPR" \
    > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -2 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
for i in $(seq 1 $REPS); do
  for v in intree $VARS; do
    lib=$GRAFT_REPO_ROOT/sg-nerf_amd/libsgn_hip.so; [ $v != intree ] && lib=$GRAFT_REPO_ROOT/$v
    SGN_VARIANT=$(basename $v .so) SGN_HIP_LIB=$lib timeout -k 10 300 python tools/agg_time.py $PREC 8 \
        >> gpurun_out/stage_$TAG.jsonl 2> gpurun_out/stage_$TAG.err || { tail -5 gpurun_out/stage_$TAG.err; exit 1; }
    tail -1 gpurun_out/stage_$TAG.jsonl
  done
done
