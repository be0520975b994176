#!/bin/bash
# Same-box training-step time (bench.py --train, fp32 unless PREC=f16) of libsgn_hip.so variants
# (SGN_HIP_LIB=) against the in-tree build, interleaved.  Usage (GPU box):
#   bash tools/train_variants_ab.sh <tag> a.so b.so ...   [env: REPS (2), PREC (f32), STEPS (40), EXTRA_ENV]
set -u
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-2}); do
  for v in base "$@"; do
    n=$(basename $v .so)
    lib=sg-nerf_amd/libsgn_hip.so; [ $v != base ] && lib=$v
    env ${EXTRA_ENV:-} SGN_HIP_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 200 python bench.py --train --train-precision ${PREC:-f32} \
        --steps ${STEPS:-40} --warmup 5 > gpurun_out/tab_${TAG}_$n$rep.json 2> gpurun_out/tab_${TAG}_$n$rep.err \
        || { echo "FAIL $v"; tail -5 gpurun_out/tab_${TAG}_$n$rep.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/tab_${TAG}_$n$rep.json')); print('$n', round(d['ms_per_step'],3), 'ms/step', 'loss', round(d['final_loss'],6))"
  done
done
echo TAB_DONE
