#!/bin/bash
# Same-box A/B of the training steps (config 5, fp32 and f16) between the round-4 tree (ab_r04/: git
# archive of f12802a with its own library built in place) and this tree, alternating, REPS rounds.
# Usage (GPU box): bash tools/ab_train_r04.sh <tag>
set -u
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=gpurun_out/abtr_$TAG.txt
: > $OUT
for rep in $(seq 1 ${REPS:-3}); do
  for prec in ${PRECS:-f32 f16}; do
    for v in r04 head; do
      f=gpurun_out/abtr_${TAG}_${v}_${prec}_$rep.json
      if [ $v = r04 ]; then
        (cd ab_r04 && timeout -k 10 200 python bench.py --train --train-precision $prec --steps ${STEPS:-100} --warmup 10) > $f 2> $f.err
      else
        timeout -k 10 200 python bench.py --train --train-precision $prec --steps ${STEPS:-100} --warmup 10 > $f 2> $f.err
      fi
      rc=$?
      [ $rc -eq 0 ] || { echo "FAIL $v $prec rc=$rc"; tail -5 $f.err; exit 1; }
      python -c "import json; d=json.load(open('$f')); print('$v', '$prec', round(d['ms_per_step'], 4), 'ms/step')" | tee -a $OUT
    done
  done
done
echo ABTR_DONE
