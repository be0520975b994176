#!/bin/bash
# Same-box f16 training-step A/B (GPU box): the HEAD copy in ab_head/ (its own built library) against
# this tree, and this tree with the rows GEMMs' bpack off (tools/train_nobpack.py).  Usage: bash tools/f16_ab.sh <tag>
set -u
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ARGS="--train --train-precision ${PREC:-f16} --steps ${STEPS:-60} --warmup 5"
for rep in $(seq 1 ${REPS:-2}); do
  for v in head new nobp; do
    out=gpurun_out/fab_${TAG}_$v$rep
    case $v in
      head) (cd ab_head && timeout -k 10 200 python bench.py $ARGS) > $out.json 2> $out.err ;;
      new) timeout -k 10 200 python bench.py $ARGS > $out.json 2> $out.err ;;
      nobp) timeout -k 10 200 python tools/train_nobpack.py $ARGS > $out.json 2> $out.err ;;
    esac
    rc=$?
    [ $rc -eq 0 ] || { echo "FAIL $v rc=$rc"; tail -5 $out.err; exit 1; }
    python -c "import json; d=json.load(open('$out.json')); print('$v', round(d['ms_per_step'],4), 'ms/step', 'loss', round(d['final_loss'],6))"
  done
done
echo FAB_DONE
