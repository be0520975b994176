#!/bin/bash
# Kernel-time A/B of the f16 training step (GPU box; robust to host noise): rocprofv3 kernel traces of
# the HEAD copy in ab_head/, this tree, and this tree without bpack, each cut into steps by
# tools/step_window.py.  Usage: bash tools/f16_prof_ab.sh <tag>
set -u
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ARGS="--train --train-precision ${PREC:-f16} --steps ${STEPS:-40} --warmup 5"
R=$GRAFT_REPO_ROOT
for v in ${VARIANTS:-head new nobp}; do
  d=$R/gpurun_out/fprof_${TAG}_$v
  case $v in
    head) (cd ab_head && timeout -k 10 300 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- python bench.py $ARGS) > $d.json 2> $d.err ;;
    new) timeout -k 10 300 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- python bench.py $ARGS > $d.json 2> $d.err ;;
    *.so) SGN_HIP_LIB=$R/build/variants/$v timeout -k 10 300 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- python bench.py $ARGS > $d.json 2> $d.err ;;
    nobp) timeout -k 10 300 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- python tools/train_nobpack.py $ARGS > $d.json 2> $d.err ;;
  esac
  rc=$?
  [ $rc -eq 0 ] || { echo "FAIL $v rc=$rc"; tail -5 $d.err; exit 1; }
  f=$(find $d -name '*kernel_trace.csv' | head -1)
  echo "== $v"; python tools/step_window.py $f 20 12 | tee $d.window.txt
done
echo FPROF_DONE
