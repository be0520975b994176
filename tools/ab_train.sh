#!/bin/bash
# A/B of the training bench in one call: abtree/ (variant A) vs the tree root (B), alternated.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2; do
  for v in A B; do
    d=.; [ $v = A ] && d=abtree
    (cd $d && timeout -k 10 200 python bench.py --train --steps 40 "$@" > $GRAFT_REPO_ROOT/gpurun_out/ab_tmp.json 2> $GRAFT_REPO_ROOT/gpurun_out/ab_$v.err) \
      || { echo "FAIL $v"; tail -20 gpurun_out/ab_$v.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_tmp.json')); print(sys.argv[1], round(d['value']), round(d['ms_per_step'],3))" $v
  done
done
