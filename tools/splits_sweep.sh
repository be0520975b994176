#!/bin/bash
# fp32 training step time against the split-K partial counts of its weight-gradient GEMMs
# (SGN_SPLITS_ROWS / SGN_SPLITS_ITEMS), alternated on one box.  Usage (GPU box): bash tools/splits_sweep.sh
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2; do
  for cfg in "84 128" "84 256" "84 64" "168 128" "42 128"; do
    set -- $cfg
    SGN_SPLITS_ROWS=$1 SGN_SPLITS_ITEMS=$2 timeout -k 10 200 python bench.py --train --steps 40 --warmup 5 \
        > gpurun_out/sp.json 2> gpurun_out/sp.err || { tail -5 gpurun_out/sp.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/sp.json')); print('rows $1 items $2', round(d['ms_per_step'], 3))"
  done
done
