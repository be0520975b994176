#!/bin/bash
# f16 training step time against the split-K batch of its weight-gradient GEMMs (SGN_DW_CHUNK),
# alternated on one box.  Usage (GPU box): bash tools/dw_chunk_sweep.sh [chunks]
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2; do
  for c in ${1:-1024 2048 4096}; do
    SGN_DW_CHUNK=$c timeout -k 10 200 python bench.py --train --train-precision f16 --steps 40 --warmup 5 \
        > gpurun_out/dw_$c.json 2> gpurun_out/dw_$c.err || { tail -5 gpurun_out/dw_$c.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/dw_$c.json')); print('chunk $c', round(d['ms_per_step'], 3))"
  done
done
