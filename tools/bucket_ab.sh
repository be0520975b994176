#!/bin/bash
# Training bench over loss-stage graph bucket sizes (SGN_GRAPH_BUCKET), alternated.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2; do
  for b in ${BUCKETS:-8192 4096 2048}; do
    SGN_GRAPH_BUCKET=$b timeout -k 10 200 python bench.py --train --steps 60 > gpurun_out/bab.json 2> gpurun_out/bab.err \
      || { echo "FAIL $b"; tail -20 gpurun_out/bab.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/bab.json')); print(sys.argv[1], round(d['value']), round(d['ms_per_step'],3))" $b
  done
done
