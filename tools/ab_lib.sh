#!/bin/bash
# Same-box A/B of two builds of libsgn_hip.so on the headline frame (no extras), alternating.
# Usage (GPU box): bash tools/ab_lib.sh <tag> <lib A> <lib B> [rounds] [extra env for both]
set -u
TAG=$1; A=$2; B=$3; N=${4:-2}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in $(seq $N); do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    SGN_HIP_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline \
        > gpurun_out/ab_${TAG}_$v$i.json 2> gpurun_out/ab_${TAG}_$v$i.err || { tail -20 gpurun_out/ab_${TAG}_$v$i.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab_${TAG}_$v$i.json')); print('$v', '$lib', round(d['value']/1e6,2), 'Mrays/s', 'rows %.2f' % d['stages_ms']['agg_rows'], 'color %.2f' % d['stages_ms']['agg_color'], 'frac', round(d['roofline']['frac'],3))"
  done
done
