#!/bin/bash
# Same-box A/B of the round-3 tree (02353b9, staged in ab_r03/ with the same pose pinning) against HEAD
# on the driver's exact headline command (no extras), alternating.  Usage (GPU box): bash tools/ab_r03.sh <tag> [rounds]
set -u
TAG=$1; N=${2:-2}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in $(seq $N); do
  for v in r03 head; do
    dir=$GRAFT_REPO_ROOT; [ $v = r03 ] && dir=$GRAFT_REPO_ROOT/ab_r03
    (cd $dir && timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline) \
        > gpurun_out/abr03_${TAG}_$v$i.json 2> gpurun_out/abr03_${TAG}_$v$i.err || { tail -20 gpurun_out/abr03_${TAG}_$v$i.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/abr03_${TAG}_$v$i.json')); print('$v', round(d['value']/1e6,3), 'Mrays/s', 'rows %.3f' % d['stages_ms']['agg_rows'], 'color %.3f' % d['stages_ms']['agg_color'], 'frac', round(d['roofline']['frac'],4), 'nb/ray %.3f' % d['occupancy']['valid_neighbours_per_ray'])"
  done
done
