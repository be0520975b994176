#!/bin/bash
# Same-box A/B of libsgn_hip.so variants on tools/agg_time.py, interleaved over two rounds.
# Usage (GPU box): bash tools/x3_ab.sh <prec> a.so b.so ...   (the in-tree lib runs as "base")
set -u
cd "$GRAFT_REPO_ROOT"
PREC=$1; shift
cp sg-nerf_amd/libsgn_hip.so /tmp/base.so
mkdir -p gpurun_out
for rep in $(seq 1 ${AB_REPS:-2}); do
    SGN_VARIANT=base timeout -k 10 120 python tools/agg_time.py $PREC >> gpurun_out/ab.jsonl 2>/dev/null || { echo FAIL base; break; }
    for v in "$@"; do
        cp "$v" sg-nerf_amd/libsgn_hip.so
        SGN_VARIANT=$(basename $v .so) timeout -k 10 120 python tools/agg_time.py $PREC >> gpurun_out/ab.jsonl 2>/dev/null || { echo "FAIL $v"; cp /tmp/base.so sg-nerf_amd/libsgn_hip.so; exit 1; }
        cp /tmp/base.so sg-nerf_amd/libsgn_hip.so
    done
done
cat gpurun_out/ab.jsonl
echo AB_DONE
