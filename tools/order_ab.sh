#!/bin/bash
# Same-box A/B of the ray order (tools/agg_time.py SGN_RAY_ORDER), interleaved.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in 1 2; do
    for b in 0 8 16 32; do
        SGN_RAY_ORDER=$b timeout -k 10 120 python tools/agg_time.py f32 >> gpurun_out/order_ab.jsonl 2>/dev/null || { echo FAIL $b; exit 1; }
    done
done
cat gpurun_out/order_ab.jsonl
