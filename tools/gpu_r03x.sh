#!/bin/bash
# GPU: k_rows16 phase cycles + in-kernel clock (timing build), ray-order A/B, lego composite time
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/x3_timing_ab.sh build/variants/tcur.so 2>&1 | tail -24 || exit 1
bash tools/order_ab.sh || exit 1
timeout -k 10 300 python bench.py --scene lego --steps 4 --warmup 2 --no-extras --no-cpu-baseline > gpurun_out/bench_lego_r03x.json 2> gpurun_out/bench_lego_r03x.err || { tail -20 gpurun_out/bench_lego_r03x.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_lego_r03x.json')); print(d['value'], d['stages_ms'])"
