#!/bin/bash
# GPU: K < 8 tests, the render / API suites and a headline bench (the fp32 row kernel changed)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_render_gpu.py tests/test_api_gpu.py tests/test_query_gpu.py -m gpu -q -s --timeout 200 --timeout-method thread > gpurun_out/pytest_k.log 2>&1; rc=$?
grep -E "K=|FAILED|ERROR" gpurun_out/pytest_k.log | head -30; tail -2 gpurun_out/pytest_k.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python bench.py --no-extras --no-cpu-baseline > gpurun_out/bench_k.json 2> gpurun_out/bench_k.err || { tail -20 gpurun_out/bench_k.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_k.json')); print(d['value'], d['stages_ms'], d['roofline']['frac'], d['roofline_query']['counter']['GBps_over_query_stage'])"
