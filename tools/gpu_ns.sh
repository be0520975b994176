#!/bin/bash
# A/B of the row kernel's row sets per wave (SGN_ROWS_NS=2: 32 rows per wave): the render parity
# subset under NS=2, then the headline frame rate (no extras) under each form.
# Usage (GPU box): bash tools/gpu_ns.sh <tag>
set -u
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
SGN_ROWS_NS=${TESTNS:-2} timeout -k 10 300 python -u -m pytest tests/test_render_gpu.py -x -v --timeout 200 --timeout-method thread \
    -k "golden or oracle_room or lego or paired or config2 or spiral" > gpurun_out/pytest_ns_$TAG.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_ns_$TAG.log
[ $rc -eq 0 ] || exit $rc
for ns in ${NSLIST:-1 2}; do
    SGN_ROWS_NS=$ns timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-extras --no-cpu-baseline \
        > gpurun_out/bench_ns${ns}_$TAG.json 2> gpurun_out/bench_ns${ns}_$TAG.err || { tail -20 gpurun_out/bench_ns${ns}_$TAG.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/bench_ns${ns}_$TAG.json')); print('NS=$ns', round(d['value']/1e6,2), 'Mrays/s', round(d['ms_per_step'],2), 'ms', d['stages_ms'], 'frac', round(d['roofline']['frac'],3))"
done
