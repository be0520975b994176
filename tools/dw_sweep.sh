#!/bin/bash
# Training bench (config 5) over split-K chunk sizes of the weight-gradient GEMMs, then the
# training GPU tests at the default chunk.  Usage (GPU box): bash tools/dw_sweep.sh <tag>
set -u
TAG=${1:-dw}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for c in ${SWEEP:-8192 4096 2048 1024 512}; do
  SGN_DW_CHUNK=$c timeout -k 10 200 python bench.py --train --steps 30 > gpurun_out/dw_${TAG}_$c.json 2> gpurun_out/dw_${TAG}_$c.err \
    || { echo "BENCH_FAIL $c"; tail -20 gpurun_out/dw_${TAG}_$c.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), round(d['ms_per_step'],3))" gpurun_out/dw_${TAG}_$c.json $c
done
timeout -k 10 300 python -u -m pytest tests/test_train_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dw_${TAG}_pytest.log 2>&1 \
  || { echo PYTEST_FAIL; tail -30 gpurun_out/dw_${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/dw_${TAG}_pytest.log
