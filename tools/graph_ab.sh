#!/bin/bash
# Training GPU tests, then the training bench with the loss-stage HIP graph off (0) and on (1), alternated.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_train_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gab_pytest.log 2>&1 \
  || { echo PYTEST_FAIL; tail -40 gpurun_out/gab_pytest.log; exit 1; }
tail -1 gpurun_out/gab_pytest.log
for i in 1 2; do
  for gph in 0 1; do
    SGN_TRAIN_GRAPH=$gph timeout -k 10 200 python bench.py --train --steps 40 > gpurun_out/gab_$gph.json 2> gpurun_out/gab_$gph.err \
      || { echo "FAIL $gph"; tail -30 gpurun_out/gab_$gph.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('graph', sys.argv[2], round(d['value']), round(d['ms_per_step'],3), d.get('final_loss'))" gpurun_out/gab_$gph.json $gph
  done
done
