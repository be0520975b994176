#!/bin/bash
# GPU: loss-stage parity + the training tests on the HIP loss stage, then training step timings
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_loss_gpu.py tests/test_train_gpu.py -m gpu -v -s --timeout 200 --timeout-method thread > gpurun_out/pytest_t2.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|rel L2|relative L2" gpurun_out/pytest_t2.log | head -60; tail -2 gpurun_out/pytest_t2.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit 1
for p in f32 f16; do
  timeout -k 10 300 python bench.py --train --train-precision $p --steps 20 --warmup 5 > gpurun_out/train_$p.json 2> gpurun_out/train_$p.err || { tail -20 gpurun_out/train_$p.err; exit 1; }
  SGN_HIP_LOSS=0 timeout -k 10 300 python bench.py --train --train-precision $p --steps 20 --warmup 5 > gpurun_out/train_${p}_torchloss.json 2> gpurun_out/train_${p}_t.err || { tail -20 gpurun_out/train_${p}_t.err; exit 1; }
  python -c "import json; a=json.load(open('gpurun_out/train_$p.json')); b=json.load(open('gpurun_out/train_${p}_torchloss.json')); print('$p hip-loss', a['ms_per_step'], a['final_loss'], ' torch-loss', b['ms_per_step'], b['final_loss'])"
done
