#!/bin/bash
# GPU: f32 training step, split-K dW A/B and a kernel trace of the current step
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for c in 1024 0 4096; do
  SGN_DW_CHUNK_F32=$c timeout -k 10 300 python bench.py --train --steps 20 --warmup 5 > gpurun_out/tr_c$c.json 2> gpurun_out/tr_c$c.err || { tail -20 gpurun_out/tr_c$c.err; exit 1; }
  python -c "import json; a=json.load(open('gpurun_out/tr_c$c.json')); print('chunk $c', a['ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/proftrain_t3 -o run --output-format csv -- \
    python bench.py --train --steps 20 --warmup 5 > gpurun_out/proftrain_t3.json 2> gpurun_out/proftrain_t3.err || { tail gpurun_out/proftrain_t3.err; exit 1; }
echo T3_DONE
