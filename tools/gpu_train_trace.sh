#!/bin/bash
# One GPU call: kernel traces of config-5 training at both precisions and their steady-state step
# windows (tools/step_window.py).  Usage (GPU box): bash tools/gpu_train_trace.sh <tag>
set -u
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for P in f32 f16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trtrace_${P}_$TAG -o run --output-format csv -- \
      python bench.py --train --train-precision $P --steps 30 --warmup 5 --no-cpu-baseline \
      > gpurun_out/trtrace_${P}_$TAG.json 2> gpurun_out/trtrace_${P}_$TAG.err || { tail -5 gpurun_out/trtrace_${P}_$TAG.err; exit 1; }
  f=$(find gpurun_out/trtrace_${P}_$TAG -name "*kernel_trace.csv" | head -1)
  python tools/step_window.py "$f" 20 40 > gpurun_out/trwin_${P}_$TAG.txt
  head -14 gpurun_out/trwin_${P}_$TAG.txt
done
