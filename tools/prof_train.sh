#!/bin/bash
# Kernel trace of the training bench (config 5).  Usage (GPU box): bash tools/prof_train.sh <tag> [bench args]
set -u
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/proftrain_$TAG -o run --output-format csv -- \
    python bench.py --train "$@" > gpurun_out/proftrain_$TAG.json 2> gpurun_out/proftrain_$TAG.err || { tail gpurun_out/proftrain_$TAG.err; exit 1; }
cat gpurun_out/proftrain_$TAG.json
