#!/bin/bash
# One GPU call: kernel-trace stats of the fp32 headline bench + PMC passes (tools/profile_pmc.sh)
# for the default kernels.  Usage (GPU box): bash tools/prof_x3.sh <tag>
set -u
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
    python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras > gpurun_out/prof_$TAG.json 2> gpurun_out/prof_$TAG.err || { echo PROF_FAIL; tail gpurun_out/prof_$TAG.err; exit 1; }
timeout -k 10 900 bash tools/profile_pmc.sh gpurun_out/pmc_$TAG > gpurun_out/pmc_$TAG.out 2>&1 || { echo PMC_FAIL; tail gpurun_out/pmc_$TAG.out; exit 1; }
echo PROF_X3_DONE
