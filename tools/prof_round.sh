#!/bin/bash
# One GPU call: kernel-trace stats + PMC passes of bench.py, the SG bench and a kernel trace of
# the training bench.  Usage (GPU box): bash tools/prof_round.sh <tag>
set -u
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
    python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_$TAG.json 2> gpurun_out/prof_$TAG.err || { echo PROF_FAIL; tail gpurun_out/prof_$TAG.err; exit 1; }
cat gpurun_out/prof_$TAG.json
timeout -k 10 300 python bench.py --no-cpu-baseline --sg > gpurun_out/benchsg_$TAG.json 2> gpurun_out/benchsg_$TAG.err || { echo SG_FAIL; tail gpurun_out/benchsg_$TAG.err; exit 1; }
cat gpurun_out/benchsg_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/proftrain_$TAG -o run --output-format csv -- \
    python bench.py --train > gpurun_out/proftrain_$TAG.json 2> gpurun_out/proftrain_$TAG.err || { echo TRAINPROF_FAIL; tail gpurun_out/proftrain_$TAG.err; exit 1; }
cat gpurun_out/proftrain_$TAG.json
KREGEX="k_agg_rows|k_knn|k_march|k_color|k_composite" timeout -k 10 900 bash tools/profile_pmc.sh gpurun_out/pmc_$TAG \
    > gpurun_out/pmc_$TAG.out 2>&1 || { echo PMC_FAIL; tail gpurun_out/pmc_$TAG.out; exit 1; }
echo PROF_ROUND_DONE
