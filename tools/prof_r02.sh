#!/bin/bash
# One GPU call for the round's profile set: kernel-trace stats + PMC passes of the f32 headline
# bench (tools/prof_x3.sh), then the lego (config 4) and SG bench lines.  Usage: bash tools/prof_r02.sh <tag>
set -u
TAG=$1
cd "$GRAFT_REPO_ROOT"
bash tools/prof_x3.sh $TAG || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --scene lego > gpurun_out/benchlego_$TAG.json 2> gpurun_out/benchlego_$TAG.err || { echo LEGO_FAIL; tail gpurun_out/benchlego_$TAG.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --sg > gpurun_out/benchsg_$TAG.json 2> gpurun_out/benchsg_$TAG.err || { echo SG_FAIL; tail gpurun_out/benchsg_$TAG.err; exit 1; }
echo PROF_R02_DONE
