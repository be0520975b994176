#!/bin/bash
# One GPU call: kernel-trace stats + PMC passes of bench.py, then optional variant benches.
# Usage (GPU box): bash tools/prof_round.sh <tag> [variant.so ...]
set -u
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
    python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || exit 1
KREGEX="k_agg_rows|k_knn|k_march|k_color|k_composite" timeout -k 10 900 bash tools/profile_pmc.sh gpurun_out/pmc_$TAG \
    > gpurun_out/pmc_$TAG.log 2>&1 || exit 1
cp sg-nerf_amd/libsgn_hip.so /tmp/base.so
for v in "$@"; do
    cp "$v" sg-nerf_amd/libsgn_hip.so
    timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$(basename $v .so).json 2>&1 || exit 1
done
cp /tmp/base.so sg-nerf_amd/libsgn_hip.so
echo PROF_ROUND_DONE
