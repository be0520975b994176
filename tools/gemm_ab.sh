#!/bin/bash
# Same-box isolated GEMM timing (tools/gemm_time.py) of libsgn_hip.so variants against the in-tree
# build.  Usage (GPU box): bash tools/gemm_ab.sh <tag> a.so b.so ...   [env: REPS (2)]
set -u
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-2}); do
  for v in base "$@"; do
    lib=sg-nerf_amd/libsgn_hip.so; [ $v != base ] && lib=$v
    SGN_HIP_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 120 python tools/gemm_time.py >> gpurun_out/gab_$TAG.jsonl 2> gpurun_out/gab_$TAG.err \
        || { echo "FAIL $v"; tail -5 gpurun_out/gab_$TAG.err; exit 1; }
    tail -1 gpurun_out/gab_$TAG.jsonl
  done
done
echo GAB_DONE
