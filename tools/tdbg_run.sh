#!/bin/bash
# Chunk-timing traces of SGN_TIMING variants (GPU box).  Usage: bash tools/tdbg_run.sh name ...
# (build/variants/<name>.so -> gpurun_out/tdbg_<name>.bin); the in-tree lib is restored after.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
cp sg-nerf_amd/libsgn_hip.so /tmp/base.so
for n in "$@"; do
    cp build/variants/$n.so sg-nerf_amd/libsgn_hip.so
    SGN_TDBG=$PWD/gpurun_out/tdbg_$n.bin timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline \
        > gpurun_out/tdbg_$n.json 2> gpurun_out/tdbg_$n.err || { echo "FAIL $n"; break; }
done
cp /tmp/base.so sg-nerf_amd/libsgn_hip.so
echo TDBG_DONE
