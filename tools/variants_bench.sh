#!/bin/bash
# Bench-only comparison of libsgn_hip.so variants in one GPU call (timing ablations whose
# results are wrong by design skip the parity tests).  Usage: bash tools/variants_bench.sh a.so ...
set -u
cd "$GRAFT_REPO_ROOT"
cp sg-nerf_amd/libsgn_hip.so /tmp/base.so
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/var_base.json 2>&1 || exit 1
for v in "$@"; do
    n=$(basename $v .so)
    cp "$v" sg-nerf_amd/libsgn_hip.so
    timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/var_$n.json 2>&1 || { echo "FAIL $n"; break; }
done
cp /tmp/base.so sg-nerf_amd/libsgn_hip.so
echo VARIANTS_DONE
