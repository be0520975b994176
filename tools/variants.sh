#!/bin/bash
# Bench (and render-parity-test) libsgn_hip.so variants in one GPU call.
# Usage (GPU box): bash tools/variants.sh variant.so ...   (the in-tree lib is benched first as "base")
set -u
cd "$GRAFT_REPO_ROOT"
cp sg-nerf_amd/libsgn_hip.so /tmp/base.so
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/var_base.json 2>&1 || exit 1
for v in "$@"; do
    n=$(basename $v .so)
    cp "$v" sg-nerf_amd/libsgn_hip.so
    timeout -k 10 300 python -m pytest tests/test_render_gpu.py tests/test_api_gpu.py -q -x > gpurun_out/var_$n.test.log 2>&1
    echo "rc=$?" >> gpurun_out/var_$n.test.log
    timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/var_$n.json 2>&1 || exit 1
done
cp /tmp/base.so sg-nerf_amd/libsgn_hip.so
echo VARIANTS_DONE
