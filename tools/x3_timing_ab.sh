#!/bin/bash
# Per-phase k_rows16 clock stamps of SGN_X3_TIMING variants (GPU box), one agg_time run each.
# Usage: bash tools/x3_timing_ab.sh a.so b.so ...
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
cp sg-nerf_amd/libsgn_hip.so /tmp/base.so
for v in "$@"; do
    n=$(basename $v .so)
    cp "$v" sg-nerf_amd/libsgn_hip.so
    SGN_X3_TDBG=$PWD/gpurun_out/t_$n.bin timeout -k 10 120 python tools/agg_time.py f32 2 > /dev/null 2>&1 || { echo "FAIL $n"; cp /tmp/base.so sg-nerf_amd/libsgn_hip.so; exit 1; }
    echo "== $n"; python tools/x3_timing16.py gpurun_out/t_$n.bin ${TIMING_ARGS:-}
done
cp /tmp/base.so sg-nerf_amd/libsgn_hip.so
echo TIMING_DONE
