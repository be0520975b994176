#!/bin/bash
# GPU: k_rows16 ablation timings (timing builds; ablated variants compute wrong results by design)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
V=build/variants
bash tools/x3_timing_ab.sh $V/tcur.so $V/tnodma.so $V/tnobar.so $V/tnodmabar.so $V/tmfma1.so $V/tmfma1nodma.so > gpurun_out/abl.txt 2>&1
rc=$?
grep -E "^==|median cycles|in-kernel|L1C1|L2C2|L0 |epilogue|tile end" gpurun_out/abl.txt
exit $rc
