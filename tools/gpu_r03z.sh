#!/bin/bash
# GPU: parity subset on the in-tree lib, then timings and same-box A/B vs the 8-wave row kernel
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -k "golden or paired or full_frame or oracle_room or api or lego or sg or config5 or range" > gpurun_out/pytest_r03z.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_r03z.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/pytest_r03z.log | head -20; exit 1; }
bash tools/x3_timing_ab.sh build/variants/t4.so build/variants/tcur.so > gpurun_out/tim_r03z.txt 2>&1 || exit 1
grep -E "^==|median cycles|in-kernel" gpurun_out/tim_r03z.txt
AB_REPS=2 bash tools/x3_ab.sh f32 build/variants/rw8.so build/variants/cw8.so | grep agg_rows
