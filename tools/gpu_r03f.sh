set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -k "golden or paired or full_frame or oracle_room or api" > gpurun_out/pytest_r03f.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_r03f.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/pytest_r03f.log | head -20; exit 1; }
bash tools/x3_timing_ab.sh build/variants/told.so build/variants/tnew.so 2>&1 | tail -44
