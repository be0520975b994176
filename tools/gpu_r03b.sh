set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -k "golden or paired or pair_slots or full_frame or oracle_room or shuffled or range_guard or api" > gpurun_out/pytest_r03b.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_r03b.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/pytest_r03b.log | head -20; exit 1; }
bash tools/x3_timing_ab.sh build/variants/tbase.so build/variants/tnew.so > gpurun_out/timing_r03b.log 2>&1 || { tail gpurun_out/timing_r03b.log; exit 1; }
cat gpurun_out/timing_r03b.log
AB_REPS=2 timeout -k 10 400 bash tools/x3_ab.sh f32 build/variants/old.so > /dev/null 2>&1; tail -6 gpurun_out/ab.jsonl
