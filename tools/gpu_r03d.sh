set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -k "golden or paired or pair_slots or full_frame or oracle_room or shuffled or range_guard or api" > gpurun_out/pytest_r03d.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_r03d.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/pytest_r03d.log | head -20; exit 1; }
rm -f gpurun_out/ab.jsonl
AB_REPS=3 timeout -k 10 600 bash tools/x3_ab.sh f32 build/variants/old.so build/variants/nosplit.so > /dev/null 2>&1; cat gpurun_out/ab.jsonl
