#!/bin/bash
# GPU: counted-ring k_rows16 (SGN_X3_RING=1): parity subset on the ring build, then same-box timing
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
cp sg-nerf_amd/libsgn_hip.so /tmp/base.so
cp build/variants/ring.so sg-nerf_amd/libsgn_hip.so
timeout -k 10 240 python -u -m pytest tests/test_render_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "golden and f32 or paired or oracle_room" > gpurun_out/pytest_ring.log 2>&1; rc=$?
cp /tmp/base.so sg-nerf_amd/libsgn_hip.so
tail -3 gpurun_out/pytest_ring.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/pytest_ring.log | head; exit 1; }
TIMING_ARGS="8 ring" bash tools/x3_timing_ab.sh build/variants/tring.so > gpurun_out/tim_ring.txt 2>&1 || exit 1; TIMING_ARGS=4 bash tools/x3_timing_ab.sh build/variants/t4.so >> gpurun_out/tim_ring.txt 2>&1 || exit 1
grep -E "^==|median cycles|in-kernel" gpurun_out/tim_ring.txt
rm -f gpurun_out/ab.jsonl; AB_REPS=2 bash tools/x3_ab.sh f32 build/variants/ring.so > /dev/null 2>&1
python -c "
import json,collections
d=collections.defaultdict(list)
for l in open('gpurun_out/ab.jsonl'):
    j=json.loads(l); d[j['lib']].append(round(j['agg_rows'],3))
for k,v in d.items(): print(k, v)
"
