#!/bin/bash
# One GPU call: a subset of the -m gpu suite (pytest -k expression), then -- unless the tests ended
# in a fault / timeout -- a same-box A/B of library variants on tools/agg_time.py.
# Usage (GPU box): bash tools/gpu_tests_ab.sh <tag> "<pytest -k expr>" [variant.so ...]
set -u
TAG=$1; KEXPR=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$KEXPR" \
    > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_$TAG.log
[ $rc -le 1 ] || exit $rc
if [ $# -gt 0 ]; then
    rm -f gpurun_out/ab.jsonl
    AB_REPS=${AB_REPS:-3} bash tools/x3_ab.sh f32 "$@" > gpurun_out/ab_$TAG.log 2>&1 || { tail gpurun_out/ab_$TAG.log; exit 1; }
    python - <<PY
import json
for l in open("gpurun_out/ab.jsonl"):
    r = json.loads(l)
    print(r["lib"], round(r["agg_rows"], 3), round(r["agg_color"], 3), round(r["frame"], 3))
PY
fi
exit $rc
