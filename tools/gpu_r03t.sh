# GPU: selected pytest subset (args: tag, -k expression)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
tag=$1; sel=$2
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s -k "$sel" > gpurun_out/pytest_$tag.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|relative L2|config 5|passed|failed" gpurun_out/pytest_$tag.log | tail -40
[ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/pytest_$tag.log | head -30; exit 1; }
exit 0
