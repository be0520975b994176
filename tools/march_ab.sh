#!/bin/bash
# Config-2 bench with the thread-per-ray march (default at 640k rays) and the wave-per-ray march.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2; do
  for m in 0 1000000000; do
    SGN_MARCH_WAVE_MAX_RAYS=$m timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/mab.json 2> gpurun_out/mab.err \
      || { echo "FAIL $m"; tail -20 gpurun_out/mab.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/mab.json')); print(sys.argv[1], round(d['value']), d['stages_ms'])" $m
  done
done
