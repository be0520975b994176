#!/bin/bash
# Round validation on one GPU box: the whole -m gpu suite, the default bench line (timed wall clock),
# and the kernel trace of the headline bench.  Usage (GPU box): bash tools/gpu_full.sh <tag>
set -u
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_full_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_full_$TAG.log
[ $rc -eq 0 ] || exit $rc
t0=$(date +%s.%N)
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
t1=$(date +%s.%N)
echo "bench wall $(python -c "print(round($t1 - $t0, 1))") s"
python - <<PY
import json
d = json.load(open("gpurun_out/bench_$TAG.json"))
print("headline", round(d["value"] / 1e6, 2), "Mrays/s", round(d["ms_per_step"], 2), "ms frac", round(d["roofline"]["frac"], 3))
for k in ("f16_mode", "lego", "sg", "config3_1gpu", "stress_dense", "train_config5", "train_config5_f16"):
    v = d.get(k)
    if v:
        print(k, round(v["value"] / 1e6, 3), "M", {kk: v.get(kk) for kk in ("ms_per_frame", "ms_per_step")},
              (v.get("roofline") or {}).get("frac", v.get("roofline_frac")))
print("cpu", d.get("cpu_baseline", {}).get("value"))
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/prof_$TAG.json 2> gpurun_out/prof_$TAG.err || { echo PROF_FAIL; tail gpurun_out/prof_$TAG.err; exit 1; }
echo FULL_DONE
