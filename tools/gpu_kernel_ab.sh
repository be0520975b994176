#!/bin/bash
# One GPU call (NOT product): kernel traces of config-5 training steps for the in-tree library and
# variant builds (SGN_HIP_LIB, tools/src_variant.sh), interleaved; prints each run's step time and the
# average duration of the kernels matching a regex (rocprofv3 --stats).
# Usage (GPU box): bash tools/gpu_kernel_ab.sh <tag> "<variant.so ...>" <kernel regex> [precisions="f32 f16"] [reps=2]
set -u
TAG=$1; VARS=$2; KRE=$3; PRECS=${4:-f32 f16}; REPS=${5:-2}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for P in $PRECS; do
  for i in $(seq 1 $REPS); do
    for v in intree $VARS; do
      lib=$GRAFT_REPO_ROOT/sg-nerf_amd/libsgn_hip.so; [ $v != intree ] && lib=$GRAFT_REPO_ROOT/$v
      b=$(basename $v .so); d=gpurun_out/kab_${TAG}_${P}_${b}_$i
      SGN_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- \
          python bench.py --train --train-precision $P --steps 30 --warmup 5 --no-cpu-baseline \
          > $d.json 2> $d.err || { tail -5 $d.err; exit 1; }
      f=$(find $d -name "*kernel_stats.csv" | head -1)
      python - "$f" "$d.json" "$KRE" "$P $b $i" <<'PY'
import csv, json, re, sys
st = [r for r in csv.DictReader(open(sys.argv[1])) if re.search(sys.argv[3], r["Name"])]
ms = json.load(open(sys.argv[2]))["ms_per_step"]
print(sys.argv[4], "step %.3f ms" % ms, " ".join("%s=%.1fus" % (re.sub(r"\(.*", "", r["Name"].replace("(anonymous namespace)::", "")).split("::")[-1], float(r["AverageNs"]) / 1e3) for r in st))
PY
    done
  done
done
