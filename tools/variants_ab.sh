#!/bin/bash
# Same-box timing of libsgn_hip.so variants (SGN_HIP_LIB=, no file swapping) on tools/agg_time.py,
# interleaved with the in-tree build.  Usage (GPU box): bash tools/variants_ab.sh <tag> <prec> a.so b.so ...
# A variant named timing*.so also dumps its k_rows16 stamps (tools/x3_timing_ns2.py).
set -u
TAG=$1; PREC=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=gpurun_out/vab_$TAG.jsonl
: > $OUT
for rep in $(seq 1 ${AB_REPS:-2}); do
    SGN_VARIANT=base timeout -k 10 150 python tools/agg_time.py $PREC >> $OUT 2> gpurun_out/vab_$TAG.err || { tail -5 gpurun_out/vab_$TAG.err; exit 1; }
    for v in "$@"; do
        n=$(basename $v .so)
        extra=""
        case $n in timing*) extra="SGN_X3_TDBG=$GRAFT_REPO_ROOT/gpurun_out/tdbg_${TAG}_$n.bin";; esac
        env $extra SGN_VARIANT=$n SGN_HIP_LIB=$GRAFT_REPO_ROOT/$v timeout -k 10 150 python tools/agg_time.py $PREC >> $OUT \
            2> gpurun_out/vab_$TAG.err || { echo "FAIL $v"; tail -5 gpurun_out/vab_$TAG.err; exit 1; }
    done
done
python - <<PY
import json, collections
rs = [json.loads(l) for l in open("$OUT")]
by = collections.defaultdict(list)
for r in rs:
    by[r["lib"]].append(r)
for k, v in by.items():
    print(f"{k:14s} rows " + " ".join(f"{r['agg_rows']:.3f}" for r in v) + "  colour " + " ".join(f"{r['agg_color']:.3f}" for r in v))
PY
for f in gpurun_out/tdbg_${TAG}_*.bin; do [ -f "$f" ] || continue; case $f in *timing2*) python tools/x3_timing2.py $f;; *) python tools/x3_timing_ns2.py $f;; esac; done
echo VAB_DONE
