#!/bin/bash
# Experiment build (NOT product): one csrc/<src>.hip taken from a file (or "HEAD": the committed one)
# linked with the in-tree objects of every other source -> build/variants/<name>.so, for same-box
# A/B through SGN_HIP_LIB (tools/agg_bwd_ab.py, tools/ab_train_lib.sh).
# Usage: bash tools/src_variant.sh <name> <src, e.g. train_x3> <file.hip | HEAD> [extra hipcc flags]
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/sg-nerf_amd/csrc
NAME=$1; SRCN=$2; SRC=$3; shift 3
make -s -C "$C" -j8 >/dev/null
W=/tmp/srcv_$NAME/pkg/csrc
rm -rf /tmp/srcv_$NAME && mkdir -p "$W" && cp "$C"/*.h "$W"/ && ln -s "$ROOT/include" /tmp/srcv_$NAME/include
if [ "$SRC" = HEAD ]; then git -C "$ROOT" show HEAD:sg-nerf_amd/csrc/$SRCN.hip > "$W/$SRCN.hip"; else cp "$SRC" "$W/$SRCN.hip"; fi
HIPCC=/opt/rocm/bin/hipcc
EXTRA=""; case $SRCN in mlp_x3|train_x3) EXTRA=-fno-slp-vectorize;; esac
$HIPCC --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -munsafe-fp-atomics $EXTRA -I"$ROOT/include" "$@" \
    -c "$W/$SRCN.hip" -o "$W/$SRCN.o"
mkdir -p "$ROOT/build/variants"
OBJS=$(ls "$C"/build/*.o | grep -v "/$SRCN.o")
$HIPCC --offload-arch=gfx950 -shared -Wl,-rpath,/opt/rocm/lib -o "$ROOT/build/variants/$NAME.so" $OBJS "$W/$SRCN.o"
echo "$ROOT/build/variants/$NAME.so"
