#!/bin/bash
# Experiment build (NOT product): link a given agg_train.hip (a file, or "HEAD" for the committed
# one) with the in-tree objects of every other source -> build/variants/<name>.so, for the same-box
# replay timing of tools/agg_bwd_ab.py.
# Usage: bash tools/agg_bwd_variant.sh <name> <agg_train.hip | HEAD> [extra hipcc flags]
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/sg-nerf_amd/csrc
NAME=$1; SRC=$2; shift 2
make -s -C "$C" -j8 >/dev/null
W=/tmp/aggv_$NAME/pkg/csrc
rm -rf /tmp/aggv_$NAME && mkdir -p "$W" && cp "$C"/*.h "$W"/ && ln -s "$ROOT/include" /tmp/aggv_$NAME/include
if [ "$SRC" = HEAD ]; then git -C "$ROOT" show HEAD:sg-nerf_amd/csrc/agg_train.hip > "$W/agg_train.hip"; else cp "$SRC" "$W/agg_train.hip"; fi
HIPCC=/opt/rocm/bin/hipcc
$HIPCC --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -munsafe-fp-atomics -I"$ROOT/include" "$@" \
    -c "$W/agg_train.hip" -o "$W/agg_train.o"
mkdir -p "$ROOT/build/variants"
OBJS=$(ls "$C"/build/*.o | grep -v "/agg_train.o")
$HIPCC --offload-arch=gfx950 -shared -Wl,-rpath,/opt/rocm/lib -o "$ROOT/build/variants/$NAME.so" $OBJS "$W/agg_train.o"
echo "$ROOT/build/variants/$NAME.so"
