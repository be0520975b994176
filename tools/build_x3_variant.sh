#!/bin/bash
# Build a variant of libsgn_hip.so with extra defines for mlp_x3.hip.
# Usage: bash tools/build_x3_variant.sh <name> "<-D flags>"   -> build/variants/<name>.so
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/sg-nerf_amd/csrc
make -s -C "$C" >/dev/null
mkdir -p "$ROOT/build/variants"
HIPCC=/opt/rocm/bin/hipcc
FL="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -munsafe-fp-atomics -fno-slp-vectorize -I$ROOT/include"
$HIPCC $FL $2 -c "$C/mlp_x3.hip" -o "/tmp/mlpx3_$1.o"
OBJS=$(ls $C/build/*.o | grep -v "/mlp_x3.o")
$HIPCC --offload-arch=gfx950 -shared -Wl,-rpath,/opt/rocm/lib -o "$ROOT/build/variants/$1.so" $OBJS "/tmp/mlpx3_$1.o"
echo "$ROOT/build/variants/$1.so"
