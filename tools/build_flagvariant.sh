#!/usr/bin/env bash
# Build libmcs.so with a given mcs_kernels.hip and extra hipcc flags into variants/libmcs_<name>.so.
#   usage: tools/build_flagvariant.sh <name> <mcs_kernels.hip> [extra hipcc flags...]
set -eu
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
NAME="$1"; SRC="$2"; shift 2
PKG="$ROOT/multi-cluster-simulator_amd"
mkdir -p "$ROOT/variants" "$PKG/build/v_$NAME"
cp "$SRC" "$PKG/build/v_$NAME/mcs_kernels.hip"
cp "$PKG"/csrc/*.h "$PKG/build/v_$NAME/"
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-result -I$ROOT/include -mllvm -amdgpu-atomic-optimizer-strategy=None"
/opt/rocm/bin/hipcc $FLAGS "$@" -I"$PKG/csrc" -c -o "$PKG/build/v_$NAME/k.o" "$PKG/build/v_$NAME/mcs_kernels.hip"
OTHERS=$(ls "$PKG"/build/*.o | grep -v '/mcs_kernels.o$')
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$ROOT/variants/libmcs_$NAME.so" "$PKG/build/v_$NAME/k.o" \
    $OTHERS -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "variants/libmcs_$NAME.so"
