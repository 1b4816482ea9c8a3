#!/usr/bin/env bash
# Build libmcs.so with one source file replaced (e.g. a mcs_fifo_asm.hip variant, or the in-tree
# mcs_trade_res.hip with -DMCS_STAMPS) into variants/libmcs_<name>.so, the other objects from the
# last in-tree build.   usage: tools/variant.sh <name> <file.hip> [hipcc flags]
# (OBJ=<object name> when the source's object is named otherwise, e.g. OBJ=mcs_dtrade_k for mcs_dtrade.hip)
set -eu
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
NAME="$1"; SRC="$2"; shift 2
PKG="$ROOT/multi-cluster-simulator_amd"
mkdir -p "$ROOT/variants" "$PKG/build/a_$NAME"
BASE="$(basename "$SRC" .hip)"
cp "$SRC" "$PKG/build/a_$NAME/$BASE.hip"
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-result -I$ROOT/include -mllvm -amdgpu-atomic-optimizer-strategy=None -mllvm -structurizecfg-skip-uniform-regions"
/opt/rocm/bin/hipcc $FLAGS "$@" -I"$PKG/csrc" -c -o "$PKG/build/a_$NAME/k.o" "$PKG/build/a_$NAME/$BASE.hip"
OTHERS=$(ls "$PKG"/build/*.o | grep -v "/${OBJ:-$BASE}.o\$")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$ROOT/variants/libmcs_$NAME.so" "$PKG/build/a_$NAME/k.o" \
    $OTHERS -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "variants/libmcs_$NAME.so"
