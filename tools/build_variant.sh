#!/usr/bin/env bash
# Build libmcs.so with a different fifo_kernel body into variants/libmcs_<name>.so (A/B timing).
#   usage: tools/build_variant.sh <name> <kernel-body.hip>
set -eu
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
NAME="$1"; BODY="$2"
PKG="$ROOT/multi-cluster-simulator_amd"
mkdir -p "$ROOT/variants" "$PKG/build/v_$NAME"
python3 - "$PKG/csrc/mcs_kernels.hip" "$BODY" "$PKG/build/v_$NAME/mcs_kernels.hip" <<'PY'
import sys
s = open(sys.argv[1]).read()
i = s.index('template <int NPL, int P, bool GEN>\n__global__ __launch_bounds__(64) void fifo_kernel(FifoArgs a) {')
j = s.index('// ---- variant table')
open(sys.argv[3], 'w').write(s[:i] + open(sys.argv[2]).read() + s[j:])
PY
cp "$PKG"/csrc/*.h "$PKG/build/v_$NAME/"
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-result -I$ROOT/include -mllvm -amdgpu-atomic-optimizer-strategy=None"
/opt/rocm/bin/hipcc $FLAGS -I"$PKG/csrc" -c -o "$PKG/build/v_$NAME/k.o" "$PKG/build/v_$NAME/mcs_kernels.hip"
OTHERS=$(ls "$PKG"/build/*.o | grep -v '/mcs_kernels.o$')
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$ROOT/variants/libmcs_$NAME.so" "$PKG/build/v_$NAME/k.o" \
    $OTHERS -L/opt/rocm/lib -lrccl \
    -Wl,-rpath,/opt/rocm/lib
echo "variants/libmcs_$NAME.so"
