#!/usr/bin/env bash
# Resident tick with workgroup-scope reloads (equality, stamps, trade subset, C5), the fused suite
# after GenStream's DPP scans / LDS period search, and the fused / streamed / DELAY-Level1 lines.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
export TAG=r03_j PYTEST_K="resident or config5 or kats or seeded or ranks"
export BENCHES="MCS_TRADE_RESIDENT=1|--config c5 --steps 1 --warmup 1 --no-cpu-baseline
MCS_TRADE_RESIDENT=0|--config c5 --steps 1 --warmup 1 --no-cpu-baseline"
bash tools/gpu_res.sh || exit $?
OUT="$ROOT/gpurun_out/r03_j"
timeout -k 10 900 python -u -m pytest tests/test_gpu_fused.py -v --timeout 400 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest_fused.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_fused.log"; echo "pytest fused rc=$rc"; [ $rc -ne 0 ] && exit $rc
export BENCHES="MCS_FIFO_ASM=1|--gen fused --steps 10 --warmup 2 --no-cpu-baseline
MCS_FIFO_ASM=1|--steps 10 --warmup 2 --no-cpu-baseline
MCS_FIFO_ASM=1|--gen fused --steps 10 --warmup 2 --no-cpu-baseline
MCS_FIFO_ASM=1|--policy delay --lam 0.9 --max-dur 1200 --steps 3 --warmup 1 --no-cpu-baseline
MCS_FIFO_ASM=1|--policy delay --lam 0.9 --max-dur 1600 --steps 3 --warmup 1 --no-cpu-baseline"
TAG=r03_j bash tools/gpu_r03_g_benches.sh
