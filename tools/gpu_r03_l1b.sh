#!/usr/bin/env bash
# DELAY suites (batch, online, fused) after a delay_kernel change, then the Level1 bench lines.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r03_l1b}"
mkdir -p "$OUT"; cd "$ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_delay.py tests/test_gpu_online.py tests/test_gpu_fused.py -m gpu -x -q \
    --timeout 200 --timeout-method thread -p no:cacheprovider ${PYK:-} > "$OUT/pytest_delay.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_delay.log"; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r03_l1b} bash tools/gpu_r03_l1.sh
