#!/usr/bin/env bash
# The resident tick after its prefetch rework (quick equality, segment stamps, C5 tick loops) and
# the hand-scheduled FIFO loop on a fused stream (its parity tests, --gen fused against the compiled
# fused kernel and the streamed headline).  Each GPU step has its own limit; a failure ends the call.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r03_g}"
mkdir -p "$OUT"
cd "$ROOT"
export PYTHONUNBUFFERED=1
TAG=${TAG:-r03_g} SKIP_PYTEST=1 bash tools/gpu_res.sh || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_fused.py "tests/test_gpu_trade.py::test_gpu_trade_resident_equals_kernels_and_oracle" \
    "tests/test_gpu_trade.py::test_gpu_trade_config5_full_size" -v --timeout 400 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest_fused_res.log" 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" "$OUT/pytest_fused_res.log" | tail -40; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_r03_g_benches.sh
