#!/usr/bin/env bash
# The fused suite after the straddling-window fix of GenStream's scratch period search, the FIFO
# kernel-variant sweep, the fused bench line and the resident tick's segment stamps on C5.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${TAG:-r03_l}"; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_fused.py "tests/test_gpu_parity.py::test_every_kernel_variant" -v \
    --timeout 400 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_fused.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_fused.log"; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --gen fused --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/bench_fused.json" 2> "$OUT/bench_fused.err"
rc=$?; head -c 400 "$OUT/bench_fused.json"; echo; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/stamp_res.py variants/libmcs_res_stamps.so 156250 > "$OUT/stamps_res.json" 2>&1
rc=$?; cat "$OUT/stamps_res.json"; echo "stamps rc=$rc"
