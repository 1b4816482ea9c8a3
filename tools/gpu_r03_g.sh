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
i=0
while IFS= read -r line; do
    [ -z "$line" ] && continue
    i=$((i+1))
    env_part="${line%%|*}"; args="${line#*|}"
    env $env_part timeout -k 10 300 python bench.py $args > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err"
    rc=$?; echo "bench $i ($env_part $args) rc=$rc"; python3 -c "
import json; d=json.loads(open('$OUT/bench_$i.json').read().strip().splitlines()[-1])
print('  %.4g' % d['value'], d['unit'], 'ms/step %.3f' % d['ms_per_step'], d.get('roofline', {}).get('kernel', ''), 'frac', d.get('roofline', {}).get('frac'))" 2>/dev/null || tail -3 "$OUT/bench_$i.err"
    [ $rc -ne 0 ] && exit $rc
done <<LIST
${BENCHES:-MCS_FIFO_ASM=1|--gen fused --steps 10 --warmup 2 --no-cpu-baseline
MCS_FIFO_ASM=0|--gen fused --steps 10 --warmup 2 --no-cpu-baseline
MCS_FIFO_ASM=1|--steps 10 --warmup 2 --no-cpu-baseline
MCS_FIFO_ASM=1|--gen fused --steps 10 --warmup 2 --no-cpu-baseline
MCS_FIFO_ASM=1|--gen fused --clusters 512 --steps 10 --warmup 2 --no-cpu-baseline
MCS_FIFO_ASM=1|--config c3 --gen fused --steps 5 --warmup 1 --no-cpu-baseline}
LIST
echo done