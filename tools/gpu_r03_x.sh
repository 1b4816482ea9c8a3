#!/usr/bin/env bash
# Workgroup-resident tick with its workers on one XCD (L2 exchange) vs across XCDs: resident parity
# cases, C5 both ways.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${TAG:-r03_x}"; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
c5() {  # $1 = MCS_MW_XCD, $2 = tag
  MCS_MW_XCD=$1 timeout -k 10 300 python bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/c5_$2.json" 2> "$OUT/c5_$2.err"
  rc=$?; python3 -c "
import json; d=json.loads(open('$OUT/c5_$2.json').read().strip().splitlines()[-1]); t=d['trading']
print('  $2 %.4g' % d['value'], d['unit'], 'us/tick %.2f' % t['us_per_tick'], 'loop_form', t['loop_form'], 'ticks', t['ticks'], 'flags', t['flags'])"
  return $rc
}
c5 1 xcd && c5 0 uc || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_trade.py -x -v -k "resident or kats or config5 or capacity" --timeout 500 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_trade.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_trade.log"; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
c5 1 xcd2
