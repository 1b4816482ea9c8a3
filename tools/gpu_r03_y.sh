#!/usr/bin/env bash
# C/D without waiting for X2 (acceptances applied at the next tick's start): resident parity cases,
# C5 A/B against the previous kernel (variants/libmcs_mw_prev.so), stamps.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${TAG:-r03_y}"; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
c5() {  # $1 = library ("" = in-tree), $2 = tag
  MCS_LIB=$1 timeout -k 10 300 python bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/c5_$2.json" 2> "$OUT/c5_$2.err"
  rc=$?; python3 -c "
import json; d=json.loads(open('$OUT/c5_$2.json').read().strip().splitlines()[-1]); t=d['trading']
print('  $2 %.4g' % d['value'], d['unit'], 'us/tick %.2f' % t['us_per_tick'], 'loop_form', t['loop_form'], 'ticks', t['ticks'], 'flags', t['flags'])"
  return $rc
}
timeout -k 10 600 python -u -m pytest tests/test_gpu_trade.py -x -v -k "resident or kats or config5 or capacity or fuzz" --timeout 500 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_trade.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_trade.log"; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
c5 "" new && c5 "$ROOT/variants/libmcs_mw_prev.so" prev && c5 "" new2 || exit $?
timeout -k 10 300 python -u tools/stamp_mw.py variants/libmcs_mw_stamps.so 40000 > "$OUT/stamps_mw.json" 2>&1
rc=$?; python3 -c "
import json; d=json.load(open('$OUT/stamps_mw.json')); print(d['us_per_tick'], d.get('sweep_passes_per_tick_x1_x2_by_wg'), d['us_per_tick_wg0_wave0'], d['us_per_tick_max_over_waves'])" || cat "$OUT/stamps_mw.json"; exit $rc
