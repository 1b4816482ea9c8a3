#!/usr/bin/env bash
# Workgroup-resident tick: stamps with sweep-pass counts, agent-scope (sc1) vs system-scope (sc0 sc1)
# granule loads.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${TAG:-r03_s}"; mkdir -p "$OUT"
for v in mw_stamps mw_stamps_sys; do
  timeout -k 10 300 python -u tools/stamp_mw.py variants/libmcs_$v.so 40000 > "$OUT/$v.json" 2>&1
  rc=$?; python3 -c "
import json; d=json.load(open('$OUT/$v.json')); print('$v', d['us_per_tick'], d['sweep_passes_per_tick_x1_x2_by_wg'], d['us_per_tick_wg0_wave0'])"; [ $rc -ne 0 ] && exit $rc
done
exit 0
