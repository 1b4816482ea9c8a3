#!/usr/bin/env bash
# Workgroup-resident tick: granules in uncached (3), fine-grained (1) and plain (0) device memory.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${TAG:-r03_t2}"; mkdir -p "$OUT"
for m in 3 1 0; do
  MCS_MW_GX=$m timeout -k 10 300 python -u tools/stamp_mw.py variants/libmcs_mw_stamps.so 40000 > "$OUT/gx$m.json" 2>&1
  rc=$?; python3 -c "
import json; d=json.load(open('$OUT/gx$m.json')); print('gx $m', d['us_per_tick'], d['sweep_passes_per_tick_x1_x2_by_wg'], d['us_per_tick_wg0_wave0'])" || cat "$OUT/gx$m.json"; [ $rc -ne 0 ] && exit $rc
done
exit 0
