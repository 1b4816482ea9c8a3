#!/usr/bin/env bash
# The fused suite (straddling-window fix + compiler barrier in GenStream's scratch search), the duo
# loop's parity cases (a decision and a release wave per cluster), then the duo / W16R A/B at the
# strong-shard sizes.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${TAG:-r03_m}"; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_fused.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_fused.log"; echo "pytest fused rc=$rc"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -v -x -k "hand_scheduled or every_kernel or config4_shape or heterogeneous or escalation or field_bounds" \
    --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_duo.log" 2>&1
rc=$?; tail -5 "$OUT/pytest_duo.log"; echo "pytest duo rc=$rc"; [ $rc -ne 0 ] && exit $rc
for n in 512 1024 2048; do for d in 0 1; do
  MCS_FIFO_DUO=$d timeout -k 10 200 python bench.py --clusters $n --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/ab_${n}_$d.json" 2> "$OUT/ab_${n}_$d.err"
  rc=$?; python3 -c "
import json; d=json.loads(open('$OUT/ab_${n}_$d.json').read().strip().splitlines()[-1])
print('$n duo=$d', '%.4g' % d['value'], 'ms/step %.3f' % d['ms_per_step'], d['roofline'].get('kernel'))" 2>/dev/null || tail -3 "$OUT/ab_${n}_$d.err"
  [ $rc -ne 0 ] && exit $rc
done; done
timeout -k 10 300 python -u tools/stamp_res.py variants/libmcs_res_stamps.so 156250 > "$OUT/stamps_res.json" 2>&1
rc=$?; cat "$OUT/stamps_res.json"; echo "stamps rc=$rc"
