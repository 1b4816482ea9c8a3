#!/usr/bin/env bash
# The workgroup-resident tick (mcs_trade_mw.hip): a quick equality check against the replayed
# kernels, the FIFO trading GPU suite, then C5 under each tick loop.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${TAG:-r03_p}"; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 120 python -u - > "$OUT/quick.log" 2>&1 <<'PY'
import os, sys
sys.path.insert(0, "multi-cluster-simulator_amd"); sys.path.insert(0, "tests")
from kat_util import seeded_workload
from mcs_amd import Engine
arrays, streams, _ = seeded_workload("n64_hot", 8, 1500)
out = {}
for mode in ("2", "0"):
    os.environ["MCS_TRADE_RESIDENT"] = mode
    with Engine(0, borrow=True, trader=True, t_max_s=20_000_000) as eng:
        eng.load_clusters(arrays); eng.submit_jobs(streams); st = eng.run()
        out[mode] = (eng.placements(), eng.trade_stats(), st.kernel_ms)
    print(mode, out[mode][1]["loop_form"], out[mode][1]["ticks"], out[mode][1]["t_final"], "ms", out[mode][2], flush=True)
a, b = out["2"][0], out["0"][0]
bad = [int((a[i] != b[i]).sum()) for i in range(3)]
print("mismatches", bad, "flags", out["2"][1]["flags"], out["0"][1]["flags"])
PY
rc=$?; cat "$OUT/quick.log"; echo "quick rc=$rc"; [ $rc -ne 0 ] && exit $rc
grep -q "mismatches \[0, 0, 0\]" "$OUT/quick.log" || exit 3
timeout -k 10 900 python -u -m pytest tests/test_gpu_trade.py -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_trade.log" 2>&1
rc=$?; tail -5 "$OUT/pytest_trade.log"; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
i=0
for mode in 2 1; do
  i=$((i+1))
  MCS_TRADE_RESIDENT=$mode timeout -k 10 300 python bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/c5_$mode.json" 2> "$OUT/c5_$mode.err"
  rc=$?; echo "c5 mode $mode rc=$rc"; python3 -c "
import json; d=json.loads(open('$OUT/c5_$mode.json').read().strip().splitlines()[-1]); t=d['trading']
print('  %.4g' % d['value'], d['unit'], 'us/tick %.2f' % t['us_per_tick'], 'loop_form', t['loop_form'], 'ticks', t['ticks'], 'flags', t['flags'])" 2>/dev/null || tail -3 "$OUT/c5_$mode.err"
  [ $rc -ne 0 ] && exit $rc
done
echo done
