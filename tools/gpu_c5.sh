#!/usr/bin/env bash
# Trading parity suites, then the C5 bench lines (FIFO and DELAY trading) on the in-tree library.
set -u
OUT=gpurun_out/${TAG:-c5}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_trade.py tests/test_gpu_dtrade.py -x -q --timeout 400 \
    --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/b7.json" || exit $?
timeout -k 10 300 python bench.py --config c5 --policy delay --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/b8.json" || exit $?
python3 - "$OUT" <<'PY'
import json, sys
for f in ("b7", "b8"):
    d = json.loads(open(f"{sys.argv[1]}/{f}.json").read().strip().splitlines()[-1])
    print(f, "%.4g" % d["value"], round(d["ms_per_step"], 1), d.get("trading", {}).get("us_per_tick"))
PY
exit 0
