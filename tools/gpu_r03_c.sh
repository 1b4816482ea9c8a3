#!/usr/bin/env bash
# Round 3: world-4 trading tests on one GPU (gloo) and the C5 tick loops side by side: one engine
# (graph-replayed ticks), the world-1 RCCL loop captured in a hipGraph, and the eager RCCL loop.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r03_c}"
mkdir -p "$OUT"
cd "$ROOT"
export PYTHONUNBUFFERED=1
fatal() { case "$1" in 0|1) return 0 ;; *) echo "GPU step exited $1: stopping"; return 1 ;; esac; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_trade.py tests/test_gpu_dtrade.py -k "four_ranks or two_ranks or rccl" -v --timeout 850 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_ranks.log" 2>&1
rc=$?; tail -12 "$OUT/pytest_ranks.log"; echo "pytest rc=$rc"; fatal $rc || exit $rc
i=0
while IFS= read -r line; do
    [ -z "$line" ] && continue
    i=$((i+1))
    env_part="${line%%|*}"; args="${line#*|}"
    env $env_part timeout -k 10 300 python bench.py $args > "$OUT/c5_$i.json" 2> "$OUT/c5_$i.err"
    rc=$?; echo "c5 $i ($env_part $args) rc=$rc"; python3 -c "
import json; d=json.loads(open('$OUT/c5_$i.json').read().strip().splitlines()[-1]); t=d['trading']
print('  %.4g' % d['value'], d['unit'], 'us/tick %.2f' % t['us_per_tick'], 'loop_form', t['loop_form'], 'ticks', t['ticks'])" 2>/dev/null || tail -3 "$OUT/c5_$i.err"
    fatal $rc || exit $rc
done <<LIST
${BENCHES:-MCS_RCCL_GRAPH=1|--config c5 --steps 1 --warmup 1 --no-cpu-baseline
MCS_RCCL_GRAPH=1|--config c5 --steps 1 --warmup 1 --no-cpu-baseline --comm
MCS_RCCL_GRAPH=0|--config c5 --steps 1 --warmup 1 --no-cpu-baseline --comm
MCS_RCCL_GRAPH=1|--config c5 --policy delay --steps 1 --warmup 1 --no-cpu-baseline
MCS_RCCL_GRAPH=1|--config c5 --policy delay --steps 1 --warmup 1 --no-cpu-baseline --comm
MCS_RCCL_GRAPH=0|--config c5 --policy delay --steps 1 --warmup 1 --no-cpu-baseline --comm}
LIST
echo done
