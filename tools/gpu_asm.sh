#!/usr/bin/env bash
# A/B of the hand-scheduled FIFO loop (mcs_fifo_asm.hip) against the compiled kernel, then the
# FIFO parity suite.  Every GPU step has its own limit; a crash / timeout ends the script.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r02_asm}"
mkdir -p "$OUT"
cd "$ROOT"
export PYTHONUNBUFFERED=1
fatal() { case "$1" in 0|1) return 0 ;; *) echo "GPU step exited $1: stopping"; return 1 ;; esac; }
i=0
while IFS= read -r line; do
    [ -z "$line" ] && continue
    i=$((i+1))
    env_part="${line%%|*}"; args="${line#*|}"
    env $env_part timeout -k 10 300 python bench.py $args --no-cpu-baseline > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err"
    rc=$?
    python3 -c "
import json,sys
d=json.loads(open('$OUT/bench_$i.json').read().strip().splitlines()[-1])
print('$i', '$env_part', '$args', '%.4g'%d['value'], round(d['roofline']['kernel_ms_avg'],3), d.get('diagnostics',{}).get('loop_passes_per_job'), d.get('slot_pool_escalations'))" 2>/dev/null || tail -3 "$OUT/bench_$i.err"
    fatal $rc || exit $rc
done <<LIST
${BENCHES:-MCS_FIFO_ASM=1|--steps 5 --warmup 1
MCS_FIFO_ASM=0|--steps 5 --warmup 1}
LIST
if [ "${TESTS:-1}" = "1" ]; then
    timeout -k 10 900 python -u -m pytest ${TESTFILES:-tests/test_gpu_parity.py} -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
    rc=$?; tail -5 "$OUT/pytest.log"; echo "pytest rc=$rc"
fi
