#!/usr/bin/env bash
# The bench lines of $BENCHES ("ENV=.. ENV=..|bench args" per line) into gpurun_out/$TAG/bench_N.json,
# each under its own time limit; the first failure ends the call.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r03_g}"
mkdir -p "$OUT"
cd "$ROOT"
i=0
while IFS= read -r line; do
    [ -z "$line" ] && continue
    i=$((i+1))
    env_part="${line%%|*}"; args="${line#*|}"
    env $env_part timeout -k 10 300 python bench.py $args > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err"
    rc=$?; echo "bench $i ($env_part $args) rc=$rc"; python3 -c "
import json; d=json.loads(open('$OUT/bench_$i.json').read().strip().splitlines()[-1])
print('  %.4g' % d['value'], d['unit'], 'ms/step %.3f' % d['ms_per_step'], d.get('roofline', {}).get('kernel', ''), 'frac', d.get('roofline', {}).get('frac'), 'l1', d.get('diagnostics', {}).get('level1_moved_frac'))" 2>/dev/null || tail -3 "$OUT/bench_$i.err"
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