#!/usr/bin/env bash
# DELAY with Level1 filling (lambda < 1 job/s at 90 % memory load): the hand-scheduled loop with
# its hand-over vs the compiled delay_kernel alone, plus a kernel trace of the default.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r03_l1}"
mkdir -p "$OUT"; cd "$ROOT"
export PYTHONUNBUFFERED=1
L1ARGS="${L1ARGS:---policy delay --lam 0.95 --max-dur 972}"
echo "default start $(date +%T)"
timeout -k 10 300 python bench.py $L1ARGS --steps 5 --warmup 1 > "$OUT/l1_default.json" 2> "$OUT/l1_default.err" || exit $?
head -c 400 "$OUT/l1_default.json"; echo
echo "compiled start $(date +%T)"
MCS_DELAY_ASM=0 timeout -k 10 300 python bench.py $L1ARGS --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/l1_compiled.json" 2> "$OUT/l1_compiled.err" || exit $?
head -c 400 "$OUT/l1_compiled.json"; echo
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/prof_l1" -o k -- python3 "$ROOT/bench.py" $L1ARGS --steps 3 --warmup 1 --no-cpu-baseline ) > "$OUT/prof_l1.log" 2>&1 || exit $?
find "$OUT/prof_l1" -name "*kernel_trace.csv" -delete
find "$OUT/prof_l1" -name "*kernel_stats.csv" -exec head -6 {} \;
echo done
