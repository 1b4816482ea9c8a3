#!/usr/bin/env bash
# rocprofv3 kernel statistics of one C5 run (FIFO trading, or DELAY trading with POLICY=delay).
set -u
OUT="$PWD/gpurun_out/${TAG:-c5prof}"
mkdir -p "$OUT"
ARGS="--config c5 --steps 1 --warmup 0 --no-cpu-baseline ${POLICY:+--policy $POLICY}"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/prof" -o k -- python3 "$GRAFT_REPO_ROOT/bench.py" $ARGS ) > "$OUT/prof.log" 2>&1
rc=$?; echo "prof rc=$rc"
find "$OUT/prof" -name "*kernel_trace.csv" -delete
find "$OUT/prof" -name "*kernel_stats.csv" -exec head -8 {} \;
exit $rc
