#!/usr/bin/env bash
# Round-2 GPU session: the given pytest targets, then optional bench lines.  Every GPU step has its
# own time limit; a crash / abort / timeout ends the script (no further GPU work in this call).
#   TESTS="tests/a.py tests/b.py" BENCHES="c4|--clusters 512" TAG=r02_x bash tools/gpu_r02.sh
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${TAG:-r02}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
export PYTHONUNBUFFERED=1
fatal() { case "$1" in 0|1) return 0 ;; *) echo "GPU step exited $1: stopping"; return 1 ;; esac; }
if [ -n "${TESTS:-}" ]; then
    echo "== pytest $TESTS"
    timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest $TESTS -m gpu -v -x --timeout ${PER_TEST:-300} \
        --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
    rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" "$OUT/pytest.log" | tail -60; echo "pytest rc=$rc"
    fatal $rc || exit $rc
fi
i=0
IFS='|' read -ra BL <<< "${BENCHES:-}"
for b in "${BL[@]}"; do
    [ -z "$b" ] && continue
    i=$((i+1))
    echo "== bench $b"
    timeout -k 10 600 python bench.py $b > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err"
    rc=$?; cat "$OUT/bench_$i.json"; tail -3 "$OUT/bench_$i.err"; echo "bench rc=$rc"; fatal $rc || exit $rc
done
echo "done $OUT"
