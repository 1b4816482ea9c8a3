#!/usr/bin/env bash
# One GPU-box session: parity tests, smoke, a short bench and a rocprofv3 kernel-trace profile.
# Every GPU step has its own time limit; any crash / abort / timeout stops the script (no further
# GPU work in this call).  Plain test failures (pytest rc 1) do not stop the later steps.
#   usage: tools/gpu_check.sh [tag] [steps...]   steps: tests smoke bench prof pmc
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r01}"
shift || true
STEPS="${*:-tests smoke bench prof}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
export PYTHONUNBUFFERED=1
BENCH_ARGS="${BENCH_ARGS:-}"
C5_ARGS="${C5_ARGS:-}"

fatal() {  # rc of a GPU step -> 0 continue, 1 stop
    case "$1" in
        0|1) return 0 ;;
        *) echo "GPU step exited $1: stopping (no further GPU work in this call)"; return 1 ;;
    esac
}

for s in $STEPS; do
    case "$s" in
    tests)
        echo "== pytest -m gpu"
        timeout -k 10 840 python -m pytest tests -m gpu -q --timeout 400 -p no:cacheprovider \
            > "$OUT/pytest_gpu.log" 2>&1
        rc=$?; tail -25 "$OUT/pytest_gpu.log"; echo "pytest rc=$rc"; fatal $rc || exit $rc ;;
    tradetests)
        echo "== pytest -m gpu tests/test_gpu_trade.py"
        timeout -k 10 600 python -m pytest tests/test_gpu_trade.py -m gpu -q --timeout 400 -p no:cacheprovider \
            > "$OUT/pytest_trade.log" 2>&1
        rc=$?; tail -25 "$OUT/pytest_trade.log"; echo "pytest rc=$rc"; fatal $rc || exit $rc ;;
    c5)
        echo "== bench C5 (lock-step trading)"
        timeout -k 10 900 python bench.py --config c5 --steps 1 --warmup 1 $C5_ARGS > "$OUT/bench_c5.json" \
            2> "$OUT/bench_c5.err"
        rc=$?; cat "$OUT/bench_c5.json"; tail -5 "$OUT/bench_c5.err"; echo "c5 rc=$rc"; fatal $rc || exit $rc ;;
    c5prof)
        echo "== rocprofv3 kernel trace, C5"
        ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats \
            --output-format csv -d "$OUT/prof_c5" -o c5 -- python3 "$ROOT/bench.py" --config c5 --steps 1 \
            --warmup 0 --no-cpu-baseline $C5_ARGS ) > "$OUT/prof_c5.log" 2>&1
        rc=$?; tail -5 "$OUT/prof_c5.log"; echo "c5prof rc=$rc"
        find "$OUT/prof_c5" -name "*stats*.csv" -exec sh -c 'echo "--- $1"; head -20 "$1"' _ {} \;
        fatal $rc || exit $rc ;;
    smoke)
        echo "== smoke"
        timeout -k 10 600 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
        rc=$?; tail -5 "$OUT/smoke.log"; echo "smoke rc=$rc"; fatal $rc || exit $rc ;;
    bench)
        echo "== bench"
        timeout -k 10 900 python bench.py --steps 5 --warmup 1 $BENCH_ARGS > "$OUT/bench.json" 2> "$OUT/bench.err"
        rc=$?; cat "$OUT/bench.json"; tail -5 "$OUT/bench.err"; echo "bench rc=$rc"; fatal $rc || exit $rc ;;
    prof)
        echo "== rocprofv3 kernel trace"
        ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats \
            --output-format csv -d "$OUT/prof" -o bench -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 \
            --no-cpu-baseline $BENCH_ARGS ) > "$OUT/prof.log" 2>&1
        rc=$?; tail -5 "$OUT/prof.log"; echo "prof rc=$rc"
        find "$OUT/prof" -name "*stats*.csv" -exec sh -c 'echo "--- $1"; head -20 "$1"' _ {} \;
        fatal $rc || exit $rc ;;
    pmc)
        echo "== rocprofv3 PMC passes (one counter group per pass; no tracing domains combined)"
        gi=0
        for ctr in "FETCH_SIZE" "WRITE_SIZE" \
                   "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES" \
                   "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
                   "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU"; do
            gi=$((gi+1))
            ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --pmc $ctr --kernel-trace \
                --output-format csv -d "$OUT/pmc_g$gi" -o pmc -- python3 "$ROOT/bench.py" --steps 1 \
                --warmup 0 --no-cpu-baseline $BENCH_ARGS ) > "$OUT/pmc_g$gi.log" 2>&1
            rc=$?; tail -3 "$OUT/pmc_g$gi.log"; echo "pmc group $gi ($ctr) rc=$rc"; fatal $rc || exit $rc
        done ;;
    pmcq)
        echo "== rocprofv3 PMC quick (instruction mix + wait states)"
        gi=0
        for ctr in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES" \
                   "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
            gi=$((gi+1))
            ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --pmc $ctr --kernel-trace \
                --output-format csv -d "$OUT/pmcq_g$gi" -o pmc -- python3 "$ROOT/bench.py" --steps 1 \
                --warmup 0 --no-cpu-baseline $BENCH_ARGS ) > "$OUT/pmcq_g$gi.log" 2>&1
            rc=$?; echo "pmcq group $gi rc=$rc"; fatal $rc || exit $rc
        done ;;
    *) echo "unknown step $s" ;;
    esac
done
echo "done: $OUT"
