#!/usr/bin/env bash
# The one GPU script (run through gpurun): STEPS picks the steps, in order, each under its own time
# limit; a crash / abort / timeout ends the script (no further GPU work in this call).
#   TAG      output directory gpurun_out/$TAG
#   STEPS    any of: tests smoke benches prof pmc ab py trace   (default: tests smoke benches prof pmc)
#   PYTEST   pytest selection for `tests` (default: the whole -m gpu suite)
#   BENCHES  one bench.py argument line per bench (default: every headline line)
#   PROFS    name|bench args lines for rocprofv3 --kernel-trace --stats (per-dispatch traces dropped)
#   PMC_ARGS bench.py arguments of the PMC passes (default: the C4 headline shape)
#   PMC_GROUPS which counter groups (1 FETCH, 2 WRITE, 3-5 SQ/GRBM; default all)
#   AB       tools/ab_bench.py arguments (interleaved variant timing)
#   TRACES   name|bench args for `trace`: rocprofv3 --kernel-trace (TRACE_RT=1: + --runtime-trace) of
#            TRACE_BENCH (default bench.py; e.g. an older tree's under variants/), summarised by
#            tools/trace_gaps.py into $OUT/trace_<name>.json (the raw CSVs are deleted on the box)
#   PY       name|script args lines for `py`: python tools (stamp probes, traces) -> $OUT/py_<name>.txt
# Summaries go to profiles/ with tools/collect_profiles.py afterwards (on the CPU side).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-gpu}"
mkdir -p "$OUT"
cd "$ROOT"
export PYTHONUNBUFFERED=1
fatal() { case "$1" in 0|1) return 0 ;; *) echo "GPU step exited $1: stopping"; return 1 ;; esac; }
STEPS="${STEPS:-tests smoke benches prof pmc}"
for s in $STEPS; do
case "$s" in
tests)
    timeout -k 10 1000 python -u -m pytest ${PYTEST:-tests -m gpu} -q --timeout 400 --timeout-method thread \
        -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
    rc=$?; tail -4 "$OUT/pytest_gpu.log"; echo "pytest rc=$rc"; fatal $rc || exit $rc ;;
smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
    rc=$?; tail -3 "$OUT/smoke.log"; echo "smoke rc=$rc"; fatal $rc || exit $rc ;;
benches)
    i=0
    while IFS= read -r b; do
        [ -z "$b" ] && continue
        i=$((i+1))
        timeout -k 10 600 python bench.py $b > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err"
        rc=$?; echo "bench $i ($b) rc=$rc"; head -c 300 "$OUT/bench_$i.json"; echo; fatal $rc || exit $rc
    done <<LIST
${BENCHES:---gpus 1 --steps 20 --warmup 5
--clusters 2048 --steps 10 --warmup 2 --no-cpu-baseline
--clusters 1024 --steps 10 --warmup 2 --no-cpu-baseline
--clusters 512 --steps 10 --warmup 2 --no-cpu-baseline
--config c3 --steps 5 --warmup 1
--config c2 --steps 3 --warmup 1
--policy delay --steps 5 --warmup 1
--policy delay --lam 0.95 --max-dur 972 --steps 5 --warmup 1
--gen fused --steps 10 --warmup 2
--config c5 --steps 1 --warmup 1
--config c5 --comm --steps 1 --warmup 1
--config c5 --policy delay --steps 1 --warmup 1}
LIST
    ;;
prof)
    while IFS= read -r spec; do
        [ -z "$spec" ] && continue
        name="${spec%%|*}"; args="${spec#*|}"
        ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
            -d "$OUT/prof_$name" -o k -- python3 "$ROOT/bench.py" $args --no-cpu-baseline ) > "$OUT/prof_$name.log" 2>&1
        rc=$?; echo "prof $name rc=$rc"
        find "$OUT/prof_$name" -name "*kernel_trace.csv" -delete
        find "$OUT/prof_$name" -name "*kernel_stats.csv" -exec head -6 {} \;
        fatal $rc || exit $rc
    done <<LIST
${PROFS:-c4|--steps 3 --warmup 1
c4_512|--clusters 512 --steps 3 --warmup 1
delay_l1|--policy delay --lam 0.95 --max-dur 972 --steps 3 --warmup 1
c5|--config c5 --steps 1 --warmup 0
c5comm|--config c5 --comm --steps 1 --warmup 0}
LIST
    ;;
pmc)
    gi=0
    for ctr in "FETCH_SIZE" "WRITE_SIZE" \
               "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES" \
               "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
               "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU"; do
        gi=$((gi+1))
        case " ${PMC_GROUPS:-1 2 3 4 5} " in *" $gi "*) ;; *) continue ;; esac
        ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace \
            --output-format csv -d "$OUT/pmc_g$gi" -o pmc -- python3 "$ROOT/bench.py" ${PMC_ARGS:-} --steps 2 \
            --warmup 0 --no-cpu-baseline ) > "$OUT/pmc_g$gi.log" 2>&1
        rc=$?; echo "pmc group $gi rc=$rc"; fatal $rc || exit $rc
    done
    # the bench line of the same shape, for collect_profiles.py's traffic file
    timeout -k 10 300 python bench.py ${PMC_ARGS:-} --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
    rc=$?; echo "pmc bench rc=$rc"; fatal $rc || exit $rc ;;
ab)
    timeout -k 10 900 python -u tools/ab_bench.py $AB > "$OUT/ab.txt" 2>&1
    rc=$?; tail -12 "$OUT/ab.txt"; echo "ab rc=$rc"; fatal $rc || exit $rc ;;
trace)
    while IFS= read -r spec; do
        [ -z "$spec" ] && continue
        name="${spec%%|*}"; args="${spec#*|}"
        ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace ${TRACE_RT:+--runtime-trace} \
            --output-format csv -d "$OUT/trace_$name" -o t -- python3 "${TRACE_BENCH:-$ROOT/bench.py}" $args --no-cpu-baseline ) \
            > "$OUT/trace_$name.log" 2>&1
        rc=$?; echo "trace $name rc=$rc"
        python tools/trace_gaps.py "$OUT/trace_$name" "$OUT/trace_$name.log" > "$OUT/trace_$name.json" 2>&1
        head -c 2500 "$OUT/trace_$name.json"; echo
        rm -rf "$OUT/trace_$name"
        fatal $rc || exit $rc
    done <<LIST
${TRACES:-}
LIST
    ;;
py)
    while IFS= read -r spec; do
        [ -z "$spec" ] && continue
        name="${spec%%|*}"; args="${spec#*|}"
        timeout -k 10 600 python -u $args > "$OUT/py_$name.txt" 2>&1
        rc=$?; echo "py $name rc=$rc"; tail -40 "$OUT/py_$name.txt"; fatal $rc || exit $rc
    done <<LIST
${PY:-}
LIST
    ;;
esac
done
echo "done $OUT"
