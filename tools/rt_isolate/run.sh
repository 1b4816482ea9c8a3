#!/usr/bin/env bash
# The rocprofv3 --runtime-trace exit-fault isolation, run through
# gpurun.  Each leg runs once bare (the control) and once under the exact profiler command of
# profiles/r05_g1/trace_c5d_comm.log, with the program itself after `--`; the exit status of every
# run is recorded in $OUT/summary.txt.  A leg's profiled exit status is data, not a failure of this
# script, but a timeout (124/137) ends it: no GPU step follows a hang.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-rt_isolate}"
mkdir -p "$OUT"
cd "$ROOT"
export PYTHONUNBUFFERED=1
: > "$OUT/summary.txt"
leg() {   # leg NAME PROGRAM ARGS...
    local name="$1"; shift
    timeout -k 10 240 "$@" > "$OUT/${name}_bare.log" 2>&1
    local rb=$?
    ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --runtime-trace \
        --output-format csv -d "$OUT/trace_$name" -o t -- "$@" ) > "$OUT/${name}_rt.log" 2>&1
    local rt=$?
    rm -rf "$OUT/trace_$name"
    echo "$name bare=$rb runtime_trace=$rt" | tee -a "$OUT/summary.txt"
    case "$rb $rt" in *124*|*137*) echo "timeout: stopping"; exit 1 ;; esac
}
# LEGS picks the legs (default: the four of the first pass, profiles/r06_rt/)
for l in ${LEGS:-comm_only torch_nccl mcs_run_notorch torch_mcs_run}; do
    case "$l" in
    comm_only) leg comm_only "$ROOT/tools/rt_isolate/comm_only" ;;
    graph_only) leg graph_only "$ROOT/tools/rt_isolate/graph_only" ;;
    bench_c5d_comm) leg bench_c5d_comm python3 "$ROOT/bench.py" --config c5 --policy delay --comm \
                        --jobs-per-cluster 200 --steps 1 --warmup 0 --no-cpu-baseline ;;
    bench_c5d) leg bench_c5d python3 "$ROOT/bench.py" --config c5 --policy delay \
                   --jobs-per-cluster 200 --steps 1 --warmup 0 --no-cpu-baseline ;;
    bench_c5d_maps) export MCS_BENCH_EXIT_MAPS="$OUT/bench_c5d_maps.txt"
                    leg bench_c5d_maps python3 "$ROOT/bench.py" --config c5 --policy delay \
                        --jobs-per-cluster 200 --steps 1 --warmup 0 --no-cpu-baseline
                    unset MCS_BENCH_EXIT_MAPS ;;
    bench_c4_small) leg bench_c4_small python3 "$ROOT/bench.py" --clusters 256 --jobs-per-cluster 2048 \
                   --steps 1 --warmup 0 --no-cpu-baseline ;;
    *) leg "$l" python3 "$ROOT/tools/rt_isolate/py_steps.py" "$l" ;;
    esac
done
echo "done $OUT"
