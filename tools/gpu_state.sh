#!/usr/bin/env bash
# ClusterState reduction: GPU parity tests, its measurement, a rocprofv3 kernel-stats pass and two
# PMC passes (FETCH_SIZE, WRITE_SIZE) for its HBM traffic.  usage: tools/gpu_state.sh [notests]
set -o pipefail
ROOT=$(pwd); out=$ROOT/gpurun_out/state; mkdir -p $out
if [ "${1:-}" != "notests" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_state.py -x -v --timeout 200 --timeout-method thread \
      -p no:cacheprovider > $out/pytest.log 2>&1
  rc=$?; tail -6 $out/pytest.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 python tools/bench_state.py > $out/bench_state.json 2> $out/bench_state.err || exit $?
cat $out/bench_state.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o state -- \
    python3 $ROOT/tools/bench_state.py --steps 10 > $out/prof.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $out/pmc_$c -o pmc -- \
      python3 $ROOT/tools/bench_state.py --steps 2 > $out/pmc_$c.log 2>&1 || exit $?
done
find $out/prof -name "*kernel_stats.csv" -exec cp {} $out/kernel_stats.csv \;
head -4 $out/kernel_stats.csv
