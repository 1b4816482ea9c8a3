#!/usr/bin/env bash
# Fused-generation GPU session: the whole GPU suite, then the C4 bench streamed vs fused (FIFO, DELAY).
set -o pipefail
out=gpurun_out/fused; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $out/pytest_gpu.log 2>&1
rc=$?; tail -8 $out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for pol in fifo delay; do
  for gen in stream fused; do
    timeout -k 10 300 python bench.py --policy $pol --gen $gen --steps 5 --warmup 1 --no-cpu-baseline \
        > $out/bench_${pol}_${gen}.json 2> $out/bench_${pol}_${gen}.err || exit $?
    cut -c1-400 $out/bench_${pol}_${gen}.json
  done
done
