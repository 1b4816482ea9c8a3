#!/usr/bin/env bash
# DELAY-policy GPU session: parity tests, then (optionally) the DELAY bench line.
#   usage: tools/gpu_delay_tests.sh [bench]
mkdir -p gpurun_out/delay1
timeout -k 10 600 python -u -m pytest tests/test_gpu_delay.py -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/delay1/pytest.log 2>&1
rc=$?; tail -22 gpurun_out/delay1/pytest.log; [ $rc -ne 0 ] && exit $rc
if [ "${1:-}" = "bench" ]; then
    timeout -k 10 600 python bench.py --policy delay --steps 5 --warmup 1 --no-cpu-baseline \
        > gpurun_out/delay1/bench.json 2> gpurun_out/delay1/bench.err
    rc=$?; cat gpurun_out/delay1/bench.json; tail -3 gpurun_out/delay1/bench.err; exit $rc
fi
