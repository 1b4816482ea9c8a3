#!/usr/bin/env bash
# DELAY-trading GPU parity tests (tests/test_gpu_dtrade.py), each run under its own time limit.
mkdir -p gpurun_out/dtrade
timeout -k 10 600 python -u -m pytest tests/test_gpu_dtrade.py -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/dtrade/pytest.log 2>&1
rc=$?; tail -25 gpurun_out/dtrade/pytest.log; exit $rc
