#!/usr/bin/env bash
# Trading GPU parity (FIFO borrow+trader and DELAY trading, incl. RCCL world-1 loops and the
# 2-rank gloo shards), then the C5-DELAY bench line.  Each step under its own time limit.
set -o pipefail
mkdir -p gpurun_out/trade_all
timeout -k 10 600 python -u -m pytest tests/test_gpu_trade.py tests/test_gpu_dtrade.py -x -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/trade_all/pytest.log 2>&1
rc=$?; tail -40 gpurun_out/trade_all/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c5 --policy delay --steps 3 --warmup 1 \
    > gpurun_out/trade_all/bench_c5d.json 2> gpurun_out/trade_all/bench_c5d.err
rc=$?; cat gpurun_out/trade_all/bench_c5d.json; exit $rc
