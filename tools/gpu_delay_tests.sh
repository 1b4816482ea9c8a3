mkdir -p gpurun_out/delay1
timeout -k 10 600 python -u -m pytest tests/test_gpu_delay.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/delay1/pytest.log 2>&1
rc=$?; tail -30 gpurun_out/delay1/pytest.log; exit $rc
