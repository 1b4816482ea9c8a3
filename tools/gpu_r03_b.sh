TAG=r03_b STEPS="prof pmc" PROFS="c4|--steps 3 --warmup 1
c4_512|--clusters 512 --steps 3 --warmup 1" bash tools/gpu_r03.sh && TAG=r03_b512 STEPS=pmc PMC_ARGS="--clusters 512" bash tools/gpu_r03.sh && timeout -k 10 300 python tools/stamp_fa.py variants/libmcs_stamps.so 256 512 1024 4096 > gpurun_out/r03_b/stamps.txt 2>&1; cat gpurun_out/r03_b/stamps.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_trade.py tests/test_gpu_dtrade.py -k rccl -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_b/rccl.log 2>&1; tail -8 gpurun_out/r03_b/rccl.log
