#!/usr/bin/env bash
# A/B of fifo_kernel variants: parity of each candidate (FIFO GPU tests through MCS_LIB), then
# interleaved timing (tools/ab_bench.py; env AB_TESTS picks the parity tests, AB_POLICY the workload).
#   usage: tools/gpu_ab.sh variants/libmcs_a.so variants/libmcs_b.so ...
mkdir -p gpurun_out/ab
for lib in "$@"; do
    MCS_LIB="$PWD/$lib" timeout -k 10 300 python -u -m pytest ${AB_TESTS:-tests/test_gpu_parity.py} -x -q --timeout 200 \
        --timeout-method thread -p no:cacheprovider > "gpurun_out/ab/$(basename $lib).log" 2>&1
    rc=$?; echo "$lib parity rc=$rc: $(tail -1 gpurun_out/ab/$(basename $lib).log)"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 600 python tools/ab_bench.py "$@" --rounds 3 --steps 5
