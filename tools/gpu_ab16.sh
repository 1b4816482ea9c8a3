#!/usr/bin/env bash
# The hand-scheduled loop's forms: tiny per-form cases, the FIFO parity suite on the new build,
# then C4 timing A/B of the forms over the occupancies a strong shard sees (16..1 waves per CU).
set -u
mkdir -p gpurun_out/ab16
timeout -k 10 240 python tools/asm_debug.py > gpurun_out/ab16/debug.txt 2>&1
rc=$?; echo "debug rc=$rc"; [ $rc -ne 0 ] && exit $rc
MCS_LIB="$PWD/${PARITY_LIB:-variants/libmcs_a17.so}" timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/ab16/parity.log 2>&1
rc=$?; tail -3 gpurun_out/ab16/parity.log; echo "parity rc=$rc"; [ $rc -ne 0 ] && exit $rc
LIBS=${LIBS:-"variants/libmcs_a17.so@MCS_FIFO_ASM=16 variants/libmcs_a17.so@MCS_FIFO_ASM=17"}
for nc in ${CLUSTERS:-4096 2048 1024 512 256}; do
    echo "== $nc clusters"
    AB_CLUSTERS=$nc timeout -k 10 600 python tools/ab_bench.py $LIBS --rounds ${ROUNDS:-2} --steps 3 | tee gpurun_out/ab16/ab$nc.txt
    rc=$?; [ $rc -ne 0 ] && exit $rc
done
exit 0
