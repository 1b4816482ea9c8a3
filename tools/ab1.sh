# A/B of the fifo_kernel variants named in $AB_LIBS (parity first, then interleaved timing)
set -o pipefail
cd $GRAFT_REPO_ROOT
export AB_TESTS=${AB_TESTS:-tests/test_gpu_parity.py}
bash tools/gpu_ab.sh $AB_LIBS > gpurun_out/ab1.log 2>&1
rc=$?; cat gpurun_out/ab1.log; exit $rc
