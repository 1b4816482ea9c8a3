# Full GPU check of the in-tree build (tests, smoke, bench) and, if given, an A/B of $AB_LIBS
# under $AB_POLICY (timing only; parity of the in-tree build is the test step).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r01_chk}
bash tools/gpu_check.sh $TAG ${STEPS:-tests smoke bench} || exit $?
if [ -n "${AB_LIBS:-}" ]; then
    timeout -k 10 600 python tools/ab_bench.py $AB_LIBS --rounds 3 --steps 5 > gpurun_out/$TAG/ab.log 2>&1
    rc=$?; cat gpurun_out/$TAG/ab.log; exit $rc
fi
