#!/usr/bin/env bash
# r06 GPU steps for the W16L lookahead loop: its parity tests, then interleaved
# A/B medians against W16R on the 512- and 1024-cluster strong shards and the 4096-cluster headline
# grid (same library, MCS_FIFO_LOOK=0|1), then the rt-isolation legs.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
LIB=multi-cluster-simulator_amd/mcs_amd/libmcs.so
TAG=r06_look STEPS=tests PYTEST="tests/test_gpu_parity.py -m gpu -k look" bash tools/gpu.sh || exit 1
for nc in ${LOOK_AB_CLUSTERS:-512 1024}; do
    AB_CLUSTERS=$nc TAG=r06_look/ab$nc STEPS=ab AB="$LIB@MCS_FIFO_LOOK=0 $LIB@MCS_FIFO_LOOK=1 --rounds 3 --steps 5" \
        bash tools/gpu.sh || exit 1
done
if [ -n "${RT_LEGS:-}" ]; then
    TAG=r06_rt2 LEGS="$RT_LEGS" bash tools/rt_isolate/run.sh || exit 1
fi
