#!/usr/bin/env bash
# r06 GPU steps for the W16T tracked-insert loop: its parity tests, then interleaved A/B medians
# against W16R on the 4096-cluster headline grid and the 512-cluster shard (same library,
# MCS_FIFO_TRACK=0|1).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
LIB=multi-cluster-simulator_amd/mcs_amd/libmcs.so
TAG=r06_track STEPS=tests PYTEST="tests/test_gpu_parity.py -m gpu -k track" bash tools/gpu.sh || exit 1
for nc in ${TRACK_AB_CLUSTERS:-4096 512}; do
    AB_CLUSTERS=$nc TAG=r06_track/ab$nc STEPS=ab AB="$LIB@MCS_FIFO_TRACK=0 $LIB@MCS_FIFO_TRACK=1 --rounds 3 --steps 5" \
        bash tools/gpu.sh || exit 1
done
