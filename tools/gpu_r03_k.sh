#!/usr/bin/env bash
# Session re-entry check at HEAD: the resident tick against the replayed kernels (quick equality),
# the whole GPU suite, smoke, and the headline / C5 / fused / DELAY bench lines.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
export TAG=${TAG:-r03_k} SKIP_PYTEST=1
export BENCHES="MCS_TRADE_RESIDENT=1|--config c5 --steps 1 --warmup 1 --no-cpu-baseline
MCS_TRADE_RESIDENT=0|--config c5 --steps 1 --warmup 1 --no-cpu-baseline"
bash tools/gpu_res.sh || exit $?
STEPS="tests smoke benches" BENCHES="--gpus 1 --steps 20 --warmup 5
--gen fused --steps 10 --warmup 2 --no-cpu-baseline
--policy delay --steps 5 --warmup 1 --no-cpu-baseline
--clusters 512 --steps 10 --warmup 2 --no-cpu-baseline
--config c5 --policy delay --steps 1 --warmup 1 --no-cpu-baseline" bash tools/gpu_r03.sh
