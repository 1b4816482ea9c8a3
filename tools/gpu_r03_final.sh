#!/usr/bin/env bash
# Round-3 final GPU session at HEAD: the whole GPU suite, smoke, every bench line (the driver's
# command first), rocprofv3 kernel traces of the headline / 512-cluster shard / C5 lines and the
# C4 PMC passes (traffic + instruction mix).  Every GPU step has its own time limit.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
export TAG=${TAG:-r03_final}
export BENCHES="--gpus 1 --steps 20 --warmup 5
--clusters 2048 --steps 10 --warmup 2 --no-cpu-baseline
--clusters 1024 --steps 10 --warmup 2 --no-cpu-baseline
--clusters 512 --steps 10 --warmup 2 --no-cpu-baseline
--config c3 --steps 5 --warmup 1
--config c2 --steps 3 --warmup 1
--policy delay --steps 5 --warmup 1
--gen fused --steps 10 --warmup 2
--config c5 --steps 1 --warmup 1
--config c5 --policy delay --steps 1 --warmup 1"
export PROFS="c4|--steps 3 --warmup 1
c4_512|--clusters 512 --steps 3 --warmup 1
c5|--config c5 --steps 1 --warmup 0"
STEPS="${STEPS:-tests smoke benches prof pmc}" bash tools/gpu_r03.sh
