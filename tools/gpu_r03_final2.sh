#!/usr/bin/env bash
# Round-3 end state at HEAD: the whole GPU suite, smoke, every bench line (the driver's command
# first; the Level1-heavy DELAY stream added), rocprofv3 kernel traces of the headline, the
# 512-cluster shard, C5 and the Level1-heavy DELAY line, and the C4 PMC passes.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
export TAG=${TAG:-r03_final2}
export BENCHES="--gpus 1 --steps 20 --warmup 5
--clusters 2048 --steps 10 --warmup 2 --no-cpu-baseline
--clusters 1024 --steps 10 --warmup 2 --no-cpu-baseline
--clusters 512 --steps 10 --warmup 2 --no-cpu-baseline
--config c3 --steps 5 --warmup 1
--config c2 --steps 3 --warmup 1
--policy delay --steps 5 --warmup 1
--policy delay --lam 0.95 --max-dur 972 --steps 5 --warmup 1
--gen fused --steps 10 --warmup 2
--config c5 --steps 1 --warmup 1
--config c5 --policy delay --steps 1 --warmup 1"
export PROFS="c4|--steps 3 --warmup 1
c4_512|--clusters 512 --steps 3 --warmup 1
delay_l1|--policy delay --lam 0.95 --max-dur 972 --steps 3 --warmup 1
c5|--config c5 --steps 1 --warmup 0"
STEPS="${STEPS:-tests smoke benches prof pmc}" bash tools/gpu_r03.sh
