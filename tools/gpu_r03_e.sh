#!/usr/bin/env bash
# HEAD check: the whole GPU suite, smoke, the DELAY line's kernel trace and PMC passes.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${TAG:-r03_e} STEPS="tests smoke" bash tools/gpu_r03.sh || exit $?
TAG=${TAG:-r03_e} STEPS="prof" PROFS="delay|--policy delay --steps 3 --warmup 1" bash tools/gpu_r03.sh || exit $?
TAG=${TAG:-r03_e}_delay STEPS="pmc" PMC_ARGS="--policy delay" bash tools/gpu_r03.sh || exit $?
