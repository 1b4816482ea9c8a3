#!/usr/bin/env bash
# Resident tick with its cluster state in lanes: equality, stamps, C5 (release groups of 4 / 8 rows,
# 256-slot pool) against the replayed kernels.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
export TAG=r03_i PYTEST_K="resident or config5 or kats or seeded"
export BENCHES="MCS_TRADE_RESIDENT=1|--config c5 --steps 1 --warmup 1 --no-cpu-baseline
MCS_TRADE_RESIDENT=1 MCS_LIB=$ROOT/variants/libmcs_res_g8.so|--config c5 --steps 1 --warmup 1 --no-cpu-baseline
MCS_TRADE_RESIDENT=1|--config c5 --steps 1 --warmup 1 --no-cpu-baseline --slot-pool 4
MCS_TRADE_RESIDENT=0|--config c5 --steps 1 --warmup 1 --no-cpu-baseline"
bash tools/gpu_res.sh
