#!/usr/bin/env bash
# Interleaved A/B of library variants on one bench line (GPU), each variant optionally with an
# environment setting:  bash tools/ab_dt.sh "<bench args>" ROUNDS name[@VAR=value] ...
# (variants/libmcs_<name>.so); writes gpurun_out/abdt_<name>_<round>.json and prints us_per_tick.
set -u
ARGS="$1"; ROUNDS="$2"; shift 2
mkdir -p gpurun_out
for r in $(seq 1 "$ROUNDS"); do
  for spec in "$@"; do
    v="${spec%%@*}"; tag="$(echo "$spec" | tr '@=' '__')"
    envs=(); [ "$spec" != "$v" ] && envs=("${spec#*@}")
    env "${envs[@]}" MCS_LIB=variants/libmcs_$v.so timeout -k 10 300 python bench.py $ARGS --no-cpu-baseline \
        > gpurun_out/abdt_${tag}_$r.json 2>/dev/null || exit 1
    echo "$spec $r $(grep -o '"us_per_tick": [0-9.]*' gpurun_out/abdt_${tag}_$r.json) $(grep -o '"loop_form": [0-9]*' gpurun_out/abdt_${tag}_$r.json)"
  done
done
