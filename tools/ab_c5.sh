#!/usr/bin/env bash
# Interleaved A/B of library variants on the C5 bench line (GPU):
#   bash tools/ab_c5.sh "<bench args>" variantA variantB ...   (variants/libmcs_<name>.so)
# writes gpurun_out/abc5_<name>_<round>.json; two rounds, A B A B ...
set -u
ARGS="$1"; shift
mkdir -p gpurun_out
for r in 1 2; do
  for v in "$@"; do
    MCS_LIB=variants/libmcs_$v.so timeout -k 10 300 python bench.py $ARGS --no-cpu-baseline > gpurun_out/abc5_${v}_$r.json 2>/dev/null || exit 1
    echo "$v $r $(grep -o '"us_per_tick": [0-9.]*' gpurun_out/abc5_${v}_$r.json)"
  done
done
