#!/usr/bin/env bash
# Instruction mix of the resident C5 tick kernel (two PMC passes on a reduced C5: 64 x 20000 jobs).
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r03_o}"; mkdir -p "$OUT"
gi=0
for ctr in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES"; do
  gi=$((gi+1))
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv \
      -d "$OUT/pmc_g$gi" -o pmc -- python3 "$ROOT/bench.py" --config c5 --jobs-per-cluster 20000 --steps 1 --warmup 0 --no-cpu-baseline ) > "$OUT/pmc_g$gi.log" 2>&1
  rc=$?; echo "pmc group $gi rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
find "$OUT" -name "*counter_collection.csv" | head; exit 0
