#!/usr/bin/env bash
# PMC passes (SQ instruction / wait counters) of one bench launch, env passed through.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r02_asmpmc}"
mkdir -p "$OUT"
gi=0
for ctr in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU"; do
    gi=$((gi+1))
    ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace \
        --output-format csv -d "$OUT/pmc_g$gi" -o pmc -- python3 "$ROOT/bench.py" --steps 1 \
        --warmup 0 --no-cpu-baseline ${BARGS:-} ) > "$OUT/pmc_g$gi.log" 2>&1
    rc=$?; echo "pmc group $gi rc=$rc"
    case $rc in 0|1) ;; *) exit $rc ;; esac
done
