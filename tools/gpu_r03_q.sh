#!/usr/bin/env bash
# Segment stamps of the workgroup-resident tick on the full C5 system, and one PMC pass on a
# reduced C5 (instructions per tick).
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${TAG:-r03_q}"; mkdir -p "$OUT"
timeout -k 10 300 python -u tools/stamp_mw.py variants/libmcs_mw_stamps.so 156250 > "$OUT/stamps_mw.json" 2>&1
rc=$?; cat "$OUT/stamps_mw.json"; echo "stamps rc=$rc"; [ $rc -ne 0 ] && exit $rc
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES --kernel-trace --output-format csv \
    -d "$OUT/pmc_g1" -o pmc -- python3 "$ROOT/bench.py" --config c5 --jobs-per-cluster 20000 --steps 1 --warmup 0 --no-cpu-baseline ) > "$OUT/pmc_g1.log" 2>&1
rc=$?; echo "pmc rc=$rc"; exit $rc
