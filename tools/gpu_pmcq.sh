# Quick PMC instruction-mix passes of the C4 bench for one library ($1), one counter group per pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
LIB=$(realpath "$1"); OUT=gpurun_out/pmcq_$(basename $1 .so); mkdir -p $OUT
gi=0
for ctr in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
    gi=$((gi+1))
    ( cd /tmp && export TMPDIR=/tmp && MCS_LIB=$LIB timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace \
        --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/g$gi" -o pmc -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 \
        --warmup 0 --no-cpu-baseline ) > "$OUT/g$gi.log" 2>&1
    rc=$?; echo "pmcq group $gi rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/g$gi.log; exit $rc; }
done
exit 0
