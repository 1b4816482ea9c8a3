#!/usr/bin/env bash
# The duo loop at 512 clusters: segment stamps (duo vs W16R, header re-reads) and an A/B of the
# release wave polling flat out vs sleeping between idle polls.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/${TAG:-r03_n}"; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
for d in 1 0; do
  MCS_FIFO_DUO=$d timeout -k 10 200 python -u tools/stamp_fa.py variants/libmcs_stamps.so 512 > "$OUT/stamps_duo$d.txt" 2>&1
  rc=$?; cat "$OUT/stamps_duo$d.txt"; [ $rc -ne 0 ] && exit $rc
done
AB_CLUSTERS=512 timeout -k 10 400 python -u tools/ab_bench.py multi-cluster-simulator_amd/mcs_amd/libmcs.so@MCS_FIFO_DUO=1 \
  variants/libmcs_hsleep.so@MCS_FIFO_DUO=1 multi-cluster-simulator_amd/mcs_amd/libmcs.so@MCS_FIFO_DUO=0 --rounds 2 --steps 3 > "$OUT/ab_512.txt" 2>&1
rc=$?; cat "$OUT/ab_512.txt"; exit $rc
