#!/usr/bin/env bash
# Form T (finish-window slot rows) on the GPU: a small parity check first, the FIFO parity suite,
# then interleaved A/B timing against W16R (MCS_FIFO_T=0) at low occupancy.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r03_t}"
mkdir -p "$OUT"
cd "$ROOT"
export PYTHONUNBUFFERED=1
LIB=multi-cluster-simulator_amd/mcs_amd/libmcs.so
timeout -k 10 120 python -u - > "$OUT/quick.log" 2>&1 <<'PY'
import sys, os
sys.path.insert(0, "multi-cluster-simulator_amd"); sys.path.insert(0, "tests")
import numpy as np
import oracle_ref as O
from kat_util import seeded_workload
from mcs_amd import Engine
os.environ["MCS_FIFO_T"] = "2"
arrays, streams, _ = seeded_workload("n256", 16, 3000)
with Engine(0) as eng:
    eng.load_clusters(arrays); eng.submit_jobs(streams); st = eng.run(); node, start, fin = eng.placements()
    print("kernel", eng.last_kernel, "escalations", st.escalations, "ms", st.kernel_ms)
on, os_, of, osd = O.fifo_run_batch(arrays, streams, n_threads=8)
bad = np.nonzero((node != on) | (start != os_) | (fin != of))[0]
print("mismatches", bad.size, bad[:10], node[bad[:5]], on[bad[:5]], start[bad[:5]], os_[bad[:5]])
PY
rc=$?; cat "$OUT/quick.log"; echo "quick rc=$rc"; [ $rc -ne 0 ] && exit $rc
grep -q "mismatches 0 " "$OUT/quick.log" || exit 3
if [ "${TESTS:-1}" = "1" ]; then
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_parity.log" 2>&1
rc=$?; tail -5 "$OUT/pytest_parity.log"; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
fi
for c in ${AB_SIZES:-512 1024 2048 4096}; do
  AB_CLUSTERS=$c timeout -k 10 600 python tools/ab_bench.py $LIB@MCS_FIFO_T=0 $LIB@MCS_FIFO_T=2 --rounds 3 --steps 5 > "$OUT/ab_$c.txt" 2>&1
  rc=$?; echo "clusters $c"; cat "$OUT/ab_$c.txt"; [ $rc -ne 0 ] && exit $rc
done
echo done
