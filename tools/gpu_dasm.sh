#!/usr/bin/env bash
# The hand-scheduled DELAY loop: a quick parity check, the DELAY GPU suite, then interleaved A/B
# timing against the compiled delay_kernel (MCS_DELAY_ASM=0) on the C4 shape.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r03_d}"
mkdir -p "$OUT"
cd "$ROOT"
export PYTHONUNBUFFERED=1
LIB=multi-cluster-simulator_amd/mcs_amd/libmcs.so
timeout -k 10 120 python -u - > "$OUT/quick.log" 2>&1 <<'PY'
import sys
sys.path.insert(0, "multi-cluster-simulator_amd"); sys.path.insert(0, "tests")
import numpy as np
import oracle_ref as O
from kat_util import seeded_workload, fuzz_workload
from mcs_amd import Engine
for name, (arrays, streams) in (("n256", seeded_workload("n256", 16, 2000)[:2]), ("fuzz", fuzz_workload("w16r", 1, n_clusters=16, J=800))):
    with Engine(0, policy="DELAY") as eng:
        eng.load_clusters(arrays); eng.submit_jobs(streams); st = eng.run(); node, start, fin = eng.placements()
        cs = eng.cluster_stats(); ds = eng.delay_stats()
        print(name, "kernel", eng.last_kernel, "ms", st.kernel_ms)
    on, os_, of, od = O.delay_run_batch(arrays, streams, n_threads=8)
    bad = np.nonzero((node != on) | (start != os_) | (fin != of))[0]
    print(name, "mismatches", bad.size, bad[:10], node[bad[:5]], on[bad[:5]], start[bad[:5]], os_[bad[:5]])
    for f in ("t_end", "placed", "peak_running", "flags"):
        print(name, f, "ok" if np.array_equal(cs[f], od[f]) else ("BAD", cs[f][:8], od[f][:8]))
    for f in ("total_wait_ms", "jobs_count", "moved_l1"):
        print(name, f, "ok" if np.array_equal(ds[f], od[f]) else ("BAD", ds[f][:8], od[f][:8]))
PY
rc=$?; cat "$OUT/quick.log"; echo "quick rc=$rc"; [ $rc -ne 0 ] && exit $rc
grep -q "BAD" "$OUT/quick.log" && exit 3
grep -q "mismatches [1-9]" "$OUT/quick.log" && exit 3
timeout -k 10 900 python -u -m pytest tests/test_gpu_delay.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_delay.log" 2>&1
rc=$?; tail -5 "$OUT/pytest_delay.log"; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
for c in ${AB_SIZES:-4096 512}; do
  AB_POLICY=DELAY AB_CLUSTERS=$c timeout -k 10 600 python tools/ab_bench.py $LIB@MCS_DELAY_ASM=0 $LIB@MCS_DELAY_ASM=1 --rounds 3 --steps 5 > "$OUT/ab_delay_$c.txt" 2>&1
  rc=$?; echo "clusters $c"; cat "$OUT/ab_delay_$c.txt"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python bench.py --policy delay --steps 10 --warmup 2 > "$OUT/bench_delay.json" 2> "$OUT/bench_delay.err"; head -c 600 "$OUT/bench_delay.json"
echo done
