"""Reproduce one tests/test_gpu_parity.py::test_hand_scheduled_fuzz case and print the first
mismatching cluster's details, with the hand-scheduled loop on and off (a debugging aid)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "multi-cluster-simulator_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import test_gpu_parity as T  # noqa: E402
import oracle_ref as O  # noqa: E402
from mcs_amd import Engine  # noqa: E402

shape, seed = sys.argv[1], int(sys.argv[2])
captured = {}
real_run_engine = T.run_engine


def fake_run_engine(eng, arrays, s):
    captured["arrays"], captured["s"] = arrays, s
    return real_run_engine(eng, arrays, s)


T.run_engine = fake_run_engine
T.assert_parity = lambda *a, **k: None
with Engine(0) as eng:
    T.test_hand_scheduled_fuzz(eng, shape, seed)
arrays, s = captured["arrays"], captured["s"]
on, os_, of, osd = O.fifo_run_batch(arrays, s, n_threads=8)
for asm in ("1", "0"):
    os.environ["MCS_FIFO_ASM"] = asm
    with Engine(0) as eng:
        eng.load_clusters(arrays)
        eng.submit_jobs(s)
        st = eng.run()
        node, start, fin = eng.placements()
        cs = eng.cluster_stats()
        k = eng.last_kernel
    bad = np.flatnonzero((node != on) | (start != os_) | (fin != of))
    print("MCS_FIFO_ASM", asm, k, "escalations", st.escalations, "pool", st.slot_pool, "mismatches", bad.size)
    if bad.size:
        off = s.job_off.astype(np.int64)
        c = int(np.searchsorted(off, bad[0], side="right") - 1)
        print(" cluster", c, "nodes", int(arrays.node_off[c + 1] - arrays.node_off[c]), "stats", cs[c], "oracle", osd[c])
        b = bad[:8]
        print(" jobs", (b - off[c]).tolist())
        print(" gpu node/start/fin", node[b].tolist(), start[b].tolist(), fin[b].tolist())
        print(" orc node/start/fin", on[b].tolist(), os_[b].tolist(), of[b].tolist())
        print(" arr/dur/c/m", s.arrival[b].tolist(), s.dur[b].tolist(), s.cores[b].tolist(), s.mem[b].tolist())
        print(" bad per cluster", np.bincount(np.searchsorted(off, bad, side="right") - 1).nonzero()[0].tolist())
