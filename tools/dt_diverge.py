"""Bounded divergence check of the DELAY-trading engine against the oracle on one seeded system:
the oracle's run sets t_max for the engine (so a run that would not end stops there), then the
first job whose placement differs is printed.  Diagnostic tool (GPU).
usage: python tools/dt_diverge.py kind C J"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "multi-cluster-simulator_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle_ref as O  # noqa: E402
from kat_util import seeded_workload  # noqa: E402
from mcs_amd import Engine  # noqa: E402

kind, C, J = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
arrays, streams, _ = seeded_workload(kind, C, J)
o = O.dtrade_run(arrays, streams)
print("oracle t_final", o["t_final"], flush=True)
with Engine(0, policy="DELAY", trader=True, t_max_s=int(o["t_final"]) + 100) as eng:
    eng.load_clusters(arrays)
    eng.submit_jobs(streams)
    st = eng.run()
    ts = eng.trade_stats()
    n, s, f = eng.placements()
print("gpu t_final", ts["t_final"], "flags", st.flags if hasattr(st, "flags") else None, flush=True)
bad = np.nonzero((n != o["node"]) | (s != o["start"]))[0]
print("mismatches", bad.size, flush=True)
if bad.size:
    i = int(bad[np.argmin(np.minimum(s[bad], o["start"][bad]))])
    print("earliest", i, "gpu", int(n[i]), int(s[i]), "oracle", int(o["node"][i]), int(o["start"][i]))
    print("first by index", bad[:10].tolist())
