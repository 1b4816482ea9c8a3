"""Repeatability of the one-launch trading tick (mcs_trade_rk.hip): one seeded fuzz system run several
times through the caller-driven path (world 1) and the RCCL loop, each compared with the oracle.
usage: python tools/rk_repeat.py [shape seed reps]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "multi-cluster-simulator_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
os.environ.setdefault("MCS_TRADE_RK", "1")
import numpy as np  # noqa: E402

import oracle_ref as O  # noqa: E402
from kat_util import fuzz_workload  # noqa: E402
from mcs_amd import Engine  # noqa: E402
from mcs_amd.shard import run_lockstep  # noqa: E402

shape = sys.argv[1] if len(sys.argv) > 1 else "w16r"
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 9
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 4
arrays, streams = fuzz_workload(shape, seed, n_clusters=12, J=500, blocking=False)
o = O.trade_run(arrays, streams)


def run(mode):
    with Engine(0, borrow=True, trader=True, t_max_s=20_000_000) as eng:
        eng.load_clusters(arrays)
        if mode == "rccl":
            eng.set_shard(0, 1)
            eng.comm_init(Engine.comm_unique_id())
        eng.submit_jobs(streams)
        if mode == "driven":
            run_lockstep(eng, lambda b: b)
        else:
            eng.run()
        node, start, fin = eng.placements()
        return node, start, fin, eng.trade_stats()


for mode in ("driven", "rccl", "driven", "rccl"):
    for r in range(reps):
        node, start, fin, ts = run(mode)
        bad = np.flatnonzero((node != o["node"]) | (start != o["start"]) | (fin != o["finish"]))
        print(mode, r, "loop_form", ts["loop_form"], "ticks", ts["ticks"], "t_final", ts["t_final"], "oracle t_final",
              o["t_final"], "mismatches", bad.size, bad[:6].tolist(),
              "gpu start", start[bad[:3]].tolist(), "oracle", o["start"][bad[:3]].tolist(), flush=True)
