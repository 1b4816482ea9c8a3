"""Engine lifecycle with an RCCL communicator, in child processes so the exit path itself is checked:
create a world-1 communicator, run both trading systems through their RCCL tick loops (captured in a
hipGraph and eager), destroy the engine and exit — the process must exit 0 (no fault in the teardown
order of graphs, communicator, device memory, or in the libraries' static destructors at exit).
DESIGN.md §15 records the r04 exit-time SIGSEGV this pins."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import os, sys
sys.path.insert(0, os.path.join(os.environ["REPO"], "multi-cluster-simulator_amd"))
sys.path.insert(0, os.path.join(os.environ["REPO"], "tests"))
if os.environ.get("WITH_TORCH") == "1":
    import torch  # bench.py's order: torch's librccl is the one libmcs binds
from kat_util import seeded_workload
from mcs_amd import Engine
policy = os.environ["POLICY"]
kind, C, J = ("small", 16, 300) if policy == "DELAY" else ("n64_hot", 8, 800)
arrays, streams, _ = seeded_workload(kind, C, J)
for rep in range(2):  # twice: a second communicator after the first was destroyed
    eng = Engine(0, policy=policy, trader=True, **({} if policy == "DELAY" else {"borrow": True, "t_max_s": 20_000_000}))
    eng.load_clusters(arrays)
    eng.set_shard(0, 1)
    eng.comm_init(Engine.comm_unique_id())
    eng.submit_jobs(streams)
    st = eng.run()
    assert st.placed > 0, st
    eng.close()
print("TEARDOWN OK", flush=True)
'''


@pytest.mark.gpu
@pytest.mark.parametrize("policy", ["FIFO", "DELAY"])
@pytest.mark.parametrize("graph", ["1", "0"])
@pytest.mark.parametrize("with_torch", ["0", "1"])
def test_rccl_engine_lifecycle_exits_cleanly(policy, graph, with_torch):
    env = dict(os.environ, REPO=REPO, POLICY=policy, MCS_RCCL_GRAPH=graph, WITH_TORCH=with_torch)
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
    assert "TEARDOWN OK" in r.stdout


REINIT = r'''
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.environ["REPO"], "multi-cluster-simulator_amd"))
sys.path.insert(0, os.path.join(os.environ["REPO"], "tests"))
from kat_util import seeded_workload
from mcs_amd import Engine
policy = os.environ["POLICY"]
kind, C, J = ("small", 16, 300) if policy == "DELAY" else ("n64_hot", 8, 800)
arrays, streams, _ = seeded_workload(kind, C, J)
kw = {} if policy == "DELAY" else {"borrow": True, "t_max_s": 20_000_000}
with Engine(0, policy=policy, trader=True, **kw) as eng:
    eng.load_clusters(arrays)
    eng.set_shard(0, 1)
    eng.submit_jobs(streams)
    eng.run()  # no communicator: the HBM tick loop
    want = eng.placements()
    forms = [eng.trade_stats()["loop_form"]]
    for rep in range(2):  # a communicator, then a re-initialised one: run() replays nothing of the old
        eng.comm_init(Engine.comm_unique_id())
        eng.run()
        forms.append(eng.trade_stats()["loop_form"])
        for a, b in zip(eng.placements(), want):
            np.testing.assert_array_equal(a, b)
print("REINIT OK", forms, flush=True)
'''


@pytest.mark.gpu
@pytest.mark.parametrize("policy", ["FIFO", "DELAY"])
def test_comm_reinit_between_runs(policy):
    """mcs_comm_init on an engine that already ran (locally, then over a communicator) releases the
    captured tick graphs, finalizes the old communicator and drops the trading state before the new
    communicator exists, so the next run captures against the new one and agrees on its shape again;
    every run's placements are equal and the process exits 0."""
    env = dict(os.environ, REPO=REPO, POLICY=policy)
    r = subprocess.run([sys.executable, "-c", REINIT], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
    assert "REINIT OK" in r.stdout
