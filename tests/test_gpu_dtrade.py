"""GPU parity of the lock-step trading system with DELAY schedulers (mcs_dtrade.hip through the
C ABI, policy MCS_POLICY_DELAY + trader) against the CPU oracle (oracle/mcs_oracle_dtrade.c) and the
hand-derived scenarios of tests/golden/kats_dtrade.json: placements (virtual nodes included),
every trader round with its contract, every Foreign job, the virtual-node capacities and the
WaitTime statistics, bit-exact.  Run on a real MI355X."""
import json
import os

import numpy as np
import pytest

import oracle_ref as O
from kat_util import GOLDEN, seeded_workload
from mcs_amd import Engine
from test_dtrade_oracle import check_kat, dt_system

pytestmark = pytest.mark.gpu
DT = json.load(open(os.path.join(GOLDEN, "kats_dtrade.json")))["dtrade"]


def run(arrays, streams, **cfg):
    with Engine(0, policy="DELAY", trader=True, **cfg) as eng:
        eng.load_clusters(arrays)
        eng.submit_jobs(streams)
        st = eng.run()
        node, start, fin = eng.placements()
        out = dict(node=node, start=start, finish=fin, trades=eng.contracts(), foreign=eng.foreign(),
                   vnodes=[eng.virtual_node_caps(c) for c in range(arrays.n_clusters)], ds=eng.delay_stats(),
                   ts=eng.trade_stats(), stats=st)
    return out


@pytest.mark.parametrize("k", DT, ids=[k["name"] for k in DT])
def test_gpu_dtrade_kats(k):
    arrays, s = dt_system(k)
    r = run(arrays, s, t_max_s=k["t_max"])
    check_kat(k, r["node"], r["start"], r["finish"], r["trades"], r["foreign"], len(r["foreign"]), r["vnodes"],
              r["ts"]["t_final"])


@pytest.mark.parametrize("kind,C,J", [("small", 8, 300), ("small", 16, 600), ("big", 8, 800), ("n64_hot", 8, 2000)])
def test_gpu_dtrade_seeded_parity(kind, C, J):
    arrays, streams, _ = seeded_workload(kind, C, J)
    g = run(arrays, streams)
    o = O.dtrade_run(arrays, streams)
    bad = np.nonzero((g["node"] != o["node"]) | (g["start"] != o["start"]) | (g["finish"] != o["finish"]))[0]
    assert bad.size == 0, f"{bad.size} mismatches, first {bad[:5]}: gpu {g['node'][bad[:5]]} {g['start'][bad[:5]]} " \
                          f"oracle {o['node'][bad[:5]]} {o['start'][bad[:5]]}"
    fields = ("t", "requester", "winner", "approvals", "policy", "cores", "mem", "time_s", "failed")
    assert len(g["trades"]) == len(o["trades"])
    for f in fields:
        np.testing.assert_array_equal(g["trades"][f], o["trades"][f], err_msg=f)
    assert len(g["foreign"]) == o["n_foreign"]
    for f in ("requester", "responder", "node", "start", "finish", "c", "m"):
        np.testing.assert_array_equal(g["foreign"][f], o["foreign"][f], err_msg=f)
    assert g["vnodes"] == o["vnodes"]
    for f in ("total_wait_ms", "jobs_count", "moved_l1", "placed_l1"):
        np.testing.assert_array_equal(g["ds"][f], o["stats"][f], err_msg=f)
    assert g["ts"]["t_final"] == o["t_final"]
    assert (g["trades"]["winner"] >= 0).sum() > 0  # the scenario exercises winning trades


def test_gpu_dtrade_without_traders_equals_delay():
    """trader_period 0 is refused; instead check the reduction with policies that never break:
    a lightly loaded 256-node system trades nothing and equals the standalone DELAY kernel."""
    arrays, streams, _ = seeded_workload("n256_delay", 4, 800)
    g = run(arrays, streams)
    assert len(g["trades"]) == 0
    with Engine(0, policy="DELAY") as eng:
        eng.load_clusters(arrays)
        eng.submit_jobs(streams)
        eng.run()
        node, start, fin = eng.placements()
    np.testing.assert_array_equal(g["node"], node)
    np.testing.assert_array_equal(g["start"], start)


def test_gpu_dtrade_caller_driven_world1_equals_run():
    """The caller-driven phase API at world 1 (phase 0 -> 1 carries this rank's exchange block back
    in unchanged) == mcs_run's graph-replayed loop, bit for bit."""
    from mcs_amd.shard import run_lockstep

    arrays, streams, _ = seeded_workload("n64_hot", 8, 2000)
    g = run(arrays, streams)
    with Engine(0, policy="DELAY", trader=True) as eng:
        eng.load_clusters(arrays)
        eng.submit_jobs(streams)
        run_lockstep(eng, lambda buf: buf)
        node, start, fin = eng.placements()
        trades, foreign = eng.contracts(), eng.foreign()
        t_final = eng.trade_stats()["t_final"]
    np.testing.assert_array_equal(node, g["node"])
    np.testing.assert_array_equal(start, g["start"])
    np.testing.assert_array_equal(fin, g["finish"])
    assert trades.tobytes() == g["trades"].tobytes()
    assert foreign.tobytes() == g["foreign"].tobytes()
    assert t_final == g["ts"]["t_final"]


def test_gpu_dtrade_two_ranks_gloo():
    """world = 2 shards (two processes, two engines on device 0) exchanging one block per rank per
    tick over gloo via the caller-driven phase API == the oracle of the whole system."""
    import subprocess
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29583")
    r = subprocess.run([sys.executable, os.path.join(here, "dtrade_2rank.py")], env=env, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "DTRADE-2RANK OK" in r.stdout


def test_gpu_dtrade_rccl_loop_world1():
    """The RCCL tick loop (shape all-reduce, one in-place ncclAllGather of the exchange blocks per
    tick, mcs_dtrade.cpp dt_run_rccl) on a world-1 communicator == the graph-replayed loop."""
    arrays, streams, _ = seeded_workload("n64_hot", 8, 2000)
    g = run(arrays, streams)
    with Engine(0, policy="DELAY", trader=True) as eng:
        eng.load_clusters(arrays)
        eng.set_shard(0, 1)
        eng.comm_init(Engine.comm_unique_id())
        eng.submit_jobs(streams)
        eng.run()
        node, start, fin = eng.placements()
        trades, foreign = eng.contracts(), eng.foreign()
        vn = eng.virtual_nodes()
        t_final = eng.trade_stats()["t_final"]
    np.testing.assert_array_equal(node, g["node"])
    np.testing.assert_array_equal(start, g["start"])
    np.testing.assert_array_equal(fin, g["finish"])
    assert trades.tobytes() == g["trades"].tobytes()
    assert foreign.tobytes() == g["foreign"].tobytes()
    assert vn.tolist() == [len(v) for v in g["vnodes"]]
    assert t_final == g["ts"]["t_final"]
