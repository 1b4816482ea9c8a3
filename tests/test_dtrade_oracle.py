"""CPU tests of the lock-step trading oracle with DELAY schedulers (oracle/mcs_oracle_dtrade.c):
hand-derived scenarios (tests/golden/kats_dtrade.json) and the exact reduction to independent
Delay loops when the traders are off or never break a policy.  No GPU needed."""
import copy
import json
import os

import numpy as np
import pytest

import oracle_ref as O
from kat_util import GOLDEN, REPO, seeded_workload
from mcs_amd import Cluster, JobStreams, pack_clusters

DT = json.load(open(os.path.join(GOLDEN, "kats_dtrade.json")))["dtrade"]


def dt_system(k):
    cls = []
    for i, name in enumerate(k["clusters"]):
        cl = copy.deepcopy(Cluster.load(os.path.join(REPO, "assets", name + ".json")))
        for node, (fc, fm) in k["override_free"].get(str(i), {}).items():
            cl.Nodes[int(node)].CoresAvailable = fc
            cl.Nodes[int(node)].MemoryAvailable = fm
        cls.append(cl)
    per = [sorted(k["jobs"], key=lambda j: j[0]) if c == 0 else
           sorted(k.get("jobs_by_cluster", {}).get(str(c), []), key=lambda j: j[0]) for c in range(len(cls))]
    jobs = [j for p in per for j in p]
    off = np.concatenate([[0], np.cumsum([len(p) for p in per])]).astype(np.uint64)
    s = JobStreams(np.array([j[1] for j in jobs], np.uint32), np.array([j[4] for j in jobs], np.uint32),
                   np.array([j[2] for j in jobs], np.uint32), np.array([j[3] for j in jobs], np.uint32), off)
    return pack_clusters(cls), s


def kat_expectations(k):
    """[(global job index, (node, start, finish))] of cluster 0 ("expect") and the others"""
    per = {"0": k["expect"], **k.get("expect_by_cluster", {})}
    sizes = [len(k["jobs"])] + [len(k.get("jobs_by_cluster", {}).get(str(c), [])) for c in range(1, len(k["clusters"]))]
    base = np.concatenate([[0], np.cumsum(sizes)])
    return [(int(base[int(c)]) + int(j), tuple(v)) for c, e in per.items() for j, v in e.items()]


def check_kat(k, node, start, fin, trades, foreign, n_foreign, vnodes, t_final):
    for g, (nd, s, f) in kat_expectations(k):
        assert (int(node[g]), int(start[g]), int(fin[g])) == (nd, s, f), (k["name"], g)
    got = [[int(r[f]) for f in ("t", "requester", "winner", "approvals", "policy", "cores", "mem", "time_s",
                                "failed")] for r in trades]
    assert got == k["trades"]
    ff = [[int(r[f]) for f in ("requester", "responder", "node", "start", "finish", "c", "m")]
          for r in foreign[:len(k["foreign_first"])]]
    assert ff == k["foreign_first"]
    assert n_foreign == k["n_foreign"]
    assert vnodes == [[tuple(v) for v in vs] for vs in k["vnodes"]]
    assert t_final == k["t_final"]


@pytest.mark.parametrize("k", DT, ids=[k["name"] for k in DT])
def test_dtrade_oracle_kats(k):
    arrays, s = dt_system(k)
    r = O.dtrade_run(arrays, s, t_max=k["t_max"])
    check_kat(k, r["node"], r["start"], r["finish"], r["trades"], r["foreign"], r["n_foreign"], r["vnodes"],
              r["t_final"])
    for key, v in k.get("stats0", {}).items():
        assert r["stats"][key][0] == v, key


@pytest.mark.parametrize("kind,C,J", [("small", 4, 300), ("big", 3, 400), ("n64_hot", 3, 800)])
def test_dtrade_without_traders_is_independent_delay(kind, C, J):
    """period 0 = no traders: every cluster runs its own Delay loop, exactly or_delay_run."""
    arrays, streams, _ = seeded_workload(kind, C, J)
    r = O.dtrade_run(arrays, streams, trader=False)
    node, st, fi, ds = O.delay_run_batch(arrays, streams)
    np.testing.assert_array_equal(r["node"], node)
    np.testing.assert_array_equal(r["start"], st)
    np.testing.assert_array_equal(r["finish"], fi)
    np.testing.assert_array_equal(r["stats"]["total_wait_ms"], ds["total_wait_ms"])
    assert r["n_trades"] == 0 and r["n_foreign"] == 0


def test_dtrade_unbroken_policies_change_nothing():
    """Light load: no WaitTime or Utilization policy ever breaks, so traders never trade and the
    placements equal the independent Delay loops."""
    arrays, streams, _ = seeded_workload("n256_delay", 3, 800)
    r = O.dtrade_run(arrays, streams)
    node, st, fi, ds = O.delay_run_batch(arrays, streams)
    assert r["n_trades"] == 0
    np.testing.assert_array_equal(r["node"], node)
    np.testing.assert_array_equal(r["start"], st)


def test_dtrade_overloaded_system_trades_and_uses_virtual_nodes():
    """cluster_small at the reference client's rate: waits exceed 600 s, traders size fast/small-node
    contracts from Level1, some trades win, and jobs run on the virtual nodes received."""
    arrays, streams, _ = seeded_workload("small", 8, 300)
    r = O.dtrade_run(arrays, streams)
    tr = r["trades"]
    assert r["n_trades"] > 100 and (tr["winner"] >= 0).sum() > 0
    assert set(np.unique(tr["policy"])) == {0, 1}
    nphys = np.repeat(np.diff(arrays.node_off), 300)
    assert (r["node"] >= nphys).sum() > 0 and (r["node"] >= 0).all()
    # every winning trade appended exactly one virtual node with the contract's capacity
    won = tr[tr["winner"] >= 0]
    for q in range(8):
        wq = won[won["requester"] == q]
        assert [(int(a), int(b)) for a, b in zip(wq["cores"], wq["mem"])] == r["vnodes"][q]


def test_small_node_time_is_the_parity_of_the_trailing_falls():
    """The small-node contract time (scheduler_client.go:263-265: endTime when the previous time is
    below it, else 0, over GetLevel1() in order) that dt_contracts computes in parallel: the last
    duration when the run of falls (d[i-1] >= d[i]) ending at the list's end is even, else 0."""
    rng = np.random.default_rng(7)
    for n in list(range(1, 70)) + [127, 128, 129, 640, 1000]:
        for hi in (1, 3, 50, 1 << 31):
            d = rng.integers(0, hi, n, dtype=np.uint64).astype(np.uint32)
            s = 0
            for x in d:
                s = int(x) if s < int(x) else 0
            run = 0
            for k in range(n - 1, 0, -1):
                if d[k - 1] >= d[k]:
                    run += 1
                else:
                    break
            assert s == (int(d[-1]) if run % 2 == 0 else 0), (n, hi)
