"""CPU checks of the lock-step trading oracle (C5; oracle/mcs_oracle_trade.c).

Pinning: hand-derived known answers (tests/golden/kats_trade.json) plus two exact reductions to
the FIFO oracle, which is itself pinned by the FIFO KATs (test_oracle.py)."""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

import oracle_ref as O
from kat_util import GOLDEN, seeded_workload
from mcs_amd import JobStreams
from mcs_amd.cluster import ClusterArrays

NONE = 0xFFFFFFFF


def load_trade_kats():
    with open(os.path.join(GOLDEN, "kats_trade.json")) as f:
        return json.load(f)["kats"]


def kat_inputs(k):
    """(ClusterArrays, JobStreams) of a trade KAT."""
    caps = [np.array(nodes, np.uint32).reshape(-1, 2) for nodes in k["clusters"]]
    off = np.zeros(len(caps) + 1, np.uint32)
    off[1:] = np.cumsum([len(c) for c in caps])
    allc = np.concatenate(caps) if caps else np.zeros((0, 2), np.uint32)
    arrays = ClusterArrays(cap_c=allc[:, 0].copy(), cap_m=allc[:, 1].copy(), free_c=allc[:, 0].copy(),
                           free_m=allc[:, 1].copy(), node_off=off)
    jobs = [np.array(j, np.uint32).reshape(-1, 4) for j in k["jobs"]]
    joff = np.zeros(len(jobs) + 1, np.uint64)
    joff[1:] = np.cumsum([len(j) for j in jobs])
    allj = np.concatenate(jobs) if jobs else np.zeros((0, 4), np.uint32)
    streams = JobStreams(allj[:, 0].copy(), allj[:, 3].copy(), allj[:, 1].copy(), allj[:, 2].copy(), joff)
    return arrays, streams


def lent_rows(lent):
    return sorted([int(r["lender"]), int(r["borrower"]), int(r["job"]), int(r["node"]), int(r["start"]),
                   int(r["finish"])] for r in lent)


def trade_rows(trades):
    return [[int(r["t"]), int(r["requester"]), int(r["winner"]), int(r["approvals"])] for r in trades]


def check_trade_kat(k, res):
    e = k["expect"]
    assert res["node"].tolist() == e["node"], k["name"]
    assert res["start"].tolist() == e["start"], k["name"]
    assert res["finish"].tolist() == e["finish"], k["name"]
    assert lent_rows(res["lent"]) == sorted(e["lent"]), k["name"]
    assert trade_rows(res["trades"]) == e["trades"], k["name"]
    assert res["virtual_nodes"].tolist() == e["virtual_nodes"], k["name"]
    assert res["t_final"] == e["t_final"], k["name"]


@pytest.mark.parametrize("k", load_trade_kats(), ids=lambda k: k["name"].split()[0])
def test_trade_kats(k):
    arrays, streams = kat_inputs(k)
    res = O.trade_run(arrays, streams, borrow=bool(k["borrow"]), trader=bool(k["trader"]))
    check_trade_kat(k, res)


@pytest.mark.parametrize("kind", ["small", "n64", "n64_hot"])
def test_reduces_to_fifo(kind):
    """Borrow and trader off -> the FIFO oracle bit for bit; trader alone -> same placements
    (its zero contract only adds zero-capacity virtual nodes)."""
    arrays, streams, _ = seeded_workload(kind, 6, 1500)
    f = O.fifo_run_batch(arrays, streams)
    for trader in (False, True):
        r = O.trade_run(arrays, streams, borrow=False, trader=trader)
        assert np.array_equal(r["node"], f[0]) and np.array_equal(r["start"], f[1])
        assert np.array_equal(r["finish"], f[2])
        assert r["n_lent"] == 0
        if not trader:
            assert r["n_trades"] == 0


def usage_ok(arrays, streams, res):
    """Node capacity is never exceeded by own placements + lent runs (event sweep per node)."""
    C = arrays.n_clusters
    ev = {}
    for c in range(C):
        j0, j1 = int(streams.job_off[c]), int(streams.job_off[c + 1])
        for j in range(j0, j1):
            nd = int(res["node"][j])
            if nd >= 0 and streams.dur[j] > 0:
                ev.setdefault((c, nd), []).append((int(res["start"][j]), int(res["finish"][j]), int(streams.cores[j]),
                                                   int(streams.mem[j])))
    for r in res["lent"]:
        j = int(r["job"])
        if streams.dur[j] > 0:
            ev.setdefault((int(r["lender"]), int(r["node"])), []).append(
                (int(r["start"]), int(r["finish"]), int(streams.cores[j]), int(streams.mem[j])))
    for (c, nd), lst in ev.items():
        g = int(arrays.node_off[c]) + nd
        pts = sorted([(s, 1, cc, mm) for s, f, cc, mm in lst] + [(f, 0, -cc, -mm) for s, f, cc, mm in lst])
        uc = um = 0
        for _, _, dc, dm in pts:  # releases (kind 0) before commits at the same second
            uc += dc
            um += dm
            assert uc <= arrays.free_c[g] and um <= arrays.free_m[g]
    return True


@pytest.mark.parametrize("kind", ["small", "n64_hot"])
def test_borrow_properties(kind):
    arrays, streams, _ = seeded_workload(kind, 5, 800)
    r = O.trade_run(arrays, streams, borrow=True, trader=True)
    assert r["decided"].sum() == streams.n_jobs and r["lent_pending"].sum() == 0
    borrowed = np.flatnonzero(r["node"] == -2)
    assert len(borrowed) > 0
    assert np.all(r["finish"][borrowed] == NONE)
    lent_jobs = {int(x) for x in r["lent"]["job"]}
    assert set(borrowed.tolist()) == lent_jobs  # every borrowed job ran somewhere, nothing else did
    for rec in r["lent"]:
        j = int(rec["job"])
        assert rec["lender"] != rec["borrower"]
        assert streams.job_off[rec["borrower"]] <= j < streams.job_off[rec["borrower"] + 1]
        assert rec["start"] >= r["start"][j] + 1  # lent queue is served after the borrow tick
        assert rec["finish"] == rec["start"] + streams.dur[j]
    own = r["node"] >= 0
    assert np.all(r["finish"][own] == r["start"][own] + streams.dur[own])
    assert np.all(r["start"][own] >= streams.arrival[own])
    assert usage_ok(arrays, streams, r)
    tr = r["trades"]
    assert np.all(np.diff(tr["t"].astype(np.int64)) >= 0)
    assert np.all(tr["t"] % 10 == 0)
    assert r["virtual_nodes"].sum() == int(np.sum(tr["winner"] >= 0))
