"""CPU tests of the DELAY oracle (oracle/mcs_oracle_delay.c, Scheduler.Delay scheduler.go:298-369)
against the hand-derived known-answer vectors (tests/golden/kats_delay.json), plus the property that
pins the fast-forward restatement to the literal one-iteration-per-second Go loop, statistics
included.  No GPU needed."""
import json
import os

import numpy as np
import pytest

import oracle_ref as O
from kat_util import GOLDEN, kat_cluster, kat_expect, kat_streams, seeded_workload
from mcs_amd import pack_clusters, replicate, uniform_cluster
from mcs_amd.engine import GenParams, gen_streams_host

DKATS = json.load(open(os.path.join(GOLDEN, "kats_delay.json")))["delay"]


def one(arrays, streams, c, literal):
    ns, js = arrays.nodes_of(c), streams.of(c)
    return O.delay_run(arrays.free_c[ns], arrays.free_m[ns], streams.arrival[js], streams.dur[js],
                       streams.cores[js], streams.mem[js], literal=literal)


@pytest.mark.parametrize("literal", [False, True])
@pytest.mark.parametrize("k", DKATS, ids=[k["name"] for k in DKATS])
def test_delay_oracle_kats(k, literal):
    arrays = pack_clusters([kat_cluster(k)])
    node, st, fi, stats = one(arrays, kat_streams(k), 0, literal)
    en, es, ef = kat_expect(k)
    np.testing.assert_array_equal(node, en)
    np.testing.assert_array_equal(st, es)
    np.testing.assert_array_equal(fi, ef)
    for key, v in k["stats"].items():
        assert stats[key] == v, key


@pytest.mark.parametrize("kind,n_clusters,jobs", [("small", 3, 400), ("big", 2, 600), ("n64", 2, 1500),
                                                  ("n64_hot", 2, 1500)])
def test_delay_fast_forward_equals_literal(kind, n_clusters, jobs):
    """The fast-forward skips only iterations that repeat the same failures: every output and every
    statistic (TotalTime included) equals the literal loop's."""
    arrays, streams, _ = seeded_workload(kind, n_clusters, jobs)
    for c in range(n_clusters):
        a = one(arrays, streams, c, True)
        b = one(arrays, streams, c, False)
        for x, y in zip(a[:3], b[:3]):
            np.testing.assert_array_equal(x, y)
        assert a[3] == b[3]


def test_delay_overloaded_small_cluster_uses_level1():
    """cluster_small under the reference client's rate (Poisson(10)/min) is overloaded: heads wait
    past MaxWaitTime and Level1 carries most jobs; every job is still placed exactly once."""
    arrays, streams, _ = seeded_workload("small", 2, 500)
    node, st, fi, ds = O.delay_run_batch(arrays, streams, n_threads=2)
    assert (node >= 0).all()
    assert (ds["moved_l1"] > 100).all() and (ds["placed_l1"] == ds["moved_l1"]).all()
    assert (st.astype(np.int64) >= streams.arrival.astype(np.int64)).all()
    np.testing.assert_array_equal(fi, st + streams.dur)


def test_delay_capacity_never_exceeded():
    """Replay the oracle's placements: no node ever goes below zero free cores or memory."""
    arrays, streams, _ = seeded_workload("small", 1, 400)
    node, st, fi, _ = O.delay_run_batch(arrays, streams)
    ev = []
    for j in range(streams.n_jobs):
        if streams.dur[j] > 0:
            ev.append((int(fi[j]), 0, j))  # releases first at equal times (D3)
            ev.append((int(st[j]), 1, j))
    fc = arrays.free_c.astype(np.int64).copy()
    fm = arrays.free_m.astype(np.int64).copy()
    for t, kind, j in sorted(ev):
        sgn = 1 if kind == 0 else -1
        fc[node[j]] += sgn * int(streams.cores[j])
        fm[node[j]] += sgn * int(streams.mem[j])
        assert fc.min() >= 0 and fm.min() >= 0


def test_delay_batch_matches_single():
    arrays, streams, _ = seeded_workload("big", 3, 300)
    node, st, fi, ds = O.delay_run_batch(arrays, streams, n_threads=3)
    for c in range(3):
        a = one(arrays, streams, c, False)
        js = streams.of(c)
        np.testing.assert_array_equal(node[js], a[0])
        np.testing.assert_array_equal(st[js], a[1])
        assert ds["total_wait_ms"][c] == a[3]["total_wait_ms"]


def test_grown_node_pass_model_equals_oracle():
    """The hand-scheduled DELAY loop's Level1 pass (r04) tests a Level1 job only against the nodes
    that grew since the last pass, measured from a snapshot lowered at every Level1 move, plus the
    D6-skipped jobs: tools/delay_g_model.py restates that algorithm in Python and must give the
    oracle's placements on randomised clusters (deadlocks, zero durations, partial availability)."""
    import importlib.util

    spec = importlib.util.spec_from_file_location(
        "delay_g_model", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools",
                                      "delay_g_model.py"))
    M = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(M)
    import sys
    argv = sys.argv
    try:
        sys.argv = ["delay_g_model.py", "80"]
        assert M.main() == 0
    finally:
        sys.argv = argv
