"""CPU tests of the oracle (oracle/mcs_oracle.c) against the known-answer vectors, plus the
properties that pin the fast-forward restatement to the literal one-second Go loop.

The reference has no tests; these KATs (tests/golden/kats.json) are hand-derived from its source
(SURVEY Appendix B).  No GPU needed.
"""
import numpy as np
import pytest

import oracle_ref as O
from kat_util import kat_cluster, kat_expect, kat_streams, load_kats, seeded_workload
from mcs_amd import pack_clusters

KATS = load_kats()


@pytest.mark.parametrize("literal", [False, True])
@pytest.mark.parametrize("k", KATS["fifo"], ids=[k["name"] for k in KATS["fifo"]])
def test_oracle_fifo_kats(k, literal):
    cl = pack_clusters([kat_cluster(k)])
    s = kat_streams(k)
    node, st, fi, stats = O.fifo_run(cl.free_c, cl.free_m, s.arrival, s.dur, s.cores, s.mem, literal=literal,
                                     cap_c=cl.cap_c, cap_m=cl.cap_m)
    en, es, ef = kat_expect(k)
    np.testing.assert_array_equal(node, en)
    np.testing.assert_array_equal(st, es)
    np.testing.assert_array_equal(fi, ef)
    assert stats["placed"] == int((en >= 0).sum())


@pytest.mark.parametrize("c", KATS["approve_trade"]["cases"])
def test_oracle_approve_trade(c):
    got = O.approve_trade(c["total_c"], c["total_m"], np.float32(c["cu"]), np.float32(c["mu"]), c["cores"],
                          c["mem"], c["time_ns"], np.float32(c["price"]))
    assert got == c["expect"]


def test_kat6_float32_availability():
    # SURVEY KAT6: util 0.79999995f gives avail 32.000008f (float32 T - T*u, trader.go:149)
    t = np.float32(160.0)
    u = np.float32(0.79999995)
    avail = np.float32(t - np.float32(t * u))
    assert avail == np.float32(32.000008)


@pytest.mark.parametrize("c", KATS["heap_order"]["cases"])
def test_oracle_heap_order(c):
    assert O.heap_order(c["prices"]) == c["expect"]


@pytest.mark.parametrize("c", KATS["allocate_virtual_node"]["cases"])
def test_oracle_allocate_virtual_node(c):
    fc = np.full(5, 32, np.uint64)
    fm = np.full(5, 24000, np.uint64)
    rc, nfc, nfm, foreign = O.allocate_virtual_node(fc, fm, c["req_c"], c["req_m"])
    assert rc == c["expect_rc"]
    assert [list(f) for f in foreign] == c["expect_foreign"]
    assert [int(nfc[0]), int(nfm[0])] == c["expect_free0"]


@pytest.mark.parametrize("c", KATS["contract"]["cases"])
def test_oracle_contract_sizing(c):
    got = O.contract(c["kind"], c["jobs"])
    assert list(got[:3]) == c["expect"][:3]
    assert got[3] == c["expect"][3]


def test_contract_small_no_padding_keeps_time():
    # 20 jobs: no nil padding (trader_server.go:79), the last job's end sets Time when it exceeds
    jobs = [(1, 1, 5)] * 19 + [(1, 1, 9)]
    c, m, t, p = O.contract("small", jobs)
    assert (c, m, t) == (20, 20, 9 * 10**9)


def test_schedule_job_and_lend_strictness():
    fc = np.array([4, 8], np.uint64)
    fm = np.array([100, 200], np.uint64)
    assert O.schedule_job(fc, fm, 4, 100) == 0  # >= (scheduler.go:131)
    assert O.schedule_job(fc, fm, 5, 100) == 1
    assert O.schedule_job(fc, fm, 9, 1) == -1
    assert not O.lend(np.array([4], np.uint64), np.array([100], np.uint64), 4, 99)  # strict > (:197)
    assert O.lend(np.array([5], np.uint64), np.array([101], np.uint64), 4, 100)


def test_resource_utilization_float32_order():
    cap_c = np.full(5, 32, np.uint64)
    cap_m = np.full(5, 24000, np.uint64)
    free_c = np.array([0, 16, 32, 31, 7], np.uint64)
    free_m = np.array([1, 24000, 12000, 5, 0], np.uint64)
    cu, mu = O.resource_utilization(cap_c, cap_m, free_c, free_m)
    # restated in numpy float32, node order (cluster.go:53-62)
    c = np.float32(0)
    m = np.float32(0)
    for i in range(5):
        c = np.float32(c + np.float32(np.float32(cap_c[i]) - np.float32(free_c[i])))
        m = np.float32(m + np.float32(np.float32(cap_m[i]) - np.float32(free_m[i])))
    assert cu == np.float32(c / np.float32(160))
    assert mu == np.float32(m / np.float32(120000))


@pytest.mark.parametrize("kind,jobs", [("small", 600), ("big", 600), ("n64", 400), ("n64_hot", 400)])
def test_fast_forward_equals_literal_loop(kind, jobs):
    """Appendix A.3: the fast-forwarded oracle equals the literal 1-second Go loop."""
    arrays, streams, _ = seeded_workload(kind, 3, jobs, seed=1234)
    for k in range(arrays.n_clusters):
        ns = arrays.nodes_of(k)
        js = streams.of(k)
        args = (arrays.free_c[ns], arrays.free_m[ns], streams.arrival[js], streams.dur[js], streams.cores[js],
                streams.mem[js])
        a = O.fifo_run(*args, literal=False)
        b = O.fifo_run(*args, literal=True)
        for x, y in zip(a[:3], b[:3]):
            np.testing.assert_array_equal(x, y)
        for key in ("t_end", "placed", "waited", "peak_running", "flags"):
            assert a[3][key] == b[3][key], key
        assert a[3]["ticks"] <= b[3]["ticks"]


@pytest.mark.parametrize("kind", ["small", "big", "n256"])
def test_oracle_properties(kind):
    """Conservation and FIFO order: every job placed, starts non-decreasing in job order (strict
    head-of-line blocking), start >= arrival, finish = start + dur, and the resources held at every
    instant fit every node."""
    arrays, streams, _ = seeded_workload(kind, 2, 500, seed=99)
    node, st, fi, sd = O.fifo_run_batch(arrays, streams)
    assert (node >= 0).all()
    np.testing.assert_array_equal(fi, st + streams.dur)
    assert (st >= streams.arrival).all()
    for k in range(arrays.n_clusters):
        js = streams.of(k)
        assert (np.diff(st[js].astype(np.int64)) >= 0).all()
        ns = arrays.nodes_of(k)
        cap_c = arrays.free_c[ns].astype(np.int64)
        cap_m = arrays.free_m[ns].astype(np.int64)
        # sweep events: usage at each start instant (after releases due then) must fit
        ev_t = np.concatenate([st[js], fi[js]])
        order = np.lexsort((np.r_[np.ones(len(st[js])), np.zeros(len(fi[js]))], ev_t))
        use_c = np.zeros_like(cap_c)
        use_m = np.zeros_like(cap_m)
        nd = np.r_[node[js], node[js]]
        cc = np.r_[streams.cores[js], -streams.cores[js].astype(np.int64)]
        mm = np.r_[streams.mem[js], -streams.mem[js].astype(np.int64)]
        for i in order:
            use_c[nd[i]] += cc[i]
            use_m[nd[i]] += mm[i]
            assert (use_c <= cap_c).all() and (use_m <= cap_m).all()


def test_oracle_batch_matches_single():
    arrays, streams, _ = seeded_workload("small", 4, 300, seed=5)
    bn, bs, bf, sd = O.fifo_run_batch(arrays, streams, n_threads=2)
    for k in range(4):
        ns, js = arrays.nodes_of(k), streams.of(k)
        n, s, f, st = O.fifo_run(arrays.free_c[ns], arrays.free_m[ns], streams.arrival[js], streams.dur[js],
                                 streams.cores[js], streams.mem[js])
        np.testing.assert_array_equal(bn[js], n)
        np.testing.assert_array_equal(bs[js], s)
        assert sd[k]["t_end"] == st["t_end"]
