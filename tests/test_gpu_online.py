"""GPU parity of the online mode (include/mcs.h: mcs_run with a finite horizon, mcs_append_jobs;
DESIGN.md §14).  The reference scheduler is an infinite loop fed by HTTP POSTs
(pkg/scheduler/server.go:23-78, scheduler.go:216-369): a Go caller advances the clock in slices and
appends the jobs POSTed meanwhile.  A run split into horizons, with each slice's arrivals appended
just before it, must equal the batch run over all the jobs and the CPU oracle bit for bit, and after
each horizon H every decision made at a simulated second < H (and no other) must be visible.
Run on a real MI355X: ``pytest -m gpu``."""
import numpy as np
import pytest

import oracle_ref as O
from kat_util import fuzz_workload, seeded_workload
from mcs_amd import Engine, JobStreams, MCSError, pack_clusters, replicate, uniform_cluster
from mcs_amd import _lib as L

pytestmark = pytest.mark.gpu


def slice_streams(streams, lo, hi):
    """the jobs of every cluster with lo <= arrival < hi, as an appended batch (CSR)"""
    parts, off = [[], [], [], []], [0]
    for k in range(len(streams.job_off) - 1):
        sl = streams.of(k)
        a = streams.arrival[sl]
        m = (a >= lo) & (a < hi)
        for i, f in enumerate(("arrival", "dur", "cores", "mem")):
            parts[i].append(getattr(streams, f)[sl][m])
        off.append(off[-1] + int(m.sum()))
    cat = [np.concatenate(p).astype(np.uint32) if p else np.zeros(0, np.uint32) for p in parts]
    return JobStreams(*cat, np.array(off, np.uint64))


def run_online(arrays, streams, horizons, policy="FIFO", check_prefix=None, **cfg):
    """append slice [h_{k-1}, h_k) then run(h_k); finally append the rest and drain."""
    with Engine(0, policy=policy, **cfg) as eng:
        eng.load_clusters(arrays)
        prev = 0
        for h in horizons:
            eng.append_jobs(slice_streams(streams, prev, h))
            st = eng.run(h)
            assert st.online and st.t_horizon == h
            if check_prefix is not None:
                check_prefix(eng, h, st)
            prev = h
        eng.append_jobs(slice_streams(streams, prev, 1 << 32))
        st = eng.run()  # drain
        node, start, fin = eng.placements()
        return node, start, fin, st, eng.cluster_stats(), (eng.delay_stats() if policy == "DELAY" else None)


def batch(arrays, streams, policy="FIFO", **cfg):
    with Engine(0, policy=policy, **cfg) as eng:
        eng.load_clusters(arrays)
        eng.submit_jobs(streams)
        st = eng.run()
        node, start, fin = eng.placements()
        return node, start, fin, st, eng.cluster_stats(), (eng.delay_stats() if policy == "DELAY" else None)


def horizons_for(streams, k):
    top = int(streams.arrival.max()) + 1
    return sorted({int(x) for x in np.linspace(0, top, k + 2)[1:-1]})


def make_prefix_check(final, full_off):
    def check(eng, h, st):
        node, start, fin = eng.placements()
        # the engine holds, per cluster, the first jobs of its stream (appended so far): map them
        # to the rows of the final run
        off = eng.job_offsets()
        idx = np.concatenate([np.arange(int(full_off[k]), int(full_off[k]) + int(off[k + 1] - off[k]))
                              for k in range(len(off) - 1)]).astype(np.int64)
        fnode, fstart, ffin = (x[idx] for x in final)
        decided = (fstart < h) & (fnode >= 0)
        assert np.array_equal(node[decided], fnode[decided]), h
        assert np.array_equal(start[decided], fstart[decided]), h
        assert np.array_equal(fin[decided], ffin[decided]), h
        und = ~decided & (fnode >= 0)
        assert (node[und] == L.MCS_NODE_UNPLACED).all() and (start[und] == L.MCS_TIME_NONE).all(), h
        assert st.placed == int(decided.sum()), (h, st.placed, int(decided.sum()))
    return check


@pytest.mark.parametrize("kind,C,J,k", [("small", 8, 3000, 7), ("n256", 32, 2500, 5), ("n256_hot", 16, 2500, 9),
                                        ("big", 1, 20000, 13)])
def test_online_fifo_slices_equal_batch_and_oracle(kind, C, J, k):
    arrays, streams, _ = seeded_workload(kind, C, J)
    b = batch(arrays, streams)
    on, os_, of, osd = O.fifo_run_batch(arrays, streams, n_threads=8)
    assert np.array_equal(b[0], on) and np.array_equal(b[1], os_) and np.array_equal(b[2], of)
    hs = horizons_for(streams, k)
    g = run_online(arrays, streams, hs, check_prefix=make_prefix_check(b[:3], streams.job_off))
    for i in range(3):
        np.testing.assert_array_equal(g[i], b[i])
    for f in ("t_end", "placed", "waited", "peak_running", "flags"):
        np.testing.assert_array_equal(g[4][f], osd[f], err_msg=f)
    assert g[3].pending == 0 and g[3].placed == b[3].placed


@pytest.mark.parametrize("kind,C,J,k", [("small", 8, 2000, 6), ("n256_delay", 16, 2500, 5), ("n64_hot", 8, 2500, 8)])
def test_online_delay_slices_equal_batch_and_oracle(kind, C, J, k):
    arrays, streams, _ = seeded_workload(kind, C, J)
    b = batch(arrays, streams, policy="DELAY")
    on, os_, of, osd = O.delay_run_batch(arrays, streams, n_threads=8)
    assert np.array_equal(b[0], on) and np.array_equal(b[1], os_) and np.array_equal(b[2], of)
    hs = horizons_for(streams, k)
    g = run_online(arrays, streams, hs, policy="DELAY", check_prefix=make_prefix_check(b[:3], streams.job_off))
    for i in range(3):
        np.testing.assert_array_equal(g[i], b[i])
    for f in ("t_end", "placed", "flags"):
        np.testing.assert_array_equal(g[4][f], osd[f], err_msg=f)
    for f in ("total_wait_ms", "jobs_count", "moved_l1", "placed_l1", "peak_l1", "l1_left"):
        np.testing.assert_array_equal(g[5][f], osd[f], err_msg=f)


def test_online_many_small_slices_grow_segments():
    """one-second-scale slices with a few jobs each: many appends, segment growth (relayout), parked
    clusters, horizons landing inside waits — still the batch result."""
    arrays, streams, _ = seeded_workload("small", 4, 600)
    b = batch(arrays, streams)
    top = int(streams.arrival.max()) + 1
    hs = list(range(7, top, max(1, top // 90)))
    g = run_online(arrays, streams, hs, check_prefix=make_prefix_check(b[:3], streams.job_off))
    for i in range(3):
        np.testing.assert_array_equal(g[i], b[i])
    gd = run_online(arrays, streams, hs, policy="DELAY")
    bd = batch(arrays, streams, policy="DELAY")
    for i in range(3):
        np.testing.assert_array_equal(gd[i], bd[i])


@pytest.mark.parametrize("policy", ["FIFO", "DELAY"])
def test_online_slot_pool_escalation(policy):
    """the smallest slot pool with > 128 concurrent jobs: a horizon that overflows is re-run from
    its untouched input state with a larger pool (DELAY: with its Level1 list restored)."""
    arrays = replicate(uniform_cluster(5), 3)
    n = 900
    a = np.repeat(np.arange(n // 3, dtype=np.uint32), 3)[:n]
    d = np.full(n, 400, np.uint32)
    c = np.zeros(n, np.uint32)
    m = np.ones(n, np.uint32)
    s = JobStreams(np.tile(a, 3), np.tile(d, 3), np.tile(c, 3), np.tile(m, 3), np.arange(4, dtype=np.uint64) * n)
    b = batch(arrays, s, policy=policy, slot_pool=2)
    g = run_online(arrays, s, [50, 120, 121, 260, 700], policy=policy, slot_pool=2)
    for i in range(3):
        np.testing.assert_array_equal(g[i], b[i])
    assert g[3].escalations + b[3].escalations >= 1


def test_online_deadlock_and_errors():
    """a head that never fits blocks its FIFO cluster for good across horizons and appends; the
    horizon order and the arrival floor are enforced."""
    from mcs_amd import Cluster
    from mcs_amd.cluster import Node

    cl = Cluster(Id=1, Nodes=[Node(Id=1, Cores=4, Memory=10, CoresAvailable=4, MemoryAvailable=10)])
    arrays = pack_clusters([cl, cl])
    first = JobStreams(np.array([0, 1, 0], np.uint32), np.array([5, 5, 5], np.uint32),
                       np.array([5, 1, 1], np.uint32), np.array([1, 1, 1], np.uint32), np.array([0, 2, 3], np.uint64))
    with Engine(0) as eng:
        eng.load_clusters(arrays)
        eng.append_jobs(first)
        eng.run(10)
        node, start, fin = eng.placements()
        assert node.tolist() == [-1, -1, 0] and start.tolist()[2] == 0
        with pytest.raises(MCSError):
            eng.run(5)  # horizons are non-decreasing
        bad = JobStreams(np.array([9], np.uint32), np.array([1], np.uint32), np.array([1], np.uint32),
                         np.array([1], np.uint32), np.array([0, 1, 1], np.uint64))
        with pytest.raises(MCSError):
            eng.append_jobs(bad)  # arrives before the last horizon run
        more = JobStreams(np.array([10, 12], np.uint32), np.array([1, 1], np.uint32), np.array([1, 1], np.uint32),
                          np.array([1, 1], np.uint32), np.array([0, 1, 2], np.uint64))
        eng.append_jobs(more)
        st = eng.run()
        node, start, fin = eng.placements()
        # cluster 0: jobs 0, 1 (initial) and 2 (appended) behind the deadlocked head; cluster 1: 2 jobs
        assert node.tolist() == [-1, -1, -1, 0, 0]
        assert start.tolist()[3:] == [0, 12]
        assert eng.cluster_stats()[0]["flags"] & L.MCS_FLAG_DEADLOCK
        assert st.unplaced == 3 and st.placed == 2 and st.pending == 0
        # rewind: the whole stream from t = 0 == the batch run
        eng.rewind()
        eng.run()
        assert eng.placements()[0].tolist() == [-1, -1, -1, 0, 0]


@pytest.mark.parametrize("policy", ["FIFO", "DELAY"])
def test_clock_overflow_is_an_error_with_unplaced_rows(policy):
    """unchecked_horizon lets a stream past the uint32 clock bound through: the kernel stops the
    cluster at the wrap, marks it MCS_FLAG_CLOCK_OVERFLOW, writes the jobs it did not decide as
    MCS_NODE_UNPLACED / MCS_TIME_NONE, and mcs_run returns MCS_E_RANGE; the checked default
    rejects the same stream up front.  A second, normal cluster is unaffected."""
    big = 0xFFFFFF00
    arrays = replicate(uniform_cluster(2, cores=4, memory=10), 2)
    # cluster 0: job 0 runs past 2^32 - 1 (its finish wraps); job 1 waits for node space
    a = np.array([big, big, 5, 6], np.uint32)
    d = np.array([0x200, 3, 4, 4], np.uint32)
    c = np.array([4, 4, 1, 1], np.uint32)
    m = np.array([1, 1, 1, 1], np.uint32)
    s = JobStreams(a, d, c, m, np.array([0, 2, 4], np.uint64))
    with Engine(0, policy=policy) as eng:
        eng.load_clusters(arrays)
        with pytest.raises(MCSError):
            eng.submit_jobs(s)
    with Engine(0, policy=policy, unchecked_horizon=1) as eng:
        eng.load_clusters(arrays)
        eng.submit_jobs(s)
        rc, st = eng.run_status()
        assert rc == L.MCS_E_RANGE
        node, start, fin = eng.placements()
        cs = eng.cluster_stats()
        assert cs[0]["flags"] & L.MCS_FLAG_CLOCK_OVERFLOW and not cs[1]["flags"]
        assert node[0] == L.MCS_NODE_UNPLACED and start[0] == L.MCS_TIME_NONE and fin[0] == L.MCS_TIME_NONE
        assert node[1] == L.MCS_NODE_UNPLACED and start[1] == L.MCS_TIME_NONE
        assert node[2:].tolist() == [0, 0] and start[2:].tolist() == [5, 6]
        if policy == "DELAY":
            assert eng.delay_stats()[0]["jobs_count"] == -1


@pytest.mark.parametrize("policy", ["FIFO", "DELAY"])
@pytest.mark.parametrize("shape,seed", [("w16s", 1), ("w16r", 2), ("w32", 3)])
def test_online_fuzz_slices_equal_batch_and_oracle(policy, shape, seed):
    """kat_util's randomised workloads (never-fitting requests, zero-duration jobs, idle stretches)
    advanced in 6 horizons with the arrivals appended between them: every prefix, the drained run,
    the batch run (the FIFO batch run goes through the hand-scheduled loop, the online one through
    the compiled kernel) and the oracle agree."""
    arrays, streams = fuzz_workload(shape, seed, n_clusters=48, J=1200)
    b = batch(arrays, streams, policy=policy)
    run_oracle = O.delay_run_batch if policy == "DELAY" else O.fifo_run_batch
    on, os_, of, osd = run_oracle(arrays, streams, n_threads=8)
    assert np.array_equal(b[0], on) and np.array_equal(b[1], os_) and np.array_equal(b[2], of)
    hs = horizons_for(streams, 6)
    g = run_online(arrays, streams, hs, policy=policy, check_prefix=make_prefix_check(b[:3], streams.job_off))
    for i in range(3):
        np.testing.assert_array_equal(g[i], b[i])
    for f in ("t_end", "placed", "flags"):
        np.testing.assert_array_equal(g[4][f], osd[f], err_msg=f)


def truncate_streams(streams, counts):
    """the first counts[k] jobs of every cluster k (ragged clusters)"""
    parts, off = [[], [], [], []], [0]
    for k, n in enumerate(counts):
        sl = streams.of(k)
        for i, f in enumerate(("arrival", "dur", "cores", "mem")):
            parts[i].append(getattr(streams, f)[sl][:n])
        off.append(off[-1] + n)
    return JobStreams(*[np.concatenate(p).astype(np.uint32) for p in parts], np.array(off, np.uint64))


@pytest.mark.parametrize("policy", ["FIFO", "DELAY"])
@pytest.mark.parametrize("kind", ["small", "n256"])
def test_online_ragged_last_cluster(policy, kind):
    """the last cluster holds fewer than 64 jobs (and one cluster none): a horizon resumes by reading
    the 64-row result batch at its cursor, which reaches past the last job (the result
    arrays carry kJobPad rows of slack).  Online slices and the unchecked-horizon batch path (the
    online kernels from t = 0) equal the batch run and the oracle."""
    arrays, full, _ = seeded_workload(kind, 4, 300)
    streams = truncate_streams(full, [300, 0, 77, 13])
    b = batch(arrays, streams, policy=policy)
    ref = (O.fifo_run_batch if policy == "FIFO" else O.delay_run_batch)(arrays, streams, n_threads=4)
    for i in range(3):
        np.testing.assert_array_equal(b[i], ref[i])
    g = run_online(arrays, streams, horizons_for(streams, 5), policy=policy)
    u = batch(arrays, streams, policy=policy, unchecked_horizon=1)
    for i in range(3):
        np.testing.assert_array_equal(g[i], b[i])
        np.testing.assert_array_equal(u[i], b[i])


def test_online_append_floor_is_per_cluster_after_a_drain():
    """after a drain each cluster accepts appended arrivals from its own clock on (mcs.h,
    mcs_append_jobs): a cluster that finished early takes a job arriving before the clock of a
    cluster that ran longer; an arrival before the cluster's own clock is refused."""
    arrays = replicate(uniform_cluster(5), 2)
    # cluster 0: one short job; cluster 1: six whole-node jobs, the sixth waits until t = 500
    s0 = JobStreams(np.zeros(7, np.uint32), np.array([5] + [500] * 6, np.uint32),
                    np.array([1] + [32] * 6, np.uint32), np.ones(7, np.uint32), np.array([0, 1, 7], np.uint64))
    with Engine(0) as eng:
        eng.load_clusters(arrays)
        eng.append_jobs(s0)
        eng.run()  # drain
        t_end = eng.cluster_stats()["t_end"]
        assert int(t_end[0]) < 100 < int(t_end[1])
        late = JobStreams(np.array([100], np.uint32), np.array([3], np.uint32), np.array([2], np.uint32),
                          np.array([2], np.uint32), np.array([0, 1, 1], np.uint64))
        eng.append_jobs(late)  # cluster 0 only: 100 >= its own clock
        eng.run()
        node, start, fin = eng.placements()
        assert (int(node[1]), int(start[1]), int(fin[1])) == (0, 100, 103)
        early = JobStreams(np.array([int(t_end[1]) - 1], np.uint32), np.array([3], np.uint32),
                           np.array([2], np.uint32), np.array([2], np.uint32), np.array([0, 0, 1], np.uint64))
        with pytest.raises(MCSError):
            eng.append_jobs(early)  # cluster 1: before its own clock


@pytest.mark.parametrize("seed", [11, 12])
def test_online_delay_level1_filter_edges(seed):
    """The Level1 fit filter's edge workload (test_gpu_delay._filter_edge_workload: 100/200-node
    clusters, keys across the clamp, zero-memory jobs) in 7 online slices: every horizon resumes a
    non-empty Level1 list (the pass-skip bound restarts from nothing) and the run equals the batch
    run and the oracle."""
    from test_gpu_delay import _filter_edge_workload

    arrays, streams = _filter_edge_workload(8, seed)
    b = batch(arrays, streams, policy="DELAY")
    g = run_online(arrays, streams, horizons_for(streams, 7), policy="DELAY",
                   check_prefix=make_prefix_check(b[:3], streams.job_off))
    for i in range(3):
        np.testing.assert_array_equal(g[i], b[i])
    for f in b[5].dtype.names:
        np.testing.assert_array_equal(g[5][f], b[5][f], err_msg=f)
    on, os_, of, od = O.delay_run_batch(arrays, streams, n_threads=8)
    np.testing.assert_array_equal(b[0], on)
    np.testing.assert_array_equal(b[1], os_)
    np.testing.assert_array_equal(b[2], of)
