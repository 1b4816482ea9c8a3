"""GPU parity of the DELAY policy: the gfx950 delay_kernel (through the C ABI, libmcs.so, engine
policy MCS_POLICY_DELAY) against the CPU oracle (oracle/mcs_oracle_delay.c) and the hand-derived
known-answer vectors.  Bit-exact on node, start, finish and on the per-cluster statistics (Delay
iterations, Level1 moves/placements/peak, WaitTime.TotalTime).  Run on a real MI355X."""
import json
import os

import numpy as np
import pytest

import oracle_ref as O
from kat_util import GOLDEN, fuzz_workload, kat_cluster, kat_expect, kat_streams, seeded_workload
from mcs_amd import Engine, JobStreams, pack_clusters, replicate, uniform_cluster
from mcs_amd import _lib as L

pytestmark = pytest.mark.gpu
DKATS = json.load(open(os.path.join(GOLDEN, "kats_delay.json")))["delay"]


@pytest.fixture(scope="module")
def delay_engine():
    e = Engine(0, policy="DELAY")
    yield e
    e.close()


def run(eng, arrays, streams):
    eng.load_clusters(arrays)
    eng.submit_jobs(streams)
    st = eng.run()
    node, start, fin = eng.placements()
    return node, start, fin, st, eng.cluster_stats(), eng.delay_stats()


def assert_delay_parity(arrays, streams, node, start, fin, cs, ds):
    on, os_, of, od = O.delay_run_batch(arrays, streams, n_threads=8)
    bad = np.nonzero((node != on) | (start != os_) | (fin != of))[0]
    assert bad.size == 0, f"{bad.size} mismatches, first at {bad[:5]}: gpu {node[bad[:5]]},{start[bad[:5]]} " \
                          f"oracle {on[bad[:5]]},{os_[bad[:5]]}"
    np.testing.assert_array_equal(cs["t_end"], od["t_end"], err_msg="t_end")
    np.testing.assert_array_equal(cs["placed"], od["placed"], err_msg="placed")
    np.testing.assert_array_equal(cs["waited"], od["moved_l1"], err_msg="moved")
    np.testing.assert_array_equal(cs["peak_running"], od["peak_running"], err_msg="peak_running")
    np.testing.assert_array_equal(cs["flags"], od["flags"], err_msg="flags")
    for key in ("total_wait_ms", "jobs_count", "moved_l1", "placed_l1", "peak_l1", "l1_left"):
        np.testing.assert_array_equal(ds[key], od[key], err_msg=key)


@pytest.mark.parametrize("k", DKATS, ids=[k["name"] for k in DKATS])
def test_gpu_delay_kats(delay_engine, k):
    arrays = pack_clusters([kat_cluster(k)])
    node, start, fin, st, cs, ds = run(delay_engine, arrays, kat_streams(k))
    en, es, ef = kat_expect(k)
    np.testing.assert_array_equal(node, en)
    np.testing.assert_array_equal(start, es)
    np.testing.assert_array_equal(fin, ef)
    for key, v in k["stats"].items():
        got = ds[key][0] if key in ds.dtype.names else cs[key][0]
        assert got == v, key


def test_gpu_delay_kats_one_launch(delay_engine):
    arrays = pack_clusters([kat_cluster(k) for k in DKATS])
    parts = [kat_streams(k) for k in DKATS]
    off = np.zeros(len(parts) + 1, np.uint64)
    off[1:] = np.cumsum([p.n_jobs for p in parts])
    s = JobStreams(*(np.concatenate([getattr(p, f) for p in parts]) for f in ("arrival", "dur", "cores", "mem")),
                   off)
    node, start, fin, st, cs, ds = run(delay_engine, arrays, s)
    assert_delay_parity(arrays, s, node, start, fin, cs, ds)


@pytest.mark.parametrize("kind,n_clusters,jobs", [
    ("small", 64, 1500),       # cluster_small at the reference client's rate: Level1-heavy
    ("big", 32, 3000),         # cluster_big, reference rate
    ("n256_delay", 64, 4000),  # 256 nodes just under one arrival per second
    ("n256", 32, 3000),        # 256 nodes above DELAY's drain rate: Level0 backlog
    ("n64_hot", 32, 3000),     # 64 nodes at 120% memory load
])
def test_gpu_delay_seeded_parity(delay_engine, kind, n_clusters, jobs):
    arrays, streams, _ = seeded_workload(kind, n_clusters, jobs)
    node, start, fin, st, cs, ds = run(delay_engine, arrays, streams)
    assert_delay_parity(arrays, streams, node, start, fin, cs, ds)
    assert st.placed + st.unplaced == streams.n_jobs


def test_gpu_delay_mixed_cluster_sizes(delay_engine):
    """cluster_small, cluster_big and 256-node clusters in one launch (NPL of the largest)."""
    a1, s1, _ = seeded_workload("small", 4, 800)
    a2, s2, _ = seeded_workload("n256_delay", 3, 800, seed=99)
    from mcs_amd import ClusterArrays
    arrays = ClusterArrays(*(np.concatenate([getattr(a1, f), getattr(a2, f)]) for f in
                             ("cap_c", "cap_m", "free_c", "free_m")),
                           np.concatenate([a1.node_off, a1.node_off[-1] + a2.node_off[1:]]))
    off = np.concatenate([s1.job_off, s1.job_off[-1] + s2.job_off[1:]])
    s = JobStreams(*(np.concatenate([getattr(s1, f), getattr(s2, f)]) for f in ("arrival", "dur", "cores", "mem")),
                   off)
    node, start, fin, st, cs, ds = run(delay_engine, arrays, s)
    assert_delay_parity(arrays, s, node, start, fin, cs, ds)


def test_gpu_delay_slot_pool_escalation():
    """A 2-row pool (128 slots) overflows on 256-node clusters; the engine re-runs those clusters
    with a doubled pool and the results still match the oracle."""
    arrays, streams, _ = seeded_workload("n256_delay", 8, 3000)
    with Engine(0, policy="DELAY", slot_pool=2) as eng:
        node, start, fin, st, cs, ds = run(eng, arrays, streams)
    assert st.escalations >= 1
    assert_delay_parity(arrays, streams, node, start, fin, cs, ds)


def test_gpu_delay_stats_state_errors(delay_engine):
    with Engine(0) as fifo:
        arrays = pack_clusters([kat_cluster(DKATS[0])])
        fifo.load_clusters(arrays)
        fifo.submit_jobs(kat_streams(DKATS[0]))
        fifo.run()
        with pytest.raises(L.MCSError):
            fifo.delay_stats()


def test_scheduler_mirror_delay():
    """The pkg/scheduler mirror with the reference's default policy (scheduler.go:116)."""
    from mcs_amd.scheduler import DELAY, Job, Scheduler

    k = [x for x in DKATS if x["name"] == "DKAT3"][0]
    s = Scheduler(device=0, policy=DELAY)
    s.Run(kat_cluster(k))
    jobs = [Job(Id=j[0], CoresNeeded=j[2], MemoryNeeded=j[3], Duration=j[4]) for j in k["jobs"]]
    pl = s.Delay([j[1] for j in k["jobs"]], jobs)
    assert [(p.Node, p.Start, p.Finish) for p in pl] == [tuple(k["expect"][str(j[0])]) for j in k["jobs"]]
    assert s.WaitTime.GetAverage() == 101000 / 8


@pytest.mark.parametrize("shape", ["w16s", "mid", "w16r", "w32"])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_gpu_delay_fuzz(delay_engine, shape, seed):
    """The randomised workloads of the FIFO fuzz cases (kat_util.fuzz_workload) under DELAY: Level1
    moves and passes, the D6 skip, WaitTime sums and never-fitting Level1 jobs, bit-exact."""
    arrays, s = fuzz_workload(shape, seed, n_clusters=96, J=1500)
    node, start, fin, st, cs, ds = run(delay_engine, arrays, s)
    assert_delay_parity(arrays, s, node, start, fin, cs, ds)


@pytest.mark.parametrize("kind", [
    "n256",        # Level0 backlog, Level1 never used: the whole run in the asm loop
    "n256_delay",  # just under one arrival per second
    "fuzz1",       # randomised w16r workloads (kat_util.fuzz_workload): heads wait MaxWaitTime and
    "fuzz2",       # their clusters hand over to delay_kernel
])
@pytest.mark.parametrize("diag", ["0", "1"])
def test_gpu_delay_hand_scheduled_loop(kind, diag, monkeypatch):
    """The hand-scheduled DELAY loop (mcs_delay_asm.hip, picked for 129-256 node clusters) with
    Level1 in LDS: its clusters, and those it hands to delay_kernel (re-run from t = 0: Level1 past
    its 640-entry LDS slice), equal the oracle and the compiled kernel alone (MCS_DELAY_ASM=0) on
    every output the oracle defines; MCS_FIFO_DIAG=1 launches its counting build."""
    if kind.startswith("fuzz"):
        arrays, streams = fuzz_workload("w16r", int(kind[4:]), n_clusters=64, J=1500)
    else:
        arrays, streams, _ = seeded_workload(kind, 64, 3000)
    monkeypatch.setenv("MCS_FIFO_DIAG", diag)
    with Engine(0, policy="DELAY") as eng:
        got = run(eng, arrays, streams)
        handed = got[3].handed_over
        assert eng.last_kernel == ("mcs::delay_asm_kernel" if handed == 0 else
                                   f"mcs::delay_asm_kernel + mcs::delay_kernel ({handed} of 64 clusters handed over)")
    assert_delay_parity(arrays, streams, *got[:3], got[4], got[5])
    if kind.startswith("n256"):
        assert handed == 0  # Level1 stays in the hand-scheduled loop
    monkeypatch.setenv("MCS_DELAY_ASM", "0")
    with Engine(0, policy="DELAY") as eng:
        ref = run(eng, arrays, streams)
        assert eng.last_kernel == "mcs::delay_kernel"
    for i in range(3):
        np.testing.assert_array_equal(got[i], ref[i])
    for f in ("t_end", "placed", "waited", "peak_running", "flags"):
        np.testing.assert_array_equal(got[4][f], ref[4][f], err_msg=f)
    for f in got[5].dtype.names:
        np.testing.assert_array_equal(got[5][f], ref[5][f], err_msg=f)
    assert got[3].placed == ref[3].placed and got[3].unplaced == ref[3].unplaced
    if diag == "1":
        assert (got[4]["release_scans"] > 0).any()
    if kind == "n256":
        assert (got[5]["moved_l1"] == 0).all()  # (no cluster needed the compiled kernel)
    if kind.startswith("fuzz"):
        assert (got[5]["moved_l1"] > 0).any()
        # Level1 placements and deadlocks (the blocking requests) inside the loop; a cluster whose
        # Level1 outgrows the LDS slice goes to delay_kernel
        assert handed < 64 and (got[4]["flags"] & L.MCS_FLAG_DEADLOCK).any()


@pytest.mark.parametrize("nodes", [64, 128, 200, 256, 512])
def test_gpu_delay_level1_heavy_generated(nodes):
    """The Level1-heavy bench stream (bench.py --policy delay --lam 0.95 --max-dur 972: fewer than
    one arrival per second at 90 % memory load, so heads wait MaxWaitTime and ~70 % of the jobs
    move to Level1) at reduced size, through every node-count class of delay_kernel (NPL 1, 2, 4,
    8; the exact fit filter in its own LDS or in the borrowed slot rows) and, for 129-256 nodes,
    the hand-scheduled loop's hand-over: bit-exact vs the oracle."""
    from mcs_amd import GenParams, gen_streams_host

    arrays = replicate(uniform_cluster(nodes), 24)
    # the offered load stays at 90 % with the arrival rate below DELAY's one-per-second drain
    gp = GenParams(seed=0x4D43535F53494D31, arrival_mode=1, lam=0.95, max_dur_s=972 * nodes // 256)
    streams = gen_streams_host(gp, arrays, 2500)
    with Engine(0, policy="DELAY") as eng:
        node, start, fin, st, cs, ds = run(eng, arrays, streams)
        if 129 <= nodes <= 256:  # the whole run in the hand-scheduled loop, Level1 included
            assert eng.last_kernel == "mcs::delay_asm_kernel" and st.handed_over == 0
    assert_delay_parity(arrays, streams, node, start, fin, cs, ds)
    assert ds["moved_l1"].sum() > streams.n_jobs // 4


def _filter_edge_workload(n_clusters, seed):
    """Clusters of 100 and 200 nodes (the fit filter in its own LDS and in the borrowed slot rows)
    whose nodes have 40-128 cores, and jobs whose cores straddle the filter's key clamp (62, 63,
    64, 100: key 63 is conservative) with zero-memory jobs among them (m = 0 passes the filter
    when no node can be told apart), arriving under DELAY's drain so Level1 fills and the pass
    skip's bound is raised, lowered and folded by D6 skips."""
    from mcs_amd.cluster import Node

    rng = np.random.default_rng(seed)
    clusters = []
    for k in range(n_clusters):
        n = 100 if k % 2 else 200
        cores = rng.choice([40, 64, 80, 128], size=n)
        mem = rng.choice([4000, 12000, 24000], size=n)
        from mcs_amd import Cluster
        clusters.append(Cluster(Id=k + 1, Nodes=[Node(Id=i + 1, Type="physical", Memory=int(mem[i]), Cores=int(cores[i]),
                                                      MemoryAvailable=int(mem[i]), CoresAvailable=int(cores[i]))
                                                 for i in range(n)]))
    arrays = pack_clusters(clusters)
    J = 1500
    parts = []
    for k in range(n_clusters):
        arr = np.cumsum(rng.poisson(1.1, size=J)).astype(np.uint32)
        dur = rng.integers(0, 900, size=J).astype(np.uint32)
        c = rng.choice([0, 1, 8, 32, 62, 63, 64, 100], size=J, p=[.05, .15, .25, .25, .1, .08, .07, .05])
        m = rng.choice([0, 1, 2000, 8000, 12000, 20000], size=J, p=[.08, .07, .3, .3, .15, .1])
        parts.append((arr, dur, c.astype(np.uint32), m.astype(np.uint32)))
    off = np.zeros(n_clusters + 1, np.uint64)
    off[1:] = np.cumsum([J] * n_clusters)
    s = JobStreams(*(np.concatenate([p[i] for p in parts]) for i in range(4)), off)
    return arrays, s


@pytest.mark.parametrize("seed", [11, 12, 13])
def test_gpu_delay_level1_filter_edges(seed):
    arrays, streams = _filter_edge_workload(16, seed)
    with Engine(0, policy="DELAY") as eng:
        node, start, fin, st, cs, ds = run(eng, arrays, streams)
    assert_delay_parity(arrays, streams, node, start, fin, cs, ds)
    assert ds["moved_l1"].sum() > 0 and ds["placed_l1"].sum() > 0


def _l1_pressure_workload(n_jobs_blocked, n_clusters=8, J=3000):
    """256-node clusters of 2-core nodes whose streams hold n_jobs_blocked 3-core requests (they fit
    no node: Level1 fills with them and the run ends in a Level1 deadlock) among small jobs."""
    from mcs_amd import Cluster
    from mcs_amd.cluster import Node

    rng = np.random.default_rng(n_jobs_blocked)
    cl = Cluster(Id=1, Nodes=[Node(Id=i + 1, Cores=2, Memory=4000, CoresAvailable=2, MemoryAvailable=4000)
                              for i in range(256)])
    arrays = replicate(cl, n_clusters)
    parts = []
    for k in range(n_clusters):
        arr = np.cumsum(rng.poisson(0.5, J)).astype(np.uint32)
        dur = rng.integers(0, 400, J).astype(np.uint32)
        c = rng.integers(0, 3, J).astype(np.uint32)
        m = rng.integers(0, 4001, J).astype(np.uint32)
        blk = rng.choice(J, n_jobs_blocked, replace=False)
        c[blk] = 3
        parts.append((arr, dur, c, m))
    off = np.arange(n_clusters + 1, dtype=np.uint64) * J
    return arrays, JobStreams(*(np.concatenate([p[i] for p in parts]) for i in range(4)), off)


@pytest.mark.parametrize("blocked,handed", [(100, False), (900, True)])
def test_gpu_delay_level1_deadlock_and_capacity(blocked, handed):
    """A Level1 that never drains: 100 never-fitting jobs end each cluster in a deadlock inside the
    hand-scheduled loop (Level1 rows written unplaced, WaitTime of the jobs left); 900 outgrow the
    640-entry LDS slice and the cluster is handed to delay_kernel.  Both bit-exact vs the oracle."""
    arrays, streams = _l1_pressure_workload(blocked)
    with Engine(0, policy="DELAY") as eng:
        node, start, fin, st, cs, ds = run(eng, arrays, streams)
        assert (st.handed_over == 8) == handed and (st.handed_over == 0) == (not handed)
    assert_delay_parity(arrays, streams, node, start, fin, cs, ds)
    assert (cs["flags"] & L.MCS_FLAG_DEADLOCK).all() and (ds["l1_left"] >= blocked).all()
