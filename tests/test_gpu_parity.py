"""GPU parity: the gfx950 FIFO kernel (through the C ABI, libmcs.so) against the CPU oracle and the
known-answer vectors.  Bit-exact on every field: node index, start and finish seconds, and the
per-cluster statistics.  Run on a real MI355X: ``pytest -m gpu``.
"""
import os

import numpy as np
import pytest

import oracle_ref as O
from kat_util import fuzz_workload, kat_cluster, kat_expect, kat_streams, load_kats, seeded_workload
from mcs_amd import (CLUSTER_STATS_DTYPE, Cluster, Engine, GenParams, JobStreams, pack_clusters, replicate,
                     uniform_cluster)
from mcs_amd import _lib as L
from mcs_amd.engine import gen_streams_host

pytestmark = pytest.mark.gpu
KATS = load_kats()



W16R = "mcs::fifo_asm_kernel<16, true, 4, 8>"
DUO = "mcs::fifo_duo_kernel"
LOOK = "mcs::fifo_asm_kernel<16, true, 4, 8, look>"


def w16r_form(n_clusters):
    """The kernel the engine picks for a streamed 129-256-node launch of n_clusters in the 16-bit
    format: W16R, the duo loop (a decision and a release wave per cluster) under MCS_FIFO_DUO=1, or
    the one-job lookahead loop W16L under MCS_FIFO_LOOK=1 (no grid picks either by default:
    kDuoMaxItems = kLookMaxItems = 0)."""
    if os.environ.get("MCS_FIFO_DUO") == "1":
        return DUO
    return LOOK if os.environ.get("MCS_FIFO_LOOK") == "1" else W16R


def set_form(monkeypatch, form):
    """form: "0" W16R, "1" the duo loop, "look" the lookahead loop (the parametrisations below)."""
    monkeypatch.setenv("MCS_FIFO_DUO", "1" if form == "1" else "0")
    monkeypatch.setenv("MCS_FIFO_LOOK", "1" if form == "look" else "0")

def run_engine(eng, arrays, streams):
    eng.load_clusters(arrays)
    eng.submit_jobs(streams)
    st = eng.run()
    node, start, fin = eng.placements()
    return node, start, fin, st, eng.cluster_stats()


def assert_parity(arrays, streams, node, start, fin, cstats, n_threads=8):
    on, os_, of, osd = O.fifo_run_batch(arrays, streams, n_threads=n_threads)
    bad = np.nonzero((node != on) | (start != os_) | (fin != of))[0]
    assert bad.size == 0, f"{bad.size} mismatches, first at job {bad[:5]}: gpu {node[bad[:5]]},{start[bad[:5]]} " \
                          f"oracle {on[bad[:5]]},{os_[bad[:5]]}"
    for key in ("t_end", "placed", "waited", "peak_running", "flags"):
        np.testing.assert_array_equal(cstats[key], osd[key], err_msg=key)


@pytest.mark.parametrize("k", KATS["fifo"], ids=[k["name"] for k in KATS["fifo"]])
def test_gpu_fifo_kats(engine, k):
    arrays = pack_clusters([kat_cluster(k)])
    node, start, fin, st, cs = run_engine(engine, arrays, kat_streams(k))
    en, es, ef = kat_expect(k)
    np.testing.assert_array_equal(node, en)
    np.testing.assert_array_equal(start, es)
    np.testing.assert_array_equal(fin, ef)
    assert st.placed == int((en >= 0).sum())
    assert st.unplaced == int((en < 0).sum())


def test_gpu_kats_batched_in_one_launch(engine):
    """All FIFO KATs as different clusters of ONE launch (independent waves)."""
    ks = KATS["fifo"]
    arrays = pack_clusters([kat_cluster(k) for k in ks])
    parts = [kat_streams(k) for k in ks]
    off = np.zeros(len(parts) + 1, np.uint64)
    off[1:] = np.cumsum([p.n_jobs for p in parts])
    s = JobStreams(*(np.concatenate([getattr(p, f) for p in parts]) for f in ("arrival", "dur", "cores", "mem")),
                   off)
    node, start, fin, st, cs = run_engine(engine, arrays, s)
    for i, k in enumerate(ks):
        en, es, ef = kat_expect(k)
        js = s.of(i)
        np.testing.assert_array_equal(node[js], en, err_msg=k["name"])
        np.testing.assert_array_equal(start[js], es, err_msg=k["name"])
    assert_parity(arrays, s, node, start, fin, cs)


def test_scheduler_mirror_kat1():
    from mcs_amd.scheduler import Job, Scheduler

    k = KATS["fifo"][0]
    s = Scheduler(device=0)
    s.Run(kat_cluster(k))
    jobs = [Job(Id=j[0], CoresNeeded=j[2], MemoryNeeded=j[3], Duration=j[4]) for j in k["jobs"]]
    pl = s.Fifo([j[1] for j in k["jobs"]], jobs)
    assert [(p.Node, p.Start, p.Finish) for p in pl] == [tuple(k["expect"][str(j[0])]) for j in k["jobs"]]
    # single-job mirrors on the live state (scheduler.go:127-139, 194-202; cluster.go:46-63,153-157)
    assert s.ScheduleJob(Job(CoresNeeded=20, MemoryNeeded=1000)) is None and s.LastNode() == 0
    assert s.ScheduleJob(Job(CoresNeeded=20, MemoryNeeded=1000)) is None and s.LastNode() == 1
    assert s.ScheduleJob(Job(CoresNeeded=33, MemoryNeeded=1)).Error() == "not enough resources in cluster"
    assert s.Lend(Job(CoresNeeded=31, MemoryNeeded=23999)) is None
    assert s.Lend(Job(CoresNeeded=32, MemoryNeeded=1)).Error() == "can't lend"
    cu, mu = s.GetResourceUtilization()
    ocu, omu = O.resource_utilization([32] * 5, [24000] * 5, [12, 12, 32, 32, 32], [23000, 23000] + [24000] * 3)
    assert (np.float32(cu), np.float32(mu)) == (np.float32(ocu), np.float32(omu))
    s.JobFinished(Job(CoresNeeded=20, MemoryNeeded=1000), 0)
    fc, fm = s.engine.live_state(0)
    assert list(fc) == [32, 12, 32, 32, 32] and list(fm) == [24000, 23000, 24000, 24000, 24000]
    s.engine.close()


def test_device_generator_matches_host(engine):
    for kind, gp in (("small", GenParams(seed=42)),
                     ("n256", GenParams(seed=43, arrival_mode=1, lam=1.5386))):
        spec = Cluster.load(os.path.join(os.path.dirname(__file__), "..", "assets", "cluster_small.json")) \
            if kind == "small" else uniform_cluster(256)
        arrays = replicate(spec, 37)
        engine.load_clusters(arrays)
        engine.generate_jobs(gp, 3001)
        dev = engine.read_jobs()
        host = gen_streams_host(gp, arrays, 3001)
        for f in ("arrival", "dur", "cores", "mem"):
            np.testing.assert_array_equal(getattr(dev, f), getattr(host, f), err_msg=f"{kind}:{f}")


@pytest.mark.parametrize("serial", ["0", "1"])
def test_device_generator_forms_all_modes(engine, serial, monkeypatch):
    """Both materialising forms (the one-wave-per-cluster GenStream writer and the per-thread scan,
    MCS_GEN_SERIAL=1) give the host generator's records for REF, SCALED and WEIBULL arrivals,
    including job counts that end mid-batch and clusters of 0 or 1 jobs' worth of rate."""
    monkeypatch.setenv("MCS_GEN_SERIAL", serial)
    arrays = replicate(uniform_cluster(64), 70)
    engine.load_clusters(arrays)
    for gp in (GenParams(seed=5), GenParams(seed=6, arrival_mode=1, lam=0.37),
               GenParams(seed=7, arrival_mode=1, lam=90.0), GenParams(seed=8, arrival_mode=2, lam=10.0),
               GenParams(seed=9, arrival_mode=2, lam=4.0, weibull_k=1.5), GenParams(seed=10, lam=0.05)):
        for J in (1, 63, 1000):
            engine.generate_jobs(gp, J)
            dev = engine.read_jobs()
            host = gen_streams_host(gp, arrays, J)
            for f in ("arrival", "dur", "cores", "mem"):
                np.testing.assert_array_equal(getattr(dev, f), getattr(host, f), err_msg=f"{gp}:{J}:{f}")


def test_config1_cluster_small_10k(engine):
    """BASELINE config 1 at its own size: cluster_small, FIFO, 10k seeded jobs."""
    arrays, streams, _ = seeded_workload("small", 1, 10_000)
    node, start, fin, st, cs = run_engine(engine, arrays, streams)
    assert st.placed == 10_000
    assert_parity(arrays, streams, node, start, fin, cs)


def test_config2_cluster_big_1m(engine):
    """BASELINE config 2 at full size: cluster_big, FIFO, 1M jobs, one cluster — bit-exact."""
    arrays, streams, _ = seeded_workload("big", 1, 1_000_000)
    node, start, fin, st, cs = run_engine(engine, arrays, streams)
    assert st.placed == 1_000_000
    assert_parity(arrays, streams, node, start, fin, cs)


def test_config3_small_replicas(engine):
    """BASELINE config 3 shape: 1024 cluster_small replicas (distinct seeds), 4k jobs each."""
    arrays, streams, _ = seeded_workload("small", 1024, 4000)
    node, start, fin, st, cs = run_engine(engine, arrays, streams)
    assert st.placed == streams.n_jobs
    assert_parity(arrays, streams, node, start, fin, cs)


@pytest.mark.parametrize("form", ["0", "look"])
@pytest.mark.parametrize("kind", ["n256", "n256_hot"])
def test_config4_shape_reduced(engine, kind, form, monkeypatch):
    """BASELINE config 4 shape (256 nodes, scaled arrivals) at 128 clusters x 6k jobs (W16R and the
    lookahead loop)."""
    set_form(monkeypatch, form)
    arrays, streams, _ = seeded_workload(kind, 128, 6000)
    node, start, fin, st, cs = run_engine(engine, arrays, streams)
    assert engine.last_kernel == w16r_form(128)
    assert_parity(arrays, streams, node, start, fin, cs)


def test_config4_strong_shard_512_lookahead(monkeypatch):
    """The strong shard an 8-GPU node runs (512 of C4's 4096 clusters, full streams) through the
    lookahead loop: every cluster bit-exact against the oracle."""
    from mcs_amd.engine import scaled_lambda

    monkeypatch.setenv("MCS_FIFO_LOOK", "1")
    n, J = 512, 16384
    arrays = replicate(uniform_cluster(256), n)
    gp = GenParams(seed=0x4D43535F53494D31, arrival_mode=1, lam=scaled_lambda(256, load=0.9))
    with Engine(0) as eng:
        eng.load_clusters(arrays)
        eng.set_shard(3, 8)  # rank 3 of 8: global clusters 1536..2047
        eng.generate_jobs(gp, J)
        st = eng.run()
        assert eng.last_kernel == LOOK
        assert st.placed == n * J
        node, start, fin = eng.placements()
        jobs = eng.read_jobs()
        cs = eng.cluster_stats()
    assert_parity(arrays, jobs, node, start, fin, cs, n_threads=16)


def test_config4_full_size_parity(engine):
    """BASELINE config 4 at full size on one GPU: 4096 clusters x 256 nodes x 16384 jobs (64M
    placements), EVERY cluster bit-exact against the oracle (OpenMP over clusters, a few seconds of
    host time), plus size-independent properties."""
    from mcs_amd.engine import scaled_lambda

    n, J = 4096, 16384
    arrays = replicate(uniform_cluster(256), n)
    gp = GenParams(seed=0x4D43535F53494D31, arrival_mode=1, lam=scaled_lambda(256, load=0.9))
    engine.load_clusters(arrays)
    engine.generate_jobs(gp, J)
    st = engine.run()
    assert st.placed == n * J and st.unplaced == 0
    node, start, fin = engine.placements()
    jobs = engine.read_jobs()
    cs = engine.cluster_stats()
    # properties on everything
    assert (node >= 0).all() and (node < 256).all()
    np.testing.assert_array_equal(fin, start + jobs.dur)
    assert (start >= jobs.arrival).all()
    s2 = start.reshape(n, J).astype(np.int64)
    assert (np.diff(s2, axis=1) >= 0).all()  # strict FIFO: starts non-decreasing in job order
    assert (cs["placed"] == J).all()
    # bit-exact on every cluster
    assert_parity(arrays, jobs, node, start, fin, cs, n_threads=16)
    # no node is ever over-committed: the ClusterState reduction at sampled seconds (a wrapped
    # free counter would show as utilization > 1)
    for t in np.linspace(0, int(fin.max()), 7).astype(int):
        cst = engine.cluster_states(int(t))
        assert (cst["cores_utilization"] <= 1.0).all() and (cst["memory_utilization"] <= 1.0).all(), t
        assert (cst["cores_utilization"] >= 0.0).all() and (cst["memory_utilization"] >= 0.0).all(), t


def test_config4_strong_shards_two_ranks_one_gpu():
    """bench.py --shard strong on two ranks (two processes, two engines on device 0): each holds a
    contiguous half of one system, generation keyed by the global cluster index; the concatenated
    outputs equal one engine holding every cluster and the oracle of the whole system."""
    import subprocess
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29587")
    r = subprocess.run([sys.executable, os.path.join(here, "c4_strong_2rank.py")], env=env, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "C4-STRONG-2RANK OK" in r.stdout


def test_config4_delay_fused_full_size_parity():
    """C4 at full size under DELAY with the stream synthesised in the kernel: every cluster
    bit-exact against the DELAY oracle over the same streams (materialised on demand by
    mcs_read_jobs, which equals the host generator), every job placed exactly once after its
    arrival, and no node over-committed."""
    from mcs_amd.engine import gen_cluster_host, scaled_lambda

    n, J = 4096, 16384
    arrays = replicate(uniform_cluster(256), n)
    gp = GenParams(seed=0x5EED5EED, arrival_mode=1, lam=scaled_lambda(256, load=0.9), fused=True)
    with Engine(0, policy="DELAY") as eng:
        eng.load_clusters(arrays)
        eng.generate_jobs(gp, J)
        st = eng.run()
        assert st.placed == n * J and st.unplaced == 0
        node, start, fin = eng.placements()
        ds = eng.delay_stats()
        cs = eng.cluster_stats()
        assert (node >= 0).all() and (node < 256).all()
        for t in np.linspace(0, int(fin.max()), 5).astype(int):
            cst = eng.cluster_states(int(t))
            assert (cst["cores_utilization"] <= 1.0).all() and (cst["memory_utilization"] <= 1.0).all(), t
        jobs = eng.read_jobs()
    for k in (0, 2049, 4095):  # the materialised stream is the host generator's
        a, d, c, m = gen_cluster_host(gp, k, 32, 24000, J)
        js = jobs.of(k)
        assert np.array_equal(jobs.arrival[js], a) and np.array_equal(jobs.dur[js], d)
        assert np.array_equal(jobs.cores[js], c) and np.array_equal(jobs.mem[js], m)
    assert (start >= jobs.arrival).all()
    np.testing.assert_array_equal(fin, start + jobs.dur)
    on, os_, of, osd = O.delay_run_batch(arrays, jobs, n_threads=16)
    bad = np.flatnonzero((node != on) | (start != os_) | (fin != of))
    assert bad.size == 0, f"{bad.size} mismatches, first jobs {bad[:5]}"
    np.testing.assert_array_equal(ds["total_wait_ms"], osd["total_wait_ms"])
    np.testing.assert_array_equal(ds["moved_l1"], osd["moved_l1"])
    np.testing.assert_array_equal(cs["t_end"], osd["t_end"])


def test_heterogeneous_cluster_sizes(engine):
    """Clusters of 0..1024 nodes in one launch (variant chosen by the largest)."""
    sizes = [0, 1, 5, 63, 64, 65, 200, 1024]
    rng = np.random.default_rng(5)
    clusters = []
    for i, nn in enumerate(sizes):
        cl = uniform_cluster(nn, cores=int(rng.integers(4, 64)), memory=int(rng.integers(1000, 50000)))
        for nd in cl.Nodes:  # partial JSON availability (KAT5 rule)
            nd.CoresAvailable = int(rng.integers(0, nd.Cores + 1))
        clusters.append(cl)
    arrays = pack_clusters(clusters)
    parts = []
    for i, cl in enumerate(clusters):
        mc = max([nd.Cores for nd in cl.Nodes], default=8)
        mm = max([nd.Memory for nd in cl.Nodes], default=1000)
        from mcs_amd.engine import gen_cluster_host

        parts.append(gen_cluster_host(GenParams(seed=77, arrival_mode=1, lam=0.02 * max(len(cl.Nodes), 1) + 0.2),
                                      i, mc, mm, 1500))
    off = np.arange(len(parts) + 1, dtype=np.uint64) * 1500
    s = JobStreams(*(np.concatenate([p[f] for p in parts]) for f in range(4)), off)
    node, start, fin, st, cs = run_engine(engine, arrays, s)
    assert_parity(arrays, s, node, start, fin, cs)
    assert cs[0]["flags"] & L.MCS_FLAG_DEADLOCK  # zero nodes: the first job never fits


@pytest.mark.parametrize("sizes", [[0, 1, 5, 63, 64, 65, 130, 200, 256], [0, 1, 2, 5, 33, 63, 64]],
                         ids=["asm_4x8", "asm_1x2"])
@pytest.mark.parametrize("duo", ["0", "1", "look"])
def test_heterogeneous_cluster_sizes_hand_scheduled(engine, sizes, duo, monkeypatch):
    """Clusters of many sizes in one launch of each hand-scheduled loop shape (the largest picks it:
    129-256 nodes -> 4 chunks x 8 slot rows, <= 64 nodes -> 1 chunk x 2 rows): padding nodes, an
    empty cluster (its first job deadlocks), partial JSON availability, zero-duration jobs."""
    from mcs_amd.engine import gen_cluster_host

    rng = np.random.default_rng(len(sizes))
    clusters, parts = [], []
    J = 2500
    for i, nn in enumerate(sizes):
        cl = uniform_cluster(nn, cores=int(rng.integers(4, 64)), memory=int(rng.integers(1000, 30000)))
        for nd in cl.Nodes:  # partial JSON availability (KAT5 rule)
            nd.CoresAvailable = int(rng.integers(0, nd.Cores + 1))
        clusters.append(cl)
        mc = max([nd.Cores for nd in cl.Nodes], default=8)
        mm = max([nd.Memory for nd in cl.Nodes], default=1000)
        a, d, c, m = gen_cluster_host(GenParams(seed=91 + i, arrival_mode=1, lam=0.02 * max(nn, 1) + 0.2), i, mc, mm, J)
        d = d.copy()
        d[rng.random(J) < 0.03] = 0  # zero-duration jobs (D3)
        parts.append((a, d, c, m))
    arrays = pack_clusters(clusters)
    off = np.arange(len(parts) + 1, dtype=np.uint64) * J
    s = JobStreams(*(np.concatenate([p[f] for p in parts]) for f in range(4)), off)
    set_form(monkeypatch, duo)
    node, start, fin, st, cs = run_engine(engine, arrays, s)
    if max(sizes) > 64:
        assert engine.last_kernel == w16r_form(len(sizes))
    else:
        assert engine.last_kernel == "mcs::fifo_asm_kernel<16, true, 1, 2>"
    assert_parity(arrays, s, node, start, fin, cs)
    assert cs[0]["flags"] & L.MCS_FLAG_DEADLOCK  # zero nodes: the first job never fits


@pytest.mark.parametrize("nodes,duo", [(256, "0"), (256, "1"), (256, "look"), (5, "0")])
def test_hand_scheduled_diag_build(nodes, duo, monkeypatch):
    """MCS_FIFO_DIAG=1 launches the counting build of the hand-scheduled loop: the same placements
    and per-cluster results, plus the pass and release-scan counters (which the production build
    leaves at the decision count and 0)."""
    set_form(monkeypatch, duo)
    arrays, streams, _ = seeded_workload("n256" if nodes == 256 else "small", 64, 3000)
    res = {}
    for diag in ("0", "1"):
        os.environ["MCS_FIFO_DIAG"] = diag
        try:
            with Engine(0) as eng:
                res[diag] = run_engine(eng, arrays, streams)
                assert eng.last_kernel == (w16r_form(64) if nodes == 256 else "mcs::fifo_asm_kernel<16, true, 1, 2>")
        finally:
            os.environ.pop("MCS_FIFO_DIAG", None)
    for i in range(3):
        np.testing.assert_array_equal(res["0"][i], res["1"][i])
    c0, c1 = res["0"][4], res["1"][4]
    for key in ("t_end", "placed", "waited", "peak_running", "flags"):
        np.testing.assert_array_equal(c0[key], c1[key], err_msg=key)
    assert (c0["iterations"] == c0["placed"]).all() and (c0["release_scans"] == 0).all()
    assert (c1["iterations"] > c1["placed"]).any() and (c1["release_scans"] > 0).any()
    assert_parity(arrays, streams, *res["1"][:3], c1)


@pytest.mark.parametrize("shape", ["w16s", "w16r", "duo", "look", "w32"])
@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5, 6])
def test_hand_scheduled_fuzz(engine, shape, seed, monkeypatch):
    """Randomised clusters and streams through each hand-scheduled loop form, bit-exact against the
    oracle: node counts across the shape's range (padding lanes and chunks), random JSON
    availability, bursts of simultaneous arrivals, zero-duration and zero-resource jobs, requests
    equal to a node's free value, and one request per cluster that fits no node (a head-of-line
    deadlock at a random point of the stream)."""
    set_form(monkeypatch, {"duo": "1", "look": "look"}.get(shape, "0"))
    arrays, s = fuzz_workload("w16r" if shape in ("duo", "look") else shape, seed)
    node, start, fin, st, cs = run_engine(engine, arrays, s)
    want = {"w16s": "mcs::fifo_asm_kernel<16, true, 1, 2>", "w16r": W16R, "duo": DUO, "look": LOOK,
            "w32": "mcs::fifo_asm_kernel<32, false, 4, 8>"}[shape]
    if st.escalations == 0:
        assert engine.last_kernel == want
    assert_parity(arrays, s, node, start, fin, cs)
    # the compiled kernel on the same case (MCS_FIFO_ASM=0) agrees as well
    os.environ["MCS_FIFO_ASM"] = "0"
    try:
        with Engine(0) as eng:
            n2, s2, f2, _, _ = run_engine(eng, arrays, s)
            assert eng.last_kernel == "mcs::fifo_kernel"
    finally:
        os.environ.pop("MCS_FIFO_ASM", None)
    np.testing.assert_array_equal(n2, node)
    np.testing.assert_array_equal(s2, start)
    np.testing.assert_array_equal(f2, fin)


def test_slot_pool_escalation():
    """Force the smallest pool (128 slots) with >128 concurrently running jobs: the engine must
    detect the overflow, re-run those clusters with a larger pool, and still be bit-exact."""
    eng = Engine(0, slot_pool=2)
    arrays = replicate(uniform_cluster(5), 3)
    n = 900
    a = np.repeat(np.arange(n // 3, dtype=np.uint32), 3)[:n]
    d = np.full(n, 400, np.uint32)
    c = np.zeros(n, np.uint32)
    m = np.ones(n, np.uint32)
    s = JobStreams(np.tile(a, 3), np.tile(d, 3), np.tile(c, 3), np.tile(m, 3),
                   np.arange(4, dtype=np.uint64) * n)
    node, start, fin, st, cs = run_engine(eng, arrays, s)
    assert st.escalations >= 1 and st.slot_pool > 2
    assert_parity(arrays, s, node, start, fin, cs)
    eng.close()


def test_slot_pool_escalation_from_hand_scheduled_loop():
    """More than 512 jobs running at once on a 200-node cluster: the hand-scheduled loop (8 slot rows)
    reports the overflow, the engine re-runs the cluster with a doubled pool on the compiled kernel,
    and the result is still bit-exact."""
    eng = Engine(0)
    arrays = replicate(uniform_cluster(200), 2)
    n = 1500
    a = np.repeat(np.arange(n // 5, dtype=np.uint32), 5)[:n]
    d = np.full(n, 700, np.uint32)
    c = np.zeros(n, np.uint32)
    m = np.ones(n, np.uint32)
    s = JobStreams(np.tile(a, 2), np.tile(d, 2), np.tile(c, 2), np.tile(m, 2), np.arange(3, dtype=np.uint64) * n)
    node, start, fin, st, cs = run_engine(eng, arrays, s)
    assert st.escalations >= 1 and st.slot_pool > 8
    assert (cs["peak_running"] > 512).all()
    assert_parity(arrays, s, node, start, fin, cs)
    eng.close()


def test_extreme_values(engine):
    """uint32 needs and capacities near 2^32: comparisons are unsigned and exact."""
    big = 0xFFFFFFF0
    cl = Cluster(Id=1, Nodes=[])
    from mcs_amd.cluster import Node

    cl.Nodes = [Node(Id=1, Cores=big, Memory=big, CoresAvailable=big, MemoryAvailable=big),
                Node(Id=2, Cores=big, Memory=big, CoresAvailable=big, MemoryAvailable=big)]
    arrays = pack_clusters([cl])
    jobs = [(0, big - 5, 7, 10), (0, 10, big, 3), (1, 6, 5, 0), (2, 1, 1, 2), (2, big, big, 1)]
    s = JobStreams(np.array([j[0] for j in jobs], np.uint32), np.array([j[3] for j in jobs], np.uint32),
                   np.array([j[1] for j in jobs], np.uint32), np.array([j[2] for j in jobs], np.uint32),
                   np.array([0, len(jobs)], np.uint64))
    node, start, fin, st, cs = run_engine(engine, arrays, s)
    assert_parity(arrays, s, node, start, fin, cs, n_threads=1)


@pytest.mark.parametrize("free", [0x7FFE, 0x7FFF])
def test_hand_scheduled_loop_field_bounds(engine, free):
    """The hand-scheduled loop's node formats at their bounds: free values up to 2^15 - 2 pick the
    16-bit format, 2^15 - 1 the 32-bit one (mcs_last_kernel says which ran).  Requests equal to a
    node's free value fit it exactly; each cluster's last job asks for one of the values around
    2^15, 2^16 and 2^31 that a truncated or unclamped request would fit, and must deadlock."""
    from mcs_amd.cluster import Node

    rng = np.random.default_rng(free)
    over = [free + 1, 0x8000, 0xFFFF, 0x10000, 0x10000 + 5, 0x17FFE, 0x7FFFFFFF, 0x80000000, 0x80000005,
            0xFFFFFFFF]
    clusters, parts = [], []
    J = 3000
    for k in range(2 * len(over)):
        cl = Cluster(Id=k + 1, Nodes=[])
        for i in range(200):
            c = free if i % 7 == 0 else int(rng.integers(0, free + 1))
            m = free if i % 5 == 0 else int(rng.integers(0, free + 1))
            cl.Nodes.append(Node(Id=i + 1, Cores=free, Memory=free, CoresAvailable=c, MemoryAvailable=m))
        clusters.append(cl)
        arr = np.cumsum(rng.poisson(0.3, J)).astype(np.uint32)
        dur = rng.integers(0, 40, J).astype(np.uint32)
        cores = rng.integers(0, free // 3, J).astype(np.uint32)
        mem = rng.integers(0, free // 3, J).astype(np.uint32)
        exact = rng.random(J) < 0.02
        cores[exact] = free
        mem[exact] = free
        o = over[k % len(over)]
        if k < len(over):
            cores[-1], mem[-1] = o, 1  # the oversize field is cores, then memory
        else:
            cores[-1], mem[-1] = 1, o
        parts.append((arr, dur, cores, mem))
    arrays = pack_clusters(clusters)
    off = np.arange(len(parts) + 1, dtype=np.uint64) * J
    s = JobStreams(*(np.concatenate([p[f] for p in parts]) for f in range(4)), off)
    node, start, fin, st, cs = run_engine(engine, arrays, s)
    assert engine.last_kernel == (w16r_form(len(clusters)) if free < 0x7FFF
                                  else "mcs::fifo_asm_kernel<32, false, 4, 8>")
    assert_parity(arrays, s, node, start, fin, cs)
    assert (cs["flags"] & L.MCS_FLAG_DEADLOCK).all()  # every cluster's last request fits nowhere
    assert (node.reshape(-1, J)[:, -1] == -1).all()


@pytest.mark.parametrize("policy", ["FIFO", "DELAY"])
def test_every_kernel_variant(policy):
    """Every compiled variant of the placement kernel — nodes per lane NPL 1..16 (the largest
    cluster: 64..1024 nodes) x slot rows 2..32 (cfg.slot_pool) x streamed / fused records — against
    the oracle (the library's kernels are built with LLVM's iterative ILP scheduler: each variant is
    its own schedule)."""
    from mcs_amd.engine import scaled_lambda

    for nn in (64, 128, 256, 512, 1024):
        arrays = pack_clusters([uniform_cluster(nn), uniform_cluster(max(1, nn // 3)), uniform_cluster(5)])
        lam = scaled_lambda(nn, load=1.1)
        gp = GenParams(seed=nn, arrival_mode=1, lam=lam, max_cores=32, max_mem=24000)
        streams = gen_streams_host(gp, arrays, 1200)
        oracle = (O.delay_run_batch if policy == "DELAY" else O.fifo_run_batch)(arrays, streams, n_threads=8)
        for pool in (2, 4, 8, 16, 32):
            # streamed FIFO has five forms: the hand-scheduled loop (mcs_fifo_asm.hip, 129-256
            # nodes and 8 slot rows) in its 16-bit node format with register slots (picked for these
            # clusters), with LDS slots (MCS_FIFO_ASM=16) and its 32-bit one (=32; =0 turns the loop
            # off), and the compiled kernel's two (the low-occupancy one is picked for small grids;
            # MCS_FIFO_LAT forces either)
            # (and the duo loop, MCS_FIFO_DUO=1, the register-slot form's two-wave variant)
            for fused, lat, asm, duo in ((False, "1", "0", None), (False, "0", "0", None), (False, None, "1", "0"),
                                         (False, None, "1", "1"), (False, None, "1", "look"),
                                         (False, None, "16", None), (False, None, "32", None),
                                         (True, None, None, None)):
                if policy == "DELAY" and lat == "0":
                    continue
                if policy == "DELAY" and asm in ("1", "16", "32"):
                    continue
                env = {"MCS_FIFO_LAT": lat, "MCS_FIFO_ASM": asm, "MCS_FIFO_DUO": "0" if duo == "look" else duo,
                       "MCS_FIFO_LOOK": "1" if duo == "look" else None}
                old = {k: os.environ.get(k) for k in env}
                for k, v in env.items():
                    if v is not None:
                        os.environ[k] = v
                try:
                    with Engine(0, slot_pool=pool, policy=policy) as eng:
                        eng.load_clusters(arrays)
                        gp.fused = fused
                        eng.generate_jobs(gp, 1200)
                        eng.run()
                        node, start, fin = eng.placements()
                finally:
                    for k, v in old.items():
                        if v is None:
                            os.environ.pop(k, None)
                        else:
                            os.environ[k] = v
                tag = f"nodes {nn} pool {pool} fused {fused} lat {lat} asm {asm} duo {duo}"
                np.testing.assert_array_equal(node, oracle[0], err_msg=tag)
                np.testing.assert_array_equal(start, oracle[1], err_msg=tag)
                np.testing.assert_array_equal(fin, oracle[2], err_msg=tag)
