"""GPU parity of on-device job generation fused into the placement kernels.

With GenParams(fused=True) no job record is stored: fifo_kernel / delay_kernel synthesise each
64-job batch in registers (csrc/mcs_gen_dev.h).  The runs must equal, bit for bit, the same runs
over the materialised records and the CPU oracle over the host generator's streams (the host
generator mcs_gen_cluster_host is the reference for the stream itself, test_abi.py).  Covered:
both arrival modes (REF per-minute spacing with empty minutes, SCALED per-second), FIFO and DELAY,
mixed cluster sizes in one launch (5, 10 and 256 nodes), explicit maxima, slot-pool escalation,
mcs_read_jobs and the trading path materialising a fused stream on demand."""
import numpy as np
import pytest

import oracle_ref as O
from mcs_amd import (Engine, GenParams, gen_streams_host, pack_clusters, replicate, scaled_lambda,
                     uniform_cluster)
from mcs_amd import _lib as L

pytestmark = pytest.mark.gpu


def mixed_arrays():
    return pack_clusters([uniform_cluster(5)] * 6 + [uniform_cluster(10)] * 4 + [uniform_cluster(256)] * 6)


def run(policy, arrays, gp, jobs, **kw):
    with Engine(0, policy=policy, **kw) as eng:
        eng.load_clusters(arrays)
        eng.generate_jobs(gp, jobs)
        st = eng.run()
        node, start, fin = eng.placements()
        cs = eng.cluster_stats()
        ds = eng.delay_stats() if policy == "DELAY" else None
    return node, start, fin, cs, ds, st


CASES = [
    ("FIFO", L.MCS_ARRIVAL_REF, 10.0, 2500),
    ("FIFO", L.MCS_ARRIVAL_SCALED, None, 2500),
    ("DELAY", L.MCS_ARRIVAL_REF, 10.0, 2000),
    ("DELAY", L.MCS_ARRIVAL_SCALED, 0.8, 1000),
    ("FIFO", L.MCS_ARRIVAL_WEIBULL, 10.0, 2500),   # the client's "weibull" mode (client.go:131-145)
    ("DELAY", L.MCS_ARRIVAL_WEIBULL, 6.0, 1500),
]
MODE_NAMES = {L.MCS_ARRIVAL_REF: "REF", L.MCS_ARRIVAL_SCALED: "SCALED", L.MCS_ARRIVAL_WEIBULL: "WEIBULL"}


@pytest.mark.parametrize("policy,mode,lam,jobs", CASES, ids=[f"{c[0]}-{MODE_NAMES[c[1]]}" for c in CASES])
def test_fused_equals_records_and_oracle(policy, mode, lam, jobs):
    arrays = mixed_arrays()
    lam = lam if lam is not None else scaled_lambda(256, load=0.9)
    gp = GenParams(seed=0x5EED + jobs, arrival_mode=mode, lam=lam)
    ref = run(policy, arrays, gp, jobs)
    gp.fused = True
    fz = run(policy, arrays, gp, jobs)
    for a, b, name in zip(ref[:3], fz[:3], ("node", "start", "finish")):
        np.testing.assert_array_equal(a, b, err_msg=name)
    for key in ("t_end", "placed", "waited", "peak_running", "flags"):
        np.testing.assert_array_equal(ref[3][key], fz[3][key], err_msg=key)
    if policy == "DELAY":
        np.testing.assert_array_equal(ref[4], fz[4])
    # and the oracle over the host generator's streams (bit-identical to the device generator)
    gp.fused = False
    streams = gen_streams_host(gp, arrays, jobs)
    if policy == "FIFO":
        on, os_, of, _ = O.fifo_run_batch(arrays, streams, n_threads=8)
    else:
        on, os_, of, _ = O.delay_run_batch(arrays, streams, n_threads=8)
    np.testing.assert_array_equal(fz[0], on)
    np.testing.assert_array_equal(fz[1], os_)
    np.testing.assert_array_equal(fz[2], of)


def test_fused_read_jobs_materialises_the_stream():
    arrays = mixed_arrays()
    gp = GenParams(seed=77, arrival_mode=L.MCS_ARRIVAL_REF, lam=10.0, max_cores=20, max_mem=9000, fused=True)
    with Engine(0) as eng:
        eng.load_clusters(arrays)
        eng.generate_jobs(gp, 1500)
        got = eng.read_jobs()
        eng.run()  # a fused run after the records exist still synthesises and matches
        node = eng.placements()[0]
    gp.fused = False
    want = gen_streams_host(gp, arrays, 1500)
    for f in ("arrival", "dur", "cores", "mem"):
        np.testing.assert_array_equal(getattr(got, f), getattr(want, f), err_msg=f)
    on, _, _, _ = O.fifo_run_batch(arrays, want, n_threads=8)
    np.testing.assert_array_equal(node, on)


def test_fused_slot_pool_escalation():
    arrays = replicate(uniform_cluster(256), 8)
    gp = GenParams(seed=5, arrival_mode=L.MCS_ARRIVAL_SCALED, lam=scaled_lambda(256, load=0.9), fused=True)
    node, start, fin, cs, _, st = run("FIFO", arrays, gp, 4000, slot_pool=2)
    assert st.escalations >= 1
    gp.fused = False
    on, os_, of, _ = O.fifo_run_batch(arrays, gen_streams_host(gp, arrays, 4000), n_threads=8)
    np.testing.assert_array_equal(node, on)
    np.testing.assert_array_equal(start, os_)


def test_fused_stream_drives_delay_trading():
    """The trading path reads job records: a fused stream is materialised for it on demand."""
    from mcs_amd import Cluster
    import os
    spec = Cluster.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets",
                                     "cluster_small.json"))
    arrays = replicate(spec, 6)
    res = []
    for fused in (False, True):
        gp = GenParams(seed=11, fused=fused)
        with Engine(0, policy="DELAY", trader=True) as eng:
            eng.load_clusters(arrays)
            eng.generate_jobs(gp, 600)
            eng.run()
            res.append((eng.placements(), eng.contracts()))
    for a, b in zip(res[0][0], res[1][0]):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(res[0][1], res[1][1])


@pytest.mark.parametrize("lam,k", [(10.0, 3.0), (2.5, 1.5), (40.0, 6.0)])
def test_weibull_device_records_equal_host(lam, k):
    """WEIBULL arrivals materialised by the device generator (gen_arrivals_kernel) and synthesised
    in the kernel both equal the host generator, for the reference's (Lambda 10, K 3) and others."""
    arrays = mixed_arrays()
    gp = GenParams(seed=99, arrival_mode=L.MCS_ARRIVAL_WEIBULL, lam=lam, weibull_k=k)
    with Engine(0) as eng:
        eng.load_clusters(arrays)
        eng.generate_jobs(gp, 3001)
        dev = eng.read_jobs()
    host = gen_streams_host(gp, arrays, 3001)
    for f in ("arrival", "dur", "cores", "mem"):
        np.testing.assert_array_equal(getattr(dev, f), getattr(host, f), err_msg=f)
    gp.fused = True
    fz = run("FIFO", arrays, gp, 3001)
    on, os_, of, _ = O.fifo_run_batch(arrays, host, n_threads=8)
    np.testing.assert_array_equal(fz[0], on)
    np.testing.assert_array_equal(fz[1], os_)


@pytest.mark.parametrize("policy", ["FIFO", "DELAY"])
@pytest.mark.parametrize("seed", [11, 12, 13, 14])
def test_fused_fuzz(policy, seed):
    """Random cluster shapes (1..300 nodes, random capacities and availability), arrival modes, rates,
    duration caps and Weibull shapes: the fused run equals the materialised run and the oracle over
    the host generator's streams."""
    from mcs_amd import Cluster
    from mcs_amd.cluster import Node

    rng = np.random.default_rng(seed)
    clusters = []
    for k in range(int(rng.integers(4, 24))):
        nn = int(rng.choice([int(rng.integers(1, 65)), int(rng.integers(65, 301))]))
        cc, cm = int(rng.integers(1, 64)), int(rng.integers(100, 60000))
        cl = Cluster(Id=k + 1, Nodes=[])
        for i in range(nn):
            cl.Nodes.append(Node(Id=i + 1, Cores=cc, Memory=cm, CoresAvailable=int(rng.integers(cc // 2, cc + 1)),
                                 MemoryAvailable=int(rng.integers(cm // 2, cm + 1))))
        clusters.append(cl)
    arrays = pack_clusters(clusters)
    mode = int(rng.choice([L.MCS_ARRIVAL_REF, L.MCS_ARRIVAL_SCALED, L.MCS_ARRIVAL_WEIBULL]))
    lam = float(rng.uniform(0.2, 3.0)) if mode == L.MCS_ARRIVAL_SCALED else float(rng.uniform(2.0, 40.0))
    gp = GenParams(seed=int(rng.integers(1, 1 << 62)), arrival_mode=mode, lam=lam,
                   max_dur_s=int(rng.integers(5, 900)), weibull_k=float(rng.choice([0.0, 1.5, 4.0])))
    if mode == L.MCS_ARRIVAL_WEIBULL and gp.weibull_k == 1.5:
        gp.lam = min(gp.lam, 18.0)  # the gap table vanishes within 256 entries only below scale ~20.5
    jobs = int(rng.integers(300, 1500))
    ref = run(policy, arrays, gp, jobs)
    gp.fused = True
    fz = run(policy, arrays, gp, jobs)
    for a, b, name in zip(ref[:3], fz[:3], ("node", "start", "finish")):
        np.testing.assert_array_equal(a, b, err_msg=name)
    for key in ("t_end", "placed", "waited", "peak_running", "flags"):
        np.testing.assert_array_equal(ref[3][key], fz[3][key], err_msg=key)
    gp.fused = False
    streams = gen_streams_host(gp, arrays, jobs)
    oracle = O.fifo_run_batch if policy == "FIFO" else O.delay_run_batch
    on, os_, of, _ = oracle(arrays, streams, n_threads=8)
    np.testing.assert_array_equal(fz[0], on)
    np.testing.assert_array_equal(fz[1], os_)
    np.testing.assert_array_equal(fz[2], of)


@pytest.mark.parametrize("serial", ["0", "1"])
@pytest.mark.parametrize("mode,lam,jobs", [(L.MCS_ARRIVAL_REF, 10.0, 777), (L.MCS_ARRIVAL_REF, 0.3, 130),
                                           (L.MCS_ARRIVAL_SCALED, 2.5, 1000), (L.MCS_ARRIVAL_SCALED, 40.0, 64),
                                           (L.MCS_ARRIVAL_WEIBULL, 10.0, 500), (L.MCS_ARRIVAL_WEIBULL, 3.0, 1)])
def test_fused_clock_bound_is_exact(serial, mode, lam, jobs, monkeypatch):
    """A fused stream is accepted iff every cluster's last arrival + jobs * max_dur stays below
    2^32-1 (FIFO; mcs_generate_jobs).  The last arrivals come from the device bound scan (one wave
    per cluster, or the per-thread scan with MCS_GEN_SERIAL=1); the host generator gives them
    exactly, so a max_dur_s one above / at the limit must flip the verdict."""
    monkeypatch.setenv("MCS_GEN_SERIAL", serial)
    arrays = replicate(uniform_cluster(64), 40)
    gp = GenParams(seed=1234, arrival_mode=mode, lam=lam, fused=True)
    last = max(int(gen_streams_host(gp, arrays, jobs).arrival.reshape(40, jobs)[:, -1].max()), 0)
    room = 0xFFFFFFFF - last
    md = (room - 1) // jobs  # the largest max_dur_s still accepted
    with Engine(0) as eng:
        eng.load_clusters(arrays)
        gp.max_dur_s = md
        eng.generate_jobs(gp, jobs)
        gp.max_dur_s = md + 1
        with pytest.raises(L.MCSError):
            eng.generate_jobs(gp, jobs)


@pytest.mark.parametrize("diag", ["0", "1"])
@pytest.mark.parametrize("nodes,kernel", [(256, "mcs::fifo_asm_fused_kernel<4, 8>"),
                                          (48, "mcs::fifo_asm_fused_kernel<1, 2>")], ids=["w16r", "w16s"])
@pytest.mark.parametrize("mode", [L.MCS_ARRIVAL_REF, L.MCS_ARRIVAL_SCALED, L.MCS_ARRIVAL_WEIBULL],
                         ids=["REF", "SCALED", "WEIBULL"])
def test_fused_hand_scheduled_loop(mode, nodes, kernel, diag, monkeypatch):
    """The hand-scheduled FIFO loop on a fused stream (MCS_FA_LOOP_F: GenStream between batches,
    the loop state held in its registers across them) equals the streamed hand-scheduled loop, the
    compiled fused kernel, and the oracle over the host generator's streams: placements, per-cluster
    statistics (with the counting build, its pass and release-scan counts too)."""
    monkeypatch.setenv("MCS_FIFO_DIAG", diag)
    arrays = replicate(uniform_cluster(nodes), 24)
    lam = {L.MCS_ARRIVAL_REF: 40.0, L.MCS_ARRIVAL_SCALED: scaled_lambda(nodes, load=0.95),
           L.MCS_ARRIVAL_WEIBULL: 10.0}[mode]
    gp = GenParams(seed=0xF05ED + nodes + mode, arrival_mode=mode, lam=lam)
    jobs = 3001  # a ragged last batch

    def go(fused, asm):
        monkeypatch.setenv("MCS_FIFO_ASM", asm)
        gp.fused = fused
        with Engine(0, policy="FIFO") as eng:
            eng.load_clusters(arrays)
            eng.generate_jobs(gp, jobs)
            eng.run()
            return eng.placements(), eng.cluster_stats(), eng.last_kernel

    fz, fcs, fk = go(True, "1")
    assert fk == kernel
    keys = ["t_end", "placed", "waited", "peak_running", "flags"] + (["iterations", "release_scans"] if diag == "1" else [])
    for fused, asm in ((False, "1"), (True, "0")):
        (pl, cs, k) = go(fused, asm)
        assert k != kernel
        for a, b, name in zip(pl, fz, ("node", "start", "finish")):
            np.testing.assert_array_equal(a, b, err_msg=f"{name} vs {k}")
        for key in keys if not (fused and asm == "0") else keys[:5]:
            np.testing.assert_array_equal(cs[key], fcs[key], err_msg=f"{key} vs {k}")
    gp.fused = False
    on, os_, of, _ = O.fifo_run_batch(arrays, gen_streams_host(gp, arrays, jobs), n_threads=8)
    np.testing.assert_array_equal(fz[0], on)
    np.testing.assert_array_equal(fz[1], os_)
    np.testing.assert_array_equal(fz[2], of)
