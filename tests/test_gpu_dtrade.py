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
from kat_util import GOLDEN, fuzz_workload, seeded_workload
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
    for key, v in k.get("stats0", {}).items():  # WaitTime statistics of cluster 0
        assert r["ds"][key][0] == v, key


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


def test_gpu_dtrade_four_ranks_gloo():
    """world = 4: a 64-cluster DELAY trading system (16 clusters per rank, reduced jobs) and a hot
    32-cluster one, four processes on device 0 over gloo == the oracle of the whole system."""
    import subprocess
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29589", MCS_WORLD="4",
               MCS_DTRADE_CASES="small:64:300,n64_hot:32:600")
    r = subprocess.run([sys.executable, os.path.join(here, "dtrade_2rank.py")], env=env, capture_output=True,
                       text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "DTRADE-2RANK OK" in r.stdout


def test_gpu_dtrade_eight_ranks_gloo():
    """world = 8, the N = 8 shape of C5-DELAY: the 64-cluster system in eight shards of 8 clusters
    (reduced jobs), eight processes on device 0 over gloo == the oracle of the whole system."""
    import subprocess
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29590", MCS_WORLD="8",
               MCS_DTRADE_CASES="small:64:300")
    r = subprocess.run([sys.executable, os.path.join(here, "dtrade_2rank.py")], env=env, capture_output=True,
                       text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "DTRADE-2RANK OK" in r.stdout


@pytest.mark.parametrize("graph", ["1", "0"])
def test_gpu_dtrade_rccl_loop_world1(graph, monkeypatch):
    """The RCCL tick loop (shape all-reduce, one in-place ncclAllGather of the exchange blocks per
    tick, mcs_dtrade.cpp dt_run_rccl) on a world-1 communicator == the graph-replayed loop."""
    monkeypatch.setenv("MCS_RCCL_GRAPH", graph)  # 1: kernels + all-gathers captured in a hipGraph; 0: eager
    arrays, streams, _ = seeded_workload("n64_hot", 8, 2000)
    g = run(arrays, streams)
    with Engine(0, policy="DELAY", trader=True) as eng:
        eng.load_clusters(arrays)
        eng.set_shard(0, 1)
        eng.comm_init(Engine.comm_unique_id())
        eng.submit_jobs(streams)
        eng.run()
        assert eng.trade_stats()["loop_form"] == (2 if graph == "1" else 1)
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


F32 = np.float32


def test_gpu_approve_trade_kat6_boundaries(engine):
    """KAT6 and neighbouring float32 boundaries of ApproveTrade (trader.go:141-167),
    evaluated by the device function both trader kernels call (mcs_approve_trade), against the
    hand-derived answers and the oracle.  TotalCore 160 / TotalMemory 120000 = cluster_small."""
    u7 = float(np.nextafter(F32(0.8), F32(0)))  # 0.79999995f
    cases = [  # (tc, tm, cu, mu, cores, mem, time_s) -> approve
        ((160, 120000, 0.5, 0.0, 80, 0, 50), 1),      # availability exactly 80.0 >= 80
        ((160, 120000, 0.5, 0.0, 81, 0, 50), 0),      # 80.0 < 81
        ((160, 120000, 0.8, 0.0, 0, 0, 0), 0),        # 0.8f < 0.8f is false
        ((160, 120000, u7, 0.0, 32, 0, 10), 1),       # 160 - 160*0.79999995f = 32.000008f >= 32
        ((160, 120000, u7, 0.0, 33, 0, 10), 0),       # 32.000008f < 33
        ((160, 120000, 0.0, 0.5, 0, 60000, 7), 1),    # memory availability exactly 60000
        ((160, 120000, 0.0, 0.5, 0, 60001, 7), 0),
        ((160, 120000, 0.0, u7, 0, 24000, 0), 1),     # 120000 - 120000*0.79999995f = 24000.006f
        ((160, 120000, 0.0, u7, 0, 24001, 0), 0),
        ((160, 120000, 0.3, 0.7, 0, 0, 0), 1),        # the zero contract: incentive -0.0 <= price 0
        ((160, 120000, float("nan"), 0.0, 0, 0, 0), 0),   # a NaN sample never passes cu < 0.8
        ((16777217, 1, 0.0, 0.0, 16777217, 0, 1), 1),  # float32(16777217) == float32(16777217): >= holds
        ((16777216, 1, 0.0, 0.0, 16777218, 0, 1), 0),  # 16777216.0 < 16777218.0
        ((0, 0, 0.0, 0.0, 0, 0, 0), 1),               # empty cluster, zero contract
    ]
    q = np.array([c for c, _ in cases], dtype=object)
    cols = [np.array([c[i] for c, _ in cases], dtype=(np.float32 if i in (2, 3) else np.uint32)) for i in range(7)]
    got = engine.approve_trade(*cols)
    want = np.array([w for _, w in cases])
    np.testing.assert_array_equal(got, want)
    orc = np.array([O.approve_trade(int(c[0]), int(c[1]), F32(c[2]), F32(c[3]), int(c[4]), int(c[5]),
                                    int(c[6]) * 1_000_000_000, 0.0) for c, _ in cases])
    np.testing.assert_array_equal(orc, want)


def test_gpu_approve_trade_sweep_vs_oracle(engine):
    """200k queries at and around the integer utilizations a cluster can sample (used/total in
    float32) with requests at the float32 availability +-1: GPU == oracle, bit for bit."""
    rng = np.random.default_rng(6)
    n = 200_000
    tc = rng.choice([160, 320, 2560, 8192, 24000, 99991, 16777215], n).astype(np.uint32)
    tm = rng.choice([120000, 240000, 6144000, 1 << 24, 3], n).astype(np.uint32)
    cu = (rng.integers(0, tc.astype(np.int64) + 1) .astype(np.float32) / tc.astype(np.float32)).astype(np.float32)
    mu = (rng.integers(0, tm.astype(np.int64) + 1).astype(np.float32) / tm.astype(np.float32)).astype(np.float32)
    av_c = (tc.astype(np.float32) - tc.astype(np.float32) * cu).astype(np.float32)
    av_m = (tm.astype(np.float32) - tm.astype(np.float32) * mu).astype(np.float32)
    kc = np.clip(np.floor(av_c).astype(np.int64) + rng.integers(-1, 2, n), 0, None).astype(np.uint32)
    km = np.clip(np.floor(av_m).astype(np.int64) + rng.integers(-1, 2, n), 0, None).astype(np.uint32)
    ks = rng.integers(0, 600, n).astype(np.uint32)
    got = engine.approve_trade(tc, tm, cu, mu, kc, km, ks)
    orc = np.array([O.approve_trade(int(tc[i]), int(tm[i]), cu[i], mu[i], int(kc[i]), int(km[i]),
                                    int(ks[i]) * 1_000_000_000, 0.0) for i in range(n)], np.int32)
    bad = np.flatnonzero(got != orc)
    assert bad.size == 0, f"{bad.size} mismatches, first {bad[:5]}"
    assert 0.2 < got.mean() < 0.8  # both outcomes are exercised


@pytest.mark.parametrize("shape,seed,J", [("w16s", 1, 300), ("w16s", 2, 300), ("mid", 3, 300),
                                          # (r04: longer streams through the grown-node pass: the
                                          # snapshot, the untested marks across rows, quiet row pairs)
                                          ("w16s", 4, 900), ("w16s", 5, 900), ("w16s", 6, 1500),
                                          ("mid", 7, 900), ("mid", 8, 1500)])
def test_gpu_dtrade_fuzz(shape, seed, J):
    """kat_util's randomised clusters and streams in a DELAY trading system (real contracts, Foreign
    jobs, virtual nodes): every output bit-exact against the oracle."""
    arrays, streams = fuzz_workload(shape, seed, n_clusters=8, J=J, blocking=False)
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


@pytest.mark.parametrize("form", ["res", "graph"])
@pytest.mark.parametrize("kind,C,J", [("small", 64, 500), ("big", 8, 800), ("n64_hot", 8, 1500), ("small", 16, 3000)])
def test_gpu_dtrade_level1_rows_equal_oracle(kind, C, J, form, monkeypatch):
    """The Level1 pass over the list with holes (DtRow summaries: only rows where a job may fit are
    visited job by job, the others take their JobsMap moves in O(1)) equals the oracle's compacted
    slice on every output: placements, contracts, Foreign jobs, virtual nodes and the WaitTime sums
    (exact clusters through the grown-node test, "big" ones through the histogram filter), in the
    resident tick (mcs_dtrade_mw.hip, loop_form 5) and the replayed kernels (MCS_DT_RESIDENT=0, 0)."""
    monkeypatch.setenv("MCS_DT_RESIDENT", "1" if form == "res" else "0")
    arrays, streams, _ = seeded_workload(kind, C, J)
    g = run(arrays, streams)
    assert g["ts"]["loop_form"] == (5 if form == "res" else 0)
    o = O.dtrade_run(arrays, streams)
    for k in ("node", "start", "finish"):
        np.testing.assert_array_equal(g[k], o[k], err_msg=k)
    assert len(g["trades"]) == len(o["trades"])
    for f in ("t", "requester", "winner", "approvals", "policy", "cores", "mem", "time_s", "failed"):
        np.testing.assert_array_equal(g["trades"][f], o["trades"][f], err_msg=f)
    assert len(g["foreign"]) == o["n_foreign"] and g["vnodes"] == o["vnodes"]
    for f in ("total_wait_ms", "jobs_count", "moved_l1", "placed_l1"):
        np.testing.assert_array_equal(g["ds"][f], o["stats"][f], err_msg=f)
    assert g["ts"]["t_final"] == o["t_final"]


@pytest.mark.parametrize("form", ["res", "graph"])
def test_gpu_dtrade_learned_capacity(form, monkeypatch):
    """C5-DELAY's own system (64 cluster_small clusters x 2000 jobs) peaks at 331 running jobs in one
    cluster: the first run overflows the 256 auto slots and escalates by half to 384; a second run of
    the same inputs starts at the learned 384 (no overflowed run), and both equal the oracle; in the
    resident tick (loop_form 5) and the replayed kernels (0)."""
    monkeypatch.setenv("MCS_DT_RESIDENT", "1" if form == "res" else "0")
    lf = 5 if form == "res" else 0
    arrays, streams, _ = seeded_workload("small", 64, 2000)
    with Engine(0, policy="DELAY", trader=True) as eng:
        eng.load_clusters(arrays)
        eng.submit_jobs(streams)
        st1 = eng.run()
        ts1 = eng.trade_stats()
        n1, s1, f1 = eng.placements()
        st2 = eng.run()
        ts2 = eng.trade_stats()
        n2, s2, f2 = eng.placements()
    assert st1.escalations == 1 and st1.slot_pool == 6 and ts1["loop_form"] == lf
    assert st2.escalations == 0 and st2.slot_pool == 6 and ts2["loop_form"] == lf
    for a, b in ((n1, n2), (s1, s2), (f1, f2)):
        np.testing.assert_array_equal(a, b)
    o = O.dtrade_run(arrays, streams)
    np.testing.assert_array_equal(n1, o["node"])
    np.testing.assert_array_equal(s1, o["start"])
    np.testing.assert_array_equal(f1, o["finish"])
    assert ts1["t_final"] == o["t_final"]


def check_equal(g, o):
    """every output of two runs of one system (run() dicts), bit for bit"""
    for k in ("node", "start", "finish"):
        np.testing.assert_array_equal(g[k], o[k], err_msg=k)
    assert g["trades"].tobytes() == o["trades"].tobytes()
    assert g["foreign"].tobytes() == o["foreign"].tobytes()
    assert g["vnodes"] == o["vnodes"]
    for f in ("total_wait_ms", "jobs_count", "moved_l1", "placed_l1"):
        np.testing.assert_array_equal(g["ds"][f], o["ds"][f], err_msg=f)
    for f in ("t_final", "ticks", "trades", "trades_won", "flags"):
        assert g["ts"][f] == o["ts"][f], f


@pytest.mark.parametrize("ticks", ["65536", "7"])
@pytest.mark.parametrize("case", ["small:64:500", "n64_hot:8:1500", "big:8:800", "small:16:3000", "n64_hot:61:400",
                                  "fuzz:w16s:4:900", "fuzz:mid:8:1500", "fuzz:w16s:6:1500"])
def test_gpu_dtrade_resident_equals_replayed(case, ticks, monkeypatch):
    """The resident tick (mcs_dtrade_mw.hip, loop_form 5: one wave per cluster keeping its nodes,
    slots and state on chip across ticks, a trader wave, granule exchange in one XCD's L2) == the
    replayed two-kernel tick (MCS_DT_RESIDENT=0, loop_form 0) on every output, and == the oracle's
    placements; MCS_DT_RES_TICKS=7 ends a launch every 7 ticks (state out and back in)."""
    p = case.split(":")
    if p[0] == "fuzz":
        arrays, streams = fuzz_workload(p[1], int(p[2]), n_clusters=8, J=int(p[3]), blocking=False)
    else:
        arrays, streams, _ = seeded_workload(p[0], int(p[1]), int(p[2]))
    monkeypatch.setenv("MCS_DT_RESIDENT", "0")
    b = run(arrays, streams)
    assert b["ts"]["loop_form"] == 0
    monkeypatch.setenv("MCS_DT_RESIDENT", "1")
    monkeypatch.setenv("MCS_DT_RES_TICKS", ticks)
    g = run(arrays, streams)
    assert g["ts"]["loop_form"] == 5, g["ts"]["loop_form"]
    check_equal(g, b)
    o = O.dtrade_run(arrays, streams)
    for k in ("node", "start", "finish"):
        np.testing.assert_array_equal(g[k], o[k], err_msg=k)
    assert g["ts"]["t_final"] == o["t_final"]


@pytest.mark.parametrize("k", DT, ids=[k["name"] for k in DT])
def test_gpu_dtrade_kats_resident(k, monkeypatch):
    """The DELAY trading KATs through the resident tick (loop_form 5), 3 ticks per launch."""
    monkeypatch.setenv("MCS_DT_RESIDENT", "1")
    monkeypatch.setenv("MCS_DT_RES_TICKS", "3")
    arrays, s = dt_system(k)
    r = run(arrays, s, t_max_s=k["t_max"])
    assert r["ts"]["loop_form"] == 5, r["ts"]["loop_form"]
    check_kat(k, r["node"], r["start"], r["finish"], r["trades"], r["foreign"], len(r["foreign"]), r["vnodes"],
              r["ts"]["t_final"])


def test_gpu_dtrade_resident_fail_over(monkeypatch):
    """A resident launch that fails over (forced after the first launch by MCS_DT_RES_FORCE_FAIL=1;
    in production: workers not all on one XCD, or an exchange timeout) redoes the run on the
    replayed kernels (loop_form 6) with the same results."""
    arrays, streams, _ = seeded_workload("n64_hot", 8, 1500)
    monkeypatch.setenv("MCS_DT_RESIDENT", "0")
    b = run(arrays, streams)
    monkeypatch.setenv("MCS_DT_RESIDENT", "1")
    monkeypatch.setenv("MCS_DT_RES_TICKS", "5")
    monkeypatch.setenv("MCS_DT_RES_FORCE_FAIL", "1")
    g = run(arrays, streams)
    assert g["ts"]["loop_form"] == 6, g["ts"]["loop_form"]
    check_equal(g, b)
