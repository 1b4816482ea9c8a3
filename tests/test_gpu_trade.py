"""GPU parity of the lock-step trading path (include/mcs_trade.h, mcs_trade.hip) against the CPU
oracle (oracle/mcs_oracle_trade.c) and the hand-derived trade KATs.  Bit-exact on every output:
own placements (node / borrowed, start, finish), the lent-run log, the trade log, the virtual
nodes and the final tick.  Run on a real MI355X: ``pytest -m gpu``."""
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle_ref as O
from kat_util import fuzz_workload, seeded_workload
from mcs_amd import Engine
from mcs_amd.shard import run_lockstep
from test_trade_oracle import kat_inputs, lent_rows, load_trade_kats, trade_rows

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def gpu_trade(arrays, streams, borrow=True, trader=True, driven=False, **cad):
    cad.setdefault("t_max_s", 20_000_000)  # a stuck clock ends the run (flagged) instead of spinning
    with Engine(0, borrow=borrow, trader=trader, **cad) as eng:
        eng.load_clusters(arrays)
        eng.submit_jobs(streams)
        if driven:  # caller-driven transport with one rank: the gather is the identity
            st = run_lockstep(eng, lambda b: b)
        else:
            st = eng.run()
        node, start, fin = eng.placements()
        return dict(node=node, start=start, finish=fin, lent=eng.lent(), trades=eng.trades(),
                    virtual_nodes=eng.virtual_nodes(), stats=st, tstats=eng.trade_stats())


def oracle_lent_local(res, streams):
    """oracle lent records with the job as an index within the borrower's stream (the ABI's)."""
    rows = lent_rows(res["lent"])
    for r in rows:
        r[2] -= int(streams.job_off[r[1]])
    return sorted(rows)


def assert_trade_parity(arrays, streams, g, borrow=True, trader=True):
    o = O.trade_run(arrays, streams, borrow=borrow, trader=trader)
    for k in ("node", "start", "finish"):
        bad = np.flatnonzero(g[k] != o[k])
        assert bad.size == 0, f"{k}: {bad.size} mismatches, first jobs {bad[:5]}: gpu {g[k][bad[:5]]} " \
                              f"oracle {o[k][bad[:5]]}"
    assert lent_rows(g["lent"]) == oracle_lent_local(o, streams)
    assert trade_rows(g["trades"]) == trade_rows(o["trades"])
    np.testing.assert_array_equal(g["virtual_nodes"], o["virtual_nodes"])
    assert g["tstats"]["t_final"] == o["t_final"]
    assert g["tstats"]["flags"] == 0, g["tstats"]["flags"]
    return o


@pytest.mark.parametrize("k", load_trade_kats(), ids=lambda k: k["name"].split()[0])
def test_gpu_trade_kats(k):
    arrays, streams = kat_inputs(k)
    g = gpu_trade(arrays, streams, borrow=bool(k["borrow"]), trader=bool(k["trader"]))
    e = k["expect"]
    assert g["node"].tolist() == e["node"]
    assert g["start"].tolist() == e["start"]
    assert g["finish"].tolist() == e["finish"]
    exp_lent = sorted([r[0], r[1], r[2] - int(streams.job_off[r[1]]), r[3], r[4], r[5]] for r in e["lent"])
    assert lent_rows(g["lent"]) == exp_lent
    assert trade_rows(g["trades"]) == e["trades"]
    assert g["virtual_nodes"].tolist() == e["virtual_nodes"]
    assert g["tstats"]["t_final"] == e["t_final"]


@pytest.mark.parametrize("kind,C,J", [("small", 16, 2000), ("n64", 8, 3000), ("n64_hot", 8, 3000),
                                      ("n256", 64, 1500)])
def test_gpu_trade_seeded(kind, C, J):
    arrays, streams, _ = seeded_workload(kind, C, J)
    g = gpu_trade(arrays, streams)
    o = assert_trade_parity(arrays, streams, g)
    assert g["tstats"]["borrowed"] == int(np.sum(o["node"] == -2))


@pytest.mark.parametrize("borrow,trader", [(True, False), (False, True)])
def test_gpu_trade_one_side(borrow, trader):
    arrays, streams, _ = seeded_workload("n64_hot", 6, 2000)
    g = gpu_trade(arrays, streams, borrow=borrow, trader=trader)
    assert_trade_parity(arrays, streams, g, borrow=borrow, trader=trader)


def test_gpu_trade_caller_driven_equals_run():
    arrays, streams, _ = seeded_workload("n64_hot", 8, 1500)
    a = gpu_trade(arrays, streams)
    b = gpu_trade(arrays, streams, driven=True)
    for k in ("node", "start", "finish", "virtual_nodes"):
        np.testing.assert_array_equal(a[k], b[k])
    assert lent_rows(a["lent"]) == lent_rows(b["lent"])
    assert trade_rows(a["trades"]) == trade_rows(b["trades"])


def test_gpu_trade_cadences_and_small_lent_queue():
    """Non-default cadences reach the kernels; a LentQueue overflow is reported, not ignored."""
    arrays, streams, _ = seeded_workload("n64_hot", 6, 1500)
    g = gpu_trade(arrays, streams, trader_period_s=20, trade_ok_sleep_s=60, trade_fail_sleep_s=30, lock_s=7)
    o = O.trade_run(arrays, streams, period_s=20, trade_ok_sleep_s=60, trade_fail_sleep_s=30, lock_s=7)
    assert trade_rows(g["trades"]) == trade_rows(o["trades"])
    np.testing.assert_array_equal(g["node"], o["node"])
    from mcs_amd import MCSError

    with pytest.raises(MCSError):
        gpu_trade(arrays, streams, lent_queue_cap=1)


def run_ranks(world, port, case=None, timeout=900, **env_extra):
    """tests/trade_2rank.py with `world` processes on device 0 over gloo; returns its stdout."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MCS_WORLD=str(world))
    if case:
        env["MCS_TRADE_CASE"] = case
    env.update({k: str(v) for k, v in env_extra.items()})
    r = subprocess.run([sys.executable, os.path.join(HERE, "trade_2rank.py")], env=env, capture_output=True,
                       text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


@pytest.mark.parametrize("rk", ["1", "0"])
def test_gpu_trade_two_ranks_one_gpu(rk):
    """world = 2 shards (two processes, two engines on device 0) exchanging records over gloo via
    the caller-driven phase API == one engine holding all clusters == the oracle; in both tick forms:
    the one-launch tick (MCS_TRADE_RK=1, loop_form 9: B/C/D of tick n + A of tick n + 1 per launch,
    mcs_trade_rk.hip; agreed layout without snapshots) and the three-kernel tick (MCS_TRADE_RK=0,
    whose blocks always carry them)."""
    out = run_ranks(2, 29581 if rk == "1" else 29582, MCS_TRADE_RK=rk, MCS_EXPECT_FORM="9" if rk == "1" else "0",
                    MCS_EXPECT_SNAPS="0" if rk == "1" else "1", timeout=600)
    assert "TRADE-2RANK OK" in out


@pytest.mark.parametrize("rk,agree", [("1", "1"), ("1", "0"), ("0", "1")])
def test_gpu_trade_four_ranks_one_gpu(rk, agree):
    """world = 4 shards of a 64-cluster system (the C5 shape: 64 clusters, reduced jobs), four
    processes on device 0 exchanging blocks over gloo: rank offsets rank * blk beyond rank 1, the
    replicated trader rounds and escalation on four ranks == the oracle of the whole system; the
    one-launch tick (loop_form 9) on agreed blocks without snapshots (320 B per cluster + the tag)
    and on per-rank blocks with them, and the three-kernel tick (0)."""
    snaps = "0" if (rk == "1" and agree == "1") else "1"
    out = run_ranks(4, {"11": 29585, "10": 29583, "01": 29586}[rk + agree], "n64_hot:64:300", MCS_TRADE_RK=rk,
                    MCS_AGREE=agree, MCS_EXPECT_FORM="9" if rk == "1" else "0", MCS_EXPECT_SNAPS=snaps)
    assert "TRADE-2RANK OK world 4" in out
    assert f"snaps {snaps}, agreed {agree}" in out


@pytest.mark.parametrize("agree", ["1", "0"])
def test_gpu_trade_eight_ranks_one_gpu(agree):
    """world = 8, the N = 8 shape of BASELINE config 5: eight shards of 8 clusters of one 64-cluster
    system, eight processes on device 0 exchanging blocks over gloo through the one-launch tick
    (loop_form 9) == the oracle of the whole system.  agree=1 is the exact block layout of an
    8-GPU RCCL run (the ranks' shape agreed, no node above 64 cores: records + G tables only,
    blocks at rank * blk with the small blk); agree=0 keeps the snapshot-carrying blocks."""
    out = run_ranks(8, 29587 if agree == "1" else 29588, "n64_hot:64:300", MCS_TRADE_RK="1", MCS_AGREE=agree,
                    MCS_EXPECT_FORM="9", MCS_EXPECT_SNAPS="0" if agree == "1" else "1")
    assert "TRADE-2RANK OK world 8" in out
    blk = int(out.split("blocks of ")[1].split(" B")[0])
    # 8 clusters per rank: 8 x (64 B record + 256 B G table) + the 16-byte tag without snapshots;
    # with them, 8 x 64 nodes x 8 B more
    assert blk == 8 * 320 + 16 + (0 if agree == "1" else 8 * 64 * 8), blk


@pytest.mark.parametrize("big,agree,form,snaps", [(100, "1", "9", "1"), (200, "1", "0", "1")])
def test_gpu_trade_ranks_heterogeneous_agreed(big, agree, form, snaps):
    """A shard that differs from the others: one rank holds a node of `big` cores.  At 100 cores its
    lender can be "big", so the agreed blocks keep the snapshots on every rank; at 200 the slot
    payload no longer packs, so the agreed form is the three-kernel tick on every rank.  Both ==
    the oracle of the whole system (world 4)."""
    out = run_ranks(4, 29589 if big == 100 else 29590, "n64_hot:32:300", MCS_BIG_NODE=big, MCS_AGREE=agree,
                    MCS_EXPECT_FORM=form, MCS_EXPECT_SNAPS=snaps)
    assert "TRADE-2RANK OK world 4" in out


def test_gpu_trade_ranks_layout_mismatch_refused():
    """Without an agreed shape, a rank with a 200-core node runs the three-kernel tick while the
    others run the one-launch tick on equally sized blocks: phase 1 sees the other ranks' layout
    tags and fails with MCS_E_INVALID on every rank instead of exchanging silently (world 4)."""
    out = run_ranks(4, 29591, "n64_hot:32:300", MCS_BIG_NODE=200, MCS_AGREE="0", MCS_EXPECT_MISMATCH="1")
    assert "TRADE-2RANK MISMATCH REFUSED world 4" in out


@pytest.mark.parametrize("rk", ["1", "0"])
@pytest.mark.parametrize("graph", ["1", "0"])
def test_gpu_trade_rccl_loop_world1(graph, rk, monkeypatch):
    """The RCCL tick loop (one ncclAllGather per tick, mcs_trade.cpp run_rccl), captured in a hipGraph or eager, on a world-1
    communicator == the HBM-exchange loop: exercises the RCCL transport on a one-GPU box."""
    monkeypatch.setenv("MCS_RCCL_GRAPH", graph)  # 1: kernels + all-gathers captured in a hipGraph; 0: eager
    monkeypatch.setenv("MCS_TRADE_RK", rk)  # 1: one launch per tick (loop_form 7 / 8), 0: three kernels (2 / 1)
    arrays, streams, _ = seeded_workload("n64_hot", 8, 1500)
    want = gpu_trade(arrays, streams)
    with Engine(0, borrow=True, trader=True, t_max_s=20_000_000) as eng:
        eng.load_clusters(arrays)
        eng.set_shard(0, 1)
        eng.comm_init(Engine.comm_unique_id())
        eng.submit_jobs(streams)
        eng.run()
        assert eng.trade_stats()["loop_form"] == ((7 if graph == "1" else 8) if rk == "1" else (2 if graph == "1" else 1))
        node, start, fin = eng.placements()
        got = dict(lent=eng.lent(), trades=eng.trades(), vn=eng.virtual_nodes(), ts=eng.trade_stats())
    np.testing.assert_array_equal(node, want["node"])
    np.testing.assert_array_equal(start, want["start"])
    np.testing.assert_array_equal(fin, want["finish"])
    assert got["lent"].tobytes() == want["lent"].tobytes()
    assert got["trades"].tobytes() == want["trades"].tobytes()
    assert got["vn"].tolist() == want["virtual_nodes"].tolist()
    assert got["ts"]["t_final"] == want["tstats"]["t_final"]


def test_gpu_trade_config5_full_size():
    """BASELINE config 5 at its stated size: 64 clusters x 256 nodes x 156,250 jobs (10M jobs),
    FIFO + borrow + trader in lock-step, against the trading oracle of the whole system (about a
    minute of host time).  Every own placement, every lent run, every trade and the final tick."""
    from mcs_amd import GenParams, replicate, uniform_cluster
    from mcs_amd.engine import scaled_lambda

    C, J = 64, 156_250
    arrays = replicate(uniform_cluster(256), C)
    gp = GenParams(seed=0x4D43535F53494D31, arrival_mode=1, lam=scaled_lambda(256, load=0.9))
    with Engine(0, borrow=True, trader=True) as eng:
        eng.load_clusters(arrays)
        eng.generate_jobs(gp, J)
        eng.run()
        node, start, fin = eng.placements()
        lent = eng.lent()
        trades = eng.trades()
        vn = eng.virtual_nodes()
        ts = eng.trade_stats()
        streams = eng.read_jobs()
    assert ts["flags"] == 0, ts["flags"]
    o = O.trade_run(arrays, streams, lent_cap=len(lent) + 1, trade_cap=len(trades) + 1)
    assert o["n_lent"] == len(lent) and o["n_trades"] == len(trades)
    for k, g in (("node", node), ("start", start), ("finish", fin)):
        bad = np.flatnonzero(g != o[k])
        assert bad.size == 0, f"{k}: {bad.size} mismatches, first jobs {bad[:5]}"
    ol = o["lent"].copy()
    ol["job"] -= streams.job_off[ol["borrower"]]  # the ABI's job index is within the borrower's stream

    def canon(x):
        x = x[np.lexsort((x["job"], x["borrower"], x["lender"], x["start"]))]
        return [x[f] for f in ("lender", "borrower", "job", "node", "start", "finish")]

    for a, b in zip(canon(lent), canon(ol)):
        np.testing.assert_array_equal(a, b)
    assert trade_rows(trades) == trade_rows(o["trades"])
    np.testing.assert_array_equal(vn, o["virtual_nodes"])
    assert ts["t_final"] == o["t_final"]


@pytest.mark.parametrize("shape,seed", [("w16s", 1), ("w16s", 2), ("mid", 3), ("w16r", 4)])
def test_gpu_trade_fuzz(shape, seed):
    """kat_util's randomised clusters and streams (mixed node counts and availability, bursts, idle
    stretches, zero-duration and zero-resource jobs) in a FIFO trading system: placements, borrows,
    lent runs, trades, virtual nodes and the final tick bit-exact against the oracle."""
    arrays, streams = fuzz_workload(shape, seed, n_clusters=12, J=500, blocking=False)
    g = gpu_trade(arrays, streams)
    assert_trade_parity(arrays, streams, g)


@pytest.mark.parametrize("kind,C,J,pool", [("n64_hot", 8, 1500, 0), ("n256", 16, 3000, 8), ("n256", 16, 3000, 0),
                                           ("small", 64, 1500, 0), ("n256", 40, 2000, 16), ("n64", 33, 2000, 4)])
def test_gpu_trade_resident_equals_kernels_and_oracle(kind, C, J, pool, monkeypatch):
    """The system resident on the GPU for the whole run, in its two forms — one workgroup per 4
    clusters trading records as tagged granules (mcs_trade_mw.hip; loop_form 4, the default for one
    engine of <= 64 clusters of <= 256 nodes with 256/512/1024 slots) and all of it in one
    workgroup (mcs_trade_res.hip; MCS_TRADE_RESIDENT=1, loop_form 3) — == the graph-replayed tick
    kernels (MCS_TRADE_RESIDENT=0, loop_form 0) == the oracle, on every output.  The workgroup form
    runs twice: its workers 8 blocks apart (the default; loop_form 5 when they all landed on one XCD
    and traded through its L2) and consecutive (MCS_MW_XCD=0: the write-through exchange across
    XCDs, loop_form 4; 5 again for a single workgroup)."""
    arrays, streams, _ = seeded_workload(kind, C, J)
    res = {}
    for mode, xcd in (("2", "1"), ("2u", "0"), ("1", "1"), ("0", "1")):
        monkeypatch.setenv("MCS_TRADE_RESIDENT", mode[0])
        monkeypatch.setenv("MCS_MW_XCD", xcd)
        res[mode] = gpu_trade(arrays, streams, slot_pool=pool)
    lf = {m: res[m]["tstats"]["loop_form"] for m in res}
    assert lf["2"] in (4, 5) and lf["1"] == 3 and lf["0"] == 0, lf
    # (one workgroup, necessarily on one XCD, when C fits the smallest workgroup the kernel is built with)
    assert lf["2u"] == 5 if C <= 4 else lf["2u"] in (4, 5), lf
    for m in ("2", "2u", "1"):
        for k in ("node", "start", "finish"):
            np.testing.assert_array_equal(res[m][k], res["0"][k], err_msg=f"{k} mode {m}")
        assert lent_rows(res[m]["lent"]) == lent_rows(res["0"]["lent"])
        assert res[m]["trades"].tobytes() == res["0"]["trades"].tobytes()
        np.testing.assert_array_equal(res[m]["virtual_nodes"], res["0"]["virtual_nodes"])
        for f in ("placed", "borrowed", "waited", "undecided", "lent_runs", "lent_pending", "trades", "trades_won",
                  "ticks", "t_final", "flags"):
            assert res[m]["tstats"][f] == res["0"]["tstats"][f], (f, m)
    assert_trade_parity(arrays, streams, res["2"])


@pytest.mark.parametrize("kind,C,J,pool", [("n256", 16, 3000, 8), ("small", 64, 1500, 0), ("n64", 33, 2000, 4)])
def test_gpu_trade_resident_write_through_form(kind, C, J, pool, monkeypatch):
    """The uncached write-through exchange of the workgroup-resident tick (loop_form 4) pinned
    explicitly: MCS_MW_FORCE_UC=1 makes every launch take it whatever XCDs its workers landed on (the
    default picks the L2 exchange, form 5, when they share one), and it must equal the oracle."""
    monkeypatch.setenv("MCS_TRADE_RESIDENT", "2")
    monkeypatch.setenv("MCS_MW_FORCE_UC", "1")
    arrays, streams, _ = seeded_workload(kind, C, J)
    g = gpu_trade(arrays, streams, slot_pool=pool)
    assert g["tstats"]["loop_form"] == 4, g["tstats"]["loop_form"]
    assert_trade_parity(arrays, streams, g)


def test_gpu_trade_resident_form_by_capacity(monkeypatch):
    """The workgroup-resident tick packs a running slot's payload into 32 bits, so the engine picks
    it only when every node's max(capacity, availability) is below 128 cores and 65536 memory: a
    system with 200-core nodes runs the one-workgroup form instead, and both equal the oracle."""
    from mcs_amd import GenParams, gen_streams_host, replicate, uniform_cluster
    from mcs_amd.engine import scaled_lambda

    monkeypatch.delenv("MCS_TRADE_RESIDENT", raising=False)
    for cores, want in ((127, 4), (200, 3)):
        arrays = replicate(uniform_cluster(64, cores=cores, memory=65535), 12)
        gp = GenParams(seed=cores, arrival_mode=1, lam=scaled_lambda(64, load=1.1), max_cores=cores, max_mem=65535)
        streams = gen_streams_host(gp, arrays, 1500)
        g = gpu_trade(arrays, streams)
        assert g["tstats"]["loop_form"] in ((4, 5) if want == 4 else (want,)), cores
        assert_trade_parity(arrays, streams, g)


@pytest.mark.parametrize("shape,seed", [("w16s", 5), ("w16s", 17), ("mid", 3), ("w16r", 9)])
def test_gpu_trade_one_launch_tick_fuzz(shape, seed, monkeypatch):
    """The one-launch tick (mcs_trade_rk.hip) on the caller-driven path at world 1 (loop_form 9) over
    kat_util's randomised systems (mixed node counts and availability, bursts, idle stretches,
    zero-duration and zero-resource jobs) == the oracle on every output."""
    monkeypatch.setenv("MCS_TRADE_RK", "1")
    arrays, streams = fuzz_workload(shape, seed, n_clusters=12, J=500, blocking=False)
    g = gpu_trade(arrays, streams, driven=True)
    assert g["tstats"]["loop_form"] == 9, g["tstats"]["loop_form"]
    assert_trade_parity(arrays, streams, g)


def test_gpu_trade_one_launch_tick_c5_shape_rccl(monkeypatch):
    """The C5 shape (64 clusters x 256 nodes, 1024 slots: 16 slot rows) through the RCCL loop of the
    one-launch tick on a world-1 communicator (loop_form 7) == the oracle."""
    monkeypatch.setenv("MCS_TRADE_RK", "1")
    arrays, streams, _ = seeded_workload("n256", 64, 400)
    want = gpu_trade(arrays, streams)
    with Engine(0, borrow=True, trader=True, t_max_s=20_000_000) as eng:
        eng.load_clusters(arrays)
        eng.set_shard(0, 1)
        eng.comm_init(Engine.comm_unique_id())
        eng.submit_jobs(streams)
        eng.run()
        assert eng.trade_stats()["loop_form"] == 7, eng.trade_stats()["loop_form"]
        node, start, fin = eng.placements()
        lent, trades, vn = eng.lent(), eng.trades(), eng.virtual_nodes()
    np.testing.assert_array_equal(node, want["node"])
    np.testing.assert_array_equal(start, want["start"])
    np.testing.assert_array_equal(fin, want["finish"])
    assert lent_rows(lent) == lent_rows(want["lent"])
    assert trade_rows(trades) == trade_rows(want["trades"])
    np.testing.assert_array_equal(vn, want["virtual_nodes"])


def test_gpu_trade_caller_driven_256_nodes_world1():
    """The caller-driven path at world 1 with 256-node clusters keeps the automatic slot pool (the
    512-slot start is trade_run's, for a resident form only): no capacity error, == the oracle."""
    arrays, streams, _ = seeded_workload("n256", 16, 1500)
    g = gpu_trade(arrays, streams, driven=True)
    assert_trade_parity(arrays, streams, g)


@pytest.mark.parametrize("ticks", ["64", "1000"])
def test_gpu_trade_resident_short_launches(ticks, monkeypatch):
    """The resident tick over many short launches (MCS_TRADE_RES_TICKS): granule epochs count from
    the run's first tick, so a line a previous launch left in an XCD's L2 never matches; placements,
    lent log and trades == the replayed kernels (MCS_TRADE_RESIDENT=0) == the oracle."""
    arrays, streams, _ = seeded_workload("n256", 64, 1200)
    monkeypatch.setenv("MCS_TRADE_RES_TICKS", ticks)
    a = gpu_trade(arrays, streams)
    assert a["tstats"]["loop_form"] in (4, 5)
    monkeypatch.delenv("MCS_TRADE_RES_TICKS")
    monkeypatch.setenv("MCS_TRADE_RESIDENT", "0")
    b = gpu_trade(arrays, streams)
    assert b["tstats"]["loop_form"] == 0
    for k in ("node", "start", "finish", "virtual_nodes"):
        np.testing.assert_array_equal(a[k], b[k])
    assert lent_rows(a["lent"]) == lent_rows(b["lent"])
    assert trade_rows(a["trades"]) == trade_rows(b["trades"])
    assert a["tstats"]["t_final"] == b["tstats"]["t_final"]
    assert_trade_parity(arrays, streams, a)


def test_gpu_trade_resident_timeout_falls_back(monkeypatch):
    """A resident exchange that times out (forced after the first launch) is redone from the start
    on the replayed kernels (loop_form 6) instead of failing the run; results == the oracle."""
    arrays, streams, _ = seeded_workload("n256", 64, 1200)
    monkeypatch.setenv("MCS_TRADE_RES_TICKS", "256")
    monkeypatch.setenv("MCS_MW_FORCE_TIMEOUT", "1")
    g = gpu_trade(arrays, streams)
    assert g["tstats"]["loop_form"] == 6
    assert_trade_parity(arrays, streams, g)
