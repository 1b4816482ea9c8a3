"""N-rank lock-step trading run on ONE GPU (tests/test_gpu_trade.py): WORLD processes (env
MCS_WORLD, default 2), each an engine holding one block of the clusters on device 0, exchanging
the per-tick records over torch.distributed gloo through the caller-driven phase API (include/mcs_trade.h).  Rank 0 checks
the union against the CPU oracle.  Prints TRADE-2RANK OK on success."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (os.path.join(REPO, "multi-cluster-simulator_amd"), REPO, HERE):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402

WORLD = int(os.environ.get("MCS_WORLD", "2"))
# MCS_AGREE=1 (default): the ranks agree on the block layout first (mcs_trade_set_shape), so a system
# with no node above 64 cores runs the one-launch tick on blocks WITHOUT node snapshots — the layout
# an 8-GPU RCCL run uses; MCS_AGREE=0 keeps per-rank decisions (blocks with snapshots)
AGREE = os.environ.get("MCS_AGREE", "1") != "0"
# MCS_BIG_NODE=<cores>: node 0 of the last rank's first cluster gets that many cores (capacity and
# availability): > 64 makes its lender "big" (the agreed blocks keep the snapshots), >= 128 rules the
# one-launch tick out on that rank (the agreed form is then the three-kernel tick on every rank);
# MCS_EXPECT_MISMATCH=1: the ranks chose different layouts (no agreement) and phase 1 must refuse
MCS_BIG_NODE = int(os.environ.get("MCS_BIG_NODE", "0"))
EXPECT_MISMATCH = os.environ.get("MCS_EXPECT_MISMATCH", "0") == "1"
# the system: env MCS_TRADE_CASE = "kind:clusters:jobs" (default 8 n64_hot clusters x 1500 jobs)
KIND, C_SYS, J_SYS = (lambda k, c, j: (k, int(c), int(j)))(*os.environ.get("MCS_TRADE_CASE", "n64_hot:8:1500").split(":"))


def shard(arrays, streams, lo, hi):
    from mcs_amd import JobStreams
    from mcs_amd.cluster import ClusterArrays

    n0, n1 = int(arrays.node_off[lo]), int(arrays.node_off[hi])
    j0, j1 = int(streams.job_off[lo]), int(streams.job_off[hi])
    a = ClusterArrays(arrays.cap_c[n0:n1].copy(), arrays.cap_m[n0:n1].copy(), arrays.free_c[n0:n1].copy(),
                      arrays.free_m[n0:n1].copy(), (arrays.node_off[lo:hi + 1] - n0).astype(np.uint32))
    s = JobStreams(streams.arrival[j0:j1].copy(), streams.dur[j0:j1].copy(), streams.cores[j0:j1].copy(),
                   streams.mem[j0:j1].copy(), (streams.job_off[lo:hi + 1] - j0).astype(np.uint64))
    return a, s


def worker(rank):
    import torch.distributed as dist

    from kat_util import seeded_workload
    from mcs_amd import Engine
    from mcs_amd.engine import gen_streams_host
    from mcs_amd.shard import run_lockstep, torch_allgather

    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    C, J = C_SYS, J_SYS
    arrays, streams, gp = seeded_workload(KIND, C, J)
    per = C // WORLD
    if MCS_BIG_NODE:
        n0 = int(arrays.node_off[(WORLD - 1) * per])
        arrays.cap_c[n0] = arrays.free_c[n0] = MCS_BIG_NODE
    a, s = shard(arrays, streams, rank * per, rank * per + per)
    with Engine(0, borrow=True, trader=True) as eng:
        eng.load_clusters(a)
        eng.set_shard(rank, WORLD)
        eng.submit_jobs(s)
        if EXPECT_MISMATCH:
            from mcs_amd import MCSError

            try:
                run_lockstep(eng, torch_allgather(), agree=AGREE)
            except MCSError as ex:
                assert "another layout" in str(ex), ex
                flag = [None] * WORLD
                dist.all_gather_object(flag, True)
                if rank == 0:
                    print("TRADE-2RANK MISMATCH REFUSED", f"world {WORLD}:", str(ex), flush=True)
                dist.barrier()
                dist.destroy_process_group()
                return
            raise AssertionError("ranks with different block layouts exchanged without an error")
        run_lockstep(eng, torch_allgather(), agree=AGREE)
        node, start, fin = eng.placements()
        ts = eng.trade_stats()
        mine = dict(node=node, start=start, finish=fin, lent=eng.lent(), trades=eng.trades(),
                    vn=eng.virtual_nodes(), t_final=ts["t_final"], form=ts["loop_form"], snaps=ts["snaps"],
                    agreed=ts["agreed"], blk=ts["block_bytes"])
    if not MCS_BIG_NODE:  # (the generator draws requests from the cluster maxima: the unchanged spec only)
        # device generation keyed by the global cluster index == the host generator of the full system
        with Engine(0) as eng:
            eng.load_clusters(a)
            eng.set_shard(rank, WORLD)
            eng.generate_jobs(gp, J)
            dev = eng.read_jobs()
        full = gen_streams_host(gp, arrays, J)
        _, want = shard(arrays, full, rank * per, rank * per + per)
        for f in ("arrival", "dur", "cores", "mem"):
            assert np.array_equal(getattr(dev, f), getattr(want, f)), f
    parts = [None] * WORLD
    dist.all_gather_object(parts, mine)
    if rank == 0:
        import oracle_ref as O
        from test_trade_oracle import lent_rows, trade_rows

        o = O.trade_run(arrays, streams)
        for k in ("node", "start", "finish"):
            got = np.concatenate([p[k] for p in parts])
            assert np.array_equal(got, o[k]), (k, np.flatnonzero(got != o[k])[:5])
        lent = np.concatenate([p["lent"] for p in parts])
        want_lent = lent_rows(o["lent"])
        for r in want_lent:
            r[2] -= int(streams.job_off[r[1]])
        assert lent_rows(lent) == sorted(want_lent)
        for p in parts:
            assert trade_rows(p["trades"]) == trade_rows(o["trades"])
            assert p["vn"].tolist() == o["virtual_nodes"].tolist()
            assert p["t_final"] == o["t_final"]
            if os.environ.get("MCS_EXPECT_FORM"):
                assert p["form"] == int(os.environ["MCS_EXPECT_FORM"]), p["form"]
            if os.environ.get("MCS_EXPECT_SNAPS"):
                assert p["snaps"] == int(os.environ["MCS_EXPECT_SNAPS"]), p["snaps"]
            assert p["agreed"] == int(AGREE), p["agreed"]
            assert p["blk"] == parts[0]["blk"]
        print("TRADE-2RANK OK", f"world {WORLD}, {C} clusters:", len(lent), "lent runs", len(o["trades"]), "trades;",
              f"blocks of {parts[0]['blk']} B, snaps {parts[0]['snaps']}, agreed {parts[0]['agreed']}", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=worker, args=(r,)) for r in range(WORLD)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=500)
    codes = [p.exitcode for p in procs]
    sys.exit(0 if all(c == 0 for c in codes) else 1)
