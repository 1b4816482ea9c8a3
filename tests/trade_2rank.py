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
    a, s = shard(arrays, streams, rank * per, rank * per + per)
    with Engine(0, borrow=True, trader=True) as eng:
        eng.load_clusters(a)
        eng.set_shard(rank, WORLD)
        eng.submit_jobs(s)
        run_lockstep(eng, torch_allgather())
        node, start, fin = eng.placements()
        mine = dict(node=node, start=start, finish=fin, lent=eng.lent(), trades=eng.trades(),
                    vn=eng.virtual_nodes(), t_final=eng.trade_stats()["t_final"],
                    form=eng.trade_stats()["loop_form"])
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
        print("TRADE-2RANK OK", f"world {WORLD}, {C} clusters:", len(lent), "lent runs", len(o["trades"]), "trades",
              flush=True)
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
