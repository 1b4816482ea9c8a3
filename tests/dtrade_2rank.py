"""N-rank lock-step DELAY trading run on ONE GPU (tests/test_gpu_dtrade.py): WORLD processes (env
MCS_WORLD, default 2), each an engine holding one block of the clusters on device 0, exchanging one block per rank per tick (cluster
records + node snapshots) over torch.distributed gloo through the caller-driven phase API
(include/mcs_trade.h).  The trader rounds run replicated on both ranks.  Rank 0 checks the union of
the placements, and every rank's replicated trade / Foreign logs, against the CPU oracle of the
whole system (oracle/mcs_oracle_dtrade.c).  Prints DTRADE-2RANK OK on success."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (os.path.join(REPO, "multi-cluster-simulator_amd"), REPO, HERE):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402

WORLD = int(os.environ.get("MCS_WORLD", "2"))
# env MCS_DTRADE_CASES = "kind:clusters:jobs,..." (default: 16 cluster_small x 600, 8 n64_hot x 2000)
CASES = [(k, int(c), int(j)) for k, c, j in
         (x.split(":") for x in os.environ.get("MCS_DTRADE_CASES", "small:16:600,n64_hot:8:2000").split(","))]


def one_case(rank, kind, C, J):
    import torch.distributed as dist

    from kat_util import seeded_workload
    from mcs_amd import Engine
    from mcs_amd.shard import run_lockstep, torch_allgather
    from trade_2rank import shard

    arrays, streams, _ = seeded_workload(kind, C, J)
    per = C // WORLD
    a, s = shard(arrays, streams, rank * per, rank * per + per)
    with Engine(0, policy="DELAY", trader=True) as eng:
        eng.load_clusters(a)
        eng.set_shard(rank, WORLD)
        eng.submit_jobs(s)
        run_lockstep(eng, torch_allgather())
        node, start, fin = eng.placements()
        mine = dict(node=node, start=start, finish=fin, trades=eng.contracts(), foreign=eng.foreign(),
                    vnodes=[eng.virtual_node_caps(c) for c in range(per)], ds=eng.delay_stats(),
                    vn=eng.virtual_nodes(), t_final=eng.trade_stats()["t_final"])
    parts = [None] * WORLD
    dist.all_gather_object(parts, mine)
    if rank == 0:
        import oracle_ref as O

        o = O.dtrade_run(arrays, streams)
        for k in ("node", "start", "finish"):
            got = np.concatenate([p[k] for p in parts])
            bad = np.flatnonzero(got != o[k])
            assert bad.size == 0, (kind, k, bad[:5], got[bad[:5]], o[k][bad[:5]])
        for p in parts:  # the replicated logs are the whole system's, on every rank
            assert len(p["trades"]) == len(o["trades"]), (kind, len(p["trades"]), len(o["trades"]))
            for f in ("t", "requester", "winner", "approvals", "policy", "cores", "mem", "time_s", "failed"):
                np.testing.assert_array_equal(p["trades"][f], o["trades"][f], err_msg=f)
            assert len(p["foreign"]) == o["n_foreign"]
            for f in ("requester", "responder", "node", "start", "finish", "c", "m"):
                np.testing.assert_array_equal(p["foreign"][f], o["foreign"][f], err_msg=f)
            assert p["vn"].tolist() == [len(v) for v in o["vnodes"]]
            assert p["t_final"] == o["t_final"]
        assert sum((p["vnodes"] for p in parts), []) == o["vnodes"]
        for f in ("total_wait_ms", "jobs_count", "moved_l1", "placed_l1"):
            got = np.concatenate([p["ds"][f] for p in parts])
            np.testing.assert_array_equal(got, o["stats"][f], err_msg=f)
        won = int((o["trades"]["winner"] >= 0).sum())
        assert won > 0, kind  # the scenario exercises winning trades (Foreign jobs across ranks)
        cross = int(np.sum((o["foreign"]["requester"] // per) != (o["foreign"]["responder"] // per)))
        print(f"DTRADE-2RANK world {WORLD} {kind} C={C} J={J}: {len(o['trades'])} trades, {won} won, "
              f"{o['n_foreign']} Foreign jobs ({cross} across ranks)", flush=True)
    dist.barrier()


def worker(rank):
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    for kind, C, J in CASES:
        one_case(rank, kind, C, J)
    if rank == 0:
        print("DTRADE-2RANK OK", flush=True)
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
