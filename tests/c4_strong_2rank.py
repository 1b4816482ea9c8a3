"""C4 strong sharding on ONE GPU (tests/test_gpu_parity.py): two processes, each an engine holding a
contiguous half of one system's clusters (mcs_set_shard, generation keyed by the global cluster
index, exactly as bench.py --shard strong runs on N GPUs).  Rank 0 checks that the concatenated
shard outputs equal one engine holding every cluster and the CPU oracle of the whole system.
Prints C4-STRONG-2RANK OK on success."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (os.path.join(REPO, "multi-cluster-simulator_amd"), REPO, HERE):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402

WORLD = 2
TOTAL, NODES, J = 192, 256, 3000


def worker(rank):
    import torch.distributed as dist

    from mcs_amd import Engine, GenParams, replicate, uniform_cluster
    from mcs_amd.engine import scaled_lambda
    from mcs_amd.shard import shard_range

    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    gp = GenParams(seed=0x4D43535F53494D31, arrival_mode=1, lam=scaled_lambda(NODES, load=0.9))
    lo, hi = shard_range(TOTAL, WORLD, rank)
    with Engine(0) as eng:
        eng.load_clusters(replicate(uniform_cluster(NODES), hi - lo))
        eng.set_shard(rank, WORLD)
        eng.generate_jobs(gp, J)
        st = eng.run()
        assert st.placed == (hi - lo) * J
        node, start, fin = eng.placements()
        mine = dict(node=node, start=start, finish=fin, cs=eng.cluster_stats())
    parts = [None] * WORLD
    dist.all_gather_object(parts, mine)
    if rank == 0:
        import oracle_ref as O
        from mcs_amd.engine import gen_streams_host

        arrays = replicate(uniform_cluster(NODES), TOTAL)
        with Engine(0) as eng:  # one engine, the whole system
            eng.load_clusters(arrays)
            eng.generate_jobs(gp, J)
            eng.run()
            one = eng.placements()
            one_cs = eng.cluster_stats()
        for i, k in enumerate(("node", "start", "finish")):
            got = np.concatenate([p[k] for p in parts])
            assert np.array_equal(got, one[i]), (k, np.flatnonzero(got != one[i])[:5])
        cs = np.concatenate([p["cs"] for p in parts])
        for f in ("t_end", "placed", "waited", "peak_running", "flags"):
            assert np.array_equal(cs[f], one_cs[f]), f
        streams = gen_streams_host(gp, arrays, J)
        on, os_, of, _ = O.fifo_run_batch(arrays, streams, n_threads=8)
        assert np.array_equal(one[0], on) and np.array_equal(one[1], os_) and np.array_equal(one[2], of)
        print("C4-STRONG-2RANK OK", TOTAL * J, "placements", flush=True)
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
