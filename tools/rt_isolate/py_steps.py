"""Python legs of the rocprofv3 --runtime-trace exit-fault isolation.

mode torch_nccl      torch alone: a world-1 'nccl' (RCCL) process group, one all_reduce, destroyed
mode mcs_run_notorch libmcs alone (no torch import: /opt/rocm's RCCL), a world-1 communicator and a
                     small C5-DELAY run through the RCCL tick loop, engine destroyed
mode torch_mcs_run   the same after `import torch` (bench.py's order: torch's librccl is the one bound)
mode graph_notorch   libmcs alone, C5-DELAY on the graph-replayed tick loop (no communicator)
mode torch_graph     the same after torch has initialised the device
mode bench_like      bench.py's C5-DELAY sequence (torch + torch.distributed imported, the device generator,
                     a CUDA synchronize, the trade statistics, contracts and Foreign jobs read back)
mode bench_like_nodist / bench_like_submit / bench_like_noreads   the same without torch.distributed,
                     with host streams submitted instead of the device generator, without the reads
mode torch_cuda_mcs_run  the same after torch has initialised the device (a CUDA tensor and a synchronize,
                     as bench.py's barrier does)
Each prints "<mode> OK" and exits 0; the profiler's own exit decides the status seen by the caller."""
import os
import sys

mode = sys.argv[1]
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "multi-cluster-simulator_amd"), os.path.join(REPO, "tests")]

if mode == "torch_nccl":
    import torch
    import torch.distributed as dist

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29655")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    t = torch.ones(1024, device="cuda")
    dist.all_reduce(t)
    torch.cuda.synchronize()
    dist.destroy_process_group()
elif mode.startswith("bench_like"):
    import torch
    if mode != "bench_like_nodist":
        import torch.distributed  # noqa: F401
    from kat_util import seeded_workload
    from mcs_amd import Cluster, Engine, GenParams, replicate

    dev = torch.device("cuda", 0)
    eng = Engine(0, policy="DELAY", trader=True)
    eng.load_clusters(replicate(Cluster.load(os.path.join(REPO, "assets", "cluster_small.json")), 64))
    eng.set_shard(0, 1)
    if mode == "bench_like_submit":
        from mcs_amd.engine import gen_streams_host
        arrays = replicate(Cluster.load(os.path.join(REPO, "assets", "cluster_small.json")), 64)
        eng.submit_jobs(gen_streams_host(GenParams(), arrays, 200))
    else:
        eng.generate_jobs(GenParams(), 200)
    torch.cuda.synchronize(dev)
    st = eng.run()
    torch.cuda.synchronize(dev)
    assert st.placed > 0
    if mode != "bench_like_noreads":
        eng.trade_stats()
        eng.contracts()
        len(eng.foreign())
    eng.close()
else:
    if mode in ("torch_mcs_run", "torch_cuda_mcs_run", "torch_graph"):
        import torch
        if mode in ("torch_cuda_mcs_run", "torch_graph"):
            x = torch.ones(1024, device="cuda")
            torch.cuda.synchronize()
    from kat_util import seeded_workload
    from mcs_amd import Engine

    arrays, streams, _ = seeded_workload("small", 64, 200)
    with Engine(0, policy="DELAY", trader=True) as eng:
        eng.load_clusters(arrays)
        eng.set_shard(0, 1)
        if mode not in ("graph_notorch", "torch_graph"):
            eng.comm_init(Engine.comm_unique_id())
        eng.submit_jobs(streams)
        st = eng.run()
        assert st.placed > 0
print(mode, "OK", flush=True)
