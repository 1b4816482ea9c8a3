#!/usr/bin/env python3
"""bench.py — headline benchmark: job placements/sec at 4096 clusters x 256 nodes (BASELINE.json).

One "step" = one full pass of the hot path over one batch of synthetic input: mcs_run simulates the
reference FIFO loop (pkg/scheduler/scheduler.go:216-296) for every cluster of the shard from its
spec until every job is placed.  Inputs (job streams) are generated on the device before the timed
region and stay resident in HBM.

Configs (BASELINE.json `configs`):
  c4 (default, the headline) — 4096 clusters x 256 nodes, FIFO, no trading.  Multi-GPU: one process
     per GPU (torchrun); with --shard strong (default) the 4096 clusters of ONE system are split in
     contiguous blocks over the ranks, each cluster keyed by its global index, so every rank
     regenerates exactly the streams the 1-GPU run simulates ("scaling": "strong"); --shard weak
     gives every rank its own 4096 clusters ("scaling": "weak").  No data-path collective: clusters
     are independent; torch.distributed carries only the barrier and the max/sum around the timed
     region.
  c3 — 1024 cluster_small replicas per GPU, FIFO, the reference client's arrivals (weak).
  c2 — one cluster_big cluster with 1M jobs (a single wave: a latency line, replicas only on N>1).
  c5 — the lock-step trading system (64 clusters, borrow + trader; --policy delay: DELAY + real
     contracts), sharded over the ranks with RCCL all-gathers.

Ranks: `python bench.py --gpus N` (WORLD_SIZE unset, N > 1) is a parent that never touches a GPU: it
spawns torchrun with N ranks on this node (127.0.0.1) and exits with their status; rank 0 prints the
line.  Under an external torchrun WORLD_SIZE must equal --gpus.  Any mismatch (WORLD_SIZE != --gpus,
fewer visible GPUs than ranks) exits 2 without printing a line, so an N-GPU line is never a 1-GPU run.

Prints ONE JSON line on rank 0 (contract in the task statement), with "roofline" (HBM-bound:
28 algorithmic bytes per placement; the kernel is latency-bound, see "limiter") and
"cpu_baseline" (the naive CPU oracle, rank 0, N=1, with the host's core count and CPU model).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "multi-cluster-simulator_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
BYTES_PER_PLACEMENT = 28  # 16 B job record read + 12 B result write
BYTES_PER_PLACEMENT_FUSED = 12  # --gen fused: the record is synthesised in registers, only results move
LIMITER = ("latency: each cluster is a serial chain of decisions (one wave per cluster); the bound is the "
           "per-decision dependency chain and issue work (DESIGN.md §7)")


def limiter_text(traffic, algorithmic):
    """The roofline limiter of this workload: the chain, with the measured HBM traffic against the
    algorithmic bytes when a PMC pass of the same shape exists (profiles/)."""
    if traffic is None:
        return LIMITER + "; HBM traffic of this workload not measured (no PMC file of this shape)"
    r = traffic / max(algorithmic, 1.0)
    return LIMITER + f"; PMC HBM traffic {r:.2f}x the algorithmic bytes" + (
        " (no wasted re-reads)" if r < 1.1 else " (bytes beyond the algorithmic ones: DESIGN.md §10)")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", choices=["c2", "c3", "c4", "c5"], default="c4",
                    help="c4: the headline FIFO benchmark; c3: 1024 cluster_small replicas per GPU; c2: one "
                         "cluster_big with 1M jobs; c5: the lock-step borrow + trader system")
    ap.add_argument("--shard", choices=["strong", "weak"], default="strong",
                    help="c4 over N GPUs: strong = the 4096 clusters of one system split over the ranks "
                         "(BASELINE configs[3]); weak = 4096 clusters per rank")
    ap.add_argument("--clusters", type=int, default=0,
                    help="c4: clusters of the system (strong) or per GPU (weak); c3: replicas per GPU; "
                         "c5: clusters of the whole trading system")
    ap.add_argument("--nodes", type=int, default=256)
    ap.add_argument("--jobs-per-cluster", type=int, default=0)
    ap.add_argument("--load", type=float, default=0.9, help="offered memory load of the scaled arrivals")
    ap.add_argument("--lam", type=float, default=0.0,
                    help="c4: per-second arrival rate of the scaled arrivals (0 = from --load)")
    ap.add_argument("--max-dur", type=int, default=600,
                    help="c4: durations U{0..max_dur-1} s (600 = rand.Intn(600), client.go:98)")
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0x4D43535F53494D31)
    ap.add_argument("--cpu-sample-clusters", type=int, default=0,
                    help="CPU baseline sample: that many clusters with full streams (0 = per-config default, "
                         "about 10-30 s of oracle work)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = every usable host cpu: the affinity set capped by the cgroup CPU quota (SURVEY §8d: "
                         "OpenMP over clusters on all host cores)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--slot-pool", type=int, default=0,
                    help="c5: running slots per cluster / 64 (0 = the engine's default, 4 x nodes)")
    ap.add_argument("--comm", action="store_true",
                    help="c5: run the RCCL tick loop (ncclAllGather per tick) even at N=1, on a world-1 "
                         "communicator (MCS_RCCL_GRAPH=0: eager launches instead of the captured hipGraph)")
    ap.add_argument("--traffic-json", default=None,
                    help="per-launch HBM bytes measured by a separate rocprofv3 --pmc pass (profile figure)")
    ap.add_argument("--policy", choices=["fifo", "delay"], default="fifo",
                    help="fifo (the headline, Scheduler.Fifo) or delay (Scheduler.Delay, the reference's "
                         "default policy, scheduler.go:116)")
    ap.add_argument("--gen", choices=["stream", "fused"], default="stream",
                    help="job stream: 'stream' = records generated before the timed region and read from HBM "
                         "(SURVEY §8d, 28 B/placement); 'fused' = synthesised inside the placement kernel "
                         "(SURVEY §8f row 3, 12 B/placement)")
    a = ap.parse_args()
    defaults = {  # (clusters, jobs per cluster, cpu sample clusters)
        "c4": (4096, 16384, 4096),
        "c3": (1024, 65536, 1024),
        "c2": (1, 1_000_000, 1),
        "c5": (64, 2000 if a.policy == "delay" else 156250, 16 if a.policy == "delay" else 64),
    }[a.config]
    a.clusters = a.clusters or defaults[0]
    a.jobs_per_cluster = a.jobs_per_cluster or defaults[1]
    a.cpu_sample_explicit = a.cpu_sample_clusters != 0
    a.cpu_sample_clusters = a.cpu_sample_clusters or defaults[2]
    if a.traffic_json is None:
        a.traffic_json = os.path.join(REPO, "profiles", "traffic_latest" + ("_delay" if a.policy == "delay" else "")
                                      + ("_fused" if a.gen == "fused" else "")
                                      + (f"_lam{a.lam:g}_dur{a.max_dur}" if a.lam or a.max_dur != 600 else "") + ".json")
    return a


def host_info(n_threads):
    """What the CPU baseline ran on: usable cores, the machine's cpus and the CPU model."""
    model = platform.processor() or "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = os.cpu_count() or 1
    quota = None
    try:  # cgroup v2 CPU quota ("max 100000" = none): the cores the threads can actually occupy
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
            quota = None if q == "max" else float(q) / float(p)
    except (OSError, ValueError):
        pass
    return {"threads": n_threads, "host_nproc": os.cpu_count(), "host_usable_cpus": usable,
            "cgroup_cpu_quota": quota, "cpu_model": model}


def usable_cpus():
    """cpus this process may run on: the affinity set, capped by the cgroup's CPU quota (on the GPU
    box 256 cpus are visible but the quota is 16: 256 threads then time-slice on 16 cpus' worth)"""
    try:
        n = len(os.sched_getaffinity(0)) or 1
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    q = host_info(0)["cgroup_cpu_quota"]
    return max(1, min(n, int(q + 0.5))) if q else n


CPU_BUDGET_S = 15.0  # target wall time of one CPU baseline sample (the pilot sizes it)
NAIVE = ("the CPU oracle is the deliberately naive restatement of the Go loop (it rescans the running "
         "list on every pass); it is a reported baseline, not the target")


def cpu_baseline_c5(args, lam, sample_jobs):
    """The trading oracle (oracle/mcs_oracle_trade.c, sequential lock-step, 1 thread) on the same
    64-cluster system with shorter streams (sample_jobs per cluster)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_ref as O
    from mcs_amd import GenParams, replicate, uniform_cluster
    from mcs_amd.engine import gen_streams_host

    arrays = replicate(uniform_cluster(args.nodes), args.clusters)
    gp = GenParams(seed=args.seed, arrival_mode=1, lam=lam)
    streams = gen_streams_host(gp, arrays, sample_jobs)
    O.lib()
    t0 = time.perf_counter()
    r = O.trade_run(arrays, streams, lent_cap=1, trade_cap=1)
    dt = time.perf_counter() - t0
    return {
        "value": streams.n_jobs / dt,
        "unit": "job decisions/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{args.clusters} clusters x {args.nodes} nodes x {sample_jobs} jobs ({streams.n_jobs} jobs, "
                  f"{r['n_lent']} lent runs, {r['t_final']} ticks), oracle/mcs_oracle_trade.c -O3, 1 thread, "
                  f"{dt:.2f} s wall; {NAIVE}",
        "seconds": dt,
        "host": host_info(1),
    }


def main_c5_delay(args, world, rank, local_rank):
    """C5 with DELAY schedulers: args.clusters cluster_small replicas with the
    reference client's arrivals, Delay loops + traders with real contracts in lock-step.  The system
    is split in equal blocks over the ranks; with world > 1 each tick all-gathers one exchange block
    per rank over RCCL (mcs_trade.h) and every rank runs the trader rounds replicated."""
    import torch
    import torch.distributed as dist

    from mcs_amd import Cluster, Engine, GenParams, replicate
    from mcs_amd.shard import aggregate

    dist_on = world > 1
    if dist_on:
        torch.cuda.set_device(local_rank)
        dist.init_process_group(backend="nccl")
    dev = torch.device("cuda", local_rank)
    spec = Cluster.load(os.path.join(REPO, "assets", "cluster_small.json"))
    if args.clusters % world:
        raise SystemExit(f"--clusters {args.clusters} must divide over {world} ranks")
    per = args.clusters // world
    eng = Engine(local_rank, policy="DELAY", trader=True)
    eng.load_clusters(replicate(spec, per))
    eng.set_shard(rank, world)
    eng.generate_jobs(GenParams(seed=args.seed), args.jobs_per_cluster)  # keyed by the global cluster
    if dist_on:
        box = [Engine.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        eng.comm_init(box[0])
    elif args.comm:
        eng.comm_init(Engine.comm_unique_id())
    n_jobs = eng.num_jobs

    def barrier():
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize(dev)

    for _ in range(args.warmup):
        eng.run()
    barrier()
    t0 = time.perf_counter()
    kernel_ms, decided, escalations = [], 0, 0
    for _ in range(args.steps):
        st = eng.run()
        kernel_ms.append(st.kernel_ms)
        decided += st.placed
        escalations += st.escalations
    barrier()
    elapsed = time.perf_counter() - t0
    elapsed_max, decided_all = aggregate(elapsed, decided, device=dev)
    ts = eng.trade_stats()
    tr = eng.contracts()
    if rank == 0:
        avg_kernel_s = sum(kernel_ms) / len(kernel_ms) / 1e3
        achieved = decided / args.steps * BYTES_PER_PLACEMENT / avg_kernel_s / 1e9
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            sys.path.insert(0, os.path.join(REPO, "tests"))
            import oracle_ref as O
            from mcs_amd.engine import gen_streams_host

            k = min(args.cpu_sample_clusters, args.clusters)
            jk = min(args.jobs_per_cluster, 1000)
            arrays = replicate(spec, k)
            streams = gen_streams_host(GenParams(seed=args.seed), arrays, jk)
            O.lib()
            c0 = time.perf_counter()
            r = O.dtrade_run(arrays, streams, trade_cap=1, foreign_cap=1)
            dt = time.perf_counter() - c0
            cpu = {"value": float((r["node"] >= 0).sum()) / dt, "unit": "job placements/s", "cores": 1,
                   "kind": "port",
                   "sample": f"{k} cluster_small x {jk} jobs ({streams.n_jobs} jobs, {r['n_trades']} trader rounds, "
                             f"{r['t_final']} ticks), oracle/mcs_oracle_dtrade.c -O3, 1 thread, {dt:.2f} s wall; "
                             f"{NAIVE}",
                   "seconds": dt, "host": host_info(1)}
        out = {
            "metric": "trading-system job placements/sec with DELAY schedulers (real contracts)",
            "value": decided_all / elapsed_max,
            "unit": "placements/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (seeded device generator restating pkg/client/client.go, Poisson(10)/min arrivals)",
            "config": {
                "workload": f"C5-DELAY: {args.clusters} cluster_small clusters, Delay + traders in lock-step, "
                            f"{args.jobs_per_cluster} jobs/cluster ({n_jobs} jobs), reference client arrivals",
                "clusters_total": args.clusters,
                "nodes": 5,
                "jobs_per_cluster": args.jobs_per_cluster,
                "parallelism": f"one system sharded over {world} GPU(s), {per} clusters each; "
                               + ("one RCCL all-gather of the exchange blocks per tick" if world > 1 else
                                  "exchange in HBM")
                               + " (tick loop: " + ("graph-replayed" if ts["loop_form"] == 0 else "graph-replayed after a resident timeout" if ts["loop_form"] == 6 else "RCCL eager" if ts["loop_form"] == 1
                                                    else "RCCL captured in a hipGraph" if ts["loop_form"] == 2
                                                    else "resident in one workgroup" if ts["loop_form"] == 3
                                                    else "one launch per tick, captured with the all-gather in a hipGraph" if ts["loop_form"] == 7
                                                    else "one launch per tick, eager" if ts["loop_form"] == 8
                                                    else "one launch per tick, caller-driven" if ts["loop_form"] == 9
                                                    else "resident, one wave per cluster (4 per workgroup) and a "
                                                         "trader wave, all on one XCD (L2 exchange)") + ")",
            },
            "roofline": {
                "bound": "hbm",
                "limiter": ("latency: one workgroup runs every cluster's Delay iteration, then the trader rounds, "
                            "per tick (DESIGN.md §11)" if ts["loop_form"] == 3 else
                            "latency: the busiest cluster's own Delay iterations (the waves run ahead of each other "
                            "between trader rounds), and a meeting of every wave at each tick with a round "
                            "(DESIGN.md §11)" if ts["loop_form"] == 5 else
                            "launch/latency: a tick is dependent launches of a few us (DESIGN.md §11)"),
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": None,
                "kernel": ("dt_res_kernel (resident tick, the whole system in one workgroup)" if ts["loop_form"] == 3
                           else "dt_mw_kernel (resident tick, one wave per cluster and a trader wave)"
                           if ts["loop_form"] == 5
                           else "lock-step tick (dt_step with the sample, dt_trader), launch/latency-bound"),
                "kernel_ms_avg": avg_kernel_s * 1e3,
                "bytes_per_placement": BYTES_PER_PLACEMENT,
            },
            "cpu_baseline": cpu,
            "trading": {"ticks": ts["ticks"], "t_final": ts["t_final"],
                        "us_per_tick": avg_kernel_s * 1e6 / max(ts["ticks"], 1), "trades": ts["trades"],
                        "trades_won": ts["trades_won"], "wait_time_rounds": int((tr["policy"] == 0).sum()),
                        "foreign_jobs": int(len(eng.foreign())), "flags": ts["flags"], "loop_form": ts["loop_form"],
                        "slot_pool": st.slot_pool, "escalations_in_timed_runs": escalations},
        }
        if dist_on:  # the RCCL communicator's size, as torch.distributed sees it
            out["world"] = world
            out["comm_world"] = dist.get_world_size()
        print(json.dumps(out), flush=True)
    eng.close()
    if dist_on:
        dist.destroy_process_group()


def main_c5(args, world, rank, local_rank):
    """C5: the whole trading system (args.clusters clusters) split in equal blocks over the ranks,
    one lock-step run per step; the per-tick record exchanges are RCCL all-gathers over xGMI
    when world > 1 (mcs_trade.h)."""
    import torch
    import torch.distributed as dist

    from mcs_amd import Engine, GenParams, replicate, uniform_cluster
    from mcs_amd.engine import scaled_lambda
    from mcs_amd.shard import aggregate

    dist_on = world > 1
    if dist_on:
        torch.cuda.set_device(local_rank)
        dist.init_process_group(backend="nccl")
    dev = torch.device("cuda", local_rank)
    if args.clusters % world:
        raise SystemExit(f"--clusters {args.clusters} must divide over {world} ranks")
    per = args.clusters // world
    lam = scaled_lambda(args.nodes, load=args.load)
    eng = Engine(local_rank, borrow=True, trader=True, slot_pool=args.slot_pool)
    eng.load_clusters(replicate(uniform_cluster(args.nodes), per))
    eng.set_shard(rank, world)
    eng.generate_jobs(GenParams(seed=args.seed, arrival_mode=1, lam=lam), args.jobs_per_cluster)
    if dist_on:
        box = [Engine.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        eng.comm_init(box[0])
    elif args.comm:
        eng.comm_init(Engine.comm_unique_id())
    n_jobs = eng.num_jobs

    def barrier():
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize(dev)

    for _ in range(args.warmup):
        eng.run()
    barrier()
    t0 = time.perf_counter()
    kernel_ms, decided = [], 0
    for _ in range(args.steps):
        st = eng.run()
        kernel_ms.append(st.kernel_ms)
        decided += st.placed + (n_jobs - st.placed - st.unplaced)  # placed + borrowed
    barrier()
    elapsed = time.perf_counter() - t0
    elapsed_max, decided_all = aggregate(elapsed, decided, device=dev)
    ts = eng.trade_stats()
    _, lent_all = aggregate(0.0, ts["lent_runs"], device=dev)
    if rank == 0:
        avg_kernel_s = sum(kernel_ms) / len(kernel_ms) / 1e3
        per_launch = decided / args.steps
        achieved = per_launch * BYTES_PER_PLACEMENT / avg_kernel_s / 1e9
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline_c5(args, lam, max(1, min(args.jobs_per_cluster, 8192)))
        out = {
            "metric": "trading-system job decisions/sec (placed locally or borrowed) at 64 clusters x 256 nodes",
            "value": decided_all / elapsed_max,
            "unit": "decisions/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (seeded device generator; scaled Poisson arrivals)",
            "config": {
                "workload": f"C5: {args.clusters} clusters x {args.nodes} nodes, FIFO + borrow + trader in lock-step, "
                            f"{args.jobs_per_cluster} jobs/cluster ({args.clusters * args.jobs_per_cluster} jobs), "
                            f"scaled arrivals at {args.load:.0%} memory load",
                "clusters_total": args.clusters,
                "nodes": args.nodes,
                "jobs_per_cluster": args.jobs_per_cluster,
                "parallelism": (f"{world} shard(s); per-tick RCCL all-gather" if dist_on or args.comm else "1 GPU, exchange in HBM")
                               + " (tick loop: " + ("graph-replayed" if ts["loop_form"] == 0 else "graph-replayed after a resident timeout" if ts["loop_form"] == 6 else "RCCL eager" if ts["loop_form"] == 1
                                                    else "RCCL captured in a hipGraph" if ts["loop_form"] == 2
                                                    else "resident in one workgroup" if ts["loop_form"] == 3
                                                    else "one launch per tick, captured with the all-gather in a hipGraph" if ts["loop_form"] == 7
                                                    else "one launch per tick, eager" if ts["loop_form"] == 8
                                                    else "one launch per tick, caller-driven" if ts["loop_form"] == 9
                                                    else "resident, one workgroup per 4 clusters"
                                                    + (", all on one XCD (L2 exchange)" if ts["loop_form"] == 5 else "")) + ")",
            },
            "roofline": {
                "bound": "hbm",
                "limiter": ("latency: the resident tick waits on the inter-workgroup X1 exchange (DESIGN.md §9)"
                            if ts["loop_form"] in (3, 4, 5) else
                            "launch/latency: a tick is dependent launches of a few us (DESIGN.md §9)"),
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": None,
                "kernel": ("tr_mw_kernel (resident tick, one workgroup per 4 clusters)" if ts["loop_form"] in (4, 5) else
                           "tr_resident_kernel (resident tick, one workgroup)" if ts["loop_form"] == 3 else
                           "tr_rk_kernel (the whole tick in one launch, one workgroup per 4 clusters), launch/latency-bound"
                           if ts["loop_form"] in (7, 8, 9) else
                           "lock-step tick (tr_step/tr_lend/tr_trader, one exchange), launch/latency-bound"),
                "kernel_ms_avg": avg_kernel_s * 1e3,
                "bytes_per_placement": BYTES_PER_PLACEMENT,
            },
            "cpu_baseline": cpu,
            "trading": {"ticks": ts["ticks"], "t_final": ts["t_final"], "us_per_tick": avg_kernel_s * 1e6 / max(ts["ticks"], 1),
                        "borrowed": ts["borrowed"], "lent_runs_all_ranks": lent_all, "trades": ts["trades"],
                        "trades_won": ts["trades_won"], "flags": ts["flags"], "loop_form": ts["loop_form"]},
        }
        if dist_on:  # the RCCL communicator's size, as torch.distributed sees it
            out["world"] = world
            out["comm_world"] = dist.get_world_size()
        print(json.dumps(out), flush=True)
    eng.close()
    if dist_on:
        dist.destroy_process_group()


# ---- C2 / C3 / C4: independent clusters, no trading --------------------------------------------
class Workload:
    """One rank's share of a FIFO/DELAY batch config."""

    def __init__(self, args, world, rank):
        from mcs_amd import Cluster, GenParams, replicate, uniform_cluster
        from mcs_amd.engine import scaled_lambda
        from mcs_amd.shard import rank_seed

        self.cfg = args.config
        self.J = args.jobs_per_cluster
        fused = args.gen == "fused"
        if args.config == "c4":
            self.spec_name = f"{args.nodes} nodes x {{32 cores, 24000 memory}}"
            spec = uniform_cluster(args.nodes)
            lam = args.lam or scaled_lambda(args.nodes, load=args.load)
            self.lam = lam
            self.arrival = (f"scaled per-second Poisson arrivals at {args.load:.0%} memory load (lambda={lam:.4f}/s)"
                            if not args.lam else f"per-second Poisson arrivals at lambda={lam:.4f}/s")
            if args.max_dur != 600:
                self.arrival += f", durations U{{0..{args.max_dur - 1}}} s"
            gp = GenParams(seed=args.seed, arrival_mode=1, lam=lam, fused=fused, max_dur_s=args.max_dur)
            if args.shard == "strong":
                if args.clusters % world:
                    raise SystemExit(f"--clusters {args.clusters} must divide over {world} ranks (strong sharding)")
                self.total = args.clusters
                self.per = args.clusters // world
                self.base = rank * self.per  # global index of this rank's first cluster
                self.shard = (rank, world)
                self.scaling = "strong"
            else:
                self.total = args.clusters * world
                self.per = args.clusters
                self.base = 0
                self.shard = None
                gp.seed = rank_seed(args.seed, rank)
                self.scaling = "weak"
        else:
            name = "cluster_small" if args.config == "c3" else "cluster_big"
            self.spec_name = f"assets/{name}.json"
            spec = Cluster.load(os.path.join(REPO, "assets", name + ".json"))
            self.lam = 10.0
            self.arrival = "reference client arrivals (Poisson(10) per minute, 60/n s spacing; client.go:107-125)"
            gp = GenParams(seed=rank_seed(args.seed, rank), fused=fused)
            self.per = args.clusters
            self.total = args.clusters * world
            self.base = 0
            self.shard = None
            self.scaling = "weak"
        self.spec = spec
        self.arrays = replicate(spec, self.per)
        self.gp = gp

    def describe(self, args, world):
        pol = "DELAY" if args.policy == "delay" else "FIFO"
        fused = "job stream synthesised inside the kernel (fused), " if args.gen == "fused" else ""
        if self.cfg == "c4":
            if self.scaling == "strong":
                head = (f"C4: {self.total} clusters total x {args.nodes} nodes, split {self.per} per GPU over "
                        f"{world} GPU(s) (strong sharding, clusters keyed by global index)")
            else:
                head = f"C4 weak: {self.per} clusters x {args.nodes} nodes per GPU ({self.total} in total)"
        elif self.cfg == "c3":
            head = f"C3: {self.per} cluster_small replicas per GPU ({self.total} in total)"
        else:
            head = f"C2: one cluster_big cluster per GPU ({world} independent replica(s))"
        return (f"{head}, {pol}, no trading, {fused}{self.J} jobs/cluster, {self.arrival}")

    def cpu_sample(self, args):
        from mcs_amd.engine import gen_streams_host

        k = min(args.cpu_sample_clusters, self.per)
        from mcs_amd import replicate

        arrays = replicate(self.spec, k)
        gp = type(self.gp)(**{**self.gp.__dict__, "fused": False})
        return arrays, gen_streams_host(gp, arrays, self.J, base=self.base), k


def cpu_baseline(args, wl, n_threads, sample_clusters=None):
    """The oracle (CPU restatement, deliberately naive, -O3) on a bounded sample of the same
    workload: the first cpu_sample_clusters clusters of rank 0, full job streams, OpenMP over
    clusters.  Test infrastructure used as the reported baseline only."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_ref as O

    O.lib()

    def run(a):
        arrays, streams, k = wl.cpu_sample(a)
        t0 = time.perf_counter()
        if a.policy == "delay":
            O.delay_run_batch(arrays, streams, n_threads=n_threads)
        else:
            O.fifo_run_batch(arrays, streams, n_threads=n_threads)
        return streams, k, time.perf_counter() - t0

    def with_k(k):
        return argparse.Namespace(**{**vars(args), "cpu_sample_clusters": k})

    if sample_clusters is not None:
        args = with_k(sample_clusters)
    elif not getattr(args, "cpu_sample_explicit", True) and args.cpu_sample_clusters > 2 * n_threads:
        # keep the sample to about CPU_BUDGET_S of work whatever the stream (a Level1-heavy DELAY
        # stream costs the naive oracle ~100x more per job): a pilot on 2 clusters per thread
        k0 = 2 * n_threads
        _, _, dt0 = run(with_k(k0))
        k = int(k0 * CPU_BUDGET_S / max(dt0, 1e-6)) // n_threads * n_threads
        args = with_k(max(k0, min(args.cpu_sample_clusters, k)))
    streams, k, dt = run(args)
    src = "oracle/mcs_oracle_delay.c" if args.policy == "delay" else "oracle/mcs_oracle.c"
    return {
        "value": streams.n_jobs / dt,
        "unit": "placements/s",
        "cores": n_threads,
        "kind": "port",
        "sample": f"{k} of {wl.per} clusters ({wl.spec_name}) x {wl.J} jobs ({streams.n_jobs} placements), "
                  f"{src} -O3, OpenMP over clusters on {n_threads} thread(s), {dt:.2f} s wall; {NAIVE}",
        "seconds": dt,
        "sample_clusters": k,
        "host": host_info(n_threads),
    }


def main_batch(args, world, rank, local_rank):
    import torch
    import torch.distributed as dist

    dist_on = world > 1
    if dist_on:
        torch.cuda.set_device(local_rank)
        dist.init_process_group(backend="nccl")
    dev = torch.device("cuda", local_rank)

    from mcs_amd import Engine
    from mcs_amd.shard import aggregate

    wl = Workload(args, world, rank)
    delay = args.policy == "delay"
    eng = Engine(local_rank, policy="DELAY" if delay else "FIFO")
    eng.load_clusters(wl.arrays)
    if wl.shard is not None:
        eng.set_shard(*wl.shard)  # generation keyed by the global cluster index rank * per + k
    fused = args.gen == "fused"
    bpp = BYTES_PER_PLACEMENT_FUSED if fused else BYTES_PER_PLACEMENT
    eng.generate_jobs(wl.gp, wl.J)
    n_jobs = eng.num_jobs

    def barrier():
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize(dev)

    for _ in range(args.warmup):
        st = eng.run()
        if st.placed + st.unplaced != n_jobs:
            raise RuntimeError(f"warmup run accounted {st.placed}+{st.unplaced} of {n_jobs} jobs")

    barrier()
    t0 = time.perf_counter()
    kernel_ms = []
    placed = 0
    escalations = 0
    handed_over = 0
    for _ in range(args.steps):
        st = eng.run()
        kernel_ms.append(st.kernel_ms)
        placed += st.placed
        escalations += st.escalations
        handed_over = st.handed_over
    barrier()
    elapsed = time.perf_counter() - t0

    elapsed_max, placed_all = aggregate(elapsed, placed, device=dev)
    kernel_name = eng.last_kernel  # the placement kernel these timings belong to
    # outside the timed region: per-cluster decision-loop diagnostics, from one more run of the
    # counting build (the hand-scheduled loop skips its pass / release counters otherwise)
    os.environ["MCS_FIFO_DIAG"] = "1"
    try:
        eng.run()
    finally:
        os.environ.pop("MCS_FIFO_DIAG", None)
    cs = eng.cluster_stats()
    diag = {
        "loop_passes_per_job": float(cs["iterations"].sum()) / max(n_jobs, 1),
        "release_scans_per_job": float(cs["release_scans"].sum()) / max(n_jobs, 1),
        "waited_frac": float(cs["waited"].sum()) / max(n_jobs, 1),
        "peak_running_max": int(cs["peak_running"].max()),
        "slot_pool": int(cs["pool"].max()),
        "clusters_per_gpu": wl.per,
    }
    if delay:
        ds = eng.delay_stats()
        diag.pop("waited_frac")
        diag["delay_iterations_per_job"] = diag.pop("loop_passes_per_job")
        diag["level1_moved_frac"] = float(ds["moved_l1"].sum()) / max(n_jobs, 1)
        # clusters the hand-scheduled loop handed to delay_kernel (re-run from t = 0, both launches in
        # kernel_ms; the engine names both kernels then): Level1 past its LDS slice, the clock range
        # after a move, or a runaway guard of the loop
        diag["clusters_handed_to_delay_kernel"] = handed_over
        diag["level1_peak_max"] = int(ds["peak_l1"].max())
        diag["avg_wait_s"] = float(ds["total_wait_ms"].sum()) / max(float(ds["jobs_count"].sum()), 1.0) / 1e3

    if rank == 0:
        avg_kernel_s = sum(kernel_ms) / len(kernel_ms) / 1e3
        placements_per_launch = placed / args.steps  # this rank
        achieved = placements_per_launch * bpp / avg_kernel_s / 1e9
        traffic = None
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f)
            if (tj.get("clusters"), tj.get("nodes"), tj.get("jobs_per_cluster"), tj.get("policy", "fifo"),
                    tj.get("gen", "stream"), tj.get("config", "c4"), tj.get("lam", 0.0), tj.get("max_dur", 600)) == \
                    (wl.per, args.nodes, wl.J, args.policy, args.gen, args.config, args.lam, args.max_dur):
                traffic = tj.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            pass
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            n_thr = args.cpu_threads or usable_cpus()
            if args.config == "c2":
                n_thr = 1  # one cluster: the oracle is one serial loop
            cpu = cpu_baseline(args, wl, n_thr)
            n_vis = host_info(0)["host_usable_cpus"] or 1
            if args.config != "c2" and not args.cpu_threads and n_vis > n_thr:
                # one thread per visible cpu as well (oversubscribed under the cgroup quota)
                sec = cpu_baseline(args, wl, n_vis, sample_clusters=cpu["sample_clusters"])
                cpu["secondary_all_visible_cpus"] = {k: sec[k] for k in ("value", "cores", "sample", "seconds")}
        value = placed_all / elapsed_max
        metric = {"c4": "job placements/sec (whole node) at 4096 clusters x 256 nodes",
                  "c3": "job placements/sec at 1024 cluster_small replicas per GPU",
                  "c2": "job placements/sec, one cluster_big cluster with 1M jobs"}[args.config]
        out = {
            "metric": metric + (", DELAY policy" if delay else ""),
            "value": value,
            "unit": "placements/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": wl.scaling,
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (seeded device generator restating pkg/client/client.go distributions)",
            "config": {
                "workload": wl.describe(args, world),
                "clusters_total": wl.total,
                "clusters_per_gpu": wl.per,
                "nodes": int(wl.arrays.node_off[1] - wl.arrays.node_off[0]),
                "jobs_per_cluster": wl.J,
                "gen": args.gen,
                "lam": args.lam,  # 0: the scaled rate of the workload string
                "max_dur": args.max_dur,
                "placements_per_step_per_gpu": placements_per_launch,
                "parallelism": (f"dp{world}: " + ("one system's clusters split over the GPUs" if wl.scaling == "strong"
                                                  else "independent replicas per GPU")
                                + ", no collective on the data path"),
            },
            "roofline": {
                "bound": "hbm",
                "limiter": limiter_text(traffic, placements_per_launch * bpp),
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "traffic_source": "profiles/ rocprofv3 --pmc pass of the same command (not measured in this run)"
                if traffic is not None else None,
                "kernel": kernel_name,
                "kernel_ms_avg": avg_kernel_s * 1e3,
                "bytes_per_placement": bpp,
                "placements_per_launch": placements_per_launch,
            },
            "cpu_baseline": cpu,
            "slot_pool_escalations": escalations,
            "diagnostics": diag,
        }
        if dist_on:  # the RCCL communicator's size, as torch.distributed sees it
            out["world"] = world
            out["comm_world"] = dist.get_world_size()
        print(json.dumps(out), flush=True)

    eng.close()
    if dist_on:
        dist.destroy_process_group()


def free_port():
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_cmd(n, argv, port):
    """The command a `bench.py --gpus N` parent (WORLD_SIZE unset) runs: torchrun with one rank per
    GPU of this node over 127.0.0.1, each rank re-entering bench.py with the same arguments (so each
    sees WORLD_SIZE == --gpus)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def world_check(gpus, env, n_devices):
    """Decide how this process runs.  Returns ("launch", n) for a parent that must spawn n ranks,
    ("run", world) for a rank (or the N=1 process), or ("refuse", message)."""
    if gpus < 1:
        return "refuse", f"--gpus {gpus}: need at least 1"
    w = env.get("WORLD_SIZE")
    if w is None:
        if gpus == 1:
            return "run", 1
        if n_devices < gpus:
            return "refuse", f"--gpus {gpus} but only {n_devices} GPU(s) are visible on this node"
        return "launch", gpus
    world = int(w)
    if world != gpus:
        return "refuse", f"WORLD_SIZE={world} (launcher) differs from --gpus {gpus}"
    local = int(env.get("LOCAL_RANK", "0"))
    if world > 1 and local >= n_devices:
        return "refuse", f"LOCAL_RANK {local} but only {n_devices} GPU(s) are visible"
    return "run", world


KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"


def _visible_list(val, n):
    """How many of n devices a *_VISIBLE_DEVICES value leaves: the leading entries that name a device
    (an index in range, or a UUID string for ROCR), stopping at the first invalid one, duplicates
    dropped; an empty value hides every device."""
    seen = []
    for tok in (x.strip() for x in val.split(",")):
        if not tok:
            break
        if tok.isdigit():
            if int(tok) >= n:
                break
        elif not tok.startswith("GPU-"):
            break
        if tok not in seen:
            seen.append(tok)
    return min(len(seen), n)


def visible_devices(env=None, root=KFD_NODES):
    """GPUs this process could use, counted from the KFD topology in sysfs (a node with SIMDs is a
    GPU), then narrowed by ROCR_VISIBLE_DEVICES and HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES (which
    index the ROCR-visible list).  No HIP, amdsmi or torch call: the `--gpus N` parent never opens
    /dev/kfd, so nothing in it can initialise a GPU before it spawns the ranks."""
    env = os.environ if env is None else env
    n = 0
    try:
        names = os.listdir(root)
    except OSError:
        names = []
    for d in names:
        try:
            with open(os.path.join(root, d, "properties")) as f:
                props = dict(line.split(None, 1) for line in f if len(line.split(None, 1)) == 2)
        except OSError:
            continue
        if int(props.get("simd_count", "0").strip() or 0) > 0:
            n += 1
    if "ROCR_VISIBLE_DEVICES" in env:
        n = _visible_list(env["ROCR_VISIBLE_DEVICES"], n)
    for var in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        if var in env:
            n = _visible_list(env[var], n)
            break
    return n


def _dump_parent_maps():
    """MCS_BENCH_PARENT_MAPS=<path>: the parent's /proc/self/maps at its decision, for the test that
    it never mapped /dev/kfd (tests/test_gpu_launcher.py, tests/test_bench_cpu.py)."""
    path = os.environ.get("MCS_BENCH_PARENT_MAPS")
    if path:
        with open("/proc/self/maps") as f, open(path, "w") as g:
            g.write(f.read())


def _dump_exit_maps():
    """MCS_BENCH_EXIT_MAPS=<path>: this process's /proc/self/maps once the run is over, so the frames
    of a fault at exit can be mapped to their libraries."""
    path = os.environ.get("MCS_BENCH_EXIT_MAPS")
    if path:
        with open("/proc/self/maps") as f, open(path, "w") as g:
            g.write(f.read())


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus == 1:
        what, val = "run", 1  # the N=1 line, unchanged
    else:
        what, val = world_check(args.gpus, os.environ, visible_devices())
        if what != "run":
            _dump_parent_maps()
    if what == "refuse":
        print(f"bench.py: refusing to run: {val}", file=sys.stderr, flush=True)
        return 2
    if what == "launch":
        import subprocess

        # a child process per rank (never exec: this parent must not replace itself); rank 0 prints
        # the JSON line on the inherited stdout; torchrun exits with the worst rank's status
        return subprocess.run(launcher_cmd(val, sys.argv[1:], free_port())).returncode
    world = val
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.config == "c5":
        rc = main_c5_delay(args, world, rank, local_rank) if args.policy == "delay" else \
            main_c5(args, world, rank, local_rank)
    else:
        rc = main_batch(args, world, rank, local_rank)
    _dump_exit_maps()
    return rc


if __name__ == "__main__":
    sys.exit(main() or 0)
