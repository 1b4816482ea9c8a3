"""Measure the ClusterState reduction (csrc/mcs_state.hip) on the C4 workload: one FIFO run of
4096 clusters x 256 nodes x 16384 jobs, then K launches of mcs_cluster_states at a mid-run second.
Algorithmic bytes per launch = 12 B per job scanned (node, start, finish) + 8 B per running job
(its cores and memory); prints one JSON line with the HBM roofline of the launch."""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "multi-cluster-simulator_amd"))
from mcs_amd import Engine, GenParams, replicate, uniform_cluster  # noqa: E402
from mcs_amd.engine import scaled_lambda  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--clusters", type=int, default=4096)
ap.add_argument("--jobs-per-cluster", type=int, default=16384)
ap.add_argument("--steps", type=int, default=20)
a = ap.parse_args()
with Engine(0) as eng:
    eng.load_clusters(replicate(uniform_cluster(256), a.clusters))
    eng.generate_jobs(GenParams(arrival_mode=1, lam=scaled_lambda(256, load=0.9)), a.jobs_per_cluster)
    eng.run()
    node, start, fin = eng.placements()
    t = int(np.median(start[node >= 0]))
    eng.cluster_states(t)  # warm-up
    ms = []
    for _ in range(a.steps):
        st, k = eng.cluster_states(t, with_time=True)
        ms.append(k)
    jobs = eng.num_jobs
    running = int(st["running"].sum())
    alg = 12.0 * jobs + 8.0 * running
    avg = sum(ms) / len(ms)
    gbs = alg / (avg / 1e3) / 1e9
    print(json.dumps({"kernel": "mcs::state_kernel", "clusters": a.clusters, "jobs": jobs, "t_s": t,
                      "running_jobs": running, "kernel_ms_avg": avg, "kernel_ms_min": min(ms),
                      "algorithmic_bytes_per_launch": alg, "records_per_s": a.clusters / (avg / 1e3),
                      "roofline": {"bound": "hbm", "achieved": gbs, "peak": 8000.0, "unit": "GB/s",
                                   "frac": gbs / 8000.0}}), flush=True)
