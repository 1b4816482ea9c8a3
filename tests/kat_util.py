"""Helpers shared by the oracle and GPU parity tests."""
from __future__ import annotations

import json
import os

import numpy as np

from mcs_amd import Cluster, JobStreams, pack_clusters, uniform_cluster
from mcs_amd.engine import GenParams, gen_streams_host

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
UNPLACED_T = 0xFFFFFFFF


def load_kats():
    with open(os.path.join(GOLDEN, "kats.json")) as f:
        return json.load(f)


def kat_cluster(k) -> Cluster:
    cl = Cluster.load(os.path.join(REPO, "assets", k["cluster"] + ".json"))
    for idx, (fc, fm) in k.get("override_free", {}).items():
        cl.Nodes[int(idx)].CoresAvailable = fc
        cl.Nodes[int(idx)].MemoryAvailable = fm
    return cl


def kat_streams(k):
    jobs = sorted(k["jobs"], key=lambda j: j[0])
    n = len(jobs)
    a = np.array([j[1] for j in jobs], np.uint32)
    c = np.array([j[2] for j in jobs], np.uint32)
    m = np.array([j[3] for j in jobs], np.uint32)
    d = np.array([j[4] for j in jobs], np.uint32)
    return JobStreams(a, d, c, m, np.array([0, n], np.uint64))


def kat_expect(k):
    n = len(k["jobs"])
    node = np.zeros(n, np.int32)
    st = np.zeros(n, np.uint32)
    fi = np.zeros(n, np.uint32)
    for sid, (nd, s, f) in k["expect"].items():
        i = int(sid)
        node[i], st[i], fi[i] = nd, s, f
    return node, st, fi


def seeded_workload(kind: str, n_clusters: int, jobs_per_cluster: int, seed: int = 0x4D43535F53494D31):
    """Seeded synthetic workloads of BASELINE.json's configs at reduced sizes.
    kind: 'small' (cluster_small, REF arrivals), 'big' (cluster_big, REF), 'n256' (256 nodes,
    SCALED arrivals at 90% memory load), 'n256_hot' (256 nodes, 120% load: heavy waiting),
    'n256_delay' (0.8 arrivals per second: just under DELAY's one Level0 decision per second)."""
    from mcs_amd.engine import scaled_lambda
    from mcs_amd import replicate

    if kind == "small":
        spec, gp = Cluster.load(os.path.join(REPO, "assets", "cluster_small.json")), GenParams(seed=seed)
    elif kind == "big":
        spec, gp = Cluster.load(os.path.join(REPO, "assets", "cluster_big.json")), GenParams(seed=seed)
    elif kind.startswith("n"):
        parts = kind[1:].split("_")
        nn = int(parts[0])
        load = 1.2 if (len(parts) > 1 and parts[1] == "hot") else 0.9
        if len(parts) > 1 and parts[1] == "delay":  # DELAY drains Level0 at one job per second
            load = 0.8 * 1.0 / scaled_lambda(nn, load=1.0)
        spec = uniform_cluster(nn)
        gp = GenParams(seed=seed, arrival_mode=1, lam=scaled_lambda(nn, load=load))
    else:
        raise ValueError(kind)
    arrays = replicate(spec, n_clusters)
    streams = gen_streams_host(gp, arrays, jobs_per_cluster)
    return arrays, streams, gp


def fuzz_workload(shape: str, seed: int, n_clusters: int = 160, J: int = 2000, blocking: bool = True):
    """Randomised clusters and job streams (tests/test_gpu_parity.py, test_gpu_delay.py): node counts
    across the shape's range ('w16s' <= 64 nodes, 'mid' 65-128, 'w16r' 129-256, 'w32' 129-256 with
    memory values past 2^15), random JSON availability, bursts of simultaneous arrivals and idle
    stretches, zero-duration and zero-resource jobs, requests up to a node's capacity, and (blocking)
    in half the clusters one request that fits no node at a random point of the stream; without
    blocking, node 0 is fully available, so no request can wait forever (a lock-step trading run
    would otherwise tick to its t_max)."""
    from mcs_amd import JobStreams, pack_clusters
    from mcs_amd.cluster import Node

    rng = np.random.default_rng(1000 * seed + {"w16s": 0, "w16r": 1, "w32": 2, "mid": 3}[shape])
    lo, hi = {"w16s": (1, 64), "mid": (65, 128)}.get(shape, (129, 256))
    clusters, parts = [], []
    for k in range(n_clusters):
        nn = int(rng.integers(lo, hi + 1)) if k else hi  # the largest picks the kernel shape
        cap_c = int(rng.integers(1, 64))
        cap_m = int(rng.integers(1, 32000)) if shape != "w32" else int(rng.integers(40000, 1 << 30))
        cl = Cluster(Id=k + 1, Nodes=[])
        for i in range(nn):
            fc = cap_c if rng.random() < 0.7 else int(rng.integers(0, cap_c + 1))
            fm = cap_m if rng.random() < 0.7 else int(rng.integers(0, cap_m + 1))
            cl.Nodes.append(Node(Id=i + 1, Cores=cap_c, Memory=cap_m, CoresAvailable=fc, MemoryAvailable=fm))
        if not blocking:  # node 0 fully available: every request fits once it drains (no stuck head)
            cl.Nodes[0].CoresAvailable, cl.Nodes[0].MemoryAvailable = cap_c, cap_m
        clusters.append(cl)
        gaps = rng.poisson(rng.uniform(0.05, 2.0), J)
        gaps[rng.random(J) < 0.05] += int(rng.integers(10, 500))  # idle stretches
        arr = np.cumsum(gaps).astype(np.uint32)
        dur = rng.integers(0, int(rng.integers(2, 300)), J).astype(np.uint32)
        cores = rng.integers(0, cap_c + 1, J).astype(np.uint32)
        mem = rng.integers(0, cap_m + 1, J).astype(np.uint32)
        z = rng.random(J) < 0.02
        cores[z] = 0
        mem[z] = 0
        if blocking and rng.random() < 0.5:  # one request that fits no node, somewhere in the stream
            i = int(rng.integers(J // 4, J))
            if rng.random() < 0.5:
                cores[i] = cap_c + 1
            else:
                mem[i] = cap_m + 1
        parts.append((arr, dur, cores, mem))
    off = np.arange(len(parts) + 1, dtype=np.uint64) * J
    return pack_clusters(clusters), JobStreams(*(np.concatenate([p[f] for p in parts]) for f in range(4)), off)
