"""Cluster specs: the reference's ``assets/cluster_*.json`` format.

Mirrors ``Cluster`` / ``Node`` of pkg/scheduler/cluster.go:14-24,127-138 and the way
cmd/scheduler/main.go:52-59 loads them (``json.Unmarshal`` into ``scheduler.Cluster``).  Go's
encoding/json matches object keys to exported field names case-insensitively and ignores unknown
keys; missing keys leave the zero value.  Both rules are reproduced here.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from typing import Any, Dict, List, Sequence

import numpy as np

U32_MAX = 0xFFFFFFFF


def _get(obj: Dict[str, Any], name: str, default=0):
    """encoding/json field lookup: exact match first, then case-insensitive."""
    if name in obj:
        return obj[name]
    low = name.lower()
    for k, v in obj.items():
        if k.lower() == low:
            return v
    return default


def _uint(v, what: str) -> int:
    if isinstance(v, bool) or not isinstance(v, (int, float)):
        raise ValueError(f"{what}: not a number: {v!r}")
    if isinstance(v, float):
        if v != int(v):
            raise ValueError(f"{what}: Go uint cannot hold {v}")
        v = int(v)
    if v < 0:
        raise ValueError(f"{what}: Go uint cannot hold {v}")
    if v > U32_MAX:
        raise ValueError(f"{what}: {v} exceeds the engine's uint32 node counters (D7)")
    return v


@dataclass
class Node:
    """pkg/scheduler/cluster.go:127-138 (RunningJobs/Time/mutex are runtime state)."""

    Id: int = 0
    Type: str = ""
    URL: str = ""
    Memory: int = 0
    Cores: int = 0
    MemoryAvailable: int = 0
    CoresAvailable: int = 0


@dataclass
class Cluster:
    """pkg/scheduler/cluster.go:14-24."""

    Id: int = 0
    Nodes: List[Node] = field(default_factory=list)
    URL: str = ""

    # SetTotalResources, cluster.go:26-40: uint32 sums (wrapping), computed once by Run
    def GetTotalResources(self):
        tc = sum(n.Cores for n in self.Nodes) & U32_MAX
        tm = sum(n.Memory for n in self.Nodes) & U32_MAX
        return tc, tm

    @staticmethod
    def from_obj(obj: Dict[str, Any]) -> "Cluster":
        nodes = []
        for i, nd in enumerate(_get(obj, "Nodes", []) or []):
            nodes.append(
                Node(
                    Id=_uint(_get(nd, "Id"), f"Nodes[{i}].Id"),
                    Type=str(_get(nd, "Type", "")),
                    URL=str(_get(nd, "URL", "")),
                    Memory=_uint(_get(nd, "Memory"), f"Nodes[{i}].Memory"),
                    Cores=_uint(_get(nd, "Cores"), f"Nodes[{i}].Cores"),
                    MemoryAvailable=_uint(_get(nd, "MemoryAvailable"), f"Nodes[{i}].MemoryAvailable"),
                    CoresAvailable=_uint(_get(nd, "CoresAvailable"), f"Nodes[{i}].CoresAvailable"),
                )
            )
        return Cluster(Id=_uint(_get(obj, "Id"), "Id"), Nodes=nodes, URL=str(_get(obj, "URL", "")))

    @staticmethod
    def from_json(text: str) -> "Cluster":
        return Cluster.from_obj(json.loads(text))

    @staticmethod
    def load(path: str) -> "Cluster":
        with open(path, "r", encoding="utf-8") as f:
            return Cluster.from_json(f.read())

    def to_obj(self) -> Dict[str, Any]:
        return {
            "Id": self.Id,
            "Nodes": [
                {
                    "Id": n.Id,
                    "Type": n.Type,
                    "Memory": n.Memory,
                    "Cores": n.Cores,
                    "MemoryAvailable": n.MemoryAvailable,
                    "CoresAvailable": n.CoresAvailable,
                }
                for n in self.Nodes
            ],
        }


def uniform_cluster(n_nodes: int, cores: int = 32, memory: int = 24000, cid: int = 1) -> Cluster:
    """A cluster of identical physical nodes, like assets/cluster_{small,big}.json (32 cores,
    24000 memory, fully available) — the synthetic N=256 config of SURVEY §8d."""
    return Cluster(
        Id=cid,
        Nodes=[Node(Id=i + 1, Type="physical", Memory=memory, Cores=cores, MemoryAvailable=memory,
                    CoresAvailable=cores) for i in range(n_nodes)],
    )


@dataclass
class ClusterArrays:
    """CSR node arrays of many clusters, the layout mcs_load_clusters takes."""

    cap_c: np.ndarray
    cap_m: np.ndarray
    free_c: np.ndarray
    free_m: np.ndarray
    node_off: np.ndarray

    @property
    def n_clusters(self) -> int:
        return len(self.node_off) - 1

    def nodes_of(self, c: int) -> slice:
        return slice(int(self.node_off[c]), int(self.node_off[c + 1]))


def pack_clusters(clusters: Sequence[Cluster]) -> ClusterArrays:
    counts = [len(c.Nodes) for c in clusters]
    off = np.zeros(len(clusters) + 1, dtype=np.uint32)
    off[1:] = np.cumsum(counts)
    cap_c = np.array([n.Cores for c in clusters for n in c.Nodes], dtype=np.uint32)
    cap_m = np.array([n.Memory for c in clusters for n in c.Nodes], dtype=np.uint32)
    free_c = np.array([n.CoresAvailable for c in clusters for n in c.Nodes], dtype=np.uint32)
    free_m = np.array([n.MemoryAvailable for c in clusters for n in c.Nodes], dtype=np.uint32)
    return ClusterArrays(cap_c, cap_m, free_c, free_m, off)


def replicate(cluster: Cluster, n: int) -> ClusterArrays:
    """n replicas of one spec (configs C3/C4) without building n Python objects."""
    k = len(cluster.Nodes)
    one = pack_clusters([cluster])
    return ClusterArrays(
        np.tile(one.cap_c, n), np.tile(one.cap_m, n), np.tile(one.free_c, n), np.tile(one.free_m, n),
        (np.arange(n + 1, dtype=np.uint64) * k).astype(np.uint32),
    )
