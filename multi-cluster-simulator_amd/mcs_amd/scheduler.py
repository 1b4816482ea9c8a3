"""Mirror of the reference's pkg/scheduler surface over the MI355X engine.

Same names, argument meaning and error behaviour as the Go code (errors are *returned*, Go style:
``None`` on success, an ``error`` instance otherwise):

  Scheduler.Run(cluster, URL)       scheduler.go:101-124 (FIFO selected, deviation D4)
  Scheduler.ScheduleJob(j) -> error scheduler.go:127-139 (+ synchronous commit, D2)
  Scheduler.Lend(j) -> error        scheduler.go:194-202
  Scheduler.JobFinished(j, node)    cluster.go:153-160 (the release half of Node.RunJob)
  Scheduler.Fifo(stream)            scheduler.go:216-296, run to completion over a job stream
  Cluster.GetResourceUtilization()  cluster.go:46-63 (here Scheduler.GetResourceUtilization)

All decisions run on the GPU through libmcs.so.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib as L
from .cluster import Cluster, pack_clusters
from .engine import Engine, JobStreams

FIFO = "FIFO"
DELAY = "DELAY"
READY = "Ready"
RUNNING = "Running"
WAITING = "Waiting"
FINISHED = "Finished"


class error(Exception):
    """A Go `error` value."""

    def Error(self) -> str:
        return str(self)


def errors_New(msg: str) -> error:
    return error(msg)


@dataclass
class Job:
    """pkg/scheduler/scheduler.go:65-73.  Duration is whole seconds (D8)."""

    Id: int = 0
    MemoryNeeded: int = 0
    CoresNeeded: int = 0
    State: str = ""
    Duration: int = 0
    WaitTime: Optional[float] = None
    Ownership: str = ""


@dataclass
class Placement:
    Id: int
    Node: int  # index into Cluster.Nodes (JSON order); -1 = never placed
    Start: int
    Finish: int


class Scheduler:
    """One reference scheduler process == one cluster on an engine."""

    def __init__(self, engine: Optional[Engine] = None, device: int = 0):
        self._eng = engine if engine is not None else Engine(device)
        self.SchedulingAlgorithm = FIFO
        self.Cluster: Optional[Cluster] = None
        self.URL = ""

    @property
    def engine(self) -> Engine:
        return self._eng

    def Run(self, clt: Cluster, URL: str = "") -> None:
        """scheduler.go:101-124: keeps JSON availability as-is; policy FIFO (D4)."""
        self.Cluster = clt
        self.URL = URL
        self._eng.load_clusters(pack_clusters([clt]))

    def ScheduleJob(self, j: Job) -> Optional[error]:
        node = self._eng.schedule_one(0, j.CoresNeeded, j.MemoryNeeded)
        if node < 0:
            return errors_New("not enough resources in cluster")  # scheduler.go:138
        self._last_node = node
        return None

    def LastNode(self) -> int:
        """Node index chosen by the last successful ScheduleJob (the Go code only logs it)."""
        return getattr(self, "_last_node", -1)

    def JobFinished(self, j: Job, node: int) -> None:
        """Completion half of Node.RunJob (cluster.go:153-157); JobFinished's queue scans are
        no-ops for own jobs (scheduler.go:158-191)."""
        self._eng.release_one(0, node, j.CoresNeeded, j.MemoryNeeded)

    def Lend(self, j: Job) -> Optional[error]:
        if self._eng.lend_check(0, j.CoresNeeded, j.MemoryNeeded):
            return None
        return errors_New("can't lend")  # scheduler.go:201

    def GetResourceUtilization(self) -> Tuple[float, float]:
        return self._eng.resource_utilization(0)

    def Fifo(self, arrivals: Sequence[int], jobs: Sequence[Job]) -> List[Placement]:
        """Scheduler.Fifo over a whole stream (jobs enter the ReadyQueue at their arrival second,
        server.go:23-51).  Runs from the cluster spec loaded by Run, on the GPU."""
        n = len(jobs)
        s = JobStreams(
            np.asarray(arrivals, np.uint32),
            np.asarray([j.Duration for j in jobs], np.uint32),
            np.asarray([j.CoresNeeded for j in jobs], np.uint32),
            np.asarray([j.MemoryNeeded for j in jobs], np.uint32),
            np.asarray([0, n], np.uint64),
        )
        self._eng.submit_jobs(s)
        self._eng.run()
        node, start, fin = self._eng.placements()
        return [Placement(jobs[i].Id, int(node[i]), int(start[i]), int(fin[i])) for i in range(n)]


__all__ = ["Scheduler", "Job", "Placement", "error", "errors_New", "FIFO", "DELAY", "READY", "RUNNING",
           "WAITING", "FINISHED", "L"]
