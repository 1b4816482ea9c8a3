"""Mirror of the reference's pkg/scheduler surface over the MI355X engine.

Same names, argument meaning and error behaviour as the Go code (errors are *returned*, Go style:
``None`` on success, an ``error`` instance otherwise):

  Scheduler.Run(cluster, URL)       scheduler.go:101-124 (FIFO selected, deviation D4)
  Scheduler.ScheduleJob(j) -> error scheduler.go:127-139 (+ synchronous commit, D2)
  Scheduler.Lend(j) -> error        scheduler.go:194-202
  Scheduler.JobFinished(j, node)    cluster.go:153-160 (the release half of Node.RunJob)
  Scheduler.Fifo(stream)            scheduler.go:216-296, run to completion over a job stream
  Scheduler.Delay(stream)           scheduler.go:298-369 (the reference default, :116), jobs
                                    ingested by "/delay" (server.go:53-78); WaitTime statistics
  WaitTime.GetAverage()             scheduler.go:56-63
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


@dataclass
class WaitTime:
    """scheduler.go:47-54 — wait-time statistics in milliseconds, as of the end of the last run."""

    TotalTime: int = 0
    JobsCount: int = 0

    def GetAverage(self) -> float:
        """scheduler.go:56-63."""
        if self.JobsCount != 0:
            return float(self.TotalTime) / float(self.JobsCount)
        return 0.0


class Scheduler:
    """One reference scheduler process == one cluster on an engine.  policy FIFO or DELAY (the
    reference hard-codes DELAY at scheduler.go:116; here it is selected, D4)."""

    def __init__(self, engine: Optional[Engine] = None, device: int = 0, policy: str = FIFO):
        self._eng = engine if engine is not None else Engine(device, policy=policy)
        self.SchedulingAlgorithm = self._eng.policy
        self.Cluster: Optional[Cluster] = None
        self.URL = ""
        self.WaitTime = WaitTime()

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
        if self.SchedulingAlgorithm != FIFO:
            raise ValueError("this scheduler runs DELAY")
        return self._run(arrivals, jobs)

    def Delay(self, arrivals: Sequence[int], jobs: Sequence[Job]) -> List[Placement]:
        """Scheduler.Delay over a whole stream (jobs enter Level0 through "/delay" at their arrival
        second, server.go:53-78).  Fills self.WaitTime like the reference's statistics."""
        if self.SchedulingAlgorithm != DELAY:
            raise ValueError("this scheduler runs FIFO")
        out = self._run(arrivals, jobs)
        ds = self._eng.delay_stats()[0]
        self.WaitTime = WaitTime(int(ds["total_wait_ms"]), int(ds["jobs_count"]))
        return out

    def _run(self, arrivals: Sequence[int], jobs: Sequence[Job]) -> List[Placement]:
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


__all__ = ["Scheduler", "WaitTime", "Job", "Placement", "error", "errors_New", "FIFO", "DELAY", "READY", "RUNNING",
           "WAITING", "FINISHED", "L"]
