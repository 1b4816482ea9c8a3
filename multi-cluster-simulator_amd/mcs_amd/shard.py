"""Multi-GPU sharding of independent clusters.

Clusters are independent, so the data path has NO collective: each rank (one process per GPU)
simulates its own shard.  torch.distributed is used only around the timed region (barrier, max of
the elapsed time, sum of the placements).
"""
from __future__ import annotations

from typing import Tuple

M64 = 0xFFFFFFFFFFFFFFFF


def rank_seed(seed: int, rank: int) -> int:
    """Distinct job streams per rank for weak scaling: rank r keys its clusters with
    seed ^ mix(r) (rank 0 keeps the base seed, so N=1 reproduces the single-GPU stream)."""
    if rank == 0:
        return seed & M64
    z = ((rank + 1) * 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    return (seed ^ z) & M64


def shard_range(total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous block of clusters for strong scaling: [lo, hi), sizes differ by at most one."""
    base, extra = divmod(total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def aggregate(elapsed_s: float, placed: int, device=None) -> Tuple[float, float]:
    """(max elapsed over ranks, total placements over ranks).  Without an initialised process
    group returns the local values."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return float(elapsed_s), float(placed)
    t = torch.tensor([elapsed_s], dtype=torch.float64, device=device)
    p = torch.tensor([float(placed)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(p, op=dist.ReduceOp.SUM)
    return float(t.item()), float(p.item())


# ---- lock-step trading over a caller-provided transport (include/mcs_trade.h) ----------------
def agree_shape(engine, allgather):
    """The caller-driven twin of the RCCL loop's shape all-reduce (mcs_trade_shape_words /
    mcs_trade_set_shape): every rank gathers every rank's layout words and applies their
    element-wise max, so all ranks lay their exchange blocks out alike (one tick form, one snapshot
    stride, and no node snapshots when no rank has a node above 64 cores)."""
    import numpy as np

    w = engine.trade_shape_words()
    allw = np.frombuffer(np.ascontiguousarray(allgather(w.view(np.uint8))).tobytes(), np.uint32)
    engine.trade_set_shape(allw.reshape(-1, w.size).max(axis=0))


def run_lockstep(engine, allgather, agree=True):
    """Drive the lock-step trading run of one shard through mcs_trade_phase.

    `allgather(buf: np.ndarray[uint8]) -> np.ndarray[uint8]` must return the concatenation, in
    rank order, of every rank's `buf` (all ranks call it the same number of times).  With `agree`
    the ranks first agree on the exchange-block layout (agree_shape).  Every tick is phases 0..3
    with an all-gather between consecutive phases; phase 3 reports `done` identically on every
    rank.  A phase whose output is empty on every rank is not gathered (both trading systems move
    bytes only from phase 0 to phase 1).  Returns the engine's RunStats."""
    def xfer(out):
        return allgather(out) if out.size else out

    if agree:
        agree_shape(engine, allgather)
    engine.trade_begin()
    while True:
        out, _ = engine.trade_phase(0, None)
        out, _ = engine.trade_phase(1, xfer(out))
        out, _ = engine.trade_phase(2, xfer(out))
        _, done = engine.trade_phase(3, xfer(out))
        if done:
            return engine.trade_end()


def torch_allgather(group=None):
    """An `allgather` for run_lockstep over torch.distributed (e.g. gloo on the host)."""
    import numpy as np
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)

    def gather(buf):
        t = torch.from_numpy(np.ascontiguousarray(buf, dtype=np.uint8).copy())
        outs = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(outs, t, group=group)
        return torch.cat(outs).numpy()

    return gather
