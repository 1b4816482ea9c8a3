"""The N>1 path on CPU: 2 ranks over gloo (127.0.0.1), each simulating its own shard of
independent clusters with no data-path collective, then the bench aggregation (max elapsed, sum of
placements).  The per-rank work is done by the oracle here (CPU); the GPU engine is the same call
per rank on its own device."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from mcs_amd.shard import rank_seed, shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.join(os.path.dirname(here), "multi-cluster-simulator_amd"), here]
    import torch.distributed as dist

    import oracle_ref as O
    from mcs_amd import GenParams, replicate, uniform_cluster
    from mcs_amd.engine import gen_streams_host
    from mcs_amd.shard import aggregate, rank_seed

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    arrays = replicate(uniform_cluster(64), 4)
    gp = GenParams(seed=rank_seed(123, rank), arrival_mode=1, lam=0.4)
    streams = gen_streams_host(gp, arrays, 500)
    node, st, fi, sd = O.fifo_run_batch(arrays, streams)
    elapsed = 1.0 + rank  # synthetic per-rank time: the max must win
    emax, ptot = aggregate(elapsed, int((node >= 0).sum()))
    q.put((rank, emax, ptot, int(st.sum() % 1000003)))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_shards_and_aggregation():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, e0, p0, h0), (r1, e1, p1, h1) = res
    assert e0 == e1 == 2.0  # max over ranks
    assert p0 == p1 == 2 * 4 * 500  # every job of both shards placed, summed over ranks
    assert h0 != h1  # the two ranks simulated different streams


def _strong_worker(rank, world, port, q):
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.join(os.path.dirname(here), "multi-cluster-simulator_amd"), here]
    import torch.distributed as dist

    import oracle_ref as O
    from mcs_amd import GenParams, replicate, uniform_cluster
    from mcs_amd.engine import gen_streams_host
    from mcs_amd.shard import shard_range

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    total, J = 10, 400
    gp = GenParams(seed=99, arrival_mode=1, lam=0.5)
    lo, hi = shard_range(total, world, rank)
    arrays = replicate(uniform_cluster(64), hi - lo)
    streams = gen_streams_host(gp, arrays, J, base=lo)  # keyed by the global cluster index
    node, st, fi, _ = O.fifo_run_batch(arrays, streams)
    parts = [None] * world
    dist.all_gather_object(parts, (node, st, fi))
    if rank == 0:
        full = replicate(uniform_cluster(64), total)
        fs = gen_streams_host(gp, full, J)
        on, os_, of, _ = O.fifo_run_batch(full, fs)
        ok = all(np.array_equal(np.concatenate([p[i] for p in parts]), w) for i, w in enumerate((on, os_, of)))
        q.put(ok)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_strong_shards_concatenate_to_one_system(world):
    """C4 strong sharding (bench.py --shard strong) on CPU over gloo: every rank simulates the
    contiguous block shard_range gives it, with streams keyed by the GLOBAL cluster index; the
    concatenated shard outputs equal the whole system run in one process."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_strong_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    ok = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert ok


def test_rank_seed_and_shard_range():
    assert rank_seed(5, 0) == 5
    assert len({rank_seed(5, r) for r in range(8)}) == 8
    spans = [shard_range(4097, 8, r) for r in range(8)]
    assert spans[0][0] == 0 and spans[-1][1] == 4097
    assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1


def test_run_lockstep_skips_empty_exchanges():
    """The caller-driven lock-step driver gathers only non-empty phase outputs (a trading tick
    moves bytes from phase 0 to phase 1 only; the driver also copes with an engine whose every
    phase moves bytes)."""
    from mcs_amd.shard import run_lockstep

    class FakeEngine:
        def __init__(self, sizes, ticks):
            self.sizes, self.ticks, self.calls = sizes, ticks, []

        def trade_begin(self):
            self.calls.append("begin")

        def trade_phase(self, phase, inp):
            n_in = 0 if inp is None else len(inp)
            self.calls.append((phase, n_in))
            if phase == 3:
                self.ticks -= 1
            return np.zeros(self.sizes[phase], np.uint8), phase == 3 and self.ticks == 0

        def trade_end(self):
            self.calls.append("end")
            return "stats"

    gathered = []

    def allgather(buf):
        gathered.append(len(buf))
        return np.concatenate([buf, buf])  # two ranks

    eng = FakeEngine([96, 0, 0, 0], ticks=3)
    assert run_lockstep(eng, allgather, agree=False) == "stats"
    assert gathered == [96] * 3
    assert eng.calls[1:5] == [(0, 0), (1, 192), (2, 0), (3, 0)]
    gathered.clear()
    eng = FakeEngine([8, 4, 12, 0], ticks=2)
    run_lockstep(eng, allgather, agree=False)
    assert gathered == [8, 4, 12] * 2


def test_agree_shape_takes_the_max_over_ranks():
    """agree_shape gathers every rank's layout words through the caller's transport and applies
    their element-wise max (the RCCL loop's shape all-reduce, mcs_trade.cpp tr_agree_shape)."""
    from mcs_amd.shard import agree_shape

    class FakeEngine:
        def trade_shape_words(self):
            return np.array([64, 8, ~np.uint32(8), 0, 0, 0, 0, 0], np.uint32)

        def trade_set_shape(self, w):
            self.agreed = np.asarray(w, np.uint32)

    other = np.array([256, 8, ~np.uint32(8), 1, 0, 64, 0, 0], np.uint32)

    def allgather(buf):
        return np.concatenate([buf, other.view(np.uint8)])

    eng = FakeEngine()
    agree_shape(eng, allgather)
    assert eng.agreed.tolist() == [256, 8, int(~np.uint32(8)), 1, 0, 64, 0, 0]
