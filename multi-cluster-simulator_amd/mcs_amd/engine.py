"""Python front end of the C ABI (include/mcs.h) — device-resident batched FIFO engine.

Every compute call goes to libmcs.so (gfx950 kernels).  There is no CPU fallback: without the
library or a HIP device the calls raise MCSError.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass
from typing import Optional, Sequence, Tuple

import numpy as np

from . import _lib as L
from .cluster import Cluster, ClusterArrays, pack_clusters


def _check(eng_handle, rc: int):
    if rc != L.MCS_OK:
        msg = ""
        if eng_handle:
            m = L.lib().mcs_last_error(eng_handle)
            msg = m.decode() if m else ""
        raise L.MCSError(rc, msg)


@dataclass
class GenParams:
    """mcs_gen_params (include/mcs.h); defaults restate pkg/client/client.go:85-147."""

    seed: int = 0x4D43535F53494D31
    arrival_mode: int = L.MCS_ARRIVAL_REF
    max_dur_s: int = 600
    lam: float = 10.0
    max_cores: int = 0
    max_mem: int = 0
    fused: bool = False  # synthesise the stream inside the placement kernels (no records in HBM)
    weibull_k: float = 0.0  # MCS_ARRIVAL_WEIBULL shape (0 = 3, client.go:134); lam is then the scale

    def to_c(self) -> L.mcs_gen_params:
        p = L.mcs_gen_params()
        L.lib().mcs_gen_params_default(C.byref(p))
        p.seed = self.seed & 0xFFFFFFFFFFFFFFFF
        p.arrival_mode = self.arrival_mode
        p.max_dur_s = self.max_dur_s
        p.lambda_ = float(self.lam)
        p.max_cores = self.max_cores
        p.max_mem = self.max_mem
        p.fused = int(bool(self.fused))
        p.weibull_k = float(self.weibull_k)
        return p


def scaled_lambda(n_nodes: int, node_mem: int = 24000, max_mem: int = 24000, max_dur_s: int = 600,
                  load: float = 0.9) -> float:
    """Per-second Poisson rate giving `load` offered memory load (SURVEY §8d 'scaled' mode)."""
    return float(L.lib().mcs_gen_scaled_lambda(n_nodes, node_mem, max_mem, max_dur_s, load))


def gen_cluster_host(params: GenParams, cluster: int, max_cores: int, max_mem: int, n_jobs: int):
    """Host generator (bit-identical to the device generator).  Returns (arrival, dur, cores, mem)."""
    a = np.empty(n_jobs, np.uint32)
    d = np.empty(n_jobs, np.uint32)
    c = np.empty(n_jobs, np.uint32)
    m = np.empty(n_jobs, np.uint32)
    p = params.to_c()
    rc = L.lib().mcs_gen_cluster_host(C.byref(p), cluster, max_cores, max_mem, n_jobs,
                                      L.ptr(a, C.c_uint32), L.ptr(d, C.c_uint32), L.ptr(c, C.c_uint32),
                                      L.ptr(m, C.c_uint32))
    _check(None, rc)
    return a, d, c, m


@dataclass
class JobStreams:
    """CSR job streams: jobs of cluster k are [job_off[k], job_off[k+1])."""

    arrival: np.ndarray
    dur: np.ndarray
    cores: np.ndarray
    mem: np.ndarray
    job_off: np.ndarray

    @property
    def n_jobs(self) -> int:
        return int(self.job_off[-1])

    def of(self, k: int) -> slice:
        return slice(int(self.job_off[k]), int(self.job_off[k + 1]))


def gen_streams_host(params: GenParams, arrays: ClusterArrays, jobs_per_cluster: int, base: int = 0) -> JobStreams:
    """Host streams of clusters base .. base + n - 1 of a (possibly sharded) system: cluster k of
    `arrays` is keyed by its global index base + k, as the device generator keys it after
    mcs_set_shard (gen.base = rank * C)."""
    n = arrays.n_clusters
    tot = n * jobs_per_cluster
    out = [np.empty(tot, np.uint32) for _ in range(4)]
    for k in range(n):
        sl = arrays.nodes_of(k)
        mc = params.max_cores or int(arrays.cap_c[sl].max(initial=0))
        mm = params.max_mem or int(arrays.cap_m[sl].max(initial=0))
        a, d, c, m = gen_cluster_host(params, base + k, mc, mm, jobs_per_cluster)
        s = slice(k * jobs_per_cluster, (k + 1) * jobs_per_cluster)
        out[0][s], out[1][s], out[2][s], out[3][s] = a, d, c, m
    off = np.arange(n + 1, dtype=np.uint64) * jobs_per_cluster
    return JobStreams(out[0], out[1], out[2], out[3], off)


@dataclass
class RunStats:
    jobs: int
    placed: int
    waited: int
    unplaced: int
    clusters: int
    deadlocked: int
    escalations: int
    slot_pool: int
    kernel_ms: float
    wall_ms: float
    pending: int = 0      # online: jobs not decided yet
    t_horizon: int = L.MCS_TIME_NONE
    online: bool = False
    handed_over: int = 0  # DELAY: clusters the hand-scheduled loop handed to delay_kernel

    @classmethod
    def from_c(cls, st: "L.mcs_stats") -> "RunStats":
        return cls(st.jobs, st.placed, st.waited, st.unplaced, st.clusters, st.deadlocked, st.escalations,
                   st.slot_pool, st.kernel_ms, st.wall_ms, st.pending, st.t_horizon, bool(st.online),
                   st.handed_over)


CLUSTER_STATS_DTYPE = np.dtype([("t_end", "<u4"), ("placed", "<u4"), ("waited", "<u4"),
                                ("peak_running", "<u4"), ("flags", "<u4"), ("pool", "<u4"),
                                ("iterations", "<u4"), ("release_scans", "<u4")])


DELAY_STATS_DTYPE = np.dtype([("total_wait_ms", "<i8"), ("jobs_count", "<i8"), ("moved_l1", "<u4"),
                              ("placed_l1", "<u4"), ("peak_l1", "<u4"), ("l1_left", "<u4")])

CLUSTER_STATE_DTYPE = np.dtype([("cores_utilization", "<f4"), ("memory_utilization", "<f4"), ("total_cpu", "<u4"),
                                ("total_memory", "<u4"), ("running", "<u4"), ("t_s", "<u4")])

CONTRACT_DTYPE = np.dtype([("t", "<u4"), ("requester", "<u4"), ("winner", "<i4"), ("approvals", "<u4"),
                           ("policy", "<u4"), ("cores", "<u4"), ("mem", "<u4"), ("time_s", "<u4"), ("failed", "<u4"),
                           ("pad", "<u4")])
FOREIGN_DTYPE = np.dtype([("requester", "<u4"), ("responder", "<u4"), ("node", "<u4"), ("start", "<u4"),
                          ("finish", "<u4"), ("pad", "<u4"), ("c", "<u8"), ("m", "<u8")])

LENT_DTYPE = np.dtype([("lender", "<u4"), ("borrower", "<u4"), ("job", "<u8"), ("node", "<u4"),
                       ("start", "<u4"), ("finish", "<u4"), ("pad", "<u4")])
TRADE_DTYPE = np.dtype([("t", "<u4"), ("requester", "<u4"), ("winner", "<i4"), ("approvals", "<u4")])


class Engine:
    """One engine = one GPU (mcs_engine_create(cfg, device))."""

    def __init__(self, device: int = 0, slot_pool: int = 0, borrow: bool = False, trader: bool = False,
                 policy: str = "FIFO", **cadences):
        """policy "FIFO" (Scheduler.Fifo) or "DELAY" (Scheduler.Delay, the reference default);
        borrow/trader select the lock-step trading path (include/mcs_trade.h); cadences override
        mcs_config fields (trader_period_s, trade_ok_sleep_s, trade_fail_sleep_s, lock_s,
        sample_period_s, lent_queue_cap, t_max_s, max_wait_s)."""
        cfg = L.mcs_config()
        L.lib().mcs_config_default(C.byref(cfg))
        if policy not in ("FIFO", "DELAY"):
            raise ValueError(f"unknown policy {policy!r}")
        cfg.policy = L.MCS_POLICY_DELAY if policy == "DELAY" else L.MCS_POLICY_FIFO
        self.policy = policy
        cfg.slot_pool = slot_pool
        cfg.borrow = int(borrow)
        cfg.trader = int(trader)
        for k, v in cadences.items():
            if k not in dict(L.mcs_config._fields_) or k in ("reserved", "policy"):
                raise TypeError(f"unknown config field {k}")
            setattr(cfg, k, int(v))
        self.cfg = cfg
        h = C.c_void_p()
        rc = L.lib().mcs_engine_create(C.byref(cfg), device, C.byref(h))
        if rc != L.MCS_OK:
            raise L.MCSError(rc, f"mcs_engine_create(device={device}) failed (is a HIP device visible?)")
        self._h = h
        self.device = device
        self.arrays: Optional[ClusterArrays] = None
        self.job_off: Optional[np.ndarray] = None

    # -- lifecycle --------------------------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None):
            L.lib().mcs_engine_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _c(self, rc):
        _check(self._h, rc)

    # -- inputs -----------------------------------------------------------------------------
    def load_clusters(self, clusters) -> ClusterArrays:
        arr = clusters if isinstance(clusters, ClusterArrays) else pack_clusters(list(clusters))
        cc = [np.ascontiguousarray(x, dtype=np.uint32) for x in (arr.cap_c, arr.cap_m, arr.free_c, arr.free_m)]
        off = np.ascontiguousarray(arr.node_off, dtype=np.uint32)
        self._c(L.lib().mcs_load_clusters(self._h, *[L.ptr(x, C.c_uint32) for x in cc],
                                          L.ptr(off, C.c_uint32), arr.n_clusters))
        self.arrays = arr
        self.job_off = None
        return arr

    def submit_jobs(self, s: JobStreams):
        a = [np.ascontiguousarray(x, dtype=np.uint32) for x in (s.arrival, s.dur, s.cores, s.mem)]
        off = np.ascontiguousarray(s.job_off, dtype=np.uint64)
        self._c(L.lib().mcs_submit_jobs(self._h, *[L.ptr(x, C.c_uint32) for x in a], L.ptr(off, C.c_uint64)))
        self.job_off = off

    def generate_jobs(self, params: GenParams, jobs_per_cluster: int):
        p = params.to_c()
        self._c(L.lib().mcs_generate_jobs(self._h, C.byref(p), jobs_per_cluster))
        n = self.num_clusters
        self.job_off = np.arange(n + 1, dtype=np.uint64) * jobs_per_cluster

    def read_jobs(self) -> JobStreams:
        n = self.num_jobs
        out = [np.empty(n, np.uint32) for _ in range(4)]
        self._c(L.lib().mcs_read_jobs(self._h, *[L.ptr(x, C.c_uint32) for x in out]))
        return JobStreams(out[0], out[1], out[2], out[3], self.job_off.copy())

    @property
    def num_clusters(self) -> int:
        return int(L.lib().mcs_num_clusters(self._h))

    @property
    def num_jobs(self) -> int:
        return int(L.lib().mcs_num_jobs(self._h))

    # -- sharding / lock-step trading (include/mcs_trade.h) -----------------------------------
    def set_shard(self, rank: int, world: int):
        """This engine holds clusters [rank*C, rank*C+C) of world*C (call before generate_jobs:
        generation is keyed by the global cluster index)."""
        self._c(L.lib().mcs_set_shard(self._h, rank, world))
        self.rank, self.world = rank, world

    @staticmethod
    def comm_unique_id() -> bytes:
        cid = L.mcs_comm_id()
        rc = L.lib().mcs_comm_unique_id(C.byref(cid))
        if rc != L.MCS_OK:
            raise L.MCSError(rc, "mcs_comm_unique_id")
        return bytes(C.string_at(C.addressof(cid), 128))

    def comm_init(self, uid: bytes):
        cid = L.mcs_comm_id()
        C.memmove(C.addressof(cid), uid, 128)
        self._c(L.lib().mcs_comm_init(self._h, C.byref(cid)))

    def trade_begin(self):
        self._c(L.lib().mcs_trade_begin(self._h))

    def trade_shape_words(self) -> np.ndarray:
        """This rank's block-layout words (mcs_trade_shape_words); agree on their max over ranks."""
        w = np.zeros(L.MCS_TRADE_SHAPE_WORDS, np.uint32)
        self._c(L.lib().mcs_trade_shape_words(self._h, L.ptr(w, C.c_uint32)))
        return w

    def trade_set_shape(self, agreed: np.ndarray):
        """Apply the element-wise max over ranks of trade_shape_words (mcs_trade_set_shape)."""
        w = np.ascontiguousarray(agreed, dtype=np.uint32)
        if w.size != L.MCS_TRADE_SHAPE_WORDS:
            raise ValueError(f"{w.size} shape words, expected {L.MCS_TRADE_SHAPE_WORDS}")
        self._c(L.lib().mcs_trade_set_shape(self._h, L.ptr(w, C.c_uint32)))

    def trade_xfer_bytes(self, phase: int):
        i, o = C.c_uint64(), C.c_uint64()
        self._c(L.lib().mcs_trade_xfer_bytes(self._h, phase, C.byref(i), C.byref(o)))
        return i.value, o.value

    def trade_phase(self, phase: int, inp: Optional[np.ndarray]):
        """One phase of a tick (caller-driven transport).  Returns (out bytes as uint8 array, done)."""
        ib, ob = self.trade_xfer_bytes(phase)
        inp = np.ascontiguousarray(inp if inp is not None else np.zeros(0, np.uint8)).view(np.uint8)
        if inp.nbytes != ib:
            raise ValueError(f"phase {phase}: input has {inp.nbytes} bytes, expected {ib}")
        out = np.empty(ob, np.uint8)
        done = C.c_uint32()
        self._c(L.lib().mcs_trade_phase(self._h, phase, inp.ctypes.data if ib else None, ib,
                                        out.ctypes.data if ob else None, ob, C.byref(done)))
        return out, bool(done.value)

    def trade_end(self) -> RunStats:
        st = L.mcs_stats()
        self._c(L.lib().mcs_trade_end(self._h, C.byref(st)))
        return RunStats.from_c(st)

    def trade_stats(self) -> dict:
        ts = L.mcs_trade_stats()
        self._c(L.lib().mcs_read_trade_stats(self._h, C.byref(ts)))
        return {k: getattr(ts, k) for k, _ in L.mcs_trade_stats._fields_ if k != "pad"}

    def lent(self) -> np.ndarray:
        """Lent runs of this engine's clusters (LENT_DTYPE), sorted by (start, lender, borrower, job)."""
        n = C.c_uint64()
        self._c(L.lib().mcs_read_lent(self._h, None, 0, C.byref(n)))
        out = np.zeros(n.value, LENT_DTYPE)
        if n.value:
            self._c(L.lib().mcs_read_lent(self._h, out.ctypes.data_as(C.POINTER(L.mcs_lent_rec)), n.value,
                                          C.byref(n)))
        return out

    def trades(self) -> np.ndarray:
        n = C.c_uint64()
        self._c(L.lib().mcs_read_trades(self._h, None, 0, C.byref(n)))
        out = np.zeros(n.value, TRADE_DTYPE)
        if n.value:
            self._c(L.lib().mcs_read_trades(self._h, out.ctypes.data_as(C.POINTER(L.mcs_trade_rec)), n.value,
                                            C.byref(n)))
        return out

    def contracts(self) -> np.ndarray:
        """Trader rounds with their contracts (DELAY trading, CONTRACT_DTYPE)."""
        n = C.c_uint64()
        self._c(L.lib().mcs_read_contracts(self._h, None, 0, C.byref(n)))
        out = np.zeros(n.value, CONTRACT_DTYPE)
        if n.value:
            self._c(L.lib().mcs_read_contracts(self._h, out.ctypes.data_as(C.POINTER(L.mcs_contract_rec)), n.value,
                                               C.byref(n)))
        return out

    def foreign(self) -> np.ndarray:
        """Foreign jobs launched by AllocateVirtualNodeResources (DELAY trading, FOREIGN_DTYPE)."""
        n = C.c_uint64()
        self._c(L.lib().mcs_read_foreign(self._h, None, 0, C.byref(n)))
        out = np.zeros(n.value, FOREIGN_DTYPE)
        if n.value:
            self._c(L.lib().mcs_read_foreign(self._h, out.ctypes.data_as(C.POINTER(L.mcs_foreign_rec)), n.value,
                                             C.byref(n)))
        return out

    def virtual_node_caps(self, cluster: int):
        """[(cores, memory)] of the virtual nodes `cluster` received (DELAY trading)."""
        n = C.c_uint32()
        self._c(L.lib().mcs_read_virtual_node_caps(self._h, cluster, None, None, 0, C.byref(n)))
        c = np.zeros(max(n.value, 1), np.uint32)
        m = np.zeros(max(n.value, 1), np.uint32)
        self._c(L.lib().mcs_read_virtual_node_caps(self._h, cluster, L.ptr(c, C.c_uint32), L.ptr(m, C.c_uint32),
                                                   n.value, C.byref(n)))
        return [(int(c[i]), int(m[i])) for i in range(n.value)]

    def virtual_nodes(self, n_total: Optional[int] = None) -> np.ndarray:
        n_total = n_total if n_total is not None else self.num_clusters * getattr(self, "world", 1)
        out = np.zeros(n_total, np.uint32)
        self._c(L.lib().mcs_read_virtual_nodes(self._h, L.ptr(out, C.c_uint32), n_total))
        return out

    # -- the hot path ---------------------------------------------------------------------------
    def run(self, t_end: Optional[int] = None) -> RunStats:
        """mcs_run: a batch run (t_end None, no online session), or online mode:
        every decision at simulated seconds < t_end, or with t_end None a drain of every job
        appended so far."""
        st = L.mcs_stats()
        self._c(L.lib().mcs_run(self._h, L.MCS_TIME_NONE if t_end is None else int(t_end), C.byref(st)))
        return RunStats.from_c(st)

    @property
    def last_kernel(self) -> str:
        """mcs_last_kernel: the placement kernel the last run launched first (its rocprofv3 name)."""
        return L.lib().mcs_last_kernel(self._h).decode()

    def run_status(self, t_end: Optional[int] = None) -> Tuple[int, RunStats]:
        """mcs_run returning (status, stats) without raising (e.g. MCS_E_RANGE, results readable)."""
        st = L.mcs_stats()
        rc = L.lib().mcs_run(self._h, L.MCS_TIME_NONE if t_end is None else int(t_end), C.byref(st))
        return rc, RunStats.from_c(st)

    def append_jobs(self, s: JobStreams):
        """mcs_append_jobs: s.job_off is the CSR of the APPENDED jobs per cluster (online mode)."""
        a = [np.ascontiguousarray(x, dtype=np.uint32) for x in (s.arrival, s.dur, s.cores, s.mem)]
        off = np.ascontiguousarray(s.job_off, dtype=np.uint64)
        self._c(L.lib().mcs_append_jobs(self._h, *[L.ptr(x, C.c_uint32) for x in a], L.ptr(off, C.c_uint64)))
        self.job_off = self.job_offsets()

    def rewind(self):
        """mcs_rewind: restart the online session at t = 0 with every job so far."""
        self._c(L.lib().mcs_rewind(self._h))

    def job_offsets(self) -> np.ndarray:
        """mcs_read_job_offsets: dense CSR of the current streams."""
        off = np.zeros(self.num_clusters + 1, np.uint64)
        self._c(L.lib().mcs_read_job_offsets(self._h, L.ptr(off, C.c_uint64)))
        return off

    def placements(self) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        n = self.num_jobs
        node = np.empty(n, np.int32)
        start = np.empty(n, np.uint32)
        fin = np.empty(n, np.uint32)
        self._c(L.lib().mcs_read_placements(self._h, L.ptr(node, C.c_int32), L.ptr(start, C.c_uint32),
                                            L.ptr(fin, C.c_uint32)))
        return node, start, fin

    def cluster_stats(self) -> np.ndarray:
        n = self.num_clusters
        out = np.zeros(n, CLUSTER_STATS_DTYPE)
        self._c(L.lib().mcs_read_cluster_stats(self._h, out.ctypes.data_as(C.POINTER(L.mcs_cluster_stats)), n))
        return out

    def delay_stats(self) -> np.ndarray:
        """Per-cluster DELAY statistics of the last DELAY run (DELAY_STATS_DTYPE)."""
        n = self.num_clusters
        out = np.zeros(n, DELAY_STATS_DTYPE)
        self._c(L.lib().mcs_read_delay_stats(self._h, out.ctypes.data_as(C.POINTER(L.mcs_delay_cluster_stats)),
                                             n))
        return out

    def cluster_states(self, t_s: int, with_time: bool = False):
        """ClusterState of every cluster at simulated second t_s, rebuilt on the GPU from the last
        FIFO/DELAY run (mcs_cluster_states; CLUSTER_STATE_DTYPE).  with_time: also the kernel ms."""
        n = self.num_clusters
        out = np.zeros(n, CLUSTER_STATE_DTYPE)
        ms = C.c_double(0.0)
        self._c(L.lib().mcs_cluster_states(self._h, int(t_s), out.ctypes.data_as(C.POINTER(L.mcs_cluster_state)),
                                           n, C.byref(ms)))
        return (out, ms.value) if with_time else out

    def approve_trade(self, total_cores, total_memory, core_util, mem_util, cores, memory, time_s) -> np.ndarray:
        """mcs_approve_trade: Trader.ApproveTrade (trader.go:141-167) on the GPU for arrays of
        (responder totals + sample, contract) queries; returns 0/1 per query."""
        arrs = np.broadcast_arrays(*(np.asarray(x) for x in (total_cores, total_memory, core_util, mem_util, cores,
                                                              memory, time_s)))
        n = arrs[0].size
        q = np.zeros(n, dtype=[("total_cores", "<u4"), ("total_memory", "<u4"), ("core_util", "<f4"),
                               ("mem_util", "<f4"), ("cores", "<u4"), ("memory", "<u4"), ("time_s", "<u4"),
                               ("pad", "<u4")])
        for f, a in zip(("total_cores", "total_memory", "core_util", "mem_util", "cores", "memory", "time_s"), arrs):
            q[f] = a.ravel()
        out = np.zeros(max(n, 1), np.int32)
        self._c(L.lib().mcs_approve_trade(self._h, q.ctypes.data_as(C.POINTER(L.mcs_approve_query)), n,
                                          L.ptr(out, C.c_int32)))
        return out[:n]

    # -- single-job mirrors (live state) --------------------------------------------------------
    def schedule_one(self, cluster: int, cores: int, mem: int) -> int:
        node = C.c_int32(-1)
        rc = L.lib().mcs_schedule_one(self._h, cluster, cores, mem, C.byref(node))
        if rc == L.MCS_NO_FIT:
            return L.MCS_NODE_UNPLACED
        self._c(rc)
        return node.value

    def release_one(self, cluster: int, node: int, cores: int, mem: int):
        self._c(L.lib().mcs_release_one(self._h, cluster, node, cores, mem))

    def lend_check(self, cluster: int, cores: int, mem: int) -> bool:
        ok = C.c_int32(0)
        self._c(L.lib().mcs_lend_check(self._h, cluster, cores, mem, C.byref(ok)))
        return bool(ok.value)

    def live_state(self, cluster: int):
        sl = self.arrays.nodes_of(cluster)
        n = sl.stop - sl.start
        fc = np.empty(max(n, 1), np.uint32)
        fm = np.empty(max(n, 1), np.uint32)
        self._c(L.lib().mcs_read_live_state(self._h, cluster, L.ptr(fc, C.c_uint32), L.ptr(fm, C.c_uint32), n))
        return fc[:n], fm[:n]

    def resource_utilization(self, cluster: int) -> Tuple[float, float]:
        cu = C.c_float()
        mu = C.c_float()
        self._c(L.lib().mcs_resource_utilization(self._h, cluster, C.byref(cu), C.byref(mu)))
        return cu.value, mu.value


def device_count() -> int:
    """HIP devices visible to this process (via torch, which does not initialise the GPU)."""
    try:
        import torch

        return int(torch.cuda.device_count())
    except Exception:
        return 0


def algorithmic_bytes_per_placement() -> int:
    """16 B job record read + 12 B result write."""
    return 28


def roofline_placements_per_s(peak_bytes_per_s: float = 8.0e12) -> float:
    return peak_bytes_per_s / algorithmic_bytes_per_placement()


__all__ = ["Engine", "GenParams", "JobStreams", "RunStats", "gen_cluster_host", "gen_streams_host",
           "scaled_lambda", "device_count", "CLUSTER_STATS_DTYPE", "DELAY_STATS_DTYPE", "math"]
