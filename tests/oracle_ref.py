"""ctypes binding of the CPU ORACLE (oracle/libmcs_oracle.so) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this, and only as
the checker / timed CPU baseline (see oracle/mcs_oracle.h).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
# MCS_ORACLE_SO: another build of the same sources (tests/test_oracle_sanitize.py runs the oracle test
# modules against the AddressSanitizer + UBSan build, oracle/asan/libmcs_oracle_asan.so)
ORACLE_SO = os.environ.get("MCS_ORACLE_SO") or os.path.join(ORACLE_DIR, "libmcs_oracle.so")


class or_stats(C.Structure):
    _fields_ = [("t_end", C.c_uint32), ("placed", C.c_uint32), ("waited", C.c_uint32),
                ("peak_running", C.c_uint32), ("flags", C.c_uint32), ("pad", C.c_uint32),
                ("ticks", C.c_uint64)]


class or_trade_cfg(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in ("borrow", "trader", "period_s", "trade_ok_sleep_s",
                                          "trade_fail_sleep_s", "lock_s", "sample_period_s", "t_max")]


class or_lent_rec(C.Structure):
    _fields_ = [("lender", C.c_uint32), ("borrower", C.c_uint32), ("job", C.c_uint64), ("node", C.c_uint32),
                ("start", C.c_uint32), ("finish", C.c_uint32), ("pad", C.c_uint32)]


class or_trade_rec(C.Structure):
    _fields_ = [("t", C.c_uint32), ("requester", C.c_uint32), ("winner", C.c_int32), ("approvals", C.c_uint32)]


class or_trade_cluster_stats(C.Structure):
    _fields_ = [("virtual_nodes", C.c_uint32), ("decided", C.c_uint32), ("lent_pending", C.c_uint32),
                ("lent_peak", C.c_uint32)]


class or_delay_stats(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in ("t_end", "placed", "moved_l1", "placed_l1", "peak_l1", "peak_running",
                                          "flags", "l1_left")] + \
               [("total_wait_ms", C.c_int64), ("jobs_count", C.c_int64), ("ticks", C.c_uint64)]


DELAY_STATS_DTYPE = np.dtype([("t_end", "<u4"), ("placed", "<u4"), ("moved_l1", "<u4"), ("placed_l1", "<u4"),
                              ("peak_l1", "<u4"), ("peak_running", "<u4"), ("flags", "<u4"), ("l1_left", "<u4"),
                              ("total_wait_ms", "<i8"), ("jobs_count", "<i8"), ("ticks", "<u8")])

class or_dtrade_cfg(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in ("period_s", "trade_ok_sleep_s", "trade_fail_sleep_s", "lock_s",
                                          "sample_period_s", "max_wait_s", "max_vnodes", "t_max")]


DTRADE_DTYPE = np.dtype([("t", "<u4"), ("requester", "<u4"), ("winner", "<i4"), ("approvals", "<u4"),
                         ("policy", "<u4"), ("cores", "<u4"), ("mem", "<u4"), ("time_s", "<u4"), ("failed", "<u4"),
                         ("pad", "<u4")])
FOREIGN_DTYPE = np.dtype([("requester", "<u4"), ("responder", "<u4"), ("node", "<u4"), ("start", "<u4"),
                          ("finish", "<u4"), ("pad", "<u4"), ("c", "<u8"), ("m", "<u8")])
DTRADE_STATS_DTYPE = np.dtype([("virtual_nodes", "<u4"), ("decided", "<u4"), ("moved_l1", "<u4"),
                               ("placed_l1", "<u4"), ("total_wait_ms", "<i8"), ("jobs_count", "<i8")])

LENT_DTYPE = np.dtype([("lender", "<u4"), ("borrower", "<u4"), ("job", "<u8"), ("node", "<u4"),
                       ("start", "<u4"), ("finish", "<u4"), ("pad", "<u4")])
TRADE_DTYPE = np.dtype([("t", "<u4"), ("requester", "<u4"), ("winner", "<i4"), ("approvals", "<u4")])

_lib = None
u32p = C.POINTER(C.c_uint32)
i32p = C.POINTER(C.c_int32)
u64p = C.POINTER(C.c_uint64)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO) and not os.environ.get("MCS_ORACLE_SO"):
            subprocess.run(["make", "-C", ORACLE_DIR], check=True, capture_output=True)
        L = C.CDLL(ORACLE_SO)
        L.or_fifo_run.argtypes = [C.c_uint32, u32p, u32p, u32p, u32p, C.c_uint64, u32p, u32p, u32p, u32p,
                                  C.c_int, i32p, u32p, u32p, C.POINTER(or_stats)]
        L.or_fifo_run.restype = C.c_int
        L.or_fifo_run_batch.argtypes = [C.c_uint32, u32p, u32p, u32p, u32p, u32p, u64p, u32p, u32p, u32p,
                                        u32p, C.c_int, i32p, u32p, u32p, C.POINTER(or_stats)]
        L.or_fifo_run_batch.restype = C.c_int
        L.or_schedule_job.argtypes = [C.c_uint32, u64p, u64p, C.c_uint64, C.c_uint64]
        L.or_schedule_job.restype = C.c_int
        L.or_lend.argtypes = [C.c_uint32, u64p, u64p, C.c_uint64, C.c_uint64]
        L.or_lend.restype = C.c_int
        L.or_resource_utilization.argtypes = [C.c_uint32, u64p, u64p, u64p, u64p, C.c_uint32, C.c_uint32,
                                              C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.or_resource_utilization.restype = None
        L.or_approve_trade.argtypes = [C.c_uint32, C.c_uint32, C.c_float, C.c_float, C.c_uint32, C.c_uint32,
                                       C.c_int64, C.c_float]
        L.or_approve_trade.restype = C.c_int
        L.or_heap_order.argtypes = [C.c_uint32, C.POINTER(C.c_float), u32p]
        L.or_heap_order.restype = None
        L.or_allocate_virtual_node.argtypes = [C.c_uint32, u64p, u64p, C.c_uint32, C.c_uint32, u32p, u32p,
                                               u64p, u64p]
        L.or_allocate_virtual_node.restype = C.c_int
        for nm in ("or_contract_fast", "or_contract_small"):
            f = getattr(L, nm)
            f.argtypes = [C.c_uint32, u32p, u32p, u32p, u32p, u32p, C.POINTER(C.c_int64), C.POINTER(C.c_float)]
            f.restype = None
        L.or_trade_run.argtypes = [C.c_uint32, u32p, u32p, u32p, u32p, u32p, u64p, u32p, u32p, u32p, u32p,
                                   C.POINTER(or_trade_cfg), i32p, u32p, u32p, C.c_void_p, C.c_uint64, u64p,
                                   C.c_void_p, C.c_uint64, u64p, C.POINTER(or_trade_cluster_stats), u32p]
        L.or_trade_run.restype = C.c_int
        L.or_dtrade_run.argtypes = [C.c_uint32, u32p, u32p, u32p, u32p, u32p, u64p, u32p, u32p, u32p, u32p,
                                    C.POINTER(or_dtrade_cfg), i32p, u32p, u32p, C.c_void_p, C.c_uint64, u64p,
                                    C.c_void_p, C.c_uint64, u64p, u32p, u32p, C.c_void_p, u32p]
        L.or_dtrade_run.restype = C.c_int
        L.or_delay_run.argtypes = [C.c_uint32, u32p, u32p, C.c_uint64, u32p, u32p, u32p, u32p, C.c_uint32, C.c_int,
                                   i32p, u32p, u32p, C.POINTER(or_delay_stats)]
        L.or_delay_run.restype = C.c_int
        L.or_delay_run_batch.argtypes = [C.c_uint32, u32p, u32p, u32p, u64p, u32p, u32p, u32p, u32p, C.c_uint32,
                                         C.c_int, i32p, u32p, u32p, C.c_void_p]
        L.or_delay_run_batch.restype = C.c_int
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


def fifo_run(free_c, free_m, arrival, dur, cores, mem, literal=False, cap_c=None, cap_m=None):
    """One cluster.  Returns (node, start, finish, stats-dict)."""
    free_c = np.ascontiguousarray(free_c, np.uint32)
    free_m = np.ascontiguousarray(free_m, np.uint32)
    cap_c = free_c if cap_c is None else np.ascontiguousarray(cap_c, np.uint32)
    cap_m = free_m if cap_m is None else np.ascontiguousarray(cap_m, np.uint32)
    a, d, c, m = (np.ascontiguousarray(x, np.uint32) for x in (arrival, dur, cores, mem))
    n = len(a)
    node = np.empty(max(n, 1), np.int32)
    st = np.empty(max(n, 1), np.uint32)
    fi = np.empty(max(n, 1), np.uint32)
    s = or_stats()
    lib().or_fifo_run(len(free_c), _p(cap_c, C.c_uint32), _p(cap_m, C.c_uint32), _p(free_c, C.c_uint32),
                      _p(free_m, C.c_uint32), n, _p(a, C.c_uint32), _p(d, C.c_uint32), _p(c, C.c_uint32),
                      _p(m, C.c_uint32), 1 if literal else 0, _p(node, C.c_int32), _p(st, C.c_uint32),
                      _p(fi, C.c_uint32), C.byref(s))
    stats = dict(t_end=s.t_end, placed=s.placed, waited=s.waited, peak_running=s.peak_running,
                 flags=s.flags, ticks=s.ticks)
    return node[:n], st[:n], fi[:n], stats


def fifo_run_batch(arrays, streams, n_threads=1):
    """Many clusters (CSR).  Returns (node, start, finish, stats structured array)."""
    n = streams.n_jobs
    node = np.empty(max(n, 1), np.int32)
    st = np.empty(max(n, 1), np.uint32)
    fi = np.empty(max(n, 1), np.uint32)
    k = arrays.n_clusters
    stats = (or_stats * k)()
    cc = [np.ascontiguousarray(x, np.uint32) for x in (arrays.cap_c, arrays.cap_m, arrays.free_c, arrays.free_m)]
    off = np.ascontiguousarray(arrays.node_off, np.uint32)
    joff = np.ascontiguousarray(streams.job_off, np.uint64)
    js = [np.ascontiguousarray(x, np.uint32) for x in (streams.arrival, streams.dur, streams.cores, streams.mem)]
    lib().or_fifo_run_batch(k, _p(off, C.c_uint32), *[_p(x, C.c_uint32) for x in cc], _p(joff, C.c_uint64),
                            *[_p(x, C.c_uint32) for x in js], n_threads, _p(node, C.c_int32),
                            _p(st, C.c_uint32), _p(fi, C.c_uint32), stats)
    sd = np.array([(s.t_end, s.placed, s.waited, s.peak_running, s.flags) for s in stats],
                  dtype=[("t_end", "<u4"), ("placed", "<u4"), ("waited", "<u4"), ("peak_running", "<u4"),
                         ("flags", "<u4")])
    return node[:n], st[:n], fi[:n], sd


def schedule_job(free_c, free_m, c, m):
    fc = np.ascontiguousarray(free_c, np.uint64)
    fm = np.ascontiguousarray(free_m, np.uint64)
    return lib().or_schedule_job(len(fc), _p(fc, C.c_uint64), _p(fm, C.c_uint64), c, m)


def lend(free_c, free_m, c, m):
    fc = np.ascontiguousarray(free_c, np.uint64)
    fm = np.ascontiguousarray(free_m, np.uint64)
    return bool(lib().or_lend(len(fc), _p(fc, C.c_uint64), _p(fm, C.c_uint64), c, m))


def resource_utilization(cap_c, cap_m, free_c, free_m):
    arrs = [np.ascontiguousarray(x, np.uint64) for x in (cap_c, cap_m, free_c, free_m)]
    tc = int(np.sum(np.asarray(cap_c, np.uint64))) & 0xFFFFFFFF
    tm = int(np.sum(np.asarray(cap_m, np.uint64))) & 0xFFFFFFFF
    cu = C.c_float()
    mu = C.c_float()
    lib().or_resource_utilization(len(arrs[0]), *[_p(x, C.c_uint64) for x in arrs], tc, tm, C.byref(cu),
                                  C.byref(mu))
    return cu.value, mu.value


def approve_trade(total_c, total_m, cu, mu, cores, mem, time_ns, price):
    return bool(lib().or_approve_trade(total_c, total_m, cu, mu, cores, mem, time_ns, price))


def heap_order(prices):
    p = np.ascontiguousarray(prices, np.float32)
    o = np.empty(max(len(p), 1), np.uint32)
    lib().or_heap_order(len(p), _p(p, C.c_float), _p(o, C.c_uint32))
    return [int(x) for x in o[: len(p)]]


def allocate_virtual_node(free_c, free_m, req_c, req_m):
    fc = np.ascontiguousarray(free_c, np.uint64).copy()
    fm = np.ascontiguousarray(free_m, np.uint64).copy()
    n = len(fc)
    nf = C.c_uint32()
    fnode = np.empty(max(n, 1), np.uint32)
    f_c = np.empty(max(n, 1), np.uint64)
    f_m = np.empty(max(n, 1), np.uint64)
    rc = lib().or_allocate_virtual_node(n, _p(fc, C.c_uint64), _p(fm, C.c_uint64), req_c, req_m, C.byref(nf),
                                        _p(fnode, C.c_uint32), _p(f_c, C.c_uint64), _p(f_m, C.c_uint64))
    k = nf.value
    return rc, fc, fm, [(int(fnode[i]), int(f_c[i]), int(f_m[i])) for i in range(k)]


def contract(kind, jobs):
    """jobs: list of (cores, mem, dur_s).  kind 'fast' or 'small'."""
    n = len(jobs)
    c = np.ascontiguousarray([j[0] for j in jobs] or [0], np.uint32)
    m = np.ascontiguousarray([j[1] for j in jobs] or [0], np.uint32)
    d = np.ascontiguousarray([j[2] for j in jobs] or [0], np.uint32)
    oc, om = C.c_uint32(), C.c_uint32()
    ot = C.c_int64()
    op = C.c_float()
    f = lib().or_contract_fast if kind == "fast" else lib().or_contract_small
    f(n, _p(c, C.c_uint32), _p(m, C.c_uint32), _p(d, C.c_uint32), C.byref(oc), C.byref(om), C.byref(ot),
      C.byref(op))
    return oc.value, om.value, ot.value, op.value


def trade_run(arrays, streams, borrow=True, trader=True, t_max=0xFFFFFFFE, lent_cap=1 << 20, trade_cap=1 << 20,
              period_s=10, trade_ok_sleep_s=240, trade_fail_sleep_s=120, lock_s=20, sample_period_s=5):
    """Lock-step trading run (C5 semantics, oracle/mcs_oracle_trade.c).  Returns a dict with node,
    start, finish (own jobs), lent (LENT_DTYPE records in execution order), trades (TRADE_DTYPE),
    virtual_nodes, decided, lent_pending (per cluster) and t_final."""
    n = streams.n_jobs
    k = arrays.n_clusters
    node = np.empty(max(n, 1), np.int32)
    st = np.empty(max(n, 1), np.uint32)
    fi = np.empty(max(n, 1), np.uint32)
    lent = np.zeros(max(lent_cap, 1), LENT_DTYPE)
    trades = np.zeros(max(trade_cap, 1), TRADE_DTYPE)
    nl, nt, tf = C.c_uint64(), C.c_uint64(), C.c_uint32()
    cs = (or_trade_cluster_stats * max(k, 1))()
    cfg = or_trade_cfg(int(borrow), int(trader), period_s, trade_ok_sleep_s, trade_fail_sleep_s, lock_s,
                       sample_period_s, t_max)
    cc = [np.ascontiguousarray(x, np.uint32) for x in (arrays.cap_c, arrays.cap_m, arrays.free_c, arrays.free_m)]
    off = np.ascontiguousarray(arrays.node_off, np.uint32)
    joff = np.ascontiguousarray(streams.job_off, np.uint64)
    js = [np.ascontiguousarray(x, np.uint32) for x in (streams.arrival, streams.dur, streams.cores, streams.mem)]
    lib().or_trade_run(k, _p(off, C.c_uint32), *[_p(x, C.c_uint32) for x in cc], _p(joff, C.c_uint64),
                       *[_p(x, C.c_uint32) for x in js], C.byref(cfg), _p(node, C.c_int32), _p(st, C.c_uint32),
                       _p(fi, C.c_uint32), lent.ctypes.data, lent_cap, C.byref(nl), trades.ctypes.data, trade_cap,
                       C.byref(nt), cs, C.byref(tf))
    return dict(node=node[:n], start=st[:n], finish=fi[:n], lent=lent[: min(nl.value, lent_cap)].copy(),
                n_lent=nl.value, trades=trades[: min(nt.value, trade_cap)].copy(), n_trades=nt.value,
                virtual_nodes=np.array([c.virtual_nodes for c in cs[:k]], np.uint32),
                decided=np.array([c.decided for c in cs[:k]], np.uint32),
                lent_pending=np.array([c.lent_pending for c in cs[:k]], np.uint32),
                lent_peak=np.array([c.lent_peak for c in cs[:k]], np.uint32), t_final=tf.value)


def _stats_dict(s):
    return {n: getattr(s, n) for n, _ in s._fields_}


def delay_run(free_c, free_m, arrival, dur, cores, mem, literal=False, max_wait_s=10):
    """DELAY policy over one cluster (oracle/mcs_oracle_delay.c).  Returns (node, start, finish, stats)."""
    fc = np.ascontiguousarray(free_c, np.uint32)
    fm = np.ascontiguousarray(free_m, np.uint32)
    a, d, c, m = (np.ascontiguousarray(x, np.uint32) for x in (arrival, dur, cores, mem))
    n = len(a)
    node = np.empty(max(n, 1), np.int32)
    st = np.empty(max(n, 1), np.uint32)
    fi = np.empty(max(n, 1), np.uint32)
    s = or_delay_stats()
    lib().or_delay_run(len(fc), _p(fc, C.c_uint32), _p(fm, C.c_uint32), n, _p(a, C.c_uint32), _p(d, C.c_uint32),
                       _p(c, C.c_uint32), _p(m, C.c_uint32), max_wait_s, 1 if literal else 0,
                       _p(node, C.c_int32), _p(st, C.c_uint32), _p(fi, C.c_uint32), C.byref(s))
    return node[:n], st[:n], fi[:n], _stats_dict(s)


def delay_run_batch(arrays, streams, n_threads=1, max_wait_s=10):
    """DELAY over many clusters (CSR).  Returns (node, start, finish, DELAY_STATS_DTYPE array)."""
    n = streams.n_jobs
    node = np.empty(max(n, 1), np.int32)
    st = np.empty(max(n, 1), np.uint32)
    fi = np.empty(max(n, 1), np.uint32)
    k = arrays.n_clusters
    stats = np.zeros(max(k, 1), DELAY_STATS_DTYPE)
    fc = np.ascontiguousarray(arrays.free_c, np.uint32)
    fm = np.ascontiguousarray(arrays.free_m, np.uint32)
    off = np.ascontiguousarray(arrays.node_off, np.uint32)
    joff = np.ascontiguousarray(streams.job_off, np.uint64)
    js = [np.ascontiguousarray(x, np.uint32) for x in (streams.arrival, streams.dur, streams.cores, streams.mem)]
    lib().or_delay_run_batch(k, _p(off, C.c_uint32), _p(fc, C.c_uint32), _p(fm, C.c_uint32), _p(joff, C.c_uint64),
                             *[_p(x, C.c_uint32) for x in js], max_wait_s, n_threads, _p(node, C.c_int32),
                             _p(st, C.c_uint32), _p(fi, C.c_uint32), stats.ctypes.data)
    return node[:n], st[:n], fi[:n], stats[:k]


def dtrade_run(arrays, streams, t_max=0xFFFFFFFE, trader=True, max_vnodes=256, period_s=10, trade_ok_sleep_s=240,
               trade_fail_sleep_s=120, lock_s=20, sample_period_s=5, max_wait_s=10, trade_cap=1 << 16,
               foreign_cap=1 << 20):
    """Lock-step DELAY clusters with traders (oracle/mcs_oracle_dtrade.c).  Returns a dict with node,
    start, finish, trades (DTRADE_DTYPE), foreign (FOREIGN_DTYPE), vnodes (list per cluster of (c, m)),
    stats (DTRADE_STATS_DTYPE) and t_final.  max_vnodes bounds the oracle's arrays only (Go's
    AddVirtualNode is unbounded): 256, the engine's own ceiling (kDtMaxVnodes, reached by escalation;
    a system that needs more fails there with MCS_E_CAPACITY), so the two agree wherever the engine runs
    (r04: at the old 64 the oracle silently dropped a 65th virtual node the engine kept)."""
    n = streams.n_jobs
    k = arrays.n_clusters
    node = np.empty(max(n, 1), np.int32)
    st = np.empty(max(n, 1), np.uint32)
    fi = np.empty(max(n, 1), np.uint32)
    trades = np.zeros(max(trade_cap, 1), DTRADE_DTYPE)
    foreign = np.zeros(max(foreign_cap, 1), FOREIGN_DTYPE)
    vc = np.zeros(max(k * max_vnodes, 1), np.uint32)
    vm = np.zeros(max(k * max_vnodes, 1), np.uint32)
    stats = np.zeros(max(k, 1), DTRADE_STATS_DTYPE)
    nt, nf, tf = C.c_uint64(), C.c_uint64(), C.c_uint32()
    cfg = or_dtrade_cfg(period_s if trader else 0, trade_ok_sleep_s, trade_fail_sleep_s, lock_s, sample_period_s,
                        max_wait_s, max_vnodes, t_max)
    cc = [np.ascontiguousarray(x, np.uint32) for x in (arrays.cap_c, arrays.cap_m, arrays.free_c, arrays.free_m)]
    off = np.ascontiguousarray(arrays.node_off, np.uint32)
    joff = np.ascontiguousarray(streams.job_off, np.uint64)
    js = [np.ascontiguousarray(x, np.uint32) for x in (streams.arrival, streams.dur, streams.cores, streams.mem)]
    lib().or_dtrade_run(k, _p(off, C.c_uint32), *[_p(x, C.c_uint32) for x in cc], _p(joff, C.c_uint64),
                        *[_p(x, C.c_uint32) for x in js], C.byref(cfg), _p(node, C.c_int32), _p(st, C.c_uint32),
                        _p(fi, C.c_uint32), trades.ctypes.data, trade_cap, C.byref(nt), foreign.ctypes.data,
                        foreign_cap, C.byref(nf), _p(vc, C.c_uint32), _p(vm, C.c_uint32), stats.ctypes.data,
                        C.byref(tf))
    stats = stats[:k].copy()
    vnodes = [[(int(vc[c * max_vnodes + i]), int(vm[c * max_vnodes + i])) for i in range(int(stats["virtual_nodes"][c]))]
              for c in range(k)]
    return dict(node=node[:n], start=st[:n], finish=fi[:n], trades=trades[: min(nt.value, trade_cap)].copy(),
                n_trades=nt.value, foreign=foreign[: min(nf.value, foreign_cap)].copy(), n_foreign=nf.value,
                vnodes=vnodes, stats=stats, t_final=tf.value)
