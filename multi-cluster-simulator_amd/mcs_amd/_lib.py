"""ctypes binding of libmcs.so (include/mcs.h, include/mcs_trade.h).

The library is loaded from this package directory (built in-tree by ``make`` /
``__graft_entry__.build()``).  There is no fallback: if the library is missing, or no HIP device
is usable, calls raise :class:`MCSError`.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# MCS_LIB overrides the library path (A/B timing of kernel variants, tools/ab_bench.py)
LIB_PATH = os.environ.get("MCS_LIB") or os.path.join(_HERE, "libmcs.so")

MCS_OK = 0
MCS_NO_FIT = 1
MCS_E_INVALID = -1
MCS_E_CAPACITY = -2
MCS_E_HIP = -3
MCS_E_RCCL = -4
MCS_E_STATE = -5
MCS_E_NOMEM = -6
MCS_E_RANGE = -7

MCS_NODE_UNPLACED = -1
MCS_NODE_BORROWED = -2
MCS_TIME_NONE = 0xFFFFFFFF
MCS_FLAG_DEADLOCK = 0x1
MCS_FLAG_OVERFLOW = 0x2
MCS_FLAG_CLOCK_OVERFLOW = 0x4
MCS_FLAG_LENT_OVERFLOW = 0x8
MCS_FLAG_LOG_OVERFLOW = 0x10
MCS_FLAG_T_MAX = 0x20
MCS_FLAG_VNODE_OVERFLOW = 0x40

MCS_POLICY_FIFO = 0
MCS_POLICY_DELAY = 1
MCS_ARRIVAL_REF = 0
MCS_ARRIVAL_SCALED = 1
MCS_ARRIVAL_WEIBULL = 2

STATUS_NAMES = {
    MCS_OK: "MCS_OK",
    MCS_NO_FIT: "MCS_NO_FIT",
    MCS_E_INVALID: "MCS_E_INVALID",
    MCS_E_CAPACITY: "MCS_E_CAPACITY",
    MCS_E_HIP: "MCS_E_HIP",
    MCS_E_RCCL: "MCS_E_RCCL",
    MCS_E_STATE: "MCS_E_STATE",
    MCS_E_NOMEM: "MCS_E_NOMEM",
    MCS_E_RANGE: "MCS_E_RANGE",
}


class MCSError(RuntimeError):
    def __init__(self, code: int, msg: str = ""):
        self.code = code
        super().__init__(f"{STATUS_NAMES.get(code, code)}: {msg}")


class mcs_config(C.Structure):
    _fields_ = [
        ("policy", C.c_uint32),
        ("borrow", C.c_uint32),
        ("trader", C.c_uint32),
        ("wait_sleep_s", C.c_uint32),
        ("idle_sleep_s", C.c_uint32),
        ("slot_pool", C.c_uint32),
        ("trader_period_s", C.c_uint32),
        ("trade_ok_sleep_s", C.c_uint32),
        ("trade_fail_sleep_s", C.c_uint32),
        ("lock_s", C.c_uint32),
        ("sample_period_s", C.c_uint32),
        ("lent_queue_cap", C.c_uint32),
        ("t_max_s", C.c_uint32),
        ("max_wait_s", C.c_uint32),
        ("unchecked_horizon", C.c_uint32),
        ("reserved", C.c_uint32 * 1),
    ]


class mcs_gen_params(C.Structure):
    _fields_ = [
        ("seed", C.c_uint64),
        ("arrival_mode", C.c_uint32),
        ("max_dur_s", C.c_uint32),
        ("lambda_", C.c_double),
        ("max_cores", C.c_uint32),
        ("max_mem", C.c_uint32),
        ("fused", C.c_uint32),
        ("weibull_k", C.c_float),
        ("reserved", C.c_uint32 * 2),
    ]


class mcs_stats(C.Structure):
    _fields_ = [
        ("jobs", C.c_uint64),
        ("placed", C.c_uint64),
        ("waited", C.c_uint64),
        ("unplaced", C.c_uint64),
        ("clusters", C.c_uint32),
        ("deadlocked", C.c_uint32),
        ("escalations", C.c_uint32),
        ("slot_pool", C.c_uint32),
        ("kernel_ms", C.c_double),
        ("wall_ms", C.c_double),
        ("pending", C.c_uint64),
        ("t_horizon", C.c_uint32),
        ("online", C.c_uint32),
        ("handed_over", C.c_uint32),
        ("reserved", C.c_uint32),
    ]


class mcs_cluster_stats(C.Structure):
    _fields_ = [
        ("t_end", C.c_uint32),
        ("placed", C.c_uint32),
        ("waited", C.c_uint32),
        ("peak_running", C.c_uint32),
        ("flags", C.c_uint32),
        ("pool", C.c_uint32),
        ("iterations", C.c_uint32),
        ("release_scans", C.c_uint32),
    ]


class mcs_cluster_state(C.Structure):
    _fields_ = [
        ("cores_utilization", C.c_float),
        ("memory_utilization", C.c_float),
        ("total_cpu", C.c_uint32),
        ("total_memory", C.c_uint32),
        ("running", C.c_uint32),
        ("t_s", C.c_uint32),
    ]


class mcs_delay_cluster_stats(C.Structure):
    _fields_ = [
        ("total_wait_ms", C.c_int64),
        ("jobs_count", C.c_int64),
        ("moved_l1", C.c_uint32),
        ("placed_l1", C.c_uint32),
        ("peak_l1", C.c_uint32),
        ("l1_left", C.c_uint32),
    ]


class mcs_lent_rec(C.Structure):
    _fields_ = [("lender", C.c_uint32), ("borrower", C.c_uint32), ("job", C.c_uint64), ("node", C.c_uint32),
                ("start_s", C.c_uint32), ("finish_s", C.c_uint32), ("pad", C.c_uint32)]


class mcs_trade_rec(C.Structure):
    _fields_ = [("t_s", C.c_uint32), ("requester", C.c_uint32), ("winner", C.c_int32), ("approvals", C.c_uint32)]


class mcs_contract_rec(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in ("t_s", "requester")] + [("winner", C.c_int32)] + \
               [(n, C.c_uint32) for n in ("approvals", "policy", "cores", "mem", "time_s", "failed", "pad")]


class mcs_foreign_rec(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in ("requester", "responder", "node", "start_s", "finish_s", "pad")] + \
               [("c", C.c_uint64), ("m", C.c_uint64)]


class mcs_trade_stats(C.Structure):
    _fields_ = [
        ("placed", C.c_uint64),
        ("borrowed", C.c_uint64),
        ("waited", C.c_uint64),
        ("undecided", C.c_uint64),
        ("lent_runs", C.c_uint64),
        ("lent_pending", C.c_uint64),
        ("trades", C.c_uint64),
        ("trades_won", C.c_uint64),
        ("ticks", C.c_uint32),
        ("t_final", C.c_uint32),
        ("flags", C.c_uint32),
        ("loop_form", C.c_uint32),
        ("kernel_ms", C.c_double),
        ("wall_ms", C.c_double),
        ("block_bytes", C.c_uint64),
        ("snaps", C.c_uint32),
        ("agreed", C.c_uint32),
    ]


MCS_TRADE_SHAPE_WORDS = 8


class mcs_approve_query(C.Structure):
    _fields_ = [("total_cores", C.c_uint32), ("total_memory", C.c_uint32), ("core_util", C.c_float),
                ("mem_util", C.c_float), ("cores", C.c_uint32), ("memory", C.c_uint32), ("time_s", C.c_uint32),
                ("pad", C.c_uint32)]


class mcs_comm_id(C.Structure):
    _fields_ = [("bytes", C.c_char * 128)]


u32p = C.POINTER(C.c_uint32)
i32p = C.POINTER(C.c_int32)
u64p = C.POINTER(C.c_uint64)
f32p = C.POINTER(C.c_float)
vp = C.c_void_p

# (name, restype, argtypes) for every symbol include/mcs.h declares
SIGNATURES = [
    ("mcs_abi_version", C.c_int, []),
    ("mcs_config_default", None, [C.POINTER(mcs_config)]),
    ("mcs_gen_params_default", None, [C.POINTER(mcs_gen_params)]),
    ("mcs_gen_cluster_host", C.c_int,
     [C.POINTER(mcs_gen_params), C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64, u32p, u32p, u32p, u32p]),
    ("mcs_gen_scaled_lambda", C.c_double, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_double]),
    ("mcs_engine_create", C.c_int, [C.POINTER(mcs_config), C.c_int, C.POINTER(vp)]),
    ("mcs_engine_destroy", C.c_int, [vp]),
    ("mcs_last_error", C.c_char_p, [vp]),
    ("mcs_last_kernel", C.c_char_p, [vp]),
    ("mcs_load_clusters", C.c_int, [vp, u32p, u32p, u32p, u32p, u32p, C.c_uint32]),
    ("mcs_submit_jobs", C.c_int, [vp, u32p, u32p, u32p, u32p, u64p]),
    ("mcs_generate_jobs", C.c_int, [vp, C.POINTER(mcs_gen_params), C.c_uint64]),
    ("mcs_read_jobs", C.c_int, [vp, u32p, u32p, u32p, u32p]),
    ("mcs_run", C.c_int, [vp, C.c_uint32, C.POINTER(mcs_stats)]),
    ("mcs_append_jobs", C.c_int, [vp, u32p, u32p, u32p, u32p, u64p]),
    ("mcs_rewind", C.c_int, [vp]),
    ("mcs_read_job_offsets", C.c_int, [vp, u64p]),
    ("mcs_read_placements", C.c_int, [vp, i32p, u32p, u32p]),
    ("mcs_read_cluster_stats", C.c_int, [vp, C.POINTER(mcs_cluster_stats), C.c_uint32]),
    ("mcs_read_delay_stats", C.c_int, [vp, C.POINTER(mcs_delay_cluster_stats), C.c_uint32]),
    ("mcs_num_clusters", C.c_uint32, [vp]),
    ("mcs_num_jobs", C.c_uint64, [vp]),
    ("mcs_schedule_one", C.c_int, [vp, C.c_uint32, C.c_uint32, C.c_uint32, i32p]),
    ("mcs_release_one", C.c_int, [vp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]),
    ("mcs_lend_check", C.c_int, [vp, C.c_uint32, C.c_uint32, C.c_uint32, i32p]),
    ("mcs_read_live_state", C.c_int, [vp, C.c_uint32, u32p, u32p, C.c_uint32]),
    ("mcs_resource_utilization", C.c_int, [vp, C.c_uint32, f32p, f32p]),
    ("mcs_cluster_states", C.c_int, [vp, C.c_uint32, C.POINTER(mcs_cluster_state), C.c_uint32,
                                     C.POINTER(C.c_double)]),
    # include/mcs_trade.h
    ("mcs_set_shard", C.c_int, [vp, C.c_uint32, C.c_uint32]),
    ("mcs_comm_unique_id", C.c_int, [C.POINTER(mcs_comm_id)]),
    ("mcs_comm_init", C.c_int, [vp, C.POINTER(mcs_comm_id)]),
    ("mcs_trade_begin", C.c_int, [vp]),
    ("mcs_trade_shape_words", C.c_int, [vp, u32p]),
    ("mcs_trade_set_shape", C.c_int, [vp, u32p]),
    ("mcs_trade_xfer_bytes", C.c_int, [vp, C.c_uint32, u64p, u64p]),
    ("mcs_trade_phase", C.c_int, [vp, C.c_uint32, vp, C.c_uint64, vp, C.c_uint64, u32p]),
    ("mcs_trade_end", C.c_int, [vp, C.POINTER(mcs_stats)]),
    ("mcs_read_trade_stats", C.c_int, [vp, C.POINTER(mcs_trade_stats)]),
    ("mcs_read_lent", C.c_int, [vp, C.POINTER(mcs_lent_rec), C.c_uint64, u64p]),
    ("mcs_read_trades", C.c_int, [vp, C.POINTER(mcs_trade_rec), C.c_uint64, u64p]),
    ("mcs_read_virtual_nodes", C.c_int, [vp, u32p, C.c_uint32]),
    ("mcs_read_contracts", C.c_int, [vp, C.POINTER(mcs_contract_rec), C.c_uint64, u64p]),
    ("mcs_read_foreign", C.c_int, [vp, C.POINTER(mcs_foreign_rec), C.c_uint64, u64p]),
    ("mcs_read_virtual_node_caps", C.c_int, [vp, C.c_uint32, u32p, u32p, C.c_uint32, u32p]),
    ("mcs_approve_trade", C.c_int, [vp, C.POINTER(mcs_approve_query), C.c_uint32, i32p]),
]

_lib = None


def lib() -> C.CDLL:
    """Load libmcs.so (once).  Raises MCSError if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise MCSError(MCS_E_STATE, f"{LIB_PATH} not built (run __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            if os.environ.get("MCS_LIB") and not hasattr(L, name):
                continue  # an older library under A/B timing (tools/ab_bench.py) lacks newer entry points
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def ptr(a, ct):
    """numpy array -> ctypes pointer (the array must stay alive during the call)."""
    return a.ctypes.data_as(C.POINTER(ct))
