"""mcs_amd — MI355X-native batched FIFO placement engine for the hot path of
hamzalsheikh/multi-cluster-simulator (pkg/scheduler FIFO loop + first-fit placement, and the
lock-step borrow / trader exchange of pkg/scheduler + pkg/trader).

Import path: add ``<repo>/multi-cluster-simulator_amd`` to sys.path (see ``mcs_amd.paths``).
"""
from ._lib import (MCS_ARRIVAL_REF, MCS_ARRIVAL_SCALED, MCS_FLAG_DEADLOCK, MCS_FLAG_OVERFLOW,
                   MCS_NODE_BORROWED, MCS_NODE_UNPLACED, MCS_TIME_NONE, LIB_PATH, MCSError, lib)
from .cluster import Cluster, ClusterArrays, Node, pack_clusters, replicate, uniform_cluster
from .engine import (CLUSTER_STATS_DTYPE, DELAY_STATS_DTYPE, LENT_DTYPE, TRADE_DTYPE, Engine, GenParams, JobStreams, RunStats, device_count,
                     gen_cluster_host, gen_streams_host, scaled_lambda)

__all__ = [
    "Cluster", "ClusterArrays", "Node", "pack_clusters", "replicate", "uniform_cluster",
    "Engine", "GenParams", "JobStreams", "RunStats", "gen_cluster_host", "gen_streams_host",
    "scaled_lambda", "device_count", "CLUSTER_STATS_DTYPE", "DELAY_STATS_DTYPE", "MCSError", "lib", "LIB_PATH",
    "MCS_ARRIVAL_REF", "MCS_ARRIVAL_SCALED", "MCS_FLAG_DEADLOCK", "MCS_FLAG_OVERFLOW",
    "MCS_NODE_UNPLACED", "MCS_NODE_BORROWED", "MCS_TIME_NONE", "LENT_DTYPE", "TRADE_DTYPE",
]
