/*
 * mcs.h — C ABI of the MI355X batched FIFO placement engine (libmcs.so).
 *
 * Drop-in boundary for the data-parallel hot path of hamzalsheikh/multi-cluster-simulator
 * (reference snapshot 2024-10-16).  The reference has no FFI: the path is a set of Go methods on
 * a global singleton.  Each entry point below names the reference symbol it replaces
 * (path:line relative to the reference root).  A Go cgo binding is shown in INTEGRATION.md.
 *
 * Rules of the ABI:
 *   - plain C99, no C++ types, no callbacks; every call is blocking;
 *   - the caller owns every host array; the engine copies inputs in during the call and never
 *     keeps host pointers; the engine owns all device memory and frees it in mcs_engine_destroy;
 *   - a handle is NOT thread-safe: one host thread (one cgo goroutine) per handle, one handle per GPU;
 *   - status codes are ints (mcs_status); details via mcs_last_error(); no exception crosses the ABI.
 *
 * Units: every time is a whole number of SECONDS in a uint32 (deviation D8 of SURVEY Appendix A:
 * the reference only produces whole seconds — pkg/client/client.go:98 and all sleeps).
 */
#ifndef MCS_H
#define MCS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MCS_ABI_VERSION 7

/* ---- status codes --------------------------------------------------------------------------- */
typedef enum mcs_status {
    MCS_OK = 0,
    /* ScheduleJob's error "not enough resources in cluster" (pkg/scheduler/scheduler.go:138) */
    MCS_NO_FIT = 1,
    MCS_E_INVALID = -1,  /* bad argument / inconsistent sizes                                     */
    MCS_E_CAPACITY = -2, /* running-slot pool overflow that survived capacity escalation          */
    MCS_E_HIP = -3,      /* a HIP runtime call failed                                             */
    MCS_E_RCCL = -4,     /* an RCCL call failed                                                   */
    MCS_E_STATE = -5,    /* call out of order (e.g. mcs_run before mcs_load_clusters)             */
    MCS_E_NOMEM = -6,    /* host or device allocation failed                                      */
    MCS_E_RANGE = -7     /* a cluster's simulated clock left the uint32 seconds range (D8): the run
                            stopped there; MCS_FLAG_CLOCK_OVERFLOW marks it and its undecided jobs
                            read MCS_NODE_UNPLACED / MCS_TIME_NONE                                 */
} mcs_status;

/* Node index written for a job that is never placed (head-of-line deadlock: the wait-queue head
 * cannot fit even on an empty cluster, so the reference's Fifo loop retries it forever,
 * scheduler.go:219-251).  start/finish are then MCS_TIME_NONE. */
#define MCS_NODE_UNPLACED (-1)
/* Node index written for a job moved to the BorrowedQueue (scheduler.go:237-242; mcs_trade.h):
 * start = the borrow tick, finish = MCS_TIME_NONE; the lender's run is in mcs_read_lent. */
#define MCS_NODE_BORROWED (-2)
#define MCS_TIME_NONE 0xFFFFFFFFu

/* per-cluster flag bits (mcs_cluster_stats.flags) */
#define MCS_FLAG_DEADLOCK 0x1u /* head-of-line job can never fit; rest of the stream unplaced     */
#define MCS_FLAG_OVERFLOW 0x2u /* running-slot pool overflow (engine re-runs with a larger pool)   */
#define MCS_FLAG_CLOCK_OVERFLOW 0x4u /* the uint32 seconds clock would wrap; results after it invalid */
#define MCS_FLAG_LENT_OVERFLOW 0x8u  /* a LentQueue exceeded lent_queue_cap (lock-step runs)          */
#define MCS_FLAG_LOG_OVERFLOW 0x10u  /* lent/trade log capacity exceeded: records dropped, counts kept */
#define MCS_FLAG_T_MAX 0x20u         /* lock-step run stopped at t_max_s with work left               */
#define MCS_FLAG_VNODE_OVERFLOW 0x40u /* DELAY trading: a cluster received more virtual nodes than the
                                         engine holds (engine re-runs with more)                      */

/* ---- configuration ------------------------------------------------------------------------- */
typedef enum mcs_policy {
    MCS_POLICY_FIFO = 0,  /* Scheduler.Fifo (scheduler.go:216-296); selected by config (D4)       */
    MCS_POLICY_DELAY = 1  /* Scheduler.Delay (scheduler.go:298-369), the reference default (:116);
                             serialized semantics SDELAY; ABI v3                   */
} mcs_policy;

typedef struct mcs_config {
    uint32_t policy;         /* mcs_policy                                                         */
    uint32_t borrow;         /* FIFO cross-cluster borrow (server.go:160-248; mcs_trade.h)          */
    uint32_t trader;         /* trader offer exchange (trader.go:193-325; mcs_trade.h)              */
    uint32_t wait_sleep_s;   /* sleep after a wait-queue attempt, scheduler.go:250 (must be 1)     */
    uint32_t idle_sleep_s;   /* sleep when all queues are empty, scheduler.go:294 (must be 1)      */
    uint32_t slot_pool;      /* running-slot pool per cluster in units of 64 (0 = auto)            */
    /* lock-step trading cadences (used when borrow or trader is set; mcs_trade.h) */
    uint32_t trader_period_s;    /* 10: time.Sleep(10 s) per monitor pass, trader.go:323            */
    uint32_t trade_ok_sleep_s;   /* 240: after a successful trade, trader.go:297                    */
    uint32_t trade_fail_sleep_s; /* 120: after a failed trade, trader.go:300                        */
    uint32_t lock_s;             /* 20: responder contract lock, pkg/trader/server.go:48-57         */
    uint32_t sample_period_s;    /* 5: scheduler state stream period, trader_server.go:44           */
    uint32_t lent_queue_cap;     /* LentQueue entries per cluster (0 = 4096)                        */
    uint32_t t_max_s;            /* stop the lock-step clock after this tick (0 = 0xFFFFFFFE)       */
    uint32_t max_wait_s;         /* DELAY: Policy.MaxWaitTime, 10 s (scheduler.go:115,353)          */
    uint32_t unchecked_horizon;  /* 0 (default): mcs_submit_jobs / mcs_generate_jobs / mcs_append_jobs
                                    reject streams whose clock bound (last arrival + sum of (dur + 1
                                    [+ max_wait_s under DELAY])) leaves the uint32 range.  1: skip that
                                    check (tests of the device-side guard: the kernels then stop the
                                    cluster with MCS_FLAG_CLOCK_OVERFLOW and mcs_run returns
                                    MCS_E_RANGE).  Not allowed with borrow or trader (the lock-step
                                    kernels have no such guard): mcs_engine_create returns
                                    MCS_E_INVALID                                                    */
    uint32_t reserved[1];
} mcs_config;

/* Fills the reference defaults (FIFO, no borrow, no trader, 1 s sleeps, trader cadences above). */
void mcs_config_default(mcs_config* cfg);

/* ---- synthetic job stream (input synthesis; restates pkg/client/client.go:85-147) ----------- */
typedef enum mcs_arrival_mode {
    MCS_ARRIVAL_REF = 0,    /* per minute n ~ Poisson(lambda), spacing floor(60/n) s (client.go:107-125);
                               n == 0 is an idle minute of 60 s (D5)                                 */
    MCS_ARRIVAL_SCALED = 1, /* per second n ~ Poisson(lambda) arrivals at that second               */
    MCS_ARRIVAL_WEIBULL = 2 /* the client's "weibull" mode (client.go:131-145): after each job a sleep of
                               floor(X) s, X ~ Weibull(scale lambda, shape weibull_k); the reference
                               uses Lambda 10, K 3 (gonum distuv.Weibull)                          */
} mcs_arrival_mode;

typedef struct mcs_gen_params {
    uint64_t seed;        /* base seed; cluster k uses key = mix(seed ^ k)                           */
    uint32_t arrival_mode;/* mcs_arrival_mode                                                        */
    uint32_t max_dur_s;   /* durations U{0..max_dur_s-1}; 600 = rand.Intn(600) (client.go:98)        */
    double lambda;        /* Poisson mean per minute (REF, 10 in client.go:108) or per second (SCALED);
                             WEIBULL: the scale (Lambda: 10, client.go:133)                          */
    uint32_t max_cores;   /* 0 = per-cluster max node Cores (setMaxCluster, client.go:68-83)          */
    uint32_t max_mem;     /* 0 = per-cluster max node Memory                                          */
    uint32_t fused;       /* 1: no job records in HBM; the FIFO/DELAY kernels synthesise each 64-job
                             batch in registers, bit-identical to the records;
                             mcs_read_jobs and the trading paths materialise them on demand      */
    float weibull_k;      /* WEIBULL: the shape (K: 3, client.go:134); 0 = 3                          */
    uint32_t reserved[2];
} mcs_gen_params;

void mcs_gen_params_default(mcs_gen_params* p);

/* Host generator (same arithmetic as the device generator, bit-identical output).  Generates the
 * jobs of ONE cluster (index `cluster`) with the given max cores/mem. */
int mcs_gen_cluster_host(const mcs_gen_params* p, uint32_t cluster, uint32_t max_cores,
                         uint32_t max_mem, uint64_t n_jobs, uint32_t* arrival_s, uint32_t* dur_s,
                         uint32_t* cores, uint32_t* mem);

/* Per-second lambda giving `load` offered memory load for n_nodes nodes of node_mem memory
 * (SCALED mode): lambda = load * n_nodes * node_mem / (E[mem] * E[dur]). */
double mcs_gen_scaled_lambda(uint32_t n_nodes, uint32_t node_mem, uint32_t max_mem,
                             uint32_t max_dur_s, double load);

/* ---- engine ---------------------------------------------------------------------------------- */
typedef struct mcs_engine mcs_engine;

typedef struct mcs_stats {
    uint64_t jobs;          /* jobs in the submitted streams                                     */
    uint64_t placed;        /* jobs placed on a node                                             */
    uint64_t waited;        /* jobs that entered the wait queue (scheduler.go:264-268)           */
    uint64_t unplaced;      /* jobs never placed (deadlocked clusters)                           */
    uint32_t clusters;
    uint32_t deadlocked;    /* clusters with MCS_FLAG_DEADLOCK                                   */
    uint32_t escalations;   /* slot-pool re-runs performed                                       */
    uint32_t slot_pool;     /* largest slot pool used (x64)                                      */
    double kernel_ms;       /* device time of the placement kernel(s), HIP events on the engine stream */
    double wall_ms;         /* host wall time of the whole mcs_run call                           */
    uint64_t pending;       /* online runs: jobs not decided yet (queued, or arriving later)       */
    uint32_t t_horizon;     /* online runs: the horizon reached (MCS_TIME_NONE after a drain)      */
    uint32_t online;        /* 1 if this run continued an online session (finite horizons)         */
    uint32_t handed_over;   /* DELAY, ABI v6: clusters the hand-scheduled loop handed to the compiled
                               delay_kernel (re-run from t = 0: Level1 past its LDS slice, the clock
                               range after a move, or a runaway guard of the loop)                           */
    uint32_t reserved;
} mcs_stats;

typedef struct mcs_cluster_stats {
    uint32_t t_end;         /* simulated clock when the cluster's queues drained (seconds)       */
    uint32_t placed;
    uint32_t waited;
    uint32_t peak_running;  /* peak jobs holding resources (dur > 0)                              */
    uint32_t flags;         /* MCS_FLAG_*                                                         */
    uint32_t pool;          /* slot pool (x64) the final result was produced with                */
    uint32_t iterations;    /* diagnostics: decision-loop passes (the hand-scheduled loop counts the
                               passes without a decision only with MCS_FIFO_DIAG=1 in the env)     */
    uint32_t release_scans; /* diagnostics: clock advances that released running jobs (ditto)    */
} mcs_cluster_stats;

/* DELAY-policy statistics of one cluster (MCS_POLICY_DELAY runs; mcs_read_delay_stats). */
typedef struct mcs_delay_cluster_stats {
    int64_t total_wait_ms;  /* WaitTime.TotalTime at t_end (scheduler.go:48-54,309-312,338-341):
                               1000 * (start - arrival) per placed job, 1000 * (t_end - arrival)
                               per job left in Level1                                             */
    int64_t jobs_count;     /* WaitTime.JobsCount: jobs received by "/delay" (server.go:72)         */
    uint32_t moved_l1;      /* Level0 -> Level1 moves after MaxWaitTime (scheduler.go:353-359)      */
    uint32_t placed_l1;     /* placements made by the Level1 pass (scheduler.go:302-329)           */
    uint32_t peak_l1;       /* peak len(Level1)                                                    */
    uint32_t l1_left;       /* Level1 jobs that can never fit (MCS_FLAG_DEADLOCK)                  */
} mcs_delay_cluster_stats;

/* scheduler.Run (scheduler.go:101-124) builds a Scheduler; here one engine batches many clusters
 * on ONE GPU (`device` = HIP ordinal). */
int mcs_engine_create(const mcs_config* cfg, int device, mcs_engine** out);
int mcs_engine_destroy(mcs_engine* eng);
const char* mcs_last_error(const mcs_engine* eng);
int mcs_abi_version(void);
/* Name of the placement kernel the last mcs_run launched first ("mcs::fifo_asm_kernel",
 * "mcs::fifo_kernel", "mcs::delay_kernel"; "" before any run): lets a caller match its timings
 * to a rocprofv3 kernel trace.  Owned by the engine. */
const char* mcs_last_kernel(const mcs_engine* eng);

/* Cluster specs (assets/cluster_*.json, Cluster/Node in pkg/scheduler/cluster.go:14-24,127-138):
 * nodes of cluster c are [node_offsets[c], node_offsets[c+1]) in JSON array order; free_* are the
 * JSON CoresAvailable/MemoryAvailable, kept as-is by Run (scheduler.go:101-109, KAT5).
 * At most 1024 nodes per cluster in ABI v1. */
int mcs_load_clusters(mcs_engine* eng, const uint32_t* cap_c, const uint32_t* cap_m,
                      const uint32_t* free_c, const uint32_t* free_m,
                      const uint32_t* node_offsets, uint32_t n_clusters);

/* Job streams (the ReadyQueue filled by the "/" handler, server.go:23-51): jobs of cluster c are
 * [job_offsets[c], job_offsets[c+1]), sorted by arrival (non-decreasing); job id = index. */
int mcs_submit_jobs(mcs_engine* eng, const uint32_t* arrival_s, const uint32_t* dur_s,
                    const uint32_t* cores, const uint32_t* mem, const uint64_t* job_offsets);

/* Same as mcs_submit_jobs but synthesises n_jobs per cluster on the device (bit-identical to
 * mcs_gen_cluster_host for every cluster).  With p->fused the records are never stored: every
 * FIFO/DELAY run regenerates them inside the placement kernels. */
int mcs_generate_jobs(mcs_engine* eng, const mcs_gen_params* p, uint64_t jobs_per_cluster);

/* Copies the (submitted or generated) job streams back to the host (sizes from the offsets). */
int mcs_read_jobs(mcs_engine* eng, uint32_t* arrival_s, uint32_t* dur_s, uint32_t* cores,
                  uint32_t* mem);

/* Runs the configured policy loop for every cluster over ScheduleJob (scheduler.go:127-139) and
 * Node.RunJob (cluster.go:141-161):
 *   MCS_POLICY_FIFO  — Scheduler.Fifo (scheduler.go:216-296), serialized semantics SFIFO
 *                      (SURVEY Appendix A); with cfg.borrow or cfg.trader set the clusters instead
 *                      advance in lock-step with the borrow and trade exchanges (mcs_trade.h);
 *   MCS_POLICY_DELAY — Scheduler.Delay (scheduler.go:298-369) with jobs ingested by the "/delay"
 *                      handler (server.go:53-78), serialized semantics SDELAY.
 *                      MCS_FLAG_DEADLOCK marks clusters whose Level1 keeps jobs that can never
 *                      fit; those jobs get MCS_NODE_UNPLACED and every other job is placed.
 *
 * Batch mode (the default after mcs_submit_jobs / mcs_generate_jobs): t_end_s = MCS_TIME_NONE runs
 * every cluster from its loaded spec until every job is decided; repeated calls repeat the run.
 *
 * Online mode (FIFO / DELAY without trading) replaces the reference's infinite loop
 * fed by HTTP POSTs (scheduler.go:216-296, 298-369; server.go:23-78): a finite t_end_s, or any
 * mcs_append_jobs, starts a session that keeps each cluster's state (clock, queues, node counters,
 * running jobs) on the device between calls.  mcs_run(t_end_s) then makes every decision the Go
 * loop makes at simulated seconds t < t_end_s and stops there; mcs_run(MCS_TIME_NONE) continues
 * until every job appended so far is decided (a drain).  Horizons are non-decreasing.  Jobs
 * appended after mcs_run(h) must arrive at or after h (they are POSTed after that moment).  Splitting
 * a run into horizons, with the jobs appended between them, gives bit-for-bit the placements of
 * the batch run over all the jobs.  Between horizons the placements of undecided jobs read
 * MCS_NODE_UNPLACED / MCS_TIME_NONE; the cluster and DELAY statistics are final after a drain.
 * Returns MCS_E_RANGE (results readable) when a cluster's clock leaves the uint32 range. */
int mcs_run(mcs_engine* eng, uint32_t t_end_s, mcs_stats* stats);

/* Online mode: append jobs to the clusters' streams (the "/" or "/delay" handler appending to the
 * ReadyQueue / Level0, server.go:38-41,67-69).  Jobs of cluster c are [job_offsets[c],
 * job_offsets[c+1]) of the given arrays, arrival-sorted, each arrival >= the cluster's last one,
 * >= the last finite horizon run, and >= the cluster's own clock after the last drain (a cluster
 * whose drain ended earlier accepts earlier arrivals than one that ran longer).  Their ids continue the cluster's stream (dense order of
 * mcs_read_placements: per cluster, submitted then appended jobs in order).  Starts an online
 * session (state at t = 0) if none is active.  Not available with borrow/trader. */
int mcs_append_jobs(mcs_engine* eng, const uint32_t* arrival_s, const uint32_t* dur_s,
                    const uint32_t* cores, const uint32_t* mem, const uint64_t* job_offsets);

/* Online mode: restart the session at t = 0 with every job submitted and appended so far. */
int mcs_rewind(mcs_engine* eng);

/* Dense CSR of the current streams (n_clusters + 1 entries): jobs of cluster c are rows
 * [off[c], off[c+1]) of mcs_read_placements / mcs_read_jobs. */
int mcs_read_job_offsets(mcs_engine* eng, uint64_t* off);

/* Per-job results of the last mcs_run, indexed like the submitted jobs. */
int mcs_read_placements(mcs_engine* eng, int32_t* node, uint32_t* start_s, uint32_t* finish_s);
int mcs_read_cluster_stats(mcs_engine* eng, mcs_cluster_stats* out, uint32_t n_clusters);
/* DELAY statistics of the last MCS_POLICY_DELAY run (MCS_E_STATE after a FIFO run). */
int mcs_read_delay_stats(mcs_engine* eng, mcs_delay_cluster_stats* out, uint32_t n_clusters);

uint32_t mcs_num_clusters(const mcs_engine* eng);
uint64_t mcs_num_jobs(const mcs_engine* eng);

/* ---- single-job mirrors (live cluster state, initialised from the spec at load time) -------- */
/* Scheduler.ScheduleJob (scheduler.go:127-139) with the commit of Node.RunJob (cluster.go:144-148)
 * done synchronously (D2): first node in order with CoresAvailable >= cores && MemoryAvailable >=
 * mem.  Returns MCS_OK and *node, or MCS_NO_FIT with *node = MCS_NODE_UNPLACED. */
int mcs_schedule_one(mcs_engine* eng, uint32_t cluster, uint32_t cores, uint32_t mem,
                     int32_t* node);
/* The completion half of Node.RunJob (cluster.go:153-157): node gives back cores/mem. */
int mcs_release_one(mcs_engine* eng, uint32_t cluster, uint32_t node, uint32_t cores,
                    uint32_t mem);
/* Scheduler.Lend (scheduler.go:194-202): strict '>' existence test, no commit. */
int mcs_lend_check(mcs_engine* eng, uint32_t cluster, uint32_t cores, uint32_t mem, int32_t* ok);
/* Live free vectors of one cluster (n = node count of the cluster). */
int mcs_read_live_state(mcs_engine* eng, uint32_t cluster, uint32_t* free_c, uint32_t* free_m,
                        uint32_t n);
/* Cluster.GetResourceUtilization (cluster.go:46-63) over the live state: float32 sums in node
 * order divided by float32 totals (SetTotalResources, cluster.go:26-40). */
int mcs_resource_utilization(mcs_engine* eng, uint32_t cluster, float* core_util,
                             float* mem_util);

/* ---- the ClusterState record as a batched reduction ---------------------- */
/* pb.ClusterState (resource-channel.proto:27-34) that each cluster's Start stream
 * (trader_server.go:24-47) would send at simulated second t_s, rebuilt from the last FIFO/DELAY
 * run's placements: the counters after second t_s (jobs with start <= t_s < finish hold their
 * node), GetResourceUtilization over them (cluster.go:46-63, float32 in node order) and the Run
 * totals (cluster.go:26-40).  average_wait_time is not part of it (host side: mcs_read_delay_stats
 * at the end of a DELAY run, 0 under FIFO where "/delay" never feeds WaitTime). */
typedef struct mcs_cluster_state {
    float cores_utilization;
    float memory_utilization;
    uint32_t total_cpu;
    uint32_t total_memory;
    uint32_t running;   /* jobs holding resources at t_s */
    uint32_t t_s;
} mcs_cluster_state;

/* One gfx950 launch over every cluster (MCS_E_STATE after a trading run).  kernel_ms (may be
 * NULL) receives the launch's device time from HIP events on the engine stream. */
int mcs_cluster_states(mcs_engine* eng, uint32_t t_s, mcs_cluster_state* out, uint32_t n_clusters,
                       double* kernel_ms);

#ifdef __cplusplus
}
#endif
#endif /* MCS_H */
