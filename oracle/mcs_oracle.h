/*
 * mcs_oracle.h — CPU ORACLE for the MI355X engine.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library, and
 * only as the checker (or the timed CPU baseline), never as the product path.
 *
 * It is a deliberately naive single-threaded restatement of the reference Go code
 * (hamzalsheikh/multi-cluster-simulator @ 2024-10-16), following it function by function; every
 * function cites the reference file:line it restates.  The semantics are SFIFO (SURVEY.md
 * Appendix A): the Go FIFO loop with each goroutine step serialized, deviations D1-D9.
 *
 * PINNING: the reference has no tests, fixtures or golden vectors, and its Go toolchain and module
 * cache are absent here, so it cannot be built or run.  This oracle is pinned by the
 * hand-derived known-answer tests KAT1-KAT9 of SURVEY Appendix B (traced from the reference
 * source), committed as tests/golden/kats.json.  Anything those KATs do not cover is
 * "parity unpinned" against the Go binary itself.
 */
#ifndef MCS_ORACLE_H
#define MCS_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Go's float64 -> uint conversion on amd64 (CVTTSD2SQ below 2^63; above, CVTTSD2SQ of x - 2^63 xor
 * 2^63, whose integer-indefinite result makes anything >= 2^64 convert to 0).  cluster.go:116 converts
 * |req - free| this way, and |req - free| reaches 2^64 once a uint counter has wrapped: a plain C cast
 * of such a value is undefined behaviour (found by the UBSan self-test, tests/test_oracle_sanitize.py). */
static inline uint64_t or_go_f64_to_u64(double x) {
    const double two63 = 9223372036854775808.0;
    if (x < two63) return (uint64_t)(int64_t)x;
    const double y = x - two63;
    if (y >= two63) return 0;
    return (uint64_t)(int64_t)y ^ 0x8000000000000000ull;
}

typedef struct or_stats {
    uint32_t t_end;
    uint32_t placed;
    uint32_t waited;
    uint32_t peak_running;
    uint32_t flags; /* 1 = deadlock */
    uint32_t pad;
    uint64_t ticks; /* loop iterations executed (literal mode: one per simulated second step) */
} or_stats;

/* FIFO run of ONE cluster.  Node arrays are the JSON order; jobs sorted by arrival.
 * literal != 0 advances the clock one second per sleep exactly as the Go loop does
 * (scheduler.go:250,289,294); literal == 0 uses the fast-forward of Appendix A.3.
 * Outputs: node (-1 unplaced), start, finish (0xFFFFFFFF unplaced).  Returns 0. */
int or_fifo_run(uint32_t n_nodes, const uint32_t* cap_c, const uint32_t* cap_m,
                const uint32_t* free_c, const uint32_t* free_m, uint64_t n_jobs,
                const uint32_t* arrival, const uint32_t* dur, const uint32_t* cores,
                const uint32_t* mem, int literal, int32_t* out_node, uint32_t* out_start,
                uint32_t* out_finish, or_stats* st);

/* Many clusters (CSR offsets like mcs.h); n_threads > 1 uses OpenMP over clusters. */
int or_fifo_run_batch(uint32_t n_clusters, const uint32_t* node_off, const uint32_t* cap_c,
                      const uint32_t* cap_m, const uint32_t* free_c, const uint32_t* free_m,
                      const uint64_t* job_off, const uint32_t* arrival, const uint32_t* dur,
                      const uint32_t* cores, const uint32_t* mem, int n_threads,
                      int32_t* out_node, uint32_t* out_start, uint32_t* out_finish,
                      or_stats* st);

/* Scheduler.ScheduleJob first-fit (scheduler.go:127-139): index or -1 (uint64 node counters). */
int or_schedule_job(uint32_t n, const uint64_t* free_c, const uint64_t* free_m, uint64_t c,
                    uint64_t m);
/* Scheduler.Lend (scheduler.go:194-202): 1 when some node has strictly more of both. */
int or_lend(uint32_t n, const uint64_t* free_c, const uint64_t* free_m, uint64_t c, uint64_t m);

/* Cluster.GetResourceUtilization (cluster.go:46-63), float32 accumulation in node order. */
void or_resource_utilization(uint32_t n, const uint64_t* cap_c, const uint64_t* cap_m,
                             const uint64_t* free_c, const uint64_t* free_m, uint32_t total_c,
                             uint32_t total_m, float* cu, float* mu);

/* Trader.ApproveTrade (trader.go:141-167) with newTrader's approvePolicy (trader.go:47-52). */
int or_approve_trade(uint32_t total_c, uint32_t total_m, float core_util, float mem_util,
                     uint32_t req_cores, uint32_t req_mem, int64_t req_time_ns, float req_price);

/* Go container/heap over contractResHeap (trader.go:169-191): push prices in order, then pop
 * everything; writes the pop order (indices into prices[]). */
void or_heap_order(uint32_t n, const float* prices, uint32_t* order);

/* Cluster.AllocateVirtualNodeResources (cluster.go:87-125) on uint64 node counters.  Foreign jobs
 * launched (go node.RunJob, cluster.go:116) are committed in place and reported (node, c, m);
 * returns 0 on success, 1 for "couldn't schedule enough resources" (cluster.go:119-121). */
int or_allocate_virtual_node(uint32_t n, uint64_t* free_c, uint64_t* free_m, uint32_t req_c,
                             uint32_t req_m, uint32_t* n_foreign, uint32_t* f_node, uint64_t* f_c,
                             uint64_t* f_m);

/* calculateFastNodeSize (scheduler_client.go:126-170) / calculateSmallNodeSize (201-289) over a
 * Level1 list delivered in ProvideJobs batches of 20 padded with zero jobs (trader_server.go:75-91,
 * D9).  MaximimumCoreCost/MemoryCost = 0 and Budget = -1 as in newTrader (trader.go:34-35,53).
 * Outputs cores, mem, time (ns), price. */
void or_contract_fast(uint32_t n, const uint32_t* c, const uint32_t* m, const uint32_t* dur_s,
                      uint32_t* oc, uint32_t* om, int64_t* otime_ns, float* oprice);
void or_contract_small(uint32_t n, const uint32_t* c, const uint32_t* m, const uint32_t* dur_s,
                       uint32_t* oc, uint32_t* om, int64_t* otime_ns, float* oprice);

/* ---- DELAY policy (mcs_oracle_delay.c) ------------------------------------------------------- */
typedef struct or_delay_stats {
    uint32_t t_end;
    uint32_t placed;
    uint32_t moved_l1;     /* Level0 -> Level1 moves (scheduler.go:353-359) */
    uint32_t placed_l1;    /* placements from the Level1 pass (scheduler.go:302-329) */
    uint32_t peak_l1;      /* peak len(Level1) */
    uint32_t peak_running;
    uint32_t flags;        /* 1 = Level1 jobs that can never fit; 4 = clock wrap */
    uint32_t l1_left;      /* len(Level1) at the end (the never-fitting jobs) */
    int64_t total_wait_ms; /* WaitTime.TotalTime at t_end (scheduler.go:48-54) */
    int64_t jobs_count;    /* WaitTime.JobsCount (server.go:72) */
    uint64_t ticks;        /* Delay iterations (literal and fast-forward count the same) */
} or_delay_stats;

/* Scheduler.Delay (scheduler.go:298-369) over one cluster, SDELAY semantics (see
 * mcs_oracle_delay.c).  max_wait_s = Policy.MaxWaitTime (10 s, scheduler.go:115). */
int or_delay_run(uint32_t n_nodes, const uint32_t* free_c, const uint32_t* free_m, uint64_t n_jobs,
                 const uint32_t* arrival, const uint32_t* dur, const uint32_t* cores,
                 const uint32_t* mem, uint32_t max_wait_s, int literal, int32_t* out_node,
                 uint32_t* out_start, uint32_t* out_finish, or_delay_stats* st);
int or_delay_run_batch(uint32_t n_clusters, const uint32_t* node_off, const uint32_t* free_c,
                       const uint32_t* free_m, const uint64_t* job_off, const uint32_t* arrival,
                       const uint32_t* dur, const uint32_t* cores, const uint32_t* mem,
                       uint32_t max_wait_s, int n_threads, int32_t* out_node, uint32_t* out_start,
                       uint32_t* out_finish, or_delay_stats* st);

#ifdef __cplusplus
}
#endif
#endif
