/*
 * mcs_oracle_trade.h — CPU ORACLE of the trading configuration (C5).  TEST INFRASTRUCTURE ONLY:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * Pinning: the reference holds no tests or fixtures for borrow or trade.  The
 * restatement is pinned by hand-derived known-answer scenarios (tests/golden/kats_trade.json,
 * each step justified against the Go file:line it follows) and by two exact reductions: with
 * borrow and trader off it must reproduce or_fifo_run_batch bit for bit, and the trader alone
 * must leave every placement unchanged (under FIFO its contract is the zero contract).
 */
#ifndef MCS_ORACLE_TRADE_H
#define MCS_ORACLE_TRADE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    uint32_t borrow;             /* BorrowResources on every failed wait-head attempt */
    uint32_t trader;             /* per-cluster trader (RequestPolicyMonitor) */
    uint32_t period_s;           /* 10: trader.go:323 */
    uint32_t trade_ok_sleep_s;   /* 240: trader.go:297 */
    uint32_t trade_fail_sleep_s; /* 120: trader.go:300 */
    uint32_t lock_s;             /* 20: server.go:49 */
    uint32_t sample_period_s;    /* 5: trader_server.go:44 */
    uint32_t t_max;              /* stop after this tick even if work remains */
} or_trade_cfg;

typedef struct {
    uint32_t lender, borrower;
    uint64_t job; /* global job index (borrower's CSR range) */
    uint32_t node, start, finish, pad;
} or_lent_rec;

typedef struct {
    uint32_t t, requester;
    int32_t winner; /* responder that provided the virtual node, -1 when the trade failed */
    uint32_t approvals;
} or_trade_rec;

typedef struct {
    uint32_t virtual_nodes, decided, lent_pending, lent_peak; /* lent_peak: LentQueue high-water */
} or_trade_cluster_stats;

/* Lock-step run of C clusters (semantics in mcs_oracle_trade.c).  Own jobs: node >= 0 placed,
 * -2 borrowed (start = borrow tick, finish = 0xFFFFFFFF), -1 never decided before t_max.
 * Logs beyond their capacity are counted but not written. */
int or_trade_run(uint32_t C, const uint32_t* node_off, const uint32_t* cap_c, const uint32_t* cap_m,
                 const uint32_t* free_c, const uint32_t* free_m, const uint64_t* job_off,
                 const uint32_t* arrival, const uint32_t* dur, const uint32_t* cores,
                 const uint32_t* mem, const or_trade_cfg* cfg, int32_t* out_node,
                 uint32_t* out_start, uint32_t* out_finish, or_lent_rec* lent_log,
                 uint64_t lent_cap, uint64_t* n_lent, or_trade_rec* trade_log, uint64_t trade_cap,
                 uint64_t* n_trades, or_trade_cluster_stats* cstats, uint32_t* t_final);

/* ---- trading with DELAY schedulers (mcs_oracle_dtrade.c) ------------------- */
typedef struct {
    uint32_t period_s;           /* 10: trader.go:323 (0 = no traders: independent Delay loops) */
    uint32_t trade_ok_sleep_s;   /* 240: trader.go:297,316 */
    uint32_t trade_fail_sleep_s; /* 120: trader.go:300,319 */
    uint32_t lock_s;             /* 20: server.go:49 */
    uint32_t sample_period_s;    /* 5: trader_server.go:42 */
    uint32_t max_wait_s;         /* 10: scheduler.go:115 */
    uint32_t max_vnodes;         /* virtual nodes a cluster can receive (capacity of the arrays) */
    uint32_t t_max;              /* stop after this tick even if work remains */
} or_dtrade_cfg;

typedef struct {
    uint32_t t, requester;
    int32_t winner;     /* responder whose allocation succeeded, -1 = "couldn't acquire resources" */
    uint32_t approvals; /* approving responses pushed on the heap */
    uint32_t policy;    /* 0 = WaitTime (fast node), 1 = Utilization (small node) */
    uint32_t cores, mem, time_s; /* the contract */
    uint32_t failed;    /* popped approvals that failed (lock lost or allocation error) */
    uint32_t pad;
} or_dtrade_rec;

typedef struct { /* one Foreign job launched by AllocateVirtualNodeResources on a responder */
    uint32_t requester, responder, node, start, finish, pad;
    uint64_t c, m; /* uint(core_diff), uint(mem_diff) (cluster.go:116) */
} or_foreign_rec;

typedef struct {
    uint32_t virtual_nodes, decided, moved_l1, placed_l1;
    int64_t total_wait_ms, jobs_count;
} or_dtrade_cluster_stats;

/* Lock-step run of C DELAY clusters with traders.  vnode_c/vnode_m: [C][max_vnodes] capacities
 * of the virtual nodes received (may be NULL).  Foreign jobs are logged in execution order. */
int or_dtrade_run(uint32_t C, const uint32_t* node_off, const uint32_t* cap_c, const uint32_t* cap_m,
                  const uint32_t* free_c, const uint32_t* free_m, const uint64_t* job_off,
                  const uint32_t* arrival, const uint32_t* dur, const uint32_t* cores,
                  const uint32_t* mem, const or_dtrade_cfg* cfg, int32_t* out_node,
                  uint32_t* out_start, uint32_t* out_finish, or_dtrade_rec* trade_log,
                  uint64_t trade_cap, uint64_t* n_trades, or_foreign_rec* foreign_log,
                  uint64_t foreign_cap, uint64_t* n_foreign, uint32_t* vnode_c, uint32_t* vnode_m,
                  or_dtrade_cluster_stats* cstats, uint32_t* t_final);

#ifdef __cplusplus
}
#endif
#endif
