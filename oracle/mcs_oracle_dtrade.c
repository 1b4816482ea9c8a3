/*
 * mcs_oracle_dtrade.c — CPU ORACLE of the trading system with DELAY schedulers (LSDELAY,
 * DESIGN.md §11).  TEST INFRASTRUCTURE ONLY (see mcs_oracle.h for the rules).
 *
 * The reference's default scheduler policy is DELAY (pkg/scheduler/scheduler.go:116), and only
 * Delay fills Level1 (scheduler.go:353-359), the job list the trader sizes its contracts from
 * (ProvideJobs, pkg/scheduler/trader_server.go:69-94).  So this is where trades carry resources:
 * AllocateVirtualNodeResources launches Foreign jobs on the responder (cluster.go:87-125) and the
 * requester appends a virtual node with the contract's capacity (cluster.go:65-85).
 *
 * Lock-step serialization (all clusters share the clock T, seconds).  Tick T, in this order:
 *   A. every cluster runs one Delay iteration at T (exactly oracle/mcs_oracle_delay.c's tick:
 *      releases due, "/delay" arrivals, the Level1 pass with its skip (D6), the Level0 head and
 *      its MaxWaitTime move).  First fit covers the physical nodes, then the virtual ones in the
 *      order they were received (Cluster.Nodes, cluster.go:79).
 *   C. at T % sample_period_s == 0 every cluster samples GetResourceUtilization (float32 over all
 *      Nodes, physical and virtual, divided by the totals SetTotalResources fixed at Run,
 *      cluster.go:46-63) and WaitTime.GetAverage() (float64 TotalTime / JobsCount,
 *      scheduler.go:56-63): the clusterState its trader holds (trader_server.go:24-47).
 *   D. trader rounds due at T, in cluster index order.  RequestPolicyMonitor (trader.go:280-325)
 *      snapshots cs, then walks [WaitTime(600000 ms), Utilization(0.8, 0.8)] (trader.go:55-62);
 *      a broken policy trades and then SLEEPS (240 s after success, 120 s after failure) before
 *      the loop moves on to the next policy with the same stale cs; after the last policy it
 *      sleeps 10 s.  So each trader is a two-stage machine: stage 0 (WaitTime) at the round's
 *      start, stage 1 (Utilization) at the same tick or after the post-trade sleep.
 *      Contract: calculateFastNodeSize (WaitTime) or calculateSmallNodeSize (Utilization) over
 *      the requester's Level1 at T (or_contract_fast/small, ProvideJobs batches padded, D9).
 *      Trade (trader.go:193-278): RequestResource to every other trader in index order
 *      (pkg/trader/server.go:31-61: refuse while locked; else ApproveTrade on the responder's
 *      sample and lock 20 s even when not approving), container/heap order over the approvals,
 *      then ApproveContract on each popped responder (server.go:63-85): a lock that no longer
 *      matches is DeadlineExceeded; otherwise AllocateVirtualNodeResources runs on the
 *      responder (or_allocate_virtual_node: Foreign jobs committed on its nodes, released after
 *      the contract time) and the lock resets either way; an allocation error moves on to the
 *      next approval; success appends the virtual node {contract cores, memory} to the
 *      requester (AddVirtualNode) and ends the trade.
 * Node counters are uint64 like Go's uint: Foreign jobs routinely wrap a node's availability
 * (cluster.go:116 commits |req - avail|), and the wrapped node then fits anything until they end.
 * float32/float64 conversions of wrapped values follow Go (convert the uint64).
 *
 * No fast-forward across queued work: every tick with a queued job runs (the Delay loop wakes
 * every second anyway).  When no cluster has a queued job the clock jumps to the next arrival,
 * sample tick or trader round.  The run stops when every job is placed or at t_max.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "mcs_oracle.h"
#include "mcs_oracle_trade.h"

typedef struct {
    uint32_t finish, node;
    uint64_t c, m;
} dt_run;

typedef struct {
    uint32_t n, n_phys, cap_nodes;
    uint64_t *cap_c, *cap_m, *fc, *fm;
    uint32_t total_c, total_m;
    uint64_t j0, J;
    uint64_t next_arrival, l0_head;
    uint64_t* l1;
    uint64_t l1_len;
    int64_t* jobs_map;
    int64_t total, count;
    dt_run* run;
    uint64_t nrun, caprun;
    uint64_t decided;
    uint32_t moved, placed_l1;
    /* trader */
    float cu, mu;
    double avgw;
    float cs_cu, cs_mu;
    double cs_avgw;
    uint32_t stage, next_due;
    uint32_t lock_id, lock_until, next_id;
} dt_cluster;

static void dt_push(dt_cluster* k, uint32_t finish, uint32_t node, uint64_t c, uint64_t m) {
    if (k->nrun == k->caprun) {
        k->caprun = k->caprun ? 2 * k->caprun : 64;
        k->run = (dt_run*)realloc(k->run, k->caprun * sizeof(dt_run));
    }
    dt_run r = {finish, node, c, m};
    k->run[k->nrun++] = r;
}

static void dt_release(dt_cluster* k, uint32_t T) {
    for (uint64_t i = 0; i < k->nrun;) {
        if (k->run[i].finish <= T) { /* cluster.go:153-157 */
            k->fc[k->run[i].node] += k->run[i].c;
            k->fm[k->run[i].node] += k->run[i].m;
            k->run[i] = k->run[--k->nrun];
        } else {
            ++i;
        }
    }
}

/* Node.RunJob (cluster.go:141-161): commit now, release after dur (0: at once, before the next
 * scheduler step). */
static void dt_run_job(dt_cluster* k, uint32_t node, uint64_t c, uint64_t m, uint32_t T, uint32_t dur) {
    k->fc[node] -= c;
    k->fm[node] -= m;
    if (dur == 0) {
        k->fc[node] += c;
        k->fm[node] += m;
        return;
    }
    dt_push(k, T + dur, node, c, m);
}

static void dt_touch(dt_cluster* k, uint64_t j, uint32_t T, const uint32_t* arrival) {
    k->total -= k->jobs_map[j];
    k->jobs_map[j] = (int64_t)(T - arrival[k->j0 + j]) * 1000;
    k->total += k->jobs_map[j];
}

/* one Delay iteration (scheduler.go:298-369) at T; returns 1 if a job was placed or moved */
static void dt_delay_tick(dt_cluster* k, uint32_t T, uint32_t max_wait, const uint32_t* arrival,
                          const uint32_t* dur, const uint32_t* cores, const uint32_t* mem,
                          int32_t* out_node, uint32_t* out_start, uint32_t* out_finish) {
    dt_release(k, T);
    while (k->next_arrival < k->J && arrival[k->j0 + k->next_arrival] <= T) {
        k->jobs_map[k->next_arrival] = 0;
        ++k->count;
        ++k->next_arrival;
    }
    for (uint64_t i = 0; i < k->l1_len; i++) {
        const uint64_t j = k->l1[i], g = k->j0 + j;
        const int nd = or_schedule_job(k->n, k->fc, k->fm, cores[g], mem[g]);
        dt_touch(k, j, T, arrival);
        if (nd >= 0) {
            dt_run_job(k, (uint32_t)nd, cores[g], mem[g], T, dur[g]);
            out_node[g] = nd;
            out_start[g] = T;
            out_finish[g] = T + dur[g];
            k->jobs_map[j] = 0;
            memmove(k->l1 + i, k->l1 + i + 1, sizeof(uint64_t) * (k->l1_len - i - 1));
            --k->l1_len;
            ++k->decided;
            ++k->placed_l1;
        }
    }
    if (k->next_arrival > k->l0_head) {
        const uint64_t j = k->l0_head, g = k->j0 + j;
        const int nd = or_schedule_job(k->n, k->fc, k->fm, cores[g], mem[g]);
        dt_touch(k, j, T, arrival);
        if (nd >= 0) {
            dt_run_job(k, (uint32_t)nd, cores[g], mem[g], T, dur[g]);
            out_node[g] = nd;
            out_start[g] = T;
            out_finish[g] = T + dur[g];
            k->jobs_map[j] = 0;
            ++k->l0_head;
            ++k->decided;
        } else if (T - arrival[g] >= max_wait) {
            k->l1[k->l1_len++] = j;
            ++k->l0_head;
            ++k->moved;
        }
    }
}

/* GetResourceUtilization (cluster.go:46-63) over every node, physical and virtual. */
static void dt_sample(dt_cluster* k) {
    float c = 0.0f, m = 0.0f;
    for (uint32_t i = 0; i < k->n; ++i) {
        c += ((float)k->cap_c[i] - (float)k->fc[i]);
        m += ((float)k->cap_m[i] - (float)k->fm[i]);
    }
    k->cu = c / (float)k->total_c;
    k->mu = m / (float)k->total_m;
    k->avgw = k->count != 0 ? (double)k->total / (double)k->count : 0.0; /* GetAverage */
}

/* Go's float64 -> uint conversion on amd64: or_go_f64_to_u64 (mcs_oracle.h) */
#define go_f64_to_u64 or_go_f64_to_u64

/* AllocateVirtualNodeResources (cluster.go:87-125) on uint64 counters, Foreign jobs released
 * after dur_s.  Returns 0 on success, 1 for "couldn't schedule enough resources". */
static int dt_allocate(dt_cluster* R, uint32_t rq, uint32_t rs, uint32_t req_c, uint32_t req_m, uint32_t dur_s,
                       uint32_t T, or_foreign_rec* flog, uint64_t fcap, uint64_t* nf) {
    for (uint32_t i = 0; i < R->n; ++i) {
        if (req_m == 0 && req_c == 0) break; /* :90-92 (uint32: <= 0 is == 0) */
        double mem_diff = 0.0, core_diff = 0.0;
        if (req_m > 0) mem_diff = fabs((double)req_m - (double)R->fm[i]);  /* :96-98 */
        if (req_c > 0) core_diff = fabs((double)req_c - (double)R->fc[i]); /* :100-102 */
        if (mem_diff > (double)req_m)
            req_m = 0;
        else
            req_m -= (uint32_t)mem_diff; /* uint32(float64) of a value <= req_m: exact */
        if (core_diff > (double)req_c)
            req_c = 0;
        else
            req_c -= (uint32_t)core_diff;
        /* go node.RunJob(Job{CoresNeeded: uint(core_diff), MemoryNeeded: uint(mem_diff),
         * Duration: req.Time}) (:116) */
        const uint64_t fc = go_f64_to_u64(core_diff), fm = go_f64_to_u64(mem_diff);
        if (*nf < fcap) {
            flog[*nf].requester = rq;
            flog[*nf].responder = rs;
            flog[*nf].pad = 0;
            flog[*nf].node = i;
            flog[*nf].start = T;
            flog[*nf].finish = T + dur_s;
            flog[*nf].c = fc;
            flog[*nf].m = fm;
        }
        ++*nf;
        dt_run_job(R, i, fc, fm, T, dur_s);
    }
    return (req_c > 0 || req_m > 0) ? 1 : 0; /* :119-121 */
}

int or_dtrade_run(uint32_t C, const uint32_t* node_off, const uint32_t* cap_c, const uint32_t* cap_m,
                  const uint32_t* free_c, const uint32_t* free_m, const uint64_t* job_off,
                  const uint32_t* arrival, const uint32_t* dur, const uint32_t* cores,
                  const uint32_t* mem, const or_dtrade_cfg* cfg, int32_t* out_node,
                  uint32_t* out_start, uint32_t* out_finish, or_dtrade_rec* trade_log,
                  uint64_t trade_cap, uint64_t* n_trades, or_foreign_rec* foreign_log,
                  uint64_t foreign_cap, uint64_t* n_foreign, uint32_t* vnode_c, uint32_t* vnode_m,
                  or_dtrade_cluster_stats* cstats, uint32_t* t_final) {
    dt_cluster* cl = (dt_cluster*)calloc(C ? C : 1, sizeof(dt_cluster));
    const uint64_t total_jobs = job_off[C];
    for (uint64_t j = 0; j < total_jobs; ++j) {
        out_node[j] = -1;
        out_start[j] = 0xFFFFFFFFu;
        out_finish[j] = 0xFFFFFFFFu;
    }
    const uint32_t vmax = cfg->max_vnodes;
    for (uint32_t c = 0; c < C; ++c) {
        dt_cluster* k = &cl[c];
        const uint32_t a = node_off[c];
        k->n = k->n_phys = node_off[c + 1] - a;
        k->cap_nodes = k->n + vmax;
        const size_t nb = 8 * (size_t)(k->cap_nodes ? k->cap_nodes : 1);
        k->cap_c = (uint64_t*)malloc(nb);
        k->cap_m = (uint64_t*)malloc(nb);
        k->fc = (uint64_t*)malloc(nb);
        k->fm = (uint64_t*)malloc(nb);
        for (uint32_t i = 0; i < k->n; ++i) {
            k->cap_c[i] = cap_c[a + i];
            k->cap_m[i] = cap_m[a + i];
            k->fc[i] = free_c[a + i];
            k->fm[i] = free_m[a + i];
            k->total_c += cap_c[a + i]; /* SetTotalResources at Run, never updated (:79) */
            k->total_m += cap_m[a + i];
        }
        k->j0 = job_off[c];
        k->J = job_off[c + 1] - job_off[c];
        k->l1 = (uint64_t*)malloc(sizeof(uint64_t) * (k->J ? k->J : 1));
        k->jobs_map = (int64_t*)calloc(k->J ? k->J : 1, sizeof(int64_t));
        k->next_id = 1; /* s.id = rand.Uint32() (server.go:26), seeded deterministically */
    }
    uint32_t* appr = (uint32_t*)malloc(sizeof(uint32_t) * (C ? C : 1));
    uint32_t* appr_id = (uint32_t*)malloc(sizeof(uint32_t) * (C ? C : 1));
    float* prices = (float*)malloc(sizeof(float) * (C ? C : 1));
    uint32_t* order = (uint32_t*)malloc(sizeof(uint32_t) * (C ? C : 1));
    uint32_t* lc = (uint32_t*)malloc(sizeof(uint32_t) * (total_jobs ? total_jobs : 1));
    uint32_t* lm = (uint32_t*)malloc(sizeof(uint32_t) * (total_jobs ? total_jobs : 1));
    uint32_t* ld = (uint32_t*)malloc(sizeof(uint32_t) * (total_jobs ? total_jobs : 1));
    uint64_t nt = 0, nf = 0;
    uint32_t T = 0;

    for (;;) {
        /* ---- A. one Delay iteration per cluster ---- */
        for (uint32_t c = 0; c < C; ++c)
            dt_delay_tick(&cl[c], T, cfg->max_wait_s, arrival, dur, cores, mem, out_node, out_start,
                          out_finish);
        /* ---- C. state samples ---- */
        if (T % cfg->sample_period_s == 0)
            for (uint32_t c = 0; c < C; ++c) dt_sample(&cl[c]);
        /* ---- D. trader rounds (period_s == 0: no traders) ---- */
        for (uint32_t q = 0; q < C && cfg->period_s; ++q) {
            dt_cluster* Q = &cl[q];
            while (Q->next_due <= T) {
                if (Q->stage == 0) { /* cs := getState() at the start of the monitor pass */
                    Q->cs_cu = Q->cu;
                    Q->cs_mu = Q->mu;
                    Q->cs_avgw = Q->avgw;
                }
                const uint32_t pol = Q->stage;
                const int broken = pol == 0 ? (Q->cs_avgw > 600000.0)                       /* :137-139 */
                                            : (Q->cs_cu > 0.8f || Q->cs_mu > 0.8f); /* :127-130 */
                Q->stage = pol == 0 ? 1u : 0u;
                if (!broken) {
                    if (pol == 1) Q->next_due = T + cfg->period_s; /* time.Sleep(10 s), :323 */
                    continue;
                }
                /* calculateContractRequest over the Level1 copy (GetLevel1, scheduler.go:204) */
                for (uint64_t i = 0; i < Q->l1_len; ++i) {
                    const uint64_t g = Q->j0 + Q->l1[i];
                    lc[i] = cores[g];
                    lm[i] = mem[g];
                    ld[i] = dur[g];
                }
                uint32_t kc, km;
                int64_t kt;
                float kp;
                if (pol == 0)
                    or_contract_fast((uint32_t)Q->l1_len, lc, lm, ld, &kc, &km, &kt, &kp);
                else
                    or_contract_small((uint32_t)Q->l1_len, lc, lm, ld, &kc, &km, &kt, &kp);
                const uint32_t ksec = (uint32_t)(kt / 1000000000LL); /* whole seconds (D8) */
                uint32_t napp = 0;
                for (uint32_t r = 0; r < C; ++r) {
                    if (r == q) continue; /* trader.go:212 */
                    dt_cluster* R = &cl[r];
                    if (R->lock_id != 0 && T >= R->lock_until) R->lock_id = 0; /* server.go:48-57 */
                    if (R->lock_id != 0) continue;                             /* :35-40 */
                    const int ok = or_approve_trade(R->total_c, R->total_m, R->cu, R->mu, kc, km, kt, kp);
                    R->lock_id = R->next_id++; /* :44-46, even when not approving */
                    R->lock_until = T + cfg->lock_s;
                    if (ok) {
                        appr[napp] = r;
                        appr_id[napp] = R->lock_id;
                        prices[napp] = kp; /* every response echoes the request's price (:44) */
                        ++napp;
                    }
                }
                int winner = -1;
                uint32_t failed = 0;
                if (napp) {
                    or_heap_order(napp, prices, order);
                    for (uint32_t i = 0; i < napp && winner < 0; ++i) {
                        dt_cluster* R = &cl[appr[order[i]]];
                        if (R->lock_id != appr_id[order[i]]) { /* DeadlineExceeded (:69-71) */
                            ++failed;
                            continue;
                        }
                        const int err = dt_allocate(R, q, appr[order[i]], kc, km, ksec, T, foreign_log, foreign_cap, &nf);
                        R->lock_id = 0; /* currentContract reset (:83) */
                        if (err) {
                            ++failed;
                            continue;
                        }
                        winner = (int)appr[order[i]];
                        if (Q->n < Q->cap_nodes) { /* AddVirtualNode (cluster.go:65-85) */
                            if (vnode_c) {
                                vnode_c[(uint64_t)q * vmax + (Q->n - Q->n_phys)] = kc;
                                vnode_m[(uint64_t)q * vmax + (Q->n - Q->n_phys)] = km;
                            }
                            Q->cap_c[Q->n] = Q->fc[Q->n] = kc;
                            Q->cap_m[Q->n] = Q->fm[Q->n] = km;
                            ++Q->n;
                        }
                    }
                }
                if (nt < trade_cap) {
                    or_dtrade_rec* tr = &trade_log[nt];
                    tr->t = T;
                    tr->requester = q;
                    tr->winner = winner;
                    tr->approvals = napp;
                    tr->policy = pol;
                    tr->cores = kc;
                    tr->mem = km;
                    tr->time_s = ksec;
                    tr->failed = failed;
                    tr->pad = 0;
                }
                ++nt;
                Q->next_due = T + (winner >= 0 ? cfg->trade_ok_sleep_s : cfg->trade_fail_sleep_s) +
                              (pol == 1 ? cfg->period_s : 0u);
            }
        }
        /* ---- termination and the next tick ---- */
        int all_done = 1, queued = 0;
        uint32_t next = T + cfg->sample_period_s - T % cfg->sample_period_s;
        for (uint32_t c = 0; c < C; ++c) {
            dt_cluster* k = &cl[c];
            if (k->decided < k->J) all_done = 0;
            if (k->l1_len > 0 || k->next_arrival > k->l0_head) queued = 1;
            if (k->next_arrival < k->J && arrival[k->j0 + k->next_arrival] < next)
                next = arrival[k->j0 + k->next_arrival];
            if (cfg->period_s && k->next_due < next) next = k->next_due;
        }
        if (all_done || T >= cfg->t_max) break;
        T = (queued || next <= T + 1u) ? T + 1u : next;
    }
    for (uint32_t c = 0; c < C; ++c) {
        dt_cluster* k = &cl[c];
        if (cstats) {
            cstats[c].virtual_nodes = k->n - k->n_phys;
            cstats[c].decided = (uint32_t)k->decided;
            cstats[c].moved_l1 = k->moved;
            cstats[c].placed_l1 = k->placed_l1;
            cstats[c].total_wait_ms = k->total;
            cstats[c].jobs_count = k->count;
        }
        free(k->cap_c);
        free(k->cap_m);
        free(k->fc);
        free(k->fm);
        free(k->l1);
        free(k->jobs_map);
        free(k->run);
    }
    if (n_trades) *n_trades = nt;
    if (n_foreign) *n_foreign = nf;
    if (t_final) *t_final = T;
    free(cl);
    free(appr);
    free(appr_id);
    free(prices);
    free(order);
    free(lc);
    free(lm);
    free(ld);
    return 0;
}
