/*
 * mcs_oracle_trade.c — CPU ORACLE of the trading configuration (C5): many FIFO clusters in
 * lock-step with the cross-cluster borrow protocol and the per-cluster trader.  TEST
 * INFRASTRUCTURE ONLY (see mcs_oracle.h).
 *
 * Lock-step serialized semantics (LSFIFO; SURVEY §8 a9, a11-a16, e).  All clusters
 * share the clock T (seconds).  Tick T, in this order:
 *   A. every cluster runs its Fifo loop at T (pkg/scheduler/scheduler.go:216-296): releases due,
 *      arrivals queued, ready-queue decisions until one ends the tick — a wait-head attempt, a
 *      lent-queue attempt or an idle sleep (each followed by time.Sleep(1 s)).  A failed
 *      wait-head attempt issues a borrow request (BorrowResources, server.go:160-248).
 *   B. borrow exchange, requests in borrower index order: every other cluster, in index order,
 *      runs Lend on its state after A (strict '>', scheduler.go:194-202) and, when it can,
 *      appends the job to its LentQueue ("/borrow" handler, server.go:80-113; every acceptor
 *      keeps a copy — the cancel is commented out, server.go:232-237).  A borrower with at least
 *      one acceptance moves the head to its BorrowedQueue (scheduler.go:237-242).
 *   C. at T % 5 == 0 every cluster samples GetResourceUtilization (cluster.go:46-63), the value
 *      its trader's clusterState holds (trader_server.go:24-47, scheduler_client.go:14-47).
 *   D. traders due at T, in cluster index order (RequestPolicyMonitor, trader.go:280-325):
 *      policies [WaitTime, Utilization]; WaitTime never breaks under FIFO (the wait-time stats are
 *      only fed by /delay, server.go:53-78); Utilization breaks when cu > 0.8f || mu > 0.8f and
 *      trades a small-node contract, which is the ZERO contract under FIFO (Level1 is only filled
 *      by Delay; scheduler_client.go:201-289 over an empty stream).  Trade (trader.go:193-278):
 *      RequestResource to every other trader in index order (server.go:31-61: refuse while
 *      locked, else ApproveTrade on the responder's sample and lock it for 20 s even when not
 *      approving), heap order over approvals (Go container/heap), ApproveContract on the first
 *      whose lock still matches (server.go:63-85) -> AllocateVirtualNodeResources of the zero
 *      request (breaks at once, cluster.go:90-92) and AddVirtualNode of a 0-core/0-memory node on
 *      the requester (cluster.go:65-85).  Next evaluation at T + 10 s, plus 240 s after a
 *      successful trade or 120 s after a failed one.
 * Lent jobs run on the lender only when its wait and ready queues are empty (scheduler.go:
 * 277-290), first fit with '>=', and are released like any job (their ReturnToBorrower only
 * empties the borrower's BorrowedQueue, no placement effect).
 */
#include <stdlib.h>
#include <string.h>

#include "mcs_oracle.h"
#include "mcs_oracle_trade.h"

typedef struct {
    uint32_t finish, node;
    uint64_t c, m;
} tr_run;

typedef struct {
    uint32_t borrower;
    uint64_t job; /* global job index */
} tr_lent;

typedef struct {
    /* node state (uint64 like Go uint) */
    uint32_t n;
    uint64_t *cap_c, *cap_m, *fc, *fm;
    uint32_t total_c, total_m; /* SetTotalResources: uint32 sums at Run */
    uint32_t virtual_nodes;    /* zero-capacity nodes appended by trades */
    /* queues */
    uint64_t j0, J;            /* own jobs [j0, j0+J) */
    uint64_t next_arrival;     /* local index */
    uint64_t rq_head, rq_tail; /* ready queue: local indices [rq_head, rq_tail) */
    int has_w;
    uint64_t w;                /* local index of the wait head */
    tr_lent* lq;
    uint64_t lq_head, lq_len, lq_cap, lq_peak;
    tr_run* run;
    uint64_t nrun, caprun;
    uint32_t minf;             /* earliest finish among run[] (0xFFFFFFFF when empty) */
    uint64_t decided;          /* own jobs placed or borrowed */
    /* trader */
    float cu, mu;              /* latest utilization sample */
    uint32_t lock_id, lock_until;
    uint32_t next_id;
    uint32_t next_due;
} tr_cluster;

static void tr_push_run(tr_cluster* cl, tr_run r) {
    if (cl->nrun == cl->caprun) {
        cl->caprun = cl->caprun ? 2 * cl->caprun : 64;
        cl->run = (tr_run*)realloc(cl->run, cl->caprun * sizeof(tr_run));
    }
    cl->run[cl->nrun++] = r;
    if (r.finish < cl->minf) cl->minf = r.finish;
}

static void tr_release(tr_cluster* cl, uint32_t T) {
    if (cl->minf > T) return;
    uint32_t mf = 0xFFFFFFFFu;
    for (uint64_t i = 0; i < cl->nrun;) {
        if (cl->run[i].finish <= T) { /* cluster.go:153-157 */
            cl->fc[cl->run[i].node] += cl->run[i].c;
            cl->fm[cl->run[i].node] += cl->run[i].m;
            cl->run[i] = cl->run[--cl->nrun];
        } else {
            if (cl->run[i].finish < mf) mf = cl->run[i].finish;
            ++i;
        }
    }
    cl->minf = mf;
}

static int tr_first_fit(const tr_cluster* cl, uint64_t c, uint64_t m) {
    /* virtual nodes (0 cores, 0 memory) follow the physical ones in Cluster.Nodes (cluster.go:79) */
    for (uint32_t i = 0; i < cl->n; ++i)
        if (cl->fc[i] >= c && cl->fm[i] >= m) return (int)i;
    if (c == 0 && m == 0 && cl->virtual_nodes > 0) return (int)cl->n; /* unreachable: node 0 fits first */
    return -1;
}

static int tr_lend(const tr_cluster* cl, uint64_t c, uint64_t m) {
    for (uint32_t i = 0; i < cl->n; ++i)
        if (cl->fc[i] > c && cl->fm[i] > m) return 1; /* scheduler.go:197 */
    return 0; /* virtual nodes have 0 free: never strictly greater */
}

static void tr_sample(tr_cluster* cl) {
    float c = 0.0f, m = 0.0f;
    for (uint32_t i = 0; i < cl->n; ++i) {
        c += ((float)cl->cap_c[i] - (float)cl->fc[i]);
        m += ((float)cl->cap_m[i] - (float)cl->fm[i]);
    }
    /* virtual nodes: float32(0) - float32(0) adds +0.0f, no change */
    cl->cu = c / (float)cl->total_c;
    cl->mu = m / (float)cl->total_m;
}

int or_trade_run(uint32_t C, const uint32_t* node_off, const uint32_t* cap_c, const uint32_t* cap_m,
                 const uint32_t* free_c, const uint32_t* free_m, const uint64_t* job_off,
                 const uint32_t* arrival, const uint32_t* dur, const uint32_t* cores,
                 const uint32_t* mem, const or_trade_cfg* cfg, int32_t* out_node,
                 uint32_t* out_start, uint32_t* out_finish, or_lent_rec* lent_log,
                 uint64_t lent_cap, uint64_t* n_lent, or_trade_rec* trade_log, uint64_t trade_cap,
                 uint64_t* n_trades, or_trade_cluster_stats* cstats, uint32_t* t_final) {
    tr_cluster* cl = (tr_cluster*)calloc(C ? C : 1, sizeof(tr_cluster));
    uint64_t total_jobs = job_off[C];
    for (uint64_t j = 0; j < total_jobs; ++j) {
        out_node[j] = -1;
        out_start[j] = 0xFFFFFFFFu;
        out_finish[j] = 0xFFFFFFFFu;
    }
    for (uint32_t c = 0; c < C; ++c) {
        tr_cluster* k = &cl[c];
        const uint32_t a = node_off[c];
        k->n = node_off[c + 1] - a;
        k->cap_c = (uint64_t*)malloc(8 * (k->n ? k->n : 1));
        k->cap_m = (uint64_t*)malloc(8 * (k->n ? k->n : 1));
        k->fc = (uint64_t*)malloc(8 * (k->n ? k->n : 1));
        k->fm = (uint64_t*)malloc(8 * (k->n ? k->n : 1));
        for (uint32_t i = 0; i < k->n; ++i) {
            k->cap_c[i] = cap_c[a + i];
            k->cap_m[i] = cap_m[a + i];
            k->fc[i] = free_c[a + i];
            k->fm[i] = free_m[a + i];
            k->total_c += cap_c[a + i];
            k->total_m += cap_m[a + i];
        }
        k->j0 = job_off[c];
        k->J = job_off[c + 1] - job_off[c];
        k->minf = 0xFFFFFFFFu;
        k->next_id = 1; /* s.id = rand.Uint32() (server.go:26), seeded deterministically */
        k->next_due = 0;
    }
    uint64_t nl = 0, nt = 0;
    uint32_t T = 0;
    int32_t* req = (int32_t*)malloc(sizeof(int32_t) * (C ? C : 1));
    uint32_t* appr = (uint32_t*)malloc(sizeof(uint32_t) * (C ? C : 1));
    uint32_t* appr_id = (uint32_t*)malloc(sizeof(uint32_t) * (C ? C : 1));
    float* prices = (float*)malloc(sizeof(float) * (C ? C : 1));
    uint32_t* order = (uint32_t*)malloc(sizeof(uint32_t) * (C ? C : 1));

    for (;;) {
        /* ---- A. scheduler step of every cluster at T ---- */
        for (uint32_t c = 0; c < C; ++c) {
            tr_cluster* k = &cl[c];
            req[c] = -1;
            tr_release(k, T);
            while (k->next_arrival < k->J && arrival[k->j0 + k->next_arrival] <= T)
                k->rq_tail = ++k->next_arrival;
            for (;;) {
                if (k->has_w) { /* scheduler.go:219-251 */
                    const uint64_t g = k->j0 + k->w;
                    const int nd = tr_first_fit(k, cores[g], mem[g]);
                    if (nd >= 0) {
                        if (dur[g]) {
                            k->fc[nd] -= cores[g];
                            k->fm[nd] -= mem[g];
                            tr_run r = {T + dur[g], (uint32_t)nd, cores[g], mem[g]};
                            tr_push_run(k, r);
                        }
                        out_node[g] = nd;
                        out_start[g] = T;
                        out_finish[g] = T + dur[g];
                        k->has_w = 0;
                        ++k->decided;
                    } else if (cfg->borrow) {
                        req[c] = (int32_t)k->w; /* BorrowResources (:234) */
                    }
                    break; /* time.Sleep(1 s), :250 */
                }
                if (k->rq_head < k->rq_tail) { /* :255-272 */
                    const uint64_t li = k->rq_head++;
                    const uint64_t g = k->j0 + li;
                    const int nd = tr_first_fit(k, cores[g], mem[g]);
                    if (nd >= 0) {
                        if (dur[g]) {
                            k->fc[nd] -= cores[g];
                            k->fm[nd] -= mem[g];
                            tr_run r = {T + dur[g], (uint32_t)nd, cores[g], mem[g]};
                            tr_push_run(k, r);
                        }
                        out_node[g] = nd;
                        out_start[g] = T;
                        out_finish[g] = T + dur[g];
                        ++k->decided;
                    } else {
                        k->has_w = 1;
                        k->w = li;
                    }
                    continue; /* no sleep */
                }
                if (k->lq_len > 0) { /* LentQueue head, :277-290 */
                    const tr_lent e = k->lq[k->lq_head];
                    const int nd = tr_first_fit(k, cores[e.job], mem[e.job]);
                    if (nd >= 0) {
                        if (nl < lent_cap) {
                            lent_log[nl].lender = c;
                            lent_log[nl].borrower = e.borrower;
                            lent_log[nl].job = e.job;
                            lent_log[nl].node = (uint32_t)nd;
                            lent_log[nl].start = T;
                            lent_log[nl].finish = T + dur[e.job];
                        }
                        if (dur[e.job]) {
                            k->fc[nd] -= cores[e.job];
                            k->fm[nd] -= mem[e.job];
                            tr_run r = {T + dur[e.job], (uint32_t)nd, cores[e.job], mem[e.job]};
                            tr_push_run(k, r);
                        }
                        ++nl;
                        ++k->lq_head;
                        --k->lq_len;
                    }
                }
                break; /* sleep 1 s (:289 or :294) */
            }
        }
        /* ---- B. borrow exchange ---- */
        if (cfg->borrow) {
            for (uint32_t b = 0; b < C; ++b) {
                if (req[b] < 0) continue;
                const uint64_t g = cl[b].j0 + (uint64_t)req[b];
                int accepted = 0;
                for (uint32_t l = 0; l < C; ++l) {
                    if (l == b) continue; /* self skipped (server.go:176-180) */
                    tr_cluster* L = &cl[l];
                    if (tr_lend(L, cores[g], mem[g])) {
                        if (L->lq_head + L->lq_len == L->lq_cap) {
                            L->lq_cap = L->lq_cap ? 2 * L->lq_cap : 64;
                            L->lq = (tr_lent*)realloc(L->lq, L->lq_cap * sizeof(tr_lent));
                        }
                        L->lq[L->lq_head + L->lq_len].borrower = b;
                        L->lq[L->lq_head + L->lq_len].job = g;
                        ++L->lq_len;
                        if (L->lq_len > L->lq_peak) L->lq_peak = L->lq_len;
                        accepted = 1;
                    }
                }
                if (accepted) { /* BorrowedQueue append, WaitQueue pop (:237-242) */
                    out_node[g] = -2;
                    out_start[g] = T;
                    out_finish[g] = 0xFFFFFFFFu;
                    cl[b].has_w = 0;
                    ++cl[b].decided;
                }
            }
        }
        /* ---- C. utilization samples ---- */
        if (cfg->trader && T % cfg->sample_period_s == 0)
            for (uint32_t c = 0; c < C; ++c) tr_sample(&cl[c]);
        /* ---- D. traders ---- */
        if (cfg->trader) {
            for (uint32_t q = 0; q < C; ++q) {
                tr_cluster* Q = &cl[q];
                if (Q->next_due > T) continue;
                /* locks expire 20 s after they were set (server.go:48-57) */
                const int broken = Q->cu > 0.8f || Q->mu > 0.8f; /* trader.go:127-130 */
                if (!broken) {
                    Q->next_due = T + cfg->period_s;
                    continue;
                }
                uint32_t napp = 0;
                for (uint32_t r = 0; r < C; ++r) {
                    if (r == q) continue; /* trader.go:212 */
                    tr_cluster* R = &cl[r];
                    if (R->lock_id != 0 && T >= R->lock_until) R->lock_id = 0;
                    if (R->lock_id != 0) continue; /* Approve: false (server.go:35-40) */
                    /* ApproveTrade of the zero contract on the responder's sample */
                    const int ok = or_approve_trade(R->total_c, R->total_m, R->cu, R->mu, 0, 0, 0, 0.0f);
                    R->lock_id = R->next_id++; /* set even when not approving (:44-46) */
                    R->lock_until = T + cfg->lock_s;
                    if (ok) {
                        appr[napp] = r;
                        appr_id[napp] = R->lock_id;
                        prices[napp] = 0.0f;
                        ++napp;
                    }
                }
                int winner = -1;
                if (napp) {
                    or_heap_order(napp, prices, order);
                    for (uint32_t i = 0; i < napp && winner < 0; ++i) {
                        tr_cluster* R = &cl[appr[order[i]]];
                        if (R->lock_id != appr_id[order[i]]) continue; /* DeadlineExceeded */
                        /* AllocateVirtualNodeResources(zero request): breaks at once, success */
                        R->lock_id = 0; /* currentContract reset (:83) */
                        ++Q->virtual_nodes; /* AddVirtualNode(0 cores, 0 memory) */
                        winner = (int)appr[order[i]];
                    }
                }
                if (nt < trade_cap) {
                    trade_log[nt].t = T;
                    trade_log[nt].requester = q;
                    trade_log[nt].winner = winner;
                    trade_log[nt].approvals = napp;
                }
                ++nt;
                Q->next_due = T + (winner >= 0 ? cfg->trade_ok_sleep_s : cfg->trade_fail_sleep_s) +
                              cfg->period_s;
            }
        }
        /* ---- termination and the next tick ---- */
        int busy = 0, all_done = 1;
        uint32_t next = 0xFFFFFFFFu;
        for (uint32_t c = 0; c < C; ++c) {
            tr_cluster* k = &cl[c];
            if (k->decided < k->J || k->lq_len > 0) all_done = 0;
            if (k->has_w || k->lq_len > 0 || k->rq_head < k->rq_tail) busy = 1;
            if (k->next_arrival < k->J) {
                const uint32_t a = arrival[k->j0 + k->next_arrival];
                if (a < next) next = a;
            }
            if (cfg->trader && k->next_due < next) next = k->next_due;
        }
        if (all_done || T >= cfg->t_max) break;
        if (busy || next <= T + 1u) {
            T = T + 1u;
        } else {
            T = next; /* nothing happens between T+1 and next (releases are applied lazily) */
        }
    }
    for (uint32_t c = 0; c < C; ++c) {
        if (cstats) {
            cstats[c].virtual_nodes = cl[c].virtual_nodes;
            cstats[c].decided = (uint32_t)cl[c].decided;
            cstats[c].lent_pending = (uint32_t)cl[c].lq_len;
            cstats[c].lent_peak = (uint32_t)cl[c].lq_peak;
        }
        free(cl[c].cap_c);
        free(cl[c].cap_m);
        free(cl[c].fc);
        free(cl[c].fm);
        free(cl[c].lq);
        free(cl[c].run);
    }
    if (n_lent) *n_lent = nl;
    if (n_trades) *n_trades = nt;
    if (t_final) *t_final = T;
    free(cl);
    free(req);
    free(appr);
    free(appr_id);
    free(prices);
    free(order);
    return 0;
}
