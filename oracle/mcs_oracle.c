/*
 * mcs_oracle.c — CPU ORACLE (test infrastructure only; see mcs_oracle.h for the rules and for how
 * the oracle is pinned).  Deliberately naive: explicit Go-shaped queues, a running list scanned on
 * every loop iteration, uint64 node counters (Go `uint`, D7).  Compiled with -ffp-contract=off so
 * the float32/float64 trader arithmetic rounds like Go on amd64 (GOAMD64=v1 emits no FMA).
 *
 * References are `path:line` in hamzalsheikh/multi-cluster-simulator @ 2024-10-16.
 */
#include "mcs_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------------------------- */
/* Scheduler.ScheduleJob — pkg/scheduler/scheduler.go:127-139: range over Cluster.Nodes in slice
 * order; first node with CoresAvailable >= CoresNeeded && MemoryAvailable >= MemoryNeeded. */
int or_schedule_job(uint32_t n, const uint64_t* free_c, const uint64_t* free_m, uint64_t c,
                    uint64_t m) {
    for (uint32_t i = 0; i < n; ++i)
        if (free_c[i] >= c && free_m[i] >= m) return (int)i; /* scheduler.go:131 */
    return -1; /* errors.New("not enough resources in cluster"), scheduler.go:138 */
}

/* Scheduler.Lend — scheduler.go:194-202: strict '>' on both, no commit, no lock. */
int or_lend(uint32_t n, const uint64_t* free_c, const uint64_t* free_m, uint64_t c, uint64_t m) {
    for (uint32_t i = 0; i < n; ++i)
        if (free_c[i] > c && free_m[i] > m) return 1; /* scheduler.go:197 */
    return 0; /* "can't lend", scheduler.go:201 */
}

/* ------------------------------------------------------------------------------------------- */
typedef struct {
    uint32_t finish;
    uint32_t node;
    uint64_t c, m;
} or_running;

typedef struct {
    uint32_t n;
    uint64_t *fc, *fm;
    or_running* run;
    uint64_t nrun, caprun;
} or_cluster;

/* Node.RunJob commit half — cluster.go:141-151 (lock; RunningJobs[id] = j; CoresAvailable -= c;
 * MemoryAvailable -= m; then Sleep(Duration)).  D2: the commit happens synchronously here. */
static void run_job(or_cluster* cl, uint32_t k, uint64_t c, uint64_t m, uint32_t t,
                    uint32_t dur) {
    cl->fc[k] -= c; /* cluster.go:146 (uint wrap as Go) */
    cl->fm[k] -= m; /* cluster.go:147 */
    if (cl->nrun == cl->caprun) {
        cl->caprun = cl->caprun ? 2 * cl->caprun : 64;
        cl->run = (or_running*)realloc(cl->run, cl->caprun * sizeof(or_running));
    }
    or_running r = {t + dur, k, c, m}; /* time.Sleep(j.Duration), cluster.go:151 */
    cl->run[cl->nrun++] = r;
}

/* Node.RunJob completion half — cluster.go:153-157: every job whose sleep has ended gives its
 * resources back.  Appendix A.2 step 1 / D3: releases precede the loop's branch. */
static void release_due(or_cluster* cl, uint32_t t) {
    for (uint64_t i = 0; i < cl->nrun;) {
        if (cl->run[i].finish <= t) {
            cl->fc[cl->run[i].node] += cl->run[i].c; /* cluster.go:155 */
            cl->fm[cl->run[i].node] += cl->run[i].m; /* cluster.go:156 */
            cl->run[i] = cl->run[--cl->nrun];
            /* sched.JobFinished(j) (cluster.go:160): for an own job it only scans Wait/Ready
             * queues for an equal job, which was already popped (scheduler.go:163-178), so it
             * is a no-op. */
        } else {
            ++i;
        }
    }
}

static uint32_t min_finish(const or_cluster* cl) {
    uint32_t mf = 0xFFFFFFFFu;
    for (uint64_t i = 0; i < cl->nrun; ++i)
        if (cl->run[i].finish < mf) mf = cl->run[i].finish;
    return mf;
}

/* Scheduler.Fifo — pkg/scheduler/scheduler.go:216-296 under SFIFO. */
int or_fifo_run(uint32_t n_nodes, const uint32_t* cap_c, const uint32_t* cap_m,
                const uint32_t* free_c, const uint32_t* free_m, uint64_t n_jobs,
                const uint32_t* arrival, const uint32_t* dur, const uint32_t* cores,
                const uint32_t* mem, int literal, int32_t* out_node, uint32_t* out_start,
                uint32_t* out_finish, or_stats* st) {
    (void)cap_c;
    (void)cap_m;
    or_cluster cl;
    memset(&cl, 0, sizeof cl);
    cl.n = n_nodes;
    cl.fc = (uint64_t*)malloc(sizeof(uint64_t) * (n_nodes ? n_nodes : 1));
    cl.fm = (uint64_t*)malloc(sizeof(uint64_t) * (n_nodes ? n_nodes : 1));
    /* Run (scheduler.go:101-109) keeps the JSON CoresAvailable/MemoryAvailable as-is (KAT5). */
    for (uint32_t i = 0; i < n_nodes; ++i) {
        cl.fc[i] = free_c[i];
        cl.fm[i] = free_m[i];
    }
    /* ReadyQueue / WaitQueue as Go slices of job ids (scheduler.go:19-20). */
    uint64_t* rq = (uint64_t*)malloc(sizeof(uint64_t) * (n_jobs ? n_jobs : 1));
    uint64_t* wq = (uint64_t*)malloc(sizeof(uint64_t) * (n_jobs ? n_jobs : 1));
    uint64_t rq_head = 0, rq_tail = 0, wq_head = 0, wq_tail = 0;
    uint64_t next_arrival = 0, decided = 0, ticks = 0;
    uint32_t t = 0, waited = 0, peak = 0, flags = 0;

    for (uint64_t j = 0; j < n_jobs; ++j) {
        out_node[j] = -1;
        out_start[j] = 0xFFFFFFFFu;
        out_finish[j] = 0xFFFFFFFFu;
    }

    for (;;) {
        ++ticks;
        release_due(&cl, t);
        /* the "/" handler appends each arriving job to the ReadyQueue (server.go:38-41) */
        while (next_arrival < n_jobs && arrival[next_arrival] <= t) rq[rq_tail++] = next_arrival++;
        if (decided == n_jobs) break;

        if (wq_tail > wq_head) { /* if len(sched.WaitQueue) > 0, scheduler.go:219 */
            const uint64_t j = wq[wq_head];
            const int k = or_schedule_job(cl.n, cl.fc, cl.fm, cores[j], mem[j]); /* :222 */
            if (k >= 0) {
                run_job(&cl, (uint32_t)k, cores[j], mem[j], t, dur[j]);
                out_node[j] = k;
                out_start[j] = t;
                out_finish[j] = t + dur[j];
                if (dur[j] > 0 && cl.nrun > peak) peak = (uint32_t)cl.nrun;
                ++wq_head; /* WaitQueue = WaitQueue[1:] (:226); D1: no panic on the log line */
                ++decided;
                t += 1; /* time.Sleep(1 * time.Second), scheduler.go:250 */
            } else {
                /* BorrowResources (:234): FIFO without peers finds no lender (server.go:220). */
                if (cl.nrun == 0) { /* nothing will ever be released: the Go loop spins forever */
                    flags |= 1u;
                    break;
                }
                if (literal) {
                    t += 1; /* scheduler.go:250 */
                } else {    /* Appendix A.3: nothing changes until the next completion */
                    const uint32_t mf = min_finish(&cl);
                    t = (mf > t + 1u) ? mf : t + 1u;
                }
            }
            continue;
        }
        if (rq_tail > rq_head) { /* if len(sched.ReadyQueue) > 0, scheduler.go:255 */
            const uint64_t j = rq[rq_head++]; /* ReadyQueue[0]; ReadyQueue = ReadyQueue[1:] :258-260 */
            const int k = or_schedule_job(cl.n, cl.fc, cl.fm, cores[j], mem[j]);
            if (k >= 0) {
                run_job(&cl, (uint32_t)k, cores[j], mem[j], t, dur[j]);
                out_node[j] = k;
                out_start[j] = t;
                out_finish[j] = t + dur[j];
                if (dur[j] > 0 && cl.nrun > peak) peak = (uint32_t)cl.nrun;
                ++decided;
            } else {
                wq[wq_tail++] = j; /* State = WAITING; WaitQueue append, scheduler.go:264-268 */
                ++waited;
            }
            continue; /* no sleep on the ready path (:272 commented out) */
        }
        /* LentQueue (scheduler.go:277) is empty without borrowing. */
        if (literal) {
            t += 1; /* time.Sleep(1 * time.Second), scheduler.go:294 */
        } else {    /* Appendix A.3 idle fast-forward */
            const uint32_t a = arrival[next_arrival];
            t = (a > t + 1u) ? a : t + 1u;
        }
    }

    if (st) {
        st->t_end = t;
        st->placed = (uint32_t)decided;
        st->waited = waited;
        st->peak_running = peak;
        st->flags = flags;
        st->pad = 0;
        st->ticks = ticks;
    }
    free(cl.fc);
    free(cl.fm);
    free(cl.run);
    free(rq);
    free(wq);
    return 0;
}

int or_fifo_run_batch(uint32_t n_clusters, const uint32_t* node_off, const uint32_t* cap_c,
                      const uint32_t* cap_m, const uint32_t* free_c, const uint32_t* free_m,
                      const uint64_t* job_off, const uint32_t* arrival, const uint32_t* dur,
                      const uint32_t* cores, const uint32_t* mem, int n_threads,
                      int32_t* out_node, uint32_t* out_start, uint32_t* out_finish,
                      or_stats* st) {
#ifdef _OPENMP
    if (n_threads < 1) n_threads = 1;
#pragma omp parallel for schedule(dynamic, 1) num_threads(n_threads)
#else
    (void)n_threads;
#endif
    for (int64_t c = 0; c < (int64_t)n_clusters; ++c) {
        const uint32_t n0 = node_off[c], nn = node_off[c + 1] - node_off[c];
        const uint64_t j0 = job_off[c], jn = job_off[c + 1] - job_off[c];
        or_fifo_run(nn, cap_c + n0, cap_m + n0, free_c + n0, free_m + n0, jn, arrival + j0,
                    dur + j0, cores + j0, mem + j0, 0, out_node + j0, out_start + j0,
                    out_finish + j0, st ? st + c : 0);
    }
    return 0;
}

/* ------------------------------------------------------------------------------------------- */
/* Cluster.GetResourceUtilization — cluster.go:46-63. */
void or_resource_utilization(uint32_t n, const uint64_t* cap_c, const uint64_t* cap_m,
                             const uint64_t* free_c, const uint64_t* free_m, uint32_t total_c,
                             uint32_t total_m, float* cu, float* mu) {
    float c = 0.0f, m = 0.0f;
    for (uint32_t i = 0; i < n; ++i) {
        c += ((float)cap_c[i] - (float)free_c[i]); /* cluster.go:55 */
        m += ((float)cap_m[i] - (float)free_m[i]); /* cluster.go:56 */
    }
    *cu = c / (float)total_c; /* cluster.go:62 */
    *mu = m / (float)total_m;
}

/* Trader.ApproveTrade — pkg/trader/trader.go:141-167 with approvePolicy{0.8, 0.8, -1, -1}
 * (trader.go:47-52).  float32 availability in Go's order T - (T*u) (148-149); float64 incentive
 * evaluated left to right (154). */
int or_approve_trade(uint32_t total_c, uint32_t total_m, float core_util, float mem_util,
                     uint32_t req_cores, uint32_t req_mem, int64_t req_time_ns,
                     float req_price) {
    const float core_thr = 0.8f, mem_thr = 0.8f;
    const double min_core_inc = -1.0, min_mem_inc = -1.0;
    if (core_util < core_thr && mem_util < mem_thr) { /* trader.go:147 */
        const float tm = (float)total_m, tc = (float)total_c;
        const float prod_m = tm * mem_util;
        const float prod_c = tc * core_util;
        const float avail_mem = tm - prod_m;  /* trader.go:148 */
        const float avail_core = tc - prod_c; /* trader.go:149 */
        if (avail_core >= (float)req_cores && avail_mem >= (float)req_mem) { /* :151 */
            /* Duration.Seconds(): float64(d/1e9) + float64(d%1e9)/1e9 */
            const int64_t sec = req_time_ns / 1000000000LL, nsec = req_time_ns % 1000000000LL;
            const double secs = (double)sec + (double)nsec / 1e9;
            const double a = min_core_inc * (double)req_cores;
            const double b = a * secs;
            const double c2 = min_mem_inc * (double)req_mem;
            const double d = c2 * secs;
            const double incentive = b + d; /* trader.go:154 */
            if ((double)req_price >= incentive) return 1; /* trader.go:155 */
        }
    }
    return 0;
}

/* ------------------------------------------------------------------------------------------- */
/* Go container/heap (Go 1.21 src/container/heap/heap.go) over contractResHeap, whose Less is
 * h[i].Price < h[j].Price (trader.go:173-175). */
typedef struct {
    float price;
    uint32_t idx;
} or_hent;

static int h_less(const or_hent* h, int i, int j) { return h[i].price < h[j].price; }
static void h_swap(or_hent* h, int i, int j) {
    or_hent x = h[i];
    h[i] = h[j];
    h[j] = x;
}
static void h_up(or_hent* h, int j) {
    for (;;) {
        int i = (j - 1) / 2; /* Go integer division truncates: (0-1)/2 == 0 */
        if (i == j || !h_less(h, j, i)) break;
        h_swap(h, i, j);
        j = i;
    }
}
static void h_down(or_hent* h, int i0, int n) {
    int i = i0;
    for (;;) {
        int j1 = 2 * i + 1;
        if (j1 >= n || j1 < 0) break;
        int j = j1;
        int j2 = j1 + 1;
        if (j2 < n && h_less(h, j2, j1)) j = j2;
        if (!h_less(h, j, i)) break;
        h_swap(h, i, j);
        i = j;
    }
}

void or_heap_order(uint32_t n, const float* prices, uint32_t* order) {
    or_hent* h = (or_hent*)malloc(sizeof(or_hent) * (n ? n : 1));
    int len = 0;
    for (uint32_t i = 0; i < n; ++i) { /* heap.Push(h, cont), trader.go:247 */
        h[len].price = prices[i];
        h[len].idx = i;
        ++len;
        h_up(h, len - 1);
    }
    for (uint32_t k = 0; k < n; ++k) { /* heap.Pop(h), trader.go:266 */
        int last = len - 1;
        h_swap(h, 0, last);
        h_down(h, 0, last);
        order[k] = h[last].idx;
        --len;
    }
    free(h);
}

/* ------------------------------------------------------------------------------------------- */
/* Cluster.AllocateVirtualNodeResources — cluster.go:87-125. */
int or_allocate_virtual_node(uint32_t n, uint64_t* free_c, uint64_t* free_m, uint32_t req_c,
                             uint32_t req_m, uint32_t* n_foreign, uint32_t* f_node, uint64_t* f_c,
                             uint64_t* f_m) {
    uint32_t nf = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if (req_m == 0 && req_c == 0) break; /* req.Memory <= 0 && req.Cores <= 0, :90-92 */
        double mem_diff = 0.0, core_diff = 0.0;
        if (req_m > 0) mem_diff = fabs((double)req_m - (double)free_m[i]);  /* :96-98 */
        if (req_c > 0) core_diff = fabs((double)req_c - (double)free_c[i]); /* :100-102 */
        if (mem_diff > (double)req_m)
            req_m = 0; /* :104-108 */
        else
            req_m -= (uint32_t)mem_diff;
        if (core_diff > (double)req_c)
            req_c = 0; /* :110-114 */
        else
            req_c -= (uint32_t)core_diff;
        /* go node.RunJob(Job{CoresNeeded: uint(core_diff), MemoryNeeded: uint(mem_diff), ...}),
         * :116 — the commit (cluster.go:146-147), uint wrap as Go (D7) */
        const uint64_t fc = or_go_f64_to_u64(core_diff), fm = or_go_f64_to_u64(mem_diff);
        free_c[i] -= fc;
        free_m[i] -= fm;
        if (f_node) {
            f_node[nf] = i;
            f_c[nf] = fc;
            f_m[nf] = fm;
        }
        ++nf;
    }
    if (n_foreign) *n_foreign = nf;
    if (req_c > 0 || req_m > 0) return 1; /* "couldn't schedule enough resources", :119-121 */
    return 0;
}

/* ------------------------------------------------------------------------------------------- */
/* ProvideJobs batching (trader_server.go:69-94): batches of BATCH=20, the last padded with nil
 * *pb.Job that reach the trader as zero jobs (D9).  Returns padded length. */
static uint32_t padded_len(uint32_t n) { return (n % 20u) ? n + (20u - n % 20u) : n; }

/* calculateFastNodeSize — pkg/trader/scheduler_client.go:126-170. */
void or_contract_fast(uint32_t n, const uint32_t* c, const uint32_t* m, const uint32_t* dur_s,
                      uint32_t* oc, uint32_t* om, int64_t* otime_ns, float* oprice) {
    uint32_t cc = 0, cm = 0;
    int64_t ct = 0;
    float cp = 0.0f;
    const float max_core_cost = 0.0f, max_mem_cost = 0.0f, budget = -1.0f; /* trader.go:34-35,53 */
    const uint32_t np = padded_len(n);
    for (uint32_t i = 0; i < np; ++i) {
        const uint32_t jc = i < n ? c[i] : 0, jm = i < n ? m[i] : 0;
        const int64_t jt = i < n ? (int64_t)dur_s[i] * 1000000000LL : 0;
        const int64_t new_time = jt > ct ? jt : ct; /* :144-148 */
        const uint32_t new_cores = cc + jc;       /* :150 uint32 wrap */
        const uint32_t new_mem = cm + jm;
        const int64_t sec = new_time / 1000000000LL, nsec = new_time % 1000000000LL;
        const double secs = (double)sec + (double)nsec / 1e9;
        const double p1 = secs * (double)new_cores;
        const double p2 = p1 * (double)max_core_cost;
        const double q1 = (double)max_mem_cost * secs;
        const double q2 = q1 * (double)new_mem;
        const double new_price = p2 + q2; /* :152 */
        if (new_price < (double)budget || budget < 0) {
            cc = new_cores;
            cm = new_mem;
            ct = new_time;
            cp = (float)new_price;
        } else {
            break; /* "fast node reached budget" */
        }
    }
    *oc = cc;
    *om = cm;
    *otime_ns = ct;
    *oprice = cp;
}

/* calculateSmallNodeSize — pkg/trader/scheduler_client.go:201-289.  atTime only ever holds the
 * initial {0,0,0} entry (nothing appends to it), and the inner costArr loop mutates copies, so each
 * job yields one startingJob; GetMin (187-198) over a one-element array returns it. */
void or_contract_small(uint32_t n, const uint32_t* c, const uint32_t* m, const uint32_t* dur_s,
                       uint32_t* oc, uint32_t* om, int64_t* otime_ns, float* oprice) {
    uint32_t cc = 0, cm = 0;
    int64_t ct = 0;
    float cp = 0.0f;
    const float max_core_cost = 0.0f, max_mem_cost = 0.0f, budget = -1.0f;
    const uint32_t np = padded_len(n);
    for (uint32_t i = 0; i < np; ++i) {
        const uint32_t jc = i < n ? c[i] : 0, jm = i < n ? m[i] : 0;
        const uint32_t jd = i < n ? dur_s[i] : 0;
        /* currState after the single atTime entry: {cores 0, memory 0} */
        const int32_t cores = (int32_t)(0u - jc); /* currState.cores - int32(CoresNeeded) :238 */
        const int32_t memv = (int32_t)(0u - jm);
        int32_t sj_cores, sj_mem;
        if (cores < 0)
            sj_cores = (int32_t)((uint32_t)(int32_t)cc - (uint32_t)cores); /* :241-245 */
        else
            sj_cores = (int32_t)cc;
        if (memv < 0)
            sj_mem = (int32_t)((uint32_t)(int32_t)cm - (uint32_t)memv); /* :246-250 */
        else
            sj_mem = (int32_t)cm;
        const double end_time = 0.0 + (double)jd; /* :253 startTime 0 + Seconds() */
        const int64_t sec = ct / 1000000000LL, nsec = ct % 1000000000LL;
        const double contract_secs = (double)sec + (double)nsec / 1e9;
        double sj_time = 0.0;
        if (contract_secs < end_time) sj_time = end_time; /* :263-265, else stays 0 */
        /* GetMin (:187-198) of the one-element costArr; price (:268) */
        const float ft = (float)sj_time;
        const float pc = (float)sj_cores * max_core_cost;
        const float pm = (float)sj_mem * max_mem_cost;
        const float price = pc * ft + pm * ft;
        if (price < budget || budget < 0) {
            cc = (uint32_t)sj_cores;
            cm = (uint32_t)sj_mem;
            ct = (int64_t)(sj_time * 1e9); /* time.Duration(min.time * float64(time.Second)) */
            cp = price;
        } else {
            break;
        }
    }
    *oc = cc;
    *om = cm;
    *otime_ns = ct;
    *oprice = cp;
}
