/*
 * oracle_selftest.c — seeded self-test of the CPU ORACLE, built only with AddressSanitizer +
 * UndefinedBehaviorSanitizer (oracle/Makefile target `asan`, run by tests/test_oracle_sanitize.py).
 * TEST INFRASTRUCTURE ONLY: it links the oracle sources, never libmcs.so, and is never shipped.
 *
 * The oracle holds every parity claim, and its Go-shaped queues (memmove / realloc growth) and
 * uint64 wrap arithmetic (cluster.go:116,146: `uint` counters that AllocateVirtualNodeResources
 * can drive below zero) are where a C restatement can corrupt memory silently.  This program drives
 * every entry point over seeded random inputs and checks the oracle's own exact identities:
 *
 *   FIFO   literal one-second loop == fast-forward (scheduler.go:216-296), per
 *          cluster and through the OpenMP batch with 1 and 4 threads;
 *   DELAY  literal == fast-forward, statistics included (scheduler.go:298-369);
 *   trade  borrow and trader off == the FIFO batch; the trader alone changes no placement (under
 *          FIFO every contract is the zero contract, trader.go:280-325); a full run with logs
 *          smaller than their counts (counted, not written) keeps every job's outcome well-formed;
 *   dtrade no traders (period 0) == the DELAY batch; a full run with small log capacities;
 *   and the single-call mirrors: first fit / Lend against a linear scan, the float32 utilization,
 *   ApproveTrade, Go heap order (a permutation in price order), AllocateVirtualNodeResources on
 *   wrapped counters, and the fast/small contract sizes over Level1 lists of every padding.
 *
 * The golden KATs themselves (tests/golden/ *.json) run through the sanitized library from Python
 * (tests/test_oracle_sanitize.py runs the oracle test modules against it).  Exit status 0 and
 * "SELFTEST OK" on success; any sanitizer report aborts (halt_on_error).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mcs_oracle.h"
#include "mcs_oracle_trade.h"

static uint64_t g_state;
static uint64_t rnd(void) { /* splitmix64 */
    uint64_t z = (g_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static uint32_t rr(uint32_t lo, uint32_t hi) { return lo + (uint32_t)(rnd() % (uint64_t)(hi - lo + 1u)); }

static int g_fail = 0;
#define CHECK(cond, ...)                                        \
    do {                                                        \
        if (!(cond)) {                                          \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                       \
            fprintf(stderr, "\n");                              \
            ++g_fail;                                           \
        }                                                       \
    } while (0)

static void* xmalloc(size_t n) {
    void* p = malloc(n ? n : 1);
    if (!p) {
        fprintf(stderr, "out of memory\n");
        exit(2);
    }
    return p;
}

/* ---- a random system: C clusters of 1..max_nodes nodes, J jobs each (kat_util.fuzz_workload's
 * shape: random availability, bursts, idle stretches, zero-duration / zero-resource jobs, and
 * optionally one request that fits no node) ----------------------------------------------------- */
typedef struct {
    uint32_t C;
    uint32_t *node_off, *cap_c, *cap_m, *free_c, *free_m;
    uint64_t* job_off;
    uint32_t *arr, *dur, *cores, *mem;
} sys_t;

static void sys_make(sys_t* s, uint32_t C, uint32_t max_nodes, uint32_t J, int blocking, uint32_t max_dur) {
    s->C = C;
    s->node_off = xmalloc((C + 1) * sizeof(uint32_t));
    s->job_off = xmalloc((C + 1) * sizeof(uint64_t));
    uint32_t* nn = xmalloc(C * sizeof(uint32_t));
    uint32_t tot = 0;
    for (uint32_t k = 0; k < C; ++k) {
        nn[k] = rr(1, max_nodes);
        s->node_off[k] = tot;
        tot += nn[k];
    }
    s->node_off[C] = tot;
    s->cap_c = xmalloc(tot * 4);
    s->cap_m = xmalloc(tot * 4);
    s->free_c = xmalloc(tot * 4);
    s->free_m = xmalloc(tot * 4);
    const uint64_t NJ = (uint64_t)C * J;
    s->arr = xmalloc(NJ * 4);
    s->dur = xmalloc(NJ * 4);
    s->cores = xmalloc(NJ * 4);
    s->mem = xmalloc(NJ * 4);
    for (uint32_t k = 0; k < C; ++k) {
        const uint32_t cc = rr(1, 63), cm = rr(1, 32000);
        for (uint32_t i = s->node_off[k]; i < s->node_off[k + 1]; ++i) {
            s->cap_c[i] = cc;
            s->cap_m[i] = cm;
            s->free_c[i] = rr(0, 9) < 7 ? cc : rr(0, cc);
            s->free_m[i] = rr(0, 9) < 7 ? cm : rr(0, cm);
        }
        if (!blocking) { /* node 0 fully available: every request fits once it drains */
            s->free_c[s->node_off[k]] = cc;
            s->free_m[s->node_off[k]] = cm;
        }
        s->job_off[k] = (uint64_t)k * J;
        uint32_t t = rr(0, 5);
        const uint32_t md = rr(1, max_dur);
        for (uint32_t j = 0; j < J; ++j) {
            const uint64_t x = (uint64_t)k * J + j;
            t += rr(0, 9) < 4 ? 0 : rr(0, 3);
            if (rr(0, 99) < 3) t += rr(10, 400); /* idle stretch */
            s->arr[x] = t;
            s->dur[x] = rr(0, md);
            s->cores[x] = rr(0, cc);
            s->mem[x] = rr(0, cm);
            if (rr(0, 49) == 0) s->cores[x] = s->mem[x] = 0;
        }
        if (blocking && rr(0, 1)) { /* one request that fits no node */
            const uint64_t x = (uint64_t)k * J + rr(J / 4, J - 1);
            if (rr(0, 1)) s->cores[x] = cc + 1;
            else s->mem[x] = cm + 1;
        }
    }
    s->job_off[C] = NJ;
    free(nn);
}

static void sys_free(sys_t* s) {
    free(s->node_off);
    free(s->job_off);
    free(s->cap_c);
    free(s->cap_m);
    free(s->free_c);
    free(s->free_m);
    free(s->arr);
    free(s->dur);
    free(s->cores);
    free(s->mem);
}

typedef struct {
    int32_t* node;
    uint32_t *start, *finish;
} res_t;
static void res_make(res_t* r, uint64_t n) {
    r->node = xmalloc(n * 4);
    r->start = xmalloc(n * 4);
    r->finish = xmalloc(n * 4);
}
static void res_free(res_t* r) {
    free(r->node);
    free(r->start);
    free(r->finish);
}
static int res_eq(const res_t* a, const res_t* b, uint64_t n) {
    return !memcmp(a->node, b->node, n * 4) && !memcmp(a->start, b->start, n * 4) &&
           !memcmp(a->finish, b->finish, n * 4);
}

/* ---- FIFO ---------------------------------------------------------------------------------- */
static void test_fifo(int iters) {
    for (int it = 0; it < iters; ++it) {
        sys_t s;
        const uint32_t C = rr(1, 6), J = rr(1, 400);
        sys_make(&s, C, it % 3 == 0 ? 300 : 64, J, 1, 300);
        const uint64_t NJ = s.job_off[C];
        res_t lit, ff, b1, b4;
        res_make(&lit, NJ);
        res_make(&ff, NJ);
        res_make(&b1, NJ);
        res_make(&b4, NJ);
        or_stats* st = xmalloc(C * sizeof(or_stats));
        for (uint32_t k = 0; k < C; ++k) {
            const uint32_t n0 = s.node_off[k], nn = s.node_off[k + 1] - n0;
            const uint64_t j0 = s.job_off[k], nj = s.job_off[k + 1] - j0;
            or_stats a, b;
            or_fifo_run(nn, s.cap_c + n0, s.cap_m + n0, s.free_c + n0, s.free_m + n0, nj, s.arr + j0, s.dur + j0,
                        s.cores + j0, s.mem + j0, 1, lit.node + j0, lit.start + j0, lit.finish + j0, &a);
            or_fifo_run(nn, s.cap_c + n0, s.cap_m + n0, s.free_c + n0, s.free_m + n0, nj, s.arr + j0, s.dur + j0,
                        s.cores + j0, s.mem + j0, 0, ff.node + j0, ff.start + j0, ff.finish + j0, &b);
            CHECK(a.placed == b.placed && a.waited == b.waited && a.flags == b.flags && a.peak_running == b.peak_running,
                  "fifo stats literal != fast-forward (iter %d cluster %u)", it, k);
        }
        CHECK(res_eq(&lit, &ff, NJ), "fifo literal != fast-forward (iter %d)", it);
        or_fifo_run_batch(C, s.node_off, s.cap_c, s.cap_m, s.free_c, s.free_m, s.job_off, s.arr, s.dur, s.cores,
                          s.mem, 1, b1.node, b1.start, b1.finish, st);
        or_fifo_run_batch(C, s.node_off, s.cap_c, s.cap_m, s.free_c, s.free_m, s.job_off, s.arr, s.dur, s.cores,
                          s.mem, 4, b4.node, b4.start, b4.finish, st);
        CHECK(res_eq(&ff, &b1, NJ) && res_eq(&ff, &b4, NJ), "fifo batch != per-cluster (iter %d)", it);
        for (uint64_t x = 0; x < NJ; ++x)
            if (ff.node[x] >= 0) CHECK(ff.start[x] >= s.arr[x] && ff.finish[x] == ff.start[x] + s.dur[x],
                                       "fifo job %llu times", (unsigned long long)x);
        free(st);
        res_free(&lit);
        res_free(&ff);
        res_free(&b1);
        res_free(&b4);
        sys_free(&s);
    }
}

/* ---- DELAY --------------------------------------------------------------------------------- */
static void test_delay(int iters) {
    for (int it = 0; it < iters; ++it) {
        sys_t s;
        const uint32_t C = rr(1, 4), J = rr(1, 300);
        sys_make(&s, C, it % 3 == 0 ? 256 : 40, J, it & 1, 200);
        const uint64_t NJ = s.job_off[C];
        res_t lit, ff, b;
        res_make(&lit, NJ);
        res_make(&ff, NJ);
        res_make(&b, NJ);
        or_delay_stats* st = xmalloc(C * sizeof(or_delay_stats));
        const uint32_t mw = rr(0, 3) ? 10u : rr(0, 30);
        for (uint32_t k = 0; k < C; ++k) {
            const uint32_t n0 = s.node_off[k], nn = s.node_off[k + 1] - n0;
            const uint64_t j0 = s.job_off[k], nj = s.job_off[k + 1] - j0;
            or_delay_stats a, c;
            or_delay_run(nn, s.free_c + n0, s.free_m + n0, nj, s.arr + j0, s.dur + j0, s.cores + j0, s.mem + j0, mw, 1,
                         lit.node + j0, lit.start + j0, lit.finish + j0, &a);
            or_delay_run(nn, s.free_c + n0, s.free_m + n0, nj, s.arr + j0, s.dur + j0, s.cores + j0, s.mem + j0, mw, 0,
                         ff.node + j0, ff.start + j0, ff.finish + j0, &c);
            CHECK(a.placed == c.placed && a.moved_l1 == c.moved_l1 && a.placed_l1 == c.placed_l1 &&
                      a.total_wait_ms == c.total_wait_ms && a.jobs_count == c.jobs_count && a.l1_left == c.l1_left,
                  "delay stats literal != fast-forward (iter %d cluster %u)", it, k);
        }
        CHECK(res_eq(&lit, &ff, NJ), "delay literal != fast-forward (iter %d)", it);
        or_delay_run_batch(C, s.node_off, s.free_c, s.free_m, s.job_off, s.arr, s.dur, s.cores, s.mem, mw, 3, b.node,
                           b.start, b.finish, st);
        CHECK(res_eq(&ff, &b, NJ), "delay batch != per-cluster (iter %d)", it);
        free(st);
        res_free(&lit);
        res_free(&ff);
        res_free(&b);
        sys_free(&s);
    }
}

/* ---- lock-step trading (FIFO) ------------------------------------------------------------- */
static or_trade_cfg trade_cfg(uint32_t borrow, uint32_t trader) {
    or_trade_cfg c = {borrow, trader, 10, 240, 120, 20, 5, 2000000u};
    return c;
}

static void trade_once(const sys_t* s, const or_trade_cfg* cfg, res_t* r, uint64_t lent_cap, uint64_t trade_cap,
                       uint64_t* n_lent, uint64_t* n_trades, uint32_t* t_final) {
    or_lent_rec* lent = xmalloc((lent_cap ? lent_cap : 1) * sizeof(or_lent_rec));
    or_trade_rec* tr = xmalloc((trade_cap ? trade_cap : 1) * sizeof(or_trade_rec));
    or_trade_cluster_stats* cs = xmalloc(s->C * sizeof(or_trade_cluster_stats));
    or_trade_run(s->C, s->node_off, s->cap_c, s->cap_m, s->free_c, s->free_m, s->job_off, s->arr, s->dur, s->cores,
                 s->mem, cfg, r->node, r->start, r->finish, lent, lent_cap, n_lent, tr, trade_cap, n_trades, cs,
                 t_final);
    for (uint64_t i = 0; i < (*n_lent < lent_cap ? *n_lent : lent_cap); ++i)
        CHECK(lent[i].lender < s->C && lent[i].borrower < s->C && lent[i].lender != lent[i].borrower,
              "lent record %llu", (unsigned long long)i);
    for (uint64_t i = 0; i < (*n_trades < trade_cap ? *n_trades : trade_cap); ++i)
        CHECK(tr[i].requester < s->C && tr[i].winner < (int32_t)s->C, "trade record %llu", (unsigned long long)i);
    free(lent);
    free(tr);
    free(cs);
}

static void test_trade(int iters) {
    for (int it = 0; it < iters; ++it) {
        sys_t s;
        const uint32_t C = rr(2, 8), J = rr(20, 300);
        sys_make(&s, C, it % 2 ? 64 : 200, J, 0, 200);
        const uint64_t NJ = s.job_off[C];
        res_t off, tro, full, fifo;
        res_make(&off, NJ);
        res_make(&tro, NJ);
        res_make(&full, NJ);
        res_make(&fifo, NJ);
        or_stats* st = xmalloc(C * sizeof(or_stats));
        or_fifo_run_batch(C, s.node_off, s.cap_c, s.cap_m, s.free_c, s.free_m, s.job_off, s.arr, s.dur, s.cores,
                          s.mem, 1, fifo.node, fifo.start, fifo.finish, st);
        uint64_t nl = 0, nt = 0;
        uint32_t tf = 0;
        or_trade_cfg c0 = trade_cfg(0, 0), c1 = trade_cfg(0, 1), c2 = trade_cfg(1, 1);
        trade_once(&s, &c0, &off, 64, 64, &nl, &nt, &tf);
        CHECK(res_eq(&off, &fifo, NJ), "trade (borrow, trader off) != FIFO batch (iter %d)", it);
        trade_once(&s, &c1, &tro, 64, 64, &nl, &nt, &tf);
        CHECK(res_eq(&tro, &fifo, NJ), "trader alone changed a placement (iter %d)", it);
        /* the full system, with logs smaller than their counts on odd iterations */
        trade_once(&s, &c2, &full, it & 1 ? 3 : 1u << 16, it & 1 ? 2 : 1u << 12, &nl, &nt, &tf);
        for (uint64_t x = 0; x < NJ; ++x) {
            const int32_t n = full.node[x];
            CHECK(n >= -2, "trade job %llu node %d", (unsigned long long)x, n);
            if (n >= 0) CHECK(full.start[x] >= s.arr[x] && full.finish[x] == full.start[x] + s.dur[x],
                              "trade job %llu times", (unsigned long long)x);
            if (n == -2) CHECK(full.start[x] >= s.arr[x], "borrowed job %llu", (unsigned long long)x);
        }
        free(st);
        res_free(&off);
        res_free(&tro);
        res_free(&full);
        res_free(&fifo);
        sys_free(&s);
    }
}

/* ---- lock-step trading (DELAY, real contracts) ------------------------------------------- */
static void test_dtrade(int iters) {
    for (int it = 0; it < iters; ++it) {
        sys_t s;
        const uint32_t C = rr(2, 8), J = rr(20, 250);
        sys_make(&s, C, it % 2 ? 12 : 64, J, 0, 150);
        const uint64_t NJ = s.job_off[C];
        const uint32_t V = 64;
        res_t ind, full, dl;
        res_make(&ind, NJ);
        res_make(&full, NJ);
        res_make(&dl, NJ);
        or_delay_stats* dst = xmalloc(C * sizeof(or_delay_stats));
        or_delay_run_batch(C, s.node_off, s.free_c, s.free_m, s.job_off, s.arr, s.dur, s.cores, s.mem, 10, 1, dl.node,
                           dl.start, dl.finish, dst);
        uint32_t* vc = xmalloc((size_t)C * V * 4);
        uint32_t* vm = xmalloc((size_t)C * V * 4);
        or_dtrade_cluster_stats* cs = xmalloc(C * sizeof(or_dtrade_cluster_stats));
        for (int pass = 0; pass < 2; ++pass) {
            or_dtrade_cfg cfg = {pass ? 10u : 0u, 240, 120, 20, 5, 10, V, 2000000u};
            const uint64_t tcap = (it & 1) ? 2 : 4096, fcap = (it & 1) ? 3 : 1u << 16;
            or_dtrade_rec* tl = xmalloc(tcap * sizeof(or_dtrade_rec));
            or_foreign_rec* fl = xmalloc(fcap * sizeof(or_foreign_rec));
            uint64_t nt = 0, nf = 0;
            uint32_t tf = 0;
            res_t* r = pass ? &full : &ind;
            or_dtrade_run(C, s.node_off, s.cap_c, s.cap_m, s.free_c, s.free_m, s.job_off, s.arr, s.dur, s.cores, s.mem,
                          &cfg, r->node, r->start, r->finish, tl, tcap, &nt, fl, fcap, &nf, vc, vm, cs, &tf);
            for (uint64_t i = 0; i < (nf < fcap ? nf : fcap); ++i)
                CHECK(fl[i].requester < C && fl[i].responder < C, "foreign record %llu", (unsigned long long)i);
            free(tl);
            free(fl);
        }
        CHECK(res_eq(&ind, &dl, NJ), "DELAY trading without traders != the DELAY batch (iter %d)", it);
        for (uint64_t x = 0; x < NJ; ++x)
            if (full.node[x] >= 0) CHECK(full.start[x] >= s.arr[x], "dtrade job %llu", (unsigned long long)x);
        free(vc);
        free(vm);
        free(cs);
        free(dst);
        res_free(&ind);
        res_free(&full);
        res_free(&dl);
        sys_free(&s);
    }
}

/* ---- single-call mirrors ------------------------------------------------------------------ */
static void test_mirrors(int iters) {
    for (int it = 0; it < iters; ++it) {
        const uint32_t n = rr(1, 300);
        uint64_t* fc = xmalloc(n * 8);
        uint64_t* fm = xmalloc(n * 8);
        uint64_t* cc = xmalloc(n * 8);
        uint64_t* cm = xmalloc(n * 8);
        for (uint32_t i = 0; i < n; ++i) {
            cc[i] = rr(1, 64);
            cm[i] = rr(1, 40000);
            fc[i] = rr(0, (uint32_t)cc[i]);
            fm[i] = rr(0, (uint32_t)cm[i]);
        }
        const uint64_t c = rr(0, 70), m = rr(0, 42000);
        int want = -1, lend = 0;
        for (uint32_t i = 0; i < n; ++i) {
            if (want < 0 && fc[i] >= c && fm[i] >= m) want = (int)i; /* scheduler.go:129-137 */
            if (fc[i] > c && fm[i] > m) lend = 1;                    /* scheduler.go:194-202 */
        }
        CHECK(or_schedule_job(n, fc, fm, c, m) == want, "first fit");
        CHECK(or_lend(n, fc, fm, c, m) == lend, "lend");
        uint32_t tc = 0, tm = 0;
        for (uint32_t i = 0; i < n; ++i) {
            tc += (uint32_t)cc[i];
            tm += (uint32_t)cm[i];
        }
        float cu = -1.0f, mu = -1.0f;
        or_resource_utilization(n, cc, cm, fc, fm, tc, tm, &cu, &mu);
        CHECK(cu >= 0.0f && cu <= 1.0f && mu >= 0.0f && mu <= 1.0f, "utilization %f %f", cu, mu);
        const int ap = or_approve_trade(tc, tm, cu, mu, rr(0, 2 * tc), rr(0, 2 * tm), (int64_t)rr(0, 1000) * 1000000000ll,
                                        0.0f);
        CHECK(ap == 0 || ap == 1, "approve %d", ap);

        /* AllocateVirtualNodeResources on counters that may already have wrapped (cluster.go:116) */
        uint32_t nf = 0, *fnode = xmalloc(n * 4);
        uint64_t *ffc = xmalloc(n * 8), *ffm = xmalloc(n * 8);
        if (it & 1) fc[rr(0, n - 1)] = (uint64_t)0 - rr(1, 5); /* a wrapped counter */
        const int rc = or_allocate_virtual_node(n, fc, fm, rr(0, 200), rr(0, 50000), &nf, fnode, ffc, ffm);
        CHECK((rc == 0 || rc == 1) && nf <= n, "allocate rc %d nf %u", rc, nf);
        for (uint32_t i = 0; i < nf; ++i) CHECK(fnode[i] < n, "foreign node");
        free(fnode);
        free(ffc);
        free(ffm);

        /* Go container/heap over contractResHeap: pops in ascending price */
        const uint32_t hn = rr(0, 40);
        float* pr = xmalloc(hn * 4 + 4);
        uint32_t* ord = xmalloc(hn * 4 + 4);
        int* seen = calloc(hn + 1, sizeof(int));
        for (uint32_t i = 0; i < hn; ++i) pr[i] = (float)rr(0, 3); /* many equal keys */
        or_heap_order(hn, pr, ord);
        for (uint32_t i = 0; i < hn; ++i) {
            CHECK(ord[i] < hn && !seen[ord[i]], "heap order not a permutation");
            if (ord[i] < hn) seen[ord[i]] = 1;
            if (i) CHECK(pr[ord[i - 1]] <= pr[ord[i]], "heap order not ascending");
        }
        free(pr);
        free(ord);
        free(seen);

        /* contract sizes over a Level1 list of any length (padded to ProvideJobs batches of 20) */
        const uint32_t ln = rr(0, 70);
        uint32_t *lc = xmalloc(ln * 4 + 4), *lm = xmalloc(ln * 4 + 4), *ld = xmalloc(ln * 4 + 4);
        for (uint32_t i = 0; i < ln; ++i) {
            lc[i] = rr(0, 64);
            lm[i] = rr(0, 40000);
            ld[i] = rr(0, 600);
        }
        uint32_t oc, om;
        int64_t ot;
        float op;
        or_contract_fast(ln, lc, lm, ld, &oc, &om, &ot, &op);
        or_contract_small(ln, lc, lm, ld, &oc, &om, &ot, &op);
        free(lc);
        free(lm);
        free(ld);
        free(fc);
        free(fm);
        free(cc);
        free(cm);
    }
}

int main(int argc, char** argv) {
    const uint64_t seed = argc > 1 ? strtoull(argv[1], NULL, 0) : 0x4D43535F53454C46ull;
    const int scale = argc > 2 ? atoi(argv[2]) : 1;
    g_state = seed;
    test_mirrors(400 * scale);
    test_fifo(40 * scale);
    test_delay(40 * scale);
    test_trade(12 * scale);
    test_dtrade(12 * scale);
    if (g_fail) {
        fprintf(stderr, "SELFTEST FAILED: %d checks\n", g_fail);
        return 1;
    }
    printf("SELFTEST OK seed 0x%llx scale %d\n", (unsigned long long)seed, scale);
    return 0;
}
