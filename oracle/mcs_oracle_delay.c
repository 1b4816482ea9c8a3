/*
 * mcs_oracle_delay.c — CPU ORACLE of the DELAY policy.  TEST INFRASTRUCTURE ONLY (see
 * mcs_oracle.h for the rules: only tests/, smoke() and bench.py's cpu_baseline may load it).
 *
 * Restates Scheduler.Delay (pkg/scheduler/scheduler.go:298-369), the shipped default policy
 * (scheduler.go:116), with the "/delay" ingestion handler (pkg/scheduler/server.go:53-78) and the
 * wait-time statistics WaitTime (scheduler.go:47-63).  Serialized semantics SDELAY (DESIGN.md
 * §10): every goroutine step completes before the next scheduler step; the clock is integer
 * seconds; each Delay iteration ends in time.Sleep(1 s) (:367), so iteration k runs at t = k.
 *
 * One iteration (tick) at time t:
 *   0. Node.RunJob releases every job with finish <= t (cluster.go:153-157; D3) and the "/delay"
 *      handler appends every arrival <= t to Level0 with WaitTime = its arrival time,
 *      JobsMap[id] = 0 and JobsCount += 1 (server.go:67-74).
 *   1. Level1 pass (:302-329): for i := 0; i < len(Level1); i++ { ScheduleJob(Level1[i]);
 *      TotalTime -= JobsMap[id]; JobsMap[id] = since(WaitTime) ms; TotalTime += JobsMap[id];
 *      on success delete(JobsMap, id) and Level1 = append(Level1[:i], Level1[i+1:]...) }.
 *      The removal has no i-- (deviation D6, replicated as written): the job that slides into
 *      slot i is not examined in this pass.
 *   2. Level0 head (:332-366): ScheduleJob(Level0[0]) with the same statistics update; success
 *      pops it; failure moves it to the tail of Level1 once since(WaitTime) >= MaxWaitTime
 *      (10 s, scheduler.go:115,353).
 *   3. time.Sleep(1 s) (:367): t += 1.
 * ScheduleJob is first fit with '>=' (scheduler.go:127-139), committed synchronously (D2).
 * since(WaitTime) is (t - arrival) whole seconds, so JobsMap values are 1000 * whole seconds
 * (D10: the serialized clock has no sub-second phase between ticks and arrivals).
 *
 * The run ends at the top of the first iteration where every job has been placed (t_end = that
 * t, like the FIFO oracle), or — when some Level1 jobs can never fit — at the end of the first
 * iteration that placed nothing while nothing runs, Level0 is empty and every job has arrived:
 * the Go loop would retry those jobs forever on a frozen cluster.  They are reported unplaced
 * (node -1, MCS_TIME_NONE), flags bit 0 is set and t_end is that iteration's t.
 *
 * Fast-forward (literal == 0) jumps over iterations that cannot change any placement: after an
 * iteration that placed nothing and moved nothing, every later iteration fails the same way until
 * the next release (min finish), the Level0 head's MaxWaitTime move (arrival + 10) or, with an
 * empty Level0, the next arrival.  The skipped iterations still examine every Level1 job and the
 * Level0 head, so their JobsMap entries are set to the last skipped t — the statistics match the
 * literal loop exactly, which tests/test_delay_oracle.py asserts.
 */
#include <stdlib.h>
#include <string.h>

#include "mcs_oracle.h"

typedef struct {
    uint32_t finish, node;
    uint64_t c, m;
} dl_run;

typedef struct {
    uint32_t n;
    uint64_t *fc, *fm;
    dl_run* run;
    uint64_t nrun, caprun;
} dl_cluster;

/* Node.RunJob commit (cluster.go:144-148), synchronous (D2); sleep(Duration) -> finish. */
static void dl_run_job(dl_cluster* cl, uint32_t k, uint64_t c, uint64_t m, uint32_t t, uint32_t dur) {
    cl->fc[k] -= c;
    cl->fm[k] -= m;
    if (dur == 0) { /* RunJob sleeps 0 and releases before the next scheduler step */
        cl->fc[k] += c;
        cl->fm[k] += m;
        return;
    }
    if (cl->nrun == cl->caprun) {
        cl->caprun = cl->caprun ? 2 * cl->caprun : 64;
        cl->run = (dl_run*)realloc(cl->run, cl->caprun * sizeof(dl_run));
    }
    dl_run r = {t + dur, k, c, m};
    cl->run[cl->nrun++] = r;
}

/* Node.RunJob completion (cluster.go:153-157). */
static void dl_release(dl_cluster* cl, uint32_t t) {
    for (uint64_t i = 0; i < cl->nrun;) {
        if (cl->run[i].finish <= t) {
            cl->fc[cl->run[i].node] += cl->run[i].c;
            cl->fm[cl->run[i].node] += cl->run[i].m;
            cl->run[i] = cl->run[--cl->nrun];
        } else {
            ++i;
        }
    }
}

static uint32_t dl_min_finish(const dl_cluster* cl) {
    uint32_t mf = 0xFFFFFFFFu;
    for (uint64_t i = 0; i < cl->nrun; ++i)
        if (cl->run[i].finish < mf) mf = cl->run[i].finish;
    return mf;
}

/* WaitTime update of one examined job (scheduler.go:309-312 / 338-341). */
static void dl_touch(int64_t* jobs_map, int64_t* total, uint64_t j, uint32_t t, uint32_t arr) {
    *total -= jobs_map[j];
    jobs_map[j] = (int64_t)(t - arr) * 1000; /* time.Since(WaitTime).Milliseconds(), D10 */
    *total += jobs_map[j];
}

int or_delay_run(uint32_t n_nodes, const uint32_t* free_c, const uint32_t* free_m, uint64_t n_jobs,
                 const uint32_t* arrival, const uint32_t* dur, const uint32_t* cores,
                 const uint32_t* mem, uint32_t max_wait_s, int literal, int32_t* out_node,
                 uint32_t* out_start, uint32_t* out_finish, or_delay_stats* st) {
    dl_cluster cl;
    memset(&cl, 0, sizeof cl);
    cl.n = n_nodes;
    cl.fc = (uint64_t*)malloc(sizeof(uint64_t) * (n_nodes ? n_nodes : 1));
    cl.fm = (uint64_t*)malloc(sizeof(uint64_t) * (n_nodes ? n_nodes : 1));
    for (uint32_t i = 0; i < n_nodes; ++i) { /* Run keeps the JSON availability (KAT5) */
        cl.fc[i] = free_c[i];
        cl.fm[i] = free_m[i];
    }
    const uint64_t nj1 = n_jobs ? n_jobs : 1;
    uint64_t* l0 = (uint64_t*)malloc(sizeof(uint64_t) * nj1); /* Level0 slice */
    uint64_t* l1 = (uint64_t*)malloc(sizeof(uint64_t) * nj1); /* Level1 slice */
    int64_t* jobs_map = (int64_t*)calloc(nj1, sizeof(int64_t)); /* WaitTime.JobsMap (0 = absent) */
    uint64_t l0_head = 0, l0_tail = 0, l1_len = 0, next_arrival = 0, decided = 0, ticks = 0;
    int64_t total = 0, count = 0;
    uint32_t t = 0, flags = 0, moved = 0, placed_l1 = 0, peak_l1 = 0, peak_run = 0;

    for (uint64_t j = 0; j < n_jobs; ++j) {
        out_node[j] = -1;
        out_start[j] = 0xFFFFFFFFu;
        out_finish[j] = 0xFFFFFFFFu;
    }

    for (;;) {
        ++ticks;
        dl_release(&cl, t);
        while (next_arrival < n_jobs && arrival[next_arrival] <= t) { /* server.go:67-74 */
            jobs_map[next_arrival] = 0;
            ++count;
            l0[l0_tail++] = next_arrival++;
        }
        if (decided == n_jobs) break;
        int changed = 0;

        /* ---- Level1 pass, scheduler.go:302-329 ---- */
        for (uint64_t i = 0; i < l1_len; i++) {
            const uint64_t j = l1[i];
            const int k = or_schedule_job(cl.n, cl.fc, cl.fm, cores[j], mem[j]); /* :307 */
            dl_touch(jobs_map, &total, j, t, arrival[j]);                       /* :309-312 */
            if (k >= 0) {
                dl_run_job(&cl, (uint32_t)k, cores[j], mem[j], t, dur[j]);
                out_node[j] = k;
                out_start[j] = t;
                out_finish[j] = t + dur[j];
                jobs_map[j] = 0; /* delete(JobsMap, id) (:316); TotalTime keeps its share */
                memmove(l1 + i, l1 + i + 1, sizeof(uint64_t) * (l1_len - i - 1)); /* :319, no i-- */
                --l1_len;
                ++decided;
                ++placed_l1;
                changed = 1;
                if (cl.nrun > peak_run) peak_run = (uint32_t)cl.nrun;
            }
        }

        /* ---- Level0 head, scheduler.go:332-366 ---- */
        if (l0_tail > l0_head) {
            const uint64_t j = l0[l0_head];
            const int k = or_schedule_job(cl.n, cl.fc, cl.fm, cores[j], mem[j]); /* :335 */
            dl_touch(jobs_map, &total, j, t, arrival[j]);                       /* :338-341 */
            if (k >= 0) {
                dl_run_job(&cl, (uint32_t)k, cores[j], mem[j], t, dur[j]);
                out_node[j] = k;
                out_start[j] = t;
                out_finish[j] = t + dur[j];
                jobs_map[j] = 0; /* :346 */
                ++l0_head;       /* Level0 = Level0[1:] (:347) */
                ++decided;
                changed = 1;
                if (cl.nrun > peak_run) peak_run = (uint32_t)cl.nrun;
            } else if (t - arrival[j] >= max_wait_s) { /* time.Since(WaitTime) >= MaxWaitTime :353 */
                l1[l1_len++] = j; /* Level1 = append(Level1, Level0[0]) (:357) */
                ++l0_head;        /* Level0 = Level0[1:] (:358) */
                ++moved;
                changed = 1;
                if (l1_len > peak_l1) peak_l1 = (uint32_t)l1_len;
            }
        }

        /* Level1 jobs that can never fit: nothing runs, nothing is queued or still to arrive, and
         * this pass placed nothing, so every later pass fails the same way forever. */
        if (!changed && cl.nrun == 0 && l0_tail == l0_head && next_arrival == n_jobs) {
            flags |= 1u;
            break;
        }

        /* ---- time.Sleep(1 s), scheduler.go:367 ---- */
        uint32_t tn = t + 1u;
        if (!literal && !changed) {
            uint32_t ev = dl_min_finish(&cl);
            if (l0_tail > l0_head) {
                const uint32_t mv = arrival[l0[l0_head]] + max_wait_s;
                if (mv < ev) ev = mv;
            } else if (next_arrival < n_jobs && arrival[next_arrival] < ev) {
                ev = arrival[next_arrival];
            }
            if (ev > tn) {
                /* iterations tn .. ev-1 examine every Level1 job and the Level0 head and fail */
                const uint32_t last = ev - 1u;
                for (uint64_t i = 0; i < l1_len; ++i)
                    dl_touch(jobs_map, &total, l1[i], last, arrival[l1[i]]);
                if (l0_tail > l0_head)
                    dl_touch(jobs_map, &total, l0[l0_head], last, arrival[l0[l0_head]]);
                ticks += (uint64_t)(ev - tn);
                tn = ev;
            }
        }
        if (tn < t) { /* u32 clock wrap (D8 range exceeded) */
            flags |= 4u;
            break;
        }
        t = tn;
    }

    if (st) {
        st->t_end = t;
        st->placed = (uint32_t)decided;
        st->moved_l1 = moved;
        st->placed_l1 = placed_l1;
        st->peak_l1 = peak_l1;
        st->peak_running = peak_run;
        st->flags = flags;
        st->l1_left = (uint32_t)l1_len;
        st->total_wait_ms = total;
        st->jobs_count = count;
        st->ticks = ticks;
    }
    free(cl.fc);
    free(cl.fm);
    free(cl.run);
    free(l0);
    free(l1);
    free(jobs_map);
    return 0;
}

int or_delay_run_batch(uint32_t n_clusters, const uint32_t* node_off, const uint32_t* free_c,
                       const uint32_t* free_m, const uint64_t* job_off, const uint32_t* arrival,
                       const uint32_t* dur, const uint32_t* cores, const uint32_t* mem,
                       uint32_t max_wait_s, int n_threads, int32_t* out_node, uint32_t* out_start,
                       uint32_t* out_finish, or_delay_stats* st) {
#ifdef _OPENMP
    if (n_threads < 1) n_threads = 1;
#pragma omp parallel for schedule(dynamic, 1) num_threads(n_threads)
#else
    (void)n_threads;
#endif
    for (int64_t c = 0; c < (int64_t)n_clusters; ++c) {
        const uint32_t n0 = node_off[c], nn = node_off[c + 1] - node_off[c];
        const uint64_t j0 = job_off[c], jn = job_off[c + 1] - job_off[c];
        or_delay_run(nn, free_c + n0, free_m + n0, jn, arrival + j0, dur + j0, cores + j0, mem + j0,
                     max_wait_s, 0, out_node + j0, out_start + j0, out_finish + j0,
                     st ? st + c : 0);
    }
    return 0;
}
