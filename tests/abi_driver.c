/*
 * abi_driver.c — a plain C99 caller of libmcs.so through include/mcs.h, as the cgo binding of
 * INTEGRATION.md would call it (tests/test_gpu_abi_driver.py builds it with gcc and runs it on the
 * GPU).  It replaces, per SURVEY §8(b), the reference's Scheduler.Run + Fifo goroutine
 * (pkg/scheduler/scheduler.go:101-124, 216-296) over ScheduleJob (:127-139):
 *
 *   1. KAT2 (head-of-line blocking and the +1 s after a wait success) as a
 *      batch run: mcs_engine_create -> mcs_load_clusters -> mcs_submit_jobs -> mcs_run ->
 *      mcs_read_placements, checked against the hand-derived answer;
 *   2. the same jobs driven online, as the Go loop fed by HTTP POSTs would see them: appended in
 *      two POST batches, the clock advanced in horizons, every intermediate result checked;
 *   3. the single-job mirrors ScheduleJob / RunJob release / Lend / GetResourceUtilization;
 *   4. the error convention: MCS_NO_FIT with the Go error text, MCS_E_INVALID / MCS_E_STATE.
 *
 * Prints ABI-DRIVER OK and exits 0 on success.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mcs.h"

static int failures = 0;
#define CHECK(cond, ...)                                          \
    do {                                                          \
        if (!(cond)) {                                            \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);  \
            fprintf(stderr, __VA_ARGS__);                         \
            fprintf(stderr, "\n");                                \
            ++failures;                                           \
        }                                                         \
    } while (0)
#define OK(call)                                                                            \
    do {                                                                                    \
        int rc_ = (call);                                                                   \
        if (rc_ != MCS_OK) {                                                                \
            fprintf(stderr, "FAIL %s:%d: %s -> %d (%s)\n", __FILE__, __LINE__, #call, rc_,  \
                    eng ? mcs_last_error(eng) : "");                                        \
            exit(2);                                                                        \
        }                                                                                   \
    } while (0)

/* assets/cluster_small.json: 5 nodes x {Cores 32, Memory 24000}, fully available */
static const uint32_t cap_c[5] = {32, 32, 32, 32, 32}, cap_m[5] = {24000, 24000, 24000, 24000, 24000};
static const uint32_t node_off[2] = {0, 5};

/* KAT2: jobs (i, 0, 32 cores, 1 mem, 10 s) for i = 0..5, then (6, 0, 0 cores, 1 mem, 3 s) */
static const uint32_t arr[7] = {0, 0, 0, 0, 0, 0, 0}, dur[7] = {10, 10, 10, 10, 10, 10, 3};
static const uint32_t cores[7] = {32, 32, 32, 32, 32, 32, 0}, mem[7] = {1, 1, 1, 1, 1, 1, 1};
/* 0..4 -> (i, 0, 10); 5 -> (0, 10, 20); 6 -> (0, 11, 14) */
static const int32_t want_node[7] = {0, 1, 2, 3, 4, 0, 0};
static const uint32_t want_start[7] = {0, 0, 0, 0, 0, 10, 11}, want_fin[7] = {10, 10, 10, 10, 10, 20, 14};

static void check_rows(mcs_engine* eng, int n_decided_max, uint32_t horizon, const char* what) {
    int32_t node[7];
    uint32_t st[7], fi[7];
    OK(mcs_read_placements(eng, node, st, fi));
    for (int j = 0; j < 7; ++j) {
        const int decided = want_start[j] < horizon && j < n_decided_max;
        if (decided) {
            CHECK(node[j] == want_node[j] && st[j] == want_start[j] && fi[j] == want_fin[j],
                  "%s: job %d got (%d, %u, %u) want (%d, %u, %u)", what, j, node[j], st[j], fi[j], want_node[j],
                  want_start[j], want_fin[j]);
        } else {
            CHECK(node[j] == MCS_NODE_UNPLACED && st[j] == MCS_TIME_NONE && fi[j] == MCS_TIME_NONE,
                  "%s: job %d should be undecided, got (%d, %u, %u)", what, j, node[j], st[j], fi[j]);
        }
    }
}

int main(void) {
    mcs_engine* eng = NULL;
    mcs_config cfg;
    mcs_config_default(&cfg);
    CHECK(mcs_abi_version() == MCS_ABI_VERSION, "ABI version %d", mcs_abi_version());
    OK(mcs_engine_create(&cfg, 0, &eng));

    /* 4. calls out of order fail with MCS_E_STATE, bad arguments with MCS_E_INVALID */
    mcs_stats stats;
    CHECK(mcs_run(eng, MCS_TIME_NONE, &stats) == MCS_E_STATE, "run before load");
    CHECK(mcs_load_clusters(eng, cap_c, cap_m, cap_c, cap_m, node_off, 0) == MCS_E_INVALID, "zero clusters");

    /* 1. batch run of KAT2 */
    OK(mcs_load_clusters(eng, cap_c, cap_m, cap_c, cap_m, node_off, 1));
    const uint64_t job_off[2] = {0, 7};
    OK(mcs_submit_jobs(eng, arr, dur, cores, mem, job_off));
    OK(mcs_run(eng, MCS_TIME_NONE, &stats));
    CHECK(stats.placed == 7 && stats.unplaced == 0 && stats.waited == 1, "batch stats %llu %llu %llu",
          (unsigned long long)stats.placed, (unsigned long long)stats.unplaced, (unsigned long long)stats.waited);
    check_rows(eng, 7, MCS_TIME_NONE, "batch");
    mcs_cluster_stats cs;
    OK(mcs_read_cluster_stats(eng, &cs, 1));
    CHECK(cs.placed == 7 && cs.flags == 0, "cluster stats");

    /* 2. online: POST jobs 0..3, advance to t = 5; POST 4..6 (arriving at 5 here, so the answer
     * shifts: recompute by hand below), then horizons 11, 12 and a drain */
    OK(mcs_load_clusters(eng, cap_c, cap_m, cap_c, cap_m, node_off, 1)); /* resets the streams */
    const uint64_t first_off[2] = {0, 7};
    OK(mcs_append_jobs(eng, arr, dur, cores, mem, first_off)); /* all seven POSTed at t = 0 */
    OK(mcs_run(eng, 1, &stats));                               /* every decision at t < 1 */
    CHECK(stats.online == 1 && stats.t_horizon == 1, "online flags");
    CHECK(stats.placed == 5 && stats.pending == 2, "after t<1: placed %llu pending %llu",
          (unsigned long long)stats.placed, (unsigned long long)stats.pending);
    check_rows(eng, 7, 1, "horizon 1");
    OK(mcs_run(eng, 11, &stats)); /* job 5 placed at 10 (the wait head), job 6 at 11 not yet */
    check_rows(eng, 7, 11, "horizon 11");
    CHECK(mcs_run(eng, 10, &stats) == MCS_E_INVALID, "decreasing horizon");
    OK(mcs_run(eng, 12, &stats));
    check_rows(eng, 7, 12, "horizon 12");
    CHECK(stats.placed == 7 && stats.pending == 0, "after t<12");
    /* a later POST: arrives at 30 on an idle cluster (job 5 still runs on node 0 until 20) */
    const uint32_t a2[1] = {30}, d2[1] = {1}, c2[1] = {32}, m2[1] = {24000};
    const uint64_t off2[2] = {0, 1};
    const uint32_t a_bad[1] = {11};
    CHECK(mcs_append_jobs(eng, a_bad, d2, c2, m2, off2) == MCS_E_INVALID, "arrival before the horizon");
    OK(mcs_append_jobs(eng, a2, d2, c2, m2, off2));
    OK(mcs_run(eng, MCS_TIME_NONE, &stats));
    uint64_t doff[2];
    OK(mcs_read_job_offsets(eng, doff));
    CHECK(doff[0] == 0 && doff[1] == 8 && mcs_num_jobs(eng) == 8, "dense offsets");
    int32_t node[8];
    uint32_t st[8], fi[8];
    OK(mcs_read_placements(eng, node, st, fi));
    CHECK(node[7] == 0 && st[7] == 30 && fi[7] == 31, "late POST got (%d, %u, %u)", node[7], st[7], fi[7]);

    /* 3. single-job mirrors over the live state (a fresh spec) */
    OK(mcs_load_clusters(eng, cap_c, cap_m, cap_c, cap_m, node_off, 1));
    int32_t k = -9;
    OK(mcs_schedule_one(eng, 0, 20, 1000, &k));
    CHECK(k == 0, "schedule_one -> %d", k);
    OK(mcs_schedule_one(eng, 0, 20, 1000, &k));
    CHECK(k == 1, "schedule_one -> %d", k);
    CHECK(mcs_schedule_one(eng, 0, 33, 1, &k) == MCS_NO_FIT && k == MCS_NODE_UNPLACED, "no fit");
    CHECK(strcmp(mcs_last_error(eng), "not enough resources in cluster") == 0, "Go error text: %s",
          mcs_last_error(eng));
    int32_t lend = -1;
    OK(mcs_lend_check(eng, 0, 31, 23999, &lend));
    CHECK(lend == 1, "lend 31/23999");
    OK(mcs_lend_check(eng, 0, 32, 1, &lend));
    CHECK(lend == 0, "lend 32 (strict >)");
    float cu = -1.0f, mu = -1.0f;
    OK(mcs_resource_utilization(eng, 0, &cu, &mu));
    CHECK(cu == 40.0f / 160.0f && mu == 2000.0f / 120000.0f, "utilization %g %g", cu, mu);
    OK(mcs_release_one(eng, 0, 0, 20, 1000));
    uint32_t fc[5], fm[5];
    OK(mcs_read_live_state(eng, 0, fc, fm, 5));
    CHECK(fc[0] == 32 && fc[1] == 12 && fm[1] == 23000, "live state");

    OK(mcs_engine_destroy(eng));
    eng = NULL;
    if (failures) {
        fprintf(stderr, "%d check(s) failed\n", failures);
        return 1;
    }
    printf("ABI-DRIVER OK\n");
    return 0;
}
