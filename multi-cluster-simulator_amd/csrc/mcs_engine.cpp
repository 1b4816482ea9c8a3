// mcs_engine.cpp — C ABI of libmcs.so (include/mcs.h): device memory, HBM layout, launch policy,
// slot-pool escalation and the single-job mirrors.  Host code; compiled by hipcc.
//
// No CPU fallback exists anywhere in this library: every placement decision is made by a gfx950
// kernel (mcs_kernels.hip).  If no HIP device is usable every compute entry point fails with
// MCS_E_HIP and a message.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "mcs_engine_impl.h"
#include "mcs_gen.h"
#include "mcs_internal.h"

namespace {

void free_clusters(mcs_engine* e) {
    dfree(e->d_free0);
    dfree(e->d_cap);
    dfree(e->d_node_off);
    dfree(e->d_live_c);
    dfree(e->d_live_m);
    dfree(e->d_max_c);
    dfree(e->d_max_m);
    dfree(e->d_cstats);
    dfree(e->d_dstats);
    dfree(e->d_list);
}

void free_jobs(mcs_engine* e) {
    mcs::online_free(e);  // a new stream ends any online session
    e->bounds_known = false;
    dfree(e->d_jobs);
    dfree(e->d_gen_max);
    dfree(e->d_wthr);
    e->gen = mcs::GenArgs{};
    dfree(e->d_job_off);
    dfree(e->d_out_node);
    dfree(e->d_out_start);
    dfree(e->d_out_finish);
    dfree(e->d_l1_cm);
    dfree(e->d_l1_jd);
}

}  // namespace

namespace mcs {
int npl_for(uint32_t max_n) {
    const int opts[] = {1, 2, 4, 8, 16};
    for (int o : opts)
        if ((uint32_t)(o * kWave) >= max_n) return o;
    return -1;
}

// Initial running-slot pool (slot rows of 64): room for ~2 running jobs per node, rounded to a
// power of two in [2, 32] (the C4 workload peaks at ~1.7 per node).  Escalation doubles it for the
// clusters that overflow, so the choice only trades occupancy against rare re-runs.
int auto_pool(uint32_t max_n) {
    const uint32_t want = (2u * max_n + 63u) / 64u;
    int p = 2;
    while ((uint32_t)p < want && p < kMaxPool) p *= 2;
    return p;
}

int ensure_job_records(mcs_engine* e) {
    if (e->d_jobs) return MCS_OK;
    const size_t nj = e->total_jobs ? e->total_jobs : 1;
    HIPCHK(e, hipMalloc(&e->d_jobs, (nj + kJobPad) * sizeof(uint4)));
    HIPCHK(e, hipMemsetAsync(e->d_jobs + nj, 0, kJobPad * sizeof(uint4), e->stream));
    // MCS_GEN_SERIAL=1: the per-thread scan (tests compare the two forms)
    const char* serial = getenv("MCS_GEN_SERIAL");
    bool wave_form = e->job_off.size() == (size_t)e->C + 1 && !(serial && atoi(serial) != 0);
    for (uint32_t c = 0; wave_form && c < e->C; ++c)
        wave_form = e->job_off[c + 1] - e->job_off[c] < (1ull << 32);
    hipError_t st;
    if (wave_form) {
        st = launch_gen_stream(e->d_jobs, e->d_job_off, e->C, e->gen, e->stream);
    } else {
        st = launch_gen_attrs(e->d_jobs, e->d_job_off, e->gen.max_c, e->gen.max_m, e->C, e->gen.seed,
                              e->gen.max_dur, e->gen.base, e->stream);
        if (st == hipSuccess) st = launch_gen_arrivals(e->d_jobs, e->d_job_off, e->C, e->gen, e->stream);
    }
    if (st == hipSuccess) st = hipStreamSynchronize(e->stream);
    if (st != hipSuccess)
        return fail(e, MCS_E_HIP, std::string("job generation: ") + hipGetErrorString(st));
    return MCS_OK;
}
}  // namespace mcs

extern "C" {

int mcs_abi_version(void) { return MCS_ABI_VERSION; }

void mcs_config_default(mcs_config* cfg) {
    if (!cfg) return;
    std::memset(cfg, 0, sizeof(*cfg));
    cfg->policy = MCS_POLICY_FIFO;
    cfg->borrow = 0;
    cfg->trader = 0;
    cfg->wait_sleep_s = 1; /* scheduler.go:250 */
    cfg->idle_sleep_s = 1; /* scheduler.go:294 */
    cfg->slot_pool = 0;
    cfg->trader_period_s = 10;     /* trader.go:323 */
    cfg->trade_ok_sleep_s = 240;   /* trader.go:297 */
    cfg->trade_fail_sleep_s = 120; /* trader.go:300 */
    cfg->lock_s = 20;              /* pkg/trader/server.go:49 */
    cfg->sample_period_s = 5;      /* trader_server.go:44 */
    cfg->lent_queue_cap = 0;
    cfg->t_max_s = 0;
    cfg->max_wait_s = 10; /* sched.Policy.MaxWaitTime = 10 * time.Second, scheduler.go:115 */
}

/* the Weibull gap table of mcs_gen.h: thr[n-1] = floor(2^64 exp(-(n/scale)^k)) while nonzero.
 * Returns its length, or -1 if it does not vanish within MCS_GEN_WEIBULL_MAX entries. */
static int weibull_table(double scale, double k, uint64_t* thr) {
    if (!(scale > 0.0) || !(k > 0.0)) return -1;
    for (uint32_t n = 1; n <= MCS_GEN_WEIBULL_MAX; ++n) {
        const double p = std::exp(-std::pow((double)n / scale, k));
        const double v = std::ldexp(p, 64);
        if (v < 1.0) return (int)n - 1;
        thr[n - 1] = v >= 18446744073709551615.0 ? 0xFFFFFFFFFFFFFFFFull : (uint64_t)v;
    }
    return -1;
}

static bool gen_params_ok(const mcs_gen_params* p) {
    if (!p || p->arrival_mode > 2u || p->max_dur_s == 0 || p->fused > 1u) return false;
    if (p->arrival_mode == 2u) {
        uint64_t thr[MCS_GEN_WEIBULL_MAX];
        return weibull_table(p->lambda, p->weibull_k > 0.0f ? p->weibull_k : 3.0, thr) >= 0;
    }
    return p->lambda > 0.0 && p->lambda <= 128.0;
}

void mcs_gen_params_default(mcs_gen_params* p) {
    if (!p) return;
    std::memset(p, 0, sizeof(*p));
    p->seed = MCS_GEN_SEED_DEFAULT;
    p->arrival_mode = MCS_ARRIVAL_REF;
    p->max_dur_s = 600; /* rand.Intn(600), client.go:98 */
    p->lambda = 10.0;   /* distuv.Poisson{Lambda: 10}, client.go:107-110 */
    p->max_cores = 0;
    p->max_mem = 0;
}

int mcs_gen_cluster_host(const mcs_gen_params* p, uint32_t cluster, uint32_t max_cores,
                         uint32_t max_mem, uint64_t n_jobs, uint32_t* arrival_s, uint32_t* dur_s,
                         uint32_t* cores, uint32_t* mem) {
    if (!p || (n_jobs && (!arrival_s || !dur_s || !cores || !mem))) return MCS_E_INVALID;
    if (!gen_params_ok(p)) return MCS_E_INVALID;
    const uint64_t key = mcs_cluster_key(p->seed, cluster);
    for (uint64_t i = 0; i < n_jobs; ++i)
        mcs_gen_job_attrs(key, i, max_cores, max_mem, p->max_dur_s, &dur_s[i], &cores[i], &mem[i]);
    uint64_t thr[MCS_GEN_WEIBULL_MAX];
    int wn = 0;
    if (p->arrival_mode == 2u) wn = weibull_table(p->lambda, p->weibull_k > 0.0f ? p->weibull_k : 3.0, thr);
    mcs_gen_arrivals(key, p->arrival_mode, std::exp(-p->lambda), thr, (uint32_t)wn, n_jobs, arrival_s);
    return MCS_OK;
}

double mcs_gen_scaled_lambda(uint32_t n_nodes, uint32_t node_mem, uint32_t max_mem,
                             uint32_t max_dur_s, double load) {
    const double e_mem = 0.5 * (double)max_mem - 0.5;   /* E[floor(B*max)], B ~ Beta(2,2) */
    const double e_dur = 0.5 * ((double)max_dur_s - 1.0); /* E[U{0..max-1}] */
    if (e_mem <= 0.0 || e_dur <= 0.0) return 0.0;
    return load * (double)n_nodes * (double)node_mem / (e_mem * e_dur);
}

int mcs_engine_create(const mcs_config* cfg, int device, mcs_engine** out) {
    if (!out) return MCS_E_INVALID;
    *out = nullptr;
    mcs_config c;
    if (cfg)
        c = *cfg;
    else
        mcs_config_default(&c);
    if (c.policy > MCS_POLICY_DELAY || c.borrow > 1 || c.trader > 1 || c.wait_sleep_s != 1 ||
        c.idle_sleep_s != 1)
        return MCS_E_INVALID; /* FIFO or DELAY with the reference sleeps */
    if (c.policy == MCS_POLICY_DELAY && c.borrow)
        return MCS_E_INVALID; /* Delay never borrows (scheduler.go:298-369) */
    if (c.policy == MCS_POLICY_DELAY && c.max_wait_s == 0) return MCS_E_INVALID;
    if (c.borrow || c.trader) {
        if (c.trader && (c.trader_period_s == 0 || c.sample_period_s == 0 || c.lock_s == 0))
            return MCS_E_INVALID;
        if (c.trader && c.trader_period_s % c.sample_period_s != 0)
            return MCS_E_INVALID; /* rounds must fall on state samples */
        if (c.slot_pool > 64) return MCS_E_INVALID; /* lock-step slots: 64 * slot_pool <= 4096 */
        if (c.unchecked_horizon)
            return MCS_E_INVALID; /* the lock-step kernels carry no run-time clock guard: keep the
                                     host bound */
    } else if (c.slot_pool != 0 && !mcs::fifo_variant_exists(1, (int)c.slot_pool)) {
        return MCS_E_INVALID;
    }
    mcs_engine* e = new (std::nothrow) mcs_engine();
    if (!e) return MCS_E_NOMEM;
    e->cfg = c;
    e->device = device;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
        delete e;
        return MCS_E_HIP;
    }
    if (hipSetDevice(device) != hipSuccess ||
        hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&e->ev0) != hipSuccess || hipEventCreate(&e->ev1) != hipSuccess ||
        hipMalloc(&e->d_totals, sizeof(mcs::Totals)) != hipSuccess ||
        hipMalloc(&e->d_scratch, 64) != hipSuccess || hipMalloc(&e->d_util, 64) != hipSuccess) {
        mcs_engine_destroy(e);
        return MCS_E_HIP;
    }
    *out = e;
    return MCS_OK;
}

int mcs_engine_destroy(mcs_engine* e) {
    if (!e) return MCS_E_INVALID;
    (void)hipSetDevice(e->device);
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    // teardown order: the captured tick graphs (they reference RCCL resources), then the RCCL
    // communicator (finalized: no proxy work outstanding), then device memory, events and the stream
    mcs::trade_release_graphs(e);
    mcs::dtrade_release_graphs(e);
    mcs::comm_free(e);
    if (e->stream) (void)hipStreamSynchronize(e->stream);  // (this engine's work only: not the device's)
    mcs::trade_free(e);
    mcs::dtrade_free(e);
    mcs::online_free(e);
    free_clusters(e);
    free_jobs(e);
    dfree(e->d_totals);
    dfree(e->d_scratch);
    dfree(e->d_util);
    if (e->ev0) (void)hipEventDestroy(e->ev0);
    if (e->ev1) (void)hipEventDestroy(e->ev1);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
    return MCS_OK;
}

const char* mcs_last_error(const mcs_engine* e) { return e ? e->err.c_str() : "null engine"; }
const char* mcs_last_kernel(const mcs_engine* e) { return e ? e->last_kernel : ""; }

uint32_t mcs_num_clusters(const mcs_engine* e) { return e ? e->C : 0; }
uint64_t mcs_num_jobs(const mcs_engine* e) { return e ? e->total_jobs : 0; }

int mcs_load_clusters(mcs_engine* e, const uint32_t* cap_c, const uint32_t* cap_m,
                      const uint32_t* free_c, const uint32_t* free_m,
                      const uint32_t* node_offsets, uint32_t n_clusters) {
    if (int st = check_engine(e)) return st;
    if (!node_offsets || n_clusters == 0) return fail(e, MCS_E_INVALID, "no clusters");
    if (node_offsets[0] != 0) return fail(e, MCS_E_INVALID, "node_offsets[0] must be 0");
    uint32_t max_n = 0;
    for (uint32_t c = 0; c < n_clusters; ++c) {
        if (node_offsets[c + 1] < node_offsets[c])
            return fail(e, MCS_E_INVALID, "node_offsets must be non-decreasing");
        max_n = std::max(max_n, node_offsets[c + 1] - node_offsets[c]);
    }
    if (max_n > (uint32_t)(mcs::kMaxNpl * mcs::kWave))
        return fail(e, MCS_E_INVALID, "more than 1024 nodes in a cluster (ABI v1 limit)");
    const uint64_t nn = node_offsets[n_clusters];
    if (nn && (!cap_c || !cap_m || !free_c || !free_m))
        return fail(e, MCS_E_INVALID, "null node array");

    HIPCHK(e, hipStreamSynchronize(e->stream));
    free_clusters(e);
    free_jobs(e);
    mcs::trade_free(e);
    mcs::dtrade_free(e);
    e->has_clusters = e->has_jobs = e->has_run = false;
    e->dt_learn_s = e->dt_learn_v = 0;
    e->tr_agreed = false;  // (an agreed block layout belongs to the clusters it was agreed for)
    e->tr_ns = e->dt_ns = 0;
    e->C = n_clusters;
    e->max_n = max_n;
    e->total_nodes = nn;
    e->total_jobs = 0;
    e->node_off.assign(node_offsets, node_offsets + n_clusters + 1);
    e->job_off.clear();

    std::vector<uint2> free0(nn ? nn : 1), cap(nn ? nn : 1);
    std::vector<uint32_t> lc(nn ? nn : 1), lm(nn ? nn : 1), mxc(n_clusters), mxm(n_clusters);
    e->free_lt31 = e->free_lt15 = true;
    for (uint64_t i = 0; i < nn; ++i) {
        free0[i] = make_uint2(free_c[i], free_m[i]);
        if (free_c[i] >= 0x7FFFFFFFu || free_m[i] >= 0x7FFFFFFFu) e->free_lt31 = false;
        if (free_c[i] >= 0x7FFFu || free_m[i] >= 0x7FFFu) e->free_lt15 = false;
        cap[i] = make_uint2(cap_c[i], cap_m[i]);
        lc[i] = free_c[i];
        lm[i] = free_m[i];
    }
    e->sums_lt24 = true;
    e->slot_pack_ok = true;
    e->cores_le64 = true;
    for (uint32_t c = 0; c < n_clusters; ++c) { /* setMaxCluster, client.go:68-83 */
        uint32_t a = 0, b = 0;
        uint64_t sc = 0, sm = 0;
        for (uint32_t i = node_offsets[c]; i < node_offsets[c + 1]; ++i) {
            a = std::max(a, cap_c[i]);
            b = std::max(b, cap_m[i]);
            sc += std::max(cap_c[i], free_c[i]);
            sm += std::max(cap_m[i], free_m[i]);
            /* a placed job's request fits some node's free value: the workgroup-resident tick
             * packs a running slot's {cores, memory} into 7 + 16 bits (mcs_trade_mw.hip) */
            if (std::max(cap_c[i], free_c[i]) > 127u || std::max(cap_m[i], free_m[i]) > 0xFFFFu)
                e->slot_pack_ok = false;
            if (std::max(cap_c[i], free_c[i]) > 64u) e->cores_le64 = false;
        }
        mxc[c] = a;
        mxm[c] = b;
        /* every partial sum of GetResourceUtilization's float32 loop is then an exact integer */
        if (sc >= (1ull << 24) || sm >= (1ull << 24)) e->sums_lt24 = false;
    }
    const size_t nb = (nn ? nn : 1);
    HIPCHK(e, hipMalloc(&e->d_free0, nb * sizeof(uint2)));
    HIPCHK(e, hipMalloc(&e->d_cap, nb * sizeof(uint2)));
    HIPCHK(e, hipMalloc(&e->d_live_c, nb * sizeof(uint32_t)));
    HIPCHK(e, hipMalloc(&e->d_live_m, nb * sizeof(uint32_t)));
    HIPCHK(e, hipMalloc(&e->d_node_off, (n_clusters + 1) * sizeof(uint32_t)));
    HIPCHK(e, hipMalloc(&e->d_max_c, n_clusters * sizeof(uint32_t)));
    HIPCHK(e, hipMalloc(&e->d_max_m, n_clusters * sizeof(uint32_t)));
    HIPCHK(e, hipMalloc(&e->d_cstats, n_clusters * sizeof(mcs_cluster_stats)));
    HIPCHK(e, hipMalloc(&e->d_dstats, n_clusters * sizeof(mcs_delay_cluster_stats)));
    HIPCHK(e, hipMalloc(&e->d_list, n_clusters * sizeof(uint32_t)));
    HIPCHK(e, hipMemcpy(e->d_free0, free0.data(), nb * sizeof(uint2), hipMemcpyHostToDevice));
    HIPCHK(e, hipMemcpy(e->d_cap, cap.data(), nb * sizeof(uint2), hipMemcpyHostToDevice));
    HIPCHK(e, hipMemcpy(e->d_live_c, lc.data(), nb * sizeof(uint32_t), hipMemcpyHostToDevice));
    HIPCHK(e, hipMemcpy(e->d_live_m, lm.data(), nb * sizeof(uint32_t), hipMemcpyHostToDevice));
    HIPCHK(e, hipMemcpy(e->d_node_off, node_offsets, (n_clusters + 1) * sizeof(uint32_t),
                        hipMemcpyHostToDevice));
    HIPCHK(e, hipMemcpy(e->d_max_c, mxc.data(), n_clusters * sizeof(uint32_t), hipMemcpyHostToDevice));
    HIPCHK(e, hipMemcpy(e->d_max_m, mxm.data(), n_clusters * sizeof(uint32_t), hipMemcpyHostToDevice));
    e->has_clusters = true;
    return MCS_OK;
}

static int alloc_jobs(mcs_engine* e, const uint64_t* job_offsets, bool records) {
    free_jobs(e);
    mcs::trade_free(e);
    mcs::dtrade_free(e);
    e->has_jobs = e->has_run = false;
    e->dt_learn_s = e->dt_learn_v = 0;
    e->job_off.assign(job_offsets, job_offsets + e->C + 1);
    e->total_jobs = job_offsets[e->C];
    const size_t nj = e->total_jobs ? e->total_jobs : 1;
    /* kJobPad records of slack after the last cluster: the FIFO kernel streams 64-record batches
     * one ahead without bounds masks (records past a cluster's end are read, never used) */
    if (records) {
        HIPCHK(e, hipMalloc(&e->d_jobs, (nj + mcs::kJobPad) * sizeof(uint4)));
        HIPCHK(e, hipMemset(e->d_jobs + nj, 0, mcs::kJobPad * sizeof(uint4)));
    }
    HIPCHK(e, hipMalloc(&e->d_job_off, (e->C + 1) * sizeof(uint64_t)));
    /* the result arrays get the same slack: a horizon resumes by reading the 64-row result batch
     * that holds its cursor ((r & ~63) + lane, mcs_kernels.hip / mcs_delay.hip), which reaches past
     * the end when the last cluster's batch is partial */
    HIPCHK(e, hipMalloc(&e->d_out_node, (nj + mcs::kJobPad) * sizeof(int32_t)));
    HIPCHK(e, hipMalloc(&e->d_out_start, (nj + mcs::kJobPad) * sizeof(uint32_t)));
    HIPCHK(e, hipMalloc(&e->d_out_finish, (nj + mcs::kJobPad) * sizeof(uint32_t)));
    HIPCHK(e, hipMemset(e->d_out_node, 0xFF, (nj + mcs::kJobPad) * sizeof(int32_t)));
    HIPCHK(e, hipMemset(e->d_out_start, 0xFF, (nj + mcs::kJobPad) * sizeof(uint32_t)));
    HIPCHK(e, hipMemset(e->d_out_finish, 0xFF, (nj + mcs::kJobPad) * sizeof(uint32_t)));
    HIPCHK(e, hipMemcpy(e->d_job_off, job_offsets, (e->C + 1) * sizeof(uint64_t),
                        hipMemcpyHostToDevice));
    return MCS_OK;
}

static int check_job_offsets(mcs_engine* e, const uint64_t* job_offsets) {
    if (!job_offsets) return fail(e, MCS_E_INVALID, "null job_offsets");
    if (job_offsets[0] != 0) return fail(e, MCS_E_INVALID, "job_offsets[0] must be 0");
    for (uint32_t c = 0; c < e->C; ++c) {
        if (job_offsets[c + 1] < job_offsets[c])
            return fail(e, MCS_E_INVALID, "job_offsets must be non-decreasing");
        if (job_offsets[c + 1] - job_offsets[c] > 0xFFFFFFFFull)
            return fail(e, MCS_E_INVALID, "more than 2^32-1 jobs in one cluster");
    }
    return MCS_OK;
}

int mcs_submit_jobs(mcs_engine* e, const uint32_t* arrival_s, const uint32_t* dur_s,
                    const uint32_t* cores, const uint32_t* mem, const uint64_t* job_offsets) {
    if (int st = check_engine(e)) return st;
    if (!e->has_clusters) return fail(e, MCS_E_STATE, "mcs_load_clusters first");
    if (int st = check_job_offsets(e, job_offsets)) return st;
    const uint64_t nj = job_offsets[e->C];
    if (nj && (!arrival_s || !dur_s || !cores || !mem)) return fail(e, MCS_E_INVALID, "null job array");
    /* the clock never passes the last arrival + sum(dur + 1) under FIFO, + max_wait_s per job under
     * DELAY (a Level0 head may wait that long before it moves): keep that inside uint32 (D8) */
    const uint32_t extra = mcs::horizon_extra(e);
    std::vector<uint32_t> last(e->C, 0u);
    std::vector<uint64_t> sum(e->C, 0ull);
    for (uint32_t c = 0; c < e->C; ++c) { /* the ReadyQueue is filled in arrival order (server.go:41) */
        for (uint64_t i = job_offsets[c]; i < job_offsets[c + 1]; ++i) {
            if (i > job_offsets[c] && arrival_s[i] < arrival_s[i - 1])
                return fail(e, MCS_E_INVALID, "arrivals must be non-decreasing within a cluster");
            sum[c] += (uint64_t)dur_s[i] + 1u + extra;
        }
        last[c] = job_offsets[c + 1] > job_offsets[c] ? arrival_s[job_offsets[c + 1] - 1] : 0u;
        if (!e->cfg.unchecked_horizon && (uint64_t)last[c] + sum[c] >= 0xFFFFFFFFull)
            return fail(e, MCS_E_INVALID, "simulated clock could exceed 2^32-1 seconds");
    }
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if (int st = alloc_jobs(e, job_offsets, true)) return st;
    e->last_arr.swap(last);
    e->sum_dur.swap(sum);
    e->bounds_known = true;
    std::vector<uint4> h(nj ? nj : 1);
    for (uint64_t i = 0; i < nj; ++i) h[i] = make_uint4(arrival_s[i], dur_s[i], cores[i], mem[i]);
    HIPCHK(e, hipMemcpy(e->d_jobs, h.data(), (nj ? nj : 1) * sizeof(uint4), hipMemcpyHostToDevice));
    e->has_jobs = true;
    return MCS_OK;
}

int mcs_generate_jobs(mcs_engine* e, const mcs_gen_params* p, uint64_t jobs_per_cluster) {
    if (int st = check_engine(e)) return st;
    if (!e->has_clusters) return fail(e, MCS_E_STATE, "mcs_load_clusters first");
    if (!gen_params_ok(p)) return fail(e, MCS_E_INVALID, "bad generator parameters");
    if (jobs_per_cluster > 0xFFFFFFFFull) return fail(e, MCS_E_INVALID, "too many jobs per cluster");
    std::vector<uint64_t> off(e->C + 1);
    for (uint32_t c = 0; c <= e->C; ++c) off[c] = (uint64_t)c * jobs_per_cluster;
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if (int st = alloc_jobs(e, off.data(), false)) return st;
    const uint32_t* mc = e->d_max_c;
    const uint32_t* mm = e->d_max_m;
    if (p->max_cores || p->max_mem) { /* explicit maxima override setMaxCluster */
        std::vector<uint32_t> hc(e->C), hm(e->C);
        HIPCHK(e, hipMemcpy(hc.data(), e->d_max_c, e->C * 4, hipMemcpyDeviceToHost));
        HIPCHK(e, hipMemcpy(hm.data(), e->d_max_m, e->C * 4, hipMemcpyDeviceToHost));
        for (uint32_t c = 0; c < e->C; ++c) {
            if (p->max_cores) hc[c] = p->max_cores;
            if (p->max_mem) hm[c] = p->max_mem;
        }
        HIPCHK(e, hipMalloc(&e->d_gen_max, 2 * (size_t)e->C * sizeof(uint32_t)));
        HIPCHK(e, hipMemcpy(e->d_gen_max, hc.data(), e->C * 4, hipMemcpyHostToDevice));
        HIPCHK(e, hipMemcpy(e->d_gen_max + e->C, hm.data(), e->C * 4, hipMemcpyHostToDevice));
        mc = e->d_gen_max;
        mm = e->d_gen_max + e->C;
    }
    /* clusters are keyed by their global index rank*C + c (mcs_set_shard), so a sharded system
     * generates exactly the streams of the same system on one engine */
    e->gen.seed = p->seed;
    e->gen.enl = std::exp(-p->lambda);
    e->gen.max_c = mc;
    e->gen.max_m = mm;
    e->gen.mode = p->arrival_mode;
    e->gen.max_dur = p->max_dur_s;
    e->gen.base = e->rank * e->C;
    e->gen.on = p->fused;
    e->gen.wthr = nullptr;
    e->gen.wn = 0;
    if (p->arrival_mode == 2u) { /* the Weibull gap table, resolved once on the host (mcs_gen.h) */
        uint64_t thr[MCS_GEN_WEIBULL_MAX];
        const int wn = weibull_table(p->lambda, p->weibull_k > 0.0f ? p->weibull_k : 3.0, thr);
        HIPCHK(e, hipMalloc(&e->d_wthr, MCS_GEN_WEIBULL_MAX * sizeof(uint64_t)));
        HIPCHK(e, hipMemcpy(e->d_wthr, thr, (size_t)wn * sizeof(uint64_t), hipMemcpyHostToDevice));
        e->gen.wthr = e->d_wthr;
        e->gen.wn = (uint32_t)wn;
    }
    /* fused: no records in HBM; the FIFO/DELAY kernels synthesise each batch (mcs_gen_dev.h) */
    if (!p->fused)
        if (int st = mcs::ensure_job_records(e)) return st;
    /* the clock range (D8), as mcs_submit_jobs checks it: exact over the records, or for a fused
     * stream its last arrival (the arrival scan, nothing stored) + jobs * (max_dur + extra) */
    if (!e->cfg.unchecked_horizon && e->C) {
        const uint32_t extra = mcs::horizon_extra(e);
        if (!p->fused) {
            if (int st = mcs::stream_bounds(e, e->last_arr, e->sum_dur)) return st;
            e->bounds_known = true;
            for (uint32_t c = 0; c < e->C; ++c)
                if ((uint64_t)e->last_arr[c] + e->sum_dur[c] >= 0xFFFFFFFFull)
                    return fail(e, MCS_E_INVALID, "simulated clock could exceed 2^32-1 seconds");
        } else {
            unsigned long long* d_last = nullptr;
            std::vector<unsigned long long> last(e->C);
            HIPCHK(e, hipMalloc(&d_last, e->C * sizeof(unsigned long long)));
            hipError_t st = mcs::launch_gen_bound(e->d_job_off, e->C, e->gen, d_last, e->stream);
            if (st == hipSuccess) st = hipStreamSynchronize(e->stream);
            if (st == hipSuccess)
                st = hipMemcpy(last.data(), d_last, e->C * sizeof(unsigned long long), hipMemcpyDeviceToHost);
            (void)hipFree(d_last);
            if (st != hipSuccess) return fail(e, MCS_E_HIP, std::string("clock bound: ") + hipGetErrorString(st));
            const uint64_t dur_bound = jobs_per_cluster * ((uint64_t)p->max_dur_s + extra);
            for (uint32_t c = 0; c < e->C; ++c)
                if (last[c] + dur_bound >= 0xFFFFFFFFull)
                    return fail(e, MCS_E_INVALID, "simulated clock could exceed 2^32-1 seconds");
        }
    }
    e->has_jobs = true;
    return MCS_OK;
}

int mcs_read_jobs(mcs_engine* e, uint32_t* arrival_s, uint32_t* dur_s, uint32_t* cores,
                  uint32_t* mem) {
    if (int st = check_engine(e)) return st;
    if (!e->has_jobs) return fail(e, MCS_E_STATE, "no jobs");
    const uint64_t nj = e->total_jobs;
    if (!nj) return MCS_OK;
    if (!arrival_s || !dur_s || !cores || !mem) return fail(e, MCS_E_INVALID, "null output");
    if (int st = mcs::ensure_job_records(e)) return st;
    std::vector<uint4> h(nj);
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if (e->segmented) {
        if (int st = mcs::online_read_jobs(e, h.data())) return st;
    } else {
        HIPCHK(e, hipMemcpy(h.data(), e->d_jobs, nj * sizeof(uint4), hipMemcpyDeviceToHost));
    }
    for (uint64_t i = 0; i < nj; ++i) {
        arrival_s[i] = h[i].x;
        dur_s[i] = h[i].y;
        cores[i] = h[i].z;
        mem[i] = h[i].w;
    }
    return MCS_OK;
}

int mcs_run(mcs_engine* e, uint32_t t_end_s, mcs_stats* stats) {
    if (int st = check_engine(e)) return st;
    if (stats) *stats = mcs_stats{};
    if (!e->has_clusters || !e->has_jobs) return fail(e, MCS_E_STATE, "load clusters and jobs first");
    if (e->online || t_end_s != MCS_TIME_NONE) { /* online mode (mcs_online.cpp) */
        if (e->cfg.borrow || e->cfg.trader)
            return fail(e, MCS_E_INVALID, "finite horizons are implemented for FIFO/DELAY without trading");
        return mcs::online_run(e, t_end_s, stats);
    }
    if (e->cfg.unchecked_horizon && !(e->cfg.borrow || e->cfg.trader)) {
        /* streams that skipped the host clock bound run through the online kernel variant, the one
         * with the device-side finish-time guard: a drain from t = 0, the batch result */
        if (int st = mcs::online_begin(e)) return st;
        const int st = mcs::online_run(e, MCS_TIME_NONE, stats);
        e->online = false; /* the next batch run starts again from t = 0 */
        if (stats) stats->online = 0;
        return st;
    }
    if (e->cfg.borrow || e->cfg.trader) /* the trading paths read the job records */
        if (int st = mcs::ensure_job_records(e)) return st;
    if (e->cfg.policy == MCS_POLICY_DELAY && e->cfg.trader) return mcs::dtrade_run(e, stats);
    if (e->cfg.borrow || e->cfg.trader) return mcs::trade_run(e, stats);
    e->trade_run = false;
    e->dtrade_run = false;
    const bool delay = e->cfg.policy == MCS_POLICY_DELAY;
    e->delay_run = delay;
    if (delay && !e->d_l1_cm) { /* Level1 can hold every job of its cluster: never overflows */
        const size_t nj = e->total_jobs ? e->total_jobs : 1;
        HIPCHK(e, hipMalloc(&e->d_l1_cm, nj * sizeof(uint64_t)));
        HIPCHK(e, hipMalloc(&e->d_l1_jd, nj * sizeof(uint64_t)));
    }
    const auto w0 = std::chrono::steady_clock::now();
    const int npl = mcs::npl_for(e->max_n ? e->max_n : 1);
    int pool = e->cfg.slot_pool ? (int)e->cfg.slot_pool : mcs::auto_pool(e->max_n);
    if (npl < 0) return fail(e, MCS_E_INVALID, "cluster too large");

    mcs::FifoArgs a{};
    a.node_free0 = e->d_free0;
    a.node_off = e->d_node_off;
    a.jobs = e->d_jobs;
    a.job_off = e->d_job_off;
    a.cluster_list = nullptr;
    a.out_node = e->d_out_node;
    a.out_start = e->d_out_start;
    a.out_finish = e->d_out_finish;
    a.cstats = e->d_cstats;
    a.totals = e->d_totals;
    a.gen = e->gen;
    a.n_items = e->C;
    a.guard_ok = (e->free_lt31 ? 1u : 0u) | (e->free_lt15 ? 2u : 0u);
    { /* the hand-scheduled loop addresses a cluster's records and results with 32-bit VGPR
       * offsets from the cluster's base ((cb + lane) << 4): keep them inside 2^32 */
        uint64_t jmax = 0;
        for (uint32_t c = 0; c < e->C; ++c) jmax = std::max<uint64_t>(jmax, e->job_off[c + 1] - e->job_off[c]);
        if (jmax <= mcs::kAsmMaxJobs) a.guard_ok |= 4u;
    }
    mcs::DelayArgs da{};
    da.node_free0 = e->d_free0;
    da.node_off = e->d_node_off;
    da.jobs = e->d_jobs;
    da.job_off = e->d_job_off;
    da.cluster_list = nullptr;
    da.out_node = e->d_out_node;
    da.out_start = e->d_out_start;
    da.out_finish = e->d_out_finish;
    da.l1_cm = e->d_l1_cm;
    da.l1_jd = e->d_l1_jd;
    da.cstats = e->d_cstats;
    da.dstats = e->d_dstats;
    da.totals = e->d_totals;
    da.gen = e->gen;
    da.max_wait_s = e->cfg.max_wait_s;
    da.n_items = e->C;

    double kms = 0.0;
    uint32_t escalations = 0;
    int pool_used = pool;
    HIPCHK(e, hipMemsetAsync(e->d_totals, 0, sizeof(mcs::Totals), e->stream));
    /* DELAY: the hand-scheduled loop first (mcs_delay_asm.hip); clusters that reach Level1 re-run on
     * delay_kernel */
    bool dasm = delay && mcs::delay_asm_eligible(npl, pool, a.guard_ok, e->gen.on);
    switch (delay ? (dasm ? -2 : -1) : mcs::fifo_asm_form(a, npl, pool, false)) {
        case -2: e->last_kernel = "mcs::delay_asm_kernel"; break;
        case -1: e->last_kernel = "mcs::delay_kernel"; break;
        case 22: e->last_kernel = "mcs::fifo_asm_kernel<16, true, 4, 8, look>"; break;
        case 21: e->last_kernel = "mcs::fifo_duo_kernel"; break;
        case 20: e->last_kernel = "mcs::fifo_asm_fused_kernel<1, 2>"; break;
        case 19: e->last_kernel = "mcs::fifo_asm_fused_kernel<4, 8>"; break;
        case 18: e->last_kernel = "mcs::fifo_asm_kernel<16, true, 1, 2>"; break;
        case 17: e->last_kernel = "mcs::fifo_asm_kernel<16, true, 4, 8>"; break;
        case 16: e->last_kernel = "mcs::fifo_asm_kernel<16, false, 4, 8>"; break;
        case 32: e->last_kernel = "mcs::fifo_asm_kernel<32, false, 4, 8>"; break;
        default: e->last_kernel = "mcs::fifo_kernel"; break;
    }
    mcs::Totals tot{};
    uint32_t handed = 0;
    for (;;) {
        HIPCHK(e, hipEventRecord(e->ev0, e->stream));
        if (dasm)
            HIPCHK(e, mcs::launch_delay_asm(da, e->stream));
        else if (delay)
            HIPCHK(e, mcs::launch_delay(da, npl, pool, false, e->stream));
        else
            HIPCHK(e, mcs::launch_fifo(a, npl, pool, false, e->stream));
        HIPCHK(e, hipEventRecord(e->ev1, e->stream));
        HIPCHK(e, hipMemcpyAsync(&tot, e->d_totals, sizeof(tot), hipMemcpyDeviceToHost, e->stream));
        HIPCHK(e, hipStreamSynchronize(e->stream));
        float ms = 0.0f;
        HIPCHK(e, hipEventElapsedTime(&ms, e->ev0, e->ev1));
        kms += ms;
        pool_used = pool;
        if (dasm && getenv("MCS_DELAY_PROBE") && getenv("MCS_FIFO_DIAG") && atoi(getenv("MCS_FIFO_DIAG"))) {
            /* the DELAY loop's probe counters (its counting build wrote 9 per cluster into the
             * start of the cluster's Level1 scratch; clusters handed over are included up to the
             * hand-over): summed over the clusters, one line on stderr (tools only) */
            unsigned long long sum[12] = {0};
            std::vector<uint32_t> w(24);
            for (uint32_t c = 0; c < e->C; ++c) {
                const uint64_t n = std::min<uint64_t>(12, 2 * (e->job_off[c + 1] - e->job_off[c]));
                if (!n) continue;
                HIPCHK(e, hipMemcpy(w.data(), e->d_l1_cm + e->job_off[c], n * 4, hipMemcpyDeviceToHost));
                for (uint64_t k = 0; k < n; ++k) sum[k] += w[k];
            }
            fprintf(stderr, "MCS_DELAY_PROBE passes_run=%llu passes_skipped=%llu rows=%llu candidates=%llu "
                            "failed_fits=%llu grown_nodes=%llu d6_skips=%llu compactions=%llu mode1_iterations=%llu "
                            "cycles_passes=%llu cycles_loop=%llu cycles_releases=%llu\n",
                    sum[0], sum[1], sum[2], sum[3], sum[4], sum[5], sum[6], sum[7], sum[8], sum[9], sum[10], sum[11]);
        }
        const bool bailed = dasm && tot.bailed != 0;
        if (bailed) {
            handed = tot.bailed;
            e->last_kernel_buf = std::string("mcs::delay_asm_kernel + mcs::delay_kernel (") +
                                 std::to_string(handed) + " of " + std::to_string(e->C) +
                                 " clusters handed over)";
            e->last_kernel = e->last_kernel_buf.c_str();
        }
        if (tot.overflowed == 0 && !bailed) break;
        /* clusters the DELAY loop handed over re-run on delay_kernel at the same pool (with the
         * loop's overflows, which then escalate there); capacity escalation: re-run only the
         * overflowed clusters with a doubled pool */
        if (!bailed && pool * 2 > mcs::kMaxPool)
            return fail(e, MCS_E_CAPACITY, "running-slot pool overflow at 2048 slots per cluster");
        std::vector<mcs_cluster_stats> cs(e->C);
        HIPCHK(e, hipMemcpy(cs.data(), e->d_cstats, e->C * sizeof(mcs_cluster_stats),
                            hipMemcpyDeviceToHost));
        std::vector<uint32_t> list;
        const uint32_t redo = MCS_FLAG_OVERFLOW | (bailed ? mcs::kDelayBail : 0u);
        for (uint32_t c = 0; c < e->C; ++c)
            if (cs[c].flags & redo) list.push_back(c);
        HIPCHK(e, hipMemcpy(e->d_list, list.data(), list.size() * sizeof(uint32_t),
                            hipMemcpyHostToDevice));
        HIPCHK(e, hipMemsetAsync(&e->d_totals->overflowed, 0, sizeof(unsigned int), e->stream));
        HIPCHK(e, hipMemsetAsync(&e->d_totals->bailed, 0, sizeof(unsigned int), e->stream));
        a.cluster_list = da.cluster_list = e->d_list;
        a.n_items = da.n_items = (uint32_t)list.size();
        if (!bailed) {
            pool *= 2;
            ++escalations;
        }
        dasm = false;
    }
    e->has_run = true;
    if (stats) {
        stats->jobs = e->total_jobs;
        stats->placed = tot.placed;
        stats->waited = tot.waited;
        stats->unplaced = tot.unplaced;
        stats->clusters = e->C;
        stats->deadlocked = tot.deadlocked;
        stats->escalations = escalations;
        stats->slot_pool = (uint32_t)pool_used;
        stats->kernel_ms = kms;
        stats->wall_ms =
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
        stats->pending = 0;
        stats->t_horizon = MCS_TIME_NONE;
        stats->online = 0;
        stats->handed_over = handed;
    }
    if (tot.clock_overflowed)
        return fail(e, MCS_E_RANGE, std::to_string(tot.clock_overflowed) +
                                        " cluster(s) stopped: the simulated clock left the uint32 seconds range");
    return MCS_OK;
}

int mcs_read_placements(mcs_engine* e, int32_t* node, uint32_t* start_s, uint32_t* finish_s) {
    if (int st = check_engine(e)) return st;
    if (!e->has_run) return fail(e, MCS_E_STATE, "mcs_run first");
    const uint64_t nj = e->total_jobs;
    if (!nj) return MCS_OK;
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if (e->segmented) return mcs::online_read_rows(e, node, start_s, finish_s);
    if (node) HIPCHK(e, hipMemcpy(node, e->d_out_node, nj * 4, hipMemcpyDeviceToHost));
    if (start_s) HIPCHK(e, hipMemcpy(start_s, e->d_out_start, nj * 4, hipMemcpyDeviceToHost));
    if (finish_s) HIPCHK(e, hipMemcpy(finish_s, e->d_out_finish, nj * 4, hipMemcpyDeviceToHost));
    return MCS_OK;
}

int mcs_read_cluster_stats(mcs_engine* e, mcs_cluster_stats* out, uint32_t n_clusters) {
    if (int st = check_engine(e)) return st;
    if (!e->has_run) return fail(e, MCS_E_STATE, "mcs_run first");
    if (!out || n_clusters > e->C) return fail(e, MCS_E_INVALID, "bad output");
    if (e->trade_run) return mcs::trade_cluster_stats(e, out, n_clusters);
    if (e->dtrade_run) return mcs::dtrade_cluster_stats(e, out, n_clusters);
    HIPCHK(e, hipStreamSynchronize(e->stream));
    HIPCHK(e, hipMemcpy(out, e->d_cstats, n_clusters * sizeof(mcs_cluster_stats),
                        hipMemcpyDeviceToHost));
    return MCS_OK;
}

int mcs_read_delay_stats(mcs_engine* e, mcs_delay_cluster_stats* out, uint32_t n_clusters) {
    if (int st = check_engine(e)) return st;
    if (!e->has_run || !e->delay_run) return fail(e, MCS_E_STATE, "no DELAY run");
    if (!out || n_clusters > e->C) return fail(e, MCS_E_INVALID, "bad output");
    if (e->dtrade_run) return mcs::dtrade_delay_stats(e, out, n_clusters);
    HIPCHK(e, hipStreamSynchronize(e->stream));
    HIPCHK(e, hipMemcpy(out, e->d_dstats, n_clusters * sizeof(mcs_delay_cluster_stats),
                        hipMemcpyDeviceToHost));
    return MCS_OK;
}

/* ---- single-job mirrors ------------------------------------------------------------------ */
static int cluster_slice(mcs_engine* e, uint32_t cluster, uint32_t* n0, uint32_t* n) {
    if (!e->has_clusters) return fail(e, MCS_E_STATE, "mcs_load_clusters first");
    if (cluster >= e->C) return fail(e, MCS_E_INVALID, "cluster index out of range");
    *n0 = e->node_off[cluster];
    *n = e->node_off[cluster + 1] - *n0;
    return MCS_OK;
}

int mcs_schedule_one(mcs_engine* e, uint32_t cluster, uint32_t cores, uint32_t mem,
                     int32_t* node) {
    if (int st = check_engine(e)) return st;
    uint32_t n0, n;
    if (int st = cluster_slice(e, cluster, &n0, &n)) return st;
    if (!node) return fail(e, MCS_E_INVALID, "null node");
    HIPCHK(e, mcs::launch_schedule_one(e->d_live_c + n0, e->d_live_m + n0, n, cores, mem,
                                       e->d_scratch, e->stream));
    HIPCHK(e, hipMemcpyAsync(node, e->d_scratch, 4, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if (*node < 0) {
        *node = MCS_NODE_UNPLACED;
        e->err = "not enough resources in cluster"; /* scheduler.go:138 */
        return MCS_NO_FIT;
    }
    return MCS_OK;
}

int mcs_release_one(mcs_engine* e, uint32_t cluster, uint32_t node, uint32_t cores,
                    uint32_t mem) {
    if (int st = check_engine(e)) return st;
    uint32_t n0, n;
    if (int st = cluster_slice(e, cluster, &n0, &n)) return st;
    if (node >= n) return fail(e, MCS_E_INVALID, "node index out of range");
    uint32_t v[2];
    HIPCHK(e, hipStreamSynchronize(e->stream));
    HIPCHK(e, hipMemcpy(&v[0], e->d_live_c + n0 + node, 4, hipMemcpyDeviceToHost));
    HIPCHK(e, hipMemcpy(&v[1], e->d_live_m + n0 + node, 4, hipMemcpyDeviceToHost));
    v[0] += cores; /* cluster.go:155-156 */
    v[1] += mem;
    HIPCHK(e, hipMemcpy(e->d_live_c + n0 + node, &v[0], 4, hipMemcpyHostToDevice));
    HIPCHK(e, hipMemcpy(e->d_live_m + n0 + node, &v[1], 4, hipMemcpyHostToDevice));
    return MCS_OK;
}

int mcs_lend_check(mcs_engine* e, uint32_t cluster, uint32_t cores, uint32_t mem, int32_t* ok) {
    if (int st = check_engine(e)) return st;
    uint32_t n0, n;
    if (int st = cluster_slice(e, cluster, &n0, &n)) return st;
    if (!ok) return fail(e, MCS_E_INVALID, "null ok");
    HIPCHK(e, mcs::launch_lend_check(e->d_live_c + n0, e->d_live_m + n0, n, cores, mem,
                                     e->d_scratch, e->stream));
    HIPCHK(e, hipMemcpyAsync(ok, e->d_scratch, 4, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return MCS_OK;
}

int mcs_read_live_state(mcs_engine* e, uint32_t cluster, uint32_t* free_c, uint32_t* free_m,
                        uint32_t n_out) {
    if (int st = check_engine(e)) return st;
    uint32_t n0, n;
    if (int st = cluster_slice(e, cluster, &n0, &n)) return st;
    if (n_out < n || !free_c || !free_m) return fail(e, MCS_E_INVALID, "output too small");
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if (n) {
        HIPCHK(e, hipMemcpy(free_c, e->d_live_c + n0, n * 4, hipMemcpyDeviceToHost));
        HIPCHK(e, hipMemcpy(free_m, e->d_live_m + n0, n * 4, hipMemcpyDeviceToHost));
    }
    return MCS_OK;
}

int mcs_resource_utilization(mcs_engine* e, uint32_t cluster, float* core_util,
                             float* mem_util) {
    if (int st = check_engine(e)) return st;
    uint32_t n0, n;
    if (int st = cluster_slice(e, cluster, &n0, &n)) return st;
    if (!core_util || !mem_util) return fail(e, MCS_E_INVALID, "null output");
    float out[2];
    HIPCHK(e, mcs::launch_utilization(e->d_cap + n0, e->d_live_c + n0, e->d_live_m + n0, n,
                                      e->d_util, e->stream));
    HIPCHK(e, hipMemcpyAsync(out, e->d_util, 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    *core_util = out[0];
    *mem_util = out[1];
    return MCS_OK;
}

int mcs_cluster_states(mcs_engine* e, uint32_t t_s, mcs_cluster_state* out, uint32_t n_clusters,
                       double* kernel_ms) {
    if (int st = check_engine(e)) return st;
    if (!e->has_run) return fail(e, MCS_E_STATE, "mcs_run first");
    if (e->trade_run || e->dtrade_run)
        return fail(e, MCS_E_STATE, "cluster states are rebuilt from a FIFO/DELAY run without trading");
    if (e->segmented)
        return fail(e, MCS_E_STATE, "cluster states are rebuilt from batch runs (not after mcs_append_jobs)");
    if (!out || n_clusters > e->C) return fail(e, MCS_E_INVALID, "bad output");
    if (int st = mcs::ensure_job_records(e)) return st;
    mcs_cluster_state* d_out = nullptr;
    HIPCHK(e, hipMalloc(&d_out, (e->C ? e->C : 1) * sizeof(mcs_cluster_state)));
    mcs::StateArgs a{};
    a.node_off = e->d_node_off;
    a.cap = e->d_cap;
    a.free0 = e->d_free0;
    a.jobs = e->d_jobs;
    a.job_off = e->d_job_off;
    a.out_node = e->d_out_node;
    a.out_start = e->d_out_start;
    a.out_finish = e->d_out_finish;
    a.out = d_out;
    a.t = t_s;
    a.n_clusters = e->C;
    hipError_t st = hipEventRecord(e->ev0, e->stream);
    if (st == hipSuccess) st = mcs::launch_state(a, e->max_n ? e->max_n : 1, e->stream);
    if (st == hipSuccess) st = hipEventRecord(e->ev1, e->stream);
    if (st == hipSuccess) st = hipStreamSynchronize(e->stream);
    float ms = 0.0f;
    if (st == hipSuccess) st = hipEventElapsedTime(&ms, e->ev0, e->ev1);
    if (st == hipSuccess && n_clusters)
        st = hipMemcpy(out, d_out, n_clusters * sizeof(mcs_cluster_state), hipMemcpyDeviceToHost);
    (void)hipFree(d_out);
    if (st != hipSuccess) return fail(e, MCS_E_HIP, std::string("cluster states: ") + hipGetErrorString(st));
    if (kernel_ms) *kernel_ms = ms;
    return MCS_OK;
}

}  // extern "C"
