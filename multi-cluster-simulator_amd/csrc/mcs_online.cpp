// mcs_online.cpp — online mode of libmcs.so: mcs_run with a finite horizon,
// mcs_append_jobs, mcs_rewind, mcs_read_job_offsets.  Host code plus the small data-movement
// kernels it needs; compiled by hipcc.
//
// The reference's scheduler is an infinite loop fed by HTTP POSTs (pkg/scheduler/server.go:23-78,
// scheduler.go:216-369).  A Go caller replacing it through cgo advances the simulated clock in
// slices and injects the jobs POSTed meanwhile.  Each cluster's loop state lives on the device
// between calls (OnlineState + node image + slot image, double-buffered: a horizon reads one copy
// and writes the other, so a slot-pool overflow re-runs the horizon from the untouched input).
// Streams live in per-cluster segments with slack (job_off = segment starts, job_cnt = lengths),
// grown by doubling when an append does not fit.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <string>
#include <vector>

#include "mcs_engine_impl.h"
#include "mcs_internal.h"

namespace mcs {
namespace {

constexpr int kBlk = 256;

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, o);
        const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), o);
        v += (unsigned long long)lo | ((unsigned long long)hi << 32);
    }
    return v;
}

// per cluster: last arrival and sum of (dur + 1 + extra) — the clock bound (D8) of its stream
__global__ __launch_bounds__(kBlk) void bounds_kernel(const uint4* jobs, const uint64_t* job_off,
                                                      const uint32_t* cnt, uint32_t extra,
                                                      uint32_t* last, unsigned long long* sum) {
    const uint32_t c = blockIdx.x;
    const uint64_t j0 = job_off[c];
    const uint64_t J = cnt ? (uint64_t)cnt[c] : job_off[c + 1] - j0;
    unsigned long long acc = 0;
    for (uint64_t i = threadIdx.x; i < J; i += kBlk) acc += (unsigned long long)jobs[j0 + i].y + 1u + extra;
    acc = wave_sum_u64(acc);
    __shared__ unsigned long long part[kBlk / kWave];
    if ((threadIdx.x & 63u) == 0u) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long tot = 0;
        for (int w = 0; w < kBlk / kWave; ++w) tot += part[w];
        sum[c] = tot;
        last[c] = J ? jobs[j0 + J - 1].x : 0u;
    }
}

// copy the first cnt[c] rows of every cluster from the old segments to the new ones
__global__ __launch_bounds__(kBlk) void relayout_kernel(const uint64_t* off_o, const uint64_t* off_n,
                                                        const uint32_t* cnt, const uint4* jo, uint4* jn,
                                                        const int32_t* no, int32_t* nn, const uint32_t* so,
                                                        uint32_t* sn, const uint32_t* fo, uint32_t* fn,
                                                        const unsigned long long* l1a_o, unsigned long long* l1a_n,
                                                        const unsigned long long* l1b_o, unsigned long long* l1b_n) {
    const uint32_t c = blockIdx.y;
    const uint64_t a = off_o[c], b = off_n[c];
    const uint32_t n = cnt[c];
    for (uint32_t i = blockIdx.x * kBlk + threadIdx.x; i < n; i += gridDim.x * kBlk) {
        jn[b + i] = jo[a + i];
        nn[b + i] = no[a + i];
        sn[b + i] = so[a + i];
        fn[b + i] = fo[a + i];
        if (l1a_n) {
            l1a_n[b + i] = l1a_o[a + i];
            l1b_n[b + i] = l1b_o[a + i];
        }
    }
}

// appended records (dense CSR src_off) into the segments after the jobs already there; their
// result rows read "not decided" until a horizon decides them
__global__ __launch_bounds__(kBlk) void append_kernel(const uint4* src, const uint64_t* src_off,
                                                      const uint64_t* job_off, const uint32_t* cnt_old,
                                                      uint4* jobs, int32_t* on, uint32_t* os, uint32_t* of) {
    const uint32_t c = blockIdx.y;
    const uint64_t s0 = src_off[c], n = src_off[c + 1] - s0;
    const uint64_t d0 = job_off[c] + cnt_old[c];
    for (uint64_t i = (uint64_t)blockIdx.x * kBlk + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlk) {
        jobs[d0 + i] = src[s0 + i];
        on[d0 + i] = MCS_NODE_UNPLACED;
        os[d0 + i] = MCS_TIME_NONE;
        of[d0 + i] = MCS_TIME_NONE;
    }
}

// segments -> dense rows (mcs_read_placements / mcs_read_jobs)
template <class T>
__global__ __launch_bounds__(kBlk) void gather_kernel(const T* src, const uint64_t* job_off,
                                                      const uint64_t* dense_off, T* dst) {
    const uint32_t c = blockIdx.y;
    const uint64_t a = job_off[c], b = dense_off[c], n = dense_off[c + 1] - b;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlk + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlk)
        dst[b + i] = src[a + i];
}

// Level1 lists (DELAY) of the listed clusters, len(Level1) entries each as the state records it
__global__ __launch_bounds__(kBlk) void l1_copy_kernel(const OnlineState* st, const uint64_t* job_off,
                                                       const uint32_t* list, const unsigned long long* sa,
                                                       const unsigned long long* sb, unsigned long long* da,
                                                       unsigned long long* db) {
    const uint32_t c = list ? list[blockIdx.y] : blockIdx.y;
    const uint32_t n = st[c].valid ? st[c].aux : 0u;
    const uint64_t o = job_off[c];
    for (uint32_t i = blockIdx.x * kBlk + threadIdx.x; i < n; i += gridDim.x * kBlk) {
        da[o + i] = sa[o + i];
        db[o + i] = sb[o + i];
    }
}

int hip_err(mcs_engine* e, const char* what, hipError_t st) {
    return fail(e, MCS_E_HIP, std::string(what) + ": " + hipGetErrorString(st));
}

size_t img_stride(const mcs_engine* e) { return (size_t)npl_for(e->max_n ? e->max_n : 1) * kWave; }

int alloc_state(mcs_engine* e) {
    if (e->d_ost[0]) return MCS_OK;
    const size_t C = e->C ? e->C : 1;
    for (int k = 0; k < 2; ++k) {
        HIPCHK(e, hipMalloc(&e->d_ost[k], C * sizeof(OnlineState)));
        HIPCHK(e, hipMalloc(&e->d_oimg[k], C * img_stride(e) * sizeof(unsigned long long)));
        HIPCHK(e, hipMalloc(&e->d_oslot[k], C * (size_t)kSlotImg * sizeof(unsigned long long)));
    }
    return MCS_OK;
}

int upload_counts(mcs_engine* e) {
    if (!e->d_job_cnt) HIPCHK(e, hipMalloc(&e->d_job_cnt, (e->C ? e->C : 1) * sizeof(uint32_t)));
    HIPCHK(e, hipMemcpy(e->d_job_cnt, e->job_cnt.data(), e->C * sizeof(uint32_t), hipMemcpyHostToDevice));
    return MCS_OK;
}

int ensure_l1(mcs_engine* e) {
    if (e->cfg.policy != MCS_POLICY_DELAY) return MCS_OK;
    const size_t cap = (size_t)(e->job_off[e->C] ? e->job_off[e->C] : 1);
    if (!e->d_l1_cm) {
        HIPCHK(e, hipMalloc(&e->d_l1_cm, cap * sizeof(uint64_t)));
        HIPCHK(e, hipMalloc(&e->d_l1_jd, cap * sizeof(uint64_t)));
    }
    if (e->l1_bak_words < 2 * cap) {
        dfree(e->d_l1_bak);
        HIPCHK(e, hipMalloc(&e->d_l1_bak, 2 * cap * sizeof(unsigned long long)));
        e->l1_bak_words = 2 * cap;
    }
    return MCS_OK;
}

}  // namespace

// a session at t = 0 over the streams in HBM
int online_begin(mcs_engine* e) {
    if (e->cfg.borrow || e->cfg.trader)
        return fail(e, MCS_E_STATE, "online mode (finite horizons, appends) is not available with borrow/trader");
    if (e->gen.on) {  // a fused synthetic stream: online runs read records
        if (int st = ensure_job_records(e)) return st;
        e->gen.on = 0;
    }
    if (!e->segmented) {
        e->job_cnt.resize(e->C);
        for (uint32_t c = 0; c < e->C; ++c) e->job_cnt[c] = (uint32_t)(e->job_off[c + 1] - e->job_off[c]);
    }
    if (int st = upload_counts(e)) return st;
    if (!e->bounds_known) {
        if (int st = stream_bounds(e, e->last_arr, e->sum_dur)) return st;
        e->bounds_known = true;
    }
    if (int st = alloc_state(e)) return st;
    if (int st = ensure_l1(e)) return st;
    e->on_cur = 0;
    HIPCHK(e, hipMemset(e->d_ost[0], 0, (e->C ? e->C : 1) * sizeof(OnlineState)));  // valid = 0: the spec
    e->on_pool = e->cfg.slot_pool ? (int)e->cfg.slot_pool : auto_pool(e->max_n);
    e->on_t_done = 0;
    e->on_t_hor = 0;
    e->on_floor.assign(e->C, 0u);
    e->online = true;
    e->has_run = false;
    return MCS_OK;
}

uint32_t horizon_extra(const mcs_engine* e) { return e->cfg.policy == MCS_POLICY_DELAY ? e->cfg.max_wait_s : 0u; }

int stream_bounds(mcs_engine* e, std::vector<uint32_t>& last, std::vector<uint64_t>& sum) {
    last.assign(e->C, 0u);
    sum.assign(e->C, 0ull);
    if (e->C == 0 || !e->d_jobs) return MCS_OK;
    uint32_t* d_last = nullptr;
    unsigned long long* d_sum = nullptr;
    hipError_t st = hipMalloc(&d_last, e->C * sizeof(uint32_t));
    if (st == hipSuccess) st = hipMalloc(&d_sum, e->C * sizeof(unsigned long long));
    if (st == hipSuccess) {
        hipLaunchKernelGGL(bounds_kernel, dim3(e->C), dim3(kBlk), 0, e->stream, e->d_jobs, e->d_job_off,
                           e->segmented ? e->d_job_cnt : nullptr, horizon_extra(e), d_last, d_sum);
        st = hipGetLastError();
    }
    if (st == hipSuccess) st = hipStreamSynchronize(e->stream);
    if (st == hipSuccess) st = hipMemcpy(last.data(), d_last, e->C * sizeof(uint32_t), hipMemcpyDeviceToHost);
    if (st == hipSuccess) st = hipMemcpy(sum.data(), d_sum, e->C * sizeof(uint64_t), hipMemcpyDeviceToHost);
    if (d_last) (void)hipFree(d_last);
    if (d_sum) (void)hipFree(d_sum);
    if (st != hipSuccess) return hip_err(e, "stream bounds", st);
    return MCS_OK;
}

void online_free(mcs_engine* e) {
    for (int k = 0; k < 2; ++k) {
        dfree(e->d_ost[k]);
        dfree(e->d_oimg[k]);
        dfree(e->d_oslot[k]);
    }
    dfree(e->d_l1_bak);
    e->l1_bak_words = 0;
    dfree(e->d_job_cnt);
    e->online = false;
    e->segmented = false;
    e->job_cnt.clear();
    e->on_t_done = 0;
    e->on_t_hor = 0;
    e->on_floor.clear();
}

int online_run(mcs_engine* e, uint32_t t_hor, mcs_stats* stats) {
    if (!e->online)
        if (int st = online_begin(e)) return st;
    if (t_hor != MCS_TIME_NONE && t_hor < e->on_t_done)
        return fail(e, MCS_E_INVALID, "horizons must be non-decreasing (last: " + std::to_string(e->on_t_done) + ")");
    const auto w0 = std::chrono::steady_clock::now();
    const bool delay = e->cfg.policy == MCS_POLICY_DELAY;
    const int npl = npl_for(e->max_n ? e->max_n : 1);
    if (npl < 0) return fail(e, MCS_E_INVALID, "cluster too large");
    int pool = e->on_pool;
    const int in = e->on_cur, out = 1 - e->on_cur;

    OnlineArgs on{};
    on.job_cnt = e->d_job_cnt;
    on.st_in = e->d_ost[in];
    on.st_out = e->d_ost[out];
    on.img_in = e->d_oimg[in];
    on.img_out = e->d_oimg[out];
    on.slot_in = e->d_oslot[in];
    on.slot_out = e->d_oslot[out];
    on.img_stride = (uint32_t)img_stride(e);
    on.t_hor = t_hor;

    FifoArgs a{};
    a.node_free0 = e->d_free0;
    a.node_off = e->d_node_off;
    a.jobs = e->d_jobs;
    a.job_off = e->d_job_off;
    a.out_node = e->d_out_node;
    a.out_start = e->d_out_start;
    a.out_finish = e->d_out_finish;
    a.cstats = e->d_cstats;
    a.totals = e->d_totals;
    a.gen = e->gen;
    a.on = on;
    a.n_items = e->C;
    DelayArgs da{};
    da.node_free0 = e->d_free0;
    da.node_off = e->d_node_off;
    da.jobs = e->d_jobs;
    da.job_off = e->d_job_off;
    da.out_node = e->d_out_node;
    da.out_start = e->d_out_start;
    da.out_finish = e->d_out_finish;
    da.l1_cm = e->d_l1_cm;
    da.l1_jd = e->d_l1_jd;
    da.cstats = e->d_cstats;
    da.dstats = e->d_dstats;
    da.totals = e->d_totals;
    da.gen = e->gen;
    da.on = on;
    da.max_wait_s = e->cfg.max_wait_s;
    da.n_items = e->C;

    unsigned long long* bak_cm = e->d_l1_bak;
    unsigned long long* bak_jd = e->d_l1_bak ? e->d_l1_bak + e->l1_bak_words / 2 : nullptr;
    if (delay && e->C) {  // Level1 at the start of the horizon, for reruns after a pool overflow
        hipLaunchKernelGGL(l1_copy_kernel, dim3(8, e->C), dim3(kBlk), 0, e->stream, on.st_in, e->d_job_off,
                           (const uint32_t*)nullptr, (const unsigned long long*)e->d_l1_cm,
                           (const unsigned long long*)e->d_l1_jd, bak_cm, bak_jd);
        HIPCHK(e, hipGetLastError());
    }
    double kms = 0.0;
    uint32_t escalations = 0;
    HIPCHK(e, hipMemsetAsync(e->d_totals, 0, sizeof(Totals), e->stream));
    e->last_kernel = delay ? "mcs::delay_kernel" : "mcs::fifo_kernel";  // the HOR variants
    Totals tot{};
    for (;;) {
        HIPCHK(e, hipEventRecord(e->ev0, e->stream));
        if (delay)
            HIPCHK(e, launch_delay(da, npl, pool, true, e->stream));
        else
            HIPCHK(e, launch_fifo(a, npl, pool, true, e->stream));
        HIPCHK(e, hipEventRecord(e->ev1, e->stream));
        HIPCHK(e, hipMemcpyAsync(&tot, e->d_totals, sizeof(tot), hipMemcpyDeviceToHost, e->stream));
        HIPCHK(e, hipStreamSynchronize(e->stream));
        float ms = 0.0f;
        HIPCHK(e, hipEventElapsedTime(&ms, e->ev0, e->ev1));
        kms += ms;
        if (tot.overflowed == 0) break;
        // slot-pool escalation: re-run the overflowed clusters from the horizon's input state
        if (pool * 2 > kMaxPool)
            return fail(e, MCS_E_CAPACITY, "running-slot pool overflow at 2048 slots per cluster");
        std::vector<mcs_cluster_stats> cs(e->C);
        HIPCHK(e, hipMemcpy(cs.data(), e->d_cstats, e->C * sizeof(mcs_cluster_stats), hipMemcpyDeviceToHost));
        std::vector<uint32_t> list;
        for (uint32_t c = 0; c < e->C; ++c)
            if (cs[c].flags & MCS_FLAG_OVERFLOW) list.push_back(c);
        HIPCHK(e, hipMemcpy(e->d_list, list.data(), list.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        if (delay) {  // the overflowed run compacted its Level1 in place: restore it
            hipLaunchKernelGGL(l1_copy_kernel, dim3(8, (uint32_t)list.size()), dim3(kBlk), 0, e->stream, on.st_in,
                               e->d_job_off, (const uint32_t*)e->d_list, (const unsigned long long*)bak_cm,
                               (const unsigned long long*)bak_jd, (unsigned long long*)e->d_l1_cm,
                               (unsigned long long*)e->d_l1_jd);
            HIPCHK(e, hipGetLastError());
        }
        HIPCHK(e, hipMemsetAsync(&e->d_totals->overflowed, 0, sizeof(unsigned int), e->stream));
        a.cluster_list = da.cluster_list = e->d_list;
        a.n_items = da.n_items = (uint32_t)list.size();
        pool *= 2;
        ++escalations;
    }
    e->on_pool = pool;
    e->on_cur = out;
    e->has_run = true;
    e->delay_run = delay;
    e->trade_run = e->dtrade_run = false;
    if (t_hor != MCS_TIME_NONE) {
        e->on_t_done = t_hor;
        e->on_t_hor = t_hor;
    } else if (e->C) {  // a drain: a cluster's later arrivals must not precede its own clock
        std::vector<mcs_cluster_stats> cs(e->C);
        HIPCHK(e, hipMemcpy(cs.data(), e->d_cstats, e->C * sizeof(mcs_cluster_stats), hipMemcpyDeviceToHost));
        e->on_floor.resize(e->C, 0u);
        for (uint32_t c = 0; c < e->C; ++c) {
            e->on_floor[c] = std::max(e->on_floor[c], cs[c].t_end);
            e->on_t_done = std::max(e->on_t_done, cs[c].t_end);  // (the next horizon's lower bound)
        }
    }
    if (stats) {
        stats->jobs = e->total_jobs;
        stats->placed = tot.placed;
        stats->waited = tot.waited;
        stats->unplaced = tot.unplaced;
        stats->clusters = e->C;
        stats->deadlocked = tot.deadlocked;
        stats->escalations = escalations;
        stats->slot_pool = (uint32_t)pool;
        stats->kernel_ms = kms;
        stats->wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
        stats->pending = e->total_jobs - tot.placed - tot.unplaced;
        stats->t_horizon = t_hor;
        stats->online = 1u;
    }
    if (tot.clock_overflowed)
        return fail(e, MCS_E_RANGE, std::to_string(tot.clock_overflowed) +
                                        " cluster(s) stopped: the simulated clock left the uint32 seconds range");
    return MCS_OK;
}

int online_read_rows(mcs_engine* e, int32_t* node, uint32_t* start_s, uint32_t* finish_s) {
    const uint64_t nj = e->total_jobs;
    std::vector<uint64_t> dense(e->C + 1, 0);
    for (uint32_t c = 0; c < e->C; ++c) dense[c + 1] = dense[c] + e->job_cnt[c];
    uint64_t* d_dense = nullptr;
    void* tmp = nullptr;
    hipError_t st = hipMalloc(&d_dense, (e->C + 1) * sizeof(uint64_t));
    if (st == hipSuccess) st = hipMalloc(&tmp, (nj ? nj : 1) * 4);
    if (st == hipSuccess)
        st = hipMemcpy(d_dense, dense.data(), (e->C + 1) * sizeof(uint64_t), hipMemcpyHostToDevice);
    void* outs[3] = {node, start_s, finish_s};
    const void* srcs[3] = {e->d_out_node, e->d_out_start, e->d_out_finish};
    for (int k = 0; k < 3 && st == hipSuccess; ++k) {
        if (!outs[k]) continue;
        hipLaunchKernelGGL(gather_kernel<uint32_t>, dim3(16, e->C), dim3(kBlk), 0, e->stream,
                           (const uint32_t*)srcs[k], e->d_job_off, (const uint64_t*)d_dense, (uint32_t*)tmp);
        st = hipGetLastError();
        if (st == hipSuccess) st = hipStreamSynchronize(e->stream);
        if (st == hipSuccess) st = hipMemcpy(outs[k], tmp, nj * 4, hipMemcpyDeviceToHost);
    }
    if (d_dense) (void)hipFree(d_dense);
    if (tmp) (void)hipFree(tmp);
    if (st != hipSuccess) return hip_err(e, "read placements (online)", st);
    return MCS_OK;
}

int online_read_jobs(mcs_engine* e, uint4* out) {
    const uint64_t nj = e->total_jobs;
    std::vector<uint64_t> dense(e->C + 1, 0);
    for (uint32_t c = 0; c < e->C; ++c) dense[c + 1] = dense[c] + e->job_cnt[c];
    uint64_t* d_dense = nullptr;
    uint4* tmp = nullptr;
    hipError_t st = hipMalloc(&d_dense, (e->C + 1) * sizeof(uint64_t));
    if (st == hipSuccess) st = hipMalloc(&tmp, (nj ? nj : 1) * sizeof(uint4));
    if (st == hipSuccess)
        st = hipMemcpy(d_dense, dense.data(), (e->C + 1) * sizeof(uint64_t), hipMemcpyHostToDevice);
    if (st == hipSuccess) {
        hipLaunchKernelGGL(gather_kernel<uint4>, dim3(16, e->C), dim3(kBlk), 0, e->stream, (const uint4*)e->d_jobs,
                           e->d_job_off, (const uint64_t*)d_dense, tmp);
        st = hipGetLastError();
    }
    if (st == hipSuccess) st = hipStreamSynchronize(e->stream);
    if (st == hipSuccess) st = hipMemcpy(out, tmp, nj * sizeof(uint4), hipMemcpyDeviceToHost);
    if (d_dense) (void)hipFree(d_dense);
    if (tmp) (void)hipFree(tmp);
    if (st != hipSuccess) return hip_err(e, "read jobs (online)", st);
    return MCS_OK;
}

}  // namespace mcs

extern "C" {

int mcs_append_jobs(mcs_engine* e, const uint32_t* arrival_s, const uint32_t* dur_s, const uint32_t* cores,
                    const uint32_t* mem, const uint64_t* job_offsets) {
    if (int st = check_engine(e)) return st;
    if (!e->has_clusters) return fail(e, MCS_E_STATE, "mcs_load_clusters first");
    if (e->cfg.borrow || e->cfg.trader)
        return fail(e, MCS_E_STATE, "online mode (finite horizons, appends) is not available with borrow/trader");
    if (!job_offsets) return fail(e, MCS_E_INVALID, "null job_offsets");
    if (job_offsets[0] != 0) return fail(e, MCS_E_INVALID, "job_offsets[0] must be 0");
    const uint32_t C = e->C;
    for (uint32_t c = 0; c < C; ++c)
        if (job_offsets[c + 1] < job_offsets[c]) return fail(e, MCS_E_INVALID, "job_offsets must be non-decreasing");
    const uint64_t na = job_offsets[C];
    if (na && (!arrival_s || !dur_s || !cores || !mem)) return fail(e, MCS_E_INVALID, "null job array");
    if (!e->has_jobs) {  // nothing submitted yet: empty streams first
        std::vector<uint64_t> z(C + 1, 0);
        uint32_t dummy = 0;
        if (int st = mcs_submit_jobs(e, &dummy, &dummy, &dummy, &dummy, z.data())) return st;
    }
    if (!e->online)
        if (int st = mcs::online_begin(e)) return st;
    // ingestion order and the clock range (server.go:38-41,67-69; D8)
    const uint32_t extra = mcs::horizon_extra(e);
    std::vector<uint64_t> add_sum(C, 0);
    for (uint32_t c = 0; c < C; ++c) {
        const uint64_t a0 = job_offsets[c], a1 = job_offsets[c + 1];
        if (a1 == a0) continue;
        if ((uint64_t)e->job_cnt[c] + (a1 - a0) > 0xFFFFFFFFull)
            return fail(e, MCS_E_INVALID, "more than 2^32-1 jobs in one cluster");
        const uint32_t floor_ = std::max({e->job_cnt[c] ? e->last_arr[c] : 0u, e->on_t_hor,
                                          c < e->on_floor.size() ? e->on_floor[c] : 0u});
        if (arrival_s[a0] < floor_)
            return fail(e, MCS_E_INVALID, "cluster " + std::to_string(c) + ": appended arrival " +
                                              std::to_string(arrival_s[a0]) + " precedes " + std::to_string(floor_) +
                                              " (the last arrival, the last horizon, or the cluster's clock after the last drain)");
        for (uint64_t i = a0; i < a1; ++i) {
            if (i > a0 && arrival_s[i] < arrival_s[i - 1])
                return fail(e, MCS_E_INVALID, "arrivals must be non-decreasing within a cluster");
            add_sum[c] += (uint64_t)dur_s[i] + 1u + extra;
        }
        if (!e->cfg.unchecked_horizon && (uint64_t)arrival_s[a1 - 1] + e->sum_dur[c] + add_sum[c] >= 0xFFFFFFFFull)
            return fail(e, MCS_E_INVALID, "simulated clock could exceed 2^32-1 seconds");
    }
    HIPCHK(e, hipStreamSynchronize(e->stream));
    // capacity: grow the segments that do not fit (doubling, 64-job granules)
    bool grow = false;
    std::vector<uint64_t> noff(C + 1, 0);
    for (uint32_t c = 0; c < C; ++c) {
        const uint64_t cap = e->job_off[c + 1] - e->job_off[c];
        const uint64_t need = (uint64_t)e->job_cnt[c] + (job_offsets[c + 1] - job_offsets[c]);
        uint64_t ncap = cap;
        if (need > cap) {
            grow = true;
            ncap = std::max<uint64_t>(std::max<uint64_t>(need, 2 * cap), 64);
            ncap = (ncap + 63) & ~63ull;
        }
        noff[c + 1] = noff[c] + ncap;
    }
    if (grow) {
        const size_t nt = noff[C] ? noff[C] : 1;
        uint4* jn = nullptr;
        int32_t* nn = nullptr;
        uint32_t *sn = nullptr, *fn = nullptr;
        uint64_t *l1a = nullptr, *l1b = nullptr, *d_noff = nullptr;
        HIPCHK(e, hipMalloc(&jn, (nt + mcs::kJobPad) * sizeof(uint4)));
        HIPCHK(e, hipMemset(jn + nt, 0, mcs::kJobPad * sizeof(uint4)));
        HIPCHK(e, hipMalloc(&nn, (nt + mcs::kJobPad) * sizeof(int32_t)));
        HIPCHK(e, hipMalloc(&sn, (nt + mcs::kJobPad) * sizeof(uint32_t)));
        HIPCHK(e, hipMalloc(&fn, (nt + mcs::kJobPad) * sizeof(uint32_t)));
        HIPCHK(e, hipMemset(nn, 0xFF, (nt + mcs::kJobPad) * sizeof(int32_t)));
        HIPCHK(e, hipMemset(sn, 0xFF, (nt + mcs::kJobPad) * sizeof(uint32_t)));
        HIPCHK(e, hipMemset(fn, 0xFF, (nt + mcs::kJobPad) * sizeof(uint32_t)));
        if (e->d_l1_cm) {
            HIPCHK(e, hipMalloc(&l1a, nt * sizeof(uint64_t)));
            HIPCHK(e, hipMalloc(&l1b, nt * sizeof(uint64_t)));
        }
        HIPCHK(e, hipMalloc(&d_noff, (C + 1) * sizeof(uint64_t)));
        HIPCHK(e, hipMemcpy(d_noff, noff.data(), (C + 1) * sizeof(uint64_t), hipMemcpyHostToDevice));
        if (C) {
            hipLaunchKernelGGL(mcs::relayout_kernel, dim3(8, C), dim3(mcs::kBlk), 0, e->stream, e->d_job_off,
                               (const uint64_t*)d_noff, (const uint32_t*)e->d_job_cnt, (const uint4*)e->d_jobs, jn,
                               (const int32_t*)e->d_out_node, nn, (const uint32_t*)e->d_out_start, sn,
                               (const uint32_t*)e->d_out_finish, fn, (const unsigned long long*)e->d_l1_cm,
                               (unsigned long long*)l1a, (const unsigned long long*)e->d_l1_jd,
                               (unsigned long long*)l1b);
            HIPCHK(e, hipGetLastError());
        }
        HIPCHK(e, hipStreamSynchronize(e->stream));
        dfree(e->d_jobs);
        dfree(e->d_out_node);
        dfree(e->d_out_start);
        dfree(e->d_out_finish);
        dfree(e->d_l1_cm);
        dfree(e->d_l1_jd);
        dfree(e->d_job_off);
        e->d_jobs = jn;
        e->d_out_node = nn;
        e->d_out_start = sn;
        e->d_out_finish = fn;
        e->d_l1_cm = l1a;
        e->d_l1_jd = l1b;
        e->d_job_off = d_noff;
        e->job_off = noff;
        e->segmented = true;
        if (int st = mcs::ensure_l1(e)) return st;  // the backup follows the capacity
    }
    // the new records, after each cluster's jobs
    if (na) {
        std::vector<uint4> h(na);
        for (uint64_t i = 0; i < na; ++i) h[i] = make_uint4(arrival_s[i], dur_s[i], cores[i], mem[i]);
        uint4* src = nullptr;
        uint64_t* d_aoff = nullptr;
        hipError_t st = hipMalloc(&src, na * sizeof(uint4));
        if (st == hipSuccess) st = hipMalloc(&d_aoff, (C + 1) * sizeof(uint64_t));
        if (st == hipSuccess) st = hipMemcpy(src, h.data(), na * sizeof(uint4), hipMemcpyHostToDevice);
        if (st == hipSuccess) st = hipMemcpy(d_aoff, job_offsets, (C + 1) * sizeof(uint64_t), hipMemcpyHostToDevice);
        if (st == hipSuccess) {
            hipLaunchKernelGGL(mcs::append_kernel, dim3(8, C), dim3(mcs::kBlk), 0, e->stream, (const uint4*)src,
                               (const uint64_t*)d_aoff, (const uint64_t*)e->d_job_off, (const uint32_t*)e->d_job_cnt,
                               e->d_jobs, e->d_out_node, e->d_out_start, e->d_out_finish);
            st = hipGetLastError();
        }
        if (st == hipSuccess) st = hipStreamSynchronize(e->stream);
        if (src) (void)hipFree(src);
        if (d_aoff) (void)hipFree(d_aoff);
        if (st != hipSuccess) return mcs::hip_err(e, "append jobs", st);
    }
    for (uint32_t c = 0; c < C; ++c) {
        const uint64_t n = job_offsets[c + 1] - job_offsets[c];
        if (!n) continue;
        e->job_cnt[c] += (uint32_t)n;
        e->last_arr[c] = arrival_s[job_offsets[c + 1] - 1];
        e->sum_dur[c] += add_sum[c];
    }
    e->total_jobs += na;
    if (int st = mcs::upload_counts(e)) return st;
    e->has_jobs = true;
    return MCS_OK;
}

int mcs_rewind(mcs_engine* e) {
    if (int st = check_engine(e)) return st;
    if (!e->has_clusters || !e->has_jobs) return fail(e, MCS_E_STATE, "load clusters and jobs first");
    HIPCHK(e, hipStreamSynchronize(e->stream));
    e->online = false;  // online_begin keeps the segments and counts
    return mcs::online_begin(e);
}

int mcs_read_job_offsets(mcs_engine* e, uint64_t* off) {
    if (int st = check_engine(e)) return st;
    if (!e->has_jobs) return fail(e, MCS_E_STATE, "no jobs");
    if (!off) return fail(e, MCS_E_INVALID, "null output");
    off[0] = 0;
    for (uint32_t c = 0; c < e->C; ++c)
        off[c + 1] = off[c] + (e->online ? e->job_cnt[c] : e->job_off[c + 1] - e->job_off[c]);
    return MCS_OK;
}

}  // extern "C"
