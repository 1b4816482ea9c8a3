// mcs_dtrade.cpp — host side of the lock-step trading system with DELAY schedulers (DESIGN.md
// §11): device state, the tick loop (two kernels per tick; world 1: 256 ticks per captured
// hipGraph, one host poll per replay; world > 1: an ncclAllGather of the exchange blocks between
// the kernels, or the caller-driven phases), capacity escalation and the result readers of
// mcs_trade.h.  Every decision is made by the gfx950 kernels of mcs_dtrade.hip; there is no CPU path.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "mcs_dtrade_internal.h"
#include "mcs_engine_impl.h"

namespace mcs {

struct DtradeDev {
    DtArgs a{};
    unsigned long long* tn = nullptr;
    unsigned long long* vn = nullptr;
    uint2* vcap = nullptr;
    uint32_t* sfin = nullptr;
    uint32_t* snode = nullptr;
    unsigned long long* scm = nullptr;
    unsigned long long* l1cm = nullptr;
    unsigned long long* l1jd = nullptr;
    unsigned long long* l1al = nullptr;
    DtCluster* cl = nullptr;
    DtTrader* tr = nullptr;
    DtCtl* ctl = nullptr;
    unsigned long long* l1snap = nullptr;
    mcs_contract_rec* trades = nullptr;
    mcs_foreign_rec* foreign = nullptr;
    unsigned char* xb = nullptr;  // world exchange blocks
    uint32_t* nv_all = nullptr;
    DtCtl* h_ctl = nullptr;  // 3 entries: [0] the control block as last read; [1], [2] the graph loop's polls
    hipEvent_t pev[2] = {nullptr, nullptr};
    hipEvent_t tev[2] = {nullptr, nullptr};  // timing: the end of each pipelined replay
    double kernel_ms = 0.0;                  // device time of the last run (mcs_read_trade_stats)
    uint32_t tag[4] = {0, 0, 0, 0};          // caller-driven blocks: the layout tag (kDtTagBytes at the end)
    hipGraphExec_t graph = nullptr;
    hipGraphExec_t rgraph = nullptr;  // RCCL loop: kernels + all-gathers of kDtGraphTicks ticks
    // the resident tick (mcs_dtrade_mw.hip): exchange granules, placement granules + failure word
    // (uncached), the queued side effects of phase D
    unsigned long long* gx = nullptr;
    unsigned long long* gu = nullptr;
    void* ops = nullptr;
    uint32_t ops_cap = 0;
    bool rgraph_tried = false;
    uint32_t loop_form = kLoopGraph;
    bool begun = false;  // caller-driven lock-step in progress
    std::chrono::steady_clock::time_point w0{};
};

namespace {

constexpr uint64_t kDtTagBytes = 16;  // caller-driven exchange blocks end in the layout tag
constexpr uint32_t kDtGraphTicks = 256;  // (r05: 64 -> 256, A/B 14.57 -> 14.44 us per C5-DELAY tick)
constexpr uint32_t kDtResTicks = 1u << 16;  // ticks per launch of the resident tick
constexpr int kDtResFallback = -100;       // dt_run_res: the launch failed over (dtrade_run re-runs)

int dt_hip_fail(mcs_engine* e, const char* what, hipError_t st) {
    return fail(e, MCS_E_HIP, std::string(what) + ": " + hipGetErrorString(st));
}

uint32_t dt_auto_slots(uint32_t max_n) {
    uint32_t s = 256;
    while (s < 4u * max_n && s < kDtMaxSlots) s *= 2;
    return s;
}

int dtrade_alloc(mcs_engine* e) {
    if (e->dtd) return MCS_OK;
    const uint32_t C = e->C, Ct = e->C * e->world;
    if (Ct > kDtMaxClusters) return fail(e, MCS_E_INVALID, "more than 1024 clusters in a trading system");
    if (e->max_n > kDtMaxNodes) return fail(e, MCS_E_INVALID, "more than 1024 nodes in a cluster");
    const uint32_t S = e->cfg.slot_pool ? 64u * e->cfg.slot_pool : (e->tr_slots ? e->tr_slots : dt_auto_slots(e->max_n));
    if (S > kDtMaxSlots) return fail(e, MCS_E_INVALID, "slot pool above 4096");
    const uint32_t V = e->dt_vnodes ? e->dt_vnodes : 64u;
    const uint32_t NS = std::max<uint32_t>(e->dt_ns ? e->dt_ns : e->max_n, 1u), W = NS + V;
    // (a caller-driven block ends in a 16-byte layout tag that phase 1 checks on every gathered block)
    const unsigned long long blk = (unsigned long long)C * sizeof(DtRec) + (unsigned long long)C * W * 8ull +
                                   (e->comm ? 0ull : kDtTagBytes);
    DtradeDev* d = new (std::nothrow) DtradeDev();
    if (!d) return fail(e, MCS_E_NOMEM, "DELAY trading state");
    e->dtd = d;
    d->tag[0] = 0x5853434Du;  // "MCSX"
    d->tag[1] = 8u | (e->tr_agreed ? 4u : 0u);  // (8: the DELAY trading block)
    d->tag[2] = W;
    d->tag[3] = C;
    const size_t nj = e->total_jobs ? e->total_jobs : 1;
    const uint64_t trade_cap = 1ull << 20, foreign_cap = 1ull << 22;
    HIPCHK(e, hipMalloc(&d->tn, std::max<uint64_t>(e->total_nodes, 1) * 8));
    HIPCHK(e, hipMalloc(&d->vn, (size_t)C * V * 8));
    HIPCHK(e, hipMalloc(&d->vcap, (size_t)C * V * sizeof(uint2)));
    HIPCHK(e, hipMalloc(&d->sfin, (size_t)C * S * 4));
    HIPCHK(e, hipMalloc(&d->snode, (size_t)C * S * 4));
    HIPCHK(e, hipMalloc(&d->scm, (size_t)C * S * 8));
    HIPCHK(e, hipMalloc(&d->l1cm, nj * 8));
    HIPCHK(e, hipMalloc(&d->l1jd, nj * 8));
    HIPCHK(e, hipMalloc(&d->l1al, nj * 8));
    HIPCHK(e, hipMalloc(&d->cl, C * sizeof(DtCluster)));
    HIPCHK(e, hipMalloc(&d->tr, Ct * sizeof(DtTrader)));
    HIPCHK(e, hipMalloc(&d->xb, std::max<unsigned long long>(blk * e->world, 8ull)));
    HIPCHK(e, hipMemset(d->xb, 0, blk * e->world));
    HIPCHK(e, hipMalloc(&d->nv_all, Ct * 4));
    HIPCHK(e, hipMalloc(&d->ctl, sizeof(DtCtl)));
    HIPCHK(e, hipMalloc(&d->l1snap, (size_t)C * W * 8));
    HIPCHK(e, hipMalloc(&d->trades, trade_cap * sizeof(mcs_contract_rec)));
    HIPCHK(e, hipMalloc(&d->foreign, foreign_cap * sizeof(mcs_foreign_rec)));
    HIPCHK(e, hipHostMalloc(&d->h_ctl, 3 * sizeof(DtCtl), hipHostMallocDefault));
    DtArgs& a = d->a;
    a.C = C;
    a.V = V;
    a.S = S;
    a.base = e->rank * C;
    a.Ct = Ct;
    a.NS = NS;
    a.W = W;
    a.rank = e->rank;
    a.blk = blk;
    a.xb = d->xb;
    a.nv_all = d->nv_all;
    a.period = e->cfg.trader_period_s;
    a.ok_sleep = e->cfg.trade_ok_sleep_s;
    a.fail_sleep = e->cfg.trade_fail_sleep_s;
    a.lock_s = e->cfg.lock_s;
    a.sample_period = e->cfg.sample_period_s ? e->cfg.sample_period_s : 5u;
    a.max_wait = e->cfg.max_wait_s;
    a.t_max = e->cfg.t_max_s ? e->cfg.t_max_s : 0xFFFFFFFEu;
    a.trade_cap = trade_cap;
    a.foreign_cap = foreign_cap;
    a.node_off = e->d_node_off;
    a.cap = e->d_cap;
    a.free0 = e->d_free0;
    a.tn = d->tn;
    a.vn = d->vn;
    a.vcap = d->vcap;
    a.jobs = e->d_jobs;
    a.job_off = e->d_job_off;
    a.out_node = e->d_out_node;
    a.out_start = e->d_out_start;
    a.out_finish = e->d_out_finish;
    a.sfin = d->sfin;
    a.snode = d->snode;
    a.scm = d->scm;
    a.l1cm = d->l1cm;
    a.l1jd = d->l1jd;
    a.l1al = d->l1al;
    a.cl = d->cl;
    a.tr = d->tr;
    a.ctl = d->ctl;
    a.l1snap = d->l1snap;
    a.trade_log = d->trades;
    a.foreign_log = d->foreign;
    return MCS_OK;
}

int dt_poll(mcs_engine* e) {
    HIPCHK(e, hipMemcpyAsync(e->dtd->h_ctl, e->dtd->ctl, sizeof(DtCtl), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return MCS_OK;
}

int dt_run_once(mcs_engine* e, double* kernel_ms) {
    DtradeDev* d = e->dtd;
    hipError_t st = launch_dtrade_init(d->a, e->stream);
    if (st != hipSuccess) return dt_hip_fail(e, "DELAY trading init", st);
    if (!d->graph) {
        hipGraph_t g = nullptr;
        HIPCHK(e, hipStreamBeginCapture(e->stream, hipStreamCaptureModeThreadLocal));
        for (uint32_t t = 0; t < kDtGraphTicks; ++t) {
            st = launch_dtrade_tick(d->a, e->stream);
            if (st != hipSuccess) {
                (void)hipStreamEndCapture(e->stream, &g);
                if (g) (void)hipGraphDestroy(g);
                return dt_hip_fail(e, "DELAY trading capture", st);
            }
        }
        HIPCHK(e, hipStreamEndCapture(e->stream, &g));
        st = hipGraphInstantiate(&d->graph, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        if (st != hipSuccess) return dt_hip_fail(e, "hipGraphInstantiate", st);
    }
    d->loop_form = kLoopGraph;
    for (hipEvent_t& ev : d->pev)
        if (!ev) HIPCHK(e, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    for (hipEvent_t& ev : d->tev)
        if (!ev) HIPCHK(e, hipEventCreate(&ev));
    // the polls are pipelined: replay k + 1 is queued before replay k's control block is read, so
    // the GPU never idles through a host round trip (a run that ended in replay k runs one more
    // replay of finished ticks, whose kernels return at once and write nothing)
    HIPCHK(e, hipEventRecord(e->ev0, e->stream));
    DtCtl* const hp = d->h_ctl + 1;
    hipEvent_t end_ev = nullptr;
    for (uint32_t k = 0;; ++k) {
        HIPCHK(e, hipGraphLaunch(d->graph, e->stream));
        HIPCHK(e, hipEventRecord(d->tev[k & 1u], e->stream));
        HIPCHK(e, hipMemcpyAsync(hp + (k & 1u), d->ctl, sizeof(DtCtl), hipMemcpyDeviceToHost, e->stream));
        HIPCHK(e, hipEventRecord(d->pev[k & 1u], e->stream));
        if (k == 0u) continue;
        HIPCHK(e, hipEventSynchronize(d->pev[(k - 1u) & 1u]));
        if (hp[(k - 1u) & 1u].done) {
            end_ev = d->tev[(k - 1u) & 1u];  // (kernel_ms ends with the replay that finished the run)
            break;
        }
    }
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if (int s = dt_poll(e)) return s;  // (the final control block into h_ctl[0])
    float ms = 0.0f;
    HIPCHK(e, hipEventElapsedTime(&ms, e->ev0, end_ev));
    *kernel_ms = ms;
    return MCS_OK;
}

// MCS_DT_RESIDENT=0 forces the replayed kernels; the resident tick needs the whole system on this
// engine (no communicator, world 1), at most 64 clusters of at most 320 nodes (physical + virtual)
// and 1024 slots each.
bool dt_res_ok(mcs_engine* e) {
    const char* env = getenv("MCS_DT_RESIDENT");
    if ((env && atoi(env) == 0) || e->tr_no_resident || e->comm || e->world != 1) return false;
    const DtArgs& a = e->dtd->a;
    return a.Ct == a.C && a.C <= kDtResMaxClusters && e->max_n + a.V <= kDtResMaxNN && a.S <= kDtResMaxSlots &&
           a.S % 64u == 0u;
}

// the resident tick: one launch per kDtResTicks ticks (MCS_DT_RES_TICKS: fewer, so tests cross
// launch boundaries); kDtResFallback when a launch's workers were not all on one XCD or an
// exchange timed out, with nothing of the run kept
int dt_run_res(mcs_engine* e, double* kernel_ms) {
    DtradeDev* d = e->dtd;
    hipError_t st = launch_dtrade_init(d->a, e->stream);
    if (st != hipSuccess) return dt_hip_fail(e, "DELAY trading init", st);
    DtResArgs m{};
    m.ops_cap = d->a.S + d->a.V + 8u;  // a tick's side effects on a cluster: one per slot it takes, per virtual node
    if (!d->gx) {
        HIPCHK(e, hipMalloc(&d->gx, dtrade_mw_gx_bytes()));
        HIPCHK(e, hipExtMallocWithFlags((void**)&d->gu, dtrade_mw_gu_bytes(), hipDeviceMallocUncached));
        HIPCHK(e, hipMalloc(&d->ops, (size_t)d->a.C * m.ops_cap * dtrade_mw_op_bytes()));
        d->ops_cap = m.ops_cap;
    }
    m.gx = d->gx;
    m.gu = d->gu;
    m.ops = d->ops;
    m.ops_cap = d->ops_cap;
    const char* tenv = getenv("MCS_DT_RES_TICKS");
    const long tv = tenv ? atol(tenv) : 0;
    m.budget = tv > 0 && tv < (long)kDtResTicks ? (uint32_t)tv : kDtResTicks;
    m.nwg = (d->a.C + 3u) / 4u;
    d->loop_form = kLoopResidentMwXcd;
    HIPCHK(e, hipEventRecord(e->ev0, e->stream));
    for (;;) {
        st = launch_dtrade_mw(d->a, m, e->stream);
        if (st != hipSuccess) return dt_hip_fail(e, "resident DELAY trading tick", st);
        unsigned long long fw = 0;
        HIPCHK(e, hipMemcpyAsync(&fw, d->gu + dtrade_mw_fail_word(), sizeof(fw), hipMemcpyDeviceToHost, e->stream));
        if (int s = dt_poll(e)) return s;
        if (fw != 0ull) return kDtResFallback;
        // (MCS_DT_RES_FORCE_FAIL=1: tests take the fail-over path after the first launch)
        if (const char* ff = getenv("MCS_DT_RES_FORCE_FAIL"); ff && atoi(ff) != 0) return kDtResFallback;
        if (d->h_ctl->done) break;
    }
    HIPCHK(e, hipEventRecord(e->ev1, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    float ms = 0.0f;
    HIPCHK(e, hipEventElapsedTime(&ms, e->ev0, e->ev1));
    *kernel_ms = ms;
    return MCS_OK;
}

// N engines (one per GPU): the exchange blocks are all-gathered in place over xGMI between the two
// kernels of every tick; one host poll per kDtGraphTicks ticks (the kernels of finished ticks
// return at once on ctl->done, identically on every rank)
int dt_run_rccl(mcs_engine* e, double* kernel_ms) {
    DtradeDev* d = e->dtd;
    ncclComm_t comm = (ncclComm_t)e->comm;
    hipError_t st = launch_dtrade_init(d->a, e->stream);
    if (st != hipSuccess) return dt_hip_fail(e, "DELAY trading init", st);
    auto tick = [&](hipStream_t s) -> bool {
        if (launch_dtrade_step(d->a, s) != hipSuccess) return false;
        if (ncclAllGather(d->xb + (size_t)e->rank * d->a.blk, d->xb, d->a.blk, ncclUint8, comm, s) != ncclSuccess)
            return false;
        return launch_dtrade_trader(d->a, s) == hipSuccess;
    };
    if (!d->rgraph_tried) {  // (no host enqueue per tick when RCCL can be captured)
        d->rgraph_tried = true;
        d->rgraph = capture_tick_graph(e->stream, kDtGraphTicks, tick);
    }
    d->loop_form = d->rgraph ? kLoopRcclGraph : kLoopRcclEager;
    HIPCHK(e, hipEventRecord(e->ev0, e->stream));
    for (;;) {
        if (d->rgraph) {
            HIPCHK(e, hipGraphLaunch(d->rgraph, e->stream));
            if (int s = dt_poll(e)) return s;
            if (d->h_ctl->done) break;
            continue;
        }
        for (uint32_t t = 0; t < kDtGraphTicks; ++t) {
            st = launch_dtrade_step(d->a, e->stream);
            if (st != hipSuccess) return dt_hip_fail(e, "dt_step_kernel", st);
            const ncclResult_t r = ncclAllGather(d->xb + (size_t)e->rank * d->a.blk, d->xb, d->a.blk, ncclUint8,
                                                 comm, e->stream);
            if (r != ncclSuccess)
                return fail(e, MCS_E_RCCL, std::string("ncclAllGather(exchange blocks): ") + ncclGetErrorString(r));
            st = launch_dtrade_trader(d->a, e->stream);
            if (st != hipSuccess) return dt_hip_fail(e, "dt_trader_kernel", st);
        }
        if (int s = dt_poll(e)) return s;
        if (d->h_ctl->done) break;
    }
    HIPCHK(e, hipEventRecord(e->ev1, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    float ms = 0.0f;
    HIPCHK(e, hipEventElapsedTime(&ms, e->ev0, e->ev1));
    *kernel_ms = ms;
    return MCS_OK;
}

// every rank must lay its exchange block out alike: the snapshot stride is the largest cluster of
// the whole system, and the cluster count per rank must match
int dt_agree_shape(mcs_engine* e) {
    uint32_t* buf = nullptr;
    HIPCHK(e, hipMalloc(&buf, 5 * sizeof(uint32_t)));
    /* max of C and of ~C (= ~min C): every rank sees the same verdict, so a mismatch fails on
     * every rank instead of leaving the ranks with the largest C in the tick loop */
    // (and the largest learned capacities, so every rank allocates the same slot and vnode pools)
    const uint32_t h[5] = {e->max_n, e->C, ~e->C, e->tr_slots, e->dt_vnodes};
    uint32_t mx[5] = {0, 0, 0, 0, 0};
    HIPCHK(e, hipMemcpy(buf, h, sizeof(h), hipMemcpyHostToDevice));
    ncclResult_t r = ncclAllReduce(buf, buf, 5, ncclUint32, ncclMax, (ncclComm_t)e->comm, e->stream);
    hipError_t st = hipStreamSynchronize(e->stream);
    if (r == ncclSuccess && st == hipSuccess) st = hipMemcpy(mx, buf, sizeof(mx), hipMemcpyDeviceToHost);
    (void)hipFree(buf);
    if (r != ncclSuccess) return fail(e, MCS_E_RCCL, std::string("ncclAllReduce(shape): ") + ncclGetErrorString(r));
    if (st != hipSuccess) return dt_hip_fail(e, "shape exchange", st);
    if (mx[1] != ~mx[2]) return fail(e, MCS_E_INVALID, "sharded DELAY trading needs the same cluster count on every rank");
    e->dt_ns = mx[0];
    e->tr_slots = mx[3];
    e->dt_vnodes = mx[4];
    return MCS_OK;
}

int dt_clusters(mcs_engine* e, std::vector<DtCluster>& cl) {
    cl.resize(e->C);
    HIPCHK(e, hipStreamSynchronize(e->stream));
    HIPCHK(e, hipMemcpy(cl.data(), e->dtd->cl, e->C * sizeof(DtCluster), hipMemcpyDeviceToHost));
    HIPCHK(e, hipMemcpy(e->dtd->h_ctl, e->dtd->ctl, sizeof(DtCtl), hipMemcpyDeviceToHost));
    return MCS_OK;
}

}  // namespace

void dtrade_release_graphs(mcs_engine* e) {
    if (DtradeDev* d = e->dtd) {
        if (d->graph) (void)hipGraphExecDestroy(d->graph);
        if (d->rgraph) (void)hipGraphExecDestroy(d->rgraph);
        d->graph = d->rgraph = nullptr;
    }
}

void dtrade_free(mcs_engine* e) {
    DtradeDev* d = e->dtd;
    if (!d) return;
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    if (d->graph) (void)hipGraphExecDestroy(d->graph);
    if (d->rgraph) (void)hipGraphExecDestroy(d->rgraph);
    dfree(d->tn);
    dfree(d->vn);
    dfree(d->vcap);
    dfree(d->sfin);
    dfree(d->snode);
    dfree(d->scm);
    dfree(d->l1cm);
    dfree(d->l1jd);
    dfree(d->l1al);
    dfree(d->cl);
    dfree(d->tr);
    dfree(d->ctl);
    dfree(d->l1snap);
    dfree(d->trades);
    dfree(d->foreign);
    dfree(d->xb);
    dfree(d->nv_all);
    dfree(d->gx);
    dfree(d->gu);
    dfree(d->ops);
    if (d->h_ctl) (void)hipHostFree(d->h_ctl);
    for (hipEvent_t& ev : d->pev)
        if (ev) (void)hipEventDestroy(ev);
    for (hipEvent_t& ev : d->tev)
        if (ev) (void)hipEventDestroy(ev);
    delete d;
    e->dtd = nullptr;
    e->dtrade_run = false;
}

int dtrade_run(mcs_engine* e, mcs_stats* stats) {
    if (e->world > 1 && !e->comm)
        return fail(e, MCS_E_STATE, "sharded DELAY trading run needs mcs_comm_init (or mcs_trade_phase)");
    const auto w0 = std::chrono::steady_clock::now();
    // the capacities the last run of these inputs escalated to (reset when clusters, jobs or the
    // shard change): a re-run of the same system starts there instead of repeating the overflowed run
    e->tr_slots = e->dt_learn_s;
    e->dt_vnodes = e->dt_learn_v;
    // a communicator selects the RCCL loop (world 1 included: one rank's all-gather is a copy)
    const bool rccl = e->comm != nullptr;
    e->tr_no_resident = false;  // (set when the resident tick fails over, for the rest of this run)
    struct Reset {
        mcs_engine* e;
        ~Reset() { e->tr_no_resident = false; }
    } reset{e};
    if (rccl) {
        dtrade_free(e);
        if (int s = dt_agree_shape(e)) return s;
    } else {
        e->dt_ns = 0;
    }
    uint32_t escalations = 0;
    double kms = 0.0;
    for (;;) {
        if (int s = dtrade_alloc(e)) return s;
        double ms = 0.0;
        int s = MCS_OK;
        if (rccl) {
            s = dt_run_rccl(e, &ms);
        } else if (dt_res_ok(e)) {
            s = dt_run_res(e, &ms);
            if (s == kDtResFallback) {  // (the run is redone from its start on the replayed kernels)
                e->tr_no_resident = true;
                s = dt_run_once(e, &ms);
                e->dtd->loop_form = kLoopGraphAfterTimeout;
            }
        } else {
            s = dt_run_once(e, &ms);
            if (e->tr_no_resident) e->dtd->loop_form = kLoopGraphAfterTimeout;
        }
        if (s) return s;
        kms += ms;
        if (int s = dt_poll(e)) return s;
        // ctl->flags is replicated (it ORs every cluster's record), so every rank escalates alike
        const uint32_t flags = e->dtd->h_ctl->flags;
        const uint32_t S = e->dtd->a.S, V = e->dtd->a.V;
        bool grow_s = (flags & MCS_FLAG_OVERFLOW) != 0, grow_v = (flags & MCS_FLAG_VNODE_OVERFLOW) != 0;
        if (!grow_s && !grow_v) break;
        if ((grow_s && (e->cfg.slot_pool || S >= kDtMaxSlots)) || (grow_v && V >= kDtMaxVnodes))
            return fail(e, MCS_E_CAPACITY, "DELAY trading capacity exhausted (slots or virtual nodes)");
        // slots grow by half (a multiple of 64): C5-DELAY peaks just above 256 (384, not 512, slots
        // for dt_step to stage through LDS every tick)
        const uint32_t ns = grow_s ? std::min<uint32_t>((S + S / 2u + 63u) / 64u * 64u, kDtMaxSlots) : S, nv = grow_v ? std::min<uint32_t>(V * 4u, kDtMaxVnodes) : V;
        dtrade_free(e);
        e->tr_slots = ns;
        e->dt_vnodes = nv;
        ++escalations;
    }
    e->dt_learn_s = e->cfg.slot_pool ? 0u : e->dtd->a.S;
    e->dt_learn_v = e->dtd->a.V;
    e->dtd->kernel_ms = kms;
    e->has_run = true;
    e->dtrade_run = true;
    e->trade_run = false;
    e->delay_run = true;
    if (stats) {
        std::vector<DtCluster> cl;
        if (int s = dt_clusters(e, cl)) return s;
        mcs_stats st{};
        st.jobs = e->total_jobs;
        for (uint32_t k = 0; k < e->C; ++k) {
            st.placed += cl[k].decided;
            st.waited += cl[k].moved;
        }
        st.unplaced = e->total_jobs - st.placed;
        st.clusters = e->C;
        st.escalations = escalations;
        st.slot_pool = e->dtd->a.S / 64u;
        st.kernel_ms = kms;
        st.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
        *stats = st;
    }
    return MCS_OK;
}

// ---- caller-driven lock-step (mcs_trade_begin/xfer_bytes/phase/end with MCS_POLICY_DELAY) ----
// A tick is phase 0 (dt_step_kernel; out = this rank's exchange block) and phase 1 (in = every
// rank's block in rank order; dt_trader_kernel).  Phases 2 and 3 move no bytes; phase 3 reports
// done.  Every rank must hold the same cluster count and the same largest cluster (block layout).
int dtrade_begin(mcs_engine* e) {
    if (int s = dtrade_alloc(e)) return s;
    DtradeDev* d = e->dtd;
    d->w0 = std::chrono::steady_clock::now();
    const hipError_t st = launch_dtrade_init(d->a, e->stream);
    if (st != hipSuccess) return dt_hip_fail(e, "DELAY trading init", st);
    HIPCHK(e, hipStreamSynchronize(e->stream));
    HIPCHK(e, hipEventRecord(e->ev0, e->stream));
    d->begun = true;
    e->has_run = false;
    e->dtrade_run = false;
    return MCS_OK;
}

int dtrade_xfer_bytes(mcs_engine* e, uint32_t phase, uint64_t* in_bytes, uint64_t* out_bytes) {
    if (int s = dtrade_alloc(e)) return s;
    const uint64_t blk = e->dtd->a.blk;
    switch (phase) {
        case 0: *in_bytes = 0; *out_bytes = blk; break;
        case 1: *in_bytes = blk * e->world; *out_bytes = 0; break;
        default: *in_bytes = 0; *out_bytes = 0; break;
    }
    return MCS_OK;
}

int dtrade_phase(mcs_engine* e, uint32_t phase, const void* in, uint64_t in_bytes, void* out,
                 uint64_t out_bytes, uint32_t* done) {
    DtradeDev* d = e->dtd;
    if (!d || !d->begun) return fail(e, MCS_E_STATE, "mcs_trade_begin first");
    uint64_t ib = 0, ob = 0;
    if (int s = dtrade_xfer_bytes(e, phase, &ib, &ob)) return s;
    if (in_bytes != ib || out_bytes != ob || (ib && !in) || (ob && !out))
        return fail(e, MCS_E_INVALID, "exchange buffer sizes do not match mcs_trade_xfer_bytes");
    if (phase == 1) {  // every gathered block must carry this rank's layout tag
        const unsigned char* p = static_cast<const unsigned char*>(in);
        for (uint32_t r = 0; r < e->world; ++r)
            if (std::memcmp(p + (size_t)(r + 1u) * d->a.blk - kDtTagBytes, d->tag, kDtTagBytes) != 0)
                return fail(e, MCS_E_INVALID, "exchange block of rank " + std::to_string(r) +
                                                  " has another layout (stride or clusters): agree on the shape"
                                                  " with mcs_trade_set_shape");
    }
    hipError_t st = hipSuccess;
    switch (phase) {
        case 0:
            st = launch_dtrade_step(d->a, e->stream);
            if (st != hipSuccess) return dt_hip_fail(e, "dt_step_kernel", st);
            HIPCHK(e, hipMemcpyAsync(out, d->xb + (size_t)e->rank * d->a.blk, ob, hipMemcpyDeviceToHost, e->stream));
            break;
        case 1:
            HIPCHK(e, hipMemcpyAsync(d->xb, in, ib, hipMemcpyHostToDevice, e->stream));
            st = launch_dtrade_trader(d->a, e->stream);
            if (st != hipSuccess) return dt_hip_fail(e, "dt_trader_kernel", st);
            HIPCHK(e, hipMemcpyAsync(d->h_ctl, d->ctl, sizeof(DtCtl), hipMemcpyDeviceToHost, e->stream));
            break;
        default:
            break;
    }
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if (phase == 0) std::memcpy(static_cast<unsigned char*>(out) + ob - kDtTagBytes, d->tag, kDtTagBytes);
    if (done) *done = phase == 3 ? d->h_ctl->done : 0u;
    return MCS_OK;
}

int dtrade_end(mcs_engine* e, mcs_stats* stats) {
    DtradeDev* d = e->dtd;
    if (!d || !d->begun) return fail(e, MCS_E_STATE, "mcs_trade_begin first");
    HIPCHK(e, hipEventRecord(e->ev1, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    d->begun = false;
    e->has_run = true;
    e->dtrade_run = true;
    e->trade_run = false;
    e->delay_run = true;
    if (int s = dt_poll(e)) return s;
    const uint32_t flags = d->h_ctl->flags;
    {
        float ms = 0.0f;
        if (hipEventElapsedTime(&ms, e->ev0, e->ev1) != hipSuccess) ms = 0.0f;
        d->kernel_ms = ms;
    }
    if (stats) {
        std::vector<DtCluster> cl;
        if (int s = dt_clusters(e, cl)) return s;
        mcs_stats st{};
        st.jobs = e->total_jobs;
        for (uint32_t k = 0; k < e->C; ++k) {
            st.placed += cl[k].decided;
            st.waited += cl[k].moved;
        }
        st.unplaced = e->total_jobs - st.placed;
        st.clusters = e->C;
        st.slot_pool = d->a.S / 64u;
        st.kernel_ms = d->kernel_ms;
        st.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - d->w0).count();
        *stats = st;
    }
    if (flags & MCS_FLAG_OVERFLOW)
        return fail(e, MCS_E_CAPACITY, "running-slot pool overflow (raise mcs_config.slot_pool)");
    if (flags & MCS_FLAG_VNODE_OVERFLOW)
        return fail(e, MCS_E_CAPACITY, "virtual-node capacity overflow");
    return MCS_OK;
}

int dtrade_cluster_stats(mcs_engine* e, mcs_cluster_stats* out, uint32_t n) {
    std::vector<DtCluster> cl;
    if (int s = dt_clusters(e, cl)) return s;
    for (uint32_t k = 0; k < n; ++k) {
        mcs_cluster_stats s{};
        s.t_end = e->dtd->h_ctl->T;
        s.placed = cl[k].decided;
        s.waited = cl[k].moved;
        s.peak_running = cl[k].peak;
        s.flags = cl[k].flags;
        s.pool = e->dtd->a.S / 64u;
        s.iterations = e->dtd->h_ctl->ticks;
        s.release_scans = 0;
        out[k] = s;
    }
    return MCS_OK;
}

int dtrade_delay_stats(mcs_engine* e, mcs_delay_cluster_stats* out, uint32_t n) {
    std::vector<DtCluster> cl;
    if (int s = dt_clusters(e, cl)) return s;
    for (uint32_t k = 0; k < n; ++k) {
        mcs_delay_cluster_stats d{};
        d.total_wait_ms = cl[k].total;
        d.jobs_count = cl[k].count;
        d.moved_l1 = cl[k].moved;
        d.placed_l1 = cl[k].placed_l1;
        d.peak_l1 = 0;
        d.l1_left = cl[k].l1n;
        out[k] = d;
    }
    return MCS_OK;
}

int dtrade_trade_stats(mcs_engine* e, mcs_trade_stats* out) {
    std::vector<DtCluster> cl;
    if (int s = dt_clusters(e, cl)) return s;
    const DtCtl& c = *e->dtd->h_ctl;
    mcs_trade_stats s{};
    uint32_t flags = c.flags;
    for (uint32_t k = 0; k < e->C; ++k) {
        const uint64_t J = e->job_off[k + 1] - e->job_off[k];
        s.placed += cl[k].decided;
        s.waited += cl[k].moved;
        s.undecided += J - cl[k].decided;
        flags |= cl[k].flags;
    }
    if (c.n_trades > e->dtd->a.trade_cap || c.n_foreign > e->dtd->a.foreign_cap) flags |= MCS_FLAG_LOG_OVERFLOW;
    s.trades = c.n_trades;
    s.trades_won = c.n_won;
    s.ticks = c.ticks;
    s.t_final = c.T;
    s.flags = flags;
    s.loop_form = e->dtd->loop_form;
    s.kernel_ms = e->dtd->kernel_ms;
    s.block_bytes = e->dtd->a.blk;
    s.snaps = 1u;
    s.agreed = (e->comm || e->tr_agreed) ? 1u : 0u;
    *out = s;
    return MCS_OK;
}

int dtrade_read_trades(mcs_engine* e, mcs_trade_rec* out, uint64_t cap, uint64_t* n) {
    HIPCHK(e, hipStreamSynchronize(e->stream));
    HIPCHK(e, hipMemcpy(e->dtd->h_ctl, e->dtd->ctl, sizeof(DtCtl), hipMemcpyDeviceToHost));
    const uint64_t total = e->dtd->h_ctl->n_trades;
    const uint64_t k = std::min<uint64_t>(std::min<uint64_t>(total, e->dtd->a.trade_cap), cap);
    if (k) {
        std::vector<mcs_contract_rec> v(k);
        HIPCHK(e, hipMemcpy(v.data(), e->dtd->trades, k * sizeof(mcs_contract_rec), hipMemcpyDeviceToHost));
        for (uint64_t i = 0; i < k; ++i) out[i] = mcs_trade_rec{v[i].t_s, v[i].requester, v[i].winner, v[i].approvals};
    }
    *n = total;
    return MCS_OK;
}

int dtrade_read_vnode_counts(mcs_engine* e, uint32_t* out, uint32_t n) {
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if (n) HIPCHK(e, hipMemcpy(out, e->dtd->nv_all, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
    return MCS_OK;
}

}  // namespace mcs

extern "C" {

int mcs_read_contracts(mcs_engine* e, mcs_contract_rec* out, uint64_t cap, uint64_t* n) {
    if (int st = check_engine(e)) return st;
    if (!n || (cap && !out)) return fail(e, MCS_E_INVALID, "bad output");
    if (!e->dtrade_run || !e->dtd) return fail(e, MCS_E_STATE, "no DELAY trading run");
    mcs::DtradeDev* d = e->dtd;
    HIPCHK(e, hipStreamSynchronize(e->stream));
    HIPCHK(e, hipMemcpy(d->h_ctl, d->ctl, sizeof(mcs::DtCtl), hipMemcpyDeviceToHost));
    const uint64_t total = d->h_ctl->n_trades;
    const uint64_t k = std::min<uint64_t>(std::min<uint64_t>(total, d->a.trade_cap), cap);
    if (k) HIPCHK(e, hipMemcpy(out, d->trades, k * sizeof(mcs_contract_rec), hipMemcpyDeviceToHost));
    *n = total;
    return MCS_OK;
}

int mcs_read_foreign(mcs_engine* e, mcs_foreign_rec* out, uint64_t cap, uint64_t* n) {
    if (int st = check_engine(e)) return st;
    if (!n || (cap && !out)) return fail(e, MCS_E_INVALID, "bad output");
    if (!e->dtrade_run || !e->dtd) return fail(e, MCS_E_STATE, "no DELAY trading run");
    mcs::DtradeDev* d = e->dtd;
    HIPCHK(e, hipStreamSynchronize(e->stream));
    HIPCHK(e, hipMemcpy(d->h_ctl, d->ctl, sizeof(mcs::DtCtl), hipMemcpyDeviceToHost));
    const uint64_t total = d->h_ctl->n_foreign;
    const uint64_t k = std::min<uint64_t>(std::min<uint64_t>(total, d->a.foreign_cap), cap);
    if (k) HIPCHK(e, hipMemcpy(out, d->foreign, k * sizeof(mcs_foreign_rec), hipMemcpyDeviceToHost));
    *n = total;
    return MCS_OK;
}

int mcs_read_virtual_node_caps(mcs_engine* e, uint32_t cluster, uint32_t* cores, uint32_t* mem,
                               uint32_t cap, uint32_t* n) {
    if (int st = check_engine(e)) return st;
    if (!n || (cap && (!cores || !mem))) return fail(e, MCS_E_INVALID, "bad output");
    if (!e->dtrade_run || !e->dtd) return fail(e, MCS_E_STATE, "no DELAY trading run");
    if (cluster >= e->C) return fail(e, MCS_E_INVALID, "cluster index out of range");
    mcs::DtradeDev* d = e->dtd;
    mcs::DtCluster k{};
    HIPCHK(e, hipStreamSynchronize(e->stream));
    HIPCHK(e, hipMemcpy(&k, d->cl + cluster, sizeof(k), hipMemcpyDeviceToHost));
    const uint32_t m = std::min<uint32_t>(std::min<uint32_t>(k.nv, d->a.V), cap);
    if (m) {
        std::vector<uint2> v(m);
        HIPCHK(e, hipMemcpy(v.data(), d->vcap + (size_t)cluster * d->a.V, m * sizeof(uint2), hipMemcpyDeviceToHost));
        for (uint32_t i = 0; i < m; ++i) {
            cores[i] = v[i].x;
            mem[i] = v[i].y;
        }
    }
    *n = k.nv;
    return MCS_OK;
}

int mcs_approve_trade(mcs_engine* e, const mcs_approve_query* q, uint32_t n, int32_t* out) {
    if (int st = check_engine(e)) return st;
    if (n && (!q || !out)) return fail(e, MCS_E_INVALID, "null query or output");
    if (!n) return MCS_OK;
    mcs_approve_query* dq = nullptr;
    int32_t* dout = nullptr;
    hipError_t st = hipMalloc(&dq, n * sizeof(mcs_approve_query));
    if (st == hipSuccess) st = hipMalloc(&dout, n * sizeof(int32_t));
    if (st == hipSuccess) st = hipMemcpy(dq, q, n * sizeof(mcs_approve_query), hipMemcpyHostToDevice);
    if (st == hipSuccess) st = mcs::launch_approve(dq, n, dout, e->stream);
    if (st == hipSuccess) st = hipStreamSynchronize(e->stream);
    if (st == hipSuccess) st = hipMemcpy(out, dout, n * sizeof(int32_t), hipMemcpyDeviceToHost);
    if (dq) (void)hipFree(dq);
    if (dout) (void)hipFree(dout);
    if (st != hipSuccess) return fail(e, MCS_E_HIP, std::string("approve_trade: ") + hipGetErrorString(st));
    return MCS_OK;
}

}  // extern "C"
