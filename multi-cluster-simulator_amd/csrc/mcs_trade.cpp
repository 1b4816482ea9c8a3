// mcs_trade.cpp — C ABI of the lock-step trading path (include/mcs_trade.h): device state,
// the tick loop (hipGraph replay on one GPU, one RCCL all-gather of the exchange blocks per tick
// over xGMI across GPUs, or the caller-driven phase API), and the result readers.  Host code;
// compiled by hipcc.
//
// Every decision is made by the gfx950 kernels of mcs_trade.hip; there is no CPU path.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "mcs_engine_impl.h"
#include "mcs_trade_internal.h"

namespace mcs {

struct TradeDev {
    TradeArgs a{};  // (the exchange blocks of every rank live in xb)
    unsigned long long* tn = nullptr;
    TrCluster* cl = nullptr;
    uint32_t* sfin = nullptr;
    uint32_t* snode = nullptr;
    unsigned long long* scm = nullptr;
    TrLq* lq = nullptr;
    unsigned char* xb = nullptr;
    unsigned long long* gx = nullptr;   // the workgroup-resident tick's granules (uncached)
    unsigned long long* gxc = nullptr;  // ... and their cached twin (workgroups on one XCD)
    uint32_t* acc = nullptr;
    uint32_t* lqp = nullptr;
    uint32_t* fb = nullptr;
    TrTrader* tr = nullptr;
    TrCtl* ctl = nullptr;
    mcs_lent_rec* lent = nullptr;
    mcs_trade_rec* trades = nullptr;
    uint4* lrp = nullptr;                // one-launch tick: pending lent-run records
    unsigned long long* tnr = nullptr;   // one-launch tick: dense node state [C_l][ns]
    bool rk = false;                     // the one-launch tick runs this system (trade_alloc)
    bool rk_started = false;             // its tick-0 phase A has run
    uint64_t rk_tick = 0;                // one-launch ticks launched (the exchange buffer's parity)
    size_t rk_lds = 0;
    TrCtl* h_ctl = nullptr;  // pinned, 3 entries: [0] the control block as last read; [1], [2] the pipelined polls
    hipEvent_t pev[2] = {nullptr, nullptr};
    hipEvent_t tev[2] = {nullptr, nullptr};  // timing: the end of each pipelined replay
    hipEvent_t end_ev = nullptr;             // the end of the replay whose control block showed done
    uint32_t tag[4] = {0, 0, 0, 0};          // caller-driven blocks: the layout tag (kTagBytes at the end)
    hipGraphExec_t graph = nullptr;
    uint32_t graph_ticks = 0;
    hipGraphExec_t rgraph = nullptr;  // RCCL loop: kernels + all-gathers of kGraphTicks ticks
    bool rgraph_tried = false;
    uint32_t loop_form = kLoopGraph;
    bool begun = false;
    std::chrono::steady_clock::time_point w0;
};

namespace {

constexpr uint64_t kTagBytes = 16;     // caller-driven exchange blocks end in the layout tag
constexpr uint32_t kTagMagic = 0x5853434Du;  // "MCSX"
constexpr uint32_t kGraphTicks = 256;  // ticks per graph replay (one host poll per replay; r05: 64 -> 256, A/B 9.60 -> 9.44 us per tick on the one-launch RCCL loop)

int hip_fail(mcs_engine* e, const char* what, hipError_t st) {
    return fail(e, MCS_E_HIP, std::string(what) + ": " + hipGetErrorString(st));
}

uint32_t auto_slots(uint32_t max_n) {
    uint32_t s = 256;
    while (s < 4u * max_n && s < kTrMaxSlots) s *= 2;
    return s;
}

// a one-engine system the resident tick kernel can hold (mcs_trade_res.hip; the LDS check is
// resident_form's).  Its slot finish times live in VGPRs, so trade_run's local loop starts such a
// system at 512 slots per cluster (8 rows; 1024 spill) when a resident form will run it: an overflow
// re-runs it at 1024 like any other pool overflow.  The caller-driven path (mcs_trade_begin) and the
// RCCL loop keep auto_slots (they have no resident form and, caller-driven, no escalation).
bool resident_wanted(const mcs_engine* e) {
    const char* env = getenv("MCS_TRADE_RESIDENT");
    if (env && atoi(env) == 0) return false;
    return e->world == 1 && e->C <= kTrResMaxClusters && e->max_n <= 256u && e->sums_lt24;
}

constexpr uint32_t kMaxLq = 1u << 24;  // LentQueue entries per cluster (512 MB per cluster)

// Every acceptor of a borrow request keeps its own copy (server.go:232-237) and an overloaded
// lender serves its LentQueue only when idle, so queues grow with the stream: start at 4 entries
// per own job of the largest cluster (measured peaks: 3-12 per job on C3/C5-shaped workloads)
uint32_t auto_lq(const mcs_engine* e) {
    uint64_t mj = 0;
    for (uint32_t c = 0; c < e->C; ++c) mj = std::max<uint64_t>(mj, e->job_off[c + 1] - e->job_off[c]);
    uint64_t q = 4096;
    while (q < 4 * mj && q < kMaxLq) q *= 2;
    return (uint32_t)q;
}

int trade_alloc(mcs_engine* e) {
    if (e->td) return MCS_OK;
    if (!e->has_clusters || !e->has_jobs) return fail(e, MCS_E_STATE, "load clusters and jobs first");
    if (int st = ensure_job_records(e)) return st;
    const uint32_t Cl = e->C, Ct = e->C * e->world;
    if (Ct > kTrMaxClusters) return fail(e, MCS_E_INVALID, "more than 1024 clusters in a trading system");
    if (e->max_n > kTrMaxNodes) return fail(e, MCS_E_INVALID, "more than 1024 nodes in a cluster");
    const uint32_t S = e->cfg.slot_pool ? 64u * e->cfg.slot_pool
                       : e->tr_slots       ? e->tr_slots
                       : e->tr_res_start   ? std::min<uint32_t>(512u, auto_slots(e->max_n))
                                           : auto_slots(e->max_n);
    if (S > kTrMaxSlots) return fail(e, MCS_E_INVALID, "slot pool above 4096");
    const uint32_t LQ = e->cfg.lent_queue_cap ? e->cfg.lent_queue_cap : (e->tr_lq ? e->tr_lq : auto_lq(e));
    TradeDev* td = new (std::nothrow) TradeDev();
    if (!td) return fail(e, MCS_E_NOMEM, "trade state");
    e->td = td;
    const uint64_t lent_cap = std::max<uint64_t>(1ull << 16, 16ull * e->total_jobs);
    const uint64_t trade_cap = 1ull << 22;
    HIPCHK(e, hipMalloc(&td->tn, std::max<uint64_t>(e->total_nodes, 1) * 8));
    HIPCHK(e, hipMalloc(&td->cl, Cl * sizeof(TrCluster)));
    HIPCHK(e, hipMalloc(&td->sfin, (size_t)Cl * S * 4));
    HIPCHK(e, hipMalloc(&td->snode, (size_t)Cl * S * 4));
    HIPCHK(e, hipMalloc(&td->scm, (size_t)Cl * S * 8));
    HIPCHK(e, hipMalloc(&td->lq, (size_t)Cl * LQ * sizeof(TrLq)));
    const uint32_t ns = std::max<uint32_t>(e->tr_ns ? e->tr_ns : e->max_n, 1u);
    // the one-launch tick (mcs_trade_rk.hip) runs sharded systems (a communicator or the caller-driven
    // API) whose shape it holds; every rank decides alike (tr_agree_shape on the RCCL path; the
    // caller-driven ranks hold alike clusters).  MCS_TRADE_RK=0 keeps the three-kernel tick.
    bool rk = false;
    size_t rk_lds = 0;
    {
        const char* rkenv = getenv("MCS_TRADE_RK");
        const bool want_rk = !rkenv || atoi(rkenv) != 0;
        TradeArgs shp{};
        shp.Ct = Ct;
        shp.Cl = Cl;
        shp.ns = ns;
        shp.S = S;
        int max_lds = 0;
        rk_lds = trade_rk_lds(ns);
        rk = want_rk && e->sums_lt24 && e->slot_pack_ok && e->tr_rk_ok && trade_rk_shape(shp) &&
             hipDeviceGetAttribute(&max_lds, hipDeviceAttributeMaxSharedMemoryPerBlock, e->device) == hipSuccess &&
             rk_lds <= (size_t)max_lds;
    }
    // (16-byte aligned blocks: the records are read as 16-byte vectors on every rank's block; the
    // one-launch tick's G tables, 256 B per cluster, follow the snapshots.  On the RCCL path, when no
    // rank has a node above 64 cores, no lender is ever "big": the one-launch tick's blocks then
    // carry no snapshots at all — 320 B per cluster instead of 320 B + 8 B per node)
    // The caller-driven path drops them too when its ranks agreed on the shape (mcs_trade_set_shape).
    // A caller-driven block ends in a 16-byte layout tag that phase 1 checks on every gathered block)
    const bool snaps = !(rk && (e->comm || e->tr_agreed) && e->tr_nosnap);
    const uint64_t tagb = e->comm ? 0ull : kTagBytes;
    const uint64_t blk = (((uint64_t)Cl * sizeof(TrXRec) + (snaps ? (uint64_t)Cl * ns * 8u : 0ull) +
                           (uint64_t)Cl * 256u + 15u) & ~15ull) + tagb;
    td->tag[0] = kTagMagic;
    td->tag[1] = (rk ? 1u : 0u) | (snaps ? 2u : 0u) | (e->tr_agreed ? 4u : 0u);
    td->tag[2] = ns;
    td->tag[3] = Cl;
    // (two buffers of world blocks: the one-launch tick alternates them by tick parity)
    HIPCHK(e, hipMalloc(&td->xb, 2u * (size_t)e->world * blk));
    HIPCHK(e, hipMalloc(&td->acc, Ct * 4));
    HIPCHK(e, hipMalloc(&td->lqp, Ct * 4));
    HIPCHK(e, hipMalloc(&td->fb, Ct * 4));
    // (two copies of the trader state and of the clock: the one-launch tick alternates them by tick
    // parity; every other form uses the first)
    HIPCHK(e, hipMalloc(&td->tr, 2u * Ct * sizeof(TrTrader)));
    HIPCHK(e, hipMalloc(&td->ctl, 2u * sizeof(TrCtl)));
    HIPCHK(e, hipMalloc(&td->lent, lent_cap * sizeof(mcs_lent_rec)));
    HIPCHK(e, hipMalloc(&td->trades, trade_cap * sizeof(mcs_trade_rec)));
    HIPCHK(e, hipHostMalloc(&td->h_ctl, 3 * sizeof(TrCtl), hipHostMallocDefault));
    HIPCHK(e, hipMalloc(&td->lrp, std::max<uint32_t>(Cl, 1u) * sizeof(uint4)));

    TradeArgs& a = td->a;
    a.Cl = Cl;
    a.Ct = Ct;
    a.base = e->rank * Cl;
    a.world = e->world;
    a.S = S;
    a.LQ = LQ;
    a.borrow = e->cfg.borrow;
    a.trader = e->cfg.trader;
    a.period = e->cfg.trader_period_s;
    a.ok_sleep = e->cfg.trade_ok_sleep_s;
    a.fail_sleep = e->cfg.trade_fail_sleep_s;
    a.lock_s = e->cfg.lock_s;
    a.sample_period = e->cfg.sample_period_s ? e->cfg.sample_period_s : 5u;
    a.t_max = e->cfg.t_max_s ? e->cfg.t_max_s : 0xFFFFFFFEu;
    a.lent_cap = lent_cap;
    a.trade_cap = trade_cap;
    a.node_off = e->d_node_off;
    a.cap = e->d_cap;
    a.free0 = e->d_free0;
    a.tn = td->tn;
    a.jobs = e->d_jobs;
    a.job_off = e->d_job_off;
    a.out_node = e->d_out_node;
    a.out_start = e->d_out_start;
    a.out_finish = e->d_out_finish;
    a.cl = td->cl;
    a.sfin = td->sfin;
    a.snode = td->snode;
    a.scm = td->scm;
    a.lq = td->lq;
    a.xb = td->xb;
    a.blk = blk;
    a.ns = ns;
    a.rank = e->rank;
    a.acc = td->acc;
    a.lqp = td->lqp;
    a.fb = td->fb;
    a.tr = td->tr;
    a.ctl = td->ctl;
    a.lent_log = td->lent;
    a.trade_log = td->trades;
    a.lrp = td->lrp;
    a.snaps = snaps ? 1u : 0u;
    if (rk) {
        td->rk_lds = rk_lds;
        HIPCHK(e, hipMalloc(&td->tnr, (size_t)Cl * ns * 8u));
        a.tnr = td->tnr;
        td->rk = true;
    }
    return MCS_OK;
}

int launch_phase(mcs_engine* e, const TradeArgs& a, int phase) {
    const hipError_t st = launch_trade_phase(a, phase, e->stream);
    if (st != hipSuccess) return hip_fail(e, "trade kernel launch", st);
    return MCS_OK;
}

int poll_ctl(mcs_engine* e) {
    HIPCHK(e, hipMemcpyAsync(e->td->h_ctl, e->td->ctl, sizeof(TrCtl), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return MCS_OK;
}

// replays of a captured tick loop until the run is done, the polls pipelined: replay k + 1 is queued
// before replay k's control block is read, so the GPU never idles through a host round trip.  A
// run that ended in replay k runs one more replay of finished ticks (their kernels return at once;
// every rank reads the same replicated flag, so the collectives stay matched).
template <class Replay>
int replay_until_done(mcs_engine* e, Replay&& replay) {
    TradeDev* td = e->td;
    for (hipEvent_t& ev : td->pev)
        if (!ev) HIPCHK(e, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    for (hipEvent_t& ev : td->tev)
        if (!ev) HIPCHK(e, hipEventCreate(&ev));
    TrCtl* const hp = td->h_ctl + 1;
    for (uint32_t k = 0;; ++k) {
        if (int s = replay()) return s;
        HIPCHK(e, hipEventRecord(td->tev[k & 1u], e->stream));
        HIPCHK(e, hipMemcpyAsync(hp + (k & 1u), td->ctl, sizeof(TrCtl), hipMemcpyDeviceToHost, e->stream));
        HIPCHK(e, hipEventRecord(td->pev[k & 1u], e->stream));
        if (k == 0u) continue;
        HIPCHK(e, hipEventSynchronize(td->pev[(k - 1u) & 1u]));
        if (hp[(k - 1u) & 1u].done) {
            // kernel_ms ends with the replay that finished the run: the one more replay of no-op
            // ticks queued behind it (the pipelined poll's price) is not part of the run
            td->end_ev = td->tev[(k - 1u) & 1u];
            break;
        }
    }
    return poll_ctl(e);  // (the final control block into h_ctl[0])
}

// one engine holds the whole system.  When it fits one workgroup (<= 64 clusters of <= 256 nodes,
// 1024 slots each, exact integer utilization sums) the tick loop runs resident (mcs_trade_res.hip),
// kResTicks ticks per launch; otherwise the four phases of kGraphTicks ticks are captured once and
// replayed.  MCS_TRADE_RESIDENT=0 forces the replayed kernels.
constexpr uint32_t kResTicks = 1u << 16;
// (MCS_TRADE_RES_TICKS: a smaller budget, so tests cross launch boundaries)
uint32_t res_ticks() {
    const char* env = getenv("MCS_TRADE_RES_TICKS");
    const long v = env ? atol(env) : 0;
    return v > 0 && v < (long)kResTicks ? (uint32_t)v : kResTicks;
}
constexpr int kMwFallback = -100;  // run_local: a resident exchange timed out (trade_run re-runs)

// MCS_TRADE_RESIDENT: 0 = the replayed kernels, 1 = one workgroup, 2 = one workgroup per 4
// clusters (the default where the shape allows it)
int resident_form(mcs_engine* e, size_t* lds) {
    const char* env = getenv("MCS_TRADE_RESIDENT");
    const int want = env ? atoi(env) : 2;
    if (want == 0 || !e->sums_lt24 || e->tr_no_resident) return 0;
    int max_lds = 0;
    if (hipDeviceGetAttribute(&max_lds, hipDeviceAttributeMaxSharedMemoryPerBlock, e->device) != hipSuccess)
        return 0;
    if (want == 2 && e->slot_pack_ok && trade_mw_shape(e->td->a)) {
        *lds = trade_mw_lds(e->td->a.ns);
        if (*lds <= (size_t)max_lds) return 2;
    }
    if (!trade_resident_shape(e->td->a)) return 0;
    *lds = trade_resident_lds(e->td->a.Ct, e->td->a.ns);
    return *lds <= (size_t)max_lds ? 1 : 0;
}

int run_local(mcs_engine* e) {
    TradeDev* td = e->td;
    size_t lds = 0;
    const int rf = resident_form(e, &lds);
    if (rf == 2) {
        td->loop_form = kLoopResidentMw;
        if (!td->gx) {
            // two granule buffers: uncached device memory (MTYPE UC) for workgroups on different
            // XCDs (a poll that re-reads a line its XCD's L2 already holds would otherwise be served
            // the stale copy until that line is evicted: ~7 sweep passes per exchange measured with
            // cached memory), and cached memory for workgroups that all run on one XCD, whose shared
            // L2 serves the polls (the kernel checks the placement; MCS_MW_GX=0 makes both cached)
            const char* gxenv = getenv("MCS_MW_GX");
            const int gxm = gxenv ? atoi(gxenv) : 3;
            const size_t gb = trade_mw_granules(td->a.Ct) * 8u;
            if (gxm == 0) HIPCHK(e, hipMalloc(&td->gx, gb));
            else HIPCHK(e, hipExtMallocWithFlags((void**)&td->gx, gb, (unsigned)gxm));
            HIPCHK(e, hipMalloc(&td->gxc, gb));
        }
        // the workgroups 8 blocks apart: one XCD under the dispatcher's round-robin (MCS_MW_XCD=0:
        // consecutive blocks, the write-through exchange)
        const char* xenv = getenv("MCS_MW_XCD");
        const bool xcd_pack = !xenv || atoi(xenv) != 0;
        const char* uenv = getenv("MCS_MW_FORCE_UC");  // tests: the write-through exchange (form 4)
        const bool force_uc = uenv && atoi(uenv) != 0;
        const uint32_t budget = res_ticks();
        for (uint32_t launch = 0;; ++launch) {
            const hipError_t st = launch_trade_mw(td->a, td->gx, td->gxc, budget, launch * budget, lds, xcd_pack,
                                                  force_uc, e->stream);
            if (st != hipSuccess) return hip_fail(e, "resident tick kernel (workgroups)", st);
            if (int s = poll_ctl(e)) return s;
            // every worker block must be resident at once; when another stream or process holds
            // CUs a bounded exchange sweep gives up: the run is redone on the replayed kernels
            // (MCS_MW_FORCE_TIMEOUT=1: tests take this path after the first launch)
            if (td->h_ctl->flags & kTrFlagMwTimeout) return kMwFallback;
            if (const char* ft = getenv("MCS_MW_FORCE_TIMEOUT"); ft && atoi(ft) != 0) return kMwFallback;
            td->loop_form = td->h_ctl->info ? kLoopResidentMwXcd : kLoopResidentMw;
            if (td->h_ctl->done) return MCS_OK;
        }
    }
    if (rf == 1) {
        td->loop_form = kLoopResident;
        for (;;) {
            const hipError_t st = launch_trade_resident(td->a, res_ticks(), lds, e->stream);
            if (st != hipSuccess) return hip_fail(e, "resident tick kernel", st);
            if (int s = poll_ctl(e)) return s;
            if (td->h_ctl->done) return MCS_OK;
        }
    }
    if (!td->graph) {
        hipGraph_t g = nullptr;
        HIPCHK(e, hipStreamBeginCapture(e->stream, hipStreamCaptureModeThreadLocal));
        for (uint32_t t = 0; t < kGraphTicks; ++t)
            for (int p = 0; p < 4; ++p) {
                const hipError_t st = launch_trade_phase(td->a, p, e->stream);
                if (st != hipSuccess) {
                    (void)hipStreamEndCapture(e->stream, &g);
                    if (g) (void)hipGraphDestroy(g);
                    return hip_fail(e, "trade kernel capture", st);
                }
            }
        HIPCHK(e, hipStreamEndCapture(e->stream, &g));
        const hipError_t st = hipGraphInstantiate(&td->graph, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        if (st != hipSuccess) return hip_fail(e, "hipGraphInstantiate", st);
        td->graph_ticks = kGraphTicks;
    }
    td->loop_form = e->tr_no_resident ? kLoopGraphAfterTimeout : kLoopGraph;
    return replay_until_done(e, [&]() -> int {
        HIPCHK(e, hipGraphLaunch(td->graph, e->stream));
        return MCS_OK;
    });
}

int nccl_fail(mcs_engine* e, const char* what, ncclResult_t r) {
    return fail(e, MCS_E_RCCL, std::string(what) + ": " + ncclGetErrorString(r));
}

// N engines (one per GPU): a tick's one exchange is the in-place ncclAllGather of the ranks'
// blocks over xGMI between phase A and the replicated phases B-D
// Captured once into a hipGraph of kGraphTicks ticks (kernels and all-gathers: no host enqueue per
// tick); eager when the capture is refused.  Every rank captures and replays the same
// sequence, so the collectives stay matched.
// The one-launch tick (r05): tick 0's phase A eagerly, then {in-place ncclAllGather of the blocks,
// tr_rk_kernel (B/C/D of tick n + A of tick n + 1)} per tick, kGraphTicks ticks per captured graph
int run_rccl_rk(mcs_engine* e) {
    TradeDev* td = e->td;
    const TradeArgs& a = td->a;
    ncclComm_t comm = (ncclComm_t)e->comm;
    {
        const hipError_t st = launch_trade_rk(a, 0u, td->rk_lds, e->stream);
        if (st != hipSuccess) return hip_fail(e, "one-launch tick (tick 0)", st);
        td->rk_started = true;
    }
    // tick n gathers buffer n & 1 (a graph replays kGraphTicks ticks, an even count, so the parity
    // of a captured tick is that of its index in the graph)
    const size_t xbuf = (size_t)e->world * a.blk;
    uint32_t cap_t = 0;
    auto gather = [&](uint64_t t, hipStream_t s) -> ncclResult_t {
        unsigned char* xb = td->xb + (size_t)(t & 1u) * xbuf;
        return ncclAllGather(xb + (size_t)e->rank * a.blk, xb, a.blk, ncclUint8, comm, s);
    };
    auto tick = [&](hipStream_t s) -> bool {
        const uint32_t t = cap_t++;
        if (gather(t, s) != ncclSuccess) return false;
        return launch_trade_rk(a, 1u + (t & 1u), td->rk_lds, s) == hipSuccess;
    };
    if (!td->rgraph_tried) {
        td->rgraph_tried = true;
        td->rgraph = capture_tick_graph(e->stream, kGraphTicks, tick);
    }
    td->loop_form = td->rgraph ? kLoopRkGraph : kLoopRkEager;
    return replay_until_done(e, [&]() -> int {
        if (td->rgraph) {
            HIPCHK(e, hipGraphLaunch(td->rgraph, e->stream));
        } else {
            for (uint32_t t = 0; t < kGraphTicks; ++t) {
                const ncclResult_t r = gather(t, e->stream);
                if (r != ncclSuccess) return nccl_fail(e, "ncclAllGather(exchange blocks)", r);
                const hipError_t st = launch_trade_rk(a, 1u + (t & 1u), td->rk_lds, e->stream);
                if (st != hipSuccess) return hip_fail(e, "one-launch tick", st);
            }
        }
        return MCS_OK;
    });
}

int run_rccl(mcs_engine* e) {
    TradeDev* td = e->td;
    if (td->rk) return run_rccl_rk(e);
    const TradeArgs& a = td->a;
    ncclComm_t comm = (ncclComm_t)e->comm;
    auto tick = [&](hipStream_t s) -> bool {
        if (launch_trade_phase(a, 0, s) != hipSuccess) return false;
        if (ncclAllGather(td->xb + (size_t)e->rank * a.blk, td->xb, a.blk, ncclUint8, comm, s) != ncclSuccess)
            return false;
        for (int p = 1; p < 4; ++p)
            if (launch_trade_phase(a, p, s) != hipSuccess) return false;
        return true;
    };
    if (!td->rgraph_tried) {
        td->rgraph_tried = true;
        td->rgraph = capture_tick_graph(e->stream, kGraphTicks, tick);
    }
    td->loop_form = td->rgraph ? kLoopRcclGraph : kLoopRcclEager;
    return replay_until_done(e, [&]() -> int {
        if (td->rgraph) {
            HIPCHK(e, hipGraphLaunch(td->rgraph, e->stream));
        } else {
            for (uint32_t t = 0; t < kGraphTicks; ++t) {
                if (int s = launch_phase(e, a, 0)) return s;
                const ncclResult_t r = ncclAllGather(td->xb + (size_t)e->rank * a.blk, td->xb, a.blk, ncclUint8,
                                                     comm, e->stream);
                if (r != ncclSuccess) return nccl_fail(e, "ncclAllGather(exchange blocks)", r);
                for (int p = 1; p < 4; ++p)
                    if (int s = launch_phase(e, a, p)) return s;
            }
        }
        return MCS_OK;
    });
}

int fill_stats(mcs_engine* e, mcs_trade_stats* ts, mcs_stats* st) {
    TradeDev* td = e->td;
    std::vector<TrCluster> cl(e->C);
    HIPCHK(e, hipStreamSynchronize(e->stream));
    HIPCHK(e, hipMemcpy(cl.data(), td->cl, e->C * sizeof(TrCluster), hipMemcpyDeviceToHost));
    HIPCHK(e, hipMemcpy(td->h_ctl, td->ctl, sizeof(TrCtl), hipMemcpyDeviceToHost));
    const TrCtl& c = *td->h_ctl;
    mcs_trade_stats s{};
    uint32_t flags = c.flags;
    for (uint32_t k = 0; k < e->C; ++k) {
        const uint64_t J = e->job_off[k + 1] - e->job_off[k];
        s.placed += cl[k].placed;
        s.borrowed += cl[k].borrowed;
        s.waited += cl[k].waited;
        s.undecided += J - cl[k].decided;
        s.lent_runs += cl[k].lent_runs;
        s.lent_pending += cl[k].lq_len;
        flags |= cl[k].flags;
    }
    if (c.n_lent > td->a.lent_cap || c.n_trades > td->a.trade_cap) flags |= MCS_FLAG_LOG_OVERFLOW;
    s.trades = c.n_trades;
    s.trades_won = c.n_won;
    s.ticks = c.ticks;
    s.t_final = c.T;
    s.flags = flags;
    s.loop_form = td->loop_form;
    s.block_bytes = td->a.blk;
    s.snaps = td->a.snaps;
    s.agreed = (e->comm || e->tr_agreed) ? 1u : 0u;
    if (ts) *ts = s;
    if (st) {
        st->jobs = e->total_jobs;
        st->placed = s.placed;
        st->waited = s.waited;
        st->unplaced = s.undecided;
        st->clusters = e->C;
        st->deadlocked = 0;
        st->escalations = 0;
        st->slot_pool = td->a.S / 64u;
    }
    return MCS_OK;
}

// a caller-driven block's last kTagBytes: the layout it was written in (TradeDev::tag)
void put_tag(const TradeDev* td, void* out, uint64_t ob) {
    std::memcpy(static_cast<unsigned char*>(out) + ob - kTagBytes, td->tag, kTagBytes);
}

// phase 1: every gathered block must carry this rank's tag (same tick form, snapshots, stride and
// cluster count), else ranks that chose different layouts would read each other's blocks wrongly
int check_tags(mcs_engine* e, const void* in, uint64_t blk) {
    const unsigned char* p = static_cast<const unsigned char*>(in);
    for (uint32_t r = 0; r < e->world; ++r)
        if (std::memcmp(p + (size_t)r * blk + blk - kTagBytes, e->td->tag, kTagBytes) != 0)
            return fail(e, MCS_E_INVALID, "exchange block of rank " + std::to_string(r) +
                                              " has another layout (tick form, snapshots, stride or clusters):"
                                              " agree on the shape with mcs_trade_set_shape");
    return MCS_OK;
}

}  // namespace

void comm_free(mcs_engine* e) {
    if (e->comm) {
        // finalize (flushes the communicator's outstanding work and stops its proxy) before the
        // destroy, so nothing of RCCL's touches the engine's buffers after mcs_engine_destroy frees them
        (void)ncclCommFinalize((ncclComm_t)e->comm);
        (void)ncclCommDestroy((ncclComm_t)e->comm);
    }
    e->comm = nullptr;
}

// the captured tick graphs hold RCCL's graph-user objects (references to the communicator's
// resources): they go before the communicator, which goes before any device memory
void trade_release_graphs(mcs_engine* e) {
    if (TradeDev* td = e->td) {
        if (td->graph) (void)hipGraphExecDestroy(td->graph);
        if (td->rgraph) (void)hipGraphExecDestroy(td->rgraph);
        td->graph = td->rgraph = nullptr;
    }
}

void trade_free(mcs_engine* e) {
    TradeDev* td = e->td;
    if (!td) return;
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    if (td->graph) (void)hipGraphExecDestroy(td->graph);
    if (td->rgraph) (void)hipGraphExecDestroy(td->rgraph);
    dfree(td->tn);
    dfree(td->cl);
    dfree(td->sfin);
    dfree(td->snode);
    dfree(td->scm);
    dfree(td->lq);
    dfree(td->xb);
    dfree(td->gx);
    dfree(td->gxc);
    dfree(td->acc);
    dfree(td->lqp);
    dfree(td->fb);
    dfree(td->tr);
    dfree(td->ctl);
    dfree(td->lent);
    dfree(td->trades);
    dfree(td->lrp);
    dfree(td->tnr);
    if (td->h_ctl) (void)hipHostFree(td->h_ctl);
    for (hipEvent_t& ev : td->pev)
        if (ev) (void)hipEventDestroy(ev);
    for (hipEvent_t& ev : td->tev)
        if (ev) (void)hipEventDestroy(ev);
    delete td;
    e->td = nullptr;
    e->trade_run = false;
}

int trade_cluster_stats(mcs_engine* e, mcs_cluster_stats* out, uint32_t n) {
    TradeDev* td = e->td;
    if (!td) return fail(e, MCS_E_STATE, "no lock-step run");
    std::vector<TrCluster> cl(e->C);
    HIPCHK(e, hipStreamSynchronize(e->stream));
    HIPCHK(e, hipMemcpy(cl.data(), td->cl, e->C * sizeof(TrCluster), hipMemcpyDeviceToHost));
    HIPCHK(e, hipMemcpy(td->h_ctl, td->ctl, sizeof(TrCtl), hipMemcpyDeviceToHost));
    for (uint32_t k = 0; k < n; ++k) {
        mcs_cluster_stats s{};
        s.t_end = td->h_ctl->T;
        s.placed = cl[k].placed;
        s.waited = cl[k].waited;
        s.peak_running = cl[k].peak;
        s.flags = cl[k].flags;
        s.pool = td->a.S / 64u;
        s.iterations = td->h_ctl->ticks;
        s.release_scans = 0;
        out[k] = s;
    }
    return MCS_OK;
}

// every rank must lay its exchange block out alike: the snapshot stride is the largest cluster of
// the whole system, and the cluster count per rank must match (one all-reduce before the run)
int tr_agree_shape(mcs_engine* e) {
    uint32_t* buf = nullptr;
    HIPCHK(e, hipMalloc(&buf, 5 * sizeof(uint32_t)));
    /* max of C and of ~C (= ~min C): every rank sees the same verdict, so a mismatch fails on
     * every rank instead of leaving the ranks with the largest C in the tick loop; the 4th word:
     * some rank cannot pack the one-launch tick's slot payload or sum utilization exactly; the 5th:
     * some rank has a node above 64 cores (a lender can be "big": the blocks carry snapshots) */
    const uint32_t h[5] = {e->max_n, e->C, ~e->C, (e->sums_lt24 && e->slot_pack_ok) ? 0u : 1u, e->cores_le64 ? 0u : 1u};
    uint32_t mx[5] = {0, 0, 0, 0, 0};
    HIPCHK(e, hipMemcpy(buf, h, sizeof(h), hipMemcpyHostToDevice));
    ncclResult_t r = ncclAllReduce(buf, buf, 5, ncclUint32, ncclMax, (ncclComm_t)e->comm, e->stream);
    hipError_t st = hipStreamSynchronize(e->stream);
    if (r == ncclSuccess && st == hipSuccess) st = hipMemcpy(mx, buf, sizeof(mx), hipMemcpyDeviceToHost);
    (void)hipFree(buf);
    if (r != ncclSuccess) return nccl_fail(e, "ncclAllReduce(shape)", r);
    if (st != hipSuccess) return hip_fail(e, "shape exchange", st);
    if (mx[1] != ~mx[2]) return fail(e, MCS_E_INVALID, "sharded lock-step trading needs the same cluster count on every rank");
    e->tr_ns = mx[0];
    e->tr_rk_ok = mx[3] == 0u;
    e->tr_nosnap = mx[4] == 0u;
    e->tr_agreed = true;
    return MCS_OK;
}

// the caller-driven twin of tr_agree_shape / dt_agree_shape's words (mcs_trade_shape_words): the
// caller takes the element-wise max over its ranks
void shape_words(const mcs_engine* e, uint32_t* w) {
    const char* rkenv = getenv("MCS_TRADE_RK");
    const bool want_rk = !rkenv || atoi(rkenv) != 0;
    w[0] = e->max_n;
    w[1] = e->C;
    w[2] = ~e->C;
    w[3] = (e->sums_lt24 && e->slot_pack_ok && want_rk) ? 0u : 1u;
    w[4] = e->cores_le64 ? 0u : 1u;
    w[5] = e->dt_vnodes;
    w[6] = 0u;
    w[7] = 0u;
}

int trade_run(mcs_engine* e, mcs_stats* stats) {
    if (e->world > 1 && !e->comm)
        return fail(e, MCS_E_STATE, "sharded lock-step run needs mcs_comm_init (or mcs_trade_phase)");
    if (e->comm && !e->td)
        if (int s = tr_agree_shape(e)) return s;
    e->tr_lq = e->tr_slots = 0;
    e->tr_no_resident = false;
    e->tr_res_start = !e->comm && !e->cfg.slot_pool && resident_wanted(e);
    struct Reset {
        mcs_engine* e;
        ~Reset() { e->tr_res_start = e->tr_no_resident = false; }
    } reset{e};
    uint32_t escalations = 0;
    for (;;) {
        if (int s = mcs_trade_begin(e)) return s;
        if (e->tr_res_start && !e->tr_slots) {
            size_t lds = 0;
            if (resident_form(e, &lds) == 0) {  // no resident form after all: the auto pool
                e->tr_res_start = false;
                trade_free(e);
                continue;
            }
        }
        // a communicator selects the RCCL loop (world 1 included: one rank's all-gather is a copy)
        const int rs = e->comm ? run_rccl(e) : run_local(e);
        if (rs == kMwFallback) {
            const uint32_t lq = e->tr_lq, sl = e->tr_slots, ns = e->tr_ns;
            trade_free(e);
            e->tr_lq = lq;
            e->tr_slots = sl;
            e->tr_ns = ns;
            e->tr_no_resident = true;
            e->tr_res_start = false;
            continue;
        }
        if (rs) return rs;
        const int s = mcs_trade_end(e, stats);
        if (s != MCS_E_CAPACITY) {
            if (stats) stats->escalations = escalations;
            return s;
        }
        // capacity escalation: the flags are replicated on every rank, so all ranks re-run alike
        const uint32_t flags = e->td->h_ctl->flags, LQ = e->td->a.LQ, S = e->td->a.S;
        bool grew = false;
        if ((flags & MCS_FLAG_LENT_OVERFLOW) && !e->cfg.lent_queue_cap && LQ < kMaxLq) {
            e->tr_lq = std::min<uint32_t>(LQ * 4u, kMaxLq);
            grew = true;
        }
        if ((flags & MCS_FLAG_OVERFLOW) && !e->cfg.slot_pool && S < kTrMaxSlots) {
            e->tr_slots = S * 2u;
            grew = true;
        }
        if (!grew) return s;
        const uint32_t lq = e->tr_lq, sl = e->tr_slots, ns = e->tr_ns;
        trade_free(e);
        e->tr_lq = lq;
        e->tr_slots = sl;
        e->tr_ns = ns;
        ++escalations;
    }
}

}  // namespace mcs

extern "C" {

int mcs_set_shard(mcs_engine* e, uint32_t rank, uint32_t world) {
    if (int st = check_engine(e)) return st;
    if (!e->has_clusters) return fail(e, MCS_E_STATE, "mcs_load_clusters first");
    if (world == 0 || rank >= world) return fail(e, MCS_E_INVALID, "rank must be < world");
    if ((uint64_t)world * e->C > 0xFFFFFFFFull) return fail(e, MCS_E_INVALID, "too many clusters");
    mcs::trade_free(e);
    mcs::dtrade_free(e);
    e->dt_learn_s = e->dt_learn_v = 0;
    e->dt_ns = 0;
    e->tr_ns = 0;
    e->tr_rk_ok = true;
    e->tr_nosnap = false;
    e->tr_agreed = false;
    e->rank = rank;
    e->world = world;
    return MCS_OK;
}

int mcs_comm_unique_id(mcs_comm_id* out) {
    if (!out) return MCS_E_INVALID;
    static_assert(sizeof(mcs_comm_id) == sizeof(ncclUniqueId), "ncclUniqueId size");
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return MCS_E_RCCL;
    std::memcpy(out->bytes, &id, sizeof(id));
    return MCS_OK;
}

int mcs_comm_init(mcs_engine* e, const mcs_comm_id* id) {
    if (int st = check_engine(e)) return st;
    if (!id) return fail(e, MCS_E_INVALID, "null id");
    // the captured tick graphs reference a previous communicator's resources, and the trading
    // states were laid out (and their shape agreed) for another transport: all of them go first, in
    // mcs_engine_destroy's order — graphs, the old communicator (finalized), then the states
    HIPCHK(e, hipStreamSynchronize(e->stream));
    mcs::trade_release_graphs(e);
    mcs::dtrade_release_graphs(e);
    mcs::comm_free(e);
    mcs::trade_free(e);
    mcs::dtrade_free(e);
    e->tr_ns = 0;
    e->dt_ns = 0;
    e->tr_rk_ok = true;
    e->tr_nosnap = false;
    e->tr_agreed = false;
    ncclUniqueId uid;
    std::memcpy(&uid, id->bytes, sizeof(uid));
    ncclComm_t comm = nullptr;
    const ncclResult_t r = ncclCommInitRank(&comm, (int)e->world, uid, (int)e->rank);
    if (r != ncclSuccess) return fail(e, MCS_E_RCCL, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    e->comm = comm;
    return MCS_OK;
}

int mcs_trade_begin(mcs_engine* e) {
    if (int st = check_engine(e)) return st;
    if (mcs::is_dtrade(e)) {
        if (!e->has_jobs) return fail(e, MCS_E_STATE, "mcs_submit_jobs first");
        if (int st = mcs::ensure_job_records(e)) return st;
        return mcs::dtrade_begin(e);
    }
    if (!(e->cfg.borrow || e->cfg.trader)) return fail(e, MCS_E_STATE, "engine config has no borrow/trader");
    if (int st = mcs::trade_alloc(e)) return st;
    mcs::TradeDev* td = e->td;
    td->w0 = std::chrono::steady_clock::now();
    const hipError_t st = mcs::launch_trade_init(td->a, e->stream);
    if (st != hipSuccess) return mcs::hip_fail(e, "trade init", st);
    td->rk_started = false;
    td->rk_tick = 0;
    td->end_ev = nullptr;
    HIPCHK(e, hipStreamSynchronize(e->stream));
    HIPCHK(e, hipEventRecord(e->ev0, e->stream));  // kernel_ms: the lock-step loop only
    td->begun = true;
    e->has_run = false;
    e->trade_run = false;
    return MCS_OK;
}

int mcs_trade_shape_words(mcs_engine* e, uint32_t* out) {
    if (int st = check_engine(e)) return st;
    if (!out) return fail(e, MCS_E_INVALID, "null output");
    if (!e->has_clusters) return fail(e, MCS_E_STATE, "mcs_load_clusters first");
    mcs::shape_words(e, out);
    return MCS_OK;
}

int mcs_trade_set_shape(mcs_engine* e, const uint32_t* w) {
    if (int st = check_engine(e)) return st;
    if (!w) return fail(e, MCS_E_INVALID, "null shape");
    if (!e->has_clusters) return fail(e, MCS_E_STATE, "mcs_load_clusters first");
    // (the max over ranks of C and of ~C: equal exactly when every rank holds the same count)
    if (w[1] != ~w[2] || w[1] != e->C)
        return fail(e, MCS_E_INVALID, "sharded lock-step trading needs the same cluster count on every rank");
    if (w[0] < e->max_n || w[0] > mcs::kTrMaxNodes)
        return fail(e, MCS_E_INVALID, "agreed snapshot stride below this rank's largest cluster (not a max over ranks)");
    uint32_t mine[MCS_TRADE_SHAPE_WORDS];
    mcs::shape_words(e, mine);
    if (w[3] < mine[3] || w[4] < mine[4] || w[5] < mine[5] || w[6] || w[7])
        return fail(e, MCS_E_INVALID, "agreed shape words are not a max over ranks that include this one");
    mcs::trade_free(e);
    mcs::dtrade_free(e);
    e->tr_ns = w[0];
    e->dt_ns = w[0];
    e->tr_rk_ok = w[3] == 0u;
    e->tr_nosnap = w[4] == 0u;
    e->dt_vnodes = w[5];
    e->tr_agreed = true;
    return MCS_OK;
}

int mcs_trade_xfer_bytes(mcs_engine* e, uint32_t phase, uint64_t* in_bytes, uint64_t* out_bytes) {
    if (!e || !in_bytes || !out_bytes || phase > 3) return MCS_E_INVALID;
    if (mcs::is_dtrade(e)) return mcs::dtrade_xfer_bytes(e, phase, in_bytes, out_bytes);
    // one exchange per tick: phase 0 writes this rank's block, phase 1 takes every rank's blocks;
    // phases 2 and 3 move no bytes.  The block layout is trade_alloc's (the state is allocated
    // here when it is not yet: mcs_trade_begin reuses it)
    if (!e->td)
        if (int st = mcs::trade_alloc(e)) return st;
    const uint64_t blk = e->td->a.blk;
    switch (phase) {
        case 0: *in_bytes = 0; *out_bytes = blk; break;
        case 1: *in_bytes = (uint64_t)e->world * blk; *out_bytes = 0; break;
        default: *in_bytes = 0; *out_bytes = 0; break;
    }
    return MCS_OK;
}

int mcs_trade_phase(mcs_engine* e, uint32_t phase, const void* in, uint64_t in_bytes, void* out,
                    uint64_t out_bytes, uint32_t* done) {
    if (int st = check_engine(e)) return st;
    if (mcs::is_dtrade(e)) return mcs::dtrade_phase(e, phase, in, in_bytes, out, out_bytes, done);
    mcs::TradeDev* td = e->td;
    if (!td || !td->begun) return fail(e, MCS_E_STATE, "mcs_trade_begin first");
    uint64_t ib = 0, ob = 0;
    if (int st = mcs_trade_xfer_bytes(e, phase, &ib, &ob)) return fail(e, st, "bad phase");
    if (in_bytes != ib || out_bytes != ob || (ib && !in) || (ob && !out))
        return fail(e, MCS_E_INVALID, "exchange buffer sizes do not match mcs_trade_xfer_bytes");
    const mcs::TradeArgs& a = td->a;
    if (phase == 1)
        if (int st = mcs::check_tags(e, in, a.blk)) return st;
    if (td->rk) {  // the one-launch tick: phase 1 runs B/C/D of tick n and A of tick n + 1
        td->loop_form = mcs::kLoopRkDriven;
        hipError_t hs = hipSuccess;
        unsigned char* const xb = td->xb + (size_t)(td->rk_tick & 1u) * ((size_t)e->world * a.blk);  // tick n's buffer
        switch (phase) {
            case 0:
                if (!td->rk_started) {
                    hs = mcs::launch_trade_rk(a, 0u, td->rk_lds, e->stream);
                    td->rk_started = true;
                }
                if (hs == hipSuccess)
                    hs = hipMemcpyAsync(out, xb + (size_t)e->rank * a.blk, ob, hipMemcpyDeviceToHost, e->stream);
                break;
            case 1:
                hs = hipMemcpyAsync(xb, in, ib, hipMemcpyHostToDevice, e->stream);
                if (hs == hipSuccess) hs = mcs::launch_trade_rk(a, 1u + (uint32_t)(td->rk_tick & 1u), td->rk_lds, e->stream);
                ++td->rk_tick;
                break;
            case 2:
                break;
            default:  // (the copy the last launch wrote)
                hs = hipMemcpyAsync(td->h_ctl, td->ctl + (td->rk_tick & 1u), sizeof(mcs::TrCtl),
                                    hipMemcpyDeviceToHost, e->stream);
                break;
        }
        if (hs != hipSuccess) return mcs::hip_fail(e, "one-launch tick (caller-driven)", hs);
        HIPCHK(e, hipStreamSynchronize(e->stream));
        if (phase == 0) mcs::put_tag(td, out, ob);
        if (done) *done = phase == 3 ? td->h_ctl->done : 0u;
        return MCS_OK;
    }
    switch (phase) {
        case 0:
            if (int s = mcs::launch_phase(e, a, 0)) return s;
            HIPCHK(e, hipMemcpyAsync(out, td->xb + (size_t)e->rank * a.blk, ob, hipMemcpyDeviceToHost, e->stream));
            break;
        case 1:
            HIPCHK(e, hipMemcpyAsync(td->xb, in, ib, hipMemcpyHostToDevice, e->stream));
            if (int s = mcs::launch_phase(e, a, 1)) return s;
            break;
        case 2:
            if (int s = mcs::launch_phase(e, a, 2)) return s;
            break;
        default:
            if (int s = mcs::launch_phase(e, a, 3)) return s;
            HIPCHK(e, hipMemcpyAsync(td->h_ctl, td->ctl, sizeof(mcs::TrCtl), hipMemcpyDeviceToHost,
                                     e->stream));
            break;
    }
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if (phase == 0) mcs::put_tag(td, out, ob);
    if (done) *done = phase == 3 ? td->h_ctl->done : 0u;
    return MCS_OK;
}

int mcs_trade_end(mcs_engine* e, mcs_stats* stats) {
    if (int st = check_engine(e)) return st;
    if (stats) *stats = mcs_stats{};
    if (mcs::is_dtrade(e)) return mcs::dtrade_end(e, stats);
    mcs::TradeDev* td = e->td;
    if (!td || !td->begun) return fail(e, MCS_E_STATE, "mcs_trade_begin first");
    if (td->rk && (td->rk_tick & 1u)) {  // caller-driven one-launch tick: the final copies into the first
        HIPCHK(e, hipMemcpyAsync(td->ctl, td->ctl + 1, sizeof(mcs::TrCtl), hipMemcpyDeviceToDevice, e->stream));
        HIPCHK(e, hipMemcpyAsync(td->tr, td->tr + td->a.Ct, td->a.Ct * sizeof(mcs::TrTrader),
                                 hipMemcpyDeviceToDevice, e->stream));
    }
    HIPCHK(e, hipEventRecord(e->ev1, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    e->has_run = true;
    e->trade_run = true;
    e->delay_run = false;
    e->dtrade_run = false;
    mcs_trade_stats ts{};
    mcs_stats st{};
    if (int s = mcs::fill_stats(e, &ts, &st)) return s;
    float ms = 0.0f;
    if (hipEventElapsedTime(&ms, e->ev0, td->end_ev ? td->end_ev : e->ev1) != hipSuccess) ms = 0.0f;
    st.kernel_ms = ms;
    st.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - td->w0).count();
    if (stats) *stats = st;
    if (ts.flags & MCS_FLAG_OVERFLOW)
        return fail(e, MCS_E_CAPACITY, "running-slot pool overflow (raise mcs_config.slot_pool)");
    if (ts.flags & MCS_FLAG_LENT_OVERFLOW)
        return fail(e, MCS_E_CAPACITY, "LentQueue overflow (raise mcs_config.lent_queue_cap)");
    return MCS_OK;
}

int mcs_read_trade_stats(mcs_engine* e, mcs_trade_stats* out) {
    if (int st = check_engine(e)) return st;
    if (!out) return fail(e, MCS_E_INVALID, "null output");
    if (e->dtrade_run && e->dtd) return mcs::dtrade_trade_stats(e, out);
    if (!e->trade_run || !e->td) return fail(e, MCS_E_STATE, "no lock-step run");
    mcs_stats st{};
    if (int s = mcs::fill_stats(e, out, &st)) return s;
    float ms = 0.0f;
    if (hipEventElapsedTime(&ms, e->ev0, e->td->end_ev ? e->td->end_ev : e->ev1) != hipSuccess) ms = 0.0f;
    out->kernel_ms = ms;
    out->wall_ms = 0.0;
    return MCS_OK;
}

int mcs_read_lent(mcs_engine* e, mcs_lent_rec* out, uint64_t cap, uint64_t* n) {
    if (int st = check_engine(e)) return st;
    if (!n || (cap && !out)) return fail(e, MCS_E_INVALID, "bad output");
    if (e->dtrade_run && e->dtd) {  // Delay never borrows: no lent runs
        *n = 0;
        return MCS_OK;
    }
    if (!e->trade_run || !e->td) return fail(e, MCS_E_STATE, "no lock-step run");
    mcs::TradeDev* td = e->td;
    HIPCHK(e, hipStreamSynchronize(e->stream));
    HIPCHK(e, hipMemcpy(td->h_ctl, td->ctl, sizeof(mcs::TrCtl), hipMemcpyDeviceToHost));
    const uint64_t total = td->h_ctl->n_lent;
    const uint64_t have = std::min<uint64_t>(total, td->a.lent_cap);
    std::vector<mcs_lent_rec> v(have);
    if (have) HIPCHK(e, hipMemcpy(v.data(), td->lent, have * sizeof(mcs_lent_rec), hipMemcpyDeviceToHost));
    std::sort(v.begin(), v.end(), [](const mcs_lent_rec& x, const mcs_lent_rec& y) {
        if (x.start_s != y.start_s) return x.start_s < y.start_s;
        if (x.lender != y.lender) return x.lender < y.lender;
        if (x.borrower != y.borrower) return x.borrower < y.borrower;
        return x.job < y.job;
    });
    const uint64_t k = std::min<uint64_t>(have, cap);
    if (k) std::memcpy(out, v.data(), k * sizeof(mcs_lent_rec));
    *n = total;
    return MCS_OK;
}

int mcs_read_trades(mcs_engine* e, mcs_trade_rec* out, uint64_t cap, uint64_t* n) {
    if (int st = check_engine(e)) return st;
    if (!n || (cap && !out)) return fail(e, MCS_E_INVALID, "bad output");
    if (e->dtrade_run && e->dtd) return mcs::dtrade_read_trades(e, out, cap, n);
    if (!e->trade_run || !e->td) return fail(e, MCS_E_STATE, "no lock-step run");
    mcs::TradeDev* td = e->td;
    HIPCHK(e, hipStreamSynchronize(e->stream));
    HIPCHK(e, hipMemcpy(td->h_ctl, td->ctl, sizeof(mcs::TrCtl), hipMemcpyDeviceToHost));
    const uint64_t total = td->h_ctl->n_trades;
    const uint64_t k = std::min<uint64_t>(std::min<uint64_t>(total, td->a.trade_cap), cap);
    if (k) HIPCHK(e, hipMemcpy(out, td->trades, k * sizeof(mcs_trade_rec), hipMemcpyDeviceToHost));
    *n = total;
    return MCS_OK;
}

int mcs_read_virtual_nodes(mcs_engine* e, uint32_t* out, uint32_t n_total) {
    if (int st = check_engine(e)) return st;
    if (e->dtrade_run && e->dtd) {
        if (!out || n_total > e->C * e->world) return fail(e, MCS_E_INVALID, "bad output");
        return mcs::dtrade_read_vnode_counts(e, out, n_total);
    }
    if (!e->trade_run || !e->td) return fail(e, MCS_E_STATE, "no lock-step run");
    const uint32_t Ct = e->C * e->world;
    if (!out || n_total > Ct) return fail(e, MCS_E_INVALID, "bad output");
    std::vector<mcs::TrTrader> t(Ct);
    HIPCHK(e, hipStreamSynchronize(e->stream));
    HIPCHK(e, hipMemcpy(t.data(), e->td->tr, Ct * sizeof(mcs::TrTrader), hipMemcpyDeviceToHost));
    for (uint32_t k = 0; k < n_total; ++k) out[k] = t[k].vnodes;
    return MCS_OK;
}

}  // extern "C"
