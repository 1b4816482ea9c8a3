// mcs_dtrade.hip — gfx950 kernels of the lock-step trading system with DELAY schedulers
// (semantics restated in oracle/mcs_oracle_dtrade.c, header of mcs_dtrade_internal.h).
//
// One tick T is two launches on the engine stream (each a grid-wide barrier); with world 1 they are
// replayed from a captured hipGraph 64 ticks at a time, with world > 1 an all-gather of the
// exchange blocks (RCCL over xGMI, or the caller's transport) sits between them:
//   A dt_step_kernel    one wave per local cluster: one Delay iteration (pkg/scheduler/scheduler.go:
//                       298-369): releases, "/delay" arrivals, the Level1 pass with its skip (D6)
//                       through an exact fit filter, the Level0 head and its MaxWaitTime move,
//                       and the WaitTime statistics (scheduler.go:309-312,338-341); then phase C,
//                       the state sample at T % 5 == 0, on the same wave (it reads only its own
//                       cluster): GetResourceUtilization over physical and virtual nodes
//                       (cluster.go:46-63, float32 in node order) and WaitTime.GetAverage
//                       (scheduler.go:56-63); then the cluster's exchange record (DtRec) and, when
//                       a trader round is due, its node snapshot and the contract sizes over its
//                       Level1 (scheduler_client.go:126-289)
//   D dt_trader_kernel  one wave for the whole system, replicated on every rank: trader rounds in
//                       cluster order (trader.go:280-325), RequestResource/ApproveTrade with locks
//                       across lanes (pkg/trader/server.go:31-61, trader.go:141-167), heap order,
//                       ApproveContract -> AllocateVirtualNodeResources on the responder's snapshot
//                       (Foreign jobs, cluster.go:87-125; the owner rank also commits them to its
//                       live nodes and running slots) and AddVirtualNode on the requester
//                       (cluster.go:65-85); then the next tick.
// Per-cluster state a wave writes and re-reads inside a kernel is staged in LDS, or read back with
// sc1 loads (L2) after an atomic write, never through this CU's non-coherent vector L1.
// The phases' code is shared with the resident tick (mcs_dtrade_mw.hip) in mcs_dtrade_dev.h.
#include "mcs_dtrade_dev.h"

namespace mcs {
namespace {

// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void dt_init_kernel(DtArgs a) {
    const uint32_t c = blockIdx.x, lane = threadIdx.x;
    const uint32_t n0 = a.node_off[c], N = a.node_off[c + 1] - n0;
    uint32_t sc = 0, sm = 0;
    for (uint32_t i = lane; i < N; i += kWave) {
        const uint2 f = a.free0[n0 + i];
        a.tn[n0 + i] = (unsigned long long)f.x | ((unsigned long long)f.y << 32);
        const uint2 cp = a.cap[n0 + i];
        sc += cp.x;  // SetTotalResources: uint32 sums (cluster.go:34-37)
        sm += cp.y;
    }
    sc = dt_wave_sum_u32(sc);
    sm = dt_wave_sum_u32(sm);
    for (uint32_t s = lane; s < a.S; s += kWave) a.sfin[(size_t)c * a.S + s] = kEmpty;
    for (uint32_t i = lane; i < a.W; i += kWave) a.l1snap[(size_t)c * a.W + i] = 0ull;  // every node "grown"
    const uint64_t j0 = a.job_off[c], j1 = a.job_off[c + 1];
    for (uint64_t j = j0 + lane; j < j1; j += kWave) {
        a.out_node[j] = MCS_NODE_UNPLACED;
        a.out_start[j] = MCS_TIME_NONE;
        a.out_finish[j] = MCS_TIME_NONE;
    }
    if (lane == 0) {
        DtCluster z{};
        z.minf = kEmpty;
        z.head_last = kEmpty;
        z.total_c = sc;
        z.total_m = sm;
        a.cl[c] = z;
    }
    // the replicated trader state of every cluster of the system: block c takes c, c + C, ...
    for (uint32_t g = c + lane * a.C; g < a.Ct; g += kWave * a.C) {
        DtTrader t{};
        t.next_id = 1u;  // s.id = rand.Uint32() (pkg/trader/server.go:26), seeded: 1
        a.tr[g] = t;
        a.nv_all[g] = 0u;
    }
    if (c == 0 && lane == 0) {
        DtCtl z{};
        z.any_due = 1u;
        *a.ctl = z;
    }
}

// ---------------------------------------------------------------------------------------------
// Phase A: one Delay iteration of cluster c at tick T.
__global__ __launch_bounds__(64) void dt_step_kernel(DtArgs a) {
    __shared__ unsigned long long nodes[kDtMaxNodes + kDtMaxVnodes];
    __shared__ uint32_t sfin[kDtMaxSlots];
    __shared__ uint32_t hist[kWave];
    if (a.ctl->done) return;
#ifdef MCS_STAMPS
    uint64_t dt_acc[7] = {0, 0, 0, 0, 0, 0, 0};
    uint64_t dt_last = wall_clock64();
#endif
    const uint32_t T = a.ctl->T;
    const uint32_t c = blockIdx.x, lane = threadIdx.x;
    const uint32_t n0 = a.node_off[c], N = a.node_off[c + 1] - n0;
    const uint64_t j0 = a.job_off[c];
    const uint32_t J = (uint32_t)(a.job_off[c + 1] - j0);
    const uint4* __restrict__ jobs = a.jobs + j0;
    unsigned long long* __restrict__ l1cm = a.l1cm + j0;
    unsigned long long* __restrict__ l1jd = a.l1jd + j0;
    unsigned long long* __restrict__ l1al = a.l1al + j0;
    const size_t sb = (size_t)c * a.S;
    const uint32_t S = a.S;
    DtCluster st = a.cl[c];
    const uint32_t NN = N + st.nv;
    const bool exact = NN <= (uint32_t)kWave;  // small clusters: per-lane exact first fit
    // (exact clusters) the node values the Level1 jobs last failed against: taken at the end of each
    // pass, lowered at each move to Level1; a job that failed every node can fit now only on a node
    // that grew past it since (releases, new virtual nodes, wrapped counters), or if it was skipped
    // (D6) and so never tested: the pass tests the others against the grown nodes only
    unsigned long long snap_l = exact && lane < NN ? a.l1snap[(size_t)c * a.W + lane] : 0ull;
    bool snap_dirty = false;
    copy_rounds<4>(nodes, a.tn + n0, N, lane);
    copy_rounds<2>(nodes + N, a.vn + (size_t)c * a.V, NN - N, lane);
    copy_rounds<8>(sfin, a.sfin + sb, S, lane);
    __syncthreads();
    DT_MARK(0);

    DtArrWin aw{kEmpty, kEmpty};  // (a fresh window every tick: the step kernel keeps nothing)
    st = dt_phase_a<false>(a, c, lane, T, N, NN, exact, j0, J, jobs, l1cm, l1jd, l1al, sb, S, nodes, sfin, hist, st, snap_l,
                      snap_dirty, aw DT_STAMP_ARGS);

    DT_MARK(4);
    if (snap_dirty && lane < NN) a.l1snap[(size_t)c * a.W + lane] = snap_l;
    __syncthreads();
    copy_rounds<4>(a.tn + n0, nodes, N, lane);
    copy_rounds<2>(a.vn + (size_t)c * a.V, nodes + N, NN - N, lane);
    copy_rounds<8>(a.sfin + sb, sfin, S, lane);
    // ---- phase C: the state stream sample (trader_server.go:24-47) every sample_period seconds ----
    dt_sample<false>(a, c, lane, T, n0, N, NN, nodes, reinterpret_cast<float*>(sfin),
                     reinterpret_cast<float*>(sfin) + (kDtMaxNodes + kDtMaxVnodes), st);
    if (lane == 0) a.cl[c] = st;
    DT_MARK(5);

    // ---- this cluster's exchange record and, when a trader round is due at T, its node
    // snapshot and both contract sizes over GetLevel1() (ProvideJobs, trader_server.go:69-94) ----
    const uint32_t g = a.base + c;
    unsigned char* blk = a.xb + (size_t)a.rank * a.blk;
    unsigned long long* snap =
        reinterpret_cast<unsigned long long*>(blk + (size_t)a.C * sizeof(DtRec)) + (size_t)c * a.W;
    const bool any_due = a.period != 0u && a.ctl->any_due != 0u;
    if (any_due)
        for (uint32_t i = lane; i < NN; i += kWave) snap[i < N ? i : a.NS + (i - N)] = nodes[i];
    uint32_t fsc = 0, fsm = 0, fmd = 0, ssc = 0, ssm = 0, sst = 0;
    dt_contracts<false>(any_due && a.tr[g].next_due <= T, lane, st.l1n, l1cm, l1jd, hist, fsc, fsm, fmd, ssc, ssm, sst);
    if (lane == 0) {
        DtRec r;
        r.cu = st.cu;
        r.mu = st.mu;
        r.avgw = st.avgw;
        r.total_c = st.total_c;
        r.total_m = st.total_m;
        r.nv = st.nv;
        r.N = N;
        r.nfree = S - st.nrun;
        r.flags = st.flags;
        r.done = st.decided == J ? 1u : 0u;
        r.queued = (st.l1n > 0u || st.next_arr > st.l0_head) ? 1u : 0u;
        r.nxt = st.next_arr < J ? jobs[st.next_arr].x : kEmpty;
        r.fc = fsc;
        r.fm = fsm;
        r.ft = fmd;
        r.sc = ssc;
        r.sm = ssm;
        r.st = sst;
        r.pad = 0u;
        reinterpret_cast<DtRec*>(blk)[c] = r;
    }
#ifdef MCS_STAMPS
    DT_MARK(6);
    if (lane == 0) {
        unsigned long long tot = 0;
        for (int i = 0; i < 7; ++i) {
            atomicAdd(&g_dt_stamps[i], (unsigned long long)dt_acc[i]);
            atomicMax(&g_dt_cur[i], (unsigned long long)dt_acc[i]);
            tot += dt_acc[i];
        }
        atomicMax(&g_dt_cur[7], tot);
        atomicAdd(&g_dt_stamps[7], 1ull);
    }
#endif
}

// ---------------------------------------------------------------------------------------------
// Phase D: trader rounds in cluster order over the whole system, then the next tick.  Every rank
// runs it on the same gathered records and replicated trader state, so every decision is identical
// on every rank; a rank applies the side effects on its own clusters (Foreign jobs, virtual nodes)
// to its live state as well as to the snapshot the later rounds of this tick read.
__global__ __launch_bounds__(64) void dt_trader_kernel(DtArgs a) {
    __shared__ DtTrader trs[kDtMaxClusters];
    __shared__ uint32_t appr[kDtMaxClusters];
    __shared__ uint32_t nvs[kDtMaxClusters];  // virtual nodes per cluster (written here)
    __shared__ uint32_t nfr[kDtMaxClusters];  // free running slots per cluster (taken here)
    // every cluster's record of the tick, copied once: the rounds read a requester's sample and
    // contract sizes and every responder's totals and sample (each an L2 round trip per round
    // otherwise); no round writes a record
    extern __shared__ DtRec srec[];  // [Ct] (dynamic)
#ifdef MCS_STAMPS
    const uint64_t tr_t0 = wall_clock64();
#endif
    // the control block and every record in one batch of loads: the done test comes after them
    // (a return before them would make every load wait for the control block's round trip)
    static_assert(sizeof(DtCtl) == 3 * sizeof(uint4), "DtCtl copy");
    DtCtl c0;
    {
        const uint4* cp = reinterpret_cast<const uint4*>(a.ctl);
        uint4* cd = reinterpret_cast<uint4*>(&c0);
        const uint4 x0 = cp[0], x1 = cp[1], x2 = cp[2];
        cd[0] = x0;
        cd[1] = x1;
        cd[2] = x2;
    }
    const uint32_t T = c0.T;
    const bool any_due = c0.any_due != 0u;
    const uint32_t lane = threadIdx.x;
    const uint32_t Ct = a.Ct;
    for (uint32_t q = lane; q < Ct; q += kWave) {
        trs[q] = a.tr[q];
        const uint4* rq = reinterpret_cast<const uint4*>(dt_rec(a, q));
        uint4* rd = reinterpret_cast<uint4*>(&srec[q]);
        static_assert(sizeof(DtRec) == 5 * sizeof(uint4), "DtRec copy");
        const uint4 w0 = rq[0], w1 = rq[1], w2 = rq[2], w3 = rq[3], w4 = rq[4];
        rd[0] = w0;
        rd[1] = w1;
        rd[2] = w2;
        rd[3] = w3;
        rd[4] = w4;
        nvs[q] = srec[q].nv;
        nfr[q] = srec[q].nfree;
    }
    __syncthreads();
    if (c0.done) return;  // (uniform: after the block-wide barrier above)
    const DtCounts k = dt_rounds<false>(a, lane, T, any_due, trs, srec, appr, nvs, nfr,
                                        DtCounts{c0.n_trades, c0.n_won, c0.n_foreign, 0u},
                                        DtOpQueue{nullptr, nullptr, 0u});
    const unsigned long long n_trades = k.n_trades, n_won = k.n_won, n_for = k.n_for;
    const uint32_t lflags = k.lflags;

    const DtCtl nc = dt_next_ctl(a, lane, c0, trs, srec, lflags, n_trades, n_won, n_for);
    __syncthreads();
    for (uint32_t q = lane; q < Ct; q += kWave) {
        a.tr[q] = trs[q];
        a.nv_all[q] = nvs[q];
    }
    if (lane == 0) {
        DtCtl* ctl = a.ctl;
        ctl->T = nc.T;
        ctl->done = nc.done;
        ctl->any_due = nc.any_due;
        ctl->ticks = nc.ticks;
        ctl->flags = nc.flags;
        ctl->n_trades = nc.n_trades;
        ctl->n_won = nc.n_won;
        ctl->n_foreign = nc.n_foreign;
#ifdef MCS_STAMPS
        for (int i = 0; i < 8; ++i) {
            g_dt_maxsum[i] += g_dt_cur[i];
            g_dt_cur[i] = 0ull;
        }
        g_dt_maxsum[8] += wall_clock64() - tr_t0;
        g_dt_maxsum[9] += 1ull;
#endif
    }
}

// The single-call mirror of ApproveTrade (mcs_approve_trade): the kernels' own device function on
// caller-given samples and contracts, one query per thread.
__global__ __launch_bounds__(256) void approve_kernel(const mcs_approve_query* q, uint32_t n, int32_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const mcs_approve_query x = q[i];
    out[i] = approve_trade_dev(x.total_cores, x.total_memory, x.core_util, x.mem_util, x.cores, x.memory,
                               x.time_s) ? 1 : 0;
}

}  // namespace

hipError_t launch_approve(const mcs_approve_query* q, uint32_t n, int32_t* out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(approve_kernel, dim3((n + 255) / 256), dim3(256), 0, s, q, n, out);
    return hipGetLastError();
}

hipError_t launch_dtrade_init(const DtArgs& a, hipStream_t s) {
    if (a.C == 0) return hipSuccess;
    hipLaunchKernelGGL(dt_init_kernel, dim3(a.C), dim3(kWave), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_dtrade_step(const DtArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(dt_step_kernel, dim3(a.C), dim3(kWave), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_dtrade_trader(const DtArgs& a, hipStream_t s) {
    const size_t lds = (size_t)a.Ct * sizeof(DtRec);
    const hipError_t st = hipFuncSetAttribute((const void*)dt_trader_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (st != hipSuccess) return st;
    hipLaunchKernelGGL(dt_trader_kernel, dim3(1), dim3(kWave), lds, s, a);
    return hipGetLastError();
}

hipError_t launch_dtrade_tick(const DtArgs& a, hipStream_t s) {
    const hipError_t st = launch_dtrade_step(a, s);
    if (st != hipSuccess) return st;
    return launch_dtrade_trader(a, s);
}

}  // namespace mcs

#ifdef MCS_STAMPS
// the probe build's dt_step segment sums (see g_dt_stamps), read and cleared
extern "C" int mcs_debug_dt_stamps(unsigned long long* out) {
    unsigned long long z[8] = {};
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(mcs::g_dt_stamps), sizeof(z)) != hipSuccess) return -1;
    return hipMemcpyToSymbol(HIP_SYMBOL(mcs::g_dt_stamps), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
// the Level1 pass's row split (see g_dt_rows), read and cleared
extern "C" int mcs_debug_dt_rows(unsigned long long* out) {
    unsigned long long z[4] = {};
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(mcs::g_dt_rows), sizeof(z)) != hipSuccess) return -1;
    return hipMemcpyToSymbol(HIP_SYMBOL(mcs::g_dt_rows), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
// the per-tick maxima summed over ticks and the trader kernel's time (see g_dt_maxsum), read and cleared
extern "C" int mcs_debug_dt_maxsum(unsigned long long* out) {
    unsigned long long z[10] = {};
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(mcs::g_dt_maxsum), sizeof(z)) != hipSuccess) return -1;
    return hipMemcpyToSymbol(HIP_SYMBOL(mcs::g_dt_maxsum), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
