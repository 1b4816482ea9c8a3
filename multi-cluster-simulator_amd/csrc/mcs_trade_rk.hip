// mcs_trade_rk.hip — the lock-step FIFO trading tick for N ranks in ONE launch per tick (r05).
//
// The RCCL tick loop used to run four launches and one all-gather per tick (tr_step / tr_lend /
// tr_trader, mcs_trade.hip).  Here a tick is {tr_rk_kernel, in-place ncclAllGather of the ranks'
// exchange blocks}, captured in a hipGraph: launch n runs phases B, C and D of tick n — replicated on
// every rank over the whole system, from the gathered blocks — and then phase A of tick n + 1 for
// this rank's clusters, which writes the rank's block for the next all-gather.  The layout is the
// workgroup-resident tick's (mcs_trade_mw.hip): one wave per cluster of the system, 4 clusters per
// workgroup, so every rank launches the same ceil(C_t / 4) workgroups:
//   X1  (launch start) wave 0 of every workgroup reads every cluster's post-A record from the
//       gathered blocks (one 64-byte record per cluster, RkRec below)
//   B   every workgroup computes the whole tick's acceptance matrix (Lend, strict '>',
//       scheduler.go:194-202, every lender against every request): lender L accepts (c, m) when
//       G_L[c] > m, G_L[x] = max free_m over L's post-A nodes with free_c > x, a 64-entry table its
//       owner builds in phase A and ships in the block (a lender with some free_c > 64 is scanned
//       from its snapshot instead).  So the acceptances need no exchange inside the launch: every
//       workgroup moves its own borrowers' WaitQueue heads to the BorrowedQueue
//       (scheduler.go:237-242), every lender's wave appends to its LentQueue in borrower order
//       (server.go:80-113, owner rank), and the append-overflow verdict is replicated
//   C+D a fifth (helper) wave of every workgroup on identical inputs, while the cluster waves run B:
//       the trader rounds (trader.go:280-325, 193-278; server.go:31-85) and the next tick's clock —
//       replicated, as in the MW tick
//   A   tick n + 1 (tr_step_kernel's phase, scheduler.go:216-296 + the borrow request): this rank's
//       waves; the record and the node snapshot go to the rank's block of the exchange buffer
// The workgroups never wait for each other (no granule exchange, no co-residency requirement).
// A launch is latency-bound: every load B-D needs issues in one batch at the start,
// phase A's nodes and slot rows right after the first barrier (they land during B-D), and phase A
// keeps the nodes in registers.
// The first launch of a run (mode 0) runs phase A of tick 0 only.  The state between launches
// (nodes, running slots, queue cursors, trader state, the clock) lives in HBM, as across the MW
// kernel's launches.  The caller-driven phase API (mcs_trade_phase) runs the same launches with the
// caller's all-gather in between, so 2- and 4-rank runs over gloo cover this path on one GPU.
// Same results bit for bit as the three-kernel tick and the oracle (tests/test_gpu_trade.py,
// tests/trade_2rank.py).
#include "mcs_trade_internal.h"
#include "mcs_trader_dev.h"
#include "mcs_wave.h"

namespace mcs {
namespace {

constexpr int kRkWaves = 4;                // clusters (waves) per workgroup
constexpr uint32_t kRkNodes = 256;         // nodes per cluster
constexpr uint32_t kRkLenders = kTrResMaxClusters / kRkWaves;  // lenders per wave in phase B
// + one helper wave per workgroup: phases C/D (the trader rounds and the clock) while the cluster
// waves run phase B, so the two overlap instead of adding up on wave 0
constexpr int kRkThreads = (kRkWaves + 1) * kWave;

// a cluster's post-A record in the exchange block: 16 words, the size of TrXRec (the three-kernel
// record), so both forms lay the blocks out alike (records, then the node snapshots)
enum : uint32_t {
    kRkJob = 0, kRkC, kRkM, kRkDur, kRkQs, kRkDecided, kRkNat, kRkFlags, kRkCu, kRkMu, kRkLq, kRkN, kRkTc, kRkTm,
    kRkWords = 16
};
static_assert(kRkWords * 4u == sizeof(TrXRec), "record size");
// qs bits: WaitQueue head, ReadyQueue busy, a lent run this tick, LentQueue non-empty, cluster done,
// some node with free_c > 64 (no G table: phase B scans the snapshot)
constexpr uint32_t kQsW = 1u, kQsRq = 2u, kQsLent = 4u, kQsLq = 8u, kQsDone = 16u, kQsBig = 32u;

// a wave's uint32 sum (wrapping), on the DPP scan: VALU steps, no LDS-pipe round trips
__device__ __forceinline__ uint32_t rk_wave_sum(uint32_t v) { return readlane(wave_scan_add_u32(v), 63u); }
// a wave's OR of a flags word: one ballot per bit some lane holds (none on most ticks)
__device__ __forceinline__ uint32_t rk_wave_or(uint32_t v) {
    uint32_t r = 0u;
    if (__ballot(v != 0u))
        for (uint32_t b = 0; b < 32u; ++b)
            if (__ballot((v >> b) & 1u)) r |= 1u << b;
    return r;
}
// The exchange blocks are double-buffered by tick parity: launch n reads tick n's blocks (buffer
// n & 1, gathered) while its phase A writes tick n + 1's (buffer (n + 1) & 1), so a workgroup that
// reaches phase A early never overwrites a record, G table or snapshot another workgroup of the
// launch is still reading (the workgroups do not wait for each other).
// cluster g's record, node snapshot and G table in the buffer at xb (its rank's block: the records,
// then the snapshots, then the G tables)
__device__ __forceinline__ unsigned char* rk_blk(const TradeArgs& a, unsigned char* xb, uint32_t g, uint32_t* c) {
    const uint32_t r = g / a.Cl;
    *c = g - r * a.Cl;
    return xb + (size_t)r * a.blk;
}
__device__ __forceinline__ uint32_t* rk_rec(const TradeArgs& a, unsigned char* xb, uint32_t g) {
    uint32_t c;
    unsigned char* b = rk_blk(a, xb, g, &c);
    return reinterpret_cast<uint32_t*>(b + (size_t)c * sizeof(TrXRec));
}
__device__ __forceinline__ unsigned long long* rk_snap(const TradeArgs& a, unsigned char* xb, uint32_t g) {
    uint32_t c;
    unsigned char* b = rk_blk(a, xb, g, &c);
    return reinterpret_cast<unsigned long long*>(b + (size_t)a.Cl * sizeof(TrXRec)) + (size_t)c * a.ns;
}
__device__ __forceinline__ uint32_t* rk_gtab(const TradeArgs& a, unsigned char* xb, uint32_t g) {
    uint32_t c;
    unsigned char* b = rk_blk(a, xb, g, &c);
    return reinterpret_cast<uint32_t*>(b + (size_t)a.Cl * sizeof(TrXRec) + (a.snaps ? (size_t)a.Cl * a.ns * 8u : 0u)) +
           (size_t)c * 64u;
}

constexpr uint32_t kStW = sizeof(TrCluster) / 4u;
constexpr uint32_t kTrW = sizeof(TrTrader) / 4u;
static_assert(sizeof(TrTrader) % 4u == 0u && kTrResMaxClusters * kTrW <= (uint32_t)kRkThreads,
              "the trader state in one word per thread");
static_assert(sizeof(TrCluster) % 4u == 0u && kStW <= (uint32_t)kWave, "TrCluster in one VGPR");
struct RkField {  // a TrCluster field held in lane f of a VGPR (phase A's cluster state)
    uint32_t& v;
    uint32_t f, lane;
    __device__ __forceinline__ operator uint32_t() const { return readlane(v, f); }
    __device__ __forceinline__ RkField& operator=(uint32_t x) {
        v = lane == f ? x : v;
        return *this;
    }
    __device__ __forceinline__ RkField& operator=(const RkField& o) { return *this = (uint32_t)o; }
    __device__ __forceinline__ RkField& operator+=(uint32_t x) { return *this = (uint32_t)*this + x; }
    __device__ __forceinline__ RkField& operator-=(uint32_t x) { return *this = (uint32_t)*this - x; }
    __device__ __forceinline__ RkField& operator|=(uint32_t x) { return *this = (uint32_t)*this | x; }
    __device__ __forceinline__ RkField& operator++() { return *this += 1u; }
    __device__ __forceinline__ RkField& operator--() { return *this -= 1u; }
    __device__ __forceinline__ uint32_t operator++(int) {
        const uint32_t o = *this;
        *this = o + 1u;
        return o;
    }
};
#define RST(field) (RkField{stv, (uint32_t)(offsetof(TrCluster, field) / 4u), lane})

#ifdef MCS_RK_STAMPS
// probe build (tools/variant.sh ... -DMCS_RK_STAMPS): per-wave segment times (s_memrealtime, 100 MHz)
// summed over the launches since the last read: [wave of the system][segment]; segments: 0 launch
// start -> state in, 1 -> B and C/D done, 2 -> acceptances applied, 3 -> phase A done, 4 -> state out
constexpr int kRkSeg = 14;
__device__ unsigned long long g_rk_stamps[kTrResMaxClusters * kRkSeg];
constexpr uint32_t kRkTl = 8192;  // timeline ring: [tick & (kRkTl - 1)][workgroup] {start, end}
__device__ unsigned long long g_rk_tl[kRkTl * 16 * 2];
#define RK_MARK(i)                                                          \
    do {                                                                    \
        const uint64_t rk_now = __builtin_amdgcn_s_memrealtime();           \
        rk_acc[i] += rk_now - rk_last;                                      \
        rk_last = rk_now;                                                   \
    } while (0)
#else
#define RK_MARK(i) \
    do {           \
    } while (0)
#endif
// the stamp build splits the launch start: kernel arguments in (0), the loads issued (1)
#ifdef MCS_RK_STAMPS
#define RK_WAIT_ARGS(v) asm volatile("s_waitcnt lgkmcnt(0)" ::"s"(v) : "memory")
#else
#define RK_WAIT_ARGS(v) \
    do {                \
    } while (0)
#endif

struct RkShared {  // (the workgroup's node vectors follow: kRkWaves * ns u64)
    // X1 of tick n, every cluster of the system (word k of cluster g at rq_job + k * 64 + g)
    uint32_t rq_job[kTrResMaxClusters], rq_c[kTrResMaxClusters], rq_m[kTrResMaxClusters];
    uint32_t rq_dur[kTrResMaxClusters], qs[kTrResMaxClusters], decided[kTrResMaxClusters];
    uint32_t nat[kTrResMaxClusters], xflags[kTrResMaxClusters];
    float cu[kTrResMaxClusters], mu[kTrResMaxClusters];
    uint32_t lq[kTrResMaxClusters], nn[kTrResMaxClusters], total_c[kTrResMaxClusters], total_m[kTrResMaxClusters];
    TrTrader trs[kTrResMaxClusters];  // replicated trader state
    TrCluster st[kRkWaves];           // this workgroup's clusters (this rank's only)
    uint32_t gtab[kRkWaves][64];
    uint32_t accm[3];  // borrowers some lender accepted (the whole system's); [2]: an append overflowed
    uint32_t T, T0, done, ticks, flags, tmax_now;
    unsigned long long n_trades, n_won, n_lent, n_lent_next;
};

template <int kRows>  // slot rows per cluster (64 slots each; a multiple of 4)
__global__ __launch_bounds__(kRkThreads) void tr_rk_kernel(TradeArgs a, uint32_t mode) {
    // mode 0: phase A of tick 0 (writes buffer 0); mode 1 / 2: tick n with n & 1 = mode - 1 (the host
    // knows the parity: a graph replays an even number of ticks, the caller-driven path counts them),
    // so every address below is known at the launch start and all of its loads issue at once
#ifdef MCS_RK_STAMPS
    uint64_t rk_acc[kRkSeg] = {};
    uint64_t rk_last = __builtin_amdgcn_s_memrealtime();
    const uint64_t rk_t0 = rk_last;
#endif
    extern __shared__ unsigned long long rk_smem[];
    RkShared& sh = *reinterpret_cast<RkShared*>(rk_smem);
    unsigned long long* const nodes_wg = rk_smem + (sizeof(RkShared) + 7) / 8;
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t C = a.Ct, ns = a.ns, S = a.S, Cl = a.Cl;
    const uint32_t wg = blockIdx.x;
    RK_WAIT_ARGS(C);
    RK_MARK(0);
    const bool helper = wave == (uint32_t)kRkWaves;  // (C/D; no cluster)
    const uint32_t g = wg * kRkWaves + (helper ? 0u : wave);  // this wave's cluster of the system
    const uint32_t lo = a.rank * Cl;          // this rank's clusters: [lo, lo + Cl)
    const bool sys = !helper && g < C;
    const bool own = sys && g >= lo && g < lo + Cl;
    // its local index (the helper: wave 0's, so its unused loads hit the lines wave 0 reads)
    const uint32_t c = g < C && g >= lo && g < lo + Cl ? g - lo : 0u;
    unsigned long long* const nodes = nodes_wg + (size_t)wave * ns;
    // tick n's blocks (read) and tick n + 1's (written); mode 0 writes tick 0's
    const size_t xbuf = (size_t)a.world * a.blk;
    const uint32_t par = mode == 2u ? 1u : 0u;  // tick n's parity (mode 0: none read)
    unsigned char* const xr = a.xb + (size_t)par * xbuf;
    unsigned char* const xw = a.xb + (size_t)(mode == 0u ? 0u : par ^ 1u) * xbuf;
    // the clock and the replicated trader state are double-buffered alike (read copy par, workgroup 0
    // writes copy par ^ 1 at its end): a workgroup that starts after workgroup 0 finished still reads
    // tick n's values.  Mode 0 changes neither.
    const TrCtl* const ctl_r = a.ctl + par;
    TrCtl* const ctl_w = a.ctl + (par ^ 1u);
    const TrTrader* const tr_r = a.tr + (size_t)par * C;
    TrTrader* const tr_w = a.tr + (size_t)(par ^ 1u) * C;

    // ---- state in: every load phases B-D need issued before any of its values is used (one round
    // trip; phase A's nodes and slot rows follow the barrier and land during B-D).  The
    // loads are unconditional, from clamped in-range addresses (a value no one uses is never read):
    // a load under a branch makes the compiler merge, and so wait for, its value at the join. ----
    // Every address first, then (past a scheduling fence) every load: a load's destination register
    // reused by an address computation after it would make the compiler wait for that load.
    const TrCtl ctlv = *ctl_r;  // (uniform: scalar loads)
    // the replicated trader state as flat words (C * kTrW <= the workgroup's threads)
    const uint32_t trn = C * kTrW, tq = threadIdx.x;
    const uint32_t* const trp0 = reinterpret_cast<const uint32_t*>(tr_r) + min(tq, trn - 1u);
    // this wave's cluster (c = 0 for a wave that owns none: its values are never read): TrCluster
    // (lane f < kStW: word f), CSR bounds, the dense node copy (tick 0's from the CSR initial state,
    // after the barrier), the running slots in registers (row r, lane l: slot (r / 4) * 256 + 4l +
    // r % 4, so a lane's four rows are one 16-byte load; finish time and payload node | cores << 9 |
    // mem << 16, in this kernel's own order in sfin / snode)
    const uint32_t* const stp = reinterpret_cast<const uint32_t*>(&a.cl[c]) + min(lane, kStW - 1u);
    const unsigned long long* np[kRkNodes / kWave];
#pragma unroll
    for (uint32_t q = 0; q < kRkNodes / kWave; ++q) np[q] = a.tnr + (size_t)c * ns + min(q * kWave + lane, ns - 1u);
    const size_t sb = (size_t)c * S;
    const uint4* const finp = reinterpret_cast<const uint4*>(a.sfin + sb) + lane;
    const uint4* const payp = reinterpret_cast<const uint4*>(a.snode + sb) + lane;
    // X1 of tick n: lane q of wave 0 takes cluster q's record from the gathered blocks
    const bool x1 = mode != 0u && wave == 0 && lane < C;
    const uint4* const rp = reinterpret_cast<const uint4*>(rk_rec(a, xr, min(lane, C - 1u)));
    const uint4* const lrpp = a.lrp + c;  // this cluster's lent run of tick n (read when it lent)
    // the G tables of this wave's lenders (w, w + 4, ...), lane x holding G_L[x]: phase B reads
    // G_L[c_b] across lanes (ds_bpermute) instead of a second round trip (L >= C: never read)
    const uint32_t* glp[kRkLenders];
#pragma unroll
    for (uint32_t k = 0; k < kRkLenders; ++k) {
        const uint32_t L = wave + k * (uint32_t)kRkWaves;
        glp[k] = rk_gtab(a, xr, L < C ? L : 0u) + lane;
    }
    __builtin_amdgcn_sched_barrier(0);
    const uint32_t trv0 = *trp0;
    const uint32_t stw = *stp;
    const uint32_t nb0 = a.node_off[c], nb1 = a.node_off[c + 1];
    const unsigned long long jb0 = a.job_off[c], jb1 = a.job_off[c + 1];
    const uint4 w0 = rp[0], w1 = rp[1], w2 = rp[2], w3 = rp[3];
    const uint4 lrv = *lrpp;
    uint32_t gl[kRkLenders];
#pragma unroll
    for (uint32_t k = 0; k < kRkLenders; ++k) gl[k] = *glp[k];
    RK_MARK(1);
    // the LDS copies
    if (own && lane < kStW) reinterpret_cast<uint32_t*>(&sh.st[wave])[lane] = stw;
    if (tq < trn) reinterpret_cast<uint32_t*>(sh.trs)[tq] = trv0;
    if (threadIdx.x == 0) {
        sh.T = sh.T0 = ctlv.T;
        sh.done = ctlv.done;
        sh.ticks = ctlv.ticks;
        sh.flags = ctlv.flags;
        sh.n_trades = ctlv.n_trades;
        sh.n_won = ctlv.n_won;
        sh.n_lent = sh.n_lent_next = ctlv.n_lent;
        sh.tmax_now = 0u;
    }
    if (x1) {
        sh.rq_job[lane] = w0.x;
        sh.rq_c[lane] = w0.y;
        sh.rq_m[lane] = w0.z;
        sh.rq_dur[lane] = w0.w;
        sh.qs[lane] = w1.x;
        sh.decided[lane] = w1.y;
        sh.nat[lane] = w1.z;
        sh.xflags[lane] = w1.w;
        sh.cu[lane] = __uint_as_float(w2.x);
        sh.mu[lane] = __uint_as_float(w2.y);
        sh.lq[lane] = w2.z;
        sh.nn[lane] = w2.w;
        sh.total_c[lane] = w3.x;
        sh.total_m[lane] = w3.y;
    }
    if (threadIdx.x < 3u) sh.accm[threadIdx.x] = 0u;
    // the barrier orders the LDS copies alone (the slot rows, nodes and TrCluster stay in flight)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    if (sh.done) {  // the graph's launches after the end of the run: the final state carried forward
        if (mode != 0u && wg == 0) {
            for (uint32_t q = threadIdx.x; q < C; q += kRkThreads) tr_w[q] = sh.trs[q];
            if (threadIdx.x == 0) *ctl_w = ctlv;
        }
        return;  // (uniform)
    }
    RK_MARK(2);
    // phase A's nodes and slot rows: issued after the barrier, they land while phases B-D run (no
    // load before A waits for them), and the launch-start batch above stays small
    unsigned long long nreg[kRkNodes / kWave];
#pragma unroll
    for (uint32_t q = 0; q < kRkNodes / kWave; ++q) nreg[q] = *np[q];
    uint32_t fin[kRows], pay[kRows];
#pragma unroll
    for (int k = 0; k < kRows / 4; ++k) {
        const uint4 f = finp[k * kWave], p = payp[k * kWave];
        fin[4 * k] = f.x;
        fin[4 * k + 1] = f.y;
        fin[4 * k + 2] = f.z;
        fin[4 * k + 3] = f.w;
        pay[4 * k] = p.x;
        pay[4 * k + 1] = p.y;
        pay[4 * k + 2] = p.z;
        pay[4 * k + 3] = p.w;
    }
    const uint32_t n0 = nb0, N = nb1 - nb0, J = (uint32_t)(jb1 - jb0);
    const uint64_t j0 = jb0;
    if (own && mode == 0u) {  // tick 0: the nodes from the CSR initial state
#pragma unroll
        for (uint32_t q = 0; q < kRkNodes / kWave; ++q)
            if (q * kWave + lane < N) nreg[q] = a.tn[n0 + q * kWave + lane];
    }
    uint32_t frm = 0u, drt = 0u;  // free rows; rows this lane changed (only those are stored back)

    const uint4* __restrict__ jobs = a.jobs + j0;
    uint4 hwin = make_uint4(0u, 0u, 0u, 0u);
    uint32_t awin = kEmpty, hwb = 0u;
    unsigned long long lqw = 0ull;
    auto prefetch_jobs = [&](uint32_t hb, uint32_t na) {
        hwb = hb;
        hwin = hb + lane < J ? jobs[hb + lane] : make_uint4(0u, 0u, 0u, 0u);
        awin = na + lane < J ? jobs[na + lane].x : kEmpty;
    };
    auto prefetch_lq = [&](uint32_t lqh, uint32_t lqn) {
        lqw = 0ull;
        if (lqn > 0u && lane < 3u)
            lqw = reinterpret_cast<const unsigned long long*>(a.lq + (size_t)c * a.LQ + lqh)[lane];
    };
    // (both windows in flight from here: the job records of the next phase A, and the LentQueue head
    // when the queue already held entries after tick n's phase A; one this launch's appends write into
    // an empty queue is taken from the request registers in phase B)
    if (own) {  // (the cluster state as loaded: lane f of stw holds word f)
#define RK_STW(field) readlane(stw, (uint32_t)(offsetof(TrCluster, field) / 4u))
        prefetch_jobs(RK_STW(has_w) ? RK_STW(w) : RK_STW(rq_head), RK_STW(next_arr));
        prefetch_lq(RK_STW(lq_head), RK_STW(lq_len));
#undef RK_STW
    }

    if (mode != 0u) {
        const uint32_t T = sh.T0;
        // ---- the lent-run records of tick n (this rank's lenders), at indices in cluster order from
        // the gathered lent bits: this rank's log counts its own runs (ctl->n_lent is per rank) ----
        {
            const unsigned long long rmask = (Cl >= 64u ? ~0ull : ((1ull << Cl) - 1ull)) << lo;
            const uint32_t qsl = lane < C ? sh.qs[lane] : 0u;
            const unsigned long long lm = __ballot(qsl & kQsLent) & rmask;
            const bool lent_g = own && ((lm >> g) & 1ull);  // (g < 64)
            if (lent_g && lane == 0) {
                const unsigned long long idx = ctlv.n_lent + (uint64_t)__builtin_popcountll(lm & ((1ull << g) - 1ull));
                if (idx < a.lent_cap) {
                    const uint4 lr = lrv;
                    mcs_lent_rec rec;
                    rec.lender = g;
                    rec.borrower = lr.x;
                    rec.job = lr.y;
                    rec.node = lr.z;
                    rec.start_s = T;
                    rec.finish_s = lr.w;
                    rec.pad = 0u;
                    a.lent_log[idx] = rec;
                }
            }
            if (threadIdx.x == 0) sh.n_lent_next = ctlv.n_lent + (uint64_t)__builtin_popcountll(lm);
        }
        RK_MARK(11);
        // ---- C and D: the helper wave of every workgroup, one lane per cluster, on X1 alone (as the MW tick:
        // every borrow request leaves its borrower busy, so the clock and the end of the run follow
        // from X1; the acceptances are applied after the X2 exchange, before phase A) ----
        if (helper) {
            const uint32_t q = lane;
            float cu = 0.0f, mu = 0.0f;
            uint32_t tot_c = 0u, tot_m = 0u, busy = 0u, next_arr_t = kEmpty, done_g = 1u, fl = 0u;
            TrTrader t{0u, 0u, 0u, kEmpty, 0u};
            if (q < C) {
                const uint32_t qs = sh.qs[q];
                cu = sh.cu[q];
                mu = sh.mu[q];
                tot_c = sh.total_c[q];
                tot_m = sh.total_m[q];
                busy = (qs & (kQsW | kQsRq | kQsLq)) ? 1u : 0u;
                next_arr_t = sh.nat[q];
                done_g = (qs & kQsDone) ? 1u : 0u;
                fl = sh.xflags[q];
                t = sh.trs[q];
            }
            unsigned long long n_trades = sh.n_trades, n_won = sh.n_won;
            uint32_t lflags = 0;
            if (a.trader) {
                const bool due = q < C && t.next_due <= T;
                const bool broken = cu > 0.8f || mu > 0.8f;  // Utilization (trader.go:127-130)
                if (due && !broken) t.next_due = T + a.period;
                const bool appr = q < C && approve_trade_dev(tot_c, tot_m, cu, mu, 0u, 0u, 0u);
                unsigned long long pend = __ballot(due && broken);
                while (pend) {  // RequestPolicyMonitor of requester r (trader.go:282-324), index order
                    const uint32_t r = (uint32_t)__builtin_ctzll(pend);
                    pend &= pend - 1ull;
                    bool app = false;
                    if (q < C && q != r) {  // RequestResource, index order
                        if (t.lock_id != 0u && T >= t.lock_until) t.lock_id = 0u;  // 20 s expiry
                        if (t.lock_id == 0u) {  // else Approve:false (server.go:35-40)
                            app = appr;
                            t.lock_id = t.next_id++;  // set even when not approving (:44-46)
                            t.lock_until = T + a.lock_s;
                        }
                    }
                    const unsigned long long ab = __ballot(app);
                    const uint32_t napp = (uint32_t)__builtin_popcountll(ab);
                    const uint32_t winner = ab ? (uint32_t)__builtin_ctzll(ab) : kEmpty;
                    if (winner != kEmpty) {
                        if (q == winner) t.lock_id = 0u;  // ApproveContract unlocks (:83)
                        if (q == r) t.vnodes += 1u;       // AddVirtualNode(0 cores, 0 memory)
                        ++n_won;
                    }
                    if (q == r) t.next_due = T + (winner != kEmpty ? a.ok_sleep : a.fail_sleep) + a.period;
                    if (lane == 0 && wg == 0) {  // (workgroup 0 keeps the log; every rank alike)
                        if (n_trades < a.trade_cap) {
                            mcs_trade_rec rec;
                            rec.t_s = T;
                            rec.requester = r;
                            rec.winner = winner == kEmpty ? -1 : (int32_t)winner;
                            rec.approvals = napp;
                            a.trade_log[n_trades] = rec;
                        }
                    }
                    if (n_trades >= a.trade_cap) lflags |= MCS_FLAG_LOG_OVERFLOW;
                    ++n_trades;
                }
            }
            // the next tick: T+1 while any queue is busy, else the next arrival or trader round
            uint32_t nxt = next_arr_t;
            if (a.trader && q < C) nxt = t.next_due < nxt ? t.next_due : nxt;
            const bool done_all = !__ballot(!done_g);
            const bool busy_any = __ballot(busy != 0u) != 0ull;
            nxt = wave_min_u32(nxt);
            fl = rk_wave_or(fl);
            // (C/D reads trs[q] of its own lane only before this barrier-free store: lane q owns q)
            if (a.trader && q < C) sh.trs[q] = t;
            if (lane == 0) {
                uint32_t flags = sh.flags | fl | lflags;
                uint32_t done = 0, Tn = T;
                const uint32_t fatal = MCS_FLAG_OVERFLOW | MCS_FLAG_LENT_OVERFLOW;
                if (done_all || (flags & fatal)) {
                    done = 1u;
                } else if (T >= a.t_max || (!busy_any && nxt == kEmpty)) {
                    done = 1u;
                    flags |= MCS_FLAG_T_MAX;
                    sh.tmax_now = 1u;
                } else {
                    Tn = (busy_any || nxt <= T + 1u) ? T + 1u : nxt;
                }
                sh.T = Tn;
                sh.done = done;
                sh.ticks += 1u;
                sh.flags = flags;
                sh.n_trades = n_trades;
                sh.n_won = n_won;
            }
        }
        RK_MARK(12);
        // ---- B (replicated in every workgroup): the acceptance matrix of tick n.  Wave w takes
        // lenders w, w + 4, ...; lane b holds borrower b's request.  Lender L accepts b when
        // G_L[c_b] > m_b (free_c > c_b and free_m > m_b on some node; c_b >= 64 fits no node of a
        // lender whose free_c are all <= 64); a "big" lender is scanned from its snapshot ----
        uint32_t rqj = kEmpty, rqc = 0u, rqm = 0u, rqd = 0u;
        if (lane < C) {
            rqj = sh.rq_job[lane];
            rqc = sh.rq_c[lane];
            rqm = sh.rq_m[lane];
            rqd = sh.rq_dur[lane];
        }
        const bool want = rqj != kEmpty;
        if (!helper && __ballot(want)) {
            // G_L[c_b] for every lender of the wave (a lane permute of the tables loaded at the start)
            uint32_t gv[kRkLenders];
            const int src = (int)(rqc < 64u ? rqc : 0u);
#pragma unroll
            for (uint32_t k = 0; k < kRkLenders; ++k) gv[k] = (uint32_t)__shfl((int)gl[k], src);
            // the wave's lenders' queue state, lane k holding lender w + 4k's (read once, before the
            // loop's LDS stores)
            const uint32_t Lk = wave + lane * (uint32_t)kRkWaves;
            const uint32_t qsk = lane < kRkLenders && Lk < C ? sh.qs[Lk] : 0u;
            const uint32_t lqk = lane < kRkLenders && Lk < C ? sh.lq[Lk] : 0u;
            uint32_t accw0 = 0u, accw1 = 0u, fbw = 0u;
#pragma unroll
            for (uint32_t k = 0; k < kRkLenders; ++k) {
                const uint32_t L = wave + k * (uint32_t)kRkWaves;
                if (L >= C) break;
                const bool want_l = want && lane != L;  // self skipped (:176)
                unsigned long long okm;
                if (!(readlane(qsk, k) & kQsBig)) {
                    okm = __ballot(want_l && rqc < 64u && gv[k] > rqm);
                } else {
                    okm = 0ull;
                    const unsigned long long* sn = rk_snap(a, xr, L);
                    const uint32_t NL = sh.nn[L];
                    unsigned long long pend = __ballot(want_l);
                    while (pend) {
                        const uint32_t bi = (uint32_t)__builtin_ctzll(pend);
                        pend &= pend - 1ull;
                        const uint32_t rc = readlane(rqc, bi), rm = readlane(rqm, bi);
                        bool ok = false;
                        for (uint32_t i0 = 0; i0 < NL; i0 += kWave) {
                            const uint32_t i = i0 + lane;
                            if (i < NL) {
                                const unsigned long long v = sn[i];
                                ok = ok || ((uint32_t)v > rc && (uint32_t)(v >> 32) > rm);
                            }
                            if (__ballot(ok)) break;
                        }
                        if (__ballot(ok)) okm |= 1ull << bi;
                    }
                }
                const uint32_t nacc = (uint32_t)__builtin_popcountll(okm);
                const uint32_t lq0 = readlane(lqk, k);  // (post-A; == the owner's own count)
                const uint32_t LQ = a.LQ;
                if (lq0 + nacc > LQ) fbw = 1u;
                accw0 |= (uint32_t)okm;
                accw1 |= (uint32_t)(okm >> 32);
                if (L == g && own) {  // the lender's own wave: appends in borrower order (owner rank)
                    const uint32_t lq_head = sh.st[wave].lq_head;
                    const uint32_t rank = (uint32_t)__builtin_popcountll(okm & ((1ull << lane) - 1ull));
                    if (((okm >> lane) & 1ull) && lq0 + rank < LQ) {
                        uint32_t at = lq_head + lq0 + rank;
                        at = at >= LQ ? at - LQ : at;
                        TrLq e{};
                        e.borrower = lane;
                        e.job = rqj;
                        e.c = rqc;
                        e.m = rqm;
                        e.dur = rqd;
                        a.lq[(size_t)c * LQ + at] = e;
                    }
                    const uint32_t lq_len = lq0 + nacc > LQ ? LQ : lq0 + nacc;
                    if (lane == 0) {
                        sh.st[wave].lq_len = lq_len;
                        if (lq0 + nacc > LQ) sh.st[wave].flags |= MCS_FLAG_LENT_OVERFLOW;
                    }
                    // the next tick's LentQueue head: an entry of an earlier tick was loaded at the
                    // launch start; one this tick's appends just wrote (the queue was empty) comes from
                    // the request registers
                    if (lq0 == 0u && okm && lq_len > 0u) {
                        const uint32_t b0 = (uint32_t)__builtin_ctzll(okm);
                        const uint32_t j = readlane(rqj, b0), ec = readlane(rqc, b0), em = readlane(rqm, b0),
                                       ed = readlane(rqd, b0);
                        lqw = lane == 0 ? ((unsigned long long)j << 32 | b0)
                            : lane == 1 ? ((unsigned long long)em << 32 | ec)
                            : lane == 2 ? (unsigned long long)ed
                                        : 0ull;
                    }
                }
            }
            if (lane == 0) {
                if (accw0) atomicOr(&sh.accm[0], accw0);
                if (accw1) atomicOr(&sh.accm[1], accw1);
                if (fbw) atomicOr(&sh.accm[2], 1u);
            }
        }
        RK_MARK(13);
        __syncthreads();
        RK_MARK(3);
        // ---- the acceptances (identical in every workgroup and on every rank): BorrowedQueue append,
        // WaitQueue pop (scheduler.go:237-242) for this workgroup's own borrowers; an append overflow
        // ends the run at tick n (clock T, no T_MAX flag of that tick) ----
        if (own && lane == 0) {  // (the owner's wave: its job offset is in registers)
            const bool acc = ((g < 32u ? sh.accm[0] >> g : sh.accm[1] >> (g - 32u)) & 1u) != 0u;
            if (acc && sh.rq_job[g] != kEmpty) {
                const uint32_t rj = sh.rq_job[g];
                a.out_node[j0 + rj] = MCS_NODE_BORROWED;
                a.out_start[j0 + rj] = T;
                a.out_finish[j0 + rj] = MCS_TIME_NONE;
                TrCluster& s = sh.st[wave];
                s.has_w = 0u;
                ++s.decided;
                ++s.borrowed;
            }
        }
        if (wave == 0) {
            if (lane == 0) {
                if (sh.accm[2]) {
                    uint32_t f = sh.flags | MCS_FLAG_LENT_OVERFLOW;
                    if (sh.tmax_now) f &= ~MCS_FLAG_T_MAX;
                    sh.flags = f;
                    sh.T = T;
                    sh.done = 1u;
                }
                sh.n_lent = sh.n_lent_next;
            }
        }
        __syncthreads();
        RK_MARK(4);
    }

    // ---- A: tick n + 1 (tick 0 in mode 0) for this rank's clusters (tr_step_kernel) ----
    // (the LDS values A starts from, read in one batch)
    const uint32_t doneA = sh.done, TA = sh.T;
    const uint32_t ndue = lane < C ? sh.trs[lane].next_due : kEmpty;  // (C <= 64)
    uint32_t stv = !helper && lane < kStW ? reinterpret_cast<const uint32_t*>(&sh.st[wave])[lane] : 0u;
    // the nodes in registers (node q * 64 + l in lane l, word q; 0 past N): the releases alone go
    // through the wave's LDS copy (a scatter), first fit and the commits stay in registers
    unsigned long long nv[kRkNodes / kWave];
#pragma unroll
    for (uint32_t q = 0; q < kRkNodes / kWave; ++q) nv[q] = q * kWave + lane < N ? nreg[q] : 0ull;
    if (own && doneA == 0u) {
        // the free slot rows
#pragma unroll
        for (int r = 0; r < kRows; ++r)
            if (fin[r] == kEmpty) frm |= 1u << r;
        const uint32_t T = TA;
        const bool sample = a.trader && T % a.sample_period == 0u && __ballot(ndue <= T) != 0ull;
        // (the WaitQueue head may have left for the BorrowedQueue in X2: the window still holds
        // the ReadyQueue head or job_at loads it)
        const uint32_t na0 = RST(next_arr);
        RK_MARK(7);
        // releases due at T (cluster.go:153-157), before the tick's decisions
        if (RST(minf) <= T) {
#pragma unroll
            for (uint32_t q = 0; q < kRkNodes / kWave; ++q)
                if (q * kWave + lane < N) nodes[q * kWave + lane] = nv[q];
            uint32_t lm = kEmpty, nrel = 0;  // (nrel: the wave's releases, from the rows' ballots)
#pragma unroll
            for (int r = 0; r < kRows; ++r) {
                const uint32_t f = fin[r];
                nrel += (uint32_t)__builtin_popcountll(__ballot(f <= T));
                if (f <= T) {
                    const uint32_t p = pay[r], kn = p & 511u;
                    if (kn < N)
                        atomicAdd(&nodes[kn], (unsigned long long)((p >> 9) & 127u) |
                                                  ((unsigned long long)(p >> 16) << 32));
                    fin[r] = kEmpty;
                    frm |= 1u << r;
                    drt |= 1u << r;
                } else {
                    lm = f < lm ? f : lm;
                }
            }
            RST(nrun) -= nrel;
            RST(minf) = wave_min_u32(lm);
#pragma unroll
            for (uint32_t q = 0; q < kRkNodes / kWave; ++q)
                if (q * kWave + lane < N) nv[q] = nodes[q * kWave + lane];
        }
        RK_MARK(8);
        // arrivals up to T join the ReadyQueue (jobs are sorted by arrival)
        uint32_t nat;
        {
            const uint32_t n = (uint32_t)__builtin_popcountll(__ballot(awin <= T && na0 + lane < J));
            RST(next_arr) = na0 + n;
            if (n < (uint32_t)kWave) {
                nat = readlane(awin, n);
            } else {
                while (RST(next_arr) < J) {
                    const uint32_t i = RST(next_arr) + lane;
                    const bool ok = i < J && jobs[i].x <= T;
                    const uint32_t m = (uint32_t)__builtin_popcountll(__ballot(ok));
                    RST(next_arr) += m;
                    if (m < (uint32_t)kWave) break;
                }
                nat = RST(next_arr) < J ? jobs[RST(next_arr)].x : kEmpty;
            }
        }
        auto job_at = [&](uint32_t j) -> uint4 {
            const uint32_t d = j - hwb;
            if (d < (uint32_t)kWave)
                return make_uint4(readlane(hwin.x, d), readlane(hwin.y, d), readlane(hwin.z, d), readlane(hwin.w, d));
            return jobs[j];
        };
        // ScheduleJob (scheduler.go:127-139); zero-capacity virtual nodes follow the physical ones
        const uint32_t vn = sh.trs[g].vnodes;
        auto first_fit = [&](uint32_t jc, uint32_t jm) -> uint32_t {
            uint32_t kk = kEmpty;
#pragma unroll
            for (uint32_t q = 0; q < kRkNodes / kWave; ++q) {
                const uint32_t i = q * kWave + lane;
                const unsigned long long m = __ballot(i < N && (uint32_t)nv[q] >= jc && (uint32_t)(nv[q] >> 32) >= jm);
                if (m && kk == kEmpty) kk = q * kWave + (uint32_t)__builtin_ctzll(m);
            }
            if (kk == kEmpty && jc == 0u && jm == 0u && vn > 0u) kk = N;
            return kk;
        };
        // Node.RunJob commit (cluster.go:144-148) + running-slot insert; false on overflow
        auto commit = [&](uint32_t kn, uint32_t jc, uint32_t jm, uint32_t f) -> bool {
            const unsigned long long need = (unsigned long long)jc | ((unsigned long long)jm << 32);
            const unsigned long long any = __ballot(frm != 0u);
            if (!any) return false;
            const uint32_t sel = (uint32_t)__builtin_ctzll(any);
            const uint32_t row = (uint32_t)__builtin_ctz(readlane(frm, sel));
            {  // node kn: lane kn % 64, word kn / 64 (masks, not an index: nv stays in registers)
                const bool mine = kn < N && lane == (kn & 63u);
#pragma unroll
                for (uint32_t q = 0; q < kRkNodes / kWave; ++q)
                    nv[q] -= need & (0ull - (unsigned long long)(mine && q == (kn >> 6)));
            }
            if (lane == sel) {
                const uint32_t p = (kn < N ? kn : 511u) | (jc << 9) | (jm << 16);
#pragma unroll
                for (int r = 0; r < kRows; ++r)
                    if ((uint32_t)r == row) {
                        fin[r] = f;
                        pay[r] = p;
                    }
                frm &= ~(1u << row);
                drt |= 1u << row;
            }
            ++RST(nrun);
            RST(peak) = RST(nrun) > RST(peak) ? RST(nrun) : RST(peak);
            RST(minf) = f < RST(minf) ? f : RST(minf);
            return true;
        };
        auto place_own = [&](uint32_t j, uint32_t kn, uint4 jb) -> bool {
            const uint32_t f = T + jb.y;
            if (jb.y != 0u && !commit(kn, jb.z, jb.w, f)) return false;
            if (lane == 0) {
                a.out_node[j0 + j] = (int32_t)kn;
                a.out_start[j0 + j] = T;
                a.out_finish[j0 + j] = f;
            }
            ++RST(placed);
            ++RST(decided);
            return true;
        };

        TrRecA req{kEmpty, 0u, 0u, 0u};
        uint32_t lent_now = 0u;
        uint4 lr = make_uint4(0u, 0u, 0u, 0u);
        for (;;) {
            if (RST(has_w)) {  // WaitQueue head (scheduler.go:219-251)
                const uint4 jb = job_at(RST(w));
                const uint32_t kn = first_fit(jb.z, jb.w);
                if (kn != kEmpty) {
                    if (!place_own(RST(w), kn, jb)) {
                        RST(flags) |= MCS_FLAG_OVERFLOW;
                        break;
                    }
                    RST(has_w) = 0u;
                } else if (a.borrow) {
                    req = TrRecA{RST(w), jb.z, jb.w, jb.y};  // BorrowResources (:234)
                }
                break;  // time.Sleep(1 s), :250
            }
            if (RST(rq_head) < RST(next_arr)) {  // ReadyQueue head (:255-272), no sleep
                const uint32_t j = RST(rq_head)++;
                const uint4 jb = job_at(j);
                const uint32_t kn = first_fit(jb.z, jb.w);
                if (kn != kEmpty) {
                    if (!place_own(j, kn, jb)) {
                        RST(flags) |= MCS_FLAG_OVERFLOW;
                        break;
                    }
                } else {
                    RST(has_w) = 1u;
                    RST(w) = j;
                    ++RST(waited);
                }
                continue;
            }
            if (RST(lq_len) > 0u) {  // LentQueue head (:277-290)
                const uint64_t w0 = readlane((uint32_t)lqw, 0) | ((uint64_t)readlane((uint32_t)(lqw >> 32), 0) << 32);
                const uint32_t eb = (uint32_t)w0, ej = (uint32_t)(w0 >> 32);
                const uint32_t ec = readlane((uint32_t)lqw, 1), em = readlane((uint32_t)(lqw >> 32), 1);
                const uint32_t ed = readlane((uint32_t)lqw, 2);
                const uint32_t kn = first_fit(ec, em);
                if (kn != kEmpty) {
                    const uint32_t f = T + ed;
                    if (ed != 0u && !commit(kn, ec, em, f)) {
                        RST(flags) |= MCS_FLAG_OVERFLOW;
                        break;
                    }
                    // the lent-run record is written by the next launch, at the index the gathered
                    // lent bits give it
                    lr = make_uint4(eb, ej, kn, f);
                    lent_now = kQsLent;
                    ++RST(lent_runs);
                    RST(lq_head) = RST(lq_head) + 1u == a.LQ ? 0u : RST(lq_head) + 1u;
                    --RST(lq_len);
                }
                break;  // sleep 1 s (:289)
            }
            break;  // idle sleep (:294)
        }
        RK_MARK(9);

        // GetResourceUtilization (cluster.go:46-63) on the ticks a trader reads it: an exact integer
        // sum (the engine's eligibility check), capacities minus free
        if (sample) {
            // (the capacities' uint32 sum is total_c / total_m, tr_init_kernel's SetTotalResources)
            uint32_t fc = 0u, fm = 0u;
#pragma unroll
            for (uint32_t q = 0; q < kRkNodes / kWave; ++q) {  // (0 past N)
                fc += (uint32_t)nv[q];
                fm += (uint32_t)(nv[q] >> 32);
            }
            const float sc = (float)(int32_t)((uint32_t)RST(total_c) - rk_wave_sum(fc));
            const float sm = (float)(int32_t)((uint32_t)RST(total_m) - rk_wave_sum(fm));
            RST(cu) = __float_as_uint(__fdiv_rn(sc, (float)RST(total_c)));
            RST(mu) = __float_as_uint(__fdiv_rn(sm, (float)RST(total_m)));
        }
        // the lender's G table of the post-A nodes (phase B of the next launch, every workgroup):
        // G[x] = max free_m over the nodes with free_c > x, x < 64; "big" when some free_c > 64
        uint32_t* const tab = sh.gtab[wave];
        tab[lane] = 0u;
        bool big = false;
#pragma unroll
        for (uint32_t q = 0; q < kRkNodes / kWave; ++q) {  // (0 past N: no entry)
            const uint32_t fc = (uint32_t)nv[q];
            if (fc > 64u)
                big = true;
            else if (fc > 0u)
                atomicMax(&tab[fc - 1u], (uint32_t)(nv[q] >> 32));
        }
        const bool bigw = __ballot(big) != 0ull;
        // (no snapshot room when the engine proved no node exceeds 64 cores: cannot happen, and is
        // refused loudly, as an overflow of this tick's record, if it ever does)
        if (bigw && !a.snaps) RST(flags) |= MCS_FLAG_OVERFLOW;
        rk_gtab(a, xw, g)[63u - lane] = wave_scan_max_u32(tab[63u - lane]);  // G[63 - lane]
        RK_MARK(10);
        // the post-A record and the node snapshot: this rank's block of the next all-gather
        const uint32_t lql = RST(lq_len);
        const uint32_t qs = (RST(has_w) ? kQsW : 0u) | (RST(rq_head) < RST(next_arr) ? kQsRq : 0u) | lent_now |
                            (lql > 0u ? kQsLq : 0u) | (RST(decided) == J && lql == 0u ? kQsDone : 0u) |
                            (bigw ? kQsBig : 0u);
        uint32_t xv = 0u;
        xv = lane == kRkJob ? req.job : xv;
        xv = lane == kRkC ? req.c : xv;
        xv = lane == kRkM ? req.m : xv;
        xv = lane == kRkDur ? req.dur : xv;
        xv = lane == kRkQs ? qs : xv;
        xv = lane == kRkDecided ? (uint32_t)RST(decided) : xv;
        xv = lane == kRkNat ? nat : xv;
        xv = lane == kRkFlags ? (uint32_t)RST(flags) : xv;
        xv = lane == kRkCu ? (uint32_t)RST(cu) : xv;
        xv = lane == kRkMu ? (uint32_t)RST(mu) : xv;
        xv = lane == kRkLq ? lql : xv;
        xv = lane == kRkN ? N : xv;
        xv = lane == kRkTc ? (uint32_t)RST(total_c) : xv;
        xv = lane == kRkTm ? (uint32_t)RST(total_m) : xv;
        uint32_t* const rp = rk_rec(a, xw, g);
        if (lane < kRkWords) rp[lane] = xv;
        if (bigw && a.snaps) {  // (read only for a big lender)
            unsigned long long* const sn = rk_snap(a, xw, g);
#pragma unroll
            for (uint32_t q = 0; q < kRkNodes / kWave; ++q)
                if (q * kWave + lane < N) sn[q * kWave + lane] = nv[q];
        }
        if (lane == 0 && lent_now) a.lrp[c] = lr;
        if (lane < kStW) reinterpret_cast<uint32_t*>(&sh.st[wave])[lane] = stv;
    }

    RK_MARK(5);
    // ---- state out (the next launch takes it from HBM) ----
    if (own) {
        // the nodes this launch changed (against the values it loaded; tick 0 writes them all): the
        // stores, and the L2 write-back at the launch end, scale with the tick's changes
#pragma unroll
        for (uint32_t q = 0; q < kRkNodes / kWave; ++q) {
            const uint32_t i = q * kWave + lane;
            if (i < N && (mode == 0u || nv[q] != nreg[q])) a.tnr[(size_t)c * ns + i] = nv[q];
        }
        if (lane < kStW) reinterpret_cast<uint32_t*>(&a.cl[c])[lane] = reinterpret_cast<const uint32_t*>(&sh.st[wave])[lane];
#pragma unroll
        for (int k = 0; k < kRows / 4; ++k) {  // a quad with a changed row, back as one 16-byte store
            if ((drt >> (4 * k)) & 15u) {
                const size_t q = sb + (size_t)k * 4u * kWave + 4u * lane;
                *reinterpret_cast<uint4*>(a.sfin + q) = make_uint4(fin[4 * k], fin[4 * k + 1], fin[4 * k + 2], fin[4 * k + 3]);
                *reinterpret_cast<uint4*>(a.snode + q) = make_uint4(pay[4 * k], pay[4 * k + 1], pay[4 * k + 2], pay[4 * k + 3]);
            }
        }
    }
    if (wg == 0 && mode != 0u) {
        for (uint32_t q = threadIdx.x; q < C; q += kRkThreads) tr_w[q] = sh.trs[q];
        if (threadIdx.x == 0) {
            TrCtl* ctl = ctl_w;
            ctl->T = sh.T;
            ctl->done = sh.done == 2u ? 1u : sh.done;
            ctl->ticks = sh.ticks;
            ctl->flags = sh.flags | (sh.done == 2u ? kTrFlagMwTimeout : 0u);
            ctl->n_trades = sh.n_trades;
            ctl->n_won = sh.n_won;
            ctl->n_lent = sh.n_lent;
        }
    }
#ifdef MCS_RK_STAMPS
    __builtin_amdgcn_s_waitcnt(0);
    RK_MARK(6);
    if (lane == 0 && !helper && g < kTrResMaxClusters)
        for (int i = 0; i < kRkSeg; ++i) atomicAdd(&g_rk_stamps[g * kRkSeg + i], (unsigned long long)rk_acc[i]);
    if (threadIdx.x == 0 && wg < 16u && mode != 0u) {
        unsigned long long* tl = g_rk_tl + ((size_t)(ctlv.ticks & (kRkTl - 1u)) * 16u + wg) * 2u;
        tl[0] = rk_t0;
        tl[1] = __builtin_amdgcn_s_memrealtime();
    }
#endif
}

}  // namespace

size_t trade_rk_lds(uint32_t ns) { return (sizeof(RkShared) + 7) / 8 * 8 + (size_t)kRkWaves * ns * 8u; }

// up to 64 clusters of the system with <= 256 nodes and 256, 512 or 1024 running slots each, any
// world size (the engine also needs the packed slot payload and exact utilization sums)
bool trade_rk_shape(const TradeArgs& a) {
    return a.Ct <= kTrResMaxClusters && a.ns <= kRkNodes && a.Cl > 0u &&
           (a.S == 4u * kWave || a.S == 8u * kWave || a.S == 16u * kWave);
}

hipError_t launch_trade_rk(const TradeArgs& a, uint32_t mode, size_t lds, hipStream_t s) {
    const uint32_t nwg = (a.Ct + kRkWaves - 1u) / kRkWaves;
    const void* fn = a.S == 4u * kWave   ? (const void*)tr_rk_kernel<4>
                     : a.S == 8u * kWave ? (const void*)tr_rk_kernel<8>
                                         : (const void*)tr_rk_kernel<16>;
    hipError_t st = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (st != hipSuccess) return st;
    if (a.S == 4u * kWave)
        hipLaunchKernelGGL(tr_rk_kernel<4>, dim3(nwg), dim3(kRkThreads), lds, s, a, mode);
    else if (a.S == 8u * kWave)
        hipLaunchKernelGGL(tr_rk_kernel<8>, dim3(nwg), dim3(kRkThreads), lds, s, a, mode);
    else
        hipLaunchKernelGGL(tr_rk_kernel<16>, dim3(nwg), dim3(kRkThreads), lds, s, a, mode);
    return hipGetLastError();
}

}  // namespace mcs

#ifdef MCS_RK_STAMPS
extern "C" int mcs_debug_rk_stamps(unsigned long long* out) {
    unsigned long long z[mcs::kTrResMaxClusters * mcs::kRkSeg] = {};
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(mcs::g_rk_stamps), sizeof(z)) != hipSuccess) return -1;
    return hipMemcpyToSymbol(HIP_SYMBOL(mcs::g_rk_stamps), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
// the launch timeline ring of the stamp build: kRkTl ticks x 16 workgroups x {start, end} (100 MHz)
extern "C" int mcs_debug_rk_timeline(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(mcs::g_rk_tl), sizeof(mcs::g_rk_tl)) == hipSuccess ? 0 : -1;
}
#endif
