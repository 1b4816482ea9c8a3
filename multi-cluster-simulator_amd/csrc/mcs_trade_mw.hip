// mcs_trade_mw.hip — the lock-step trading system (mcs_trade.h) resident in a few
// workgroups that trade records through tagged granules: up to 64 clusters x 256 nodes, one
// cluster per wave, 4 clusters per workgroup (one CU each), the whole run in one launch per
// 64k ticks.
//
// The one-workgroup resident tick (mcs_trade_res.hip) holds all 64 clusters on ONE CU: four
// clusters per wave, their slot rows copied into a working set and back around every step, and
// the tick ran VALU-bound on that CU's four SIMDs (~24k VALU instructions per tick, PMC pass in
// profiles/r03_res).  Here each wave owns one cluster (its slot finish times in registers, no
// copies), so a tick's phase A runs on ceil(C / 4) CUs, and the workgroups meet twice per tick:
//   A  each wave, its cluster: releases, arrivals, the Fifo decisions of the tick
//      (scheduler.go:216-296), the borrow request (server.go:160-248), the utilization sample
//      (cluster.go:46-63); it publishes the cluster's post-A record (10 words)
//   X1 wave 0 of every workgroup gathers all records (the requests for B, the queue state and
//      samples for C/D)
//   B  each wave, its cluster as lender: Lend (strict '>', scheduler.go:194-202) against the
//      tick's requests in borrower order, LentQueue appends (server.go:80-113); the workgroup's
//      acceptances (a borrower mask) and an append-overflow bit are published (X2)
//   C+D wave 0 of EVERY workgroup, on identical inputs from X1: the trader rounds
//      (trader.go:280-325, 193-278; server.go:31-85) and the next tick — the trader state is
//      replicated, so the workgroups agree on the clock without another exchange
//   X2 at the start of the next tick, wave 0 of every workgroup gathers the acceptances and the
//      owner workgroup applies its borrowers' BorrowedQueue moves (C/D does not wait for them).
// Exchange: the data is the flag (cdna_hip_programming.md Guideline 16, R2): every word travels
// as an 8-byte granule {value, tag} stored write-through (agent-scope atomic store) with
// tag = the exchange's epoch counted from the run's first tick, across launches (2 * tick + 1 for
// X1, + 2 for X2, the tick taken modulo 2^31 - 1 so no tag is 0); the gathering
// wave re-reads its granules (agent-scope atomic loads) until every tag matches.  A workgroup
// publishes X1 of tick n + 1 only after gathering X2 of tick n, which every workgroup published
// after its own X1 sweep of tick n; and it publishes X2 of tick n + 1 only after its X1 sweep of
// tick n + 1, which needed every workgroup's X1 of tick n + 1, each published after that
// workgroup's X2 gather of tick n: so a granule is never overwritten before every workgroup has
// read it.  The engine zeroes the granules before each
// launch; every sweep is bounded (a timeout stops the run with an internal error).
// Same results bit for bit as the three-kernel tick and the one-workgroup resident tick
// (tests/test_gpu_trade.py).
#include "mcs_trade_internal.h"
#include "mcs_trader_dev.h"
#include "mcs_wave.h"

namespace mcs {
namespace {

// clusters (waves) per workgroup: 4, one wave per SIMD of the worker's CU (r04: 16 put four cluster
// waves on each SIMD, and the last-issued of them published their records last; 4 -> 5.56, 8 -> 5.78,
// 16 -> 6.59 us per C5 tick).  At most 64 / 3 workgroups (the X2 sweep's one granule per lane) and 32
// (one XCD's CUs for the L2 exchange): with 64 clusters, 16.  (MCS_MW_WAVES: A/B builds.)
#ifndef MCS_MW_WAVES
#define MCS_MW_WAVES 4
#endif
constexpr int kMwWaves = MCS_MW_WAVES;
static_assert(3 * ((int)kTrResMaxClusters / kMwWaves) <= kWave, "X2: one granule per lane");
// the control wave: X2's gather (x2_apply), the X1 sweep, phases C and D and X2's publication.  With
// MCS_MW_HELPER a fifth wave of its own, so C/D runs beside every cluster wave's phase B and the
// sweep starts at the tick's start; else cluster wave 0 after its own phase A
#ifndef MCS_MW_HELPER
#define MCS_MW_HELPER 1
#endif
constexpr uint32_t kMwCtl = MCS_MW_HELPER ? (uint32_t)kMwWaves : 0u;
constexpr int kMwThreads = (kMwWaves + (MCS_MW_HELPER ? 1 : 0)) * kWave;
constexpr uint32_t kMwNodes = 256;       // nodes per cluster
constexpr uint32_t kX1Words = 10;        // granules of a cluster's post-A record
constexpr uint32_t kSpinLimit = 1u << 20;  // sweeps per exchange before the run gives up

// a wave's uint32 sum / OR on the DPP scans: VALU steps, no chain of LDS-pipe permutes (every
// lane active)
__device__ __forceinline__ uint32_t mw_wave_sum(uint32_t v) { return readlane(wave_scan_add_u32(v), 63u); }
__device__ __forceinline__ uint32_t mw_wave_or(uint32_t v) { return readlane(wave_scan_or_u32(v), 63u); }
// HBM this kernel's own wave wrote in an earlier tick and reads back (LentQueue entries)
__device__ __forceinline__ uint64_t mld64(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
#ifdef MCS_MW_SYSLOAD
#define MW_LOAD_SCOPE __HIP_MEMORY_SCOPE_SYSTEM
#else
#define MW_LOAD_SCOPE __HIP_MEMORY_SCOPE_AGENT
#endif
__device__ __forceinline__ void put_granule(unsigned long long* g, uint32_t tag, uint32_t v) {
    __hip_atomic_store(g, ((unsigned long long)tag << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the same granule when every workgroup of the launch runs on this XCD (checked at the start of the
// launch from HW_REG_XCC_ID): a plain store keeps the line in the XCD's shared L2, where the readers'
// agent-scope loads (L1 bypassed) find it, instead of dropping it to the fabric (write-through)
// (inline asm: as an atomic store of a narrower scope, LLVM merged it with put_granule's store in
// the other branch and kept the write-through one)
__device__ __forceinline__ void put_granule_xcd(unsigned long long* g, uint32_t tag, uint32_t v) {
    const unsigned long long x = ((unsigned long long)tag << 32) | v;
    asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(g), "v"(x) : "memory");
}
__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & 0xFu;
}

#ifdef MCS_STAMPS
// the probe build's per-wave segment times (s_memrealtime, 100 MHz) summed over the launches since
// the last read: [workgroup][wave][segment], segments as MW_MARK below
constexpr int kMwSeg = 12, kMwMaxWg = 64 / kMwWaves;  // (10, 11: sweep passes of X1, X2)
__device__ unsigned long long g_mw_stamps[kMwMaxWg * kMwWaves * kMwSeg];
// absolute times (s_memrealtime) of every 64th tick of the launch (up to kMwLogTicks of them), to split the X1 wait into
// skew (the last record's publication after this wave's own) and propagation (the sweep's end after
// the last publication): [tick][workgroup][slot], slots 0-15 each wave's phase-A end (its X1
// granules stored), 16-31 each wave's arrival at the X1 barrier, 32 wave 0's first sweep pass, 33
// its last, 34 wave 0 past the X1 barrier
constexpr int kMwLogTicks = 1024, kMwLogSlots = 2 * kMwWaves + 3;
__device__ unsigned long long g_mw_tlog[kMwLogTicks * kMwMaxWg * kMwLogSlots];
#define MW_TLOG(it, slot, v)                                                                   \
    do {                                                                                       \
        if (((it) & 63u) == 0u && ((it) >> 6) < (uint32_t)kMwLogTicks && wg < (uint32_t)kMwMaxWg && lane == 0) \
            g_mw_tlog[((size_t)((it) >> 6) * kMwMaxWg + wg) * kMwLogSlots + (slot)] = (v);                   \
    } while (0)
#define MW_MARK(i)                              \
    do {                                        \
        const uint64_t mw_now = wall_clock64(); \
        mw_acc[i] += mw_now - mw_last;          \
        mw_last = mw_now;                       \
    } while (0)
#else
#define MW_MARK(i) \
    do {           \
    } while (0)
#define MW_TLOG(it, slot, v) \
    do {                     \
    } while (0)
#endif

constexpr uint32_t kStWords = sizeof(TrCluster) / 4u;
static_assert(sizeof(TrCluster) % 4u == 0u && kStWords <= (uint32_t)kWave, "TrCluster in one VGPR");
struct MwField {  // a TrCluster field held in lane f of a VGPR (phase A's cluster state)
    uint32_t& v;
    uint32_t f, lane;
    __device__ __forceinline__ operator uint32_t() const { return readlane(v, f); }
    __device__ __forceinline__ MwField& operator=(uint32_t x) {
        v = lane == f ? x : v;
        return *this;
    }
    __device__ __forceinline__ MwField& operator=(const MwField& o) { return *this = (uint32_t)o; }
    __device__ __forceinline__ MwField& operator+=(uint32_t x) { return *this = (uint32_t)*this + x; }
    __device__ __forceinline__ MwField& operator-=(uint32_t x) { return *this = (uint32_t)*this - x; }
    __device__ __forceinline__ MwField& operator|=(uint32_t x) { return *this = (uint32_t)*this | x; }
    __device__ __forceinline__ MwField& operator++() { return *this += 1u; }
    __device__ __forceinline__ MwField& operator--() { return *this -= 1u; }
    __device__ __forceinline__ uint32_t operator++(int) {
        const uint32_t o = *this;
        *this = o + 1u;
        return o;
    }
};
#define MST(field) (MwField{stv, (uint32_t)(offsetof(TrCluster, field) / 4u), lane})

struct MwShared {  // (this workgroup's node vectors follow: kMwWaves * ns u64)
    // gathered each tick (X1): every cluster's request and queue state
    uint32_t rq_job[kTrResMaxClusters], rq_c[kTrResMaxClusters], rq_m[kTrResMaxClusters];
    uint32_t rq_dur[kTrResMaxClusters];
    uint32_t qs[kTrResMaxClusters];  // has_w | rq_busy << 1 | lent run this tick << 2
    uint32_t decided[kTrResMaxClusters], next_arr_t[kTrResMaxClusters], xflags[kTrResMaxClusters];
    float cu[kTrResMaxClusters], mu[kTrResMaxClusters];
    // constants of the run, every cluster
    uint32_t total_c[kTrResMaxClusters], total_m[kTrResMaxClusters], J[kTrResMaxClusters];
    unsigned long long j0[kTrResMaxClusters];
    TrTrader trs[kTrResMaxClusters];  // replicated trader state
    // this workgroup's clusters
    TrCluster st[kMwWaves];
    uint32_t capc[kMwWaves], capm[kMwWaves];
    uint32_t gtab[kMwWaves][64];
    uint32_t accm[3];  // borrowers some lender of this workgroup accepted this tick; [2]: an append overflowed
    uint32_t T, done, ticks, flags, xcd, tmax_now;
    unsigned long long n_trades, n_won, n_lent;
    unsigned long long n_lent_next;  // C/D's lent-run count for the next tick (phase B still reads n_lent)
};
// X1 stores a record's word w at rq_job + w * 64: the ten arrays must stay consecutive, in word order
static_assert(offsetof(MwShared, rq_c) == offsetof(MwShared, rq_job) + 1 * kTrResMaxClusters * 4 &&
                  offsetof(MwShared, rq_m) == offsetof(MwShared, rq_job) + 2 * kTrResMaxClusters * 4 &&
                  offsetof(MwShared, rq_dur) == offsetof(MwShared, rq_job) + 3 * kTrResMaxClusters * 4 &&
                  offsetof(MwShared, qs) == offsetof(MwShared, rq_job) + 4 * kTrResMaxClusters * 4 &&
                  offsetof(MwShared, decided) == offsetof(MwShared, rq_job) + 5 * kTrResMaxClusters * 4 &&
                  offsetof(MwShared, next_arr_t) == offsetof(MwShared, rq_job) + 6 * kTrResMaxClusters * 4 &&
                  offsetof(MwShared, xflags) == offsetof(MwShared, rq_job) + 7 * kTrResMaxClusters * 4 &&
                  offsetof(MwShared, cu) == offsetof(MwShared, rq_job) + 8 * kTrResMaxClusters * 4 &&
                  offsetof(MwShared, mu) == offsetof(MwShared, rq_job) + 9 * kTrResMaxClusters * 4,
              "X1 record arrays out of word order");

template <int kRows>  // slot rows per cluster (64 slots each)
__global__ __launch_bounds__(kMwThreads) void tr_mw_kernel(TradeArgs a, unsigned long long* gx_uc,
                                                                 unsigned long long* gx_c, uint32_t tick_budget,
                                                                 uint32_t nwg, uint32_t stride, uint32_t tick0,
                                                                 uint32_t force_uc) {
    // the workers are blocks 0, stride, 2 * stride, ...: with stride 8 they share one XCD under the
    // dispatcher's observed round-robin placement (speed only: the check below decides the protocol)
    if (blockIdx.x % stride != 0u) return;
    extern __shared__ unsigned long long mw_smem[];
    MwShared& sh = *reinterpret_cast<MwShared*>(mw_smem);
    unsigned long long* const nodes_wg = mw_smem + (sizeof(MwShared) + 7) / 8;
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t C = a.Ct, ns = a.ns, S = a.S;
    const uint32_t wg = blockIdx.x / stride;
    const uint32_t c = wg * kMwWaves + wave;  // this wave's cluster
    const bool own = wave < (uint32_t)kMwWaves && c < C;

    // ---- the exchange protocol of this launch: every workgroup publishes its XCD id (write-through
    // granule in uncached memory, valid under any placement); when all are equal the tick's granules
    // use the cached buffer and plain stores (put_granule_xcd), else uncached memory and write-through
    if (threadIdx.x < 64u) {
        unsigned long long* const gid = gx_uc + trade_mw_xcc_off();
        if (threadIdx.x == 0) put_granule(gid + wg, 1u, xcc_id());
        uint32_t v = 0u;
        bool ok = false;
        for (uint32_t spins = 0; spins <= kSpinLimit; ++spins) {
            const unsigned long long x = lane < nwg ? __hip_atomic_load(gid + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : (1ull << 32);
            v = (uint32_t)x;
            if (__all((uint32_t)(x >> 32) == 1u)) {
                ok = true;
                break;
            }
        }
        const uint32_t v0 = readlane(v, 0);
        // (force_uc, MCS_MW_FORCE_UC=1: the write-through exchange whatever the placement, so the
        // tests pin loop_form 4 even when every worker landed on one XCD)
        const bool same = ok && force_uc == 0u && __all(lane >= nwg || v == v0);
        if (threadIdx.x == 0) sh.xcd = same ? 1u : 0u;
    }
    __syncthreads();
    const bool xcd = sh.xcd != 0u;
    unsigned long long* const gx = xcd ? gx_c : gx_uc;
    auto put = [&](unsigned long long* g, uint32_t tag, uint32_t v) {
        if (xcd) put_granule_xcd(g, tag, v);
        else put_granule(g, tag, v);
    };
    // X1, two buffers by tick parity: [kX1Words][64] each, word w of cluster g at w * 64 + g (r04).
    // (A tick without a borrow request has no X2, so a workgroup may publish tick n + 1's X1 while
    // another still sweeps tick n's: it writes the other buffer.  It can write this one again only
    // at tick n + 2, after its own sweep of tick n + 1, i.e. after every workgroup published tick
    // n + 1's record, which each did after its sweep of tick n.)
    unsigned long long* const gx1b[2] = {gx, gx + trade_mw_x1b_off()};
    unsigned long long* const gx2 = gx + (size_t)kTrResMaxClusters * kX1Words;  // [C] lender words, [nwg][2]

    // ---- state in ----
    unsigned long long* const nodes = nodes_wg + (size_t)(wave < (uint32_t)kMwWaves ? wave : 0u) * ns;
    uint32_t N = 0, n0 = 0, J = 0;
    uint64_t j0 = 0;
    if (own) {
        n0 = a.node_off[c];
        N = a.node_off[c + 1] - n0;
        j0 = a.job_off[c];
        J = (uint32_t)(a.job_off[c + 1] - j0);
        for (uint32_t i = lane; i < N; i += kWave) nodes[i] = a.tn[n0 + i];
        if (lane < kStWords) reinterpret_cast<uint32_t*>(&sh.st[wave])[lane] = reinterpret_cast<const uint32_t*>(&a.cl[c])[lane];
        uint32_t uc = 0u, um = 0u;
        for (uint32_t i = lane; i < N; i += kWave) {
            const uint2 cp = a.cap[n0 + i];
            uc += cp.x;
            um += cp.y;
        }
        uc = mw_wave_sum(uc);
        um = mw_wave_sum(um);
        if (lane == 0) {
            sh.capc[wave] = uc;
            sh.capm[wave] = um;
        }
    }
    for (uint32_t g = threadIdx.x; g < C; g += kMwThreads) {
        sh.trs[g] = a.tr[g];
        sh.total_c[g] = a.cl[g].total_c;
        sh.total_m[g] = a.cl[g].total_m;
        sh.j0[g] = a.job_off[g];
        sh.J[g] = (uint32_t)(a.job_off[g + 1] - a.job_off[g]);
    }
    if (threadIdx.x == 0) {
        const TrCtl ctl = *a.ctl;
        sh.T = ctl.T;
        sh.done = ctl.done;
        sh.ticks = ctl.ticks;
        sh.flags = ctl.flags;
        sh.n_trades = ctl.n_trades;
        sh.n_won = ctl.n_won;
        sh.n_lent = ctl.n_lent;
    }
    // the wave's running slots in registers (row r, lane l = slot r * 64 + l): finish time, and the
    // payload packed as node | cores << 9 | mem << 16 (the engine picks this form only when every
    // node capacity is below 128 cores and 65536 memory; node >= N: a virtual node, nothing to
    // release); across launches the payload is kept in snode
    uint32_t fin[kRows], pay[kRows];
    uint32_t frm = 0u;  // free rows of this lane
    const size_t sb = (size_t)c * S;
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
        fin[r] = own ? a.sfin[sb + r * kWave + lane] : kEmpty;
        pay[r] = own ? a.snode[sb + r * kWave + lane] : 0u;
        if (fin[r] == kEmpty) frm |= 1u << r;
    }
    __syncthreads();
    const uint4* __restrict__ jobs = a.jobs + j0;
    // the next tick's records, loaded during the previous tick's exchanges: 64 records from the
    // window base hwb (the WaitQueue head, else the ReadyQueue head), 64 arrival times from the
    // first unqueued job, the LentQueue head entry
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
        if (lqn > 0u && lane < 3u) lqw = mld64(reinterpret_cast<const unsigned long long*>(a.lq + (size_t)c * a.LQ + lqh) + lane);
    };
    if (own) {
        const TrCluster& s0 = sh.st[wave];
        prefetch_jobs(s0.has_w ? s0.w : s0.rq_head, s0.next_arr);
        prefetch_lq(s0.lq_head, s0.lq_len);
    }
    uint32_t lent_tick = 0u;  // lent runs of the whole system this tick
    uint32_t lent_now = 0u, lr_b = 0u, lr_j = 0u, lr_n = 0u, lr_f = 0u;  // this tick's lent run (bit 2 of qs)
    bool timed_out = false;
#ifdef MCS_STAMPS
    uint64_t mw_acc[kMwSeg];
#pragma unroll
    for (int i = 0; i < kMwSeg; ++i) mw_acc[i] = 0u;
    uint64_t mw_last = wall_clock64();
#endif

    // X2 of tick n at the start of tick n + 1 (and after the last tick of the launch): wave 0 gathers
    // every workgroup's borrower masks; the owner workgroup moves its accepted borrowers' WaitQueue
    // heads to the BorrowedQueue (scheduler.go:237-242) with tick n's clock Tn; an append overflow
    // ends the run at tick n, as the three-kernel tick does (clock Tn, no T_MAX flag of that tick)
    auto x2_apply = [&](uint32_t tg, uint32_t Tn) {
        if (wave == kMwCtl) {
            const uint32_t nw = 3u * nwg;
            unsigned long long x = 0ull;
            bool got = false;
            for (uint32_t spins = 0; spins <= kSpinLimit; ++spins) {
                x = lane < nw ? __hip_atomic_load(gx2 + lane, __ATOMIC_RELAXED, MW_LOAD_SCOPE) : ((unsigned long long)tg << 32);
#ifdef MCS_STAMPS
                mw_acc[11] += 1u;
#endif
                if (__all((uint32_t)(x >> 32) == tg)) {
                    got = true;
                    break;
                }
            }
            if (!got) {
                timed_out = true;
                if (lane == 0) sh.done = 2u;
            } else {
                const uint32_t v = (uint32_t)x, k = lane % 3u;
                uint32_t m0 = lane < nw && k == 0u ? v : 0u, m1 = lane < nw && k == 1u ? v : 0u,
                         fb = lane < nw && k == 2u ? v : 0u;
                m0 = mw_wave_or(m0);
                m1 = mw_wave_or(m1);
                fb = mw_wave_or(fb);
                const uint32_t g = lane;
                const bool acc = ((g < 32u ? m0 >> g : m1 >> (g - 32u)) & 1u) != 0u;
                if (acc && g < C && g / kMwWaves == wg && sh.rq_job[g] != kEmpty) {
                    const uint32_t rj = sh.rq_job[g];
                    const uint64_t gj0 = sh.j0[g];
                    a.out_node[gj0 + rj] = MCS_NODE_BORROWED;
                    a.out_start[gj0 + rj] = Tn;
                    a.out_finish[gj0 + rj] = MCS_TIME_NONE;
                    TrCluster& s = sh.st[g - wg * kMwWaves];
                    s.has_w = 0u;
                    ++s.decided;
                    ++s.borrowed;
                }
                if (fb && lane == 0) {
                    uint32_t f = sh.flags | MCS_FLAG_LENT_OVERFLOW;
                    if (sh.tmax_now) f &= ~MCS_FLAG_T_MAX;
                    sh.flags = f;
                    sh.T = Tn;
                    sh.done = 1u;
                }
            }
        }
        __syncthreads();
    };
    bool pend = false;  // a tick's X2 not applied yet
    uint32_t pend_tag = 0u, pend_T = 0u;

    for (uint32_t it = 0; it < tick_budget; ++it) {
        if (pend) {
            x2_apply(pend_tag, pend_T);
            pend = false;
        }
        if (sh.done) break;
        MW_MARK(9);
        const uint32_t T = sh.T;
        // epochs count from the run's first tick, across launches: a granule line another launch
        // left in an XCD's L2 never carries a current tag.  Taken modulo 2^31 - 1, so tag1 is odd in
        // [1, 2^32 - 3] and tag2 = tag1 + 1 never wraps to 0 (the zeroed granules' tag)
        const uint32_t ep = (tick0 + it) % 0x7FFFFFFFu;
        const uint32_t tag1 = 2u * ep + 1u, tag2 = tag1 + 1u;
        unsigned long long* const gx1 = gx1b[(tick0 + it) & 1u];

        // GetResourceUtilization runs on the ticks a trader reads it (see tr_step_kernel)
        bool sample = false;
        if (a.trader && T % a.sample_period == 0u) {
            bool due = false;
            for (uint32_t q = lane; q < C; q += kWave) due = due || sh.trs[q].next_due <= T;
            sample = __ballot(due) != 0ull;
        }

        // ---- phase A: this wave's cluster (tr_step_kernel) ----
        if (own) {
            uint32_t stv = lane < kStWords ? reinterpret_cast<const uint32_t*>(&sh.st[wave])[lane] : 0u;
            // the tick's job records, every load in flight at once: 64 records from the WaitQueue
            // head (else the ReadyQueue head), 64 arrival times from the first unqueued job, and
            // the LentQueue head entry
            const uint32_t na0 = MST(next_arr);
            MW_MARK(0);

            // releases due at T (cluster.go:153-157), before the tick's decisions
            if (MST(minf) <= T) {
                uint32_t lm = kEmpty, nrel = 0;
#pragma unroll
                for (int r = 0; r < kRows; ++r) {
                    const uint32_t f = fin[r];
                    nrel += (uint32_t)__builtin_popcountll(__ballot(f <= T));  // (the wave's releases)
                    if (f <= T) {
                        const uint32_t p = pay[r], kn = p & 511u;
                        if (kn < N)
                            atomicAdd(&nodes[kn], (unsigned long long)((p >> 9) & 127u) |
                                                      ((unsigned long long)(p >> 16) << 32));
                        fin[r] = kEmpty;
                        frm |= 1u << r;
                    } else {
                        lm = f < lm ? f : lm;
                    }
                }
                MST(nrun) -= nrel;
                MST(minf) = wave_min_u32(lm);
            }
            MW_MARK(1);
            // arrivals up to T join the ReadyQueue (jobs are sorted by arrival)
            uint32_t nat;  // the arrival second of the first job not yet queued (kEmpty: none)
            {
                const uint32_t n = (uint32_t)__builtin_popcountll(__ballot(awin <= T && na0 + lane < J));
                MST(next_arr) = na0 + n;
                if (n < (uint32_t)kWave) {
                    nat = readlane(awin, n);
                } else {
                    while (MST(next_arr) < J) {
                        const uint32_t i = MST(next_arr) + lane;
                        const bool ok = i < J && jobs[i].x <= T;
                        const uint32_t m = (uint32_t)__builtin_popcountll(__ballot(ok));
                        MST(next_arr) += m;
                        if (m < (uint32_t)kWave) break;
                    }
                    nat = MST(next_arr) < J ? jobs[MST(next_arr)].x : kEmpty;
                }
            }
            MW_MARK(2);
            auto job_at = [&](uint32_t j) -> uint4 {
                const uint32_t d = j - hwb;
                if (d < (uint32_t)kWave)
                    return make_uint4(readlane(hwin.x, d), readlane(hwin.y, d), readlane(hwin.z, d), readlane(hwin.w, d));
                return jobs[j];
            };
            // ScheduleJob (scheduler.go:127-139): lowest node with both >=; zero-capacity virtual
            // nodes (AddVirtualNode, cluster.go:79) follow the physical ones
            const uint32_t vn = sh.trs[c].vnodes;
            auto first_fit = [&](uint32_t jc, uint32_t jm) -> uint32_t {
                unsigned long long v[kMwNodes / kWave];
#pragma unroll
                for (uint32_t q = 0; q < kMwNodes / kWave; ++q) {
                    const uint32_t i = q * kWave + lane;
                    v[q] = i < N ? nodes[i] : 0ull;
                }
                uint32_t kk = kEmpty;
#pragma unroll
                for (uint32_t q = 0; q < kMwNodes / kWave; ++q) {
                    const uint32_t i = q * kWave + lane;
                    const unsigned long long m =
                        __ballot(i < N && (uint32_t)v[q] >= jc && (uint32_t)(v[q] >> 32) >= jm);
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
                if (lane == sel) {
                    if (kn < N) atomicSub(&nodes[kn], need);
                    const uint32_t p = (kn < N ? kn : 511u) | (jc << 9) | (jm << 16);
#pragma unroll
                    for (int r = 0; r < kRows; ++r)
                        if ((uint32_t)r == row) {
                            fin[r] = f;
                            pay[r] = p;
                        }
                    frm &= ~(1u << row);
                }
                ++MST(nrun);
                MST(peak) = MST(nrun) > MST(peak) ? MST(nrun) : MST(peak);
                MST(minf) = f < MST(minf) ? f : MST(minf);
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
                ++MST(placed);
                ++MST(decided);
                return true;
            };

            TrRecA req{kEmpty, 0u, 0u, 0u};
            lent_now = 0u;
            for (;;) {
                if (MST(has_w)) {  // WaitQueue head (scheduler.go:219-251)
                    const uint4 jb = job_at(MST(w));
                    const uint32_t kn = first_fit(jb.z, jb.w);
                    if (kn != kEmpty) {
                        if (!place_own(MST(w), kn, jb)) {
                            MST(flags) |= MCS_FLAG_OVERFLOW;
                            break;
                        }
                        MST(has_w) = 0u;
                    } else if (a.borrow) {
                        req = TrRecA{MST(w), jb.z, jb.w, jb.y};  // BorrowResources (:234)
                    }
                    break;  // time.Sleep(1 s), :250
                }
                if (MST(rq_head) < MST(next_arr)) {  // ReadyQueue head (:255-272), no sleep
                    const uint32_t j = MST(rq_head)++;
                    const uint4 jb = job_at(j);
                    const uint32_t kn = first_fit(jb.z, jb.w);
                    if (kn != kEmpty) {
                        if (!place_own(j, kn, jb)) {
                            MST(flags) |= MCS_FLAG_OVERFLOW;
                            break;
                        }
                    } else {
                        MST(has_w) = 1u;
                        MST(w) = j;
                        ++MST(waited);
                    }
                    continue;
                }
                if (MST(lq_len) > 0u) {  // LentQueue head (:277-290), appended by this wave in phase B
                    const uint64_t w0 = readlane((uint32_t)lqw, 0) | ((uint64_t)readlane((uint32_t)(lqw >> 32), 0) << 32);
                    const uint32_t eb = (uint32_t)w0, ej = (uint32_t)(w0 >> 32);
                    const uint32_t ec = readlane((uint32_t)lqw, 1), em = readlane((uint32_t)(lqw >> 32), 1);
                    const uint32_t ed = readlane((uint32_t)lqw, 2);
                    const uint32_t kn = first_fit(ec, em);
                    if (kn != kEmpty) {
                        const uint32_t f = T + ed;
                        if (ed != 0u && !commit(kn, ec, em, f)) {
                            MST(flags) |= MCS_FLAG_OVERFLOW;
                            break;
                        }
                        // the lent-run record is written after X1, at the index every workgroup
                        // derives from the tick's lent bits (no global counter on this path)
                        lr_b = eb;
                        lr_j = ej;
                        lr_n = kn;
                        lr_f = f;
                        lent_now = 4u;
                        ++MST(lent_runs);
                        MST(lq_head) = MST(lq_head) + 1u == a.LQ ? 0u : MST(lq_head) + 1u;
                        --MST(lq_len);
                    }
                    break;  // sleep 1 s (:289)
                }
                break;  // idle sleep (:294)
            }
            MW_MARK(3);

            // GetResourceUtilization (cluster.go:46-63) on the ticks a trader reads it: an exact
            // integer sum (the engine's eligibility check), capacities minus free
            if (sample) {
                uint32_t fc = 0u, fm = 0u;
                for (uint32_t i = lane; i < N; i += kWave) {
                    const unsigned long long v = nodes[i];
                    fc += (uint32_t)v;
                    fm += (uint32_t)(v >> 32);
                }
                const float sc = (float)(int32_t)(sh.capc[wave] - mw_wave_sum(fc));
                const float sm = (float)(int32_t)(sh.capm[wave] - mw_wave_sum(fm));
                MST(cu) = __float_as_uint(__fdiv_rn(sc, (float)MST(total_c)));
                MST(mu) = __float_as_uint(__fdiv_rn(sm, (float)MST(total_m)));
            }
            // the post-A record, one granule per lane
            uint32_t xv = 0u;
            xv = lane == 0 ? req.job : xv;
            xv = lane == 1 ? req.c : xv;
            xv = lane == 2 ? req.m : xv;
            xv = lane == 3 ? req.dur : xv;
            const uint32_t qs = (MST(has_w) ? 1u : 0u) | (MST(rq_head) < MST(next_arr) ? 2u : 0u) | lent_now |
                                (MST(lq_len) > 0u ? 8u : 0u);
            xv = lane == 4 ? qs : xv;
            xv = lane == 5 ? (uint32_t)MST(decided) : xv;
            xv = lane == 6 ? nat : xv;
            xv = lane == 7 ? (uint32_t)MST(flags) : xv;
            xv = lane == 8 ? (uint32_t)MST(cu) : xv;
            xv = lane == 9 ? (uint32_t)MST(mu) : xv;
            if (lane < kX1Words) put(gx1 + (size_t)lane * kTrResMaxClusters + c, tag1, xv);
            MW_TLOG(it, wave, wall_clock64());
            if (lane < kStWords) reinterpret_cast<uint32_t*>(&sh.st[wave])[lane] = stv;
            // the next tick's records (only phase A moves these cursors; a WaitQueue head that C/D
            // moves to the BorrowedQueue leaves the ReadyQueue head inside the same window, or
            // job_at loads it directly)
            prefetch_jobs(MST(has_w) ? MST(w) : MST(rq_head), MST(next_arr));
        }
        MW_MARK(4);

        // ---- X1: every cluster's record (one wave sweeps, the others wait at the barrier) ----
        if (wave == kMwCtl) {
            // word-major granules: lane g sweeps cluster g's ten words (granule k * 64 + g), and stores
            // word k of it at rq_job + k * 64 + g: consecutive LDS words, no division, no bank
            // conflict (record-major, lane i held word i % 10 of cluster i / 10: up to ten lanes of
            // one store on one bank)
            static_assert(kTrResMaxClusters == (uint32_t)kWave, "one lane per cluster in the X1 sweep");
            constexpr int kPer = (int)kX1Words;  // granules per lane
            uint32_t xv[kPer];
            unsigned long long xg[kPer];
            for (uint32_t spins = 0;; ++spins) {
                bool ok = true;
#pragma unroll
                for (int k = 0; k < kPer; ++k)  // (every load issued before the first compare; the
                    // granule block is allocated for 64 clusters, so no index is clamped)
                    xg[k] = __hip_atomic_load(gx1 + lane + (uint32_t)k * kWave, __ATOMIC_RELAXED, MW_LOAD_SCOPE);
#pragma unroll
                for (int k = 0; k < kPer; ++k) {
                    ok = ok && (lane >= C || (uint32_t)(xg[k] >> 32) == tag1);
                    xv[k] = (uint32_t)xg[k];
                }
#ifdef MCS_STAMPS
                mw_acc[10] += 1u;
                if (spins == 0u) MW_TLOG(it, 2 * kMwWaves, wall_clock64());
#endif
                if (__all(ok)) break;
                if (spins > kSpinLimit) {
                    timed_out = true;
                    break;
                }
            }
            MW_TLOG(it, 2 * kMwWaves + 1, wall_clock64());
            // the record's ten words land in ten consecutive [64]-arrays of MwShared (rq_job .. mu)
            // (r04: a switch on the word index here ran as a divergent chain, ~8 us of the tick)
            if (lane < C) {
#pragma unroll
                for (int k = 0; k < kPer; ++k)
                    reinterpret_cast<uint32_t*>(sh.rq_job)[(uint32_t)k * kTrResMaxClusters + lane] = xv[k];
            }
            if (lane < 3) sh.accm[lane] = 0u;
            if (timed_out && lane == 0) sh.done = 2u;
        }
        if (wave < (uint32_t)kMwWaves) MW_TLOG(it, kMwWaves + wave, wall_clock64());
        __syncthreads();
        if (wave == kMwCtl) MW_TLOG(it, 2 * kMwWaves + 2, wall_clock64());
        MW_MARK(5);
        if (sh.done == 2u) break;
        // a tick without a borrow request has no acceptance and no append to overflow: its X2 is
        // neither published nor gathered (every workgroup sees the same requests in X1)
        const bool any_req = __ballot(lane < C && sh.rq_job[lane] != kEmpty) != 0ull;

        // ---- phase B: this wave's cluster as lender, requests in borrower order (tr_lend_kernel) ----
        // Lend (scheduler.go:194-202) accepts a request (c, m) when some node has free_c > c and
        // free_m > m.  With every free_c of the lender at most 64 that is G[c] > m for
        // G[x] = max free_m over the nodes with free_c > x (0 when none): the lender builds G in a
        // 64-entry LDS table, and every request of the tick is tested at once, one borrower per
        // lane (C <= 64); the accepted ones join its LentQueue in borrower order.  A lender with a
        // larger free_c scans its nodes per request instead.
        // the tick's lent-run records at indices in cluster order, from the gathered lent bits
        // (every workgroup computes the same ones; the log counter is replicated in LDS)
        {
            const bool ln = lane < C && (sh.qs[lane] & 4u);
            const unsigned long long lm = __ballot(ln);
            if (own && lent_now && lane == 0) {
                const unsigned long long idx = sh.n_lent + (uint64_t)__builtin_popcountll(lm & ((1ull << c) - 1ull));
                if (idx < a.lent_cap) {
                    mcs_lent_rec rec;
                    rec.lender = c;
                    rec.borrower = lr_b;
                    rec.job = lr_j;
                    rec.node = lr_n;
                    rec.start_s = T;
                    rec.finish_s = lr_f;
                    rec.pad = 0u;
                    a.lent_log[idx] = rec;
                }
            }
            lent_tick = (uint32_t)__builtin_popcountll(lm);
        }
        // ---- phases C and D: wave 0 of every workgroup, one lane per cluster (C <= 64), while the
        // other waves run phase B (r04: C/D needs X1 alone, and its writes are read only after the
        // phase-B barrier; the lent-run count goes to n_lent_next, since phase B indexes by n_lent) ----
        // They need nothing from phase B: every borrow request leaves its borrower busy (its WaitQueue
        // head, or the lender's LentQueue when accepted) and not done, so the next tick's clock and
        // the end of the run follow from X1 alone (queue bits: WaitQueue, ReadyQueue, LentQueue
        // after A); the acceptances (X2: the workgroup's borrower masks and append-overflow bit) are
        // published here and applied at the start of the next tick (x2_apply), while C/D runs
        if (wave == kMwCtl) {
            const uint32_t g = lane;
            float cu = 0.0f, mu = 0.0f;
            uint32_t tot_c = 0u, tot_m = 0u, busy = 0u, next_arr_t = kEmpty, done_g = 1u, fl = 0u;
            TrTrader t{0u, 0u, 0u, kEmpty, 0u};
            if (g < C && !timed_out) {
                const uint32_t qs = sh.qs[g], has_w = qs & 1u, lq = (qs >> 3) & 1u, decided = sh.decided[g];
                cu = sh.cu[g];
                mu = sh.mu[g];
                tot_c = sh.total_c[g];
                tot_m = sh.total_m[g];
                busy = (has_w || lq > 0u || (qs & 2u)) ? 1u : 0u;
                next_arr_t = sh.next_arr_t[g];
                done_g = (decided == sh.J[g] && lq == 0u) ? 1u : 0u;
                fl = sh.xflags[g];
                t = sh.trs[g];
            }
            unsigned long long n_trades = sh.n_trades, n_won = sh.n_won;
            uint32_t lflags = 0;
            if (a.trader && !timed_out) {
                const bool due = g < C && t.next_due <= T;
                const bool broken = cu > 0.8f || mu > 0.8f;  // Utilization (trader.go:127-130)
                if (due && !broken) t.next_due = T + a.period;
                // ApproveTrade of this lane as a responder: its sample is fixed for the tick
                const bool appr = g < C && approve_trade_dev(tot_c, tot_m, cu, mu, 0u, 0u, 0u);
                unsigned long long pend = __ballot(due && broken);
                while (pend) {  // RequestPolicyMonitor of requester q (trader.go:282-324)
                    const uint32_t q = (uint32_t)__builtin_ctzll(pend);
                    pend &= pend - 1ull;
                    bool app = false;
                    if (g < C && g != q) {  // RequestResource, index order
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
                        if (g == winner) t.lock_id = 0u;  // ApproveContract unlocks (:83)
                        if (g == q) t.vnodes += 1u;       // AddVirtualNode(0 cores, 0 memory)
                        ++n_won;
                    }
                    if (g == q) t.next_due = T + (winner != kEmpty ? a.ok_sleep : a.fail_sleep) + a.period;
                    if (lane == 0 && wg == 0) {  // (workgroup 0 keeps the log)
                        if (n_trades < a.trade_cap) {
                            mcs_trade_rec rec;
                            rec.t_s = T;
                            rec.requester = q;
                            rec.winner = winner == kEmpty ? -1 : (int32_t)winner;
                            rec.approvals = napp;
                            a.trade_log[n_trades] = rec;
                        }
                    }
                    if (n_trades >= a.trade_cap) lflags |= MCS_FLAG_LOG_OVERFLOW;
                    ++n_trades;
                }
                if (g < C) sh.trs[g] = t;
            }
            // the next tick: T+1 while any queue is busy, else the next arrival or trader round
            uint32_t nxt = next_arr_t;
            if (a.trader && g < C) nxt = t.next_due < nxt ? t.next_due : nxt;
            const bool done_all = !__ballot(!done_g);
            const bool busy_any = __ballot(busy != 0u) != 0ull;
            nxt = wave_min_u32(nxt);
            fl = mw_wave_or(fl);
            if (lane == 0) {
                uint32_t flags = sh.flags | fl | lflags;
                uint32_t done = 0, Tn = T;
                const uint32_t fatal = MCS_FLAG_OVERFLOW | MCS_FLAG_LENT_OVERFLOW;
                sh.tmax_now = 0u;
                if (timed_out) {
                    done = 2u;
                } else if (done_all || (flags & fatal)) {
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
                sh.n_lent_next = sh.n_lent + lent_tick;
                sh.flags = flags;
                sh.n_trades = n_trades;
                sh.n_won = n_won;
            }
        }
        if (own) {
            const uint32_t L = c;
            uint32_t rqj = kEmpty, rqc = 0u, rqm = 0u, rqd = 0u;
            if (lane < C) {
                rqj = sh.rq_job[lane];
                rqc = sh.rq_c[lane];
                rqm = sh.rq_m[lane];
                rqd = sh.rq_dur[lane];
            }
            uint32_t* const tab = sh.gtab[wave];
            uint32_t lq_len = sh.st[wave].lq_len, fb = 0;
            const uint32_t lq0 = lq_len;
            const uint32_t lq_head = sh.st[wave].lq_head;
            const uint32_t LQ = a.LQ;
            const bool want = rqj != kEmpty && lane != L;  // self skipped (:176)
            unsigned long long okm = 0ull;
            if (__ballot(want)) {
                tab[lane] = 0u;
                bool big = false;
                for (uint32_t i = lane; i < N; i += kWave) {
                    const unsigned long long v = nodes[i];
                    const uint32_t fc = (uint32_t)v;
                    if (fc > 64u)
                        big = true;
                    else if (fc > 0u)
                        atomicMax(&tab[fc - 1u], (uint32_t)(v >> 32));
                }
                if (!__ballot(big)) {
                    const uint32_t gm = wave_scan_max_u32(tab[63u - lane]);  // G[63 - lane]
                    tab[63u - lane] = gm;
                    okm = __ballot(want && rqc < 64u && tab[rqc < 64u ? rqc : 0u] > rqm);
                } else {
                    unsigned long long pend = __ballot(want);
                    while (pend) {
                        const uint32_t bi = (uint32_t)__builtin_ctzll(pend);
                        pend &= pend - 1ull;
                        const uint32_t rc = readlane(rqc, bi), rm = readlane(rqm, bi);
                        bool ok = false;
                        for (uint32_t i0 = 0; i0 < N; i0 += kWave) {
                            const uint32_t i = i0 + lane;
                            if (i < N) {
                                const unsigned long long v = nodes[i];
                                ok = ok || ((uint32_t)v > rc && (uint32_t)(v >> 32) > rm);
                            }
                            if (__ballot(ok)) break;
                        }
                        if (__ballot(ok)) okm |= 1ull << bi;
                    }
                }
            }
            // appends (server.go:80-113): the first LQ - lq_len accepted, in borrower order
            const uint32_t rank = (uint32_t)__builtin_popcountll(okm & ((1ull << lane) - 1ull));
            if (((okm >> lane) & 1ull) && lq_len + rank < LQ) {
                uint32_t at = lq_head + lq_len + rank;
                at = at >= LQ ? at - LQ : at;
                TrLq e{};
                e.borrower = lane;
                e.job = rqj;
                e.c = rqc;
                e.m = rqm;
                e.dur = rqd;
                a.lq[(size_t)L * LQ + at] = e;
            }
            const uint32_t nacc = (uint32_t)__builtin_popcountll(okm);
            if (lq_len + nacc > LQ) {
                fb |= MCS_FLAG_LENT_OVERFLOW;
                lq_len = LQ;
            } else {
                lq_len += nacc;
            }
            if (lane == 0) {
                sh.st[wave].lq_len = lq_len;
                sh.st[wave].flags |= fb;
                if (okm) {
                    atomicOr(&sh.accm[0], (uint32_t)okm);
                    atomicOr(&sh.accm[1], (uint32_t)(okm >> 32));
                }
                if (fb) atomicOr(&sh.accm[2], 1u);
            }
            // the next tick's LentQueue head: an entry of an earlier tick is loaded; one this tick's
            // appends just wrote (the queue was empty) is taken from the request registers
            if (lq0 > 0u) {
                prefetch_lq(lq_head, lq0);
            } else if (okm && lq_len > 0u) {
                const uint32_t b0 = (uint32_t)__builtin_ctzll(okm);
                const uint32_t j = readlane(rqj, b0), ec = readlane(rqc, b0), em = readlane(rqm, b0),
                               ed = readlane(rqd, b0);
                lqw = lane == 0 ? ((unsigned long long)j << 32 | b0)
                    : lane == 1 ? ((unsigned long long)em << 32 | ec)
                    : lane == 2 ? (unsigned long long)ed
                                : 0ull;
            } else {
                lqw = 0ull;
            }
        }
        MW_MARK(6);
        __syncthreads();
        MW_MARK(7);
        // X2: this workgroup's acceptances and append-overflow bit (applied at the next tick's start)
        if (wave == kMwCtl) {
            if (any_req && lane < 3) put(gx2 + 3u * wg + lane, tag2, sh.accm[lane]);
            if (lane == 0) sh.n_lent = sh.n_lent_next;
        }

        MW_MARK(8);
        if (sh.done == 2u) break;  // (C/D wrote it before the phase-B barrier)
        pend = any_req;
        pend_tag = tag2;
        pend_T = T;
    }
    if (pend && sh.done != 2u) x2_apply(pend_tag, pend_T);
#ifdef MCS_STAMPS
    if (lane == 0 && wg < (uint32_t)kMwMaxWg && wave < (uint32_t)kMwWaves)
        for (int i = 0; i < kMwSeg; ++i)
            atomicAdd(&g_mw_stamps[(wg * kMwWaves + wave) * kMwSeg + i], (unsigned long long)mw_acc[i]);
#endif

    // ---- state out (the next launch, the stats and the readers take it from HBM) ----
    if (own) {
        for (uint32_t i = lane; i < N; i += kWave) a.tn[n0 + i] = nodes[i];
        if (lane < kStWords) reinterpret_cast<uint32_t*>(&a.cl[c])[lane] = reinterpret_cast<const uint32_t*>(&sh.st[wave])[lane];
#pragma unroll
        for (int r = 0; r < kRows; ++r) {
            a.sfin[sb + r * kWave + lane] = fin[r];
            a.snode[sb + r * kWave + lane] = pay[r];
        }
    }
    if (wg == 0) {
        for (uint32_t g = threadIdx.x; g < C; g += kMwThreads) a.tr[g] = sh.trs[g];
        if (threadIdx.x == 0) {
            TrCtl* ctl = a.ctl;
            ctl->T = sh.T;
            ctl->done = sh.done == 2u ? 1u : sh.done;
            ctl->ticks = sh.ticks;
            ctl->flags = sh.flags | (sh.done == 2u ? kTrFlagMwTimeout : 0u);
            ctl->n_trades = sh.n_trades;
            ctl->n_won = sh.n_won;
            ctl->n_lent = sh.n_lent;
            ctl->info = sh.xcd;
        }
    }
}

}  // namespace

size_t trade_mw_lds(uint32_t ns) { return (sizeof(MwShared) + 7) / 8 * 8 + (size_t)kMwWaves * ns * 8u; }

// up to 64 clusters of <= 256 nodes with 256, 512 or 1024 running slots each on one engine
bool trade_mw_shape(const TradeArgs& a) {
    return a.world == 1 && a.Ct <= kTrResMaxClusters && a.ns <= kMwNodes &&
           (a.S == 4u * kWave || a.S == 8u * kWave || a.S == 16u * kWave);
}

// X1 for 64 clusters, then X2 (64 lender words + 4 x 2 mask words) padded to 128: every sweep load
// lies inside the block (a multiple of 16 bytes); then the workgroups' XCD ids (uncached buffer)
size_t trade_mw_granules(uint32_t) { return trade_mw_x1b_off() + (size_t)kTrResMaxClusters * kX1Words; }

hipError_t launch_trade_mw(const TradeArgs& a, unsigned long long* gx_uc, unsigned long long* gx_c,
                           uint32_t tick_budget, uint32_t tick0, size_t lds, bool xcd_pack, bool force_uc,
                           hipStream_t s) {
    const uint32_t nwg = (a.Ct + kMwWaves - 1) / kMwWaves;
    const uint32_t stride = xcd_pack ? 8u : 1u, nblk = stride * (nwg - 1u) + 1u;
    // the granules carry epochs counted from the run's first tick (tick0 = the ticks of the run's
    // earlier launches); zeroed before every launch as well (no tag is 0)
    hipError_t st = hipMemsetAsync(gx_uc, 0, trade_mw_granules(a.Ct) * 8u, s);
    if (st != hipSuccess) return st;
    st = hipMemsetAsync(gx_c, 0, trade_mw_granules(a.Ct) * 8u, s);
    if (st != hipSuccess) return st;
    const void* fn = a.S == 4u * kWave   ? (const void*)tr_mw_kernel<4>
                     : a.S == 8u * kWave ? (const void*)tr_mw_kernel<8>
                                         : (const void*)tr_mw_kernel<16>;
    st = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (st != hipSuccess) return st;
    if (a.S == 4u * kWave)
        hipLaunchKernelGGL(tr_mw_kernel<4>, dim3(nblk), dim3(kMwThreads), lds, s, a, gx_uc, gx_c, tick_budget,
                           nwg, stride, tick0, force_uc ? 1u : 0u);
    else if (a.S == 8u * kWave)
        hipLaunchKernelGGL(tr_mw_kernel<8>, dim3(nblk), dim3(kMwThreads), lds, s, a, gx_uc, gx_c, tick_budget,
                           nwg, stride, tick0, force_uc ? 1u : 0u);
    else
        hipLaunchKernelGGL(tr_mw_kernel<16>, dim3(nblk), dim3(kMwThreads), lds, s, a, gx_uc, gx_c, tick_budget,
                           nwg, stride, tick0, force_uc ? 1u : 0u);
    return hipGetLastError();
}

}  // namespace mcs

#ifdef MCS_STAMPS
// the probe build's per-wave segment times (kMwMaxWg workgroups x kMwWaves waves x segments, 100 MHz)
extern "C" int mcs_debug_mw_stamps(unsigned long long* out) {
    unsigned long long z[mcs::kMwMaxWg * mcs::kMwWaves * mcs::kMwSeg] = {};  // (64 waves x 12)
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(mcs::g_mw_stamps), sizeof(z)) != hipSuccess) return -1;
    return hipMemcpyToSymbol(HIP_SYMBOL(mcs::g_mw_stamps), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
// the last launch's absolute-time log ([1024 ticks][kMwMaxWg][2 kMwWaves + 3 slots], see g_mw_tlog)
extern "C" int mcs_debug_mw_tlog(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(mcs::g_mw_tlog), sizeof(mcs::g_mw_tlog)) == hipSuccess ? 0 : -1;
}
#endif
