// mcs_trade_res.hip — the lock-step trading system (mcs_trade.h) resident in ONE
// workgroup: the tick loop of a whole one-GPU system of up to 64 clusters x 256 nodes with 256,
// 512 or 1024 running slots each (C5: 64 x 256) as one launch of 16 waves on one CU, its phases
// separated by s_barrier instead of kernel boundaries.
//
// The three-kernel tick (mcs_trade.hip) spends its ~18 us re-staging every cluster's state: node
// vectors and slot finish times HBM -> LDS -> HBM in tr_step, lender snapshots in tr_lend, trader
// state in tr_trader, each a dependent memory round trip behind a kernel boundary.  Here the state
// stays on the CU across ticks:
//   * every cluster's node vector in LDS (u64 {free_c | free_m << 32}, 128 KiB for 64 x 256);
//   * each wave owns up to 4 clusters; their running-slot finish times live in that wave's VGPRs
//     (4, 8 or 16 rows of 64 lanes per cluster; the cluster being stepped is copied into a working
//     set), the slots' {node, payload} in HBM (written at a commit, read back only when the slot
//     expires, through L2), the clusters' queue state in LDS;
//   * the exchange records, acceptances, LentQueue lengths, trader locks and the clock in LDS.
// One tick (LSFIFO), each phase the body of the kernel it replaces:
//   A  every wave, its clusters in turn: releases, arrivals, the Fifo decisions of the tick
//      (scheduler.go:216-296), the borrow request (server.go:160-248), the utilization sample
//      (cluster.go:46-63), the exchange record                                   [tr_step_kernel]
//   B  every wave, its clusters as lenders: Lend (strict '>', scheduler.go:194-202) against the
//      tick's requests in borrower order, LentQueue appends (server.go:80-113)    [tr_lend_kernel]
//   C+D wave 0: the borrowers' BorrowedQueue moves, the trader rounds (trader.go:280-325,
//      193-278; server.go:31-85) and the next tick                              [tr_trader_kernel]
// The utilization sample is an integer wave sum converted once: exact against Go's float32 sum
// in node order because the engine picks this kernel only when every cluster's sum of
// max(capacity, JSON availability) per resource is below 2^24 (every partial sum is then an
// integer float32 represents exactly).  Same results bit for bit as the three-kernel tick
// (tests/test_gpu_trade.py, MCS_TRADE_RESIDENT=0 forces that path).
#include "mcs_trade_internal.h"
#include "mcs_trader_dev.h"
#include "mcs_wave.h"

namespace mcs {
namespace {

constexpr int kResWaves = 16;
constexpr int kResCpw = 4;      // clusters per wave
constexpr uint32_t kResMaxNodes = 256;

__device__ __forceinline__ uint32_t rwave_sum(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o);
    return v;
}

// HBM this kernel wrote and reads back (slot payloads, LentQueue entries): all of it is written and
// read by the one CU, whose vector L1 sees its own stores, so workgroup-scope loads (served by the
// L1 or this XCD's L2) suffice.  (Agent-scope loads would go past the XCD's L2 to keep 8 XCDs
// coherent: about 2 us each, measured as most of a release and of a lent run.)
__device__ __forceinline__ uint64_t rld64(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint32_t rld32(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// a TrCluster field held in lane f of a VGPR (phase A's per-cluster state)
constexpr uint32_t kStWords = sizeof(TrCluster) / 4u;
static_assert(sizeof(TrCluster) % 4u == 0u && kStWords <= (uint32_t)kWave, "TrCluster in one VGPR");
struct LaneField {
    uint32_t& v;
    uint32_t f, lane;
    __device__ __forceinline__ operator uint32_t() const { return readlane(v, f); }
    __device__ __forceinline__ LaneField& operator=(uint32_t x) {
        v = lane == f ? x : v;
        return *this;
    }
    __device__ __forceinline__ LaneField& operator=(const LaneField& o) { return *this = (uint32_t)o; }
    __device__ __forceinline__ LaneField& operator+=(uint32_t x) { return *this = (uint32_t)*this + x; }
    __device__ __forceinline__ LaneField& operator-=(uint32_t x) { return *this = (uint32_t)*this - x; }
    __device__ __forceinline__ LaneField& operator|=(uint32_t x) { return *this = (uint32_t)*this | x; }
    __device__ __forceinline__ LaneField& operator++() { return *this += 1u; }
    __device__ __forceinline__ LaneField& operator--() { return *this -= 1u; }
    __device__ __forceinline__ uint32_t operator++(int) {
        const uint32_t o = *this;
        *this = o + 1u;
        return o;
    }
};
#define ST(field) (LaneField{stv, (uint32_t)(offsetof(TrCluster, field) / 4u), lane})

struct ResShared {  // (the node vectors follow, Ct * ns u64)
    TrXRec x[kTrResMaxClusters];
    TrCluster st[kTrResMaxClusters];
    TrTrader trs[kTrResMaxClusters];
    TrRecC rcs[kTrResMaxClusters];
    uint32_t acc[kTrResMaxClusters], lqp[kTrResMaxClusters], fb[kTrResMaxClusters];
    uint32_t capc[kTrResMaxClusters], capm[kTrResMaxClusters];  // sums of capacities (mod 2^32)
    uint32_t gtab[kResWaves][64];  // phase B: a lender's G table, one per wave
    uint32_t T, done, ticks, flags;
    unsigned long long n_trades, n_won, n_lent;  // (n_lent: the lent log's cursor)
};

#ifdef MCS_STAMPS
// the probe build's per-wave segment times (s_memrealtime, 100 MHz) summed over the launches since
// the last read: [wave][segment], segments as RS_MARK below
constexpr int kResSeg = 10;
__device__ unsigned long long g_res_stamps[kResWaves * kResSeg];
#define RS_MARK(i)                                  \
    do {                                            \
        const uint64_t rs_now = wall_clock64();     \
        rs_acc[i] += rs_now - rs_last;              \
        rs_last = rs_now;                           \
    } while (0)
#else
#define RS_MARK(i) \
    do {           \
    } while (0)
#endif

template <int kResRows>  // slot rows per cluster (64 slots each)
__global__ __launch_bounds__(kResWaves * kWave) void tr_resident_kernel(TradeArgs a, uint32_t tick_budget) {
    extern __shared__ unsigned long long res_smem[];
    ResShared& sh = *reinterpret_cast<ResShared*>(res_smem);
    unsigned long long* const nodes_all = res_smem + (sizeof(ResShared) + 7) / 8;
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t C = a.Ct, ns = a.ns, S = a.S;

    // ---- state in: the node vectors, the clusters, the traders, the clock ----
    for (uint32_t c = 0; c < C; ++c) {
        const uint32_t n0 = a.node_off[c], N = a.node_off[c + 1] - n0;
        for (uint32_t i = threadIdx.x; i < N; i += kResWaves * kWave) nodes_all[(size_t)c * ns + i] = a.tn[n0 + i];
    }
    for (uint32_t c = threadIdx.x; c < C; c += kResWaves * kWave) {
        sh.st[c] = a.cl[c];
        sh.trs[c] = a.tr[c];
        sh.acc[c] = 0u;
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
    // this wave's clusters: slot finish times in registers (row r, lane l = slot r * 64 + l), and
    // the sums of capacities the utilization sample subtracts the free vector from
    uint32_t fin[kResCpw][kResRows];
    uint32_t frm[kResCpw];  // free rows of this lane
#pragma unroll
    for (int k = 0; k < kResCpw; ++k) {
        const uint32_t c = wave * kResCpw + k;
        frm[k] = 0u;
#pragma unroll
        for (int r = 0; r < kResRows; ++r) {
            fin[k][r] = c < C ? a.sfin[(size_t)c * S + r * kWave + lane] : kEmpty;
            if (fin[k][r] == kEmpty) frm[k] |= 1u << r;
        }
        if (c < C) {
            const uint32_t n0 = a.node_off[c], N = a.node_off[c + 1] - n0;
            uint32_t uc = 0u, um = 0u;
            for (uint32_t i = lane; i < N; i += kWave) {
                const uint2 cp = a.cap[n0 + i];
                uc += cp.x;
                um += cp.y;
            }
            uc = rwave_sum(uc);
            um = rwave_sum(um);
            if (lane == 0) {
                sh.capc[c] = uc;
                sh.capm[c] = um;
            }
        }
    }
#ifdef MCS_STAMPS
    uint64_t rs_acc[kResSeg];
#pragma unroll
    for (int i = 0; i < kResSeg; ++i) rs_acc[i] = 0u;
    uint64_t rs_last = wall_clock64();
#endif
    __syncthreads();

    for (uint32_t it = 0; it < tick_budget; ++it) {
        if (sh.done) break;
        const uint32_t T = sh.T;
        RS_MARK(9);

        // the tick's job records, all loads in flight at once: lanes 16k..16k+15 hold, for the
        // wave's cluster k, the 16 records from its WaitQueue head (else its ReadyQueue head) and
        // the arrival times of the 16 jobs from its first unqueued one (a tick's decisions and
        // arrivals stay within them but for bursts, which load the records they pass directly)
        uint4 hwin = make_uint4(0u, 0u, 0u, 0u);
        uint32_t awin = kEmpty, hbase = 0u;
        {
            const uint32_t c = wave * kResCpw + (lane >> 4), d = lane & 15u;
            if (c < C) {
                const uint64_t j0 = a.job_off[c];
                const uint32_t J = (uint32_t)(a.job_off[c + 1] - j0);
                const TrCluster& s = sh.st[c];
                const uint32_t hb = s.has_w ? s.w : s.rq_head;
                const uint32_t na = s.next_arr;
                hbase = hb;
                if (hb + d < J) hwin = a.jobs[j0 + hb + d];
                if (na + d < J) awin = a.jobs[j0 + na + d].x;
            }
        }
        // GetResourceUtilization runs on the ticks a trader reads it (see tr_step_kernel)
        bool sample = false;
        if (a.trader && T % a.sample_period == 0u) {
            bool due = false;
            for (uint32_t q = lane; q < C; q += kWave) due = due || sh.trs[q].next_due <= T;
            sample = __ballot(due) != 0ull;
        }
        RS_MARK(0);

        // ---- phase A: each wave's clusters, in turn (tr_step_kernel) ----
        // (one cluster's 16 slot rows are copied into a working set and back: the loop body is
        // not unrolled over the wave's clusters, which keeps it within 128 VGPRs)
#pragma unroll 1
        for (int k = 0; k < kResCpw; ++k) {
            const uint32_t c = wave * kResCpw + k;
            if (c >= C) break;
            uint32_t wf[kResRows];
            uint32_t wfrm = k == 0 ? frm[0] : k == 1 ? frm[1] : k == 2 ? frm[2] : frm[3];
#pragma unroll
            for (int r = 0; r < kResRows; ++r)
                wf[r] = k == 0 ? fin[0][r] : k == 1 ? fin[1][r] : k == 2 ? fin[2][r] : fin[3][r];
            const uint32_t wl = (uint32_t)k * 16u;  // the cluster's window lanes
            const uint32_t hb = readlane(hbase, wl);
            unsigned long long* const nodes = nodes_all + (size_t)c * ns;
            const uint32_t n0 = a.node_off[c], N = a.node_off[c + 1] - n0;
            const uint64_t j0 = a.job_off[c];
            const uint32_t J = (uint32_t)(a.job_off[c + 1] - j0);
            const uint4* __restrict__ jobs = a.jobs + j0;
            const size_t sb = (size_t)c * S;
            const uint32_t vn = sh.trs[c].vnodes;
            // the cluster's queue state: word f of its TrCluster in lane f of one VGPR (uniform
            // reads are v_readlane, writes a lane select; never written under a lane-divergent
            // branch)
            uint32_t stv = lane < kStWords ? reinterpret_cast<const uint32_t*>(&sh.st[c])[lane] : 0u;

            // releases due at T (cluster.go:153-157), before the tick's decisions
            if (ST(minf) <= T) {
                // the expired slots' {node, payload} loads of up to 8 rows issued together, then
                // their node updates
                constexpr int kG = kResRows < 4 ? kResRows : 4;
                uint32_t lm = kEmpty, nrel = 0;
#pragma unroll
                for (int g = 0; g < kResRows; g += kG) {
                    uint32_t nd[kG];
                    unsigned long long cm[kG];
#pragma unroll
                    for (int r = 0; r < kG; ++r) {
                        nd[r] = kEmpty;
                        cm[r] = 0ull;
                        if (wf[g + r] <= T) {
                            const uint32_t slot = (g + r) * kWave + lane;
                            nd[r] = rld32(a.snode + sb + slot);
                            cm[r] = rld64(a.scm + sb + slot);
                        }
                    }
#pragma unroll
                    for (int r = 0; r < kG; ++r) {
                        const uint32_t f = wf[g + r];
                        if (f <= T) {
                            if (nd[r] < N) atomicAdd(&nodes[nd[r]], cm[r]);
                            wf[g + r] = kEmpty;
                            wfrm |= 1u << (g + r);
                            ++nrel;
                        } else {
                            lm = f < lm ? f : lm;
                        }
                    }
                }
                ST(nrun) -= rwave_sum(nrel);
                ST(minf) = wave_min_u32(lm);
            }
            RS_MARK(1);
            // arrivals up to T join the ReadyQueue (jobs are sorted by arrival): the arrival
            // window, then direct loads past a full window
            uint32_t nat;  // the arrival second of the first job not yet queued (kEmpty: none)
            {
                const uint32_t na = ST(next_arr);
                const uint32_t n = (uint32_t)__builtin_popcountll(
                    (__ballot(awin <= T && na + (lane & 15u) < J) >> wl) & 0xffffull);
                ST(next_arr) = na + n;
                if (n < 16u) {
                    nat = readlane(awin, wl + n);
                } else {
                    while (ST(next_arr) < J) {
                        const uint32_t i = ST(next_arr) + lane;
                        const bool ok = i < J && jobs[i].x <= T;
                        const uint32_t m = (uint32_t)__builtin_popcountll(__ballot(ok));
                        ST(next_arr) += m;
                        if (m < (uint32_t)kWave) break;
                    }
                    nat = ST(next_arr) < J ? jobs[ST(next_arr)].x : kEmpty;
                }
            }
            // record j: from the head window when it holds it
            auto job_at = [&](uint32_t j) -> uint4 {
                const uint32_t d = j - hb;
                if (d < 16u) {
                    const uint32_t l = wl + d;
                    return make_uint4(readlane(hwin.x, l), readlane(hwin.y, l), readlane(hwin.z, l), readlane(hwin.w, l));
                }
                return jobs[j];
            };
            RS_MARK(2);

            // ScheduleJob (scheduler.go:127-139): lowest node with both >=; zero-capacity virtual
            // nodes (AddVirtualNode, cluster.go:79) follow the physical ones
            // (every node read issued before the first compare: one LDS round trip for <= 256 nodes)
            auto first_fit = [&](uint32_t jc, uint32_t jm) -> uint32_t {
                unsigned long long v[kResMaxNodes / kWave];
#pragma unroll
                for (uint32_t q = 0; q < kResMaxNodes / kWave; ++q) {
                    const uint32_t i = q * kWave + lane;
                    v[q] = i < N ? nodes[i] : 0ull;
                }
                uint32_t kk = kEmpty;
#pragma unroll
                for (uint32_t q = 0; q < kResMaxNodes / kWave; ++q) {
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
                const unsigned long long any = __ballot(wfrm != 0u);
                if (!any) return false;
                const uint32_t sel = (uint32_t)__builtin_ctzll(any);
                const uint32_t row = (uint32_t)__builtin_ctz(readlane(wfrm, sel));
                if (lane == sel) {
                    if (kn < N) atomicSub(&nodes[kn], need);
                    a.snode[sb + row * kWave + sel] = kn;
                    a.scm[sb + row * kWave + sel] = need;
#pragma unroll
                    for (int r = 0; r < kResRows; ++r)
                        if ((uint32_t)r == row) wf[r] = f;
                    wfrm &= ~(1u << row);
                }
                ++ST(nrun);
                ST(peak) = ST(nrun) > ST(peak) ? ST(nrun) : ST(peak);
                ST(minf) = f < ST(minf) ? f : ST(minf);
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
                ++ST(placed);
                ++ST(decided);
                return true;
            };

            TrRecA req{kEmpty, 0u, 0u, 0u};
            for (;;) {
                if (ST(has_w)) {  // WaitQueue head (scheduler.go:219-251)
                    const uint4 jb = job_at(ST(w));
                    const uint32_t kn = first_fit(jb.z, jb.w);
                    if (kn != kEmpty) {
                        if (!place_own(ST(w), kn, jb)) {
                            ST(flags) |= MCS_FLAG_OVERFLOW;
                            break;
                        }
                        ST(has_w) = 0u;
                    } else if (a.borrow) {
                        req = TrRecA{ST(w), jb.z, jb.w, jb.y};  // BorrowResources (:234)
                    }
                    break;  // time.Sleep(1 s), :250
                }
                if (ST(rq_head) < ST(next_arr)) {  // ReadyQueue head (:255-272), no sleep
                    const uint32_t j = ST(rq_head)++;
                    const uint4 jb = job_at(j);
                    const uint32_t kn = first_fit(jb.z, jb.w);
                    if (kn != kEmpty) {
                        if (!place_own(j, kn, jb)) {
                            ST(flags) |= MCS_FLAG_OVERFLOW;
                            break;
                        }
                    } else {
                        ST(has_w) = 1u;
                        ST(w) = j;
                        ++ST(waited);
                    }
                    continue;
                }
                if (ST(lq_len) > 0u) {  // LentQueue head (:277-290), written by this wave in phase B
                    const TrLq* q = a.lq + (size_t)c * a.LQ + ST(lq_head);
                    const uint64_t w0 = rld64(reinterpret_cast<const unsigned long long*>(q));
                    const uint64_t w1 = rld64(reinterpret_cast<const unsigned long long*>(q) + 1);
                    const uint64_t w2 = rld64(reinterpret_cast<const unsigned long long*>(q) + 2);
                    const uint32_t eb = (uint32_t)w0, ej = (uint32_t)(w0 >> 32);
                    const uint32_t ec = (uint32_t)w1, em = (uint32_t)(w1 >> 32), ed = (uint32_t)w2;
                    const uint32_t kn = first_fit(ec, em);
                    if (kn != kEmpty) {
                        const uint32_t f = T + ed;
                        if (ed != 0u && !commit(kn, ec, em, f)) {
                            ST(flags) |= MCS_FLAG_OVERFLOW;
                            break;
                        }
                        if (lane == 0) {
                            const unsigned long long idx = atomicAdd(&sh.n_lent, 1ull);
                            if (idx < a.lent_cap) {
                                mcs_lent_rec rec;
                                rec.lender = c;
                                rec.borrower = eb;
                                rec.job = ej;
                                rec.node = kn;
                                rec.start_s = T;
                                rec.finish_s = f;
                                rec.pad = 0u;
                                a.lent_log[idx] = rec;
                            }
                        }
                        ++ST(lent_runs);
                        ST(lq_head) = ST(lq_head) + 1u == a.LQ ? 0u : ST(lq_head) + 1u;
                        --ST(lq_len);
                    }
                    break;  // sleep 1 s (:289)
                }
                break;  // idle sleep (:294)
            }

            RS_MARK(3);
            // GetResourceUtilization (cluster.go:46-63) on the ticks a trader reads it: an exact
            // integer sum (the engine's eligibility check, above), capacities minus free
            if (sample) {
                uint32_t fc = 0u, fm = 0u;
                for (uint32_t i = lane; i < N; i += kWave) {
                    const unsigned long long v = nodes[i];
                    fc += (uint32_t)v;
                    fm += (uint32_t)(v >> 32);
                }
                // (mod 2^32: the signed sum, < 2^24 in size)
                const float sc = (float)(int32_t)(sh.capc[c] - rwave_sum(fc));
                const float sm = (float)(int32_t)(sh.capm[c] - rwave_sum(fm));
                ST(cu) = __float_as_uint(__fdiv_rn(sc, (float)ST(total_c)));
                ST(mu) = __float_as_uint(__fdiv_rn(sm, (float)ST(total_m)));
            }
            if (lane == 0) {
                TrXRec x;
                x.req = req;
                x.n = N;
                x.has_w = ST(has_w);
                x.lq_len = ST(lq_len);
                x.rq_busy = ST(rq_head) < ST(next_arr) ? 1u : 0u;
                x.decided = ST(decided);
                x.J = J;
                x.next_arr_t = nat;
                x.flags = ST(flags);
                x.cu = __uint_as_float(ST(cu));
                x.mu = __uint_as_float(ST(mu));
                x.total_c = ST(total_c);
                x.total_m = ST(total_m);
                sh.x[c] = x;
            }
#pragma unroll
            for (int r = 0; r < kResRows; ++r) {
                fin[0][r] = k == 0 ? wf[r] : fin[0][r];
                fin[1][r] = k == 1 ? wf[r] : fin[1][r];
                fin[2][r] = k == 2 ? wf[r] : fin[2][r];
                fin[3][r] = k == 3 ? wf[r] : fin[3][r];
            }
            frm[0] = k == 0 ? wfrm : frm[0];
            frm[1] = k == 1 ? wfrm : frm[1];
            frm[2] = k == 2 ? wfrm : frm[2];
            frm[3] = k == 3 ? wfrm : frm[3];
            if (lane < kStWords) reinterpret_cast<uint32_t*>(&sh.st[c])[lane] = stv;
            RS_MARK(4);
        }
        __syncthreads();
        RS_MARK(5);

        // ---- phase B: each wave's clusters as lenders, requests in borrower order (tr_lend_kernel) ----
        // Lend (scheduler.go:194-202) accepts a request (c, m) when some node has free_c > c and
        // free_m > m.  With every free_c of the lender at most 64 that is G[c] > m for
        // G[x] = max free_m over the nodes with free_c > x (0 when none): the lender builds G in a
        // 64-entry LDS table (an atomic max per node into A[free_c - 1], then a suffix maximum),
        // and every request of the tick is tested at once, one borrower per lane (C <= 64); the
        // accepted ones join its LentQueue in borrower order by their rank among them.  A lender
        // with a larger free_c scans its nodes per request instead.
        {
            TrRecA rq{kEmpty, 0u, 0u, 0u};
            if (lane < C) rq = sh.x[lane].req;
            uint32_t* const tab = sh.gtab[wave];
#pragma unroll 1
            for (int k = 0; k < kResCpw; ++k) {
                const uint32_t L = wave * kResCpw + k;
                if (L >= C) break;
                const unsigned long long* const nodes = nodes_all + (size_t)L * ns;
                const uint32_t N = sh.x[L].n;
                uint32_t lq_len = sh.x[L].lq_len, fb = 0;
                const uint32_t lq_head = sh.st[L].lq_head;
                const uint32_t LQ = a.LQ;
                const bool want = rq.job != kEmpty && lane != L;  // self skipped (:176)
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
                        const uint32_t g = wave_scan_max_u32(tab[63u - lane]);  // G[63 - lane]
                        tab[63u - lane] = g;
                        okm = __ballot(want && rq.c < 64u && tab[rq.c < 64u ? rq.c : 0u] > rq.m);
                    } else {
                        unsigned long long pend = __ballot(want);
                        while (pend) {
                            const uint32_t bi = (uint32_t)__builtin_ctzll(pend);
                            pend &= pend - 1ull;
                            const uint32_t rc = readlane(rq.c, bi), rm = readlane(rq.m, bi);
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
                    e.job = rq.job;
                    e.c = rq.c;
                    e.m = rq.m;
                    e.dur = rq.dur;
                    a.lq[(size_t)L * LQ + at] = e;
                    sh.acc[lane] = 1u;  // (every accepting lender writes the same value)
                }
                const uint32_t nacc = (uint32_t)__builtin_popcountll(okm);
                if (lq_len + nacc > LQ) {
                    fb |= MCS_FLAG_LENT_OVERFLOW;
                    lq_len = LQ;
                } else {
                    lq_len += nacc;
                }
                if (lane == 0) {
                    sh.lqp[L] = lq_len;
                    sh.fb[L] = fb;
                    sh.st[L].lq_len = lq_len;
                    sh.st[L].flags |= fb;
                }
            }
        }
        RS_MARK(6);
        __syncthreads();
        RS_MARK(7);

        // ---- phases C and D: wave 0 (tr_trader_kernel), one lane per cluster (C <= 64) ----
        // The borrower step, then the trader rounds with every trader's state in the lanes'
        // registers: a due requester that is not over the utilization threshold only moves its own
        // due time (all of them at once); the others run their RequestResource rounds in index
        // order, each a ballot over the responders' lock states, with no LDS round trip.
        if (wave == 0) {
            const uint32_t g = lane;
            float cu = 0.0f, mu = 0.0f;
            uint32_t tot_c = 0u, tot_m = 0u, busy = 0u, next_arr_t = kEmpty, done_g = 1u, fl = 0u;
            TrTrader t{0u, 0u, 0u, kEmpty, 0u};
            if (g < C) {
                const TrXRec x = sh.x[g];
                const uint32_t accg = sh.acc[g], lq = sh.lqp[g], fbg = sh.fb[g];
                uint32_t has_w = x.has_w, decided = x.decided;
                if (x.req.job != kEmpty && accg) {  // BorrowedQueue append (scheduler.go:237-242)
                    has_w = 0u;
                    ++decided;
                    const uint64_t j0 = a.job_off[g];
                    a.out_node[j0 + x.req.job] = MCS_NODE_BORROWED;
                    a.out_start[j0 + x.req.job] = T;
                    a.out_finish[j0 + x.req.job] = MCS_TIME_NONE;
                    sh.st[g].has_w = 0u;
                    ++sh.st[g].decided;
                    ++sh.st[g].borrowed;
                }
                sh.acc[g] = 0u;
                cu = x.cu;
                mu = x.mu;
                tot_c = x.total_c;
                tot_m = x.total_m;
                busy = (has_w || lq > 0u || x.rq_busy) ? 1u : 0u;
                next_arr_t = x.next_arr_t;
                done_g = (decided == x.J && lq == 0u) ? 1u : 0u;
                fl = x.flags | fbg;
                t = sh.trs[g];
            }
            unsigned long long n_trades = sh.n_trades, n_won = sh.n_won;
            uint32_t lflags = 0;
            if (a.trader) {
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
                    if (lane == 0) {
                        if (n_trades < a.trade_cap) {
                            mcs_trade_rec rec;
                            rec.t_s = T;
                            rec.requester = q;
                            rec.winner = winner == kEmpty ? -1 : (int32_t)winner;
                            rec.approvals = napp;
                            a.trade_log[n_trades] = rec;
                        } else {
                            lflags |= MCS_FLAG_LOG_OVERFLOW;
                        }
                    }
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
            for (int o = 32; o > 0; o >>= 1) fl |= (uint32_t)__shfl_xor((int)fl, o);
            lflags = (uint32_t)__shfl((int)lflags, 0);
            if (lane == 0) {
                uint32_t flags = sh.flags | fl | lflags;
                uint32_t done = 0, Tn = T;
                const uint32_t fatal = MCS_FLAG_OVERFLOW | MCS_FLAG_LENT_OVERFLOW;
                if (done_all || (flags & fatal)) {
                    done = 1u;
                } else if (T >= a.t_max || (!busy_any && nxt == kEmpty)) {
                    done = 1u;
                    flags |= MCS_FLAG_T_MAX;
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
        RS_MARK(8);
        __syncthreads();
    }
#ifdef MCS_STAMPS
    if (lane == 0)
        for (int i = 0; i < kResSeg; ++i) atomicAdd(&g_res_stamps[wave * kResSeg + i], (unsigned long long)rs_acc[i]);
#endif

    // ---- state out (the next launch, the stats and the readers take it from HBM) ----
    for (uint32_t c = 0; c < C; ++c) {
        const uint32_t n0 = a.node_off[c], N = a.node_off[c + 1] - n0;
        for (uint32_t i = threadIdx.x; i < N; i += kResWaves * kWave) a.tn[n0 + i] = nodes_all[(size_t)c * ns + i];
    }
    for (uint32_t c = threadIdx.x; c < C; c += kResWaves * kWave) {
        a.cl[c] = sh.st[c];
        a.tr[c] = sh.trs[c];
    }
#pragma unroll
    for (int k = 0; k < kResCpw; ++k) {
        const uint32_t c = wave * kResCpw + k;
        if (c < C) {
#pragma unroll
            for (int r = 0; r < kResRows; ++r) a.sfin[(size_t)c * S + r * kWave + lane] = fin[k][r];
        }
    }
    if (threadIdx.x == 0) {
        TrCtl ctl{};
        ctl.T = sh.T;
        ctl.done = sh.done;
        ctl.ticks = sh.ticks;
        ctl.flags = sh.flags;
        ctl.n_lent = sh.n_lent;
        ctl.n_trades = sh.n_trades;
        ctl.n_won = sh.n_won;
        *a.ctl = ctl;
    }
}

}  // namespace

size_t trade_resident_lds(uint32_t n_clusters, uint32_t ns) {
    return (sizeof(ResShared) + 7) / 8 * 8 + (size_t)n_clusters * ns * 8u;
}

// one workgroup holds the whole system: one engine (world 1), <= 64 clusters of <= 256 nodes,
// 1024 running slots each, and the LDS to hold them (checked against the device by the caller)
bool trade_resident_shape(const TradeArgs& a) {
    return a.world == 1 && a.Ct <= (uint32_t)(kResWaves * kResCpw) && a.Ct <= kTrResMaxClusters &&
           a.ns <= kResMaxNodes && (a.S == 4u * kWave || a.S == 8u * kWave || a.S == 16u * kWave);
}

hipError_t launch_trade_resident(const TradeArgs& a, uint32_t tick_budget, size_t lds, hipStream_t s) {
    // 256 / 512 slots per cluster: 16 / 32 VGPRs of finish times per wave; 1024: 64 (that variant
    // spills registers)
    const void* fn = a.S == 4u * kWave   ? (const void*)tr_resident_kernel<4>
                     : a.S == 8u * kWave ? (const void*)tr_resident_kernel<8>
                                         : (const void*)tr_resident_kernel<16>;
    const hipError_t st = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (st != hipSuccess) return st;
    if (a.S == 4u * kWave)
        hipLaunchKernelGGL(tr_resident_kernel<4>, dim3(1), dim3(kResWaves * kWave), lds, s, a, tick_budget);
    else if (a.S == 8u * kWave)
        hipLaunchKernelGGL(tr_resident_kernel<8>, dim3(1), dim3(kResWaves * kWave), lds, s, a, tick_budget);
    else
        hipLaunchKernelGGL(tr_resident_kernel<16>, dim3(1), dim3(kResWaves * kWave), lds, s, a, tick_budget);
    return hipGetLastError();
}

}  // namespace mcs

#ifdef MCS_STAMPS
// the probe build's per-wave segment times (16 waves x 10 segments, 100 MHz ticks); read and reset
extern "C" int mcs_debug_res_stamps(unsigned long long* out) {
    unsigned long long z[mcs::kResWaves * mcs::kResSeg] = {};
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(mcs::g_res_stamps), sizeof(z)) != hipSuccess) return -1;
    return hipMemcpyToSymbol(HIP_SYMBOL(mcs::g_res_stamps), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
