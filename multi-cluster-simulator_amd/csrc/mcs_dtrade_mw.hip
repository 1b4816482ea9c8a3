// mcs_dtrade_mw.hip — the lock-step trading system with DELAY schedulers resident
// in a few workgroups on one XCD: up to 64 clusters of <= 320 nodes (physical + virtual), one wave
// per cluster, four per workgroup, plus one trader wave; a launch runs up to `budget` ticks.
//   A+C  each cluster wave, its cluster, with its nodes, running slots and DtCluster state held in
//        the wave's LDS and registers from tick to tick (the replayed step kernel copies them in and
//        out of HBM every tick): phase A and the sample (dt_phase_a, dt_sample of
//        mcs_dtrade_dev.h), then its exchange record and, when a trader round is due, its node
//        snapshot and both contract sizes; it publishes the record (X1)
//   D    on a tick with a trader round due (any_due), the trader wave gathers every record (X1), runs
//        the rounds in cluster order on its own copy of the trader state (dt_rounds<true>: the same
//        code as dt_trader_kernel), and publishes the next tick's clock, each cluster's next round
//        and the count of the rounds' side effects on that cluster's live state, queued in HBM in
//        the rounds' order (X2); each cluster wave applies them (Foreign commits to a node and a
//        running slot, virtual nodes: pkg/scheduler/cluster.go:65-125) and starts the next tick
//   --   on a tick without a round (9 in 10 of C5-DELAY's) there is no phase D and no X2: a cluster
//        wave with queued jobs of its own knows the next clock is T + 1 (dt_next_ctl: queued_any,
//        not every job decided) and goes straight on; one with nothing queued reads every cluster's
//        four clock words of X1 and computes the clock itself (dm_next_clock: dt_next_ctl's T, done
//        and any_due).  So between two ticks with rounds the waves run ahead of each other, and a
//        tick costs the busiest cluster's average work rather than the maximum over the clusters of
//        every tick's (r06: 10.0 -> 9.0 us per C5-DELAY tick without X2, 8.2 -> 4.55 running ahead).
//        The trader reads every tick's clock words in order to keep the control block.
// Exchange: the worker workgroups run 8 blocks apart, which the dispatcher's round-robin puts on
// one XCD (checked at the launch's start: a launch whose workers landed on more than one XCD does
// nothing, and the engine runs the replayed kernels instead), so that XCD's L2 is the meeting
// point.  Every exchanged word travels as an 8-byte granule {value, tag} written with a plain store
// (write-through L1, so it lands in the L2) and read with agent-scope loads (L1 bypassed) until
// its tag is the exchange's epoch (tick + 1; the granules are zeroed before every launch): the data
// is the flag (cdna_hip_programming.md Guideline 16).  The bulk data behind a granule (node
// snapshots, the queued operations) is stored before it and drained with s_waitcnt vmcnt(0).
// X1 is a ring of kDmRing (32) buffers: a wave publishes tick n's records only after every reader (the
// trader and each cluster wave, through their progress granules) is done with tick n - kDmRing's.
// X2 needs one buffer: at a tick with rounds every wave waits for it, and the trader publishes the
// next one only after every wave has published a later tick's records.  A slot overflow (the run
// is redone with more slots) publishes its tick in an abort granule: every wave finishes that tick,
// so the trader finds its records and stops, and every wait watches the granule.
// Every wait is bounded (1 s without the epoch ends the launch with a failure word, and the engine
// redoes the run on the replayed kernels).  Same results bit for bit as the replayed tick
// (tests/test_gpu_dtrade.py).
#include "mcs_dtrade_dev.h"

namespace mcs {
namespace {

constexpr uint32_t kDmWaves = 4;  // cluster waves per workgroup, one per SIMD
constexpr uint32_t kDmThreads = kDmWaves * kWave;
constexpr uint32_t kDmRecWords = (uint32_t)(sizeof(DtRec) / 4u);
static_assert(sizeof(DtRec) % 4u == 0u && kDmRecWords <= (uint32_t)kWave, "a record word per lane");
// granules (u64) of gx: X1 records word-major [2][kDmRecWords][64] (word w of cluster q at w * 64 + q,
// one buffer per tick parity), X2 per-cluster words [64] (queued operations) and [64] (the cluster's
// next trader round), X2 clock words [4] (T, done, any_due, the earliest next round over the system),
// the trader's progress [1] (tag: the last tick whose records it has read, + 1)
constexpr uint32_t kDmRing = 32;  // X1 buffers: a cluster wave runs up to kDmRing ticks ahead of X1's readers (8: +0.8 %)
constexpr uint32_t kDmX1Buf = kDmRecWords * kDtResMaxClusters;
constexpr uint32_t kDmX2 = kDmRing * kDmX1Buf;
constexpr uint32_t kDmX2Due = kDmX2 + kDtResMaxClusters;
constexpr uint32_t kDmX2Ctl = kDmX2Due + kDtResMaxClusters;
constexpr uint32_t kDmTR = kDmX2Ctl + 4u;
constexpr uint32_t kDmP = kDmTR + 1u;                      // [64] each cluster wave's progress (tag: tick + 1)
constexpr uint32_t kDmAbort = kDmP + kDtResMaxClusters;    // an overflow's tick (tag 1: set)
constexpr uint32_t kDmGranules = kDmAbort + 1u;
// the record words the next tick's clock needs (DtRec: flags, done, queued, nxt), and nv
constexpr uint32_t kDmWFlags = (uint32_t)(offsetof(DtRec, flags) / 4u);
constexpr uint32_t kDmWNv = (uint32_t)(offsetof(DtRec, nv) / 4u);
static_assert(offsetof(DtRec, done) == offsetof(DtRec, flags) + 4 && offsetof(DtRec, queued) == offsetof(DtRec, flags) + 8 &&
                  offsetof(DtRec, nxt) == offsetof(DtRec, flags) + 12,
              "clock words contiguous");
// gu (uncached): [0, 32) one placement granule per worker, [32] the failure word
constexpr uint32_t kDmMaxWorkers = 32;  // one XCD's CUs
constexpr uint32_t kDmFail = kDmMaxWorkers;
static_assert(kDtResMaxClusters / kDmWaves + 1u <= kDmMaxWorkers, "workers on one XCD");
constexpr uint64_t kDmTimeout = 100000000ull;  // s_memrealtime ticks (100 MHz): 1 s

#ifdef MCS_STAMPS
// the probe build's tick timeline (s_memrealtime, 100 MHz), tools/stamp_dm.py: per cluster wave
// [c][0..4] phase A, sample, record + snapshot + contracts + X1 put, the X2 wait, the side effects;
// [c][5] ticks.  Per tick (ring of 1024, read and cleared by the trader after X1), each the slowest
// wave's: [0] side effects of the previous tick + work up to the X1 put, [1] phase A, [2] releases,
// [3] arrivals (+ the pass's first loads), [4] the Level1 pass, [5] the Level0 head, [6] the sample,
// [7] record + snapshot + contracts + X1 put.
// Trader sums: [0] X1 wait (from its X2 put), [1] the rounds, [2] next clock + X2 put, [3] ticks,
// [6] ticks with a round due, [8 + i] the per-tick maxima [i] summed
__device__ unsigned long long g_dm_cl[kDtResMaxClusters][6];
__device__ unsigned long long g_dm_tick[1024][8];
__device__ unsigned long long g_dm_tr[16];
#endif

__device__ __forceinline__ void dm_put(unsigned long long* g, uint32_t tag, uint32_t v) {
    const unsigned long long x = ((unsigned long long)tag << 32) | v;
    asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(g), "v"(x) : "memory");
}
__device__ __forceinline__ unsigned long long dm_get(const unsigned long long* g) {
    return __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t dm_xcc() {
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & 0xFu;
}
__device__ __forceinline__ void dm_fail(const DtResArgs& m, uint32_t why) {
    __hip_atomic_store(m.gu + kDmFail, (unsigned long long)why, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The clock after a tick with no trader round, from every cluster's record words of the tick (lane q:
// cluster q's flags, done, queued, nxt) and the earliest next round ndue: dt_next_ctl's T, done and
// any_due (its OVERFLOW test reads the records' flags alone: a round's overflow ends the run at its
// own tick, and a cluster's flags are sticky)
struct DmClock {
    uint32_t T;
    bool done, any_due;
};
__device__ __forceinline__ DmClock dm_next_clock(const DtArgs& a, const uint32_t lane, const uint32_t T,
                                                 const uint32_t fw, const uint32_t dw, const uint32_t qw,
                                                 const uint32_t xw, const uint32_t ndue) {
    const bool valid = lane < a.Ct;
    const bool done_all = __ballot(valid && dw == 0u) == 0ull;
    const bool queued_any = __ballot(valid && qw != 0u) != 0ull;
    uint32_t nxt = T + a.sample_period - T % a.sample_period;
    const uint32_t rn = wave_min_u32(valid ? xw : kEmpty);
    nxt = rn < nxt ? rn : nxt;
    nxt = ndue < nxt ? ndue : nxt;
    const bool ovf = __ballot(valid && (fw & MCS_FLAG_OVERFLOW) != 0u) != 0ull;
    DmClock k{T, false, false};
    if (done_all || ovf || T >= a.t_max) {
        k.done = true;
    } else {
        k.T = (queued_any || nxt <= T + 1u) ? T + 1u : nxt;
    }
    k.any_due = ndue <= k.T;
    return k;
}

// ---- a cluster wave: phases A and C of its cluster every tick, X1, X2 and the queued side effects ----
__device__ __forceinline__ void dm_cluster(const DtArgs& a, const DtResArgs& m, const uint32_t c, const uint32_t lane,
                                           unsigned long long* nodes, uint32_t* sfin, uint32_t* hist, float* dc,
                                           float* dm, DtRec* rec) {
    const uint32_t n0 = a.node_off[c], N = a.node_off[c + 1] - n0;
    const uint64_t j0 = a.job_off[c];
    const uint32_t J = (uint32_t)(a.job_off[c + 1] - j0);
    const uint4* jobs = a.jobs + j0;
    unsigned long long* l1cm = a.l1cm + j0;
    unsigned long long* l1jd = a.l1jd + j0;
    unsigned long long* l1al = a.l1al + j0;
    const size_t sb = (size_t)c * a.S;
    const uint32_t S = a.S;
    DtCluster st = a.cl[c];
    const DtCtl c0 = *a.ctl;
    uint32_t my_due = a.tr[c].next_due;  // this cluster's next trader round
    // the earliest next round over the system (kEmpty without traders)
    uint32_t ndue = wave_min_u32(a.period != 0u && lane < a.Ct ? a.tr[lane].next_due : kEmpty);
    uint32_t NN = N + st.nv;
    // (the replayed step kernel's per-tick state in, once per launch)
    unsigned long long snap_l = NN <= (uint32_t)kWave && lane < NN ? a.l1snap[(size_t)c * a.W + lane] : 0ull;
    copy_rounds<4>(nodes, a.tn + n0, N, lane);
    copy_rounds<2>(nodes + N, a.vn + (size_t)c * a.V, NN - N, lane);
    copy_rounds<8>(sfin, a.sfin + sb, S, lane);
    uint32_t T = c0.T;
    bool done = c0.done != 0u;
    bool any_due = a.period != 0u && c0.any_due != 0u;
    bool due = any_due && my_due <= T;
    unsigned long long* const gx = m.gx;
    unsigned long long* const snap = dt_snap(a, c);
    const unsigned long long* const ops =
        reinterpret_cast<const unsigned long long*>(m.ops) + (size_t)c * m.ops_cap * (sizeof(DtOp) / 8u);
    dt_wave_sync();
#ifdef MCS_STAMPS
    uint64_t dt_acc[7] = {0, 0, 0, 0, 0, 0, 0};
    uint64_t dt_last = 0;
#endif
    bool failed = false;
    bool aborted = false;  // another cluster's slot overflow ended the run (it is redone bigger)
    DtArrWin aw{kEmpty, kEmpty};  // the next 64 arrival times, kept from tick to tick
    uint32_t seen = 0;     // every reader has read X1 up to this tick (cached)
#ifdef MCS_STAMPS
    uint64_t sm[5] = {0, 0, 0, 0, 0}, sticks = 0, s_prev = wall_clock64(), s_ops = 0;
#endif
    for (uint32_t it = 0; it < m.budget && !done; ++it) {
#ifdef MCS_STAMPS
        const uint64_t s0 = wall_clock64();
        dt_last = s0;
        const uint64_t p1 = dt_acc[1], p2 = dt_acc[2], p3 = dt_acc[3];
#endif
        NN = N + st.nv;
        const bool exact = NN <= (uint32_t)kWave;
        if (!exact) snap_l = 0ull;  // (the replayed kernel loads it for exact clusters only)
        bool snap_dirty = false;
        st = dt_phase_a<true>(a, c, lane, T, N, NN, exact, j0, J, jobs, l1cm, l1jd, l1al, sb, S, nodes, sfin, hist, st,
                              snap_l, snap_dirty, aw DT_STAMP_ARGS);
        (void)snap_dirty;  // (written back at the launch's end)
#ifdef MCS_STAMPS
        const uint64_t s1 = wall_clock64();
#endif
        dt_sample<true>(a, c, lane, T, n0, N, NN, nodes, dc, dm, st);
#ifdef MCS_STAMPS
        const uint64_t s2 = wall_clock64();
#endif
        // the record, and when a trader round is due the node snapshot and the contract sizes
        if (any_due)
            for (uint32_t i = lane; i < NN; i += kWave) snap[i < N ? i : a.NS + (i - N)] = nodes[i];
        uint32_t fsc = 0, fsm = 0, fmd = 0, ssc = 0, ssm = 0, sst = 0;
        dt_contracts<true>(due, lane, st.l1n, l1cm, l1jd, hist, fsc, fsm, fmd, ssc, ssm, sst);
        uint32_t nxt = kEmpty;  // the next arrival, from the window (moved on when it is used up)
        if (st.next_arr < J) {
            dt_win_at(aw, st.next_arr, J, jobs, lane);
            nxt = readlane(aw.arr, st.next_arr - aw.base);
        }
        if (lane == 0u) {
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
            r.nxt = nxt;
            r.fc = fsc;
            r.fm = fsm;
            r.ft = fmd;
            r.sc = ssc;
            r.sm = ssm;
            r.st = sst;
            r.pad = 0u;
            *rec = r;
        }
        dt_wave_sync();
        if (any_due) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the snapshot lands before X1
        const uint32_t tag = it + 1u;
        unsigned long long* const x1 = gx + (size_t)(it % kDmRing) * kDmX1Buf;
        // the buffer's last records (tick it - kDmRing) must have been read by every reader: the
        // trader and every cluster wave (each publishes its progress after its tick's clock); the
        // minimum seen is cached, so the sweep runs about once per kDmRing ticks
        if (it >= kDmRing && it - kDmRing + 1u > seen) {
            const uint64_t t0 = wall_clock64();
            for (;;) {
                const unsigned long long x = lane < a.Ct ? dm_get(gx + kDmP + lane) : ~0ull;
                const unsigned long long tr = lane == 0u ? dm_get(gx + kDmTR) : 0ull;
                const unsigned long long ab = lane == 0u ? dm_get(gx + kDmAbort) : 0ull;
                const uint32_t mp = wave_min_u32((uint32_t)(x >> 32)), mt = readlane((uint32_t)(tr >> 32), 0u);
                const uint32_t mn = mp < mt ? mp : mt;
                if (readlane((uint32_t)(ab >> 32), 0u) != 0u) {  // (a run that overflowed: stop)
                    aborted = true;
                    break;
                }
                if (mn >= it - kDmRing + 1u) {
                    seen = mn;
                    break;
                }
                if (wall_clock64() - t0 > kDmTimeout) {
                    failed = true;
                    break;
                }
            }
            if (failed || aborted) break;
        }
        if (lane < kDmRecWords)
            dm_put(x1 + (size_t)lane * kDtResMaxClusters + c, tag, reinterpret_cast<const uint32_t*>(rec)[lane]);
#ifdef MCS_STAMPS
        const uint64_t s3 = wall_clock64();
        if (lane == 0u) {
            unsigned long long* tk = g_dm_tick[it & 1023u];
            atomicMax(&tk[0], (unsigned long long)(s_ops + (s3 - s0)));
            atomicMax(&tk[1], (unsigned long long)(s1 - s0));
            atomicMax(&tk[2], (unsigned long long)(dt_acc[1] - p1));
            atomicMax(&tk[3], (unsigned long long)(dt_acc[2] - p2));
            atomicMax(&tk[4], (unsigned long long)(dt_acc[3] - p3));
            atomicMax(&tk[5], (unsigned long long)(s1 - dt_last));
            atomicMax(&tk[6], (unsigned long long)(s2 - s1));
            atomicMax(&tk[7], (unsigned long long)(s3 - s2));
        }
        sm[0] += s1 - s0;
        sm[1] += s2 - s1;
        sm[2] += s3 - s2;
#endif
        uint32_t nops = 0u;
        if (any_due) {
            // X2 of a tick with trader rounds: lane 0 this cluster's queued operations, lane 1 its next
            // round, lanes 2-5 the clock
            const unsigned long long* src =
                gx + (lane == 0u ? kDmX2 + c : lane == 1u ? kDmX2Due + c : kDmX2Ctl + (lane < 6u ? lane - 2u : 0u));
            uint32_t v = 0u;
            const uint64_t t0 = wall_clock64();
            for (;;) {
                const unsigned long long x = lane < 6u ? dm_get(src)
                                             : lane == 63u ? dm_get(gx + kDmAbort) : ((unsigned long long)tag << 32);
                v = (uint32_t)x;
                if (readlane((uint32_t)(x >> 32), 63u) != 0u && readlane((uint32_t)x, 63u) < it) {
                    aborted = true;  // (the trader stopped at an earlier tick)
                    break;
                }
                if (__all(lane == 63u || (uint32_t)(x >> 32) == tag)) break;
                if (wall_clock64() - t0 > kDmTimeout) {
                    failed = true;
                    break;
                }
            }
            if (failed || aborted) break;
            nops = readlane(v, 0u);
            my_due = readlane(v, 1u);
            T = readlane(v, 2u);
            done = readlane(v, 3u) != 0u;
            any_due = a.period != 0u && readlane(v, 4u) != 0u;
            ndue = readlane(v, 5u);
        } else if (rec->queued != 0u && !(st.flags & MCS_FLAG_OVERFLOW) && T < a.t_max) {
            // no round, and this cluster has queued jobs: dt_next_ctl's clock is T + 1 whatever the
            // other records hold (queued_any; not every job is decided; an overflow elsewhere ends
            // the run, which is redone), so the wave goes on without reading them
            T = T + 1u;
            done = false;
            any_due = a.period != 0u && ndue <= T;
        } else {
            // no round: the clock from every cluster's records of the tick (lane q: cluster q)
            uint32_t fw = 0u, dw = 0u, qw = 0u, xw = 0u;
            const unsigned long long* src = x1 + (size_t)kDmWFlags * kDtResMaxClusters + lane;
            const bool valid = lane < a.Ct;
            const uint64_t t0 = wall_clock64();
            for (;;) {
                const unsigned long long tg = (unsigned long long)tag << 32;
                const unsigned long long x0 = valid ? dm_get(src) : tg;
                const unsigned long long x1w = valid ? dm_get(src + kDtResMaxClusters) : tg;
                const unsigned long long x2w = valid ? dm_get(src + 2u * kDtResMaxClusters) : tg;
                const unsigned long long x3w = valid ? dm_get(src + 3u * kDtResMaxClusters) : tg;
                fw = (uint32_t)x0;
                dw = (uint32_t)x1w;
                qw = (uint32_t)x2w;
                xw = (uint32_t)x3w;
                if (__all((uint32_t)(x0 >> 32) == tag && (uint32_t)(x1w >> 32) == tag &&
                          (uint32_t)(x2w >> 32) == tag && (uint32_t)(x3w >> 32) == tag))
                    break;
                const unsigned long long ab = lane == 0u ? dm_get(gx + kDmAbort) : 0ull;
                if (readlane((uint32_t)(ab >> 32), 0u) != 0u && readlane((uint32_t)ab, 0u) < it) {
                    aborted = true;  // (a cluster stopped at an earlier tick)
                    break;
                }
                if (wall_clock64() - t0 > kDmTimeout) {
                    failed = true;
                    break;
                }
            }
            if (failed || aborted) break;
            const DmClock k = dm_next_clock(a, lane, T, fw, dw, qw, xw, ndue);
            T = k.T;
            done = k.done;
            any_due = a.period != 0u && k.any_due;
        }
        due = any_due && my_due <= T;
        // this wave is done with tick it's records; a slot overflow here ends the run at tick it for
        // every wave (the others finish tick it, so every reader finds its records, and stop)
        if (lane == 0u) {
            dm_put(gx + kDmP + c, tag, 0u);
            if (st.flags & MCS_FLAG_OVERFLOW) dm_put(gx + kDmAbort, 1u, it);
        }
        {
            const unsigned long long ab = lane == 0u ? dm_get(gx + kDmAbort) : 0ull;
            if (readlane((uint32_t)(ab >> 32), 0u) != 0u && readlane((uint32_t)ab, 0u) <= it) done = true;
        }
#ifdef MCS_STAMPS
        const uint64_t s4 = wall_clock64();
        sm[3] += s4 - s3;
#endif
        // phase D's side effects on this cluster, in the rounds' order (what dt_trader_kernel writes
        // to the live state of a local cluster)
        for (uint32_t i = 0; i < nops; ++i) {
            const unsigned long long* op = ops + (size_t)i * (sizeof(DtOp) / 8u);
            const unsigned long long q0 = dm_get(op), q1 = dm_get(op + 1), q2 = dm_get(op + 2), q3 = dm_get(op + 3);
            const uint32_t kind = (uint32_t)q0, nd = (uint32_t)(q0 >> 32);
            if (kind == 1u) {  // go node.RunJob(Foreign) (cluster.go:116): the node and a running slot
                const uint32_t fin = (uint32_t)q2;
                uint32_t slot = kEmpty;
                for (uint32_t b = 0; b < S; b += kWave) {
                    const unsigned long long fr = __ballot(sfin[b + lane] == kEmpty);
                    if (fr) {
                        slot = b + (uint32_t)__builtin_ctzll(fr);
                        break;
                    }
                }
                if (slot != kEmpty) {
                    if (lane == 0u) {
                        nodes[nd] = q1;
                        sfin[slot] = fin;
                        a.snode[sb + slot] = nd;
                        a.scm[sb + slot] = (q2 >> 32) | (q3 << 32);
                    }
                    ++st.nrun;
                    st.minf = fin < st.minf ? fin : st.minf;
                    st.l1_dirty = 1u;  // the commit may wrap a counter
                }
            } else if (kind == 2u) {  // AddVirtualNode (cluster.go:65-85)
                if (lane == 0u) {
                    nodes[N + nd] = q1;
                    a.vcap[(size_t)c * a.V + nd] = make_uint2((uint32_t)q1, (uint32_t)(q1 >> 32));
                }
                ++st.nv;
                st.l1_dirty = 1u;
            } else {
                st.flags |= MCS_FLAG_VNODE_OVERFLOW;
            }
            dt_wave_sync();
        }
#ifdef MCS_STAMPS
        s_prev = wall_clock64();
        s_ops = s_prev - s4;
        sm[4] += s_ops;
        ++sticks;
#endif
    }
#ifdef MCS_STAMPS
    (void)s_prev;
    if (lane == 0u) {
        for (int i = 0; i < 5; ++i) atomicAdd(&g_dm_cl[c][i], (unsigned long long)sm[i]);
        atomicAdd(&g_dm_cl[c][5], (unsigned long long)sticks);
    }
#endif
    if (failed) {
        if (lane == 0u) dm_fail(m, 2u);
        return;
    }
    if (aborted) return;  // (the run overflowed and is redone: no state out)
    // the state out, for the next launch and the engine's readers
    dt_wave_sync();
    if (lane == 0u) a.cl[c] = st;
    NN = N + st.nv;
    copy_rounds<4>(a.tn + n0, nodes, N, lane);
    copy_rounds<2>(a.vn + (size_t)c * a.V, nodes + N, NN - N, lane);
    copy_rounds<8>(a.sfin + sb, sfin, S, lane);
    if (NN <= (uint32_t)kWave && lane < NN) a.l1snap[(size_t)c * a.W + lane] = snap_l;
}

// ---- the trader wave: X1 every tick; on a tick with a round due, phase D and X2 ----
__device__ __forceinline__ void dm_trader(const DtArgs& a, const DtResArgs& m, const uint32_t lane, DtTrader* trs,
                                          DtRec* srec, uint32_t* appr, uint32_t* nvs, uint32_t* nfr, uint32_t* opn) {
    const uint32_t Ct = a.Ct;
    for (uint32_t q = lane; q < Ct; q += kWave) trs[q] = a.tr[q];
    DtCtl c0 = *a.ctl;
    dt_wave_sync();
    if (c0.done) return;
    unsigned long long n_trades = c0.n_trades, n_won = c0.n_won, n_for = c0.n_foreign;
    unsigned long long* const gx = m.gx;
    DtOp* const ops = reinterpret_cast<DtOp*>(m.ops);
    bool failed = false;
#ifdef MCS_STAMPS
    uint64_t tsum[6] = {0, 0, 0, 0, 0, 0}, t_put = wall_clock64();
#endif
    for (uint32_t it = 0; it < m.budget; ++it) {
        const uint32_t T = c0.T;
        const bool any_due = c0.any_due != 0u;
        const uint32_t tag = it + 1u;
        const unsigned long long* const x1 = gx + (size_t)(it % kDmRing) * kDmX1Buf;
        const uint64_t t0 = wall_clock64();
        if (any_due) {
            // X1: lane q gathers cluster q's record
            uint32_t w[kDmRecWords];
            for (;;) {
                bool ok = true;
#pragma unroll
                for (uint32_t k = 0; k < kDmRecWords; ++k) {
                    const unsigned long long x = lane < Ct ? dm_get(x1 + (size_t)k * kDtResMaxClusters + lane)
                                                           : ((unsigned long long)tag << 32);
                    w[k] = (uint32_t)x;
                    ok = ok && (uint32_t)(x >> 32) == tag;
                }
                if (__all(ok)) break;
                if (wall_clock64() - t0 > kDmTimeout) {
                    failed = true;
                    break;
                }
            }
            if (failed) break;
            if (lane == 0u) dm_put(gx + kDmTR, tag, 0u);  // (this tick's records read)
            if (lane < Ct) {
                uint32_t* d = reinterpret_cast<uint32_t*>(&srec[lane]);
#pragma unroll
                for (uint32_t k = 0; k < kDmRecWords; ++k) d[k] = w[k];
                nvs[lane] = srec[lane].nv;
                nfr[lane] = srec[lane].nfree;
                opn[lane] = 0u;
            }
        } else {
            // a tick without rounds: the words of the next clock (and nv, for nv_all)
            uint32_t w[5];
            for (;;) {
                bool ok = true;
#pragma unroll
                for (uint32_t k = 0; k < 5u; ++k) {
                    const uint32_t wi = k == 4u ? kDmWNv : kDmWFlags + k;
                    const unsigned long long x = lane < Ct ? dm_get(x1 + (size_t)wi * kDtResMaxClusters + lane)
                                                           : ((unsigned long long)tag << 32);
                    w[k] = (uint32_t)x;
                    ok = ok && (uint32_t)(x >> 32) == tag;
                }
                if (__all(ok)) break;
                if (wall_clock64() - t0 > kDmTimeout) {
                    failed = true;
                    break;
                }
            }
            if (failed) break;
            if (lane == 0u) dm_put(gx + kDmTR, tag, 0u);
            if (lane < Ct) {
                srec[lane].flags = w[0];
                srec[lane].done = w[1];
                srec[lane].queued = w[2];
                srec[lane].nxt = w[3];
                nvs[lane] = w[4];
            }
        }
#ifdef MCS_STAMPS
        const uint64_t t1 = wall_clock64();
        tsum[0] += t1 - t_put;
        if (lane < 8u)  // (lane i sums the tick's [i])
            tsum[4] += __hip_atomic_exchange(&g_dm_tick[it & 1023u][lane], 0ull, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
#endif
        dt_wave_sync();
#ifdef MCS_STAMPS
        const uint64_t t2 = wall_clock64();
#endif
        const DtCounts k = dt_rounds<true>(a, lane, T, any_due, trs, srec, appr, nvs, nfr,
                                           DtCounts{n_trades, n_won, n_for, 0u}, DtOpQueue{ops, opn, m.ops_cap});
#ifdef MCS_STAMPS
        const uint64_t t3 = wall_clock64();
        tsum[1] += t3 - t2;
#endif
        n_trades = k.n_trades;
        n_won = k.n_won;
        n_for = k.n_for;
        const uint32_t lflags = k.lflags;
        const DtCtl nc = dt_next_ctl(a, lane, c0, trs, srec, lflags, n_trades, n_won, n_for);
        if (any_due) {  // X2: the rounds' side effects, every cluster's next round and the clock
            dt_wave_sync();
            const uint32_t on = lane < Ct ? opn[lane] : 0u;
            if (__ballot(on > m.ops_cap)) {  // (the run fails over; the cluster waves time out)
                failed = true;
                break;
            }
            const uint32_t nd = lane < Ct ? trs[lane].next_due : kEmpty;
            const uint32_t ndue = a.period != 0u ? wave_min_u32(nd) : kEmpty;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the operations and snapshot writes before X2
            if (lane < Ct) {
                dm_put(gx + kDmX2 + lane, tag, on);
                dm_put(gx + kDmX2Due + lane, tag, nd);
            }
            if (lane < 4u)
                dm_put(gx + kDmX2Ctl + lane, tag,
                       lane == 0u ? nc.T : (lane == 1u ? nc.done : (lane == 2u ? nc.any_due : ndue)));
        }
#ifdef MCS_STAMPS
        t_put = wall_clock64();
        tsum[2] += t_put - t3;
        tsum[3] += 1u;
        tsum[5] += any_due ? 1u : 0u;
#endif
        c0 = nc;
        if (nc.done) break;
    }
    if (failed) {
        if (lane == 0u) dm_fail(m, 3u);
        return;
    }
#ifdef MCS_STAMPS
    if (lane == 0u)
        for (int i = 0; i < 4; ++i) atomicAdd(&g_dm_tr[i], (unsigned long long)tsum[i]);
    if (lane == 0u) atomicAdd(&g_dm_tr[6], (unsigned long long)tsum[5]);
    if (lane < 8u) atomicAdd(&g_dm_tr[8 + lane], (unsigned long long)tsum[4]);
#endif
    dt_wave_sync();
    for (uint32_t q = lane; q < Ct; q += kWave) {
        a.tr[q] = trs[q];
        a.nv_all[q] = nvs[q];
    }
    if (lane == 0u) *a.ctl = c0;
}

__global__ __launch_bounds__(kDmThreads) void dt_mw_kernel(DtArgs a, DtResArgs m) {
    // the workers are blocks 0, 8, 16, ...: one XCD under the dispatcher's round-robin placement
    if (blockIdx.x % 8u != 0u) return;
    __shared__ unsigned long long s_nodes[kDmWaves][kDtResMaxNN];
    __shared__ uint32_t s_sfin[kDmWaves][kDtResMaxSlots];
    __shared__ uint32_t s_hist[kDmWaves][kWave];
    __shared__ float s_dcm[kDmWaves][2 * kDtResMaxNN];  // the sample's per-node differences
    __shared__ DtRec s_rec[kDmWaves];
    __shared__ DtTrader s_trs[kDtResMaxClusters];
    __shared__ DtRec s_srec[kDtResMaxClusters];
    __shared__ uint32_t s_appr[kDtResMaxClusters], s_nvs[kDtResMaxClusters], s_nfr[kDtResMaxClusters],
        s_opn[kDtResMaxClusters];
    __shared__ uint32_t s_ok;
    const uint32_t wg = blockIdx.x / 8u, lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t nw = m.nwg + 1u;  // the cluster workgroups and the trader's
    const bool trader = wg == m.nwg;
    if (trader && wave != 0u) return;
    // the placement: every worker publishes its XCD (uncached memory: valid on any XCD)
    if (wave == 0u) {
        if (lane == 0u)
            __hip_atomic_store(m.gu + wg, (1ull << 32) | dm_xcc(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bool ok = false;
        uint32_t v = 0u;
        const uint64_t t0 = wall_clock64();
        for (;;) {
            const unsigned long long x =
                lane < nw ? __hip_atomic_load(m.gu + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : (1ull << 32);
            v = (uint32_t)x;
            if (__all((uint32_t)(x >> 32) == 1u)) {
                ok = true;
                break;
            }
            if (wall_clock64() - t0 > kDmTimeout) break;
        }
        const uint32_t v0 = readlane(v, 0u);
        const bool same = ok && __all(lane >= nw || v == v0);
        if (!same && lane == 0u) dm_fail(m, 1u);
        if (lane == 0u) s_ok = same ? 1u : 0u;
    }
    if (!trader) __syncthreads();  // (the trader's workgroup is its wave 0 alone)
    if (s_ok == 0u) return;
    if (trader) {
        dm_trader(a, m, lane, s_trs, s_srec, s_appr, s_nvs, s_nfr, s_opn);
        return;
    }
    const uint32_t c = wg * kDmWaves + wave;
    if (c >= a.C) return;
    dm_cluster(a, m, c, lane, s_nodes[wave], s_sfin[wave], s_hist[wave], s_dcm[wave], s_dcm[wave] + kDtResMaxNN,
               &s_rec[wave]);
}

}  // namespace

size_t dtrade_mw_gx_bytes() { return (size_t)kDmGranules * 8u; }
size_t dtrade_mw_gu_bytes() { return (size_t)(kDmFail + 1u) * 8u; }
size_t dtrade_mw_op_bytes() { return sizeof(DtOp); }
uint32_t dtrade_mw_fail_word() { return kDmFail; }

}  // namespace mcs

// the probe build's tick timeline (g_dm_cl [64][6] then g_dm_tr [16]), read and cleared; -2 in the
// product build
extern "C" int mcs_debug_dm_stamps(unsigned long long* out) {
#ifdef MCS_STAMPS
    static unsigned long long z[mcs::kDtResMaxClusters * 6 + 16];
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(mcs::g_dm_cl), sizeof(mcs::g_dm_cl)) != hipSuccess ||
        hipMemcpyFromSymbol(out + mcs::kDtResMaxClusters * 6, HIP_SYMBOL(mcs::g_dm_tr), sizeof(mcs::g_dm_tr)) !=
            hipSuccess)
        return -1;
    if (hipMemcpyToSymbol(HIP_SYMBOL(mcs::g_dm_cl), z, sizeof(mcs::g_dm_cl)) != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(mcs::g_dm_tr), z, sizeof(mcs::g_dm_tr)) != hipSuccess)
        return -1;
    return 0;
#else
    (void)out;
    return -2;
#endif
}
// the probe build's Level1 row counters of the resident tick (g_dt_rows [21]), read and cleared
extern "C" int mcs_debug_dm_rows(unsigned long long* out) {
#ifdef MCS_STAMPS
    unsigned long long z[21] = {};
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(mcs::g_dt_rows), sizeof(z)) != hipSuccess) return -1;
    return hipMemcpyToSymbol(HIP_SYMBOL(mcs::g_dt_rows), z, sizeof(z)) == hipSuccess ? 0 : -1;
#else
    (void)out;
    return -2;
#endif
}

namespace mcs {

hipError_t launch_dtrade_mw(const DtArgs& a, const DtResArgs& m, hipStream_t s) {
    if (a.Ct != a.C || a.C > kDtResMaxClusters || a.S > kDtResMaxSlots || m.nwg != (a.C + kDmWaves - 1) / kDmWaves)
        return hipErrorInvalidValue;
    hipError_t st = hipMemsetAsync(m.gx, 0, dtrade_mw_gx_bytes(), s);
    if (st != hipSuccess) return st;
    st = hipMemsetAsync(m.gu, 0, dtrade_mw_gu_bytes(), s);
    if (st != hipSuccess) return st;
    hipLaunchKernelGGL(dt_mw_kernel, dim3(8u * m.nwg + 1u), dim3(kDmThreads), 0, s, a, m);
    return hipGetLastError();
}

}  // namespace mcs
