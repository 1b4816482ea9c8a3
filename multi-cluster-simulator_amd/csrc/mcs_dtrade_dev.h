// mcs_dtrade_dev.h — device code of the DELAY trading tick shared by its two loops:
// the replayed two-kernel tick (mcs_dtrade.hip: dt_step_kernel + dt_trader_kernel, any world size)
// and the resident tick (mcs_dtrade_mw.hip: one launch for many ticks, world 1).  RES = true is the
// resident form: several cluster waves share a workgroup, so every sync is a wave-level one, and
// phase D queues its side effects on a cluster's live state (Foreign commits, virtual nodes) as
// operations for the cluster's own wave instead of writing that state, which lives in the wave's LDS.
#pragma once
#include "mcs_dtrade_internal.h"
#include "mcs_trader_dev.h"
#include "mcs_wave.h"

namespace mcs {
namespace {

// dt_step_kernel is one wave per block (launch_bounds 64): its LDS traffic is ordered by the wave's
// own in-order LDS queue, so between its phases a compiler barrier suffices.  __syncthreads() would
// also wait for every outstanding global load, i.e. drain the Level1 rows prefetched ahead.
__device__ __forceinline__ void dt_wave_sync() {
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}


// wave reductions on the DPP scans of mcs_wave.h, read at lane 63: VALU steps instead of a chain
// of six dependent ds_bpermute round trips (every lane active at every call site)
__device__ __forceinline__ uint32_t dt_wave_sum_u32(uint32_t v) { return readlane(wave_scan_add_u32(v), 63u); }

__device__ __forceinline__ long long dt_wave_sum_i64(long long v) {
    unsigned long long u = (unsigned long long)v;  // (two's complement: the same adds)
    auto step = [&](unsigned long long w) { u += w; };
#define DT_DPP64(CTRL, MASK)                                                                  \
    step((unsigned long long)dpp_src0<CTRL, MASK>((uint32_t)u) |                              \
         ((unsigned long long)dpp_src0<CTRL, MASK>((uint32_t)(u >> 32)) << 32))
    DT_DPP64(0x111, 0xf);
    DT_DPP64(0x112, 0xf);
    DT_DPP64(0x114, 0xf);
    DT_DPP64(0x118, 0xf);
    DT_DPP64(0x142, 0xa);
    DT_DPP64(0x143, 0xc);
#undef DT_DPP64
    return (long long)(((unsigned long long)readlane((uint32_t)(u >> 32), 63u) << 32) | readlane((uint32_t)u, 63u));
}

__device__ __forceinline__ uint32_t dt_wave_max_u32(uint32_t v) { return readlane(wave_scan_max_u32(v), 63u); }

// Go uint64 value of a device free counter (sign extension of the u32, see the header)
__device__ __forceinline__ unsigned long long go_u64(uint32_t x) {
    return (unsigned long long)(long long)(int32_t)x;
}
__device__ __forceinline__ float go_f32(uint32_t x) { return (float)go_u64(x); }
__device__ __forceinline__ double go_f64(uint32_t x) { return (double)go_u64(x); }

// Go's float64 -> uint conversion on amd64 (mcs_oracle_dtrade.c: go_f64_to_u64)
__device__ __forceinline__ unsigned long long go_f64_to_u64(double x) {
    const double two63 = 9223372036854775808.0;
    if (x < two63) return (unsigned long long)(long long)x;
    const double y = x - two63;
    if (y >= two63) return 0ull;
    return (unsigned long long)(long long)y ^ 0x8000000000000000ull;
}

__device__ __forceinline__ uint32_t ld32(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld64(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// rank block of global cluster g: its exchange record and node snapshot
__device__ __forceinline__ const DtRec* dt_rec(const DtArgs& a, uint32_t g) {
    const uint32_t r = g / a.C, c = g - r * a.C;
    return reinterpret_cast<const DtRec*>(a.xb + (size_t)r * a.blk) + c;
}
__device__ __forceinline__ unsigned long long* dt_snap(const DtArgs& a, uint32_t g) {
    const uint32_t r = g / a.C, c = g - r * a.C;
    return reinterpret_cast<unsigned long long*>(a.xb + (size_t)r * a.blk + (size_t)a.C * sizeof(DtRec)) +
           (size_t)c * a.W;
}

#ifdef MCS_STAMPS
// the probe build's dt_step segment times (s_memrealtime, 100 MHz), summed over clusters and ticks:
// 0 state in + LDS copies, 1 releases, 2 arrivals, 3 Level1 pass, 4 Level0 head, 5 copies out +
// sample, 6 record + snapshot + contract sizes; [7] dt_step calls (clusters x ticks)
__device__ unsigned long long g_dt_stamps[8];
// per tick: the slowest cluster's step (and each segment's slowest), summed over ticks by the trader
// kernel of the tick ([0-6] segments, [7] the whole step); [8] the trader kernel's own time, [9] ticks
__device__ unsigned long long g_dt_cur[8];
__device__ unsigned long long g_dt_maxsum[10];
// inside the Level1 pass, summed over every row of every pass: [0] the fit tests and placements,
// [1] the WaitTime and compaction bookkeeping, [2] rows, [3] placements (of the general rows);
// [4] quiet rows, [5] passes, [6] candidates given a first fit, [7] the passes' time; of which
// [8] before the row loop, [9] the row loop, [10] after it
// (the probe's per-pair split, [11]-[16], is not built here); the trader rounds: [17]/[18] time/count
// of stage steps that trade (a request), [19]/[20] of those that do not
__device__ unsigned long long g_dt_rows[21];
#define DT_MARK(i)                                  \
    do {                                            \
        const uint64_t dt_now = wall_clock64();     \
        dt_acc[i] += dt_now - dt_last;              \
        dt_last = dt_now;                           \
    } while (0)
#define DT_STAMP_PARAMS , uint64_t(&dt_acc)[7], uint64_t& dt_last
#define DT_STAMP_ARGS , dt_acc, dt_last
#else
#define DT_MARK(i) \
    do {           \
    } while (0)
#define DT_STAMP_PARAMS
#define DT_STAMP_ARGS
#endif

// a wave-level sync in the resident form (each wave its own cluster), the workgroup's barrier in the
// replayed step kernel (one wave per workgroup: the r05 schedule, which it keeps)
template <bool RES>
__device__ __forceinline__ void dt_bar() {
    if constexpr (RES) dt_wave_sync();
    else __syncthreads();
}

// (resident tick) a side effect of phase D on one cluster's live state, applied by its own wave in
// phase D's order: 1 a Foreign job's commit (go node.RunJob(Foreign), cluster.go:116: the node's new
// free vector {lo, hi} and a running slot until fin holding {fc, fm}), 2 the virtual node nd with
// capacity {lo, hi} (AddVirtualNode, cluster.go:65-85), 3 the virtual-node pool overflowed
struct DtOp {
    uint32_t kind, nd, lo, hi, fin, fc, fm, pad;
};
static_assert(sizeof(DtOp) == 32, "DtOp layout");
struct DtOpQueue {
    DtOp* ops;     // [cluster][cap]
    uint32_t* n;   // per cluster, this tick (LDS)
    uint32_t cap;
    __device__ __forceinline__ void push(uint32_t q, const DtOp& o) {  // (one lane)
        const uint32_t k = n[q];
        if (k < cap) ops[(size_t)q * cap + k] = o;
        n[q] = k + 1u;  // (above cap: the run fails over to the replayed kernels)
    }
};

// The arrival times of 64 jobs from `base` (lane i: job base + i, kEmpty past the cluster's last):
// the resident tick keeps them in a register from tick to tick, so the arrivals and the record's next
// arrival read no job record from HBM until the window is used up (the replayed step kernel starts
// every tick with base = kEmpty: one load, as before)
struct DtArrWin {
    uint32_t base;
    uint32_t arr;
};
__device__ __forceinline__ void dt_win_at(DtArrWin& w, const uint32_t at, const uint32_t J, const uint4* jobs,
                                          const uint32_t lane) {
    if (at < w.base || at - w.base >= (uint32_t)kWave) {
        w.base = at;
        const uint32_t i = at + lane;
        w.arr = i < J ? jobs[i].x : kEmpty;
    }
}

// ---------------------------------------------------------------------------------------------
// Phase A of cluster c at tick T, after its state, nodes and slots are in place (nodes and sfin in
// LDS, the cluster state st): releases, "/delay" arrivals, the Level1 pass, the Level0 head.  j0, J:
// the cluster's jobs (loaded by the caller with its first batch of loads).
template <bool RES>
__device__ __forceinline__ DtCluster dt_phase_a(const DtArgs& a, const uint32_t c, const uint32_t lane, const uint32_t T,
                                           const uint32_t N, const uint32_t NN, const bool exact, const uint64_t j0,
                                           const uint32_t J, const uint4* jobs, unsigned long long* l1cm,
                                           unsigned long long* l1jd, unsigned long long* l1al, const size_t sb,
                                           const uint32_t S,
                                           unsigned long long* nodes, uint32_t* sfin, uint32_t* hist, DtCluster st,
                                           unsigned long long& snap_l, bool& snap_dirty, DtArrWin& aw DT_STAMP_PARAMS) {

    // releases due at T (cluster.go:153-157), Foreign jobs included
    if (st.minf <= T) {
        uint32_t lm = kEmpty, nrel = 0;
        for (uint32_t s = lane; s < S; s += kWave) {
            const uint32_t f = sfin[s];
            if (f <= T) {
                // per u32 half: a wrapped counter's low half may carry (Go's uint64 wraps back)
                const unsigned long long cm = a.scm[sb + s];
                uint32_t* h = reinterpret_cast<uint32_t*>(&nodes[a.snode[sb + s]]);
                atomicAdd(h, (uint32_t)cm);
                atomicAdd(h + 1, (uint32_t)(cm >> 32));
                sfin[s] = kEmpty;
                ++nrel;
            } else {
                lm = f < lm ? f : lm;
            }
        }
        const uint32_t nr = dt_wave_sum_u32(nrel);
        st.nrun -= nr;
        st.l1_dirty |= nr != 0u ? 1u : 0u;
        st.minf = wave_min_u32(lm);
        dt_bar<RES>();
    }
    DT_MARK(1);
    // "/delay" arrivals up to T join Level0 (server.go:67-74): JobsMap[id] = 0, JobsCount++
    {
        const uint32_t before = st.next_arr;
        while (st.next_arr < J) {
            dt_win_at(aw, st.next_arr, J, jobs, lane);
            const uint32_t off = st.next_arr - aw.base;
            // (arrival-sorted: the jobs arrived by T are the window's lanes [off, off + n))
            const bool ok = lane >= off && aw.arr <= T;
            const uint32_t n = (uint32_t)__builtin_popcountll(__ballot(ok));
            st.next_arr += n;
            if (off + n < (uint32_t)kWave) break;
        }
        st.count += (long long)(st.next_arr - before);
    }

    // the Level1 pass's first rows, in flight from here (vmcnt waits in issue order: a load issued
    // before the copies, the releases or the arrivals would be drained by their waits)
    // (8 or 12 rows ahead in the resident tick measured slower: 10.85 -> 11.03 / 11.37 us per C5-DELAY
    // tick, profiles/r06_dm/ab_ahead.txt)
    constexpr int kL1Ahead = 4;
    unsigned long long pcm[kL1Ahead], pjd[kL1Ahead], pal[kL1Ahead];
    // (every lane loads, at an index clamped into the list: a load under a lane condition ends in a
    // merge of old and new values that waits for it on the spot)
    if (st.l1n != 0u) {
        const uint32_t n1 = st.l1n;
#pragma unroll
        for (int r = 0; r < kL1Ahead; ++r) {
            const uint32_t p = (uint32_t)r * kWave + lane, pi = p < n1 ? p : n1 - 1u;
            pcm[r] = l1cm[pi];
            pjd[r] = l1jd[pi];
            pal[r] = l1al[pi];
        }
    } else {
#pragma unroll
        for (int r = 0; r < kL1Ahead; ++r) pcm[r] = pjd[r] = pal[r] = 0ull;
    }
    DT_MARK(2);
    // ScheduleJob (scheduler.go:127-139) over Cluster.Nodes: physical, then virtual
    auto first_fit = [&](uint32_t jc, uint32_t jm) -> uint32_t {
        uint32_t best = kEmpty;
        for (uint32_t b = 0; b < NN; b += kWave) {
            const uint32_t i = b + lane;
            if (i < NN) {
                const unsigned long long v = nodes[i];
                if ((uint32_t)v >= jc && (uint32_t)(v >> 32) >= jm) best = i;
            }
            if (__ballot(best != kEmpty)) break;
        }
        return wave_min_u32(best);
    };
    // Node.RunJob commit (cluster.go:144-148) + running slot; false on slot overflow
    auto commit = [&](uint32_t k, uint32_t jc, uint32_t jm, uint32_t fin) -> bool {
        const unsigned long long need = (unsigned long long)jc | ((unsigned long long)jm << 32);
        uint32_t slot = kEmpty;
        for (uint32_t b = 0; b < S; b += kWave) {
            const unsigned long long fr = __ballot(sfin[b + lane] == kEmpty);
            if (fr) {
                slot = b + (uint32_t)__builtin_ctzll(fr);
                break;
            }
        }
        if (slot == kEmpty) return false;
        if (lane == 0) {
            // u32 halves: a wrapped node may borrow across them (Go's uint64 counters would
            // wrap the same way), so update each half on its own
            nodes[k] = (unsigned long long)((uint32_t)nodes[k] - jc) |
                       ((unsigned long long)((uint32_t)(nodes[k] >> 32) - jm) << 32);
            sfin[slot] = fin;
            a.snode[sb + slot] = k;
            a.scm[sb + slot] = need;
        }
        dt_wave_sync();
        ++st.nrun;
        st.peak = st.nrun > st.peak ? st.nrun : st.peak;
        st.minf = fin < st.minf ? fin : st.minf;
        return true;
    };

    // ---- Level1 pass (scheduler.go:302-329) ----
    if (st.l1n != 0u && !st.l1_dirty) {
        // nothing raised a free counter since the last pass and it placed nothing: every entry
        // fails again; each JobsMap entry becomes 1000 * (T - arrival)
        st.total += 1000ll * (long long)((unsigned long long)st.l1n * T - st.s_last);
        st.s_last = (unsigned long long)st.l1n * T;
        st.t_all = T;
    } else if (st.l1n != 0u) {
#ifdef MCS_STAMPS
        const uint64_t pt0 = wall_clock64();
#endif
        // bigger clusters: exact fit filter (see mcs_delay.hip): lane l holds the max free memory
        // over nodes with min(free cores, 63) >= l; conservative for wrapped counters
        uint32_t best = 0u, max_c = 0u;
        if (!exact) {
            hist[lane] = 0u;
            dt_bar<RES>();
            uint32_t mc = 0u;
            for (uint32_t i = lane; i < NN; i += kWave) {
                const unsigned long long v = nodes[i];
                const uint32_t fc = (uint32_t)v;
                atomicMax(&hist[fc < 63u ? fc : 63u], (uint32_t)(v >> 32));
                mc = fc > mc ? fc : mc;
            }
            dt_bar<RES>();
            max_c = dt_wave_max_u32(mc);
            // suffix maximum: a DPP prefix scan of the reversed histogram, reversed back
            const uint32_t sc = wave_scan_max_u32(hist[63u - lane]);
            best = (uint32_t)__shfl((int)sc, (int)(63u - lane));
        }
        // per lane: the lowest node (physical, then virtual) that fits this lane's entry
        // (the node values come from one LDS read per lane, node i in lane i, then readlanes: no
        // chain of dependent LDS reads per entry test; called with every lane active)
        auto lane_fit = [&](uint32_t c_l, uint32_t m_l) -> uint32_t {
            const unsigned long long nv = lane < NN ? nodes[lane] : 0ull;
            const uint32_t nc = (uint32_t)nv, nm = (uint32_t)(nv >> 32);
            uint32_t kl = kEmpty;
            for (uint32_t i = NN; i-- > 0u;) {
                const uint32_t vc = readlane(nc, i), vm = readlane(nm, i);
                kl = (vc >= c_l && vm >= m_l) ? i : kl;
            }
            return kl;
        };
        // the grown nodes (exact clusters): more than 16 -> every job is tested on every node
        unsigned long long gmask = 0ull;
        if (exact) {
            const unsigned long long cur = lane < NN ? nodes[lane] : 0ull;
            gmask = __ballot(lane < NN && ((uint32_t)cur > (uint32_t)snap_l ||
                                           (uint32_t)(cur >> 32) > (uint32_t)(snap_l >> 32)));
        }
        const bool g_all = __builtin_popcountll(gmask) > 16;
        // does this lane's job fit some grown node (current values)?  (every lane active)
        // (the node values in a register for the pass, node i in lane i; refreshed after a commit)
        unsigned long long nvv = exact && lane < NN ? nodes[lane] : 0ull;
#ifndef MCS_DT_GLOOP
        // G as a staircase: lane 63 - x holds the largest free memory over the grown nodes with
        // min(free cores, 63) >= x (0: none), so a job (c, m) fits some grown node only if
        // gtab[63 - min(c, 63)] >= m: one permute per test instead of a readlane chain over G.  A
        // superset (cores clamped at 63, m = 0): every candidate still gets the real first fit, and a
        // quiet row is one where nothing passes.  Rebuilt after each commit (nodes only shrink).
        uint32_t gtab = 0u;
        // (r06: one or two grown nodes tested exactly against their values in scalars instead, no
        // permute: 8.92 -> 10.69 us per C5-DELAY tick, profiles/r06_dm/ab_ct.txt)
        auto g_build = [&]() {
            hist[lane] = 0u;
            dt_wave_sync();
            if ((gmask >> lane) & 1ull) {
                const uint32_t nc = (uint32_t)nvv;
                atomicMax(&hist[nc < 63u ? nc : 63u], (uint32_t)(nvv >> 32));
            }
            dt_wave_sync();
            gtab = wave_scan_max_u32(hist[63u - lane]);
        };
        if (exact && !g_all && gmask) g_build();
        auto g_fit = [&](uint32_t c_l, uint32_t m_l) -> bool {
            const uint32_t t = (uint32_t)__shfl((int)gtab, (int)(63u - (c_l < 63u ? c_l : 63u)));
            return gmask != 0ull && t >= m_l;
        };
#else
        auto g_build = [&]() {};
        auto g_fit = [&](uint32_t c_l, uint32_t m_l) -> bool {
            const uint32_t nc = (uint32_t)nvv, nm = (uint32_t)(nvv >> 32);
            bool f = false;
            for (unsigned long long g = gmask; g; g &= g - 1ull) {
                const uint32_t k = (uint32_t)__builtin_ctzll(g);
                f = f || (readlane(nc, k) >= c_l && readlane(nm, k) >= m_l);
            }
            return f;
        };
#endif
        uint32_t wr = 0;
        bool carry_skip = false;  // the last entry of the previous row was placed
        const uint32_t n1 = st.l1n, t_all = st.t_all;
        // WaitTime in closed form: s_last is the sum of every entry's effective last examination, so
        // the pass's JobsMap moves are 1000 * (n_examined * T - (s_last - the skipped entries' sum))
        // and the kept entries' new sum is (kept - skipped) * T + the skipped entries' sum; only the
        // entries a D6 skip passes over (general rows) need their own stamp (per-lane partial sum,
        // reduced once after the sweep), and a quiet row does no WaitTime arithmetic
        unsigned long long sk_eff = 0ull;
        uint32_t n_skip = 0;
        // rows of 64 entries; each row's three coalesced loads are issued kL1Ahead rows ahead (the
        // first ones before the pass), so a row's HBM latency hides behind the rows before it
        // (compaction writes only at or below the row in hand: never into a prefetched row)
        // one row of the pass; false: a slot overflow (the run stops, the engine re-runs bigger)
        auto row = [&](const uint32_t base, const unsigned long long cm, const unsigned long long jdv,
                       const unsigned long long al) -> bool {
            const uint32_t pos = base + lane;
            const bool live = pos < n1;
#ifdef MCS_STAMPS
            const uint64_t rt0 = wall_clock64();
#endif
            const uint32_t jc_l = (uint32_t)cm, jm_l = (uint32_t)(cm >> 32);
            unsigned long long placedm = 0ull, skipm = carry_skip ? 1ull : 0ull;
            bool overflow = false;
            if (exact) {
                const bool untested = ((uint32_t)jdv >> 31) != 0u;
                uint32_t from = 0;
                for (;;) {  // the next entry in list order that fits now and is not skipped
                    dt_wave_sync();
                    // candidates: jobs that fit a grown node, and the untested (all lanes: the
                    // tests read across lanes)
                    bool cf;
                    if (g_all) {
                        cf = lane_fit(jc_l, jm_l) != kEmpty;
                    } else {
                        cf = g_fit(jc_l, jm_l) || untested;
                    }
                    const unsigned long long fitm = __ballot(live && cf) & ~skipm &
                                                    (from < 64u ? (~0ull << from) : 0ull);
                    if (!fitm) break;
                    const uint32_t b = (uint32_t)__builtin_ctzll(fitm);
                    const uint32_t jc = readlane(jc_l, b), jm = readlane(jm_l, b);
                    const uint32_t k = first_fit(jc, jm);
#ifdef MCS_STAMPS
                    if (lane == 0) atomicAdd(&g_dt_rows[6], 1ull);
#endif
                    if (k == kEmpty) {  // an untested job that fits no node after all
                        from = b + 1u;
                        continue;
                    }
                    const uint32_t jd = readlane((uint32_t)(jdv >> 32), b),
                                   jj = readlane((uint32_t)jdv, b) & 0x7FFFFFFFu;
                    const uint32_t fin = T + jd;
                    if (jd != 0u && !commit(k, jc, jm, fin)) {
                        overflow = true;
                        break;
                    }
                    if (jd != 0u) {  // (node k shrank)
                        nvv = lane < NN ? nodes[lane] : 0ull;
                        if (!g_all && ((gmask >> k) & 1ull)) g_build();
                    }
                    if (lane == 0) {
                        a.out_node[j0 + jj] = (int32_t)k;
                        a.out_start[j0 + jj] = T;
                        a.out_finish[j0 + jj] = fin;
                    }
                    placedm |= 1ull << b;
                    if (b < 63u) skipm |= 1ull << (b + 1u);
                    from = b + 2u;
                    ++st.decided;
                    ++st.placed_l1;
                }
            } else {
                const uint32_t bm = (uint32_t)__shfl((int)best, (int)(jc_l < 63u ? jc_l : 63u));
                unsigned long long cand = __ballot(live && jc_l <= max_c && bm >= jm_l);
                while (cand) {
                    const uint32_t b = (uint32_t)__builtin_ctzll(cand);
                    cand &= cand - 1ull;
                    if ((skipm >> b) & 1ull) continue;  // slid into slot i: not examined (D6)
                    const uint32_t jc = readlane(jc_l, b), jm = readlane(jm_l, b);
                    const uint32_t k = first_fit(jc, jm);
                    if (k == kEmpty) continue;
                    const uint32_t jd = readlane((uint32_t)(jdv >> 32), b),
                                   jj = readlane((uint32_t)jdv, b) & 0x7FFFFFFFu;
                    const uint32_t fin = T + jd;
                    if (jd != 0u && !commit(k, jc, jm, fin)) {
                        overflow = true;
                        break;
                    }
                    if (lane == 0) {
                        a.out_node[j0 + jj] = (int32_t)k;
                        a.out_start[j0 + jj] = T;
                        a.out_finish[j0 + jj] = fin;
                    }
                    placedm |= 1ull << b;
                    if (b < 63u) skipm |= 1ull << (b + 1u);
                    ++st.decided;
                    ++st.placed_l1;
                }
            }
            if (overflow) {
                st.flags |= MCS_FLAG_OVERFLOW;
                wr = n1;  // state is abandoned (the engine re-runs with more slots)
                return false;
            }
#ifdef MCS_STAMPS
            const uint64_t rt1 = wall_clock64();
#endif
            const unsigned long long livem = __ballot(live);
            const uint32_t last = 63u - (uint32_t)__builtin_clzll(livem);
            carry_skip = ((placedm >> last) & 1ull) != 0ull && last == 63u;
            // WaitTime update of every examined job (the skipped one is not examined): its
            // JobsMap entry goes from 1000 * (last - arrival) to 1000 * (T - arrival)
            const bool examined = live && !((skipm >> lane) & 1ull);
            const bool placed = ((placedm >> lane) & 1ull) != 0ull;
            const uint32_t sl = (uint32_t)(al >> 32);
            // the entry's last examination: its own stamp while it is marked untested (a D6 skip
            // materialised it), else the later of the stamp and the list's floor t_all
            const uint32_t eff = ((uint32_t)jdv >> 31) != 0u ? sl : (sl > t_all ? sl : t_all);
            sk_eff += live && !examined ? (unsigned long long)eff : 0ull;
            n_skip += (uint32_t)__builtin_popcountll(skipm & livem);
            // compaction in the same sweep (append(Level1[:i], Level1[i+1:]...), :319)
            const unsigned long long kept = livem & ~placedm;
            const uint32_t nl = examined ? T : eff;  // the kept entry's last examination
            if (live && !placed) {
                const uint32_t np = wr + (uint32_t)__builtin_amdgcn_mbcnt_hi(
                                             (uint32_t)(kept >> 32),
                                             __builtin_amdgcn_mbcnt_lo((uint32_t)kept, 0u));
                // the untested mark (bit 31 of the job word): set on a skipped job, cleared on an
                // examined one
                const unsigned long long jdn = examined ? (jdv & ~0x80000000ull) : (jdv | 0x80000000ull);
                if (np != pos) {
                    l1cm[np] = cm;
                    l1jd[np] = jdn;
                } else if (jdn != jdv) {
                    l1jd[np] = jdn;
                }
                // (an examined entry left in place keeps its stamp: the floor t_all = T set after
                // the pass makes its last examination T; a skipped one carries its own)
                // (an examined entry left in place could keep its stamp, the floor t_all = T set after
                // the pass makes its last examination T, but testing for it here costs the kernel 50
                // more SGPR spills: rows with a candidate are rare, quiet rows skip the store)
                if (np != pos || nl != sl) l1al[np] = (al & 0xFFFFFFFFull) | ((unsigned long long)nl << 32);
            }
            wr += (uint32_t)__builtin_popcountll(kept);
#ifdef MCS_STAMPS
            if (lane == 0) {
                atomicAdd(&g_dt_rows[0], (unsigned long long)(rt1 - rt0));
                atomicAdd(&g_dt_rows[1], (unsigned long long)(wall_clock64() - rt1));
                atomicAdd(&g_dt_rows[2], 1ull);
                atomicAdd(&g_dt_rows[3], (unsigned long long)__builtin_popcountll(placedm));
            }
#endif
            return true;
        };
        // a quiet row: no job of it fits now (none fits a grown node, none is untested) and its first
        // job is examined (no skip carried in): only the compaction, as the general row does it with
        // nothing placed (the live jobs are a prefix: rank = lane; the shift wr0 - base is uniform, no
        // entry is untested, and a moved entry keeps its stamp: its last examination is the floor
        // t_all = T set after the pass)
        auto quiet_row = [&](const uint32_t base, const unsigned long long cm, const unsigned long long jdv,
                             const unsigned long long al, const uint32_t wr0) {
            if (wr0 != base && base + lane < n1) {
                const uint32_t np = wr0 + lane;
                l1cm[np] = cm;
                l1jd[np] = jdv;
                l1al[np] = al;
            }
        };
        const bool quiet_ok = exact && !g_all;
        bool ok_pass = true;
#ifdef MCS_STAMPS
        const uint64_t pt1 = wall_clock64();
#endif
        // rows in pairs: two quiet rows are tested and booked together (independent instruction
        // streams for the one wave of the CU); a row with a candidate, or with a skip carried into
        // it, goes through row()  (r04: 19.2 -> 17.1 us per C5-DELAY tick; testing and booking a
        // whole group of four first measured 17.6)
        for (uint32_t base0 = 0; base0 < n1 && ok_pass; base0 += kL1Ahead * kWave) {
#pragma unroll
            for (int r = 0; r < kL1Ahead; r += 2) {
                const uint32_t ba = base0 + (uint32_t)r * kWave, bb = ba + kWave;
                if (!ok_pass || ba >= n1) break;
                const unsigned long long cma = pcm[r], jda = pjd[r], ala = pal[r];
                const unsigned long long cmb = pcm[r + 1], jdb = pjd[r + 1], alb = pal[r + 1];
                const uint32_t nxa = ba + kL1Ahead * kWave + lane, nxb = nxa + kWave;
                const uint32_t nia = nxa < n1 ? nxa : n1 - 1u, nib = nxb < n1 ? nxb : n1 - 1u;
                pcm[r] = l1cm[nia];  // (unconditional: see the first rows' loads)
                pjd[r] = l1jd[nia];
                pal[r] = l1al[nia];
                pcm[r + 1] = l1cm[nib];
                pjd[r + 1] = l1jd[nib];
                pal[r + 1] = l1al[nib];
                const bool has_b = bb < n1;
                bool qa = false, qb = false;
                if (quiet_ok && !carry_skip) {  // (both rows' permutes in flight together)
                    const bool fa = g_fit((uint32_t)cma, (uint32_t)(cma >> 32)) || ((uint32_t)jda >> 31) != 0u;
                    const bool fb = g_fit((uint32_t)cmb, (uint32_t)(cmb >> 32)) || ((uint32_t)jdb >> 31) != 0u;
                    qa = __ballot(ba + lane < n1 && fa) == 0ull;
                    qb = has_b && __ballot(bb + lane < n1 && fb) == 0ull;
                }
#ifdef MCS_STAMPS
                if (lane == 0 && (qa || qb)) atomicAdd(&g_dt_rows[4], (unsigned long long)(qa ? 1 : 0) + (qa && qb ? 1 : 0));
#endif
                if (qa) {
                    const uint32_t ka = n1 - ba < (uint32_t)kWave ? n1 - ba : (uint32_t)kWave;
                    quiet_row(ba, cma, jda, ala, wr);
                    if (qb) quiet_row(bb, cmb, jdb, alb, wr + ka);
                    wr += ka;
                    if (qb) wr += n1 - bb < (uint32_t)kWave ? n1 - bb : (uint32_t)kWave;
                    else if (has_b) ok_pass = row(bb, cmb, jdb, alb);
                } else {
                    ok_pass = row(ba, cma, jda, ala);
                    if (ok_pass && has_b) ok_pass = row(bb, cmb, jdb, alb);
                }
            }
        }
#ifdef MCS_STAMPS
        const uint64_t pt2 = wall_clock64();
#endif
        st.l1n = wr;
        {
            const unsigned long long s_sk = (unsigned long long)dt_wave_sum_i64((long long)sk_eff);
            st.total += 1000ll * ((long long)(n1 - n_skip) * (long long)T - (long long)(st.s_last - s_sk));
            st.s_last = (unsigned long long)(wr - n_skip) * T + s_sk;
        }
        st.t_all = T;  // every entry examined at T: its stamp is not rewritten (the skipped ones are marked)
        st.l1_dirty = wr != n1 ? 1u : 0u;  // a pass that placed: its skipped entries come next
        if (exact) {  // the jobs left failed every node as they are now
            snap_l = lane < NN ? nodes[lane] : 0ull;
            snap_dirty = true;
        }
#ifdef MCS_STAMPS
        if (lane == 0) {
            const uint64_t pt3 = wall_clock64();
            atomicAdd(&g_dt_rows[8], (unsigned long long)(pt1 - pt0));
            atomicAdd(&g_dt_rows[9], (unsigned long long)(pt2 - pt1));
            atomicAdd(&g_dt_rows[10], (unsigned long long)(pt3 - pt2));
            atomicAdd(&g_dt_rows[5], 1ull);
            atomicAdd(&g_dt_rows[7], (unsigned long long)(pt3 - pt0));
        }
#endif
    }

    DT_MARK(3);
    // ---- Level0 head (scheduler.go:332-366) ----
    if (!(st.flags & MCS_FLAG_OVERFLOW) && st.l0_head < st.next_arr) {
        const uint32_t j = st.l0_head;
        const uint4 jb = jobs[j];
        const uint32_t k = first_fit(jb.z, jb.w);
        // JobsMap: 0 until the head is first examined, then 1000 * (last - arrival)
        const long long old = st.head_last == kEmpty ? 0ll : (long long)(st.head_last - jb.x) * 1000ll;
        st.total += (long long)(T - jb.x) * 1000ll - old;
        st.head_last = T;
        if (k != kEmpty) {
            const uint32_t fin = T + jb.y;
            if (jb.y != 0u && !commit(k, jb.z, jb.w, fin)) {
                st.flags |= MCS_FLAG_OVERFLOW;
            } else {
                if (lane == 0) {
                    a.out_node[j0 + j] = (int32_t)k;
                    a.out_start[j0 + j] = T;
                    a.out_finish[j0 + j] = fin;
                }
                ++st.l0_head;
                ++st.decided;
                st.head_last = kEmpty;
            }
        } else if (T - jb.x >= a.max_wait) {  // MaxWaitTime (:353): Level1 append (:357)
            if (lane == 0) {
                l1cm[st.l1n] = (unsigned long long)jb.z | ((unsigned long long)jb.w << 32);
                l1jd[st.l1n] = (unsigned long long)j | ((unsigned long long)jb.y << 32);
                l1al[st.l1n] = (unsigned long long)jb.x | ((unsigned long long)T << 32);
            }
            ++st.l1n;
            st.s_last += T;
            ++st.l0_head;
            ++st.moved;
            if (exact) {  // it failed every node as they are now: the snapshot may not exceed them
                const unsigned long long cur = lane < NN ? nodes[lane] : 0ull;
                const uint32_t lo = (uint32_t)cur < (uint32_t)snap_l ? (uint32_t)cur : (uint32_t)snap_l;
                const uint32_t hi = (uint32_t)(cur >> 32) < (uint32_t)(snap_l >> 32) ? (uint32_t)(cur >> 32)
                                                                                     : (uint32_t)(snap_l >> 32);
                snap_l = (unsigned long long)lo | ((unsigned long long)hi << 32);
                snap_dirty = true;
            }
            st.head_last = kEmpty;
        }
    }
    return st;
}

// Phase C: the state stream sample (trader_server.go:24-47) every sample_period seconds, into st;
// dc, dm: NN floats each of scratch LDS
template <bool RES>
__device__ __forceinline__ void dt_sample(const DtArgs& a, const uint32_t c, const uint32_t lane, const uint32_t T,
                                          const uint32_t n0, const uint32_t N, const uint32_t NN,
                                          const unsigned long long* __restrict__ nodes, float* dc, float* dm,
                                          DtCluster& st) {
    if (T % a.sample_period == 0u) {
        dt_bar<RES>();  // (the scratch may be the slots' LDS, copied out)
        for (uint32_t i = lane; i < NN; i += kWave) {
            const unsigned long long v = nodes[i];
            const uint2 cp = i < N ? a.cap[n0 + i] : a.vcap[(size_t)c * a.V + (i - N)];
            // float32(node.Cores) - float32(node.CoresAvailable) (cluster.go:55-56), uint64 -> float32
            dc[i] = __fsub_rn((float)cp.x, go_f32((uint32_t)v));
            dm[i] = __fsub_rn((float)cp.y, go_f32((uint32_t)(v >> 32)));
        }
        dt_bar<RES>();
        if (lane == 0) {
            float sc = 0.0f, sm = 0.0f;
            for (uint32_t i = 0; i < NN; ++i) {  // node order, float32 like Go
                sc = __fadd_rn(sc, dc[i]);
                sm = __fadd_rn(sm, dm[i]);
            }
            st.cu = __fdiv_rn(sc, (float)st.total_c);
            st.mu = __fdiv_rn(sm, (float)st.total_m);
            // WaitTime.GetAverage (scheduler.go:56-63)
            st.avgw = st.count != 0 ? __ddiv_rn((double)st.total, (double)st.count) : 0.0;
        }
    }
}

// both contract sizes over GetLevel1() (ProvideJobs, trader_server.go:69-94) when this cluster's
// trader round is due: ln entries of l1cm / l1jd; hist: 64 words of scratch LDS
template <bool RES>
__device__ __forceinline__ void dt_contracts(const bool due, const uint32_t lane, const uint32_t ln,
                                             const unsigned long long* l1cm, const unsigned long long* l1jd,
                                             uint32_t* hist, uint32_t& fsc, uint32_t& fsm, uint32_t& fmd,
                                             uint32_t& ssc, uint32_t& ssm, uint32_t& sst) {
    if (due) {
        // Level1 rows were compacted by other lanes in this kernel: read them back through L2
        // (resident: this wave's stores complete first; every reader of them is on this CU)
        if constexpr (RES) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        dt_bar<RES>();
        // 8 rows of loads in flight per round (every lane loads, at an index clamped into the list;
        // a row at a time waited one L2 round trip per 64 entries)
        constexpr uint32_t kR = 8;
        for (uint32_t b = 0; b < ln; b += kR * kWave) {
            unsigned long long cmv[kR], jdv[kR];
#pragma unroll
            for (uint32_t u = 0; u < kR; ++u) {
                const uint32_t i = b + u * kWave + lane, pi = i < ln ? i : ln - 1u;
                cmv[u] = ld64(&l1cm[pi]);
                jdv[u] = ld64(&l1jd[pi]);
            }
#pragma unroll
            for (uint32_t u = 0; u < kR; ++u) {
                const bool in = b + u * kWave + lane < ln;
                const uint32_t jc = in ? (uint32_t)cmv[u] : 0u, jm = in ? (uint32_t)(cmv[u] >> 32) : 0u;
                const uint32_t d = in ? (uint32_t)(jdv[u] >> 32) : 0u;
                fsc += jc;  // fast node: uint32 sums and the longest duration (:138-155)
                fsm += jm;
                fmd = d > fmd ? d : fmd;
                ssc += (int32_t)(0u - jc) < 0 ? jc : 0u;  // small node: int32 arithmetic (:232-259)
                ssm += (int32_t)(0u - jm) < 0 ? jm : 0u;
            }
        }
        fsc = dt_wave_sum_u32(fsc);
        fsm = dt_wave_sum_u32(fsm);
        fmd = dt_wave_max_u32(fmd);
        ssc = dt_wave_sum_u32(ssc);
        ssm = dt_wave_sum_u32(ssm);
        // small node contract.Time per job: endTime if the previous time < endTime, else 0
        // (:263-265); a padded last batch (len % 20 != 0) ends with zero jobs -> 0.  The recurrence
        // s = s < d ? d : 0 from s = 0 leaves s = d_k exactly when the run of "falls" (d_(i-1) >= d_i)
        // ending at k is even (a non-fall takes d_i whatever s was; a fall takes it only after a 0),
        // so the answer is the last duration or 0 by the parity of the list's trailing run of falls,
        // read backwards a row at a time from the end (usually one row)
        if (ln % 20u == 0u && ln != 0u) {
            const uint32_t dl = (uint32_t)(ld64(&l1jd[ln - 1u]) >> 32);
            uint32_t run = 0;  // falls ending at the list's last entry
            for (uint32_t top = ln;;) {  // entries [top - 64, top) by lane (the row's last in lane 63)
                const uint32_t base = top > (uint32_t)kWave ? top - (uint32_t)kWave : 0u;
                const uint32_t k = base + lane;  // entry k: a fall when d_(k-1) >= d_k (k >= 1)
                const bool in = k < top;
                const uint32_t dk = (uint32_t)(ld64(&l1jd[in ? k : top - 1u]) >> 32);
                const uint32_t dp = k >= 1u && in ? (uint32_t)(ld64(&l1jd[k - 1u]) >> 32) : 0u;
                const bool fall = in && k >= 1u && dp >= dk;
                // the last non-fall in the row (entry 0 counts as one)
                const unsigned long long nf = __ballot(in && !fall);
                if (nf) {
                    run += top - 1u - (base + 63u - (uint32_t)__builtin_clzll(nf));
                    break;
                }
                run += top - base;
                top = base;
            }
            sst = (run & 1u) == 0u ? dl : 0u;
        }
    }
}

// Phase D's trader rounds of tick T in cluster order over the whole system, on the records of the
// tick (srec) and the replicated trader state (trs); appr, nvs, nfr: per-cluster scratch, virtual
// node and free slot counts (LDS).  The replayed form commits a local cluster's side effects to its
// live state; the resident form queues them (oq).
struct DtCounts {  // the logs' counters and the round flags, carried through the rounds
    unsigned long long n_trades, n_won, n_for;
    uint32_t lflags;
};
template <bool RES>
__device__ __forceinline__ DtCounts dt_rounds(const DtArgs& a, const uint32_t lane, const uint32_t T,
                                              const bool any_due, DtTrader* __restrict__ trs,
                                              const DtRec* __restrict__ srec, uint32_t* __restrict__ appr,
                                              uint32_t* __restrict__ nvs, uint32_t* __restrict__ nfr, DtCounts k,
                                              DtOpQueue oq) {
    const uint32_t Ct = a.Ct;
    unsigned long long n_trades = k.n_trades, n_won = k.n_won, n_for = k.n_for;
    uint32_t lflags = k.lflags;
    for (uint32_t q0 = 0; q0 < Ct && a.period && any_due; q0 += kWave) {
        const uint32_t ql = q0 + lane;
        unsigned long long due = __ballot(ql < Ct && trs[ql].next_due <= T);
        while (due) {
            const uint32_t q = q0 + (uint32_t)__builtin_ctzll(due);
            due &= due - 1ull;
            const DtRec* rq = &srec[q];
            const uint32_t ql_ = q - a.base;  // local index when q is on this rank
            const bool qloc = ql_ < a.C;
            // RequestPolicyMonitor of requester q (trader.go:282-324): two-stage machine
            while (trs[q].next_due <= T) {
#ifdef MCS_STAMPS
                const uint64_t rq0 = wall_clock64();
#endif
                DtTrader tq = trs[q];
                if (tq.stage == 0u) {  // cs := t.State.getState() (:284)
                    tq.cs_cu = rq->cu;
                    tq.cs_mu = rq->mu;
                    tq.cs_avgw = rq->avgw;
                }
                const uint32_t pol = tq.stage;
                const bool broken = pol == 0u ? (tq.cs_avgw > 600000.0)                     // :137-139
                                              : (tq.cs_cu > 0.8f || tq.cs_mu > 0.8f);       // :127-130
                tq.stage = pol == 0u ? 1u : 0u;
                if (!broken) {
                    if (pol == 1u) tq.next_due = T + a.period;  // time.Sleep(10 s) (:323)
                    dt_bar<RES>();
                    if (lane == 0) trs[q] = tq;
                    dt_bar<RES>();
#ifdef MCS_STAMPS
                    if (lane == 0) {
                        atomicAdd(&g_dt_rows[19], (unsigned long long)(wall_clock64() - rq0));
                        atomicAdd(&g_dt_rows[20], 1ull);
                    }
#endif
                    continue;
                }
                // calculateContractRequest over GetLevel1() (scheduler_client.go:126-289), sized
                // by the owner's step kernel after phase A: Level1 does not change in phase D
                const uint32_t kc = pol == 0u ? rq->fc : rq->sc;
                const uint32_t km = pol == 0u ? rq->fm : rq->sm;
                const uint32_t ksec = pol == 0u ? rq->ft : rq->st;
                // ---- Trade (trader.go:193-278): RequestResource to every other trader ----
                uint32_t napp = 0;
                for (uint32_t r0 = 0; r0 < Ct; r0 += kWave) {
                    const uint32_t r = r0 + lane;
                    bool app = false;
                    if (r < Ct && r != q) {
                        DtTrader t = trs[r];
                        if (t.lock_id != 0u && T >= t.lock_until) t.lock_id = 0u;  // 20 s expiry
                        if (t.lock_id == 0u) {  // else Approve:false (server.go:35-40)
                            const DtRec* rr = &srec[r];
                            app = approve_trade_dev(rr->total_c, rr->total_m, rr->cu, rr->mu, kc, km, ksec);
                            t.lock_id = t.next_id++;  // set even when not approving (:44-46)
                            t.lock_until = T + a.lock_s;
                        }
                        trs[r] = t;
                    }
                    const unsigned long long ab = __ballot(app);
                    if (app) {
                        const uint32_t at = napp + (uint32_t)__builtin_amdgcn_mbcnt_hi(
                                                       (uint32_t)(ab >> 32),
                                                       __builtin_amdgcn_mbcnt_lo((uint32_t)ab, 0u));
                        appr[at] = r;
                    }
                    napp += (uint32_t)__builtin_popcountll(ab);
                }
                dt_bar<RES>();
                // container/heap of equal prices (every response echoes the request's price,
                // server.go:44) pops pushes a0, a1, ..., a(n-1) as a0, a(n-1), ..., a1
                int32_t winner = -1;
                uint32_t failed = 0;
                for (uint32_t i = 0; i < napp && winner < 0; ++i) {
                    const uint32_t r = appr[i == 0u ? 0u : napp - i];
                    // ApproveContract (server.go:63-85): the lock set in this round still
                    // matches; AllocateVirtualNodeResources on the responder (cluster.go:87-125)
                    uint32_t rc_ = kc, rm_ = km;
                    const uint32_t rN = srec[r].N;
                    const uint32_t rNN = rN + nvs[r];
                    unsigned long long* rs = dt_snap(a, r);
                    const uint32_t rl = r - a.base;  // local index when r is on this rank
                    const bool rloc = rl < a.C;
                    bool ovf = false;
                    for (uint32_t nd = 0; nd < rNN; ++nd) {
                        if (rm_ == 0u && rc_ == 0u) break;  // :90-92
                        unsigned long long* sp = nd < rN ? &rs[nd] : &rs[a.NS + (nd - rN)];
                        const unsigned long long v = ld64(sp);
                        double mem_diff = 0.0, core_diff = 0.0;
                        if (rm_ > 0u) mem_diff = fabs(__dsub_rn((double)rm_, go_f64((uint32_t)(v >> 32))));
                        if (rc_ > 0u) core_diff = fabs(__dsub_rn((double)rc_, go_f64((uint32_t)v)));
                        if (mem_diff > (double)rm_)
                            rm_ = 0u;
                        else
                            rm_ -= (uint32_t)mem_diff;
                        if (core_diff > (double)rc_)
                            rc_ = 0u;
                        else
                            rc_ -= (uint32_t)core_diff;
                        const unsigned long long fc = go_f64_to_u64(core_diff), fm = go_f64_to_u64(mem_diff);
                        if (lane == 0) {
                            if (n_for < a.foreign_cap) {
                                mcs_foreign_rec fr;
                                fr.requester = q;
                                fr.responder = r;
                                fr.node = nd;
                                fr.start_s = T;
                                fr.finish_s = T + ksec;
                                fr.pad = 0u;
                                fr.c = fc;
                                fr.m = fm;
                                a.foreign_log[n_for] = fr;
                            } else {
                                lflags |= MCS_FLAG_LOG_OVERFLOW;
                            }
                        }
                        ++n_for;
                        if (ksec == 0u) continue;  // RunJob sleeps 0: commit and release at once
                        // go node.RunJob(Foreign) (:116): commit now, release at T + time.  The
                        // free-slot count is replicated, so every rank sees the same overflow.
                        if (nfr[r] == 0u) {
                            ovf = true;
                            break;
                        }
                        const unsigned long long nv_ = (unsigned long long)((uint32_t)v - (uint32_t)fc) |
                                                       ((unsigned long long)((uint32_t)(v >> 32) - (uint32_t)fm) << 32);
                        if (lane == 0) {
                            __hip_atomic_store(sp, nv_, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            nfr[r] -= 1u;
                        }
                        if constexpr (RES) {  // the owner wave applies it after the tick (dt_apply_ops)
                            if (lane == 0)
                                oq.push(r, DtOp{1u, nd, (uint32_t)nv_, (uint32_t)(nv_ >> 32), T + ksec, (uint32_t)fc,
                                                (uint32_t)fm, 0u});
                        } else if (rloc) {  // the owner: live node counter and a running slot
                            uint32_t slot = kEmpty;
                            const size_t rsb = (size_t)rl * a.S;
                            for (uint32_t b = 0; b < a.S; b += kWave) {
                                const unsigned long long fr = __ballot(ld32(&a.sfin[rsb + b + lane]) == kEmpty);
                                if (fr) {
                                    slot = b + (uint32_t)__builtin_ctzll(fr);
                                    break;
                                }
                            }
                            if (lane == 0 && slot != kEmpty) {
                                unsigned long long* np_ = nd < rN ? &a.tn[a.node_off[rl] + nd]
                                                                  : &a.vn[(size_t)rl * a.V + (nd - rN)];
                                __hip_atomic_store(np_, nv_, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                __hip_atomic_store(&a.sfin[rsb + slot], T + ksec, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
                                a.snode[rsb + slot] = nd;
                                a.scm[rsb + slot] = (unsigned long long)(uint32_t)fc |
                                                    ((unsigned long long)(uint32_t)fm << 32);
                                atomicAdd(&a.cl[rl].nrun, 1u);  // atomics: never read back in here
                                atomicMin(&a.cl[rl].minf, T + ksec);
                                atomicOr(&a.cl[rl].l1_dirty, 1u);  // the commit may wrap a counter
                            }
                        }
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                        dt_bar<RES>();
                    }
                    if (ovf) {
                        lflags |= MCS_FLAG_OVERFLOW;
                        break;
                    }
                    if (lane == 0) trs[r].lock_id = 0u;  // currentContract reset (:83)
                    dt_bar<RES>();
                    if (rc_ > 0u || rm_ > 0u) {  // "couldn't schedule enough resources" (:119-121)
                        ++failed;
                        continue;
                    }
                    winner = (int32_t)r;
                    // AddVirtualNode on the requester (cluster.go:65-85)
                    if (lane == 0) {
                        const uint32_t nv = nvs[q];
                        const unsigned long long cap = (unsigned long long)kc | ((unsigned long long)km << 32);
                        if (nv < a.V) {
                            __hip_atomic_store(&dt_snap(a, q)[a.NS + nv], cap, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
                            nvs[q] = nv + 1u;
                            if constexpr (RES) {
                                oq.push(q, DtOp{2u, nv, kc, km, 0u, 0u, 0u, 0u});
                            } else if (qloc) {
                                __hip_atomic_store(&a.vn[(size_t)ql_ * a.V + nv], cap, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
                                a.vcap[(size_t)ql_ * a.V + nv] = make_uint2(kc, km);
                                atomicAdd(&a.cl[ql_].nv, 1u);
                                atomicOr(&a.cl[ql_].l1_dirty, 1u);
                            }
                        } else {
                            lflags |= MCS_FLAG_VNODE_OVERFLOW;
                            if constexpr (RES) oq.push(q, DtOp{3u, 0u, 0u, 0u, 0u, 0u, 0u, 0u});
                            else if (qloc) atomicOr(&a.cl[ql_].flags, (uint32_t)MCS_FLAG_VNODE_OVERFLOW);
                        }
                    }
                    dt_bar<RES>();
                }
                if (lane == 0) {
                    if (winner >= 0) ++n_won;
                    if (n_trades < a.trade_cap) {
                        mcs_contract_rec rec;
                        rec.t_s = T;
                        rec.requester = q;
                        rec.winner = winner;
                        rec.approvals = napp;
                        rec.policy = pol;
                        rec.cores = kc;
                        rec.mem = km;
                        rec.time_s = ksec;
                        rec.failed = failed;
                        rec.pad = 0u;
                        a.trade_log[n_trades] = rec;
                    } else {
                        lflags |= MCS_FLAG_LOG_OVERFLOW;
                    }
                    tq.next_due = T + (winner >= 0 ? a.ok_sleep : a.fail_sleep) + (pol == 1u ? a.period : 0u);
                    tq.lock_id = trs[q].lock_id;  // q's own lock may have been set as a responder
                    tq.lock_until = trs[q].lock_until;
                    tq.next_id = trs[q].next_id;
                    trs[q] = tq;
                }
                ++n_trades;
                dt_bar<RES>();
#ifdef MCS_STAMPS
                if (lane == 0) {
                    atomicAdd(&g_dt_rows[17], (unsigned long long)(wall_clock64() - rq0));
                    atomicAdd(&g_dt_rows[18], 1ull);
                }
#endif
                if (lflags & MCS_FLAG_OVERFLOW) break;
            }
            if (lflags & MCS_FLAG_OVERFLOW) break;
        }
        if (lflags & MCS_FLAG_OVERFLOW) break;
    }
    return DtCounts{n_trades, n_won, n_for, lflags};
}

// the next tick: T+1 while any cluster has a queued job, else the next arrival, sample tick or
// trader round (oracle/mcs_oracle_dtrade.c); the control block that follows tick T
__device__ __forceinline__ DtCtl dt_next_ctl(const DtArgs& a, const uint32_t lane, const DtCtl& c0,
                                             const DtTrader* trs, const DtRec* srec, const uint32_t lflags,
                                             const unsigned long long n_trades, const unsigned long long n_won,
                                             const unsigned long long n_for) {
    const uint32_t T = c0.T, Ct = a.Ct;
    bool all_done = true, queued = false;
    uint32_t nxt = T + a.sample_period - T % a.sample_period, fl = 0, ndue = kEmpty;
    for (uint32_t q = lane; q < Ct; q += kWave) {
        const DtRec* rq = &srec[q];
        all_done = all_done && rq->done != 0u;
        queued = queued || rq->queued != 0u;
        nxt = rq->nxt < nxt ? rq->nxt : nxt;
        if (a.period) ndue = trs[q].next_due < ndue ? trs[q].next_due : ndue;
        fl |= rq->flags;
    }
    const bool done_all = !__ballot(!all_done);
    const bool queued_any = __ballot(queued) != 0ull;
    ndue = wave_min_u32(ndue);
    nxt = wave_min_u32(nxt);
    nxt = ndue < nxt ? ndue : nxt;
    fl = readlane(wave_scan_or_u32(fl), 63u);
    DtCtl n = c0;
    uint32_t flags = c0.flags | fl | lflags;
    uint32_t done = 0, Tn = T;
    if (done_all || (flags & MCS_FLAG_OVERFLOW)) {
        done = 1u;
    } else if (T >= a.t_max) {
        done = 1u;
        flags |= MCS_FLAG_T_MAX;
    } else {
        Tn = (queued_any || nxt <= T + 1u) ? T + 1u : nxt;
    }
    n.T = Tn;
    n.done = done;
    n.any_due = ndue <= Tn ? 1u : 0u;
    n.ticks = c0.ticks + 1u;
    n.flags = flags;
    n.n_trades = n_trades;
    n.n_won = n_won;
    n.n_foreign = n_for;
    return n;
}

}  // namespace
}  // namespace mcs
