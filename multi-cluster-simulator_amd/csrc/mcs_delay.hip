// mcs_delay.hip — gfx950 kernel of the DELAY policy (Scheduler.Delay, pkg/scheduler/scheduler.go:
// 298-369, the reference's shipped default, scheduler.go:116) for one cluster per wave64
// workgroup, under the serialized semantics SDELAY (oracle/mcs_oracle_delay.c).
//
// One Delay iteration at time t (every iteration ends in time.Sleep(1 s), :367):
//   * releases due at t (cluster.go:153-157) — the same wave-parallel slot scan as fifo_kernel;
//   * the Level1 pass (:302-329): every Level1 job in list order gets ScheduleJob; a placed job is
//     removed with append(Level1[:i], Level1[i+1:]...) and no i--, so the job sliding into slot i
//     is skipped this pass (D6, replicated);
//   * the Level0 head (:332-366): ScheduleJob; on failure it moves to the Level1 tail once it has
//     waited MaxWaitTime (10 s, :353).
//
// Layout and the MI355X choices:
//   * node free vectors, running slots and releases are fifo_kernel's (LDS packed u64 nodes,
//     first fit = per-lane select + DPP wave minimum, commit = one ds_sub_u64);
//   * Level0 is a cursor h into the arrival-sorted SoA stream (jobs leave Level0 in stream order,
//     either placed or moved), streamed 64 records at a time like fifo_kernel's ready queue, or
//     synthesised in registers with fused generation (GEN, mcs_gen_dev.h);
//   * Level1 is a dense list in HBM scratch (capacity = the cluster's job count, so it never
//     overflows): {cores | mem << 32} and {job | dur << 32}, 16 B per entry.  A pass reads it 64
//     entries per coalesced load (sc1: served by L2, never a stale L1 line of this CU) and
//     compacts it in the same sweep, so removals cost no extra pass;
//   * a per-lane fit filter rejects every Level1 entry that fits no node without a first fit:
//     lane l holds best[l] = max free memory over nodes with min(free cores, 63) >= l (an LDS
//     ds_max_u32 histogram + a wave suffix max), so job (c, m) can fit iff c <= max free cores and
//     best[min(c, 63)] >= m (exact for c < 63, conservative above).  Clusters of > 128 nodes
//     build it in 256 B borrowed from the running-slot rows (fifo_kernel's 10 KB of LDS per wave,
//     16 waves per CU); the filter is rebuilt only after a commit or a release (r03: the
//     per-resource maxima it replaced let ~88 first fits through per placement on a Level1-heavy
//     stream).  Resources only shrink inside a pass, so a job rejected at the start of the pass
//     stays rejected; the survivors get a real first fit in list order;
//   * Level0 results leave in 64-job register batches (masked: moved jobs are written when Level1
//     places them); Level1 results are three single-lane stores.
// Fast-forward: after an iteration that placed and moved nothing, the next iteration that can
// change anything is the next release, the Level0 head's MaxWaitTime move, or (empty Level0) the
// next arrival — the skipped iterations repeat the same failures (exact, oracle-tested).
#define MCS_GEN_FN __host__ __device__ static inline
#include "mcs_gen_dev.h"
#include "mcs_internal.h"
#include "mcs_lds.h"
#include "mcs_wave.h"

namespace mcs {

// unsigned max over the wave (DPP row shifts + row broadcasts, identity 0), see wave_min_u32
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#define MCS_DPP_MAX(CTRL, RM)                                                                      \
    {                                                                                              \
        const uint32_t w = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, RM, 0xf, false); \
        v = w > v ? w : v;                                                                         \
    }
    MCS_DPP_MAX(0x111, 0xf)
    MCS_DPP_MAX(0x112, 0xf)
    MCS_DPP_MAX(0x114, 0xf)
    MCS_DPP_MAX(0x118, 0xf)
    MCS_DPP_MAX(0x142, 0xa)
    MCS_DPP_MAX(0x143, 0xc)
#undef MCS_DPP_MAX
    return readlane(v, 63);
}

// inclusive prefix max over the wave (lane i: max of lanes 0..i), the DPP steps of wave_max_u32
__device__ __forceinline__ uint32_t wave_prefix_max_u32(uint32_t v) {
#define MCS_DPP_MAX(CTRL, RM)                                                                      \
    {                                                                                              \
        const uint32_t w = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, RM, 0xf, false); \
        v = w > v ? w : v;                                                                         \
    }
    MCS_DPP_MAX(0x111, 0xf)
    MCS_DPP_MAX(0x112, 0xf)
    MCS_DPP_MAX(0x114, 0xf)
    MCS_DPP_MAX(0x118, 0xf)
    MCS_DPP_MAX(0x142, 0xa)
    MCS_DPP_MAX(0x143, 0xc)
#undef MCS_DPP_MAX
    return v;
}

// HBM scratch of the Level1 list, read by the wave that wrote it: bypass this CU's vector L1.
__device__ __forceinline__ uint64_t ld_l2(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// HOR: the online variant, as fifo_kernel's: resume from the previous horizon's
// OnlineState / node image / slot image (Level1 stays in its HBM list), run every iteration at
// t < a.on.t_hor, save.  A cluster with nothing queued parks without advancing its clock (the
// iteration is idempotent when re-run); only a drain (t_hor = kEmpty) ends a run the way the
// one-shot kernel does.
// online sessions: the run's final iteration (t + 1 after the last placement) has been taken; kept
// in the saved state's flags only (a drain must take it once, whichever horizon placed the job)
constexpr uint32_t kOnEnded = 0x80000000u;

template <int NPL, int P, bool GEN, bool HOR>
__global__ __launch_bounds__(64) void delay_kernel(DelayArgs a) {
    static_assert(P <= 32, "free-row mask is one u32 per lane");
    static_assert(!(HOR && GEN), "online runs stream records");
    constexpr bool kHist = NPL <= 2;  // exact Level1 fit histogram (256 B of LDS)
    const uint32_t item = blockIdx.x;
    const uint32_t ci = a.cluster_list ? a.cluster_list[item] : item;
    const uint32_t lane = threadIdx.x;

    __shared__ uint64_t nodes[NPL * kWave];
    __shared__ uint64_t pay[2 * P * kWave];  // running slots: {cores|mem} rows, then {node|finish}
    uint64_t* const pay_cm = pay;
    uint64_t* const pay_nf = pay + P * kWave;

    // ---- cluster spec: Run() keeps the JSON availability (scheduler.go:101-109) ----
    const uint32_t n0 = a.node_off[ci];
    const uint32_t N = a.node_off[ci + 1] - n0;
    uint32_t nid[NPL];
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
        const uint32_t idx = k * kWave + lane;
        uint2 v = make_uint2(0u, 0u);
        if (idx < N) v = a.node_free0[n0 + idx];
        nodes[idx] = (uint64_t)v.x | ((uint64_t)v.y << 32);
        nid[k] = idx < N ? idx : kEmpty;
    }

    const uint64_t j0 = a.job_off[ci];
    const uint32_t J = HOR ? a.on.job_cnt[ci] : (uint32_t)(a.job_off[ci + 1] - j0);
    const uint4* __restrict__ jobs = GEN ? nullptr : a.jobs + j0;
    int32_t* __restrict__ o_node = a.out_node + j0;
    uint32_t* __restrict__ o_start = a.out_start + j0;
    uint32_t* __restrict__ o_finish = a.out_finish + j0;
    uint64_t* l1_cm = a.l1_cm + j0;  // Level1 entries: {cores | mem << 32}
    uint64_t* l1_jd = a.l1_jd + j0;  //                  {job | dur << 32}
    const uint32_t max_wait = a.max_wait_s;

    uint32_t frm = (P == 32) ? 0xFFFFFFFFu : ((1u << (P & 31)) - 1u);
    uint32_t lmin = kEmpty;
#pragma unroll
    for (int p = 0; p < P; ++p) pay_nf[p * kWave + lane] = (uint64_t)kEmpty << 32;

    // Level0 batches: streamed from HBM, or synthesised in registers (GEN, mcs_gen_dev.h)
    GenStream gs;
    if constexpr (GEN) gs.init(a.gen, ci, lane);
    auto load_batch = [&](uint32_t base) __attribute__((always_inline)) -> uint4 {
        if constexpr (GEN)
            return gs.next(base, lane);
        else
            return jobs[base + lane];
    };
    uint32_t t = 0, h = 0, l1n = 0, minf = kEmpty, flags = 0;
    // Counters and the WaitTime sums live in VGPRs (the asm hides their uniformity): the CU's scalar
    // unit is the scarcer issue resource (fifo_kernel's measurements).
    uint32_t used = 0, peak = 0, placed = 0, moved = 0, placed_l1 = 0, peak_l1 = 0;
    uint32_t n_iter = 0, n_rel = 0;
    // WaitTime.TotalTime / 1000 = sum over placed jobs of (start - arrival) [+ left jobs]:
    //   wacc  per lane: Level0 placements of that lane's batch slots, added at each batch flush;
    //   l1_t  t of every Level1 placement;  mv_a  arrival of every job moved to Level1
    uint64_t wacc = 0, l1_t = 0, mv_a = 0;
    uint32_t ovf = 0u;  // a finish time left the u32 clock range (recorded in VALU)
    bool live = true;
    // the Level1 fit filter (lane l: best[l]) and the largest free core count, valid until a
    // commit or a release (hdirty)
    uint32_t best = 0u;
    bool hdirty = true;
    // lmv (lane i, as best): a lower bound of the smallest memory demand among the Level1 jobs of
    // core key 63 - i (~0u: none).  A pass that cannot place anything (best < lmv in every lane)
    // is skipped whole: it would only have re-read the list (its JobsMap updates are closed-form)
    uint32_t lmv = ~0u;
    if constexpr (HOR) {  // resume from the previous horizon
        const OnlineState st = a.on.st_in[ci];
        if (st.valid) {
            const unsigned long long* img = a.on.img_in + (size_t)ci * a.on.img_stride;
#pragma unroll
            for (int k = 0; k < NPL; ++k) nodes[k * kWave + lane] = img[k * kWave + lane];
            const unsigned long long* sl = a.on.slot_in + (size_t)ci * kSlotImg;
#pragma unroll
            for (int p = 0; p < P; ++p) {
                if ((uint32_t)p < st.pool) {
                    const uint64_t nf = sl[(kMaxPool + p) * kWave + lane];
                    pay_cm[p * kWave + lane] = sl[p * kWave + lane];
                    pay_nf[p * kWave + lane] = nf;
                    const uint32_t f = (uint32_t)(nf >> 32);
                    if (f != kEmpty) {
                        frm &= ~(1u << p);
                        lmin = f < lmin ? f : lmin;
                    }
                }
            }
            minf = wave_min_u32(lmin);
            t = st.t;
            h = st.cursor;
            l1n = st.aux;
            // a drained deadlock is not final online: later arrivals still reach Level0
            flags = st.flags & ~MCS_FLAG_DEADLOCK;
            placed = st.placed;
            moved = st.waited;
            peak = st.peak;
            used = st.used;
            n_iter = st.n_iter;
            n_rel = st.n_rel;
            placed_l1 = st.placed_l1;
            peak_l1 = st.peak_l1;
            l1_t = st.l1_t;
            mv_a = st.mv_a;
            if (lane == 0) wacc = st.wsum;
        }
        // nothing to do: a clock overflow is final, the horizon may be reached, and a cluster
        // with nothing queued keeps its clock — except that a drain ends a run whose last job was
        // placed in an earlier (non-drain) horizon with the batch run's final iteration (t + 1,
        // below), once (kOnEnded in the saved flags)
        if ((flags & kOnEnded) && h < J) {  // jobs appended after that: the run had not ended
            t = t - 1u;
            flags &= ~kOnEnded;
        }
        live = !(flags & MCS_FLAG_CLOCK_OVERFLOW) && t < a.on.t_hor && (h < J || l1n != 0u);
        if (st.valid && !live && a.on.t_hor == kEmpty && h >= J && l1n == 0u &&
            !(flags & (kOnEnded | MCS_FLAG_CLOCK_OVERFLOW))) {
            t = t + 1u;
            flags |= kOnEnded;
        }
    }
    asm volatile("" : "+v"(used), "+v"(peak), "+v"(n_iter), "+v"(n_rel), "+v"(placed), "+v"(moved),
                 "+v"(placed_l1), "+v"(peak_l1), "+v"(l1_t), "+v"(mv_a), "+v"(ovf));

    const uint32_t cb0 = HOR ? (h & ~63u) : 0u;
    uint32_t cb = cb0;
    uint4 cur = load_batch(cb0);
    // wait for the first batch here, so the only load pending at the pass loop's entry is the
    // prefetch, which the loop never reads (no flush of it at every pass; fifo_kernel v18)
    asm volatile("" ::"v"(cur.x), "v"(cur.y), "v"(cur.z), "v"(cur.w));
    uint4 nxt = make_uint4(0u, 0u, 0u, 0u);
    // Level0 result batch: lane (job & 63) holds its record; ov = written by Level0
    int32_t on = -1;
    uint32_t os = kEmpty, of = kEmpty, ov = 0u;

    // release every running job with finish <= t (cluster.go:153-157), row by row as in
    // fifo_kernel: row p's expired test over all lanes is one compare whose lane mask drives the
    // payload hand-back of that row and its free-row bits
    // LDS byte addresses (single-address b64 accesses: mcs_lds.h)
    const uint32_t pay_lds = lds_addr(pay);
    auto release = [&]() __attribute__((always_inline)) {
        ++n_rel;
        uint32_t lm = kEmpty;
        uint64_t nf[P];
        bool ex[P];
        read_finish_rows<P>(nf, pay_lds + lane * 8u + P * kWave * 8u);
#pragma unroll
        for (int p = 0; p < P; ++p) {  // free rows hold kEmpty: never expired, min-neutral
            const uint32_t f = (uint32_t)(nf[p] >> 32);
            ex[p] = f <= t;
            const uint32_t fl = ex[p] ? kEmpty : f;
            lm = fl < lm ? fl : lm;
        }
        lmin = lm;
        uint32_t nexp = 0u;
#pragma unroll
        for (int p = 0; p < P; ++p) {
            const uint64_t m = __ballot(ex[p]);
            if (m) {
                nexp += (uint32_t)__builtin_popcountll(m);
                if (ex[p]) {
                    atomicAdd((unsigned long long*)&nodes[(uint32_t)nf[p]],
                              (unsigned long long)pay_cm[p * kWave + lane]);
                    reinterpret_cast<uint32_t*>(pay_nf)[2 * (p * kWave + lane) + 1] = kEmpty;
                    frm |= 1u << p;
                }
            }
        }
        used -= nexp;
        minf = wave_min_u32(lmin);
        hdirty = true;
    };

    // ScheduleJob (scheduler.go:127-139): lowest node index with both >=
    auto first_fit = [&](uint32_t jc, uint32_t jm) __attribute__((always_inline)) -> uint32_t {
        asm volatile("" ::: "memory");  // another lane may have committed since the last read
        uint32_t best = kEmpty;
#pragma unroll
        for (int k = NPL - 1; k >= 0; --k) {
            const uint64_t v = nodes[k * kWave + lane];
            // descending chunks: a fit replaces best (padding chunks sit above every real one)
            best = ((uint32_t)v >= jc && (uint32_t)(v >> 32) >= jm) ? nid[k] : best;
        }
        return wave_min_u32(best);
    };

    // Node.RunJob commit (cluster.go:144-148, synchronous D2) and the running slot; returns false
    // on slot-pool overflow.  A zero-duration job is committed and released before the next
    // ScheduleJob can read the node, so it changes nothing.
    auto commit = [&](uint32_t k, uint32_t jc, uint32_t jm, uint32_t fin, uint32_t jd)
        __attribute__((always_inline)) -> bool {
        if (jd == 0u) return true;
        const uint64_t need = (uint64_t)jc | ((uint64_t)jm << 32);
        const uint64_t any = __ballot(frm != 0u);
        if (!any) return false;  // pool overflow: the run stops and the cluster is re-run
        hdirty = true;
        if (lane == (uint32_t)__builtin_ctzll(any)) {  // the slot's lane also commits the node
            __hip_atomic_fetch_sub(&nodes[k], need, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const uint32_t ad = (uint32_t)__builtin_ctz(frm) * kWave + lane;
            frm &= frm - 1u;
            // two single-address writes (LLVM pairs them into one write2st64, 2x the LDS time)
            const uint64_t nfw = (uint64_t)k | ((uint64_t)fin << 32);
            asm volatile("ds_write_b64 %0, %1\n\tds_write_b64 %0, %2 offset:%3"
                         :: "v"(pay_lds + ad * 8u), "v"(need), "v"(nfw), "i"(P * kWave * 8) : "memory");
            lmin = fin < lmin ? fin : lmin;
        }
        ++used;
        peak = used > peak ? used : peak;
        minf = fin < minf ? fin : minf;
        return true;
    };

    // the Level1 fit filter (scheduler.go:305, ScheduleJob's outcome without its node): lane i
    // holds best[63 - i] = max free memory over nodes with min(free cores, 63) >= 63 - i, so job
    // (c, m) fits some node iff best[min(c, 63)] >= m (exact for c < 63 and m > 0; a job without
    // memory demand passes whenever it cannot be told apart, and its first fit decides).  An LDS
    // ds_max_u32 histogram over the reversed core keys, then a DPP inclusive prefix max.  Clusters
    // of <= 128 nodes own 256 B of LDS for it; bigger ones keep fifo_kernel's 10 KB per wave (16
    // waves per CU) and borrow the first 256 B of the running slots' {node | finish} rows: each
    // lane saves its own word and puts it back (the wave is the workgroup, nothing reads them in
    // between)
    auto build_filter = [&]() __attribute__((always_inline)) {
        hdirty = false;
        asm volatile("" ::: "memory");  // other lanes' commits and releases since
        uint32_t* hist;
        if constexpr (kHist) {
            __shared__ uint32_t hist_own[kWave];
            hist = hist_own;
        } else {
            hist = reinterpret_cast<uint32_t*>(pay_nf);
        }
        const uint32_t haddr = lds_addr(hist) + lane * 4u;
        uint32_t saved = 0u;
        if constexpr (!kHist)
            asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(saved) : "v"(haddr) : "memory");
        asm volatile("ds_write_b32 %0, %1" ::"v"(haddr), "v"(0u) : "memory");
#pragma unroll
        for (int k = 0; k < NPL; ++k) {
            const uint64_t v = nodes[k * kWave + lane];
            const uint32_t fc = (uint32_t)v;
            if (nid[k] != kEmpty) atomicMax(&hist[63u - (fc < 63u ? fc : 63u)], (uint32_t)(v >> 32));
        }
        // the histogram is written by other lanes: without a fence the compiler may forward this
        // lane's own 0 store to the load below (it reasons per thread)
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
        uint32_t v;
        asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(haddr) : "memory");
        if constexpr (!kHist) asm volatile("ds_write_b32 %0, %1" ::"v"(haddr), "v"(saved) : "memory");
        best = wave_prefix_max_u32(v);
    };

    // Level1 rows in flight: a pass reads rows 0.. kPf - 1 from these registers, loaded at the end of
    // the iteration before (one L2 round trip per pass instead of one per row; the pass was bound
    // by them: 57 % of the wave's time waiting on a Level1-heavy stream)
    constexpr int kPf = 4;
    uint64_t pf_cm[kPf], pf_jd[kPf];
    auto prefetch_l1 = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int r = 0; r < kPf; ++r) {
            const uint32_t q = (uint32_t)r * kWave + lane;
            const bool ql = q < l1n;
            pf_cm[r] = ql ? ld_l2(l1_cm + q) : 0ull;
            pf_jd[r] = ql ? ld_l2(l1_jd + q) : 0ull;
        }
    };

    // writes the Level0 results of batch [base, base + 64); `cur` holds that batch's records
    auto flush = [&](uint32_t base) __attribute__((always_inline)) {
        const uint32_t i = base + lane;
        if (ov && i < J) {
            __builtin_nontemporal_store(on, o_node + i);
            __builtin_nontemporal_store(os, o_start + i);
            __builtin_nontemporal_store(of, o_finish + i);
            wacc += (uint64_t)(os - cur.x);
        }
        ov = 0u;
    };

    // Outer loop: one 64-record Level0 batch (records in `cur`); inner loop: the passes whose head
    // h is in it.  rend bounds h: the batch end, or 0 once the run stops.  A batch's results are
    // stored at the next batch boundary, after the wait for the prefetched records.
    uint32_t stop = 0u, rend = 0u;
    if (l1n != 0u) {  // (online resume)
        lmv = 0u;       // nothing known about the resumed list
        prefetch_l1();
    }
    if (live && (HOR || J != 0u)) for (;;) {
    if (cb != cb0) {
        const uint4 nb = nxt;  // waits for the prefetch, issued a whole batch ago
        flush(cb - kWave);     // the previous batch (all 64 decided), with its arrivals in cur
        cur = nb;
    }
    nxt = load_batch(cb + kWave);
    rend = cb + kWave;
    do {
        ++n_iter;
        uint32_t changed = 0u, l1w = 0u;

        // ---- Level1 pass (scheduler.go:302-329) ----
        if (l1n != 0u) {
            // the fit filter (build_filter) is rebuilt when a commit or a release changed the
            // nodes since the last build, and after every placement of the pass
            if (hdirty) build_filter();

            uint32_t wr = 0u, skip = kEmpty, dfold = ~0u;
            const bool any = __ballot(best >= lmv) != 0ull;
            for (uint32_t base = 0; any && base < l1n && !stop; base += kWave) {
                const uint32_t pos = base + lane;
                const bool live = pos < l1n;
                // the row was loaded kPf rows ahead (the first kPf at the previous iteration's
                // end): rotate the window and issue row + kPf
                const uint64_t cm = pf_cm[0], jdv = pf_jd[0];
#pragma unroll
                for (int r = 0; r + 1 < kPf; ++r) {
                    pf_cm[r] = pf_cm[r + 1];
                    pf_jd[r] = pf_jd[r + 1];
                }
                {
                    const uint32_t q = pos + kPf * kWave;
                    const bool ql = q < l1n;
                    pf_cm[kPf - 1] = ql ? ld_l2(l1_cm + q) : 0ull;
                    pf_jd[kPf - 1] = ql ? ld_l2(l1_jd + q) : 0ull;
                }
                const uint32_t c = (uint32_t)cm, m = (uint32_t)(cm >> 32);
                const uint32_t key = 63u - (c < 63u ? c : 63u);
                // the lookup outside the && (a ds_bpermute under a partial exec mask reads 0 from
                // the disabled lanes that hold the filter)
                uint32_t bm = (uint32_t)__shfl((int)best, (int)key);
                uint64_t cand = __ballot(live && bm >= m);
                uint64_t rem = 0ull;
                while (cand) {
                    const uint32_t b = (uint32_t)__builtin_ctzll(cand);
                    cand &= cand - 1ull;
                    if (base + b == skip) {  // slid into slot i: not examined (D6)
                        const uint32_t sk = readlane(key, b), sm = readlane(m, b);
                        dfold = (lane == sk && sm < dfold) ? sm : dfold;
                        continue;
                    }
                    const uint32_t jc = readlane(c, b), jm = readlane(m, b);
                    const uint32_t k = first_fit(jc, jm);
                    if (k == kEmpty) continue;
                    const uint32_t jw = readlane((uint32_t)jdv, b);
                    const uint32_t jd = readlane((uint32_t)(jdv >> 32), b);
                    const uint32_t fin = t + jd;
                    if constexpr (HOR) ovf |= (fin + 1u <= t) ? 1u : 0u;  // D8 guard, online variant only
                    if (!commit(k, jc, jm, fin, jd)) {
                        flags |= MCS_FLAG_OVERFLOW;
                        stop = 1u;
                        break;
                    }
                    if (lane == 0u) {
                        o_node[jw] = (int32_t)k;
                        o_start[jw] = t;
                        o_finish[jw] = fin;
                    }
                    rem |= 1ull << b;
                    skip = base + b + 1u;
                    // the commit shrank node k: the rest of this row is re-tested on the rebuilt
                    // filter (the stale one let every entry that only fitted k's old room through
                    // to a failing first fit: ~29 per placement on a Level1-heavy stream)
                    build_filter();
                    bm = (uint32_t)__shfl((int)best, (int)key);
                    cand &= __ballot(live && bm >= m);
                    ++placed;
                    ++placed_l1;
                    l1_t += t;
                    changed = 1u;
                }
                // compaction in the same sweep: survivors move down to the write cursor
                const uint64_t kept = __ballot(live) & ~rem;
                if ((wr != base || rem != 0ull) && live && !((rem >> lane) & 1ull)) {
                    const uint32_t np = wr + (uint32_t)__builtin_amdgcn_mbcnt_hi(
                                                 (uint32_t)(kept >> 32),
                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)kept, 0u));
                    if (np != pos) {
                        l1_cm[np] = cm;
                        l1_jd[np] = jdv;
                    }
                }
                l1w |= (wr != base || rem != 0ull) ? 1u : 0u;
                wr += (uint32_t)__builtin_popcountll(kept);
            }
            if (any && !stop) {
                l1n = wr;
                // every job left was tested on a filter no smaller than the final one and failed
                // (exact below key 63 where some node has memory), except the D6-skipped ones
                const uint32_t raised = best + 1u;
                if (lane != 0u && best != 0u && raised != 0u) lmv = raised > lmv ? raised : lmv;
                lmv = dfold < lmv ? dfold : lmv;
            }
        }

        // ---- Level0 head (scheduler.go:332-366) ----
        // (unmasked batch loads: the job array has kJobPad records of slack)
        const uint32_t l = (h - cb) & 63u;
        const uint32_t arr = readlane(cur.x, l);
        if (!stop && h < J && arr <= t) {  // Level0 is non-empty: its head has arrived
            const uint32_t jd = readlane(cur.y, l);
            const uint32_t jc = readlane(cur.z, l);
            const uint32_t jm = readlane(cur.w, l);
            const uint32_t k = first_fit(jc, jm);
            const uint32_t ol = h & 63u;
            if (k != kEmpty) {
                const uint32_t fin = t + jd;
                if constexpr (HOR) ovf |= (fin + 1u <= t) ? 1u : 0u;  // D8 guard, online variant only
                if (!commit(k, jc, jm, fin, jd)) {
                    flags |= MCS_FLAG_OVERFLOW;
                    stop = 1u;
                } else {
                    // lane ol of the batch takes (k, t, fin, written): v_writelane with the
                    // lane select in m0 (m0 is used nowhere else in these kernels)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
                    asm("s_mov_b32 m0, %4\n\ts_nop 0\n\t"
                        "v_writelane_b32 %0, %5, m0\n\t"
                        "v_writelane_b32 %1, %6, m0\n\t"
                        "v_writelane_b32 %2, %7, m0\n\t"
                        "v_writelane_b32 %3, 1, m0"
                        : "+v"(on), "+v"(os), "+v"(of), "+v"(ov)
                        : "s"(sgpr(ol)), "s"(sgpr(k)), "s"(sgpr(t)), "s"(sgpr(fin))
                        : "m0");
#pragma clang diagnostic pop
                    ++placed;
                    ++h;
                    changed = 1u;
                }
            } else if (t - arr >= max_wait) {  // time.Since(WaitTime) >= MaxWaitTime (:353)
                if (lane == 0u) {
                    l1_cm[l1n] = (uint64_t)jc | ((uint64_t)jm << 32);
                    l1_jd[l1n] = (uint64_t)h | ((uint64_t)jd << 32);
                }
                ++l1n;
                peak_l1 = l1n > peak_l1 ? l1n : peak_l1;
                {
                    const uint32_t kk = 63u - (jc < 63u ? jc : 63u);
                    lmv = (lane == kk && jm < lmv) ? jm : lmv;
                }
                ++moved;
                mv_a += arr;
                ++h;
                changed = 1u;
                l1w = 1u;
            }
        }
        // Level1 stores must have reached L2 before the next pass's sc1 loads
        if (l1w) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        // the next pass's first rows, in flight during the clock advance, the releases and the
        // filter build (the list does not change until that pass).  The moves' appends and the
        // pass's compaction stores are waited for explicitly first: a one-wave workgroup's release
        // fence waits on LDS only, and the re-read rows are the ones just written.
        if (l1n != 0u) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            prefetch_l1();
        }

        // ---- time.Sleep(1 s) (:367) and the fast-forward; one exit, tested at the bottom ----
        uint32_t tn = t + 1u;
        if (!changed) {
            // the next iteration that can differ: a release, the head's MaxWaitTime move, or
            // (empty Level0) the next arrival; arr is still job h's arrival
            uint32_t ev = minf;
            const uint32_t e2 = arr <= t ? arr + max_wait : arr;
            ev = (h < J && e2 < ev) ? e2 : ev;
            tn = ev > tn ? ev : tn;
            if constexpr (HOR) {
                // online, an empty Level0 waits for jobs not appended yet: one arriving at or after
                // the horizon but before the jump's target would be the head at its own second, so
                // the jump stops at the horizon (the skipped seconds repeat the same failures either way)
                // (nothing to come at all, kEmpty: parked below, as before)
                if (h >= J && tn != kEmpty && tn > a.on.t_hor) tn = a.on.t_hor;
            }
        }
        if (!stop) {
            if (h >= J && l1n == 0u) {  // every job placed: the run ends at the next iteration
                // (online: parked; the next horizon re-runs this iteration, which is idempotent
                // with nothing queued, unless this is a drain)
                if (!HOR || a.on.t_hor == kEmpty) {
                    t = t + 1u;
                    if constexpr (HOR) flags |= kOnEnded;
                }
                stop = 1u;
            } else if (!changed && tn == kEmpty) {  // nothing runs or arrives: Level1 never fits
                if (!HOR || a.on.t_hor == kEmpty) flags |= MCS_FLAG_DEADLOCK;  // (online: parked)
                stop = 1u;
            } else if (tn <= t) {
                flags |= MCS_FLAG_CLOCK_OVERFLOW;
                stop = 1u;
            } else {
                t = tn;
                if (minf <= t) release();
                if constexpr (HOR) {
                    if (t >= a.on.t_hor) stop = 1u;  // the horizon: resume here next time
                }
            }
        }
        if (stop) rend = 0u;
    } while (h < rend);
    if (rend == 0u) break;
    cb += kWave;
    wave_progress_prio(cb, J);
    }

    // a finish past the u32 clock released its job early: every result of the cluster is void
    const bool ovf_fin = sgpr(ovf) != 0u;
    if (ovf_fin) flags |= MCS_FLAG_CLOCK_OVERFLOW;
    if (!(flags & MCS_FLAG_OVERFLOW)) {
        if (h > cb) flush(cb);  // the current batch's decided jobs (earlier batches are stored)
        if (flags & (MCS_FLAG_DEADLOCK | MCS_FLAG_CLOCK_OVERFLOW)) {
            // the Level1 jobs left are retried forever (deadlock) or were not decided before the
            // clock left the u32 range (the run fails with MCS_E_RANGE): never placed
            for (uint32_t base = 0; base < l1n; base += kWave) {
                const uint32_t pos = base + lane;
                if (pos < l1n) {
                    const uint32_t jw = (uint32_t)ld_l2(l1_jd + pos);
                    o_node[jw] = MCS_NODE_UNPLACED;
                    o_start[jw] = MCS_TIME_NONE;
                    o_finish[jw] = MCS_TIME_NONE;
                }
            }
        }
        if (flags & MCS_FLAG_CLOCK_OVERFLOW) {  // and so were the Level0 jobs h..J-1
            for (uint32_t i = (ovf_fin ? 0u : h) + lane; i < J; i += kWave) {
                o_node[i] = MCS_NODE_UNPLACED;
                o_start[i] = MCS_TIME_NONE;
                o_finish[i] = MCS_TIME_NONE;
            }
        }
    }
    // WaitTime.TotalTime (scheduler.go:309-312,338-341): a placed job keeps 1000 * (start -
    // arrival); a job left in Level1 holds 1000 * (t - arrival) from the last pass.  Every moved
    // job's arrival is in mv_a, so Level1 contributes l1_t + left * t - mv_a.
    // (online: the Level1 jobs still queued count at t as well; the values are final after a drain)
    const uint32_t left = (HOR || (flags & MCS_FLAG_DEADLOCK)) ? l1n : 0u;
    uint64_t wsum = wacc;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)wsum, o);
        const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(wsum >> 32), o);
        wsum += (uint64_t)lo | ((uint64_t)hi << 32);
    }
    const uint64_t wait_s = wsum + l1_t + (uint64_t)left * t - mv_a;
    // WaitTime.JobsCount counts the jobs POSTed to "/delay" (server.go:72): all of them at the
    // end of a run; online, those that arrived before the horizon
    int64_t jobs_count = (int64_t)J;
    if constexpr (HOR) {
        if (a.on.t_hor != kEmpty) {
            uint32_t n = h;
            for (uint32_t b = h; b < J; b += kWave) {
                const uint32_t i = b + lane;
                const uint64_t got = __ballot(i < J && jobs[i].x < a.on.t_hor);
                n += (uint32_t)__builtin_popcountll(got);
                if (got != ~0ull) break;  // arrivals are sorted: the first late one ends the count
            }
            jobs_count = (int64_t)n;
        }
        if (!(flags & MCS_FLAG_OVERFLOW)) {  // save the state the next horizon resumes from
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");  // other lanes' LDS atomics
            unsigned long long* img = a.on.img_out + (size_t)ci * a.on.img_stride;
#pragma unroll
            for (int k = 0; k < NPL; ++k) img[k * kWave + lane] = nodes[k * kWave + lane];
            unsigned long long* sl = a.on.slot_out + (size_t)ci * kSlotImg;
#pragma unroll
            for (int p = 0; p < P; ++p) {
                sl[p * kWave + lane] = pay_cm[p * kWave + lane];
                sl[(kMaxPool + p) * kWave + lane] = pay_nf[p * kWave + lane];
            }
            if (lane == 0) {
                OnlineState st{};
                st.valid = 1u;
                st.t = t;
                st.cursor = h;
                st.aux = l1n;
                st.flags = flags;
                st.pool = (uint32_t)P;
                st.placed = placed;
                st.waited = moved;
                st.peak = peak;
                st.used = used;
                st.n_iter = n_iter;
                st.n_rel = n_rel;
                st.placed_l1 = placed_l1;
                st.peak_l1 = peak_l1;
                st.l1_t = l1_t;
                st.mv_a = mv_a;
                st.wsum = wsum;
                a.on.st_out[ci] = st;
            }
        }
    }

    if (lane == 0) {
        mcs_cluster_stats st;
        st.t_end = t;
        st.placed = placed;
        st.waited = moved;
        st.peak_running = peak;
        st.flags = flags & ~kOnEnded;
        st.pool = (uint32_t)P;
        st.iterations = n_iter;
        st.release_scans = n_rel;
        a.cstats[ci] = st;
        mcs_delay_cluster_stats ds;
        ds.total_wait_ms = (int64_t)(wait_s * 1000ull);
        // every job has arrived when the run ends; a run stopped by the clock range is an error
        // (MCS_E_RANGE) whose wait statistics mean nothing: marked -1
        ds.jobs_count = (flags & MCS_FLAG_CLOCK_OVERFLOW) ? -1 : jobs_count;
        ds.moved_l1 = moved;
        ds.placed_l1 = placed_l1;
        ds.peak_l1 = peak_l1;
        ds.l1_left = left;
        a.dstats[ci] = ds;
        if (flags & MCS_FLAG_OVERFLOW) {
            atomicAdd(&a.totals->overflowed, 1u);
        } else {
            atomicAdd(&a.totals->placed, (unsigned long long)placed);
            atomicAdd(&a.totals->waited, (unsigned long long)moved);
            // online: jobs not decided yet are pending, not unplaced (a drain decides them)
            const bool final_ = !HOR || a.on.t_hor == kEmpty || (flags & MCS_FLAG_CLOCK_OVERFLOW);
            if (final_) atomicAdd(&a.totals->unplaced, (unsigned long long)(J - placed));
            if (flags & MCS_FLAG_DEADLOCK) atomicAdd(&a.totals->deadlocked, 1u);
            if (flags & MCS_FLAG_CLOCK_OVERFLOW) atomicAdd(&a.totals->clock_overflowed, 1u);
        }
    }
}

template <int NPL, int P, bool GEN, bool HOR>
static hipError_t launch_delay_one(const DelayArgs& a, hipStream_t s) {
    hipLaunchKernelGGL((delay_kernel<NPL, P, GEN, HOR>), dim3(a.n_items), dim3(kWave), 0, s, a);
    return hipGetLastError();
}

template <int NPL, bool GEN, bool HOR>
static hipError_t launch_delay_npl(const DelayArgs& a, int pool, hipStream_t s) {
    switch (pool) {
        case 2: return launch_delay_one<NPL, 2, GEN, HOR>(a, s);
        case 4: return launch_delay_one<NPL, 4, GEN, HOR>(a, s);
        case 8: return launch_delay_one<NPL, 8, GEN, HOR>(a, s);
        case 16: return launch_delay_one<NPL, 16, GEN, HOR>(a, s);
        case 32: return launch_delay_one<NPL, 32, GEN, HOR>(a, s);
        default: return hipErrorInvalidValue;
    }
}

template <bool GEN, bool HOR>
static hipError_t launch_delay_gen(const DelayArgs& a, int npl, int pool, hipStream_t s) {
    switch (npl) {
        case 1: return launch_delay_npl<1, GEN, HOR>(a, pool, s);
        case 2: return launch_delay_npl<2, GEN, HOR>(a, pool, s);
        case 4: return launch_delay_npl<4, GEN, HOR>(a, pool, s);
        case 8: return launch_delay_npl<8, GEN, HOR>(a, pool, s);
        case 16: return launch_delay_npl<16, GEN, HOR>(a, pool, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_delay(const DelayArgs& a, int npl, int pool, bool hor, hipStream_t s) {
    if (a.n_items == 0) return hipSuccess;
    if (hor) return a.gen.on ? hipErrorInvalidValue : launch_delay_gen<false, true>(a, npl, pool, s);
    return a.gen.on ? launch_delay_gen<true, false>(a, npl, pool, s)
                    : launch_delay_gen<false, false>(a, npl, pool, s);
}

}  // namespace mcs
