// mcs_kernels.hip — gfx950 kernels of the batched FIFO placement engine.
//
// The hot kernel (fifo_kernel) runs the reference's FIFO policy loop — Scheduler.Fifo
// (pkg/scheduler/scheduler.go:216-296) over the first-fit primitive ScheduleJob (:127-139) and the
// commit/release of Node.RunJob (pkg/scheduler/cluster.go:141-161) — for one cluster per wave64
// workgroup, under the serialized semantics SFIFO of SURVEY Appendix A with the exact fast-forward
// of A.3.  Every decision is wave-uniform, so the wave never diverges on control flow:
//
//   * node free vectors are staged in LDS as packed u64 {free_c, free_m}, lane l owning the NPL
//     consecutive nodes l*NPL.. (chunk c at nodes[c*64 + l]); first fit = one ds_read_b64 per
//     chunk (issued at the end of the previous pass, after its commit and releases), a per-lane
//     lowest-fitting-chunk select, a ballot + ff1 for the lowest lane with a fit and one readlane
//     of its chunk; commit is one ds_sub_u64 (by the slot-insert lane) and a release one
//     ds_add_u64 (the packed halves never borrow or carry: a placed job fits and resources are
//     conserved);
//   * the running set is a pool of 64*P slots (row p, lane l): finish times in VGPRs (one
//     register per row, static indices only), payload {cores|mem, node} in LDS [P][64]
//     (lane-contiguous, bank-conflict-free); a free slot is the lowest free row of the lowest
//     lane that has one (ballot + ffbl);
//   * releases at a clock advance go row by row: the expired test of row p over all lanes is one
//     compare whose lane mask drives that row's payload hand-back (ds_add_u64, order-free integer
//     adds) and its free-row bits; the next completion time is a DPP wave minimum;
//   * job records are streamed from HBM 64 at a time with one coalesced 16 B/lane load (uint4
//     {arrival, dur, cores, mem}), double-buffered one batch ahead, and broadcast to the scalar
//     unit with v_readlane; with fused generation (GEN) each batch is synthesised in registers
//     instead and no record is read (mcs_gen_dev.h);
//   * results are gathered 64 jobs per register batch (placements happen in job order because
//     FIFO head-of-line blocking is strict) and written with three coalesced 256 B stores.
//
// Codegen notes (measured with rocprofv3 SQ counters, profiles/): the kernel is issue-bound on
// the CU's shared scalar unit and VALU, not on HBM.  Keeping node state in LDS and the loop
// single-exit removed the whole-state register copies LLVM inserted at control-flow merges.
//
// Compiled with -ffp-contract=off (no FP in this file's hot kernel; the utilization mirror is
// float32 and must round like Go).
#define MCS_GEN_FN __host__ __device__ static inline
#include "mcs_gen.h"
#include "mcs_gen_dev.h"
#include "mcs_internal.h"
#include "mcs_lds.h"
#include "mcs_wave.h"

#ifdef MCS_STAMPS
// diagnostic build only (tools/stamp_probe.py): per-segment cycle sums of the pass loop
#define MCS_STAMP(v)                                                                    \
    do {                                                                                \
        __builtin_amdgcn_sched_barrier(0);                                              \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");       \
        __builtin_amdgcn_sched_barrier(0);                                              \
    } while (0)
__device__ unsigned long long g_stamps[8];
#else
#define MCS_STAMP(v) \
    do {             \
    } while (0)
#endif

namespace mcs {


// HOR: the online variant.  The cluster resumes from the OnlineState, node image
// and slot image of the previous horizon (or its spec when the state is not valid), runs every
// iteration at t < a.on.t_hor, and saves them again; job counts come from a.on.job_cnt.  The
// one-shot variant (HOR = false) is the batch hot path and does none of this.
// LAT: the low-occupancy form (a few cluster waves per CU, e.g. one system sharded over several
// GPUs): the fitting chunk is picked by scalar bit tests and a release reads every slot payload
// with the finish words (one wait), which shortens one decision's chain at the price of scalar
// work and LDS time, the shared resources at 16 waves per CU.
template <int NPL, int P, bool GEN, bool HOR, bool LAT>
__global__ __launch_bounds__(64) void fifo_kernel(FifoArgs a) {
    static_assert(P <= 32, "free-row mask is one u32 per lane");
    static_assert(!(HOR && GEN), "online runs stream records");
    const uint32_t item = blockIdx.x;
    const uint32_t ci = a.cluster_list ? a.cluster_list[item] : item;
    const uint32_t lane = threadIdx.x;

    // Node free vectors staged in LDS as packed u64 {free_c, free_m}: commit is one ds_sub_u64
    // (the job fits, so the low half never borrows) and a release one ds_add_u64 (resources are
    // conserved, so the low half never carries).  Node k lives at nodes[k].
    __shared__ uint64_t nodes[NPL * kWave];
    // running slots, row-major [P][64]: {cores | mem << 32} and {node | finish << 32}
    // (one array, so a slot's two words share one address register and differ by an offset)
    __shared__ uint64_t pay[2 * P * kWave];
    uint64_t* const pay_cm = pay;
    uint64_t* const pay_nf = pay + P * kWave;

    // ---- cluster spec: Run() keeps the JSON availability (scheduler.go:101-109) ----
    const uint32_t n0 = a.node_off[ci];
    const uint32_t N = a.node_off[ci + 1] - n0;
    // Lane l holds the NPL consecutive nodes l * NPL + c (c = chunk), stored at nodes[c * 64 + l]
    // (lane-contiguous rows, conflict-free): the lowest fitting node is then in the lowest lane
    // with any fit, at that lane's lowest fitting chunk.
#pragma unroll
    for (int c = 0; c < NPL; ++c) {
        const uint32_t node = lane * NPL + c;
        uint2 v = make_uint2(0u, 0u);  // padding: free 0 fits only a zero job, which node 0 takes
        if (node < N) v = a.node_free0[n0 + node];
        nodes[c * kWave + lane] = (uint64_t)v.x | ((uint64_t)v.y << 32);
    }
    const uint64_t vmask = __ballot(lane * NPL < N);  // lanes holding a real node

    // ---- job stream ----
    const uint64_t j0 = a.job_off[ci];
    const uint32_t J = HOR ? a.on.job_cnt[ci] : (uint32_t)(a.job_off[ci + 1] - j0);
    const uint4* __restrict__ jobs = GEN ? nullptr : a.jobs + j0;
    int32_t* __restrict__ o_node = a.out_node + j0;
    uint32_t* __restrict__ o_start = a.out_start + j0;
    uint32_t* __restrict__ o_finish = a.out_finish + j0;

    // Unmasked: the job array has kJobPad records of slack, and records past this cluster's end
    // (the next cluster's, or the pad) are read but never used, because r < J guards every use.
    // An unmasked load can land straight in the loop-carried batch registers, so the prefetch one
    // batch ahead is not waited for until that batch is needed.
    // GEN: the batch is synthesised in registers instead (mcs_gen_dev.h; bases come in order)
    GenStream gs;
    if constexpr (GEN) gs.init(a.gen, ci, lane);
    auto load_batch = [&](uint32_t base) __attribute__((always_inline)) -> uint4 {
        if constexpr (GEN)
            return gs.next(base, lane);
        else
            return jobs[base + lane];
    };

    // running slots: frm = this lane's free rows (bit p), lmin = earliest finish among its
    // occupied rows (kEmpty if none); finish times and payloads live in LDS
    uint32_t frm = (P == 32) ? 0xFFFFFFFFu : ((1u << P) - 1u);
    uint32_t lmin = kEmpty;
#pragma unroll
    for (int p = 0; p < P; ++p) pay_nf[p * kWave + lane] = (uint64_t)kEmpty << 32;  // free: never expires

    uint32_t t = 0, r = 0, flags = 0;
    // Counters that no decision reads live in VGPRs (the asm hides their uniformity): the CU's
    // one scalar unit is shared by 16 cluster waves and is the scarcer issue resource.
    uint32_t used = 0, peak = 0, waited = 0, placed = 0;
    uint32_t n_iter = 0, n_rel = 0;  // diagnostics: loop passes, release scans
    uint32_t ovf_r = kEmpty;         // first job whose finish left the u32 clock range
    // have_w: the job at the ready cursor r already failed once and is the WaitQueue head
    // (|WaitQueue| <= 1, scheduler.go:264-268), so the candidate is always job r
    uint32_t have_w = 0u;
    int32_t on = -1;
    uint32_t os = kEmpty, of = kEmpty;
    bool live = true;  // the loop runs (online: not parked, not stopped for good)
    uint32_t r_in = 0;
    if constexpr (HOR) {  // resume from the previous horizon
        const OnlineState st = a.on.st_in[ci];
        if (st.valid) {
            const unsigned long long* img = a.on.img_in + (size_t)ci * a.on.img_stride;
#pragma unroll
            for (int c = 0; c < NPL; ++c) nodes[c * kWave + lane] = img[c * kWave + lane];
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
            t = st.t;
            r = st.cursor;
            have_w = st.aux;
            flags = st.flags;
            placed = st.placed;
            waited = st.waited;
            peak = st.peak;
            used = st.used;
            n_iter = st.n_iter;
            n_rel = st.n_rel;
        }
        r_in = r;
        // a deadlocked head blocks the cluster for good (nothing runs, nothing can overtake it);
        // a clock overflow is final; a parked cluster waits for jobs; the horizon may be reached
        live = !(flags & (MCS_FLAG_DEADLOCK | MCS_FLAG_CLOCK_OVERFLOW)) && r < J && t < a.on.t_hor;
        // the register result batch holds the rows already decided in the current batch
        const uint32_t i = (r & ~63u) + lane;
        on = o_node[i];
        os = o_start[i];
        of = o_finish[i];
    }
    asm volatile("" : "+v"(used), "+v"(peak), "+v"(waited), "+v"(placed), "+v"(n_iter), "+v"(n_rel),
                 "+v"(ovf_r));

    const uint32_t cb0 = HOR ? (r & ~63u) : 0u;
    uint32_t cb = cb0;
    uint4 nxt = load_batch(cb0);
    // wait for the first batch here: the only load pending at the pass loop's entry is then the
    // prefetch, which the loop never reads, so the waitcnt pass does not flush it at every batch
    asm volatile("" ::"v"(nxt.x), "v"(nxt.y), "v"(nxt.z), "v"(nxt.w));

    // LDS byte addresses of the node vector and of this lane's slot column
    const uint32_t nodes_lds = lds_addr(nodes);
    const uint32_t pay_lds = lds_addr(pay) + lane * 8u;

    // Node free vectors in registers (nvr[c]: node lane * NPL + c), the state every decision
    // reads: a commit updates them in place, so a decision never waits on LDS.  The LDS copy
    // nodes[] follows every change (ds_sub_u64 at a commit, ds_add_u64 at a release hand-back)
    // and is read back only after a release.
    uint64_t nvr[NPL];
#pragma unroll
    for (int c = 0; c < NPL; ++c) {
        nvr[c] = nodes[c * kWave + lane];
        asm volatile("" ::"v"(nvr[c]));  // waited for here, not at the loop's first compare
    }

    // release every running job with finish <= t (cluster.go:153-157; A.2 step 1).  Row by row:
    // the expired test of row p over all lanes is one compare straight into a lane mask, which
    // drives the payload hand-back of that row (only rows with an expiry branch off the straight
    // line) and the free-row bits; the lane's next finish is the min over its unexpired rows.
    auto release = [&]() __attribute__((always_inline)) {
        ++n_rel;
        const uint32_t t1 = t + 1u;  // t < kEmpty here (a wrap stops the run first)
        uint64_t nf[P];
        uint64_t cm[LAT ? P : 1];
        if constexpr (LAT) {  // payload rows 0..P-1 and finish rows P..2P-1, one wait
            uint64_t rows[2 * P];
            read_finish_rows<2 * P>(rows, pay_lds);
#pragma unroll
            for (int p = 0; p < P; ++p) {
                cm[p] = rows[p];
                nf[p] = rows[P + p];
            }
        } else {
            read_finish_rows<P>(nf, pay_lds + P * kWave * 8u);
        }
        // lane's next finish: min over unexpired rows, as min(f - (t + 1)) + (t + 1) in u32: an
        // expired row (f <= t) wraps above every unexpired and free one, and the bound ~t1 caps
        // the result at kEmpty when the lane has none left
        uint32_t lm = ~t1;
        uint32_t nexp = 0u;
#pragma unroll
        for (int p = 0; p < P; ++p) {  // free rows hold kEmpty: never expired
            const uint32_t f = (uint32_t)(nf[p] >> 32);
            const uint64_t m = lanes_ge(t, f);
            const uint32_t d = f - t1;
            lm = d < lm ? d : lm;
            if (__builtin_expect(m != 0ull, 0)) {
                nexp += (uint32_t)__builtin_popcountll(m);
                // the expired lanes (exec = m) give their payloads back to their nodes and free
                // the row: (read payload,) ds_add_u64 on the node, finish word := kEmpty
                const uint32_t na = nodes_lds + (uint32_t)nf[p] * 8u;
                uint64_t sv;
                if constexpr (LAT) {
                    asm volatile(
                        "s_mov_b64 %[sv], exec\n\t"
                        "s_mov_b64 exec, %[m]\n\t"
                        "ds_add_u64 %[na], %[cm]\n\t"
                        "ds_write_b32 %[pa], %[emp] offset:%[of]\n\t"
                        "v_or_b32 %[frm], %[bit], %[frm]\n\t"
                        "s_mov_b64 exec, %[sv]"
                        : [sv] "=&s"(sv), [frm] "+v"(frm)
                        : [m] "s"(m), [pa] "v"(pay_lds), [na] "v"(na), [cm] "v"(cm[p]), [emp] "v"(kEmpty),
                          [bit] "i"(1u << p), [of] "i"((P + p) * kWave * 8 + 4)
                        : "memory");
                } else {
                    uint64_t cmr;
                    asm volatile(
                        "s_mov_b64 %[sv], exec\n\t"
                        "s_mov_b64 exec, %[m]\n\t"
                        "ds_read_b64 %[cm], %[pa] offset:%[oc]\n\t"
                        "s_waitcnt lgkmcnt(0)\n\t"
                        "ds_add_u64 %[na], %[cm]\n\t"
                        "ds_write_b32 %[pa], %[emp] offset:%[of]\n\t"
                        "v_or_b32 %[frm], %[bit], %[frm]\n\t"
                        "s_mov_b64 exec, %[sv]"
                        : [sv] "=&s"(sv), [cm] "=&v"(cmr), [frm] "+v"(frm)
                        : [m] "s"(m), [pa] "v"(pay_lds), [na] "v"(na), [emp] "v"(kEmpty), [bit] "i"(1u << p),
                          [oc] "i"(p * kWave * 8), [of] "i"((P + p) * kWave * 8 + 4)
                        : "memory");
                }
            }
        }
        used -= nexp;
        // read the node vectors back (the hand-backs are ahead of the reads in LDS order)
        reload_nodes(nvr, nodes_lds + lane * 8u);
        lmin = lm + t1;
    };

    // rend bounds the ready cursor of the inner pass loop: the end of the current batch, or 0 once
    // the run stops, so one scalar compare ends both loops
    uint32_t rend = 0u;
    // a placement of job ri on node k = fl * NPL + fch at t: the result record (lane ri & 63 of
    // the register batch) and, for a job that runs, Node.RunJob's commit (cluster.go:146-147,
    // synchronous D2) with the running-slot insert.  fr: lanes with a free slot row.
    auto place = [&](uint32_t ri, uint32_t jd, uint32_t jc, uint32_t jm, uint32_t fl, uint32_t fch,
                     uint64_t fr) __attribute__((always_inline)) {
        const uint32_t k = fl * NPL + fch;     // the node (Go index)
        const uint32_t kx = fch * kWave + fl;  // its place in nodes[]
        const uint32_t ol = ri & 63u;
        const uint32_t fin = t + jd;
        // lane ol of the batch takes (k, t, fin): three v_writelane (lane select in m0, the one
        // scalar operand gfx950 allows beside the data SGPR); m0 is reserved to the compiler,
        // which uses it nowhere in these kernels
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
        asm("s_mov_b32 m0, %3\n\ts_nop 0\n\t"
            "v_writelane_b32 %0, %4, m0\n\t"
            "v_writelane_b32 %1, %5, m0\n\t"
            "v_writelane_b32 %2, %6, m0"
            : "+v"(on), "+v"(os), "+v"(of)
            : "s"(sgpr(ol)), "s"(sgpr(k)), "s"(sgpr(t)), "s"(sgpr(fin))
            : "m0");
#pragma clang diagnostic pop
        // A zero-duration job is committed and released before the next decision can read the
        // node (RunJob sleeps 0; the release precedes the next branch, D3).
        if (jd != 0u) {
            // a finish that wraps the u32 clock or hits the kEmpty sentinel (D8 range) is
            // recorded off the decision chain, in VALU: the first such job ends the valid
            // results.  Only the online variant carries this guard: the host bound keeps checked
            // streams away from it, and the engine runs batch runs of unchecked streams
            // (cfg.unchecked_horizon) through the online variant
            if constexpr (HOR) {
                uint32_t tv = t, jv = jd;  // VGPR copies: the check stays in VALU
                asm volatile("" : "+v"(tv), "+v"(jv));
                const uint32_t fv = tv + jv;
                const uint32_t cand = (fv + 1u <= tv) ? ri : kEmpty;
                ovf_r = cand < ovf_r ? cand : ovf_r;
            }
            // slot insert: the lowest lane with a free row, its lowest free row.  On a pool
            // overflow the run stops and the cluster is re-run with a bigger pool.
            if (!fr) {
                flags |= MCS_FLAG_OVERFLOW;
                rend = 0u;
            } else {
                // commit in registers: lane fl, chunk fch (packed halves: the job fits, so the
                // low half never borrows)
                const bool me = lane == fl;
                const uint32_t dc = me ? jc : 0u, dm = me ? jm : 0u;
#pragma unroll
                for (int c = 0; c < NPL; ++c)
                    if ((uint32_t)c == fch)
                        nvr[c] = (uint64_t)((uint32_t)nvr[c] - dc) |
                                 ((uint64_t)((uint32_t)(nvr[c] >> 32) - dm) << 32);
                // That one lane (exec = its bit) writes the slot {need, node | fin << 32}; its
                // free rows and earliest finish follow.  One asm block: exec is restored before
                // anything else issues.
                const uint64_t need = (uint64_t)jc | ((uint64_t)jm << 32);
                const uint64_t nfw = (uint64_t)kx | ((uint64_t)fin << 32);  // release target
                // (under that exec: slot row = lowest free bit, address = row * 512 + lane * 8)
                uint64_t sv;
                uint32_t ta, tf;
                asm volatile(
                    "s_mov_b64 %[sv], exec\n\t"
                    "s_mov_b64 exec, %[m]\n\t"
                    "v_ffbl_b32 %[ta], %[frm]\n\t"
                    "v_lshl_add_u32 %[ta], %[ta], 9, %[pl]\n\t"
                    "ds_sub_u64 %[na], %[nd]\n\t"
                    "ds_write_b64 %[ta], %[nd]\n\t"
                    "ds_write_b64 %[ta], %[nf] offset:%[off]\n\t"
                    "v_add_u32 %[tf], -1, %[frm]\n\t"
                    "v_and_b32 %[frm], %[tf], %[frm]\n\t"
                    "v_min_u32 %[lmin], %[fin], %[lmin]\n\t"
                    "s_mov_b64 exec, %[sv]"
                    : [sv] "=&s"(sv), [ta] "=&v"(ta), [tf] "=&v"(tf), [frm] "+v"(frm), [lmin] "+v"(lmin)
                    : [m] "s"(1ull << __builtin_ctzll(fr)), [nd] "v"(need), [pl] "v"(pay_lds),
                      [nf] "v"(nfw), [fin] "s"(sgpr(fin)), [off] "i"(P * kWave * 8),
                      [na] "v"(nodes_lds + kx * 8u)
                    : "memory");
                ++used;
                peak = used > peak ? used : peak;
            }
        }
    };

    // ---- Scheduler.Fifo (scheduler.go:216-296) ----
    // One pass = one decision; the loop has a single exit (the structurizer then needs no flow
    // copies of the loop-carried registers).  rend (declared above) bounds the ready cursor of
    // the inner loop.
#ifdef MCS_STAMPS
    unsigned long long t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0;
    unsigned long long ss[7] = {};
#endif
    // advance the clock to tn (> t): releases at the new instant (A.2 step 1), then the online
    // horizon; a tn below t means the u32 seconds clock wrapped (D8 range exceeded): stop, flagged
    auto advance = [&](uint32_t tn) __attribute__((always_inline)) {
        if (tn < t) {
            flags |= MCS_FLAG_CLOCK_OVERFLOW;
            rend = 0u;
        } else {
            t = tn;
            if (lanes_ge(t, lmin) != 0ull) {  // a running job finishes by t
                release();
                MCS_STAMP(t3);
            }
            if constexpr (HOR) {
                if (t >= a.on.t_hor) rend = 0u;  // the horizon: resume here next time
            }
        }
    };

    // The ReadyQueue head's record {arrival, dur, cores, mem} (jr, job r) in scalar registers,
    // broadcast from the batch registers (v_readlane) when the cursor moves.
    uint4 jr = make_uint4(0u, 0u, 0u, 0u);
    if (live) {
    // Outer loop: one 64-job result batch (and, fused, one 64-record batch); inner loop: the
    // passes whose ready cursor is in it.  The previous batch's results (all 64 placed) are
    // stored here.
    do {
    const uint4 cur = nxt;
    if (cb != cb0) {  // a full batch: every lane's job cb - 64 + lane < J, no mask
        const uint32_t i = cb - kWave + lane;
        __builtin_nontemporal_store(on, o_node + i);
        __builtin_nontemporal_store(os, o_start + i);
        __builtin_nontemporal_store(of, o_finish + i);
    }
    nxt = load_batch(cb + kWave);  // prefetch (or generate) one batch ahead
    {
        const uint32_t l = r - cb;
        jr = make_uint4(readlane(cur.x, l), readlane(cur.y, l), readlane(cur.z, l), readlane(cur.w, l));
    }
    rend = cb + kWave;
    do {
        MCS_STAMP(t0);
#ifdef MCS_STAMPS
        t1 = t0;
        t3 = 0;
#endif
        ++n_iter;
        // ReadyQueue head (:255-260): the next stream job, queued once its arrival has passed.
        // Streamed: one scalar load per pass, a value of this pass only (a loop-carried record
        // made LLVM copy it at the latch, waiting for the load there)
        const uint32_t arr = jr.x, jd = jr.y, jc = jr.z, jm = jr.w;
        if (__builtin_expect(r >= J, 0)) {  // every job decided
            MCS_STAMP(t2);
            rend = 0u;
        } else if (__builtin_expect(arr > t, 0)) {  // all queues empty: 1 s sleeps to the arrival
            MCS_STAMP(t2);                           // (:294); a wait head has always arrived,
            advance(arr);                            // so this is never taken with have_w
        } else {
            // first fit — ScheduleJob, scheduler.go:129-137: lowest node index with both >=.
            // One lane mask per chunk (two compares straight into scalar registers); the lowest
            // lane with any fit holds the node, at the lowest chunk whose mask has that lane.
            uint64_t F[NPL];
            uint64_t fit = 0ull;
#pragma unroll
            for (int c = 0; c < NPL; ++c) {
                const uint64_t v = nvr[c];
                F[c] = lanes_ge((uint32_t)v, jc) & lanes_ge((uint32_t)(v >> 32), jm);
                fit |= F[c];
            }
            fit &= vmask;
            // each lane's lowest fitting chunk, selected in VALU by the chunk masks (the scalar
            // unit is shared by the CU's waves; the vector unit is per SIMD)
            uint32_t bc = NPL - 1;
            if constexpr (!LAT) {
#pragma unroll
                for (int c = NPL - 2; c >= 0; --c)  // bc = F[c] has this lane ? c : bc (mask operand)
                    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(bc) : "v"(bc), "i"(c), "s"(F[c]));
            }
#ifdef MCS_STAMPS
            asm volatile("" ::"s"(fit));
#endif
            MCS_STAMP(t1);
            if (__builtin_expect(fit != 0ull, 1)) {
                const uint32_t fl = (uint32_t)__builtin_ctzll(fit);
                uint32_t fch = 0u;
                if constexpr (LAT) {  // lowest chunk whose mask has lane fl: scalar bit tests
                    fch = NPL - 1;
#pragma unroll
                    for (int c = NPL - 2; c >= 0; --c) fch = ((F[c] >> fl) & 1ull) ? (uint32_t)c : fch;
                } else if constexpr (NPL > 1) {
                    fch = readlane(bc, fl);
                }
                place(r, jd, jc, jm, fl, fch, lanes_ne(frm, 0u));
                ++r;
                {
                    const uint32_t l = (r - cb) & 63u;  // (a batch boundary reloads it above)
                    jr = make_uint4(readlane(cur.x, l), readlane(cur.y, l), readlane(cur.z, l),
                                    readlane(cur.w, l));
                }
                MCS_STAMP(t2);
                // wait head: WaitQueue = WaitQueue[1:] (:226; D1) and time.Sleep(1 s) (:250);
                // ready head: next job, no sleep (:272)
                if (__builtin_expect(have_w != 0u, 0)) {
                    have_w = 0u;
                    advance(t + 1u);
                }
            } else {
                // State = WAITING; WaitQueue append (:264-268).  The Go loop's next pass retries
                // the new head at this same instant on an unchanged cluster (certain to fail),
                // then sleeps: folded into the fast-forward.
                waited += 1u - have_w;
                have_w = 1u;
                MCS_STAMP(t2);
                // the next completion, over every lane's earliest finish (only waits need it)
                const uint32_t minf = wave_min_u32(lmin);
                if (minf == kEmpty) {  // nothing running: the head can never fit
                    flags |= MCS_FLAG_DEADLOCK;
                    rend = 0u;
                } else {  // A.3: 1 s retries until the next completion (no lender, :234)
                    advance(minf > t + 1u ? minf : t + 1u);
                }
            }
        }
#ifdef MCS_STAMPS
        if (t3 == 0) t3 = t2;
#endif
        MCS_STAMP(t4);
#ifdef MCS_STAMPS
        ss[0] += t1 - t0;
        ss[1] += t2 - t1;
        ss[2] += t3 - t2;
        ss[3] += t4 - t3;
        ss[4] += 1u;
        ss[5] += t3 != t2 ? 1u : 0u;
        ss[6] += t1 != t0 ? 1u : 0u;
#endif
    } while (r < rend);
    cb += kWave;
    wave_progress_prio(cb, J);
    } while (rend != 0u);
    }  // live

    placed = r;  // FIFO places every job it decides, in order
    // [rs, J) is undecided: a deadlocked head and everything behind it (the Go loop retries the
    // head forever), or every job from the first one whose clock left the u32 range (the run
    // fails with MCS_E_RANGE)
    const uint32_t ovf_job = sgpr(ovf_r);
    if (ovf_job != kEmpty) flags |= MCS_FLAG_CLOCK_OVERFLOW;
    const uint32_t rs = ovf_job < r ? ovf_job : r;
    if (!(flags & MCS_FLAG_OVERFLOW)) {
        // the batch holding the last decision, lanes decided (a batch boundary reached in the
        // same pass is rewritten with the same values); earlier batches are stored
        if (r > r_in) {
            const uint32_t i = ((r - 1u) & ~63u) + lane;
            if (i < rs) {
                __builtin_nontemporal_store(on, o_node + i);
                __builtin_nontemporal_store(os, o_start + i);
                __builtin_nontemporal_store(of, o_finish + i);
            }
        }
        if (flags & (MCS_FLAG_DEADLOCK | MCS_FLAG_CLOCK_OVERFLOW)) {
            for (uint32_t i = rs + lane; i < J; i += kWave) {
                o_node[i] = MCS_NODE_UNPLACED;
                o_start[i] = MCS_TIME_NONE;
                o_finish[i] = MCS_TIME_NONE;
            }
        }
    }
    if (flags & MCS_FLAG_CLOCK_OVERFLOW) placed = rs < placed ? rs : placed;

    if constexpr (HOR) {  // save the state the next horizon resumes from (rerun on overflow)
        if (!(flags & MCS_FLAG_OVERFLOW)) {
            unsigned long long* img = a.on.img_out + (size_t)ci * a.on.img_stride;
#pragma unroll
            for (int c = 0; c < NPL; ++c) img[c * kWave + lane] = nvr[c];  // the register truth
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
                st.cursor = rs;
                st.aux = have_w;
                st.flags = flags;
                st.pool = (uint32_t)P;
                st.placed = placed;
                st.waited = waited;
                st.peak = peak;
                st.used = used;
                st.n_iter = n_iter;
                st.n_rel = n_rel;
                a.on.st_out[ci] = st;
            }
        }
    }

#ifdef MCS_STAMPS
    if (lane == 0)
        for (int q = 0; q < 7; ++q) atomicAdd(&g_stamps[q], ss[q]);
#endif
    if (lane == 0) {
        mcs_cluster_stats st;
        st.t_end = t;
        st.placed = placed;
        st.waited = waited;
        st.peak_running = peak;
        st.flags = flags;
        st.pool = (uint32_t)P;
        st.iterations = n_iter;
        st.release_scans = n_rel;
        a.cstats[ci] = st;
        if (flags & MCS_FLAG_OVERFLOW) {
            atomicAdd(&a.totals->overflowed, 1u);
        } else {
            atomicAdd(&a.totals->placed, (unsigned long long)placed);
            atomicAdd(&a.totals->waited, (unsigned long long)waited);
            // online: jobs not decided yet are pending, not unplaced
            const bool final_ = !HOR || (flags & (MCS_FLAG_DEADLOCK | MCS_FLAG_CLOCK_OVERFLOW));
            if (final_) atomicAdd(&a.totals->unplaced, (unsigned long long)(J - placed));
            if (flags & MCS_FLAG_DEADLOCK) atomicAdd(&a.totals->deadlocked, 1u);
            if (flags & MCS_FLAG_CLOCK_OVERFLOW) atomicAdd(&a.totals->clock_overflowed, 1u);
        }
    }
}

// ---- variant table ------------------------------------------------------------------------------
template <int NPL, int P, bool GEN, bool HOR, bool LAT>
static hipError_t launch_one(const FifoArgs& a, hipStream_t s) {
    hipLaunchKernelGGL((fifo_kernel<NPL, P, GEN, HOR, LAT>), dim3(a.n_items), dim3(kWave), 0, s, a);
    return hipGetLastError();
}

template <int NPL, bool GEN, bool HOR>
static hipError_t launch_npl(const FifoArgs& a, int pool, bool lat, hipStream_t s) {
    switch (pool) {
        case 2: return lat ? launch_one<NPL, 2, GEN, HOR, !GEN && !HOR>(a, s)
                             : launch_one<NPL, 2, GEN, HOR, false>(a, s);
        case 4: return lat ? launch_one<NPL, 4, GEN, HOR, !GEN && !HOR>(a, s)
                             : launch_one<NPL, 4, GEN, HOR, false>(a, s);
        case 8: return lat ? launch_one<NPL, 8, GEN, HOR, !GEN && !HOR>(a, s)
                             : launch_one<NPL, 8, GEN, HOR, false>(a, s);
        case 16: return lat ? launch_one<NPL, 16, GEN, HOR, !GEN && !HOR>(a, s)
                             : launch_one<NPL, 16, GEN, HOR, false>(a, s);
        case 32: return lat ? launch_one<NPL, 32, GEN, HOR, !GEN && !HOR>(a, s)
                             : launch_one<NPL, 32, GEN, HOR, false>(a, s);
        default: return hipErrorInvalidValue;
    }
}

template <bool GEN, bool HOR>
static hipError_t launch_fifo_gen(const FifoArgs& a, int npl, int pool, bool lat, hipStream_t s) {
    switch (npl) {
        case 1: return launch_npl<1, GEN, HOR>(a, pool, lat, s);
        case 2: return launch_npl<2, GEN, HOR>(a, pool, lat, s);
        case 4: return launch_npl<4, GEN, HOR>(a, pool, lat, s);
        case 8: return launch_npl<8, GEN, HOR>(a, pool, lat, s);
        case 16: return launch_npl<16, GEN, HOR>(a, pool, lat, s);
        default: return hipErrorInvalidValue;
    }
}

bool fifo_variant_exists(int npl, int pool) {
    const bool np = npl == 1 || npl == 2 || npl == 4 || npl == 8 || npl == 16;
    const bool pp = pool == 2 || pool == 4 || pool == 8 || pool == 16 || pool == 32;
    return np && pp;
}

// The low-occupancy form for grids of at most kLatWavesPerCu cluster waves per CU (the streamed
// batch path only): measured on C4 shards, 2.3-2.4 % faster at 1-4 waves per CU, 1.5 % slower at 8
// (DESIGN.md §4).  MCS_FIFO_LAT=0/1 forces it off/on (A/B timing, the variant test).
uint32_t cu_count() {
    static int n_cu = 0;
    if (n_cu == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0)
            n_cu = 256;
    }
    return (uint32_t)n_cu;
}

hipError_t launch_fifo(const FifoArgs& a, int npl, int pool, bool hor, hipStream_t s) {
    const char* env = getenv("MCS_FIFO_LAT");
    const int g_lat_env = env ? atoi(env) : -1;
    const bool lat = g_lat_env >= 0 ? g_lat_env != 0 : a.n_items <= kLatWavesPerCu * cu_count();
    if (fifo_asm_eligible(a, npl, pool, hor)) return launch_fifo_asm(a, npl, pool, s);
    if (hor) return a.gen.on ? hipErrorInvalidValue : launch_fifo_gen<false, true>(a, npl, pool, false, s);
    return a.gen.on ? launch_fifo_gen<true, false>(a, npl, pool, false, s)
                    : launch_fifo_gen<false, false>(a, npl, pool, lat, s);
}

// ---- device job-stream synthesis (mcs_gen.h; bit-identical to the host generator) -------------
__global__ __launch_bounds__(256) void gen_attrs_kernel(uint4* jobs, const uint64_t* job_off,
                                                       const uint32_t* max_c,
                                                       const uint32_t* max_m, uint64_t seed,
                                                       uint32_t max_dur, uint32_t base) {
    const uint32_t c = blockIdx.y;
    const uint64_t j0 = job_off[c], J = job_off[c + 1] - j0;
    const uint64_t key = mcs_cluster_key(seed, base + c);  // keyed by the global cluster index
    const uint32_t mc = max_c[c], mm = max_m[c];
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < J;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t d, cc, m;
        mcs_gen_job_attrs(key, i, mc, mm, max_dur, &d, &cc, &m);
        jobs[j0 + i] = make_uint4(0u, d, cc, m);
    }
}

__global__ __launch_bounds__(64) void gen_arrivals_kernel(uint4* jobs, const uint64_t* job_off,
                                                         uint32_t n_clusters, GenArgs g) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n_clusters) return;
    const uint64_t j0 = job_off[c], J = job_off[c + 1] - j0;
    const uint64_t akey = mcs_arrival_key(mcs_cluster_key(g.seed, g.base + c));
    uint64_t j = 0, period = 0;
    uint32_t T = 0;
    // same scan as mcs_gen_arrivals (mcs_gen.h), writing into the .x lane of the records
    if (g.mode == 2u) {
        for (; j < J; ++j) {
            jobs[j0 + j].x = T;
            T += mcs_weibull_gap(mcs_draw(akey, j), (const uint64_t*)g.wthr, g.wn);
        }
        return;
    }
    while (j < J) {
        const uint32_t n = mcs_poisson(akey, period++, g.enl);
        if (g.mode == 0u) {
            if (n == 0u) {
                T += 60u;
                continue;
            }
            const uint32_t sp = 60u / n;
            for (uint32_t i = 0; i < n && j < J; ++i) {
                jobs[j0 + j].x = T;
                ++j;
                T += sp;
            }
        } else {
            for (uint32_t i = 0; i < n && j < J; ++i) {
                jobs[j0 + j].x = T;
                ++j;
            }
            T += 1u;
        }
    }
}

// last arrival of every cluster's synthetic stream (the scan of mcs_gen_arrivals in 64-bit time,
// nothing stored): the clock-range check of a fused stream in mcs_generate_jobs
__global__ __launch_bounds__(64) void gen_bound_kernel(const uint64_t* job_off, uint32_t n_clusters, GenArgs g,
                                                      unsigned long long* last) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n_clusters) return;
    const uint64_t J = job_off[c + 1] - job_off[c];
    const uint64_t akey = mcs_arrival_key(mcs_cluster_key(g.seed, g.base + c));
    uint64_t j = 0, period = 0, T = 0, lastT = 0;
    if (g.mode == 2u) {
        for (; j + 1u < J; ++j) T += mcs_weibull_gap(mcs_draw(akey, j), (const uint64_t*)g.wthr, g.wn);
        last[c] = T;
        return;
    }
    while (j < J) {
        const uint32_t n = mcs_poisson(akey, period++, g.enl);
        if (g.mode == 0u) {
            if (n == 0u) {
                T += 60u;
                continue;
            }
            const uint64_t take = (J - j) < n ? (J - j) : n;
            lastT = T + (take - 1u) * (60u / n);
            T += (uint64_t)n * (60u / n);
            j += take;
        } else {
            if (n) lastT = T;
            j += n;
            T += 1u;
        }
    }
    last[c] = lastT;
}

// The same bound, one wave per cluster, in 64-bit time: windows of 64 periods (lane l = period
// pw + l) are prefix-summed as in GenStream::fill until the window holding job J-1, whose lane is
// the first with an inclusive count above J-1-jw; WEIBULL sums the gaps of jobs 0..J-2, 64 a step.
__global__ __launch_bounds__(256) void gen_bound_wave_kernel(const uint64_t* job_off, uint32_t n_clusters,
                                                            GenArgs g, unsigned long long* last) {
    const uint32_t c = blockIdx.x * (256u / kWave) + threadIdx.x / kWave;
    const uint32_t lane = threadIdx.x % kWave;
    if (c >= n_clusters) return;  // wave-uniform
    const uint64_t J = job_off[c + 1] - job_off[c];
    const uint64_t akey = mcs_arrival_key(mcs_cluster_key(g.seed, g.base + c));
    uint64_t T = 0;
    if (g.mode == 2u) {
        for (uint64_t b = 0; b + 1u < J; b += kWave) {
            const uint32_t gap = b + lane + 1u < J
                                     ? mcs_weibull_gap(mcs_draw(akey, b + lane), (const uint64_t*)g.wthr, g.wn)
                                     : 0u;
            T += readlane(wave_incl_sum_u32(gap, lane), 63);  // 64 gaps < 2^32 (table length bound)
        }
        if (lane == 0) last[c] = T;
        return;
    }
    uint64_t pw = 0, jw = 0;
    while (J != 0) {
        const uint32_t n = mcs_poisson(akey, pw + lane, g.enl);
        const uint32_t d = g.mode == 0u ? (n == 0u ? 60u : n * (60u / n)) : 1u;
        const uint32_t cum = wave_incl_sum_u32(n, lane);
        const uint32_t dinc = wave_incl_sum_u32(d, lane);
        const uint32_t tot = readlane(cum, 63);
        if (jw + tot >= J) {  // job J-1 lies in this window
            const uint32_t rel = (uint32_t)(J - 1u - jw);
            const uint32_t lo = (uint32_t)__builtin_ctzll(__ballot(cum > rel));
            const uint32_t np = (uint32_t)__shfl((int)n, (int)lo);
            const uint32_t cp = (uint32_t)__shfl((int)cum, (int)lo);
            const uint32_t te = (uint32_t)__shfl((int)(dinc - d), (int)lo);
            const uint64_t lt = g.mode == 0u ? T + te + (uint64_t)(rel - (cp - np)) * (60u / np) : T + lo;
            if (lane == 0) last[c] = lt;
            return;
        }
        jw += tot;
        T += readlane(dinc, 63);
        pw += kWave;
    }
    if (lane == 0) last[c] = 0u;
}

hipError_t launch_gen_bound(const uint64_t* job_off, uint32_t n_clusters, const GenArgs& g,
                            unsigned long long* last, hipStream_t s) {
    if (n_clusters == 0) return hipSuccess;
    const char* serial = getenv("MCS_GEN_SERIAL");  // the per-thread scan (tests compare the forms)
    if (!(serial && atoi(serial) != 0)) {
        const uint32_t per = 256u / kWave;
        hipLaunchKernelGGL(gen_bound_wave_kernel, dim3((n_clusters + per - 1) / per), dim3(256), 0, s, job_off,
                           n_clusters, g, last);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(gen_bound_kernel, dim3((n_clusters + 63) / 64), dim3(64), 0, s, job_off, n_clusters, g,
                       last);
    return hipGetLastError();
}

hipError_t launch_gen_attrs(uint4* jobs, const uint64_t* job_off, const uint32_t* max_c,
                            const uint32_t* max_m, uint32_t n_clusters, uint64_t seed,
                            uint32_t max_dur, uint32_t base, hipStream_t s) {
    if (n_clusters == 0) return hipSuccess;
    hipLaunchKernelGGL(gen_attrs_kernel, dim3(64, n_clusters), dim3(256), 0, s, jobs, job_off,
                       max_c, max_m, seed, max_dur, base);
    return hipGetLastError();
}

// Whole records, one wave per cluster: the fused kernels' batch generator (GenStream) writing its
// batches out.  The per-thread arrival scan above walks a cluster's stream serially (one lane per
// cluster, 64 clusters per wave: 9.5 ms for C4); the wave form draws 64 periods and 64 jobs at a
// time.  Its 32-bit job counters need every cluster below 2^32 jobs (the caller checks).
__global__ __launch_bounds__(256) void gen_stream_kernel(uint4* jobs, const uint64_t* job_off,
                                                        uint32_t n_clusters, GenArgs g) {
    const uint32_t c = blockIdx.x * (256u / kWave) + threadIdx.x / kWave;
    const uint32_t lane = threadIdx.x % kWave;
    if (c >= n_clusters) return;  // wave-uniform
    const uint64_t j0 = job_off[c];
    const uint32_t J = (uint32_t)(job_off[c + 1] - j0);
    GenStream gs;
    gs.init(g, c, lane);
    for (uint32_t b = 0; b < J; b += kWave) {
        const uint4 rec = gs.next(b, lane);
        if (b + lane < J) jobs[j0 + b + lane] = rec;
    }
}

hipError_t launch_gen_stream(uint4* jobs, const uint64_t* job_off, uint32_t n_clusters, const GenArgs& g,
                             hipStream_t s) {
    if (n_clusters == 0) return hipSuccess;
    const uint32_t per = 256u / kWave;
    hipLaunchKernelGGL(gen_stream_kernel, dim3((n_clusters + per - 1) / per), dim3(256), 0, s, jobs, job_off,
                       n_clusters, g);
    return hipGetLastError();
}

hipError_t launch_gen_arrivals(uint4* jobs, const uint64_t* job_off, uint32_t n_clusters, const GenArgs& g,
                               hipStream_t s) {
    if (n_clusters == 0) return hipSuccess;
    hipLaunchKernelGGL(gen_arrivals_kernel, dim3((n_clusters + 63) / 64), dim3(64), 0, s, jobs, job_off,
                       n_clusters, g);
    return hipGetLastError();
}

// ---- single-job mirrors over the live state ---------------------------------------------------
// ScheduleJob (scheduler.go:127-139) + synchronous commit (cluster.go:146-147)
__global__ __launch_bounds__(64) void schedule_one_kernel(uint32_t* live_c, uint32_t* live_m,
                                                         uint32_t n, uint32_t c, uint32_t m,
                                                         int32_t* out) {
    const uint32_t lane = threadIdx.x;
    int found = -1;
    for (uint32_t b = 0; b < n && found < 0; b += kWave) {
        const uint32_t i = b + lane;
        const bool fit = i < n && live_c[i] >= c && live_m[i] >= m;
        const uint64_t hit = __ballot(fit);
        if (hit) found = (int)(b + (uint32_t)__builtin_ctzll(hit));
    }
    if (lane == 0) {
        if (found >= 0) {
            live_c[found] -= c;
            live_m[found] -= m;
        }
        *out = found;
    }
}

// Lend (scheduler.go:194-202): strict '>' existence, no commit
__global__ __launch_bounds__(64) void lend_kernel(const uint32_t* live_c, const uint32_t* live_m,
                                                 uint32_t n, uint32_t c, uint32_t m,
                                                 int32_t* out) {
    const uint32_t lane = threadIdx.x;
    bool any = false;
    for (uint32_t b = 0; b < n; b += kWave) {
        const uint32_t i = b + lane;
        any = any || (i < n && live_c[i] > c && live_m[i] > m);
    }
    const uint64_t hit = __ballot(any);
    if (lane == 0) *out = hit ? 1 : 0;
}

// GetResourceUtilization (cluster.go:46-63): float32 accumulation in node order — a serial
// dependency chain by definition, so one lane walks it (this is a mirror, not a hot op).
__global__ void utilization_kernel(const uint2* cap, const uint32_t* live_c,
                                   const uint32_t* live_m, uint32_t n, float* out2) {
    if (threadIdx.x != 0) return;
    float cu = 0.0f, mu = 0.0f;
    uint32_t tc = 0, tm = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const float a = __fsub_rn((float)cap[i].x, (float)live_c[i]);
        const float b = __fsub_rn((float)cap[i].y, (float)live_m[i]);
        cu = __fadd_rn(cu, a);
        mu = __fadd_rn(mu, b);
        tc += cap[i].x;  // SetTotalResources: uint32 sums (cluster.go:34-37)
        tm += cap[i].y;
    }
    out2[0] = __fdiv_rn(cu, (float)tc);
    out2[1] = __fdiv_rn(mu, (float)tm);
}

hipError_t launch_schedule_one(uint32_t* live_c, uint32_t* live_m, uint32_t n, uint32_t c,
                               uint32_t m, int32_t* out_node, hipStream_t s) {
    hipLaunchKernelGGL(schedule_one_kernel, dim3(1), dim3(kWave), 0, s, live_c, live_m, n, c, m,
                       out_node);
    return hipGetLastError();
}

hipError_t launch_lend_check(const uint32_t* live_c, const uint32_t* live_m, uint32_t n,
                             uint32_t c, uint32_t m, int32_t* out_ok, hipStream_t s) {
    hipLaunchKernelGGL(lend_kernel, dim3(1), dim3(kWave), 0, s, live_c, live_m, n, c, m, out_ok);
    return hipGetLastError();
}

hipError_t launch_utilization(const uint2* cap, const uint32_t* live_c, const uint32_t* live_m,
                              uint32_t n, float* out2, hipStream_t s) {
    hipLaunchKernelGGL(utilization_kernel, dim3(1), dim3(kWave), 0, s, cap, live_c, live_m, n,
                       out2);
    return hipGetLastError();
}

}  // namespace mcs

#ifdef MCS_STAMPS
// sums [decide, place, release, reload, passes, releasing passes, deciding passes, -]; reset after read
extern "C" int mcs_debug_stamps(unsigned long long* out) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(g_stamps)) != hipSuccess) return -1;
    unsigned long long z[8] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
