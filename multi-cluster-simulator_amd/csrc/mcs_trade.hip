// mcs_trade.hip — gfx950 kernels of the lock-step trading path (mcs_trade.h).
//
// One tick of the lock-step semantics is three launches on the engine stream, each a kernel
// boundary (= grid-wide barrier), with ONE exchange: on N GPUs an RCCL all-gather of the ranks'
// blocks (post-A records + node snapshots) between A and B; B, C and D then run replicated on
// every rank over the whole system, so they need nothing more from the other ranks:
//   A tr_step_kernel    one wave per local cluster: releases, arrivals, the Fifo decisions of the
//                       tick (scheduler.go:216-296), the tick's borrow request (server.go:160-248),
//                       the float32 utilization sample (cluster.go:46-63) on trader ticks; then
//                       the cluster's exchange record and node snapshot
//   B tr_lend_kernel    one wave per cluster of the system as lender: Lend (strict '>',
//                       scheduler.go:194-202) on its snapshot against every request of the tick,
//                       in borrower order; the owner rank appends to its LentQueue
//   C (in the trader kernel) one lane per cluster of the system as borrower: BorrowedQueue move
//                       when some lender accepted (scheduler.go:237-242, owner rank); clock hints
//   D tr_trader_kernel  one wave for the whole system: trader rounds in cluster order
//                       (trader.go:280-325, 193-278; server.go:31-85) with the responders
//                       evaluated across lanes, then the next tick (fast-forward)
// Work per tick is a handful of decisions per cluster: the path is launch/latency-bound, so the
// engine replays the four launches from a captured hipGraph.  Within a kernel the per-cluster
// state a wave both writes and re-reads (node free vectors, slot finish times, trader locks) is
// staged in LDS: an L2 atomic or store followed by a plain global load of the same line from the
// same wave could be served stale by the non-coherent vector L1.
#include "mcs_trade_internal.h"
#include "mcs_trader_dev.h"
#include "mcs_wave.h"

namespace mcs {
namespace {

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o);
    return v;
}

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x; }

// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void tr_init_kernel(TradeArgs a) {
    const uint32_t c = blockIdx.x, lane = lane_id();
    const uint32_t n0 = a.node_off[c], N = a.node_off[c + 1] - n0;
    uint32_t sc = 0, sm = 0;
    for (uint32_t i = lane; i < N; i += kWave) {
        const uint2 f = a.free0[n0 + i];
        a.tn[n0 + i] = (unsigned long long)f.x | ((unsigned long long)f.y << 32);
        const uint2 cp = a.cap[n0 + i];
        sc += cp.x;  // uint32 sums, wrapping like SetTotalResources (cluster.go:34-37)
        sm += cp.y;
    }
    sc = wave_sum_u32(sc);
    sm = wave_sum_u32(sm);
    for (uint32_t s = lane; s < a.S; s += kWave) a.sfin[(size_t)c * a.S + s] = kEmpty;
    const uint64_t j0 = a.job_off[c], j1 = a.job_off[c + 1];
    for (uint64_t j = j0 + lane; j < j1; j += kWave) {
        a.out_node[j] = MCS_NODE_UNPLACED;
        a.out_start[j] = MCS_TIME_NONE;
        a.out_finish[j] = MCS_TIME_NONE;
    }
    if (lane == 0) {
        TrCluster z{};
        z.minf = kEmpty;
        z.total_c = sc;
        z.total_m = sm;
        a.cl[c] = z;
    }
    if (c == 0) {
        for (uint32_t g = lane; g < a.Ct; g += kWave) {
            TrTrader t{};
            t.next_id = 1u;  // s.id = rand.Uint32() (pkg/trader/server.go:26), seeded: 1
            a.tr[g] = t;
            a.acc[g] = 0u;
        }
        if (lane == 0) {
            TrCtl z{};
            *a.ctl = z;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Phase A: the cluster's scheduler step at tick T.
__global__ __launch_bounds__(64) void tr_step_kernel(TradeArgs a) {
    __shared__ unsigned long long nodes[kTrMaxNodes];
    __shared__ uint32_t sfin[kTrMaxSlots];
    if (a.ctl->done) return;
    const uint32_t T = a.ctl->T;
    const uint32_t c = blockIdx.x, lane = lane_id(), g = a.base + c;
    const uint32_t n0 = a.node_off[c], N = a.node_off[c + 1] - n0;
    const uint64_t j0 = a.job_off[c];
    const uint32_t J = (uint32_t)(a.job_off[c + 1] - j0);
    const uint4* __restrict__ jobs = a.jobs + j0;
    const size_t sb = (size_t)c * a.S;
    const uint32_t S = a.S;
    const uint32_t vn = a.tr[g].vnodes;
    TrCluster st = a.cl[c];

    copy_rounds<4>(nodes, a.tn + n0, N, lane);
    copy_rounds<8>(sfin, a.sfin + sb, S, lane);
    __syncthreads();

    // releases due at T (cluster.go:153-157), before the tick's decisions
    if (st.minf <= T) {
        uint32_t lm = kEmpty, nrel = 0;
        for (uint32_t s = lane; s < S; s += kWave) {
            const uint32_t f = sfin[s];
            if (f <= T) {
                const uint32_t nd = a.snode[sb + s];
                if (nd < N) atomicAdd(&nodes[nd], a.scm[sb + s]);
                sfin[s] = kEmpty;
                ++nrel;
            } else {
                lm = f < lm ? f : lm;
            }
        }
        st.nrun -= wave_sum_u32(nrel);
        st.minf = wave_min_u32(lm);
        __syncthreads();
    }
    // arrivals up to T join the ReadyQueue (jobs are sorted by arrival)
    while (st.next_arr < J) {
        const uint32_t i = st.next_arr + lane;
        const bool ok = i < J && jobs[i].x <= T;
        const uint32_t n = (uint32_t)__builtin_popcountll(__ballot(ok));
        st.next_arr += n;
        if (n < (uint32_t)kWave) break;
    }

    // ScheduleJob (scheduler.go:127-139): lowest node with both >=; zero-capacity virtual nodes
    // (AddVirtualNode, cluster.go:79) follow the physical ones
    auto first_fit = [&](uint32_t jc, uint32_t jm) -> uint32_t {
        uint32_t best = kEmpty;
        for (uint32_t b = 0; b < N; b += kWave) {
            const uint32_t i = b + lane;
            if (i < N) {
                const unsigned long long v = nodes[i];
                if ((uint32_t)v >= jc && (uint32_t)(v >> 32) >= jm) best = i;
            }
            if (__ballot(best != kEmpty)) break;
        }
        uint32_t k = wave_min_u32(best);
        if (k == kEmpty && jc == 0u && jm == 0u && vn > 0u) k = N;
        return k;
    };
    // Node.RunJob commit (cluster.go:144-148) + running-slot insert; false on slot overflow
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
            if (k < N) atomicSub(&nodes[k], need);
            sfin[slot] = fin;
            a.snode[sb + slot] = k;
            a.scm[sb + slot] = need;
        }
        __syncthreads();
        ++st.nrun;
        st.peak = st.nrun > st.peak ? st.nrun : st.peak;
        st.minf = fin < st.minf ? fin : st.minf;
        return true;
    };
    auto place_own = [&](uint32_t j, uint32_t k, uint4 jb) -> bool {
        const uint32_t fin = T + jb.y;
        if (jb.y != 0u && !commit(k, jb.z, jb.w, fin)) return false;
        if (lane == 0) {
            a.out_node[j0 + j] = (int32_t)k;
            a.out_start[j0 + j] = T;
            a.out_finish[j0 + j] = fin;
        }
        ++st.placed;
        ++st.decided;
        return true;
    };

    TrRecA req{kEmpty, 0u, 0u, 0u};
    for (;;) {
        if (st.has_w) {  // WaitQueue head (scheduler.go:219-251)
            const uint4 jb = jobs[st.w];
            const uint32_t k = first_fit(jb.z, jb.w);
            if (k != kEmpty) {
                if (!place_own(st.w, k, jb)) {
                    st.flags |= MCS_FLAG_OVERFLOW;
                    break;
                }
                st.has_w = 0u;
            } else if (a.borrow) {
                req = TrRecA{st.w, jb.z, jb.w, jb.y};  // BorrowResources (:234)
            }
            break;  // time.Sleep(1 s), :250
        }
        if (st.rq_head < st.next_arr) {  // ReadyQueue head (:255-272), no sleep
            const uint32_t j = st.rq_head++;
            const uint4 jb = jobs[j];
            const uint32_t k = first_fit(jb.z, jb.w);
            if (k != kEmpty) {
                if (!place_own(j, k, jb)) {
                    st.flags |= MCS_FLAG_OVERFLOW;
                    break;
                }
            } else {
                st.has_w = 1u;
                st.w = j;
                ++st.waited;
            }
            continue;
        }
        if (st.lq_len > 0u) {  // LentQueue head (:277-290)
            const TrLq e = a.lq[(size_t)c * a.LQ + st.lq_head];
            const uint32_t k = first_fit(e.c, e.m);
            if (k != kEmpty) {
                const uint32_t fin = T + e.dur;
                if (e.dur != 0u && !commit(k, e.c, e.m, fin)) {
                    st.flags |= MCS_FLAG_OVERFLOW;
                    break;
                }
                if (lane == 0) {
                    const unsigned long long idx = atomicAdd(&a.ctl->n_lent, 1ull);
                    if (idx < a.lent_cap) {
                        mcs_lent_rec r;
                        r.lender = g;
                        r.borrower = e.borrower;
                        r.job = e.job;
                        r.node = k;
                        r.start_s = T;
                        r.finish_s = fin;
                        r.pad = 0u;
                        a.lent_log[idx] = r;
                    }
                }
                ++st.lent_runs;
                st.lq_head = st.lq_head + 1u == a.LQ ? 0u : st.lq_head + 1u;
                --st.lq_len;
            }
            break;  // sleep 1 s (:289)
        }
        break;  // idle sleep (:294)
    }

    __syncthreads();
    // GetResourceUtilization (cluster.go:46-63) when a trader reads it at this tick: the state
    // stream samples every sample_period_s (trader_server.go:24-47) and trader rounds fall on
    // multiples of the period, so the sample a round reads is the one taken at its own tick
    // (phases B-C do not change node counters)
    if (a.trader && T % a.sample_period == 0u) {
        bool due = false;
        for (uint32_t q = lane; q < a.Ct; q += kWave) due = due || a.tr[q].next_due <= T;
        if (__ballot(due)) {
            __shared__ float dcs[kTrMaxNodes], dms[kTrMaxNodes];
            for (uint32_t i = lane; i < N; i += kWave) {
                const unsigned long long v = nodes[i];
                const uint2 cp = a.cap[n0 + i];
                dcs[i] = __fsub_rn((float)cp.x, (float)(uint32_t)v);
                dms[i] = __fsub_rn((float)cp.y, (float)(uint32_t)(v >> 32));
            }
            __syncthreads();
            if (lane == 0) {
                float sc = 0.0f, sm = 0.0f;
                for (uint32_t i = 0; i < N; ++i) {  // node order, float32 (Go)
                    sc = __fadd_rn(sc, dcs[i]);
                    sm = __fadd_rn(sm, dms[i]);
                }
                st.cu = __fdiv_rn(sc, (float)st.total_c);
                st.mu = __fdiv_rn(sm, (float)st.total_m);
            }
            st.cu = __shfl(st.cu, 0);
            st.mu = __shfl(st.mu, 0);
        }
    }
    unsigned long long* snap = tr_snap(a, g);
    copy_rounds<4>(a.tn + n0, nodes, N, lane);
    copy_rounds<4>(snap, nodes, N, lane);
    copy_rounds<8>(a.sfin + sb, sfin, S, lane);
    if (lane == 0) {
        a.cl[c] = st;
        TrXRec x;
        x.req = req;
        x.n = N;
        x.has_w = st.has_w;
        x.lq_len = st.lq_len;
        x.rq_busy = st.rq_head < st.next_arr ? 1u : 0u;
        x.decided = st.decided;
        x.J = J;
        x.next_arr_t = st.next_arr < J ? jobs[st.next_arr].x : kEmpty;
        x.flags = st.flags;
        x.cu = st.cu;
        x.mu = st.mu;
        x.total_c = st.total_c;
        x.total_m = st.total_m;
        *tr_xrec(a, g) = x;
    }
}

// ---------------------------------------------------------------------------------------------
// Phase B: cluster L of the system as lender, requests in borrower order ("/borrow",
// server.go:80-113), on L's post-A snapshot.  Every rank runs it for every lender, so the
// acceptances (acc) and LentQueue lengths (lqp) are replicated; only L's owner appends.
__global__ __launch_bounds__(64) void tr_lend_kernel(TradeArgs a) {
    __shared__ unsigned long long sn[kTrMaxNodes];
    if (a.ctl->done) return;
    const uint32_t L = blockIdx.x, lane = lane_id();
    const bool own = L / a.Cl == a.rank;
    const uint32_t c = L - a.rank * a.Cl;  // (own only)
    // every read of the tick issued together (one round trip): the first 64 borrowers' requests
    // (one per lane), the lender's snapshot — the whole stride, since its node count arrives only
    // with its record — staged once for every request, and the record
    TrRecA rl0{kEmpty, 0u, 0u, 0u};
    if (lane < a.Ct && lane != L) rl0 = tr_xrec(a, lane)->req;  // self skipped (:176)
    copy_rounds<4>(sn, tr_snap(a, L), a.ns, lane);
    const TrXRec xl = *tr_xrec(a, L);
    const uint32_t N = xl.n;
    __syncthreads();
    uint32_t lq_len = xl.lq_len, lq_head = own ? a.cl[c].lq_head : 0u, fb = 0;
    const uint32_t LQ = a.LQ;
    for (uint32_t b0 = 0; b0 < a.Ct; b0 += kWave) {
        const uint32_t bl = b0 + lane;
        // this block of 64 borrowers' requests, one per lane, broadcast per pending request
        TrRecA rl = rl0;
        if (b0 != 0u) {
            rl = TrRecA{kEmpty, 0u, 0u, 0u};
            if (bl < a.Ct && bl != L) rl = tr_xrec(a, bl)->req;  // self skipped (:176)
        }
        unsigned long long pend = __ballot(rl.job != kEmpty);
        while (pend) {
            const uint32_t bi = (uint32_t)__builtin_ctzll(pend);
            const uint32_t b = b0 + bi;
            pend &= pend - 1ull;
            const TrRecA r{readlane(rl.job, bi), readlane(rl.c, bi), readlane(rl.m, bi), readlane(rl.dur, bi)};
            bool ok = false;
            for (uint32_t i0 = 0; i0 < N; i0 += kWave) {
                const uint32_t i = i0 + lane;
                if (i < N) {
                    const unsigned long long v = sn[i];
                    ok = ok || ((uint32_t)v > r.c && (uint32_t)(v >> 32) > r.m);
                }
                if (__ballot(ok)) break;
            }
            if (!__ballot(ok)) continue;  // "can't lend" (scheduler.go:201)
            if (lq_len >= LQ) {
                fb |= MCS_FLAG_LENT_OVERFLOW;
                continue;
            }
            if (lane == 0) {
                if (own) {
                    uint32_t at = lq_head + lq_len;
                    at = at >= LQ ? at - LQ : at;
                    TrLq e{};
                    e.borrower = b;
                    e.job = r.job;
                    e.c = r.c;
                    e.m = r.m;
                    e.dur = r.dur;
                    a.lq[(size_t)c * LQ + at] = e;
                }
                a.acc[b] = 1u;  // (every accepting lender writes the same value)
            }
            ++lq_len;
        }
    }
    if (lane == 0) {
        a.lqp[L] = lq_len;
        a.fb[L] = fb;
        if (own) {
            a.cl[c].lq_len = lq_len;
            a.cl[c].flags |= fb;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Phase C: cluster g of the system as borrower (the owner rank moves the job) and its clock
// hints for the trader phase; run by one lane of the trader wave per cluster (replicated).
__device__ __forceinline__ TrRecC post_cluster(const TradeArgs& a, uint32_t g, uint32_t T) {
    // every input read first (one round trip): the record, the acceptance, the LentQueue length
    // and the lender flags
    const TrXRec x = *tr_xrec(a, g);
    const uint32_t accg = a.acc[g], lq = a.lqp[g], fbg = a.fb[g];
    const bool own = g / a.Cl == a.rank;
    uint32_t has_w = x.has_w, decided = x.decided;
    if (x.req.job != kEmpty && accg) {  // BorrowedQueue append, WaitQueue pop (scheduler.go:237-242)
        has_w = 0u;
        ++decided;
        if (own) {
            const uint32_t c = g - a.rank * a.Cl;
            const uint64_t j0 = a.job_off[c];
            a.out_node[j0 + x.req.job] = MCS_NODE_BORROWED;
            a.out_start[j0 + x.req.job] = T;
            a.out_finish[j0 + x.req.job] = MCS_TIME_NONE;
            TrCluster st = a.cl[c];
            st.has_w = 0u;
            ++st.decided;
            ++st.borrowed;
            a.cl[c] = st;
        }
    }
    a.acc[g] = 0u;  // (only this lane reads it; cleared for the next tick)
    TrRecC o;
    o.cu = x.cu;
    o.mu = x.mu;
    o.total_c = x.total_c;
    o.total_m = x.total_m;
    o.busy = (has_w || lq > 0u || x.rq_busy) ? 1u : 0u;
    o.next_arr_t = x.next_arr_t;
    o.done = (decided == x.J && lq == 0u) ? 1u : 0u;
    o.flags = x.flags | fbg;
    return o;
}

// ---------------------------------------------------------------------------------------------
// ApproveTrade (trader.go:141-167) of the contract {cores 0, mem 0, time 0 s, price 0} that every
// FIFO trade carries (the small-node contract over an empty Level1), on the responder's sample:
// mcs_trader_dev.h's function, shared with the DELAY trader and the mcs_approve_trade mirror.
__device__ __forceinline__ bool approve_zero_contract(uint32_t tc, uint32_t tm, float cu, float mu) {
    return approve_trade_dev(tc, tm, cu, mu, 0u, 0u, 0u);
}

// Phases C and D: every cluster's borrower step and sample record (one lane each), then the
// trader rounds (replicated) and the next tick.
__global__ __launch_bounds__(64) void tr_trader_kernel(TradeArgs a) {
    __shared__ TrTrader trs[kTrMaxClusters];
    __shared__ TrRecC rcs[kTrMaxClusters];
    if (a.ctl->done) return;
    const uint32_t T = a.ctl->T;
    const uint32_t lane = lane_id();
    const uint32_t Ct = a.Ct;
    for (uint32_t q = lane; q < Ct; q += kWave) {
        trs[q] = a.tr[q];
        rcs[q] = post_cluster(a, q, T);
    }
    __syncthreads();
    unsigned long long n_trades = a.ctl->n_trades, n_won = a.ctl->n_won;
    uint32_t lflags = 0;

    if (a.trader) {
        for (uint32_t q0 = 0; q0 < Ct; q0 += kWave) {
            const uint32_t ql = q0 + lane;
            unsigned long long due = __ballot(ql < Ct && trs[ql].next_due <= T);
            while (due) {  // RequestPolicyMonitor of requester q (trader.go:282-324), index order
                const uint32_t q = q0 + (uint32_t)__builtin_ctzll(due);
                due &= due - 1ull;
                const TrRecC rq = rcs[q];
                // policies [WaitTime, Utilization] (trader.go:55-62): WaitTime never breaks under
                // FIFO (its average is only fed by /delay); Utilization (trader.go:127-130)
                const bool broken = rq.cu > 0.8f || rq.mu > 0.8f;
                if (!broken) {
                    if (lane == 0) trs[q].next_due = T + a.period;
                    __syncthreads();
                    continue;
                }
                // Trade (trader.go:193-278): RequestResource to every other trader, index order
                uint32_t napp = 0, winner = kEmpty;
                for (uint32_t r0 = 0; r0 < Ct; r0 += kWave) {
                    const uint32_t r = r0 + lane;
                    bool app = false;
                    if (r < Ct && r != q) {
                        TrTrader t = trs[r];
                        if (t.lock_id != 0u && T >= t.lock_until) t.lock_id = 0u;  // 20 s expiry
                        if (t.lock_id == 0u) {  // else Approve:false (server.go:35-40)
                            const TrRecC rr = rcs[r];
                            app = approve_zero_contract(rr.total_c, rr.total_m, rr.cu, rr.mu);
                            t.lock_id = t.next_id++;  // set even when not approving (:44-46)
                            t.lock_until = T + a.lock_s;
                        }
                        trs[r] = t;
                    }
                    const unsigned long long ab = __ballot(app);
                    napp += (uint32_t)__builtin_popcountll(ab);
                    // every response echoes the requester's price (server.go:44): the Go heap of
                    // equal keys pops the first push first (Appendix C), whose lock still matches
                    // (nothing intervenes), and the zero allocation cannot fail -> first approver
                    if (winner == kEmpty && ab) winner = r0 + (uint32_t)__builtin_ctzll(ab);
                }
                __syncthreads();
                if (lane == 0) {
                    if (winner != kEmpty) {
                        trs[winner].lock_id = 0u;  // ApproveContract resets currentContract (:83)
                        trs[q].vnodes += 1u;       // AddVirtualNode(0 cores, 0 memory)
                        ++n_won;
                    }
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
                    trs[q].next_due = T + (winner != kEmpty ? a.ok_sleep : a.fail_sleep) + a.period;
                }
                ++n_trades;
                __syncthreads();
            }
        }
    }

    // the next tick: T+1 while any queue is busy, else the next arrival or trader round
    bool all_done = true, busy = false;
    uint32_t nxt = kEmpty, fl = 0;
    for (uint32_t q = lane; q < Ct; q += kWave) {
        const TrRecC rc = rcs[q];
        all_done = all_done && rc.done;
        busy = busy || rc.busy;
        nxt = rc.next_arr_t < nxt ? rc.next_arr_t : nxt;
        if (a.trader) nxt = trs[q].next_due < nxt ? trs[q].next_due : nxt;
        fl |= rc.flags;
    }
    const bool done_all = !__ballot(!all_done);
    const bool busy_any = __ballot(busy) != 0ull;
    nxt = wave_min_u32(nxt);
    for (int o = 32; o > 0; o >>= 1) fl |= (uint32_t)__shfl_xor((int)fl, o);
    __syncthreads();
    for (uint32_t q = lane; q < Ct; q += kWave) a.tr[q] = trs[q];
    if (lane == 0) {
        TrCtl* ctl = a.ctl;
        uint32_t flags = ctl->flags | fl | lflags;
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
        ctl->T = Tn;
        ctl->done = done;
        ctl->ticks += 1u;
        ctl->flags = flags;
        ctl->n_trades = n_trades;
        ctl->n_won = n_won;
    }
}

}  // namespace

hipError_t launch_trade_init(const TradeArgs& a, hipStream_t s) {
    if (a.Cl == 0) return hipSuccess;
    hipLaunchKernelGGL(tr_init_kernel, dim3(a.Cl), dim3(kWave), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_trade_phase(const TradeArgs& a, int phase, hipStream_t s) {
    switch (phase) {
        case 0:
            hipLaunchKernelGGL(tr_step_kernel, dim3(a.Cl), dim3(kWave), 0, s, a);
            break;
        case 1:
            hipLaunchKernelGGL(tr_lend_kernel, dim3(a.Ct), dim3(kWave), 0, s, a);
            break;
        case 2:  // (phase C runs inside the trader kernel)
            return hipSuccess;
        case 3:
            hipLaunchKernelGGL(tr_trader_kernel, dim3(1), dim3(kWave), 0, s, a);
            break;
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace mcs
