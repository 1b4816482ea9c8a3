// mcs_dtrade_res.hip — the lock-step DELAY trading system resident on one CU.
//
// The graph-replayed tick (mcs_dtrade.hip) is two dependent launches per tick that re-stage every
// cluster's node vector, running slots and state through HBM: ~20 us per tick on C5-DELAY (64
// cluster_small clusters), most of it launch seams and HBM round trips for a few hundred
// instructions of work.  For one-engine systems that fit one CU's LDS (world 1, at most 64
// clusters of at most 64 physical nodes) this kernel keeps the whole system on chip for up to
// `budget` ticks per launch:
//   * one workgroup of 16 waves; wave w runs phase A (one Delay iteration, scheduler.go:298-369, and
//     the phase-C sample, trader_server.go:24-47) of clusters w, w + 16, w + 32, w + 48 on their
//     LDS-resident state (DtCluster, nodes physical then virtual, running-slot finish times; the
//     slots' node and payload words and the Level1 lists stay in HBM);
//   * s_barrier, then wave 0 runs phase D (the trader rounds, trader.go:280-325, with ApproveTrade,
//     the Go heap order and AllocateVirtualNodeResources, cluster.go:87-125) on the same LDS
//     records and nodes — with one engine the responder's snapshot IS its live node vector;
//   * s_barrier, the next tick.
// The code of both phases is mcs_dtrade.hip's (same statements, same order), with HBM staging
// replaced by the resident arrays and __syncthreads of a one-wave workgroup by a wave-local LDS
// fence.  Bit-exact against the replayed kernels and the oracle (tests/test_gpu_dtrade.py).
#include "mcs_dtrade_internal.h"
#include "mcs_trader_dev.h"
#include "mcs_wave.h"

namespace mcs {
namespace {

constexpr uint32_t kDrWaves = 16;
constexpr uint32_t kDrMaxClusters = 64;
constexpr uint32_t kDrMaxNodes = 64;  // physical nodes per cluster

// LDS order of one wave's lanes among themselves (the wave is not the workgroup here)
__device__ __forceinline__ void wsync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

__device__ __forceinline__ uint32_t dr_sum_u32(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o);
    return v;
}
__device__ __forceinline__ long long dr_sum_i64(long long v) {
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)(unsigned long long)v, o);
        const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)((unsigned long long)v >> 32), o);
        v += (long long)((unsigned long long)lo | ((unsigned long long)hi << 32));
    }
    return v;
}
__device__ __forceinline__ uint32_t dr_max_u32(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t w = (uint32_t)__shfl_xor((int)v, o);
        v = w > v ? w : v;
    }
    return v;
}
__device__ __forceinline__ unsigned long long dr_go_u64(uint32_t x) {
    return (unsigned long long)(long long)(int32_t)x;
}
__device__ __forceinline__ float dr_go_f32(uint32_t x) { return (float)dr_go_u64(x); }
__device__ __forceinline__ double dr_go_f64(uint32_t x) { return (double)dr_go_u64(x); }
__device__ __forceinline__ unsigned long long dr_f64_to_u64(double x) {
    const double two63 = 9223372036854775808.0;
    if (x < two63) return (unsigned long long)(long long)x;
    const double y = x - two63;
    if (y >= two63) return 0ull;
    return (unsigned long long)(long long)y ^ 0x8000000000000000ull;
}
// HBM words this kernel writes and re-reads (Level1 rows, slot payloads, virtual-node capacities):
// read through L2 (agent scope), never a stale line of this CU's vector L1, after the writer's
// agent-scope release fence and a barrier
__device__ __forceinline__ unsigned long long dr_ld64(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t dr_ld32(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the resident state, in dynamic LDS (dtrade_res_lds gives its size)
struct DrShared {
    DtCtl ctl;
    uint32_t period_due;  // (pad)
    uint32_t pad[3];
    DtCluster cl[kDrMaxClusters];
    DtRec rec[kDrMaxClusters];
    DtTrader trs[kDrMaxClusters];
    uint32_t appr[kDrMaxClusters];
    uint32_t nvs[kDrMaxClusters];
    uint32_t nfr[kDrMaxClusters];
    uint32_t hist[kDrWaves][kWave];
};
static_assert(sizeof(DrShared) % 8 == 0, "the node array follows DrShared at an 8-byte boundary");
// then: unsigned long long nodes[Ct][W] (W = NS + V, physical then virtual, contiguous);
//       uint32_t sfin[Ct][S]; float samp[kDrWaves][2 * W]

size_t dr_lds(uint32_t Ct, uint32_t W, uint32_t S) {
    return sizeof(DrShared) + (size_t)Ct * W * 8u + (size_t)Ct * S * 4u + (size_t)kDrWaves * 2u * W * 4u;
}

__global__ __launch_bounds__(kDrWaves * kWave) void dt_res_kernel(DtArgs a, uint32_t budget) {
    extern __shared__ unsigned long long dr_smem[];
    DrShared& sh = *reinterpret_cast<DrShared*>(dr_smem);
    const uint32_t W = a.W, S = a.S, Ct = a.Ct;
    unsigned long long* const NODES = dr_smem + sizeof(DrShared) / 8u;
    uint32_t* const SFIN = reinterpret_cast<uint32_t*>(NODES + (size_t)Ct * W);
    float* const SAMP = reinterpret_cast<float*>(SFIN + (size_t)Ct * S);
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;

    // ---- load the system (written by dt_init_kernel or the previous launch) ----
    for (uint32_t i = threadIdx.x; i < Ct; i += blockDim.x) {
        sh.cl[i] = a.cl[i];
        sh.trs[i] = a.tr[i];
        sh.nvs[i] = a.nv_all[i];
    }
    if (threadIdx.x == 0) sh.ctl = *a.ctl;
    for (uint32_t c = wave; c < Ct; c += kDrWaves) {
        const uint32_t n0 = a.node_off[c], N = a.node_off[c + 1] - n0;
        const uint32_t nv = a.cl[c].nv;
        for (uint32_t i = lane; i < N; i += kWave) NODES[(size_t)c * W + i] = a.tn[n0 + i];
        for (uint32_t i = lane; i < nv && i < a.V; i += kWave)
            NODES[(size_t)c * W + N + i] = a.vn[(size_t)c * a.V + i];
        for (uint32_t s = lane; s < S; s += kWave) SFIN[(size_t)c * S + s] = a.sfin[(size_t)c * S + s];
    }
    __syncthreads();

    for (uint32_t it = 0; it < budget; ++it) {
        if (sh.ctl.done) break;
        const uint32_t T = sh.ctl.T;
        // ================= phase A (+ C): one Delay iteration per cluster =================
        for (uint32_t c = wave; c < Ct; c += kDrWaves) {
            unsigned long long* nodes = NODES + (size_t)c * W;
            uint32_t* sfin = SFIN + (size_t)c * S;
            uint32_t* hist = sh.hist[wave];
            const uint32_t n0 = a.node_off[c], N = a.node_off[c + 1] - n0;
            const uint64_t j0 = a.job_off[c];
            const uint32_t J = (uint32_t)(a.job_off[c + 1] - j0);
            const uint4* __restrict__ jobs = a.jobs + j0;
            unsigned long long* __restrict__ l1cm = a.l1cm + j0;
            unsigned long long* __restrict__ l1jd = a.l1jd + j0;
            unsigned long long* __restrict__ l1al = a.l1al + j0;
            const size_t sb = (size_t)c * S;
            DtCluster st = sh.cl[c];
            const uint32_t NN = N + st.nv;

            // releases due at T (cluster.go:153-157), Foreign jobs included
            if (st.minf <= T) {
                uint32_t lm = kEmpty, nrel = 0;
                for (uint32_t s = lane; s < S; s += kWave) {
                    const uint32_t f = sfin[s];
                    if (f <= T) {
                        const unsigned long long cm = dr_ld64(&a.scm[sb + s]);
                        uint32_t* h = reinterpret_cast<uint32_t*>(&nodes[dr_ld32(&a.snode[sb + s])]);
                        atomicAdd(h, (uint32_t)cm);
                        atomicAdd(h + 1, (uint32_t)(cm >> 32));
                        sfin[s] = kEmpty;
                        ++nrel;
                    } else {
                        lm = f < lm ? f : lm;
                    }
                }
                const uint32_t nr = dr_sum_u32(nrel);
                st.nrun -= nr;
                st.l1_dirty |= nr != 0u ? 1u : 0u;
                st.minf = wave_min_u32(lm);
                wsync();
            }
            // "/delay" arrivals up to T join Level0 (server.go:67-74)
            {
                const uint32_t before = st.next_arr;
                while (st.next_arr < J) {
                    const uint32_t i = st.next_arr + lane;
                    const bool ok = i < J && jobs[i].x <= T;
                    const uint32_t n = (uint32_t)__builtin_popcountll(__ballot(ok));
                    st.next_arr += n;
                    if (n < (uint32_t)kWave) break;
                }
                st.count += (long long)(st.next_arr - before);
            }
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
                    nodes[k] = (unsigned long long)((uint32_t)nodes[k] - jc) |
                               ((unsigned long long)((uint32_t)(nodes[k] >> 32) - jm) << 32);
                    sfin[slot] = fin;
                    a.snode[sb + slot] = k;
                    a.scm[sb + slot] = need;
                }
                wsync();
                ++st.nrun;
                st.peak = st.nrun > st.peak ? st.nrun : st.peak;
                st.minf = fin < st.minf ? fin : st.minf;
                return true;
            };

            // ---- Level1 pass (scheduler.go:302-329) ----
            if (st.l1n != 0u && !st.l1_dirty) {
                st.total += 1000ll * (long long)((unsigned long long)st.l1n * T - st.s_last);
                st.s_last = (unsigned long long)st.l1n * T;
                st.t_all = T;
            } else if (st.l1n != 0u) {
                const bool exact = NN <= (uint32_t)kWave;
                uint32_t best = 0u, max_c = 0u;
                if (!exact) {
                    hist[lane] = 0u;
                    wsync();
                    uint32_t mc = 0u;
                    for (uint32_t i = lane; i < NN; i += kWave) {
                        const unsigned long long v = nodes[i];
                        const uint32_t fc = (uint32_t)v;
                        atomicMax(&hist[fc < 63u ? fc : 63u], (uint32_t)(v >> 32));
                        mc = fc > mc ? fc : mc;
                    }
                    wsync();
                    max_c = dr_max_u32(mc);
                    best = hist[lane];
                    for (int o = 1; o < kWave; o <<= 1) {
                        const uint32_t w = (uint32_t)__shfl_down((int)best, o);
                        best = (lane + (uint32_t)o < (uint32_t)kWave && w > best) ? w : best;
                    }
                }
                auto lane_fit = [&](uint32_t c_l, uint32_t m_l) -> uint32_t {
                    uint32_t kl = kEmpty;
                    for (uint32_t i = NN; i-- > 0u;) {
                        const unsigned long long v = nodes[i];
                        kl = ((uint32_t)v >= c_l && (uint32_t)(v >> 32) >= m_l) ? i : kl;
                    }
                    return kl;
                };
                uint32_t wr = 0;
                bool carry_skip = false;
                const uint32_t n1 = st.l1n, t_all = st.t_all;
                long long tot_l = 0ll;
                unsigned long long snew_l = 0ull;
                unsigned long long ncm = 0, njd = 0, nal = 0;
                if (lane < n1) {
                    ncm = dr_ld64(&l1cm[lane]);
                    njd = dr_ld64(&l1jd[lane]);
                    nal = dr_ld64(&l1al[lane]);
                }
                for (uint32_t base = 0; base < n1; base += kWave) {
                    const uint32_t pos = base + lane;
                    const bool live = pos < n1;
                    const unsigned long long cm = ncm, jdv = njd, al = nal;
                    if (pos + kWave < n1) {
                        ncm = dr_ld64(&l1cm[pos + kWave]);
                        njd = dr_ld64(&l1jd[pos + kWave]);
                        nal = dr_ld64(&l1al[pos + kWave]);
                    }
                    const uint32_t jc_l = (uint32_t)cm, jm_l = (uint32_t)(cm >> 32);
                    unsigned long long placedm = 0ull, skipm = carry_skip ? 1ull : 0ull;
                    bool overflow = false;
                    if (exact) {
                        uint32_t from = 0;
                        for (;;) {
                            wsync();
                            const uint32_t kl = live ? lane_fit(jc_l, jm_l) : kEmpty;
                            const unsigned long long fitm = __ballot(kl != kEmpty) & ~skipm &
                                                            (from < 64u ? (~0ull << from) : 0ull);
                            if (!fitm) break;
                            const uint32_t b = (uint32_t)__builtin_ctzll(fitm);
                            const uint32_t k = readlane(kl, b);
                            const uint32_t jc = readlane(jc_l, b), jm = readlane(jm_l, b);
                            const uint32_t jd = readlane((uint32_t)(jdv >> 32), b), jj = readlane((uint32_t)jdv, b);
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
                            if ((skipm >> b) & 1ull) continue;
                            const uint32_t jc = readlane(jc_l, b), jm = readlane(jm_l, b);
                            const uint32_t k = first_fit(jc, jm);
                            if (k == kEmpty) continue;
                            const uint32_t jd = readlane((uint32_t)(jdv >> 32), b), jj = readlane((uint32_t)jdv, b);
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
                        wr = n1;
                        break;
                    }
                    const unsigned long long livem = __ballot(live);
                    const uint32_t last = 63u - (uint32_t)__builtin_clzll(livem);
                    carry_skip = ((placedm >> last) & 1ull) != 0ull && last == 63u;
                    const bool examined = live && !((skipm >> lane) & 1ull);
                    const bool placed = ((placedm >> lane) & 1ull) != 0ull;
                    const uint32_t sl = (uint32_t)(al >> 32);
                    const uint32_t eff = sl > t_all ? sl : t_all;
                    const long long delta = examined ? (long long)(T - eff) * 1000ll : 0ll;
                    tot_l += delta;
                    const unsigned long long kept = livem & ~placedm;
                    const uint32_t nl = examined ? T : eff;
                    if (live && !placed) {
                        const uint32_t np = wr + (uint32_t)__builtin_amdgcn_mbcnt_hi(
                                                     (uint32_t)(kept >> 32),
                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)kept, 0u));
                        if (np != pos) {
                            l1cm[np] = cm;
                            l1jd[np] = jdv;
                        }
                        if (np != pos || nl != sl) l1al[np] = (al & 0xFFFFFFFFull) | ((unsigned long long)nl << 32);
                    }
                    snew_l += live && !placed ? (unsigned long long)nl : 0ull;
                    wr += (uint32_t)__builtin_popcountll(kept);
                }
                st.l1n = wr;
                st.total += dr_sum_i64(tot_l);
                st.s_last = (unsigned long long)dr_sum_i64((long long)snew_l);
                st.l1_dirty = wr != n1 ? 1u : 0u;
            }

            // ---- Level0 head (scheduler.go:332-366) ----
            if (!(st.flags & MCS_FLAG_OVERFLOW) && st.l0_head < st.next_arr) {
                const uint32_t j = st.l0_head;
                const uint4 jb = jobs[j];
                const uint32_t k = first_fit(jb.z, jb.w);
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
                } else if (T - jb.x >= a.max_wait) {
                    if (lane == 0) {
                        l1cm[st.l1n] = (unsigned long long)jb.z | ((unsigned long long)jb.w << 32);
                        l1jd[st.l1n] = (unsigned long long)j | ((unsigned long long)jb.y << 32);
                        l1al[st.l1n] = (unsigned long long)jb.x | ((unsigned long long)T << 32);
                    }
                    ++st.l1n;
                    st.s_last += T;
                    ++st.l0_head;
                    ++st.moved;
                    st.head_last = kEmpty;
                }
            }
            wsync();
            // ---- phase C: the state sample (trader_server.go:24-47) every sample_period seconds ----
            if (T % a.sample_period == 0u) {
                float* dc = SAMP + (size_t)wave * 2u * W;
                float* dm = dc + W;
                for (uint32_t i = lane; i < NN; i += kWave) {
                    const unsigned long long v = nodes[i];
                    uint2 cp;
                    if (i < N) {
                        cp = a.cap[n0 + i];
                    } else {
                        const unsigned long long w = dr_ld64(reinterpret_cast<const unsigned long long*>(
                            &a.vcap[(size_t)c * a.V + (i - N)]));
                        cp = make_uint2((uint32_t)w, (uint32_t)(w >> 32));
                    }
                    dc[i] = __fsub_rn((float)cp.x, dr_go_f32((uint32_t)v));
                    dm[i] = __fsub_rn((float)cp.y, dr_go_f32((uint32_t)(v >> 32)));
                }
                wsync();
                if (lane == 0) {
                    float sc = 0.0f, sm = 0.0f;
                    for (uint32_t i = 0; i < NN; ++i) {
                        sc = __fadd_rn(sc, dc[i]);
                        sm = __fadd_rn(sm, dm[i]);
                    }
                    st.cu = __fdiv_rn(sc, (float)st.total_c);
                    st.mu = __fdiv_rn(sm, (float)st.total_m);
                    st.avgw = st.count != 0 ? __ddiv_rn((double)st.total, (double)st.count) : 0.0;
                }
                st.cu = __shfl(st.cu, 0);
                st.mu = __shfl(st.mu, 0);
                st.avgw = __shfl(st.avgw, 0);
            }
            // ---- the cluster's record, and its contract sizes over GetLevel1() when its trader is
            // due at T (ProvideJobs, trader_server.go:69-94) ----
            const bool any_due = a.period != 0u && sh.ctl.any_due != 0u;
            uint32_t fsc = 0, fsm = 0, fmd = 0, ssc = 0, ssm = 0, sst = 0;
            if (any_due && sh.trs[c].next_due <= T) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // this wave's compaction stores
                wsync();
                const uint32_t ln = st.l1n;
                for (uint32_t i = lane; i < ln; i += kWave) {
                    const unsigned long long cm = dr_ld64(&l1cm[i]);
                    const uint32_t jc = (uint32_t)cm, jm = (uint32_t)(cm >> 32);
                    const uint32_t d = (uint32_t)(dr_ld64(&l1jd[i]) >> 32);
                    fsc += jc;
                    fsm += jm;
                    fmd = d > fmd ? d : fmd;
                    ssc += (int32_t)(0u - jc) < 0 ? jc : 0u;
                    ssm += (int32_t)(0u - jm) < 0 ? jm : 0u;
                }
                fsc = dr_sum_u32(fsc);
                fsm = dr_sum_u32(fsm);
                fmd = dr_max_u32(fmd);
                ssc = dr_sum_u32(ssc);
                ssm = dr_sum_u32(ssm);
                if (ln % 20u == 0u) {
                    for (uint32_t b = 0; b < ln; b += kWave) {
                        wsync();
                        if (b + lane < ln) hist[lane] = (uint32_t)(dr_ld64(&l1jd[b + lane]) >> 32);
                        wsync();
                        if (lane == 0) {
                            const uint32_t m = ln - b < (uint32_t)kWave ? ln - b : (uint32_t)kWave;
                            for (uint32_t i = 0; i < m; ++i) sst = sst < hist[i] ? hist[i] : 0u;
                        }
                    }
                    sst = readlane(sst, 0);
                }
            }
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
                sh.rec[c] = r;
                sh.cl[c] = st;
            }
            wsync();
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // Level1 rows, slot payloads
        __syncthreads();

        // ================= phase D: the trader rounds, wave 0 =================
        if (wave == 0) {
            const bool any_due = sh.ctl.any_due != 0u;
            for (uint32_t q = lane; q < Ct; q += kWave) sh.nfr[q] = sh.rec[q].nfree;
            wsync();
            unsigned long long n_trades = sh.ctl.n_trades, n_won = sh.ctl.n_won, n_for = sh.ctl.n_foreign;
            uint32_t lflags = 0;
            for (uint32_t q0 = 0; q0 < Ct && a.period && any_due; q0 += kWave) {
                const uint32_t ql = q0 + lane;
                unsigned long long due = __ballot(ql < Ct && sh.trs[ql].next_due <= T);
                while (due) {
                    const uint32_t q = q0 + (uint32_t)__builtin_ctzll(due);
                    due &= due - 1ull;
                    const DtRec* rq = &sh.rec[q];
                    while (sh.trs[q].next_due <= T) {
                        DtTrader tq = sh.trs[q];
                        if (tq.stage == 0u) {
                            tq.cs_cu = rq->cu;
                            tq.cs_mu = rq->mu;
                            tq.cs_avgw = rq->avgw;
                        }
                        const uint32_t pol = tq.stage;
                        const bool broken = pol == 0u ? (tq.cs_avgw > 600000.0)
                                                      : (tq.cs_cu > 0.8f || tq.cs_mu > 0.8f);
                        tq.stage = pol == 0u ? 1u : 0u;
                        if (!broken) {
                            if (pol == 1u) tq.next_due = T + a.period;
                            wsync();
                            if (lane == 0) sh.trs[q] = tq;
                            wsync();
                            continue;
                        }
                        const uint32_t kc = pol == 0u ? rq->fc : rq->sc;
                        const uint32_t km = pol == 0u ? rq->fm : rq->sm;
                        const uint32_t ksec = pol == 0u ? rq->ft : rq->st;
                        uint32_t napp = 0;
                        for (uint32_t r0 = 0; r0 < Ct; r0 += kWave) {
                            const uint32_t r = r0 + lane;
                            bool app = false;
                            if (r < Ct && r != q) {
                                DtTrader t = sh.trs[r];
                                if (t.lock_id != 0u && T >= t.lock_until) t.lock_id = 0u;
                                if (t.lock_id == 0u) {
                                    const DtRec* rr = &sh.rec[r];
                                    app = approve_trade_dev(rr->total_c, rr->total_m, rr->cu, rr->mu, kc, km, ksec);
                                    t.lock_id = t.next_id++;
                                    t.lock_until = T + a.lock_s;
                                }
                                sh.trs[r] = t;
                            }
                            const unsigned long long ab = __ballot(app);
                            if (app) {
                                const uint32_t at = napp + (uint32_t)__builtin_amdgcn_mbcnt_hi(
                                                               (uint32_t)(ab >> 32),
                                                               __builtin_amdgcn_mbcnt_lo((uint32_t)ab, 0u));
                                sh.appr[at] = r;
                            }
                            napp += (uint32_t)__builtin_popcountll(ab);
                        }
                        wsync();
                        int32_t winner = -1;
                        uint32_t failed = 0;
                        for (uint32_t i = 0; i < napp && winner < 0; ++i) {
                            const uint32_t r = sh.appr[i == 0u ? 0u : napp - i];
                            uint32_t rc_ = kc, rm_ = km;
                            const uint32_t rN = sh.rec[r].N;
                            const uint32_t rNN = rN + sh.nvs[r];
                            unsigned long long* rs = NODES + (size_t)r * W;  // live = snapshot (one engine)
                            bool ovf = false;
                            for (uint32_t nd = 0; nd < rNN; ++nd) {
                                if (rm_ == 0u && rc_ == 0u) break;
                                const unsigned long long v = rs[nd];
                                double mem_diff = 0.0, core_diff = 0.0;
                                if (rm_ > 0u) mem_diff = fabs(__dsub_rn((double)rm_, dr_go_f64((uint32_t)(v >> 32))));
                                if (rc_ > 0u) core_diff = fabs(__dsub_rn((double)rc_, dr_go_f64((uint32_t)v)));
                                if (mem_diff > (double)rm_)
                                    rm_ = 0u;
                                else
                                    rm_ -= (uint32_t)mem_diff;
                                if (core_diff > (double)rc_)
                                    rc_ = 0u;
                                else
                                    rc_ -= (uint32_t)core_diff;
                                const unsigned long long fc = dr_f64_to_u64(core_diff), fm = dr_f64_to_u64(mem_diff);
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
                                if (ksec == 0u) continue;
                                if (sh.nfr[r] == 0u) {
                                    ovf = true;
                                    break;
                                }
                                const unsigned long long nv_ = (unsigned long long)((uint32_t)v - (uint32_t)fc) |
                                                               ((unsigned long long)((uint32_t)(v >> 32) - (uint32_t)fm) << 32);
                                uint32_t slot = kEmpty;
                                const size_t rsb = (size_t)r * S;
                                for (uint32_t b = 0; b < S; b += kWave) {
                                    const unsigned long long fr = __ballot(SFIN[rsb + b + lane] == kEmpty);
                                    if (fr) {
                                        slot = b + (uint32_t)__builtin_ctzll(fr);
                                        break;
                                    }
                                }
                                if (lane == 0) {
                                    rs[nd] = nv_;
                                    sh.nfr[r] -= 1u;
                                    if (slot != kEmpty) {
                                        SFIN[rsb + slot] = T + ksec;
                                        a.snode[rsb + slot] = nd;
                                        a.scm[rsb + slot] = (unsigned long long)(uint32_t)fc |
                                                            ((unsigned long long)(uint32_t)fm << 32);
                                        DtCluster& k = sh.cl[r];
                                        k.nrun += 1u;
                                        k.minf = (T + ksec) < k.minf ? (T + ksec) : k.minf;
                                        k.l1_dirty |= 1u;
                                    }
                                }
                                wsync();
                            }
                            if (ovf) {
                                lflags |= MCS_FLAG_OVERFLOW;
                                break;
                            }
                            if (lane == 0) sh.trs[r].lock_id = 0u;
                            wsync();
                            if (rc_ > 0u || rm_ > 0u) {
                                ++failed;
                                continue;
                            }
                            winner = (int32_t)r;
                            if (lane == 0) {
                                const uint32_t nv = sh.nvs[q];
                                const unsigned long long cap = (unsigned long long)kc | ((unsigned long long)km << 32);
                                if (nv < a.V) {
                                    NODES[(size_t)q * W + rq->N + nv] = cap;
                                    sh.nvs[q] = nv + 1u;
                                    a.vn[(size_t)q * a.V + nv] = cap;
                                    a.vcap[(size_t)q * a.V + nv] = make_uint2(kc, km);
                                    sh.cl[q].nv += 1u;
                                    sh.cl[q].l1_dirty |= 1u;
                                } else {
                                    lflags |= MCS_FLAG_VNODE_OVERFLOW;
                                    sh.cl[q].flags |= (uint32_t)MCS_FLAG_VNODE_OVERFLOW;
                                }
                            }
                            wsync();
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
                            tq.lock_id = sh.trs[q].lock_id;
                            tq.lock_until = sh.trs[q].lock_until;
                            tq.next_id = sh.trs[q].next_id;
                            sh.trs[q] = tq;
                        }
                        ++n_trades;
                        wsync();
                        if (lflags & MCS_FLAG_OVERFLOW) break;
                    }
                    if (lflags & MCS_FLAG_OVERFLOW) break;
                }
                if (lflags & MCS_FLAG_OVERFLOW) break;
            }
            lflags = readlane(lflags, 0);
            // the next tick (as dt_trader_kernel)
            bool all_done = true, queued = false;
            uint32_t nxt = T + a.sample_period - T % a.sample_period, fl = 0, ndue = kEmpty;
            for (uint32_t q = lane; q < Ct; q += kWave) {
                const DtRec* rq = &sh.rec[q];
                all_done = all_done && rq->done != 0u;
                queued = queued || rq->queued != 0u;
                nxt = rq->nxt < nxt ? rq->nxt : nxt;
                if (a.period) ndue = sh.trs[q].next_due < ndue ? sh.trs[q].next_due : ndue;
                fl |= rq->flags;
            }
            const bool done_all = !__ballot(!all_done);
            const bool queued_any = __ballot(queued) != 0ull;
            ndue = wave_min_u32(ndue);
            nxt = wave_min_u32(nxt);
            nxt = ndue < nxt ? ndue : nxt;
            for (int o = 32; o > 0; o >>= 1) fl |= (uint32_t)__shfl_xor((int)fl, o);
            if (lane == 0) {
                DtCtl& ctl = sh.ctl;
                uint32_t flags = ctl.flags | fl | lflags;
                uint32_t done = 0, Tn = T;
                if (done_all || (flags & MCS_FLAG_OVERFLOW)) {
                    done = 1u;
                } else if (T >= a.t_max) {
                    done = 1u;
                    flags |= MCS_FLAG_T_MAX;
                } else {
                    Tn = (queued_any || nxt <= T + 1u) ? T + 1u : nxt;
                }
                ctl.T = Tn;
                ctl.done = done;
                ctl.any_due = ndue <= Tn ? 1u : 0u;
                ctl.ticks += 1u;
                ctl.flags = flags;
                ctl.n_trades = n_trades;
                ctl.n_won = n_won;
                ctl.n_foreign = n_for;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // Foreign slots, virtual-node caps
        }
        __syncthreads();
    }

    // ---- store the system back (the host polls ctl; a next launch reloads it) ----
    for (uint32_t i = threadIdx.x; i < Ct; i += blockDim.x) {
        a.cl[i] = sh.cl[i];
        a.tr[i] = sh.trs[i];
        a.nv_all[i] = sh.nvs[i];
    }
    for (uint32_t c = wave; c < Ct; c += kDrWaves) {
        const uint32_t n0 = a.node_off[c], N = a.node_off[c + 1] - n0;
        const uint32_t nv = sh.cl[c].nv;
        for (uint32_t i = lane; i < N; i += kWave) a.tn[n0 + i] = NODES[(size_t)c * W + i];
        for (uint32_t i = lane; i < nv && i < a.V; i += kWave)
            a.vn[(size_t)c * a.V + i] = NODES[(size_t)c * W + N + i];
        for (uint32_t s = lane; s < S; s += kWave) a.sfin[(size_t)c * S + s] = SFIN[(size_t)c * S + s];
    }
    if (threadIdx.x == 0) *a.ctl = sh.ctl;
}

}  // namespace

// The shape this kernel holds: one engine, at most 64 clusters of at most 64 physical nodes, and the
// resident arrays within the device's LDS per workgroup.
bool dtrade_res_shape(const DtArgs& a, uint32_t world, size_t* lds) {
    if (world != 1 || a.Ct > kDrMaxClusters || a.NS > kDrMaxNodes || a.S % kWave != 0u) return false;
    *lds = dr_lds(a.Ct, a.W, a.S);
    return true;
}

hipError_t launch_dtrade_res(const DtArgs& a, uint32_t budget, size_t lds, hipStream_t s) {
    const hipError_t st = hipFuncSetAttribute((const void*)dt_res_kernel,
                                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (st != hipSuccess) return st;
    hipLaunchKernelGGL(dt_res_kernel, dim3(1), dim3(kDrWaves * kWave), lds, s, a, budget);
    return hipGetLastError();
}

}  // namespace mcs
