// mcs_kernels.hip — gfx950 kernels of the batched FIFO placement engine.
//
// The hot kernel (fifo_kernel) runs the reference's FIFO policy loop — Scheduler.Fifo
// (pkg/scheduler/scheduler.go:216-296) over the first-fit primitive ScheduleJob (:127-139) and the
// commit/release of Node.RunJob (pkg/scheduler/cluster.go:141-161) — for one cluster per wave64
// workgroup, under the serialized semantics SFIFO of SURVEY Appendix A with the exact fast-forward
// of A.3.  Every decision is wave-uniform, so the wave never diverges on control flow:
//
//   * node free vectors live in VGPRs: lane l holds nodes l, l+64, ... (NPL nodes per lane);
//     first fit = one v_cmp pair per 64-node chunk whose SGPR mask IS the ballot, then s_ff1;
//   * the running set is a pool of 64*P slots (row p, lane l): finish times in VGPRs (one row per
//     register), payload {cores, mem, node} in LDS as three [P][64] u32 arrays (lane-contiguous,
//     bank-conflict-free); a free slot is found by ballot over finish == EMPTY;
//   * releases at a clock advance are wave-parallel: every lane whose slot expired scatters its
//     cores/mem into a per-node LDS accumulator with ds_add_u32 (order-free integer adds), and
//     each node owner lane folds its accumulator back with one ds_wrxchg per chunk;
//   * job records are streamed from HBM 64 at a time with one coalesced 16 B/lane load (uint4
//     {arrival, dur, cores, mem}), double-buffered one batch ahead, and broadcast to the scalar
//     unit with v_readlane;
//   * results are gathered 64 jobs per register batch (placements happen in job order because
//     FIFO head-of-line blocking is strict) and written with three coalesced 256 B stores.
//
// Compiled with -ffp-contract=off (no FP in this file's hot kernel; the utilization mirror is
// float32 and must round like Go).
#define MCS_GEN_FN __host__ __device__ static inline
#include "mcs_gen.h"
#include "mcs_internal.h"

namespace mcs {

__device__ __forceinline__ uint32_t readlane(uint32_t v, uint32_t l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t w = (uint32_t)__shfl_xor((int)v, o);
        v = w < v ? w : v;
    }
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

template <int NPL, int P>
__global__ __launch_bounds__(64) void fifo_kernel(FifoArgs a) {
    const uint32_t item = blockIdx.x;
    const uint32_t ci = a.cluster_list ? a.cluster_list[item] : item;
    const uint32_t lane = threadIdx.x;

    __shared__ uint32_t rel_c[NPL * kWave];  // release scatter accumulators, one per node
    __shared__ uint32_t rel_m[NPL * kWave];
    __shared__ uint32_t pay_c[P * kWave];    // running-slot payload, slot (p, l) at p*64 + l
    __shared__ uint32_t pay_m[P * kWave];
    __shared__ uint32_t pay_n[P * kWave];

    // ---- cluster spec: Run() keeps the JSON availability (scheduler.go:101-109) ----
    const uint32_t n0 = a.node_off[ci];
    const uint32_t N = a.node_off[ci + 1] - n0;
    uint32_t fc[NPL], fm[NPL];
    uint64_t valid[NPL];
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
        const uint32_t idx = k * kWave + lane;
        uint2 v = make_uint2(0u, 0u);
        if (idx < N) v = a.node_free0[n0 + idx];
        fc[k] = v.x;
        fm[k] = v.y;
        valid[k] = __ballot(idx < N);
        rel_c[idx] = 0u;
        rel_m[idx] = 0u;
    }

    // ---- job stream ----
    const uint64_t j0 = a.job_off[ci];
    const uint32_t J = (uint32_t)(a.job_off[ci + 1] - j0);
    const uint4* __restrict__ jobs = a.jobs + j0;
    int32_t* __restrict__ o_node = a.out_node + j0;
    uint32_t* __restrict__ o_start = a.out_start + j0;
    uint32_t* __restrict__ o_finish = a.out_finish + j0;

    auto load_batch = [&](uint32_t base) __attribute__((always_inline)) -> uint4 {
        const uint32_t i = base + lane;
        uint4 v = make_uint4(kEmpty, 0u, 0u, 0u);
        if (i < J) v = jobs[i];
        return v;
    };

    // running-slot finish times: row p of the pool in register sf[p] (static indices only)
    uint32_t sf[P];
#pragma unroll
    for (int p = 0; p < P; ++p) sf[p] = kEmpty;

    uint32_t cb = 0;
    uint4 cur = load_batch(0);
    uint4 nxt = load_batch(kWave);

    uint32_t t = 0, r = 0, minf = kEmpty, used = 0, peak = 0, waited = 0, placed = 0, flags = 0;
    bool have_w = false;
    uint32_t wi = 0, wc = 0, wm = 0, wd = 0;
    int32_t on = -1;
    uint32_t os = kEmpty, of = kEmpty;

    // first fit — ScheduleJob, scheduler.go:129-137 (lowest node index with both >=)
    auto first_fit = [&](uint32_t c, uint32_t m) __attribute__((always_inline)) -> int {
#pragma unroll
        for (int k = 0; k < NPL; ++k) {
            const uint64_t hit = __ballot(fc[k] >= c && fm[k] >= m) & valid[k];
            if (hit) return k * kWave + (int)__builtin_ctzll(hit);
        }
        return -1;
    };

    // commit — Node.RunJob, cluster.go:146-147 (synchronous, D2)
    auto commit = [&](int k, uint32_t c, uint32_t m) __attribute__((always_inline)) {
        const int kc = k >> 6;
        const uint32_t kl = (uint32_t)(k & 63);
#pragma unroll
        for (int kk = 0; kk < NPL; ++kk) {
            if (kk == kc && lane == kl) {
                fc[kk] -= c;
                fm[kk] -= m;
            }
        }
    };

    // running set insert (finish = start + Duration, cluster.go:151): first free slot in row-major
    // order; the finish goes to its register row by a select (no dynamic register index), the
    // payload to LDS by the one owning lane
    auto insert = [&](uint32_t fin, uint32_t c, uint32_t m, uint32_t node)
                      __attribute__((always_inline)) -> bool {
        int ps = -1;
        uint64_t e = 0;
#pragma unroll
        for (int p = P - 1; p >= 0; --p) {
            const uint64_t b = __ballot(sf[p] == kEmpty);
            if (b) {
                ps = p;
                e = b;
            }
        }
        if (ps < 0) return false;
        const uint32_t L = (uint32_t)__builtin_ctzll(e);
        const bool me = lane == L;
#pragma unroll
        for (int p = 0; p < P; ++p) sf[p] = (me && p == ps) ? fin : sf[p];
        if (me) {
            const uint32_t a = (uint32_t)ps * kWave + L;
            pay_c[a] = c;
            pay_m[a] = m;
            pay_n[a] = node;
        }
        ++used;
        peak = used > peak ? used : peak;
        minf = fin < minf ? fin : minf;
        return true;
    };

    // release every running job with finish <= t (cluster.go:153-157; A.2 step 1)
    auto release = [&]() __attribute__((always_inline)) {
        if (minf > t) return;
        uint32_t nexp = 0;
#pragma unroll
        for (int p = 0; p < P; ++p) {
            const bool ex = sf[p] <= t;
            const uint64_t b = __ballot(ex);
            if (b) {
                nexp += (uint32_t)__builtin_popcountll(b);
                if (ex) {
                    const uint32_t a = (uint32_t)p * kWave + lane;
                    const uint32_t nd = pay_n[a];
                    atomicAdd(&rel_c[nd], pay_c[a]);
                    atomicAdd(&rel_m[nd], pay_m[a]);
                }
                sf[p] = ex ? kEmpty : sf[p];
            }
        }
        used -= nexp;
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
        for (int k = 0; k < NPL; ++k) {
            if (valid[k]) {
                fc[k] += atomicExch(&rel_c[k * kWave + lane], 0u);
                fm[k] += atomicExch(&rel_m[k * kWave + lane], 0u);
            }
        }
        uint32_t lm = kEmpty;
#pragma unroll
        for (int p = 0; p < P; ++p) lm = sf[p] < lm ? sf[p] : lm;
        minf = wave_min_u32(lm);
    };

    auto flush = [&](uint32_t base) __attribute__((always_inline)) {
        const uint32_t i = base + lane;
        if (i < J) {
            __builtin_nontemporal_store(on, o_node + i);
            __builtin_nontemporal_store(os, o_start + i);
            __builtin_nontemporal_store(of, o_finish + i);
        }
    };

    auto place = [&](uint32_t ji, int k, uint32_t start, uint32_t fin) __attribute__((always_inline)) {
        const uint32_t ol = ji & 63u;
        if (lane == ol) {
            on = k;
            os = start;
            of = fin;
        }
        ++placed;
        if (ol == 63u) flush(ji - 63u);
    };

    // ---- Scheduler.Fifo (scheduler.go:216-296) ----
    // One pass = one decision.  Every helper has a single call site (one inlined copy each), and
    // the clock only moves at the bottom, where the completions due by then are released.
    for (;;) {
        uint32_t tn = t;
        bool attempt = true;
        uint32_t ji, jc, jm, jd;
        if (have_w) {  // len(WaitQueue) > 0, scheduler.go:219 -> ScheduleJob(WaitQueue[0]) :222
            ji = wi;
            jc = wc;
            jm = wm;
            jd = wd;
        } else {
            if (r >= J) break;
            if (r - cb >= (uint32_t)kWave) {
                cur = nxt;
                cb += kWave;
                nxt = load_batch(cb + kWave);
            }
            const uint32_t l = r - cb;
            const uint32_t arr = readlane(cur.x, l);
            // ReadyQueue head (:255-260); the job is in the queue once its arrival has passed
            ji = r;
            jd = readlane(cur.y, l);
            jc = readlane(cur.z, l);
            jm = readlane(cur.w, l);
            if (arr > t) {  // all queues empty: 1 s sleeps until the arrival (:294, A.3)
                tn = arr;
                attempt = false;
            } else {
                ++r;
            }
        }
        if (attempt) {
            const int k = first_fit(jc, jm);
            if (k >= 0) {
                place(ji, k, t, t + jd);
                // A zero-duration job is committed and released before the next decision can
                // read the node (RunJob sleeps 0; the release precedes the next branch, D3), so
                // it leaves no trace on the cluster: only its fit test matters.
                if (jd != 0u) {
                    commit(k, jc, jm);
                    if (!insert(t + jd, jc, jm, (uint32_t)k)) {
                        flags |= MCS_FLAG_OVERFLOW;
                        break;
                    }
                }
                if (have_w) {       // WaitQueue = WaitQueue[1:] (:226; D1)
                    have_w = false;
                    tn = t + 1u;    // time.Sleep(1 s) after every wait attempt (:250)
                }                   // ready path: no sleep (:272)
            } else {
                if (!have_w) {  // State = WAITING; WaitQueue append (:264-268)
                    have_w = true;
                    wi = ji;
                    wc = jc;
                    wm = jm;
                    wd = jd;
                    ++waited;
                    // The next pass of the Go loop retries the head at this same instant on an
                    // unchanged cluster (certain to fail) before sleeping: folded in here.
                }
                // no lender without borrowing (:234, server.go:220)
                if (minf == kEmpty) {  // nothing running: the head can never fit
                    flags |= MCS_FLAG_DEADLOCK;
                    break;
                }
                tn = (minf > t + 1u) ? minf : t + 1u;  // A.3: 1 s retries until a completion
            }
        }
        if (tn != t) {
            if (tn < t) {  // the u32 seconds clock would wrap (D8 range exceeded): stop, flagged
                flags |= MCS_FLAG_CLOCK_OVERFLOW;
                break;
            }
            t = tn;
            release();
        }
    }

    if (flags & MCS_FLAG_DEADLOCK) {
        // jobs wi..J-1 are never placed (the Go loop retries the head forever)
        const uint32_t b0 = wi & ~63u;
        if (lane >= (wi & 63u)) {
            on = MCS_NODE_UNPLACED;
            os = MCS_TIME_NONE;
            of = MCS_TIME_NONE;
        }
        flush(b0);
        on = MCS_NODE_UNPLACED;
        os = MCS_TIME_NONE;
        of = MCS_TIME_NONE;
        for (uint32_t b = b0 + kWave; b < J; b += kWave) flush(b);
    } else if (!(flags & (MCS_FLAG_OVERFLOW | MCS_FLAG_CLOCK_OVERFLOW)) && J > 0u &&
               ((J - 1u) & 63u) != 63u) {
        flush((J - 1u) & ~63u);
    }

    if (lane == 0) {
        mcs_cluster_stats st;
        st.t_end = t;
        st.placed = placed;
        st.waited = waited;
        st.peak_running = peak;
        st.flags = flags;
        st.pool = (uint32_t)P;
        st.reserved[0] = 0u;
        st.reserved[1] = 0u;
        a.cstats[ci] = st;
        if (flags & MCS_FLAG_OVERFLOW) {
            atomicAdd(&a.totals->overflowed, 1u);
        } else {
            atomicAdd(&a.totals->placed, (unsigned long long)placed);
            atomicAdd(&a.totals->waited, (unsigned long long)waited);
            atomicAdd(&a.totals->unplaced, (unsigned long long)(J - placed));
            if (flags & MCS_FLAG_DEADLOCK) atomicAdd(&a.totals->deadlocked, 1u);
        }
    }
}

// ---- variant table ------------------------------------------------------------------------------
template <int NPL, int P>
static hipError_t launch_one(const FifoArgs& a, hipStream_t s) {
    hipLaunchKernelGGL((fifo_kernel<NPL, P>), dim3(a.n_items), dim3(kWave), 0, s, a);
    return hipGetLastError();
}

template <int NPL>
static hipError_t launch_npl(const FifoArgs& a, int pool, hipStream_t s) {
    switch (pool) {
        case 2: return launch_one<NPL, 2>(a, s);
        case 4: return launch_one<NPL, 4>(a, s);
        case 8: return launch_one<NPL, 8>(a, s);
        case 16: return launch_one<NPL, 16>(a, s);
        case 32: return launch_one<NPL, 32>(a, s);
        default: return hipErrorInvalidValue;
    }
}

bool fifo_variant_exists(int npl, int pool) {
    const bool np = npl == 1 || npl == 2 || npl == 4 || npl == 8 || npl == 16;
    const bool pp = pool == 2 || pool == 4 || pool == 8 || pool == 16 || pool == 32;
    return np && pp;
}

hipError_t launch_fifo(const FifoArgs& a, int npl, int pool, hipStream_t s) {
    if (a.n_items == 0) return hipSuccess;
    switch (npl) {
        case 1: return launch_npl<1>(a, pool, s);
        case 2: return launch_npl<2>(a, pool, s);
        case 4: return launch_npl<4>(a, pool, s);
        case 8: return launch_npl<8>(a, pool, s);
        case 16: return launch_npl<16>(a, pool, s);
        default: return hipErrorInvalidValue;
    }
}

// ---- device job-stream synthesis (mcs_gen.h; bit-identical to the host generator) -------------
__global__ __launch_bounds__(256) void gen_attrs_kernel(uint4* jobs, const uint64_t* job_off,
                                                       const uint32_t* max_c,
                                                       const uint32_t* max_m, uint64_t seed,
                                                       uint32_t max_dur) {
    const uint32_t c = blockIdx.y;
    const uint64_t j0 = job_off[c], J = job_off[c + 1] - j0;
    const uint64_t key = mcs_cluster_key(seed, c);
    const uint32_t mc = max_c[c], mm = max_m[c];
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < J;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t d, cc, m;
        mcs_gen_job_attrs(key, i, mc, mm, max_dur, &d, &cc, &m);
        jobs[j0 + i] = make_uint4(0u, d, cc, m);
    }
}

__global__ __launch_bounds__(64) void gen_arrivals_kernel(uint4* jobs, const uint64_t* job_off,
                                                         uint32_t n_clusters, uint64_t seed,
                                                         uint32_t mode, double enl) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n_clusters) return;
    const uint64_t j0 = job_off[c], J = job_off[c + 1] - j0;
    const uint64_t akey = mcs_arrival_key(mcs_cluster_key(seed, c));
    uint64_t j = 0, period = 0;
    uint32_t T = 0;
    // same scan as mcs_gen_arrivals (mcs_gen.h), writing into the .x lane of the records
    while (j < J) {
        const uint32_t n = mcs_poisson(akey, period++, enl);
        if (mode == 0u) {
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

hipError_t launch_gen_attrs(uint4* jobs, const uint64_t* job_off, const uint32_t* max_c,
                            const uint32_t* max_m, uint32_t n_clusters, uint64_t seed,
                            uint32_t max_dur, hipStream_t s) {
    if (n_clusters == 0) return hipSuccess;
    hipLaunchKernelGGL(gen_attrs_kernel, dim3(64, n_clusters), dim3(256), 0, s, jobs, job_off,
                       max_c, max_m, seed, max_dur);
    return hipGetLastError();
}

hipError_t launch_gen_arrivals(uint4* jobs, const uint64_t* job_off, uint32_t n_clusters,
                               uint64_t seed, uint32_t mode, double exp_neg_lambda,
                               hipStream_t s) {
    if (n_clusters == 0) return hipSuccess;
    hipLaunchKernelGGL(gen_arrivals_kernel, dim3((n_clusters + 63) / 64), dim3(64), 0, s, jobs,
                       job_off, n_clusters, seed, mode, exp_neg_lambda);
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
