// mcs_gen_dev.h — the job stream synthesised inside the placement kernels.
//
// With mcs_gen_params.fused the FIFO and DELAY kernels never read job records from HBM: each
// 64-job batch is generated in registers when the kernel reaches it.  Job j of cluster k gets
// exactly the record mcs_gen_job_attrs + mcs_gen_arrivals (mcs_gen.h) give it, so a fused run
// equals the materialised run bit for bit (tests/test_gpu_fused.py).
//
//   * Attributes are counter-based (key, j): one job per lane.
//   * Arrivals are mcs_gen_arrivals' sequential scan over Poisson periods.  Here a wave draws the
//     counts of 64 periods at once (lane l = period pw + l), prefix-sums the counts and the period
//     lengths (REF: n * floor(60 / n) s, or 60 s for an empty minute; SCALED: 1 s), and each lane
//     finds its job's period with a 6-step binary search over the inclusive counts.  A window of
//     64 periods holds ~64 * lambda jobs, so at the C4 rate the scan costs about one window per
//     two batches.
//   * WEIBULL arrivals (client.go:131-145) are a running sum of per-job gaps: each lane draws its
//     job's gap from the host-resolved table (mcs_weibull_gap), the wave prefix-sums them and the
//     batch total carries to the next batch.
// The host resolves exp(-lambda) and the Weibull gap table once (like mcs_generate_jobs), so device
// and host draws match.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef MCS_GEN_FN
#define MCS_GEN_FN __host__ __device__ static inline
#endif
#include "mcs_gen.h"
#include "mcs_internal.h"
#include "mcs_wave.h"

namespace mcs {

// (DPP row shifts and broadcasts, mcs_wave.h: no LDS round trip)
__device__ __forceinline__ uint32_t wave_incl_sum_u32(uint32_t v, uint32_t) { return wave_scan_add_u32(v); }

constexpr uint32_t kGenScratch = 4u * kWave;  // LDS words of GenStream's optional scratch

struct GenStream {
    uint64_t ckey, akey;
    double enl;
    uint32_t mode, mc, mm, md;
    uint32_t pw, jw, tw;   // window: first period, its first job, its start second
    uint32_t n, cum, tex;  // lane l: jobs of period pw + l, inclusive job count, start offset
    uint32_t tot, span;    // jobs and seconds of the whole window
    const uint64_t* wthr;  // WEIBULL: gap table; wcarry = arrival of the next batch's first job
    uint32_t wn, wcarry;
    // Optional per-wave LDS scratch (kGenScratch words): the period search below runs as a scatter
    // of period starts and a prefix maximum instead of the 6-step shuffle search
    uint32_t* scr;

    __device__ __forceinline__ void fill(uint32_t lane) {
        n = mcs_poisson(akey, (uint64_t)pw + lane, enl);
        const uint32_t d = mode == 0u ? (n == 0u ? 60u : n * (60u / n)) : 1u;  // client.go:116-125, D5
        cum = wave_incl_sum_u32(n, lane);
        const uint32_t dinc = wave_incl_sum_u32(d, lane);
        tex = dinc - d;
        tot = readlane(cum, 63);
        span = readlane(dinc, 63);
    }

    __device__ __forceinline__ void init(const GenArgs& g, uint32_t cluster, uint32_t lane,
                                         uint32_t* scratch = nullptr) {
        scr = scratch;
        ckey = mcs_cluster_key(g.seed, g.base + cluster);
        akey = mcs_arrival_key(ckey);
        enl = g.enl;
        mode = g.mode;
        mc = g.max_c[cluster];
        mm = g.max_m[cluster];
        md = g.max_dur;
        pw = 0u;
        jw = 0u;
        tw = 0u;
        wthr = (const uint64_t*)g.wthr;
        wn = g.wn;
        wcarry = 0u;
        if (mode != 2u) fill(lane);
    }

    // the records {arrival, dur, cores, mem} of jobs [base, base + 64); bases must increase
    __device__ __forceinline__ uint4 next(uint32_t base, uint32_t lane) {
        const uint32_t j = base + lane;
        uint32_t arr = 0u, done = 0u;
        if (mode == 2u) {  // job j arrives after the gaps of jobs 0..j-1 (consecutive batches)
            const uint32_t g = mcs_weibull_gap(mcs_draw(akey, j), wthr, wn);
            const uint32_t inc = wave_incl_sum_u32(g, lane);
            arr = wcarry + inc - g;
            wcarry += readlane(inc, 63);
        }
        if (mode != 2u) for (;;) {  // (a wave-uniform loop: every lane takes part in the shuffles)
            // every lane searches (the shuffles need all lanes); lanes outside the window discard
            const uint32_t rel = j - jw;
            uint32_t lo = 0u, np, cp, te;
            if (scr) {
                // job lane l's period = the last period starting at or before it: each period with
                // jobs marks its first job's lane (distinct lanes), the period holding the batch's
                // first job comes from a ballot, and a prefix maximum spreads them; the period's
                // {n, cum, tex} are then read back from its slot.  The period's first job sits in
                // lane d = st - off; off < 0 when the batch straddles into this window (its first
                // lanes were decided in the previous one): no period then covers lane 0.
                const int32_t off = (int32_t)(base - jw);
                const int32_t d = (int32_t)(cum - n) - off;
                const uint64_t cov = __ballot(n != 0u && d <= 0);
                scr[lane] = 0u;
                if (n != 0u && d > 0 && d < (int32_t)kWave) scr[d] = lane + 1u;
                scr[kWave + lane * 3u] = n;
                scr[kWave + lane * 3u + 1u] = cum;
                scr[kWave + lane * 3u + 2u] = tex;
                // the reads below take other lanes' stores: a compiler memory barrier, or LLVM
                // forwards this lane's own `scr[lane] = 0` (measured: it did, and read the slot only
                // under the marking lanes' exec).  The wave's LDS ops run in order, so no wait.
                asm volatile("" ::: "memory");
                uint32_t mk = scr[lane];
                if (lane == 0u && cov) mk = mk > 64u - (uint32_t)__builtin_clzll(cov) ? mk : 64u - (uint32_t)__builtin_clzll(cov);
                const uint32_t sm = wave_scan_max_u32(mk);
                lo = sm != 0u ? sm - 1u : 0u;
                np = scr[kWave + lo * 3u];
                cp = scr[kWave + lo * 3u + 1u];
                te = scr[kWave + lo * 3u + 2u];
            } else {
#pragma unroll
                for (uint32_t s = 32u; s != 0u; s >>= 1) {
                    const uint32_t c = (uint32_t)__shfl((int)cum, (int)(lo + s - 1u));
                    lo += c <= rel ? s : 0u;
                }
                np = (uint32_t)__shfl((int)n, (int)lo);
                cp = (uint32_t)__shfl((int)cum, (int)lo);
                te = (uint32_t)__shfl((int)tex, (int)lo);
            }
            const uint32_t a = mode == 0u ? tw + te + (rel - (cp - np)) * (60u / (np != 0u ? np : 1u))
                                          : pw + lo;
            if (!done && rel < tot) {
                arr = a;
                done = 1u;
            }
            if (base + 63u - jw < tot) break;  // the batch's last job lies in this window
            jw += tot;
            tw += span;
            pw += (uint32_t)kWave;
            fill(lane);
        }
        uint32_t d, c, m;
        mcs_gen_job_attrs(ckey, j, mc, mm, md, &d, &c, &m);
        return make_uint4(arr, d, c, m);
    }
};

}  // namespace mcs
