/*
 * mcs_gen.h — seeded synthetic job streams (INPUT synthesis, not the checked algorithm).
 *
 * Restates the distributions of the reference client (pkg/client/client.go:85-147):
 *   cores = floor(B  * maxCores)   B  ~ Beta(2,2)   (client.go:87-90, 97)
 *   mem   = floor(B' * maxMem)     B' ~ Beta(2,2)   (client.go:99); maxima from setMaxCluster (68-83)
 *   dur   = rand.Intn(600) s                         (client.go:98)
 *   arrivals, REF mode:    per "minute" n ~ Poisson(10) (client.go:107-114); the n jobs are sent
 *                          floor(60/n) s apart, the loop sleeping after every send (116-125), so a
 *                          minute lasts n*floor(60/n) s; n == 0 panics in Go (60/0) -> idle 60 s (D5)
 *   arrivals, SCALED mode: per second n ~ Poisson(lambda_s), all n arrive at that second
 *   arrivals, WEIBULL mode: the client's "weibull" time_dist (client.go:131-145): after each job it
 *                          sleeps time.Duration(X) * time.Second with X ~ Weibull(Lambda 10, K 3),
 *                          i.e. floor(X) whole seconds (the float64 -> Duration conversion truncates)
 *
 * Beta(2,2) is drawn as the median of three U(0,1) (the median of 3 iid uniforms is exactly
 * Beta(2,2)); floor(B*max) is computed on 32-bit fixed point: (median_u32 * max) >> 32.  Poisson is
 * Knuth's product method on IEEE doubles (single multiplies, no contraction possible) against
 * exp(-lambda) computed ONCE on the host and passed in, so host and device streams are bit-identical.
 * The reference stream itself is unreproducible (gonum v0.14.0 samplers; math/rand.Intn is
 * auto-seeded since Go 1.20), so the stream is treated as input.
 *
 * Randomness is counter-based (SplitMix64 finaliser of key + counter*gamma): job i's attributes
 * depend only on (cluster key, i), so attributes are generated in parallel; only the arrival scan
 * is sequential per cluster.
 *
 * Included by C (gcc) and HIP (hipcc) translation units.  The includer may define MCS_GEN_FN
 * (e.g. `__host__ __device__ static inline`) before including.
 */
#ifndef MCS_GEN_H
#define MCS_GEN_H

#include <stdint.h>

#ifndef MCS_GEN_FN
#define MCS_GEN_FN static inline
#endif

#define MCS_GEN_GAMMA 0x9E3779B97F4A7C15ULL
#define MCS_GEN_SEED_DEFAULT 0x4D43535F53494D31ULL /* "MCS_SIM1" */
#define MCS_GEN_POISSON_MAX_DRAWS 256u

MCS_GEN_FN uint64_t mcs_mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

/* counter-based draw: value number `ctr` of the stream `key` */
MCS_GEN_FN uint64_t mcs_draw(uint64_t key, uint64_t ctr) {
    return mcs_mix64(key + (ctr + 1u) * MCS_GEN_GAMMA);
}

/* attribute key of cluster k ("cluster k uses stream seed xor k") */
MCS_GEN_FN uint64_t mcs_cluster_key(uint64_t seed, uint32_t cluster) {
    return mcs_mix64(seed ^ (uint64_t)cluster);
}
/* arrival-process key of cluster k (an independent stream) */
MCS_GEN_FN uint64_t mcs_arrival_key(uint64_t ckey) {
    return mcs_mix64(ckey ^ 0xA5A5A5A55A5A5A5AULL);
}

MCS_GEN_FN uint32_t mcs_med3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t lo = a < b ? a : b, hi = a < b ? b : a;
    return c < lo ? lo : (c > hi ? hi : c);
}

/* floor(u * max) for u = x / 2^32 */
MCS_GEN_FN uint32_t mcs_scale(uint32_t x, uint32_t max) {
    return (uint32_t)(((uint64_t)x * (uint64_t)max) >> 32);
}

/* attributes of job i: cores, mem (Beta(2,2)*max), duration (U{0..max_dur-1}) */
MCS_GEN_FN void mcs_gen_job_attrs(uint64_t ckey, uint64_t i, uint32_t max_cores, uint32_t max_mem,
                                  uint32_t max_dur, uint32_t* dur, uint32_t* cores,
                                  uint32_t* mem) {
    const uint64_t h0 = mcs_draw(ckey, 4u * i + 0u);
    const uint64_t h1 = mcs_draw(ckey, 4u * i + 1u);
    const uint64_t h2 = mcs_draw(ckey, 4u * i + 2u);
    const uint64_t h3 = mcs_draw(ckey, 4u * i + 3u);
    *cores = mcs_scale(mcs_med3((uint32_t)h0, (uint32_t)(h0 >> 32), (uint32_t)h1), max_cores);
    *mem = mcs_scale(mcs_med3((uint32_t)(h1 >> 32), (uint32_t)h2, (uint32_t)(h2 >> 32)), max_mem);
    *dur = mcs_scale((uint32_t)h3, max_dur);
}

/* U(0,1) with 53 random bits */
MCS_GEN_FN double mcs_u01(uint64_t h) { return (double)(h >> 11) * (1.0 / 9007199254740992.0); }

/* Poisson(lambda) draw number `idx` of the arrival stream, Knuth: count uniforms until the running
 * product falls to exp(-lambda) or below.  exp_neg_lambda is host-computed. */
MCS_GEN_FN uint32_t mcs_poisson(uint64_t akey, uint64_t idx, double exp_neg_lambda) {
    double p = 1.0;
    uint32_t k = 0;
    for (;;) {
        p = p * mcs_u01(mcs_draw(akey, idx * MCS_GEN_POISSON_MAX_DRAWS + k));
        if (!(p > exp_neg_lambda)) break;
        ++k;
        if (k + 1u >= MCS_GEN_POISSON_MAX_DRAWS) break;
    }
    return k;
}

/* Weibull gaps: floor(X), X ~ Weibull(lambda, k), from the 64-bit draw u by inverse CDF on the
 * integer grid: floor(X) >= n  <=>  X >= n  <=>  U <= exp(-(n/lambda)^k).  thr[n-1] =
 * floor(2^64 * exp(-(n/lambda)^k)) is resolved ONCE on the host (like exp(-lambda) for Poisson) and
 * decreases to 0 within MCS_GEN_WEIBULL_MAX entries; the gap is the number of leading entries with
 * u < thr (binary search), so host and device gaps are identical integers. */
#define MCS_GEN_WEIBULL_MAX 256u
MCS_GEN_FN uint32_t mcs_weibull_gap(uint64_t u, const uint64_t* thr, uint32_t nthr) {
    uint32_t lo = 0, hi = nthr;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (u < thr[mid])
            lo = mid + 1u;
        else
            hi = mid;
    }
    return lo;
}

/* Sequential arrival scan of one cluster: arrival[j] for j < n_jobs.  mode 0 = REF, 1 = SCALED,
 * 2 = WEIBULL (thr / nthr: the gap table above; unused by the Poisson modes). */
MCS_GEN_FN void mcs_gen_arrivals(uint64_t ckey, uint32_t mode, double exp_neg_lambda,
                                 const uint64_t* thr, uint32_t nthr, uint64_t n_jobs, uint32_t* arrival) {
    const uint64_t akey = mcs_arrival_key(ckey);
    uint64_t j = 0, period = 0;
    uint32_t T = 0;
    if (mode == 2u) { /* SendJob, then Sleep(floor(X)) (client.go:136-145): job 0 at t = 0 */
        for (j = 0; j < n_jobs; ++j) {
            arrival[j] = T;
            T += mcs_weibull_gap(mcs_draw(akey, j), thr, nthr);
        }
        return;
    }
    while (j < n_jobs) {
        const uint32_t n = mcs_poisson(akey, period++, exp_neg_lambda);
        if (mode == 0u) {
            if (n == 0u) { /* D5: 60/0 panics in Go; an idle minute here */
                T += 60u;
                continue;
            }
            const uint32_t spacing = 60u / n; /* client.go:116 integer division */
            for (uint32_t i = 0; i < n && j < n_jobs; ++i) {
                arrival[j++] = T; /* SendJob then Sleep(spacing), client.go:121-124 */
                T += spacing;
            }
        } else {
            for (uint32_t i = 0; i < n && j < n_jobs; ++i) arrival[j++] = T;
            T += 1u;
        }
    }
}

#endif /* MCS_GEN_H */
