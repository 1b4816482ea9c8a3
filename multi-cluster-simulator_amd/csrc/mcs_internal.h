// mcs_internal.h — device data layout shared by the kernels and the C-ABI engine (libmcs.so).
//
// HBM layout:
//   jobs      uint4  {arrival_s, dur_s, cores, mem} per job, clusters contiguous (CSR job_off)  16 B/job
//   out_node  int32  per job; out_start, out_finish uint32 per job (SoA)                      12 B/job
//   node_free0 uint2 {free_c, free_m} per node (JSON CoresAvailable/MemoryAvailable), CSR node_off
//   node_cap   uint2 {cores, memory} per node; live_c/live_m uint32 per node (single-job mirrors)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mcs.h"

namespace mcs {

constexpr uint32_t kEmpty = 0xFFFFFFFFu;  // empty running slot (finish time never reached)
constexpr int kWave = 64;
constexpr int kMaxNpl = 16;   // nodes per lane -> at most 1024 nodes per cluster in ABI v1
constexpr int kMaxPool = 32;  // running-slot registers per lane -> 2048 slots per cluster
constexpr uint32_t kAsmMaxJobs = (1u << 28) - 128u;  // hand-scheduled loop: 32-bit record offsets
// grids up to this many clusters would pick the duo loop by default: none (measured 1.5x slower than
// W16R at 512-2048 clusters; MCS_FIFO_DUO=1 runs it)
constexpr uint32_t kDuoMaxItems = 0u;
// the W16L lookahead loop: picked for grids of at most this many clusters (0: only MCS_FIFO_LOOK=1)
constexpr uint32_t kLookMaxItems = 0u;
constexpr uint32_t kJobPad = 128;  // records of slack after the job array (unmasked batch loads)

struct Totals {  // device-side accumulation of mcs_stats (only clusters that did not overflow)
    unsigned long long placed;
    unsigned long long waited;
    unsigned long long unplaced;
    unsigned int deadlocked;
    unsigned int overflowed;
    unsigned int clock_overflowed;  // clusters stopped by MCS_FLAG_CLOCK_OVERFLOW (run fails, MCS_E_RANGE)
    unsigned int bailed;            // DELAY clusters the hand-scheduled loop hands to delay_kernel
};

// In-kernel synthesis of the job stream (mcs_gen_dev.h): with `on` the FIFO and
// DELAY kernels generate each 64-job batch in registers and `jobs` is not read (may be null).
struct GenArgs {
    unsigned long long seed;
    double enl;             // exp(-lambda), resolved once on the host like mcs_generate_jobs
    const uint32_t* max_c;  // per-cluster maxima: setMaxCluster (client.go:68-83) or explicit
    const uint32_t* max_m;
    uint32_t mode;          // mcs_arrival_mode
    uint32_t max_dur;
    uint32_t base;          // global index of the engine's cluster 0 (mcs_set_shard)
    uint32_t on;
    const unsigned long long* wthr;  // WEIBULL gap table (mcs_gen.h), resolved on the host
    uint32_t wn;
    uint32_t pad;
};

// Online mode (mcs_run with a finite horizon, mcs_append_jobs): one record per
// cluster carried between horizons, plus the node image (the LDS layout of nodes[]) and the running
// slots.  valid == 0 starts the cluster from its spec at t = 0.
struct OnlineState {
    uint32_t valid;
    uint32_t t;       // the next loop iteration's time (not yet executed)
    uint32_t cursor;  // FIFO: ready cursor r; DELAY: Level0 head h
    uint32_t aux;     // FIFO: have_w (job r is the WaitQueue head); DELAY: len(Level1)
    uint32_t flags;
    uint32_t pool;    // slot rows saved in the slot image (rows >= pool are free)
    uint32_t placed, waited, peak, used, n_iter, n_rel, placed_l1, peak_l1;  // DELAY: waited = moved
    unsigned long long l1_t, mv_a, wsum;  // DELAY WaitTime sums (mcs_delay.hip)
};
constexpr uint32_t kSlotImg = 2u * kMaxPool * kWave;  // u64 words of one cluster's slot image

struct OnlineArgs {  // read only by the HOR kernel variants
    const uint32_t* job_cnt;   // jobs in each cluster's segment (job_off = segment starts)
    const OnlineState* st_in;  // state at the start of this horizon (read only: reruns reuse it)
    OnlineState* st_out;
    const unsigned long long* img_in;  // node image, img_stride words per cluster
    unsigned long long* img_out;
    const unsigned long long* slot_in;  // slot image: kSlotImg words per cluster ([cm rows][nf rows])
    unsigned long long* slot_out;
    uint32_t img_stride;
    uint32_t t_hor;  // stop before any iteration at t >= t_hor; kEmpty = drain
};

struct FifoArgs {
    const uint2* node_free0;
    const uint32_t* node_off;
    const uint4* jobs;
    const uint64_t* job_off;
    const uint32_t* cluster_list;  // grid item -> cluster (nullptr = identity)
    int32_t* out_node;
    uint32_t* out_start;
    uint32_t* out_finish;
    mcs_cluster_stats* cstats;
    Totals* totals;
    GenArgs gen;
    OnlineArgs on;
    uint32_t n_items;
    uint32_t guard_ok;  // bit 0: every node's free values < 2^31 - 1 (the hand-scheduled loop
                        // may run, W32 node format); bit 1: < 2^15 - 1 (W16 node format);
                        // bit 2: every cluster holds at most kAsmMaxJobs jobs
};

struct DelayArgs {
    const uint2* node_free0;
    const uint32_t* node_off;
    const uint4* jobs;
    const uint64_t* job_off;
    const uint32_t* cluster_list;  // grid item -> cluster (nullptr = identity)
    int32_t* out_node;
    uint32_t* out_start;
    uint32_t* out_finish;
    uint64_t* l1_cm;  // Level1 scratch, one entry per job: {cores | mem << 32}
    uint64_t* l1_jd;  //                                    {job | dur << 32}
    mcs_cluster_stats* cstats;
    mcs_delay_cluster_stats* dstats;
    Totals* totals;
    GenArgs gen;
    OnlineArgs on;
    uint32_t max_wait_s;
    uint32_t n_items;
};

// hor: the online variant (OnlineArgs; records streamed, never fused)
hipError_t launch_delay(const DelayArgs& a, int npl, int pool, bool hor, hipStream_t s);  // mcs_delay.hip
// the hand-scheduled DELAY loop (mcs_delay_asm.hip): Level1-empty iterations; a cluster whose head
// moves to Level1 stops with kDelayBail in its cstats flags and is re-run on delay_kernel
constexpr uint32_t kDelayBail = 0x40000000u;
bool delay_asm_eligible(int npl, int pool, uint32_t guard_ok, bool gen_on);
hipError_t launch_delay_asm(const DelayArgs& a, hipStream_t s);

struct StateArgs {  // the ClusterState reduction over a run's placements (mcs_state.hip)
    const uint32_t* node_off;
    const uint2* cap;
    const uint2* free0;
    const uint4* jobs;
    const uint64_t* job_off;
    const int32_t* out_node;
    const uint32_t* out_start;
    const uint32_t* out_finish;
    mcs_cluster_state* out;
    uint32_t t;
    uint32_t n_clusters;
};
hipError_t launch_state(const StateArgs& a, uint32_t max_n, hipStream_t s);  // mcs_state.hip

// Launchers (mcs_kernels.hip).  Return hipSuccess or the launch error.
hipError_t launch_fifo(const FifoArgs& a, int npl, int pool, bool hor, hipStream_t s);
uint32_t cu_count();  // CUs of the current device (256 on MI355X)
// the low-occupancy forms are picked for grids of at most this many cluster waves per CU
constexpr uint32_t kLatWavesPerCu = 4;
bool fifo_variant_exists(int npl, int pool);
// the hand-scheduled decision loop (mcs_fifo_asm.hip): NPL 4 / P 8 or NPL 1 / P 2, streamed
// batch runs; MCS_FIFO_ASM=0 turns it off
bool fifo_asm_eligible(const FifoArgs& a, int npl, int pool, bool hor);
int fifo_asm_form(const FifoArgs& a, int npl, int pool, bool hor);  // 22, 21, 20, 19, 18, 17, 16, 32 or 0
hipError_t launch_fifo_asm(const FifoArgs& a, int npl, int pool, hipStream_t s);
hipError_t launch_gen_attrs(uint4* jobs, const uint64_t* job_off, const uint32_t* max_c,
                            const uint32_t* max_m, uint32_t n_clusters, uint64_t seed,
                            uint32_t max_dur, uint32_t cluster_base, hipStream_t s);
hipError_t launch_gen_arrivals(uint4* jobs, const uint64_t* job_off, uint32_t n_clusters, const GenArgs& g,
                               hipStream_t s);
// whole records through GenStream, one wave per cluster (every cluster below 2^32 jobs)
hipError_t launch_gen_stream(uint4* jobs, const uint64_t* job_off, uint32_t n_clusters, const GenArgs& g,
                             hipStream_t s);
hipError_t launch_gen_bound(const uint64_t* job_off, uint32_t n_clusters, const GenArgs& g,
                            unsigned long long* last, hipStream_t s);
hipError_t launch_schedule_one(uint32_t* live_c, uint32_t* live_m, uint32_t n, uint32_t c,
                               uint32_t m, int32_t* out_node, hipStream_t s);
hipError_t launch_lend_check(const uint32_t* live_c, const uint32_t* live_m, uint32_t n,
                             uint32_t c, uint32_t m, int32_t* out_ok, hipStream_t s);
hipError_t launch_utilization(const uint2* cap, const uint32_t* live_c, const uint32_t* live_m,
                              uint32_t n, float* out2, hipStream_t s);

}  // namespace mcs
