// mcs_trade_internal.h — device layout of the lock-step trading path (mcs_trade.h).
//
// HBM, per local cluster c (C_l of them) unless noted:
//   tn      u64 packed {free_c | free_m << 32} per node (CSR node_off), live across ticks
//   cl      TrCluster: queue cursors, counters, last utilization sample
//   sfin    u32 [S] running-slot finish times (kEmpty = free); snode u32 [S]; scm u64 [S]
//   lq      TrLq [LQ] LentQueue ring
// Exchange blocks, one per rank (world * blk bytes), the tick's only exchange (all-gathered once):
//   rank r's block holds TrXRec[C_l] (the post-A record of its clusters: borrow request, queue
//   state, utilization sample) followed by the node snapshots u64 [C_l][ns] (post-A free vectors,
//   which every rank's lender scan reads) and, for the one-launch tick, the lenders' G tables
//   u32 [C_l][64] (mcs_trade_rk.hip)
// Replicated per global cluster (C_t = world * C_l); every rank computes them alike from the
// gathered blocks:
//   acc     u32 [C_t] "some lender accepted borrower b this tick" (phase B -> C)
//   lqp     u32 [C_t] LentQueue length after phase B; fb u32 [C_t] flags raised in phase B
//   (TrRecC, the sample + clock hints of phase C, lives in the trader kernel's LDS)
//   tr      TrTrader [C_t] trader/lock state: every rank runs the identical trader rounds
//   ctl     TrCtl    the lock-step clock and log counters
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mcs_trade.h"
#include "mcs_internal.h"

namespace mcs {

constexpr uint32_t kTrMaxNodes = 1024;     // nodes per cluster (LDS staging, 8 KB)
constexpr uint32_t kTrMaxSlots = 4096;     // running slots per cluster (LDS staging, 16 KB)
constexpr uint32_t kTrMaxClusters = 1024;  // clusters in one trading system (trader LDS state)

struct TrCluster {
    uint32_t next_arr;  // first job (local index) not yet queued; ready queue = [rq_head, next_arr)
    uint32_t rq_head;
    uint32_t has_w;     // WaitQueue head present (scheduler.go:219)
    uint32_t w;         // its local index
    uint32_t lq_head;   // LentQueue ring cursor and length
    uint32_t lq_len;
    uint32_t decided;   // own jobs placed or borrowed
    uint32_t placed;
    uint32_t waited;
    uint32_t borrowed;
    uint32_t minf;      // earliest running finish (kEmpty = none)
    uint32_t nrun;
    uint32_t peak;
    uint32_t flags;     // MCS_FLAG_*
    uint32_t lent_runs;
    uint32_t total_c;   // SetTotalResources (cluster.go:26-40): uint32 sums of capacities
    uint32_t total_m;
    float cu, mu;       // latest utilization sample
    uint32_t pad[3];
};

struct TrRecA {  // phase A -> B: the tick's borrow request (job == kEmpty: none)
    uint32_t job, c, m, dur;
};

struct TrXRec {  // a cluster's post-A exchange record (64 B)
    TrRecA req;           // the tick's borrow request (req.job == kEmpty: none)
    uint32_t n;           // nodes (of the snapshot)
    uint32_t has_w, lq_len, rq_busy;  // wait head, LentQueue length, ready jobs queued
    uint32_t decided, J, next_arr_t, flags;
    float cu, mu;         // latest utilization sample (taken in phase A on sample ticks)
    uint32_t total_c, total_m;
};
static_assert(sizeof(TrXRec) == 64, "exchange record");

struct TrRecC {  // phase C -> D
    float cu, mu;
    uint32_t total_c, total_m;
    uint32_t busy;        // wait head, ready jobs or lent jobs pending: next tick is T+1
    uint32_t next_arr_t;  // arrival of the next unqueued job (kEmpty = none)
    uint32_t done;        // every own job decided and the LentQueue empty
    uint32_t flags;
};

struct TrTrader {  // replicated per global cluster
    uint32_t lock_id, lock_until, next_id, next_due, vnodes;
};

struct TrLq {
    uint32_t borrower, job, c, m, dur, pad0, pad1, pad2;
};

struct TrCtl {
    uint32_t T, done, ticks, flags;
    unsigned long long n_lent, n_trades, n_won;
    uint32_t info, pad;  // info: the workgroup-resident tick exchanged through one XCD's L2 (1)
};

struct TradeArgs {
    uint32_t Cl, Ct, base, world;
    uint32_t S, LQ, borrow, trader;
    uint32_t period, ok_sleep, fail_sleep, lock_s;
    uint32_t sample_period, t_max;
    unsigned long long lent_cap, trade_cap;
    const uint32_t* node_off;  // local CSR
    const uint2* cap;          // {cores, memory} per node
    const uint2* free0;        // JSON availability
    unsigned long long* tn;
    const uint4* jobs;
    const uint64_t* job_off;
    int32_t* out_node;
    uint32_t* out_start;
    uint32_t* out_finish;
    TrCluster* cl;
    uint32_t* sfin;
    uint32_t* snode;
    unsigned long long* scm;
    TrLq* lq;
    unsigned char* xb;       // world exchange blocks
    unsigned long long blk;  // bytes of one rank's block
    uint32_t ns, rank;       // snapshot stride (nodes), this rank
    uint32_t snaps;          // one-launch tick: 1 = the blocks carry node snapshots (a lender may be
                             // "big"), 0 = records and G tables only
    uint32_t* acc;
    uint32_t* lqp;
    uint32_t* fb;
    TrTrader* tr;
    TrCtl* ctl;
    mcs_lent_rec* lent_log;
    mcs_trade_rec* trade_log;
    unsigned long long* tnr;  // (one-launch tick) this rank's nodes, dense [C_l][ns], across launches
    uint4* lrp;  // (one-launch tick) this rank's lent run of the last phase A per cluster {b, j, node, fin}
};

// the exchange record and node snapshot of global cluster g
__device__ __forceinline__ TrXRec* tr_xrec(const TradeArgs& a, uint32_t g) {
    const uint32_t r = g / a.Cl, c = g - r * a.Cl;
    return reinterpret_cast<TrXRec*>(a.xb + (size_t)r * a.blk) + c;
}
__device__ __forceinline__ unsigned long long* tr_snap(const TradeArgs& a, uint32_t g) {
    const uint32_t r = g / a.Cl, c = g - r * a.Cl;
    return reinterpret_cast<unsigned long long*>(a.xb + (size_t)r * a.blk + (size_t)a.Cl * sizeof(TrXRec)) +
           (size_t)c * a.ns;
}

hipError_t launch_trade_init(const TradeArgs& a, hipStream_t s);
hipError_t launch_trade_phase(const TradeArgs& a, int phase, hipStream_t s);
// the whole system resident in one workgroup (mcs_trade_res.hip): shape check, LDS bytes, launch
constexpr uint32_t kTrResMaxClusters = 64;
bool trade_resident_shape(const TradeArgs& a);
size_t trade_resident_lds(uint32_t n_clusters, uint32_t ns);
hipError_t launch_trade_resident(const TradeArgs& a, uint32_t tick_budget, size_t lds, hipStream_t s);
// the system resident in ceil(C / kMwWaves) workgroups (4 clusters each), one cluster per wave, records traded as tagged
// granules (mcs_trade_mw.hip): shape check, LDS bytes, granule count, launch
bool trade_mw_shape(const TradeArgs& a);
size_t trade_mw_lds(uint32_t ns);
size_t trade_mw_granules(uint32_t n_clusters);
// the workgroups' XCD-id granules follow X1 (10 per cluster) and X2 (128) in the uncached buffer
constexpr size_t trade_mw_xcc_off() { return (size_t)kTrResMaxClusters * 10u + 128u; }
constexpr size_t trade_mw_x1b_off() { return trade_mw_xcc_off() + 64u; }  // X1's second buffer
// gx_uc: uncached granules (any placement); gx_c: cached granules, used when every workgroup runs on
// one XCD; xcd_pack: launch the workers 8 blocks apart (one XCD under round-robin dispatch)
hipError_t launch_trade_mw(const TradeArgs& a, unsigned long long* gx_uc, unsigned long long* gx_c,
                           uint32_t tick_budget, uint32_t tick0, size_t lds, bool xcd_pack, bool force_uc,
                           hipStream_t s);
constexpr uint32_t kTrFlagMwTimeout = 0x80000000u;  // internal: an exchange sweep gave up
// N ranks, one launch per tick (mcs_trade_rk.hip): B/C/D of tick n + A of tick n + 1, the ranks'
// blocks all-gathered between launches; mode 0 = phase A of tick 0 only
bool trade_rk_shape(const TradeArgs& a);
size_t trade_rk_lds(uint32_t ns);
hipError_t launch_trade_rk(const TradeArgs& a, uint32_t mode, size_t lds, hipStream_t s);

}  // namespace mcs
