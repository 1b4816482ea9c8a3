// mcs_dtrade_internal.h — device layout of the lock-step trading system with DELAY schedulers
// (mcs_trade.h; oracle/mcs_oracle_dtrade.c).  The system of Ct = world * C clusters
// is sharded over `world` engines in contiguous blocks of C; the trader rounds run replicated.
//
// HBM, per local cluster c (C of them):
//   tn     u64 {free_c | free_m << 32} per physical node (CSR node_off), live across ticks
//   vn     u64 free vector of virtual node v at [c * V + v]; vcap uint2 its capacity
//   sfin/snode/scm  running slots (finish, node, {c | m << 32}); Foreign jobs included
//   l1cm/l1jd/l1al  the Level1 list, capacity = the cluster's job count (at job_off), one u64 each:
//          {cores | mem << 32}, {job | dur << 32}, {arrival | last examined << 32}; the JobsMap
//          entry of a Level1 job is 1000 * (last - arrival), so no per-job map is kept
//   cl     DtCluster queue cursors, counters, WaitTime sums, last sample
//   tr     DtTrader trader state (two-stage RequestPolicyMonitor, responder lock)
//   ctl    DtCtl the lock-step clock and log counters (replicated: identical on every rank)
//   xb     the exchange blocks, one per rank (world * blk bytes): rank r's block holds DtRec[C] and
//          the node snapshots u64[C * W] of clusters [r*C, r*C + C) after phase A (physical nodes
//          at [0, N), virtual node v at [NS + v]).  Phase D reads every block (gathered by RCCL or
//          the caller; with world 1 the step kernel writes the only block in place).
// Free counters are u32 halves read as Go uint64 values by sign extension: a Foreign job can take
// more than a node has (cluster.go:116), and the wrapped uint64 is 2^64 - x for small x, which
// the device keeps as the u32 2^32 - x (same comparisons against needs < 2^31; conversions to
// float32/float64 go through the sign-extended uint64 like Go's).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mcs_trade.h"
#include "mcs_internal.h"

namespace mcs {

constexpr uint32_t kDtMaxNodes = 1024;  // physical nodes per cluster
constexpr uint32_t kDtMaxVnodes = 256;  // virtual nodes a cluster can receive
constexpr uint32_t kDtMaxSlots = 4096;  // running slots per cluster (LDS staging, 16 KB)
constexpr uint32_t kDtMaxClusters = 1024;  // in the whole system (all ranks)

struct DtCluster {
    uint32_t next_arr;  // jobs [0, next_arr) have arrived
    uint32_t l0_head;   // Level0 = [l0_head, next_arr)
    uint32_t l1n;       // len(Level1)
    uint32_t nv;        // virtual nodes received
    uint32_t decided;
    uint32_t moved;
    uint32_t placed_l1;
    uint32_t minf;      // earliest running finish (kEmpty = none)
    uint32_t nrun;
    uint32_t peak;
    uint32_t flags;
    uint32_t total_c;   // SetTotalResources at Run (cluster.go:26-40), physical nodes only
    uint32_t total_m;
    float cu, mu;       // last sample
    uint32_t head_last; // last tick the Level0 head was examined (kEmpty: not yet)
    double avgw;        // last WaitTime.GetAverage()
    long long total;    // WaitTime.TotalTime (ms)
    long long count;    // WaitTime.JobsCount
    // Level1 pass elision: a pass can only place a job after something raised a free counter
    // (a release, a new virtual node, a Foreign job wrapping a counter) or after a pass that
    // placed (its skipped entries).  Otherwise every entry fails again and only its JobsMap entry
    // moves to T: entries' effective last = max(stored last, t_all), s_last = their sum.  A pass
    // that runs sets t_all = T too and rewrites no stamp of an examined entry left in place; an entry
    // the pass skips (D6, marked untested in bit 31 of its job word) carries its own last
    // examination in its stamp, which is then its effective last whatever t_all holds (r06).
    uint32_t l1_dirty;
    uint32_t t_all;
    unsigned long long s_last;
};

// What the replicated trader rounds need of a cluster after phase A (one per cluster, in xb).
struct DtRec {
    float cu, mu;       // last sample
    double avgw;
    uint32_t total_c, total_m, nv, N;
    uint32_t nfree;     // free running slots (Foreign jobs need one each)
    uint32_t flags;
    uint32_t done;      // every job decided
    uint32_t queued;    // Level0 or Level1 non-empty
    uint32_t nxt;       // next arrival (kEmpty: none)
    uint32_t fc, fm, ft;  // the fast-node contract over Level1 (computed when the trader is due)
    uint32_t sc, sm, st;  // the small-node contract
    uint32_t pad;
};
static_assert(sizeof(DtRec) == 80, "DtRec layout");

struct DtTrader {
    uint32_t lock_id, lock_until, next_id, next_due;
    uint32_t stage;     // 0: WaitTime next (a fresh cs), 1: Utilization (stale cs)
    float cs_cu, cs_mu;
    uint32_t pad;
    double cs_avgw;
};

struct DtCtl {
    uint32_t T, done, ticks, flags;
    uint32_t any_due, pad0;  // a trader round is due at T (phase A then sizes contracts)
    unsigned long long n_trades, n_won, n_foreign;
};

struct DtArgs {
    uint32_t C, V, S;
    uint32_t base, Ct;   // global index of local cluster 0; clusters in the system (world * C)
    uint32_t NS, W;      // snapshot stride: physical nodes, physical + virtual
    uint32_t rank;
    unsigned long long blk;  // bytes of one rank's exchange block
    unsigned char* xb;       // world exchange blocks
    uint32_t* nv_all;        // virtual nodes of every cluster (replicated)
    uint32_t period, ok_sleep, fail_sleep, lock_s, sample_period, max_wait, t_max;
    unsigned long long trade_cap, foreign_cap;
    const uint32_t* node_off;
    const uint2* cap;
    const uint2* free0;
    unsigned long long* tn;
    unsigned long long* vn;
    uint2* vcap;
    const uint4* jobs;
    const uint64_t* job_off;
    int32_t* out_node;
    uint32_t* out_start;
    uint32_t* out_finish;
    uint32_t* sfin;
    uint32_t* snode;
    unsigned long long* scm;
    unsigned long long* l1cm;
    unsigned long long* l1jd;
    unsigned long long* l1al;
    DtCluster* cl;
    DtTrader* tr;  // Ct entries, replicated
    DtCtl* ctl;
    unsigned long long* l1snap;  // [C][W] node values the Level1 jobs last failed against (dt_step)
    mcs_contract_rec* trade_log;
    mcs_foreign_rec* foreign_log;
};

// The resident tick (mcs_dtrade_mw.hip, world 1): one wave per cluster, 4 per workgroup, and a
// trader wave, exchanging granules through one XCD's L2; a launch runs up to `budget` ticks.
constexpr uint32_t kDtResMaxClusters = 64;  // clusters in the system
constexpr uint32_t kDtResMaxNN = 320;       // physical + virtual nodes per cluster
constexpr uint32_t kDtResMaxSlots = 1024;   // running slots per cluster
struct DtResArgs {
    unsigned long long* gx;  // exchange granules (cached device memory), dtrade_mw_gx_bytes()
    unsigned long long* gu;  // placement granules and the failure word (uncached), dtrade_mw_gu_bytes()
    void* ops;               // phase D's side effects, [cluster][ops_cap] of dtrade_mw_op_bytes() each
    uint32_t ops_cap, budget, nwg, pad;
};
size_t dtrade_mw_gx_bytes();
size_t dtrade_mw_gu_bytes();
size_t dtrade_mw_op_bytes();
uint32_t dtrade_mw_fail_word();  // index in gu: 0 ok, 1 placement, 2 a cluster wave's wait, 3 the trader's
hipError_t launch_dtrade_mw(const DtArgs& a, const DtResArgs& m, hipStream_t s);

hipError_t launch_dtrade_init(const DtArgs& a, hipStream_t s);
hipError_t launch_approve(const mcs_approve_query* q, uint32_t n, int32_t* out, hipStream_t s);  // the mirror
// one tick: phases A and C (dt_step_kernel, writes this rank's exchange block), then phase D
hipError_t launch_dtrade_step(const DtArgs& a, hipStream_t s);
hipError_t launch_dtrade_trader(const DtArgs& a, hipStream_t s);
hipError_t launch_dtrade_tick(const DtArgs& a, hipStream_t s);  // world 1: both

}  // namespace mcs
