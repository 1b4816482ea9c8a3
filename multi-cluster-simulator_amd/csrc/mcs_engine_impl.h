// mcs_engine_impl.h — the engine handle behind the C ABI (mcs.h, mcs_trade.h), shared by the
// FIFO engine (mcs_engine.cpp) and the lock-step trading path (mcs_trade.cpp).  Host code.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/mcs_trade.h"
#include "mcs_internal.h"

namespace mcs {
struct TradeDev;  // mcs_trade.cpp
void trade_free(mcs_engine* e);
void trade_release_graphs(mcs_engine* e);  // the captured tick graphs only (before comm_free)
void comm_free(mcs_engine* e);
int trade_run(mcs_engine* e, mcs_stats* stats);
int trade_cluster_stats(mcs_engine* e, mcs_cluster_stats* out, uint32_t n_clusters);
struct DtradeDev;  // mcs_dtrade.cpp: lock-step trading with DELAY schedulers
void dtrade_free(mcs_engine* e);
void dtrade_release_graphs(mcs_engine* e);
int dtrade_run(mcs_engine* e, mcs_stats* stats);
int dtrade_cluster_stats(mcs_engine* e, mcs_cluster_stats* out, uint32_t n);
int dtrade_delay_stats(mcs_engine* e, mcs_delay_cluster_stats* out, uint32_t n);
int dtrade_trade_stats(mcs_engine* e, mcs_trade_stats* out);
// job records in HBM for the paths that read them (trading, mcs_read_jobs): a fused synthetic
// stream is materialised by the generator kernels (mcs_engine.cpp)
int ensure_job_records(mcs_engine* e);
int dtrade_read_trades(mcs_engine* e, mcs_trade_rec* out, uint64_t cap, uint64_t* n);
int dtrade_read_vnode_counts(mcs_engine* e, uint32_t* out, uint32_t n);
// caller-driven lock-step of a sharded DELAY trading system (mcs_trade_begin/xfer/phase/end)
int dtrade_begin(mcs_engine* e);
int dtrade_xfer_bytes(mcs_engine* e, uint32_t phase, uint64_t* in_bytes, uint64_t* out_bytes);
int dtrade_phase(mcs_engine* e, uint32_t phase, const void* in, uint64_t in_bytes, void* out,
                 uint64_t out_bytes, uint32_t* done);
int dtrade_end(mcs_engine* e, mcs_stats* stats);
inline bool is_dtrade(const mcs_engine* e);
// online mode (mcs_online.cpp)
void online_free(mcs_engine* e);
int online_begin(mcs_engine* e);
int online_run(mcs_engine* e, uint32_t t_hor, mcs_stats* stats);
int online_read_rows(mcs_engine* e, int32_t* node, uint32_t* start_s, uint32_t* finish_s);
int online_read_jobs(mcs_engine* e, uint4* out);
int npl_for(uint32_t max_n);
int auto_pool(uint32_t max_n);
// per-cluster clock bound of the streams in HBM: last arrival and sum of (dur + 1 + extra)
int stream_bounds(mcs_engine* e, std::vector<uint32_t>& last, std::vector<uint64_t>& sum);
uint32_t horizon_extra(const mcs_engine* e);  // max_wait_s under DELAY, else 0

// Lock-step tick loops: mcs_trade_stats.loop_form
constexpr uint32_t kLoopGraph = 0;      // one engine, ticks replayed from a captured hipGraph
constexpr uint32_t kLoopRcclEager = 1;  // RCCL all-gather per tick, launches enqueued eagerly
constexpr uint32_t kLoopRcclGraph = 2;  // RCCL all-gather per tick, captured with the kernels
constexpr uint32_t kLoopResident = 3;   // one engine, the whole system resident in one workgroup
constexpr uint32_t kLoopResidentMwXcd = 5;  // the same, its workgroups on one XCD (L2 exchange)
constexpr uint32_t kLoopResidentMw = 4;  // one engine, resident in ceil(C / kMwWaves) workgroups, 4 clusters each (granules)
constexpr uint32_t kLoopGraphAfterTimeout = 6;  // the replayed kernels after a resident exchange timed out
constexpr uint32_t kLoopRkGraph = 7;  // RCCL: one launch + one all-gather per tick, captured in a hipGraph
constexpr uint32_t kLoopRkEager = 8;  // the same, enqueued eagerly
constexpr uint32_t kLoopRkDriven = 9;  // the one-launch tick on the caller-driven phase API

// Capture `ticks` ticks of `tick(stream)` (kernels and the RCCL all-gather) into one executable
// graph.  Returns nullptr, with the stream out of capture mode and the HIP error state cleared, when
// any step of the capture fails (the caller then keeps the eager loop); MCS_RCCL_GRAPH=0 skips it.
template <class F>
hipGraphExec_t capture_tick_graph(hipStream_t s, uint32_t ticks, F&& tick) {
    if (const char* env = getenv("MCS_RCCL_GRAPH"))
        if (atoi(env) == 0) return nullptr;
    hipGraph_t g = nullptr;
    if (hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    bool ok = true;
    for (uint32_t t = 0; t < ticks && ok; ++t) ok = tick(s);
    const hipError_t ec = hipStreamEndCapture(s, &g);
    hipGraphExec_t x = nullptr;
    if (ok && ec == hipSuccess && g) {
        if (hipGraphInstantiate(&x, g, nullptr, nullptr, 0) != hipSuccess) x = nullptr;
    }
    if (g) (void)hipGraphDestroy(g);
    (void)hipGetLastError();
    return x;
}
}  // namespace mcs

struct mcs_engine {
    mcs_config cfg{};
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    std::string err;
    const char* last_kernel = "";  // mcs_last_kernel: the first placement launch of the last run
    std::string last_kernel_buf;   // (when last_kernel names a DELAY hand-over)

    uint32_t C = 0;
    uint32_t max_n = 0;
    bool free_lt31 = false;  // every node free value < 2^31 - 1 (fifo_asm_kernel<32> guard bits)
    bool free_lt15 = false;  // every node free value < 2^15 - 1 (fifo_asm_kernel<16>)
    bool sums_lt24 = false;  // every cluster's sum of max(capacity, availability) < 2^24 per resource
    bool slot_pack_ok = false;  // every node's max(capacity, availability) < 128 cores, < 65536 memory
    bool cores_le64 = false;    // every node's max(capacity, availability) <= 64 cores (no "big" lender)
    uint64_t total_nodes = 0, total_jobs = 0;
    std::vector<uint32_t> node_off;
    std::vector<uint64_t> job_off;

    uint2* d_free0 = nullptr;
    uint2* d_cap = nullptr;
    uint32_t* d_node_off = nullptr;
    uint32_t* d_live_c = nullptr;
    uint32_t* d_live_m = nullptr;
    uint32_t* d_max_c = nullptr;
    uint32_t* d_max_m = nullptr;
    uint4* d_jobs = nullptr;        // null while a fused synthetic stream is not materialised
    mcs::GenArgs gen{};             // the synthetic stream of mcs_generate_jobs (gen.on: fused)
    uint32_t* d_gen_max = nullptr;  // its explicit maxima: [C] cores, then [C] memory
    unsigned long long* d_wthr = nullptr;  // its Weibull gap table (MCS_ARRIVAL_WEIBULL)
    uint64_t* d_job_off = nullptr;
    int32_t* d_out_node = nullptr;
    uint32_t* d_out_start = nullptr;
    uint32_t* d_out_finish = nullptr;
    mcs_cluster_stats* d_cstats = nullptr;
    mcs_delay_cluster_stats* d_dstats = nullptr;
    uint64_t* d_l1_cm = nullptr;  // DELAY Level1 scratch (allocated by the first DELAY run)
    uint64_t* d_l1_jd = nullptr;
    bool delay_run = false;       // results of the last run come from the DELAY kernel
    mcs::Totals* d_totals = nullptr;
    uint32_t* d_list = nullptr;
    int32_t* d_scratch = nullptr;
    float* d_util = nullptr;
    bool has_clusters = false, has_jobs = false, has_run = false;
    // sharding (mcs_set_shard) and the lock-step trading state (mcs_trade.cpp)
    uint32_t rank = 0, world = 1;
    void* comm = nullptr;  // ncclComm_t
    mcs::TradeDev* td = nullptr;
    bool trade_run = false;  // results of the last run come from the lock-step path
    uint32_t tr_lq = 0, tr_slots = 0;  // capacity escalation of the lock-step path (0 = auto)
    bool tr_res_start = false;  // trade_run's local loop on a resident form: start at 512 slots
    bool tr_no_resident = false;  // a resident tick timed out in this run: the replayed kernels
    mcs::DtradeDev* dtd = nullptr;     // DELAY trading state (mcs_dtrade.cpp)
    bool dtrade_run = false;           // results of the last run come from DELAY trading
    uint32_t dt_vnodes = 0;            // virtual-node capacity per cluster (0 = auto)
    uint32_t dt_learn_s = 0, dt_learn_v = 0;  // the capacities a DELAY-trading run of these inputs ended at
    uint32_t dt_ns = 0;                // node-snapshot stride over all ranks (0 = max_n)
    uint32_t tr_ns = 0;                // the same for FIFO lock-step trading
    bool tr_rk_ok = true;              // every rank can run the one-launch tick (tr_agree_shape)
    bool tr_nosnap = false;            // no rank has a node above 64 cores: the one-launch tick's
                                       // exchange blocks carry no node snapshots (tr_agree_shape)
    bool tr_agreed = false;            // the ranks agreed on the block layout (tr_agree_shape on the
                                       // RCCL path, mcs_trade_set_shape on the caller-driven one)
    // online mode (mcs_online.cpp): per-cluster state kept on the device between horizons
    bool online = false;               // a session is active
    bool segmented = false;            // job_off holds segment starts with slack (appends)
    uint32_t on_t_done = 0;            // the last horizon run (appended arrivals must be >= it)
    uint32_t on_t_hor = 0;             // the last finite horizon (appended arrivals must be >= it)
    std::vector<uint32_t> on_floor;    // per cluster: its clock after the last drain (appends >= it)
    int on_pool = 0;                   // slot rows that every saved state fits in
    int on_cur = 0;                    // which of the double-buffered states is current
    mcs::OnlineState* d_ost[2] = {nullptr, nullptr};
    unsigned long long* d_oimg[2] = {nullptr, nullptr};
    unsigned long long* d_oslot[2] = {nullptr, nullptr};
    unsigned long long* d_l1_bak = nullptr;  // DELAY: Level1 lists at the start of a horizon
    size_t l1_bak_words = 0;
    uint32_t* d_job_cnt = nullptr;
    std::vector<uint32_t> job_cnt;     // jobs per cluster (online; job_off = segment starts)
    std::vector<uint32_t> last_arr;    // last arrival per cluster (append checks)
    std::vector<uint64_t> sum_dur;     // sum of (dur + 1 [+ max_wait]) per cluster (clock bound)
    bool bounds_known = false;         // last_arr / sum_dur filled
};

inline bool mcs::is_dtrade(const mcs_engine* e) { return e->cfg.policy == MCS_POLICY_DELAY && e->cfg.trader; }

inline int fail(mcs_engine* e, int code, const std::string& msg) {
    if (e) e->err = msg;
    return code;
}

#define HIPCHK(e, call)                                                                      \
    do {                                                                                     \
        hipError_t _st = (call);                                                             \
        if (_st != hipSuccess)                                                               \
            return fail((e), MCS_E_HIP,                                                      \
                        std::string(#call) + ": " + hipGetErrorString(_st));                 \
    } while (0)

template <class T>
inline void dfree(T*& p) {
    if (p) (void)hipFree(p);
    p = nullptr;
}


inline int check_engine(mcs_engine* e) {
    if (!e) return MCS_E_INVALID;
    hipError_t st = hipSetDevice(e->device);
    if (st != hipSuccess) return fail(e, MCS_E_HIP, std::string("hipSetDevice: ") + hipGetErrorString(st));
    return MCS_OK;
}
