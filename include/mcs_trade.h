/*
 * mcs_trade.h — lock-step trading extension of the MI355X engine (libmcs.so): the FIFO borrow
 * protocol and the per-cluster trader, batched over many clusters and sharded over GPUs.
 *
 * Replaces (reference snapshot 2024-10-16):
 *   Scheduler.BorrowResources        pkg/scheduler/server.go:160-248  (borrow broadcast)
 *   "/borrow" handler + Lend         pkg/scheduler/server.go:80-113, scheduler.go:194-202
 *   LentQueue service in Fifo        pkg/scheduler/scheduler.go:277-290
 *   Trader.RequestPolicyMonitor      pkg/trader/trader.go:280-325
 *   Trader.Trade + contractResHeap   pkg/trader/trader.go:169-278
 *   traderServer.RequestResource /
 *   ApproveContract                  pkg/trader/server.go:31-85
 *   ApproveTrade                     pkg/trader/trader.go:141-167
 *   Start (state stream)             pkg/scheduler/trader_server.go:24-47
 *   AddVirtualNode /
 *   AllocateVirtualNodeResources     pkg/scheduler/cluster.go:65-125
 * Semantics: the lock-step serialization of DESIGN.md §9 (tick T: scheduler steps, borrow
 * exchange, state samples, trader rounds), bit-identical to oracle/mcs_oracle_trade.c.  With
 * MCS_POLICY_DELAY the schedulers run Scheduler.Delay and the traders size real contracts from
 * Level1 (oracle/mcs_oracle_dtrade.c): Foreign jobs on responders, virtual nodes
 * with capacity on requesters.  DELAY trading shards too: its tick exchanges one block per rank
 * (per-cluster records + node snapshots) and runs the trader rounds replicated on every rank.
 *
 * Sharding: the clusters are split in equal contiguous blocks over `world` engines (one per GPU,
 * usually one process each).  A tick of either policy needs one all-gather of one block per rank
 * (per-cluster records + node snapshots; phase 0 -> 1; phases 2 and 3 move no bytes): the
 * remaining phases run replicated over the whole system on every rank.  Every rank must hold the
 * same number of clusters and the same largest cluster (the block layout).
 * Two transports:
 *   - RCCL (mcs_comm_unique_id on rank 0, shared out of band, then mcs_comm_init on every rank):
 *     mcs_run drives the whole lock-step loop with ncclAllGather over xGMI;
 *   - caller-driven (no communicator): the caller runs the ticks with mcs_trade_phase and moves
 *     the bytes between ranks itself (any transport; tests use torch.distributed gloo).
 * With world == 1 neither is needed: mcs_run keeps the exchange in HBM.
 */
#ifndef MCS_TRADE_H
#define MCS_TRADE_H

#include "mcs.h"

#ifdef __cplusplus
extern "C" {
#endif

/* One lent-job execution: the lender ran the borrower's job (index within the BORROWER's stream)
 * after accepting it on a /borrow request.  Every acceptor runs its own copy (server.go:232-237). */
typedef struct mcs_lent_rec {
    uint32_t lender, borrower; /* global cluster indices */
    uint64_t job;              /* job index in the borrower's stream */
    uint32_t node, start_s, finish_s, pad;
} mcs_lent_rec;

/* One trader round whose request policy broke (trader.go:288-303). */
typedef struct mcs_trade_rec {
    uint32_t t_s;       /* tick of the round */
    uint32_t requester; /* global cluster index */
    int32_t winner;     /* responder whose virtual node was received, -1 = "couldn't acquire resources" */
    uint32_t approvals; /* approving responses pushed on the heap */
} mcs_trade_rec;

/* One trader round of a DELAY system (MCS_POLICY_DELAY + trader), with its contract
 * (calculateFastNodeSize / calculateSmallNodeSize, pkg/trader/scheduler_client.go:126-289). */
typedef struct mcs_contract_rec {
    uint32_t t_s, requester;
    int32_t winner;     /* responder whose AllocateVirtualNodeResources succeeded, -1 = none    */
    uint32_t approvals;
    uint32_t policy;    /* 0 = WaitTime (fast node, trader.go:304-320), 1 = Utilization (small) */
    uint32_t cores, mem, time_s; /* the ContractRequest (trader.proto:20-27); price is 0        */
    uint32_t failed;    /* popped approvals whose ApproveContract failed before the winner       */
    uint32_t pad;
} mcs_contract_rec;

/* One Foreign job launched on a responder by AllocateVirtualNodeResources (cluster.go:87-125):
 * it holds {c, m} of node `node` of cluster `responder` from start_s to finish_s.  c and m are
 * Go uint values (cluster.go:116): they may exceed what the node had (the counter wraps). */
typedef struct mcs_foreign_rec {
    uint32_t requester, responder, node, start_s, finish_s, pad;
    uint64_t c, m;
} mcs_foreign_rec;

typedef struct mcs_trade_stats {
    uint64_t placed;       /* own jobs placed locally */
    uint64_t borrowed;     /* own jobs moved to the BorrowedQueue */
    uint64_t waited;       /* own jobs that entered the WaitQueue */
    uint64_t undecided;    /* own jobs neither placed nor borrowed (t_max reached) */
    uint64_t lent_runs;    /* lent-job executions on this engine's clusters */
    uint64_t lent_pending; /* LentQueue entries never run */
    uint64_t trades;       /* trader rounds with a broken policy (all clusters, replicated) */
    uint64_t trades_won;   /* ... that received a virtual node */
    uint32_t ticks;        /* lock-step ticks executed (fast-forward skips idle seconds) */
    uint32_t t_final;      /* last tick */
    uint32_t flags;        /* OR of MCS_FLAG_* over clusters and logs */
    uint32_t loop_form;    /* tick loop that ran: 0 = one engine, hipGraph-replayed ticks; 1 = RCCL
                              all-gather per tick, eager launches; 2 = RCCL, kernels and all-gathers
                              captured in a hipGraph (MCS_RCCL_GRAPH=0 forces 1); 3 = one
                              engine, the whole system resident in one workgroup; 4 = resident,
                              one workgroup per 4 clusters, exchange written through to memory;
                              5 = the same with every workgroup on one XCD, exchange in its L2;
                              6 = form 0 after a resident exchange timed out (workers not all
                              resident at once: the run was redone on the replayed kernels);
                              7 = RCCL, ONE launch per tick (phases B-D of tick n + A of tick
                              n + 1, mcs_trade_rk.hip) and one all-gather, captured in a hipGraph;
                              8 = the same, eager; 9 = the one-launch tick on the caller-driven
                              phase API (MCS_TRADE_RK=0: the three-kernel forms 0-2) */
    double kernel_ms;      /* device time of the lock-step loop (HIP events) */
    double wall_ms;
    /* ABI v7: the exchange-block layout the run used (equal on every rank) */
    uint64_t block_bytes;  /* bytes of one rank's exchange block (the all-gather's per-rank slice) */
    uint32_t snaps;        /* 1 = the blocks carry node snapshots; 0 = records + G tables only
                              (the one-launch tick when no rank has a node above 64 cores) */
    uint32_t agreed;       /* 1 = the layout was agreed over all ranks (the RCCL loop's shape
                              all-reduce, or mcs_trade_set_shape on the caller-driven path) */
} mcs_trade_stats;

/* ---- sharding and transport ------------------------------------------------------------------- */
typedef struct mcs_comm_id {
    char bytes[128]; /* ncclUniqueId */
} mcs_comm_id;

/* This engine holds clusters [rank*C, rank*C + C) of world*C (C = mcs_num_clusters).  Call after
 * mcs_load_clusters; default is rank 0 of 1. */
int mcs_set_shard(mcs_engine* eng, uint32_t rank, uint32_t world);
/* RCCL transport: ncclGetUniqueId (rank 0) and ncclCommInitRank on this engine's device. */
int mcs_comm_unique_id(mcs_comm_id* out);
int mcs_comm_init(mcs_engine* eng, const mcs_comm_id* id);

/* ---- caller-driven lock-step ---------------------------------------------------------------- */
/* One tick is phases 0..3.  Phase p reads `in` (the all-gather, in rank order, of every rank's
 * `out` of phase p-1; phase 0 takes no input) and writes this rank's slice for the next
 * exchange.  Sizes per phase from mcs_trade_xfer_bytes: today only phase 0 writes (this rank's
 * block) and only phase 1 reads (every rank's blocks); the other sizes are 0 and an empty output
 * need not be gathered.  *done becomes 1 (identically on every rank) after the phase 3
 * that ends the run; keep calling phase 0..3 until then.  mcs_trade_begin resets the lock-step
 * state; mcs_trade_end fills the stats and makes the results readable. */
int mcs_trade_begin(mcs_engine* eng);
/* Agreed block layout (ABI v7).  The RCCL loop agrees on the exchange-block layout with one
 * all-reduce (MAX) before the run.  The caller-driven transport does the same through these two
 * calls, made after mcs_set_shard / mcs_submit_jobs and before mcs_trade_begin:
 * mcs_trade_shape_words writes this rank's MCS_TRADE_SHAPE_WORDS words; the caller takes their
 * element-wise MAX over all ranks and passes the result to mcs_trade_set_shape on every rank.  The
 * agreed shape fixes the snapshot stride (the largest cluster of the system), whether every rank
 * runs the one-launch tick (one rank that cannot, or has MCS_TRADE_RK=0, turns it off for all) and
 * whether the blocks drop the node snapshots (no node above 64 cores on any rank: 320 B per
 * cluster, the layout an 8-GPU RCCL run uses).  A cluster-count mismatch fails (MCS_E_INVALID) on
 * every rank.  Without an agreed shape each rank decides from its own shard and the blocks keep
 * the snapshots.  Every caller-driven phase-0 block ends in a 16-byte layout tag (tick form,
 * snapshots, stride, clusters, policy); phase 1 fails with MCS_E_INVALID when the gathered blocks'
 * tags differ, so ranks that chose different layouts never exchange silently. */
#define MCS_TRADE_SHAPE_WORDS 8
int mcs_trade_shape_words(mcs_engine* eng, uint32_t* out);
int mcs_trade_set_shape(mcs_engine* eng, const uint32_t* agreed);
int mcs_trade_xfer_bytes(mcs_engine* eng, uint32_t phase, uint64_t* in_bytes, uint64_t* out_bytes);
int mcs_trade_phase(mcs_engine* eng, uint32_t phase, const void* in, uint64_t in_bytes, void* out,
                    uint64_t out_bytes, uint32_t* done);
int mcs_trade_end(mcs_engine* eng, mcs_stats* stats);

/* ---- results (after mcs_run or mcs_trade_end) ---------------------------------------------- */
int mcs_read_trade_stats(mcs_engine* eng, mcs_trade_stats* out);
/* Lent runs executed by this engine's clusters, sorted by (start_s, lender, borrower, job).
 * *n = total count (may exceed cap: then only cap records are written). */
int mcs_read_lent(mcs_engine* eng, mcs_lent_rec* out, uint64_t cap, uint64_t* n);
/* Trader rounds of ALL clusters in (t_s, requester) order (identical on every rank). */
int mcs_read_trades(mcs_engine* eng, mcs_trade_rec* out, uint64_t cap, uint64_t* n);
/* Virtual nodes received by each of the world*C clusters (AddVirtualNode, cluster.go:65-85):
 * zero-capacity under FIFO, the contract's capacity under DELAY. */
int mcs_read_virtual_nodes(mcs_engine* eng, uint32_t* out, uint32_t n_total);

/* ---- DELAY trading (MCS_POLICY_DELAY with cfg.trader) ----------------------------------------- */
/* Trader rounds of ALL clusters with their contracts, in (t_s, requester) order, identical on
 * every rank; *n = total count. */
int mcs_read_contracts(mcs_engine* eng, mcs_contract_rec* out, uint64_t cap, uint64_t* n);
/* Foreign jobs of ALL clusters in launch order (global indices, identical on every rank). */
int mcs_read_foreign(mcs_engine* eng, mcs_foreign_rec* out, uint64_t cap, uint64_t* n);
/* Capacities {cores, memory} of the virtual nodes local cluster `cluster` received, in order (node
 * index n_physical + i); *n = their count. */
int mcs_read_virtual_node_caps(mcs_engine* eng, uint32_t cluster, uint32_t* cores, uint32_t* mem,
                               uint32_t cap, uint32_t* n);

/* ---- single-call mirror of the approval rule ---------------------------------------------------- */
/* Trader.ApproveTrade (pkg/trader/trader.go:141-167) with the reference's approvePolicy{0.8, 0.8, -1,
 * -1} (trader.go:47-52): a responder whose sample is {core_util, mem_util} and whose totals are
 * {total_cores, total_memory} (SetTotalResources, uint32) asked for the contract {cores, memory,
 * time_s, price 0}.  Evaluated on the GPU by the same device function both trader kernels call
 * (float32 availability T - T*u and float64 incentive in Go's order, no FMA contraction). */
typedef struct mcs_approve_query {
    uint32_t total_cores, total_memory;
    float core_util, mem_util;
    uint32_t cores, memory, time_s, pad;
} mcs_approve_query;

/* out[i] = 1 (approve) or 0 for each of the n queries. */
int mcs_approve_trade(mcs_engine* eng, const mcs_approve_query* q, uint32_t n, int32_t* out);

#ifdef __cplusplus
}
#endif
#endif /* MCS_TRADE_H */
