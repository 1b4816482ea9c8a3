// mcs_fifo_asm.hip — the batched FIFO decision loop, hand-scheduled for gfx950.
//
// Same algorithm and results as fifo_kernel<4, 8, false, false, false> (mcs_kernels.hip):
// Scheduler.Fifo (pkg/scheduler/scheduler.go:216-296) over ScheduleJob's first fit (:127-139) and
// Node.RunJob's commit/release (pkg/scheduler/cluster.go:141-161), one cluster (up to 256 nodes)
// per wave64, SFIFO semantics with the exact fast-forward of SURVEY Appendix A.3.  The whole
// decision loop (batches, passes, releases, waits) is one asm statement on fixed registers, so
// the shape of each pass is chosen here instead of by the CFG structurizer.  Two node formats:
//
//   * W32 (every node free value < 2^31 - 1, checked on the host): node c of a lane is a VGPR
//     pair C = 2^31 + free_c, M = 2^31 + free_m; requests are clamped to 2^31 - 1 when a batch is
//     loaded (which cannot change a fit).  a = C - cores and b = M - mem keep bit 31 exactly when
//     the node fits, so (a & b) >> 31 is the fit bit; two v_perm (sign-replicating selectors)
//     gather the four chunks' bits into one byte mask per lane.
//   * W16 (every node free value < 2^15 - 1: the reference's cluster specs, 32 cores / 24000 MB):
//     node c is ONE VGPR {2^15 + free_c | (2^15 + free_m) << 16} and the request one SGPR
//     {cores | mem << 16} (each clamped to 2^15 - 1); one v_pk_sub_u16 per chunk leaves bits 15
//     and 31 set exactly when the node fits, one SDWA v_and per chunk folds them into one bit per
//     half word, and one v_perm gathers the byte mask: 10 VALU per first fit instead of 16, one
//     register move per commit, one record broadcast less per pass, u32 LDS node words.
//   Padding nodes hold 2^(W-1) - 1 in each field (no guard, and no clamped request wraps it):
//   they never fit, not even a zero job.  One v_cmp gives the lanes with a fit.
//   * Commit without branches: the lowest set byte of lane fl's mask is its first fitting chunk
//     c; under exec = lane fl, an indexed move (s_set_gpr_idx_on) copies the already computed
//     fit-test difference into that chunk's register(s).
//   * Slot insert under exec = the lowest lane with a free row (s_ff1 of the free-row lanes,
//     ANDed back with them); a full pool leaves exec empty and is caught by peak > 64*P at the
//     batch end (the cluster is re-run with a bigger pool by the engine, as for the compiled
//     kernel).  The counters (used, peak, waited, passes) are scalar.
//   * The cursor's lane in the batch lives in m0 for the result batch writes (v_writelane) and
//     in s47 for the record broadcasts (v_readlane).
//   * Release at a clock advance: every slot row's expiry lane mask is computed before the first
//     row is visited (no row waits on its own compare), then each row with an expiry hands its
//     payloads back under exec = that mask.  The slot's node word is the node's LDS address.
//   * The ready head's arrival/clock checks and the WaitQueue bookkeeping follow fifo_kernel line
//     by line (see the comments there); the result batch keeps the node's LDS index
//     (chunk * 64 + lane) and converts it to the node index when it is stored.
//
// Hazards (wait states are not inserted by the compiler inside asm): DPP reads a VGPR 2 states
// after its write (s_nop 1), v_readlane reads a VGPR at least 1 instruction after its write, m0
// is read by v_writelane at least 1 state after an SALU write.  Loads and stores issued here are
// waited for before the statement ends.  The loop runs with the full wave in exec.
#include "mcs_gen_dev.h"
#include "mcs_internal.h"
#include "mcs_lds.h"
#include "mcs_wave.h"

namespace mcs {

namespace {

#ifdef MCS_STAMPS
__device__ unsigned long long g_fa_stamps[5];  // [4]: the duo loop's header re-reads
#endif

#include "mcs_fa_macros.h"

// ---- the decision loop ------------------------------------------------------------------------
#define MCS_FA_ENTRY_S(W)                                                                         \
    /* ---- entry: state into the fixed registers ---- */                                        \
    "s_mov_b32 s40, %[t]\n\t"                                                                     \
    "s_mov_b32 s42, %[J]\n\t"                                                                     \
    "s_mov_b32 s43, 0\n\t"                                                                        \
    "s_mov_b32 s44, 0\n\t"                                                                        \
    "s_mov_b32 s47, 0\n\t"                                                                        \
    "s_mov_b32 s57, 0\n\t"                                                                        \
    "s_mov_b32 s78, 0\n\t"                                                                        \
    "s_lshl2_add_u32 s79, s42, 0x100\n\t"                                                         \
    "s_mov_b32 s80, 0\n\t"                                                                        \
    "s_mov_b32 s81, 0\n\t"                                                                        \
    "s_mov_b32 s82, 0\n\t"                                                                        \
    "s_mov_b32 s83, 0\n\t"                                                                        \
    "s_mov_b32 s84, 0\n\t"                                                                        \
    "s_mov_b32 s77, -1\n\t" /* nothing running */                                                \
    "s_mov_b64 s[64:65], %[jobs]\n\t"                                                             \
    "s_mov_b64 s[66:67], %[onp]\n\t"                                                              \
    "s_mov_b64 s[68:69], %[osp]\n\t"                                                              \
    "s_mov_b64 s[70:71], %[ofp]\n\t"                                                              \
    "s_mov_b32 s72, %[sel0]\n\t"                                                                  \
    "s_mov_b32 s73, %[sel1]\n\t"                                                                  \
    "v_mov_b32 v89, %[frm]\n\t"                                                                   \
    "v_mov_b32 v90, %[lmin]\n\t"                                                                  \
    "v_mov_b32 v94, %[c0]\n\t"                                                                    \
    "v_mov_b32 v95, %[c1]\n\t"                                                                    \
    "v_mov_b32 v96, %[c2]\n\t"                                                                    \
    "v_mov_b32 v97, %[c3]\n\t"                                                                    \
    "v_mov_b32 v107, %[pay]\n\t"                                                                  \
    "v_mov_b32 v108, %[nb]\n\t"                                                                   \
    "v_mov_b32 v109, %[nbase]\n\t"                                                                \
    "v_mov_b32 v110, %[lane]\n\t"                                                                 \
    "v_mov_b32 v111, -1\n\t" MCS_FA_INIT##W MCS_FA_RELOAD##W "s_waitcnt lgkmcnt(0)\n\t" MCS_FA_TSTART \
    /* prefetch batch 1 */                                                                        \
    "v_lshlrev_b32 v121, 4, v110\n\t"                                                             \
    "v_add_u32 v121, 0x400, v121\n\t"                                                             \
    "global_load_dwordx4 v[98:101], v121, s[64:65]\n\t"                                           \
    "s_min_u32 s41, s42, 64\n\t" MCS_FA_REC##W                                                    \
    "s_cmp_lt_u32 s47, s41\n\t"                                                                   \
    "s_cbranch_scc0 mcsfa_bend_%=\n"

#define MCS_FA_BODY(W, D, F)                                                                      \
    /* ---- one pass = one decision (scheduler.go:216-296) ---- */                               \
    "mcsfa_inner_%=:\n\t"                                                                         \
    "s_cmp_gt_u32 s45, s40\n\t" /* ready head not arrived: sleep to it */                         \
    "s_cbranch_scc1 mcsfa_arrive_%=\n\t" MCS_FA_FIT##W MCS_FA_ANYFIT##W                           \
    "s_add_u32 s55, s40, s46\n\t"                                                                 \
    "s_cbranch_vccz mcsfa_nofit_%=\n\t"                                                           \
    "s_ff1_i32_b64 s50, vcc\n\t" /* lowest lane with a fit */                                     \
    "s_cmp_eq_u32 s46, 0\n\t"                                                                     \
    "s_cbranch_scc1 mcsfa_zero_%=\n\t"                                                            \
    MCS_FA_DECIDE##W                                                                              \
    "s_min_u32 s77, s77, s55\n\t" /* the wave's earliest finish */                                \
    "s_mov_b64 exec, -1\n\t"                                                                      \
    "s_mov_b32 m0, s47\n\t"                                                                       \
    "s_add_u32 s80, s80, 1\n\t"                                                                   \
    "v_writelane_b32 v91, s54, m0\n\t"                                                            \
    "v_writelane_b32 v92, s40, m0\n"                                                              \
    /* next ready job; a WaitQueue head placed sleeps 1 s (:250) */                               \
    "mcsfa_placed_%=:\n\t"                                                                        \
    "s_add_u32 s47, s47, 1\n\t"                                                                   \
 MCS_FA_REC##W                                                                                   \
    "mcsfa_loopend_%=:\n\t"                                                                       \
    "s_cmp_lt_u32 s47, s41\n\t"                                                                   \
    "s_cbranch_scc1 mcsfa_inner_%=\n\t"                                                           \
    /* the pass bound ends here after a placed WaitQueue head (s41 = its cursor + 1 while one */  \
    /* waits): it sleeps 1 s (:250) with the batch bound restored */                             \
    "s_cmp_lg_u32 s43, 0\n\t"                                                                     \
    "s_cbranch_scc0 mcsfa_bend_%=\n\t"                                                            \
    "s_sub_u32 s41, s42, s57\n\t"                                                                 \
    "s_min_u32 s41, s41, 64\n\t"                                                                  \
    /* (the clock moves by t + 1 here and on a failed fit: the carry is the u32 clock's overflow) */ \
    "s_mov_b32 s43, 0\n\t"                                                                        \
    "s_add_u32 s40, s40, 1\n\t"                                                                   \
    "s_cbranch_scc1 mcsfa_clkovf_%=\n\t"                                                          \
    "s_branch mcsfa_adv_%=\n"                                                                     \
                                                                                                  \
    /* zero-duration job: committed and released before the next decision (D3) */               \
    "mcsfa_zero_%=:\n\t" MCS_FA_ZEROKX##W                                                        \
    "v_writelane_b32 v91, s54, m0\n\t"                                                            \
    "v_writelane_b32 v92, s40, m0\n\t"                                                            \
    "s_branch mcsfa_placed_%=\n"                                                                  \
                                                                                                  \
    "mcsfa_arrive_%=:\n\t"                                                                        \
    "s_mov_b32 s40, s45\n\t" /* (> t) */                                                         \
    MCS_FA_CNTS_##D                                                                               \
    "s_branch mcsfa_adv_%=\n"                                                                     \
                                                                                                  \
    /* no node fits: WaitQueue append (:264-268), sleep to the next completion (A.3); falls */   \
    /* through to the release (a failed head sleeps to a completion, so it always releases) */  \
    "mcsfa_nofit_%=:\n\t" MCS_FA_T0                                                              \
    "s_sub_u32 s76, 1, s43\n\t"                                                                   \
    "s_add_u32 s82, s82, s76\n\t"                                                                 \
    "s_mov_b32 s43, 1\n\t"                                                                        \
    "s_add_u32 s41, s47, 1\n\t" /* the passes stop right after this head is placed */             \
    MCS_FA_CNTS_##D                                                                               \
    /* runaway guard: every advance moves the clock forward and a loop without decisions goes */  \
    /* through here; at most 2 failed fits per job (one per arrival, one per completion) */      \
    "s_add_u32 s78, s78, 1\n\t"                                                                   \
    "s_cmp_gt_u32 s78, s79\n\t"                                                                   \
    "s_cbranch_scc1 mcsfa_poolovf_%=\n\t"                                                         \
    "s_cmp_eq_u32 s77, -1\n\t"                                                                    \
    "s_cbranch_scc1 mcsfa_deadlock_%=\n\t"                                                        \
    "s_add_u32 s40, s40, 1\n\t"                                                                   \
    "s_cbranch_scc1 mcsfa_clkovf_%=\n\t"                                                          \
    "s_max_u32 s40, s40, s77\n\t" /* (every running job finishes after t: no wrap) */           \
    MCS_FA_T1("s95")                                                                              \
    /* the clock has advanced: releases at the new instant (A.2 step 1) */                       \
    "mcsfa_adv_%=:\n\t"                                                                           \
    "s_cmp_lt_u32 s40, s77\n\t" /* nothing finishes by t: no release */                          \
    "s_cbranch_scc1 mcsfa_loopend_%=\n\t"                                                         \
    /* release every running job with finish <= t (cluster.go:153-157) */                        \
    MCS_FA_CNTR_##D MCS_FA_T0                                                                     \
    "s_max_u32 s81, s81, s80\n\t" /* peak: used only grows between releases */                   \
    "s_add_u32 s74, s40, 1\n\t" MCS_FA_SCAN##W MCS_FA_SCANEND##W MCS_FA_T1("s94")                \
    /* (loopend's test, so the usual continuation is one taken branch) */                        \
    "s_cmp_lt_u32 s47, s41\n\t"                                                                   \
    "s_cbranch_scc1 mcsfa_inner_%=\n\t"                                                           \
    "s_branch mcsfa_loopend_%=\n" MCS_FA_RBODY##W                                                 \
                                                                                                  \
    "mcsfa_deadlock_%=:\n\t"                                                                      \
    "s_or_b32 s44, s44, %[fdl]\n\t"                                                               \
    "s_branch mcsfa_exit_%=\n"                                                                    \
    "mcsfa_clkovf_%=:\n\t"                                                                        \
    "s_mov_b32 s40, -1\n\t" /* the clock stays at the last second it reached */                   \
    "s_or_b32 s44, s44, %[fck]\n\t"                                                               \
    "s_branch mcsfa_exit_%=\n"                                                                    \
    "mcsfa_poolovf_%=:\n\t"                                                                       \
    "s_or_b32 s44, s44, %[fov]\n\t"                                                               \
    "s_branch mcsfa_exit_%=\n"                                                                    \
                                                                                                  \
    /* ---- batch end: store the 64 results, take the prefetched records, prefetch the next ---- */ \
    "mcsfa_bend_%=:\n\t" MCS_FA_T0                                                               \
    "s_max_u32 s81, s81, s80\n\t"                                                                 \
    "s_cmp_gt_u32 s81, " MCS_FA_POOLMAX##W "\n\t"                                                 \
    "s_cbranch_scc1 mcsfa_poolovf_%=\n\t" MCS_FA_BENDCHK##W                                       \
    "s_add_u32 s76, s57, s47\n\t"                                                                 \
    "s_cmp_ge_u32 s76, s42\n\t"                                                                   \
    "s_cbranch_scc1 mcsfa_exit_%=\n\t"                                                            \
    "s_waitcnt vmcnt(0)\n\t"                                                                      \
    "v_add_u32 v125, s57, v110\n\t"                                                               \
    "v_lshlrev_b32 v125, 2, v125\n\t"                                                             \
    MCS_FA_NODEIDX##W                                                                             \
    "global_store_dword v125, v126, s[66:67] nt\n\t"                                              \
    "global_store_dword v125, v92, s[68:69] nt\n\t"                                               \
    "v_add_u32 v93, v92, v95\n\t" /* finish = start + the batch's duration column */            \
    "global_store_dword v125, v93, s[70:71] nt\n\t"                                               \
    "s_add_u32 s57, s57, 64\n\t" MCS_FA_PRIO("mcsfa_") MCS_FA_BENDTAIL_##F(W)

// streamed records: the prefetched batch becomes current, the next one is prefetched
#define MCS_FA_BENDTAIL_S(W)                                                                      \
    MCS_FA_TAKE##W                                                                                \
    "v_add_u32 v121, s57, v110\n\t"                                                               \
    "v_lshlrev_b32 v121, 4, v121\n\t"                                                             \
    "v_add_u32 v121, 0x400, v121\n\t"                                                             \
    "global_load_dwordx4 v[98:101], v121, s[64:65]\n\t"                                           \
    "s_sub_u32 s41, s42, s57\n\t"                                                                 \
    "s_min_u32 s41, s41, 64\n\t"                                                                  \
    "s_mov_b32 s47, 0\n\t" MCS_FA_REC##W MCS_FA_T1("s96")                                         \
    "s_branch mcsfa_inner_%=\n"
// fused records: the statement ends with s59 = 1 and the kernel synthesises the next batch
#define MCS_FA_BENDTAIL_F(W)                                                                      \
    "s_mov_b32 s47, 0\n\t"                                                                        \
    "s_mov_b32 s59, 1\n\t" MCS_FA_T1("s96")                                                      \
    "s_branch mcsfa_exit_%=\n"

#define MCS_FA_EXIT_S                                                                             \
    /* ---- exit: state back to the compiler's registers ---- */                                 \
    "mcsfa_exit_%=:\n\t"                                                                          \
    "s_waitcnt vmcnt(0) lgkmcnt(0)\n\t" MCS_FA_TEND                                               \
    "s_mov_b32 %[t], s40\n\t"                                                                     \
    "s_add_u32 %[r], s57, s47\n\t"                                                                \
    "s_mov_b32 %[flags], s44\n\t"                                                                 \
    "s_mov_b32 %[hw], s43\n\t"                                                                    \
    "s_mov_b32 %[used], s80\n\t"                                                                  \
    "s_max_u32 %[peak], s81, s80\n\t"                                                             \
    "s_mov_b32 %[waited], s82\n\t"                                                                \
    "s_mov_b32 %[nslow], s83\n\t"                                                                 \
    "s_mov_b32 %[nrel], s84\n\t"                                                                  \
    "v_mov_b32 %[on], v91\n\t"                                                                    \
    "v_mov_b32 %[os], v92\n\t"                                                                    \
    /* finish = start + duration of the batch the result registers hold: the current records', */ \
    /* unless the run stopped at the first job of a new batch, whose previous batch was stored */  \
    /* with its finishes already formed in v93 (tests/test_gpu_parity.py fuzz cases) */           \
    "s_cmp_eq_u32 s47, 0\n\t"                                                                     \
    "s_cbranch_scc1 mcsfa_xf_%=\n\t"                                                              \
    "v_add_u32 v93, v92, v95\n"                                                                   \
    "mcsfa_xf_%=:\n\t"                                                                            \
    "v_mov_b32 %[of], v93\n\t"                                                                    \
    "v_mov_b32 %[frm], v89\n\t"                                                                   \
    "v_mov_b32 %[lmin], v90\n\t"                                                                  \
    "s_nop 1"

#define MCS_FA_LOOP(W, D) MCS_FA_ENTRY_S(W) MCS_FA_BODY(W, D, S) MCS_FA_EXIT_S

// ---- W16L: W16R with a one-job lookahead (r06; form 22) -----------------------
// Every pass also tests the NEXT job's request (s92, read one record ahead) against the nodes as they
// stand before this pass's commit (v76-v79 / v82-v83 -> byte masks v87, lanes s[94:95]), and picks
// its first fit s58 (kx = chunk * 64 + lane) at the end of the pass.  The next pass decides from s58
// without a fit test on its chain (the L pass) when nothing has changed since that test but this
// pass's commit: its node s59 (h) is then the only node whose fit may have changed, and it can only
// have lost one, so s58 != h is the exact first fit (scheduler.go:127-139: every lower node failed
// before and still fails; s58 itself is unchanged).  s58 == h (the next job's first fit is the node
// just committed; also the "no lookahead" code, s58 := s59) runs the full pass (F): W16R's fit test
// of the job interleaved with the next one's.  A release (nodes gain) and a batch end (new records)
// invalidate; an arrival advance without a release changes no node and keeps the lookahead.
// The insert's slot (lowest lane with a free row: s85, its row s86, exec mask s[62:63]) is picked at
// the end of the pass that changed the free rows (and after a release), off the next decision's chain.
// Each pass type ends with its own copy of the tail, so a pass takes one taken branch, to the next
// pass of either type.  The L pass commits with one indexed v_subrev (the job fits: the packed
// halves do not borrow).
//   s58 lookahead kx   s59 h   s92 next request   s[94:95] lanes where it fits   s96-s98 temps
//   v76-v79 next diffs   v82-v83 next fit bits   v87 next byte masks
// (r06 A/B against W16R, profiles/r06_look/: the first form, with the insert's slot on the chain and
// two taken branches per pass, measured 6.44 vs 4.96 ms at 512 clusters)
#define MCS_FL_SWEEP_A                                                                            \
    "v_pk_sub_u16 v76, v64, s92\n\t"                                                              \
    "v_pk_sub_u16 v77, v65, s92\n\t"                                                              \
    "v_pk_sub_u16 v78, v66, s92\n\t"                                                              \
    "v_pk_sub_u16 v79, v67, s92\n\t"                                                              \
    "v_and_b32_sdwa v82, v76, v76 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_0\n\t" \
    "v_and_b32_sdwa v83, v78, v78 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_0\n\t" \
    "v_and_b32_sdwa v82, v77, v77 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_0\n\t" \
    "v_and_b32_sdwa v83, v79, v79 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_0\n\t"
// (two instructions of the caller between A and B: the SDWA-preserve hazard of MCS_FA_FIT16)
#define MCS_FL_SWEEP_B                                                                            \
    "v_perm_b32 v87, v83, v82, s72\n\t"                                                           \
    "v_cmp_ne_u32_e64 s[94:95], 0, v87\n\t"
// the F pass's two fit tests (the job's: v72-v75 -> v80/v81 -> v86 and vcc; the next one's),
// interleaved so that each SDWA-preserve write has two instructions before its reader
#define MCS_FL_FIT2                                                                               \
    "v_pk_sub_u16 v72, v64, s48\n\t"                                                              \
    "v_pk_sub_u16 v73, v65, s48\n\t"                                                              \
    "v_pk_sub_u16 v74, v66, s48\n\t"                                                              \
    "v_pk_sub_u16 v75, v67, s48\n\t"                                                              \
    "v_pk_sub_u16 v76, v64, s92\n\t"                                                              \
    "v_pk_sub_u16 v77, v65, s92\n\t"                                                              \
    "v_pk_sub_u16 v78, v66, s92\n\t"                                                              \
    "v_pk_sub_u16 v79, v67, s92\n\t"                                                              \
    "v_and_b32_sdwa v80, v72, v72 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_0\n\t" \
    "v_and_b32_sdwa v81, v74, v74 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_0\n\t" \
    "v_and_b32_sdwa v82, v76, v76 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_0\n\t" \
    "v_and_b32_sdwa v83, v78, v78 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_0\n\t" \
    "v_and_b32_sdwa v80, v73, v73 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_0\n\t" \
    "v_and_b32_sdwa v81, v75, v75 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_0\n\t" \
    "v_and_b32_sdwa v82, v77, v77 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_0\n\t" \
    "v_and_b32_sdwa v83, v79, v79 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_0\n\t" \
    "v_perm_b32 v86, v81, v80, s72\n\t"                                                           \
    "v_cmp_ne_u32_e32 vcc, 0, v86\n\t"                                                            \
    "v_perm_b32 v87, v83, v82, s72\n\t"                                                           \
    "s_add_u32 s55, s40, s46\n\t"                                                                 \
    "v_cmp_ne_u32_e64 s[94:95], 0, v87\n\t"
// the record at the cursor, and the next record's request (lane 64 wraps to lane 0: a batch end
// invalidates whatever the last pass of the batch looked ahead at)
#define MCS_FL_REC                                                                                \
    "v_readlane_b32 s45, v94, s47\n\t"                                                            \
    "v_readlane_b32 s46, v95, s47\n\t"                                                            \
    "v_readlane_b32 s48, v96, s47\n\t"                                                            \
    "s_add_u32 s97, s47, 1\n\t"                                                                   \
    "s_and_b32 s97, s97, 63\n\t"                                                                  \
    "v_readlane_b32 s92, v96, s97\n\t"
// the next insert's slot from the free rows v89 (exec = the full wave): the vector half, then the
// scalar half a few instructions later (pool full: s[62:63] empty, s86 = 8, as MCS_FA_DECIDE16R)
#define MCS_FL_INSPICK_V                                                                          \
    "v_cmp_lt_u32_e64 s[60:61], s49, v89\n\t"                                                    \
    "v_ffbl_b32 v117, v89\n\t"
#define MCS_FL_INSPICK_S                                                                          \
    "s_ff1_i32_b64 s85, s[60:61]\n\t"                                                             \
    "v_readlane_b32 s86, v117, s85\n\t"                                                           \
    "s_lshl_b64 s[62:63], 1, s85\n\t"                                                             \
    "s_and_b64 s[62:63], s[62:63], s[60:61]\n\t"
// the L pass's decision: node s58 (lane s50); commit + slot insert in one register-index region
#define MCS_FL_DECIDE_L                                                                           \
    "s_lshr_b32 s53, s58, 6\n\t"                                                                  \
    "s_lshl_b64 exec, 1, s50\n\t"                                                                 \
    "s_lshl2_add_u32 s87, s58, s73\n\t"                                                           \
    "s_mov_b32 s54, s58\n\t"                                                                      \
    "s_set_gpr_idx_on s53, gpr_idx(SRC1,DST)\n\t"                                                 \
    "v_subrev_u32 v64, s48, v64\n\t" /* the commit (cluster.go:146-147) */                        \
    "s_mov_b64 exec, s[62:63]\n\t"                                                                \
    "s_set_gpr_idx_idx s86\n\t"                                                                   \
    "v_mov_b32 v32, s55\n\t"                                                                      \
    "v_mov_b32 v40, s48\n\t"                                                                      \
    "v_mov_b32 v48, s87\n\t"                                                                      \
    "s_set_gpr_idx_off\n\t"                                                                       \
    "s_lshl_b32 s76, 1, s86\n\t"                                                                  \
    "v_xor_b32 v89, s76, v89\n\t"
// the F pass's decision: MCS_FA_DECIDE16R with the insert's slot already picked
#define MCS_FL_DECIDE_F                                                                           \
    "v_readlane_b32 s51, v86, s50\n\t"                                                            \
    "s_lshl_b64 exec, 1, s50\n\t"                                                                 \
    "s_ff1_i32_b32 s52, s51\n\t"                                                                  \
    "s_lshr_b32 s53, s52, 3\n\t"                                                                  \
    "s_lshl3_add_u32 s54, s52, s50\n\t"                                                           \
    "s_set_gpr_idx_on s53, gpr_idx(SRC0,DST)\n\t"                                                 \
    "v_mov_b32 v64, v72\n\t" /* the commit (cluster.go:146-147) */                                \
    "s_mov_b64 exec, s[62:63]\n\t"                                                                \
    "s_lshl2_add_u32 s87, s54, s73\n\t"                                                           \
    "s_set_gpr_idx_idx s86\n\t"                                                                   \
    "v_mov_b32 v32, s55\n\t"                                                                      \
    "v_mov_b32 v40, s48\n\t"                                                                      \
    "v_mov_b32 v48, s87\n\t"                                                                      \
    "s_set_gpr_idx_off\n\t"                                                                       \
    "s_lshl_b32 s76, 1, s86\n\t"                                                                  \
    "v_xor_b32 v89, s76, v89\n\t"
// the end of a placing pass of type X (L or F): exec back, the next insert's slot, counters and
// results, the next job's first fit from the sweep (none: s58 = h, the next pass is an F pass),
// and the branch to the next pass (cursor past the pass bound: mcsfl_pend)
#define MCS_FL_TAIL(X, BACK)                                                                      \
    "s_mov_b32 s59, s54\n\t" /* h: the node this pass committed */                                \
    "s_mov_b64 exec, -1\n\t" MCS_FL_INSPICK_V                                                    \
    "s_min_u32 s77, s77, s55\n\t" /* the wave's earliest finish */                                \
    "s_mov_b32 m0, s47\n\t"                                                                       \
    "s_add_u32 s80, s80, 1\n\t"                                                                   \
    "v_writelane_b32 v91, s54, m0\n\t"                                                            \
    "v_writelane_b32 v92, s40, m0\n"                                                              \
    "mcsfl_pick" X "_%=:\n\t"                                                                     \
    "s_mov_b32 s58, s59\n\t"                                                                      \
    "s_cmp_lg_u64 s[94:95], 0\n\t"                                                                \
    "s_cbranch_scc0 mcsfl_nopick_%=\n\t"                                                          \
    "s_ff1_i32_b64 s96, s[94:95]\n\t"                                                             \
    "v_readlane_b32 s98, v87, s96\n\t" MCS_FL_INSPICK_S                                          \
    "s_add_u32 s47, s47, 1\n\t" MCS_FL_REC                                                        \
    "s_ff1_i32_b32 s98, s98\n\t"                                                                  \
    "s_lshl3_add_u32 s58, s98, s96\n\t"                                                           \
    "s_cmp_lt_u32 s47, s41\n\t"                                                                   \
    "s_cbranch_scc0 mcsfl_pend_%=\n\t"                                                            \
    "s_cmp_eq_u32 s58, s59\n\t" BACK
#define MCS_FL_BACK_L "s_cbranch_scc0 mcsfl_innerL_%=\n\ts_branch mcsfl_innerF_%=\n"
#define MCS_FL_BACK_F "s_cbranch_scc1 mcsfl_innerF_%=\n\ts_branch mcsfl_innerL_%=\n"

// W16R's release scan with the next insert's slot picked after its rows (they free slot rows)
#define MCS_FL_SCAN                                                                               \
    "ds_write_b32 v108, v64 offset:0\n\t"                                                        \
    "ds_write_b32 v108, v65 offset:256\n\t"                                                      \
    "ds_write_b32 v108, v66 offset:512\n\t"                                                      \
    "ds_write_b32 v108, v67 offset:768\n\t"                                                      \
    "s_mov_b32 s75, 0\n\t"                                                                       \
    "v_cmp_ge_u32_e64 s[50:51], s40, v32\n\t"                                                    \
    "v_cmp_ge_u32_e64 s[52:53], s40, v33\n\t"                                                    \
    "v_cmp_ge_u32_e64 s[54:55], s40, v34\n\t"                                                    \
    "v_cmp_ge_u32_e64 s[60:61], s40, v35\n\t"                                                    \
    "v_cmp_ge_u32_e64 s[62:63], s40, v36\n\t"                                                    \
    "v_cmp_ge_u32_e64 s[86:87], s40, v37\n\t"                                                    \
    "v_cmp_ge_u32_e64 s[88:89], s40, v38\n\t"                                                    \
    "v_cmp_ge_u32_e64 s[90:91], s40, v39\n\t"                                                    \
    MCS_FR_ROW(0, "s[50:51]", "v32", "v40", "v48") MCS_FR_ROW(1, "s[52:53]", "v33", "v41", "v49")  \
    MCS_FR_ROW(2, "s[54:55]", "v34", "v42", "v50") MCS_FR_ROW(3, "s[60:61]", "v35", "v43", "v51")  \
    MCS_FR_ROW(4, "s[62:63]", "v36", "v44", "v52") MCS_FR_ROW(5, "s[86:87]", "v37", "v45", "v53")  \
    MCS_FR_ROW(6, "s[88:89]", "v38", "v46", "v54") MCS_FR_ROW(7, "s[90:91]", "v39", "v47", "v55")  \
    "s_mov_b64 exec, -1\n\t" MCS_FL_INSPICK_V                                                    \
    "s_sub_u32 s80, s80, s75\n\t" MCS_FA_RELOAD16                                               \
    "v_min3_u32 v90, v32, v33, v34\n\t"                                                          \
    "v_min3_u32 v90, v90, v35, v36\n\t"                                                          \
    "v_min3_u32 v90, v90, v37, v38\n\t"                                                          \
    "v_min_u32 v90, v90, v39\n\t" MCS_FA_SCANEND16R MCS_FL_INSPICK_S

#define MCS_FL_ENTRY                                                                              \
    "s_mov_b32 s58, -1\n\t"                                                                       \
    "s_mov_b32 s59, -1\n\t" MCS_FA_ENTRY_S(16R)
// (MCS_FA_ENTRY_S(16R) ends with MCS_FA_REC16R and a branch to the batch end when the first batch is
// empty; the first pass also needs the next request and the insert's slot)
#define MCS_FL_BODY(D)                                                                            \
    "s_add_u32 s97, s47, 1\n\t"                                                                   \
    "s_and_b32 s97, s97, 63\n\t"                                                                  \
    "v_readlane_b32 s92, v96, s97\n\t" MCS_FL_INSPICK_V                                          \
    "s_nop 4\n\t" MCS_FL_INSPICK_S                                                                \
    "s_branch mcsfa_inner_%=\n"                                                                   \
    "mcsfa_loopend_%=:\n\t"                                                                       \
    "s_cmp_lt_u32 s47, s41\n\t"                                                                   \
    "s_cbranch_scc0 mcsfl_pend_%=\n"                                                              \
    "mcsfa_inner_%=:\n\t"                                                                         \
    "s_cmp_eq_u32 s58, s59\n\t" /* no usable lookahead: the F pass */                            \
    "s_cbranch_scc1 mcsfl_innerF_%=\n"                                                            \
    /* ---- L pass: the job's first fit is s58 ---- */                                            \
    "mcsfl_innerL_%=:\n\t"                                                                        \
    "s_cmp_gt_u32 s45, s40\n\t" /* ready head not arrived: sleep to it */                         \
    "s_cbranch_scc1 mcsfa_arrive_%=\n\t" MCS_FL_SWEEP_A                                          \
    "s_add_u32 s55, s40, s46\n\t"                                                                 \
    "s_and_b32 s50, s58, 63\n\t" MCS_FL_SWEEP_B                                                  \
    "s_cmp_eq_u32 s46, 0\n\t"                                                                     \
    "s_cbranch_scc1 mcsfl_lzero_%=\n\t" MCS_FL_DECIDE_L MCS_FL_TAIL("L", MCS_FL_BACK_L)          \
    "mcsfl_lzero_%=:\n\t"                                                                         \
    "s_mov_b32 m0, s47\n\t"                                                                       \
    "s_mov_b32 s54, s58\n\t"                                                                      \
    "v_writelane_b32 v91, s54, m0\n\t"                                                            \
    "v_writelane_b32 v92, s40, m0\n\t"                                                            \
    "s_branch mcsfl_pickL_%=\n"                                                                   \
    /* ---- F pass: W16R's fit test of the job, with the next one's ---- */                      \
    "mcsfl_innerF_%=:\n\t"                                                                        \
    "s_cmp_gt_u32 s45, s40\n\t"                                                                   \
    "s_cbranch_scc1 mcsfa_arrive_%=\n\t" MCS_FL_FIT2                                             \
    "s_cbranch_vccz mcsfa_nofit_%=\n\t"                                                           \
    "s_ff1_i32_b64 s50, vcc\n\t" /* lowest lane with a fit */                                     \
    "s_cmp_eq_u32 s46, 0\n\t"                                                                     \
    "s_cbranch_scc1 mcsfa_zero_%=\n\t" MCS_FL_DECIDE_F MCS_FL_TAIL("F", MCS_FL_BACK_F)           \
    "mcsfa_zero_%=:\n\t" MCS_FA_ZEROKX16R                                                        \
    "v_writelane_b32 v91, s54, m0\n\t"                                                            \
    "v_writelane_b32 v92, s40, m0\n\t"                                                            \
    "s_branch mcsfl_pickF_%=\n"                                                                   \
    /* a pass whose next job fits no node (before the commit, so none after it either) */        \
    "mcsfl_nopick_%=:\n\t" MCS_FL_INSPICK_S                                                       \
    "s_add_u32 s47, s47, 1\n\t" MCS_FL_REC                                                        \
    "s_branch mcsfa_loopend_%=\n"                                                                 \
    /* the cursor reached the pass bound: a placed WaitQueue head sleeps 1 s (:250), or the */    \
    /* batch ends */                                                                              \
    "mcsfl_pend_%=:\n\t"                                                                          \
    "s_cmp_lg_u32 s43, 0\n\t"                                                                     \
    "s_cbranch_scc0 mcsfa_bend_%=\n\t"                                                            \
    "s_sub_u32 s41, s42, s57\n\t"                                                                 \
    "s_min_u32 s41, s41, 64\n\t"                                                                  \
    "s_mov_b32 s43, 0\n\t"                                                                        \
    "s_add_u32 s40, s40, 1\n\t"                                                                   \
    "s_cbranch_scc1 mcsfa_clkovf_%=\n\t"                                                          \
    "s_branch mcsfa_adv_%=\n"                                                                     \
                                                                                                  \
    "mcsfa_arrive_%=:\n\t"                                                                        \
    "s_mov_b32 s40, s45\n\t"                                                                      \
    MCS_FA_CNTS_##D                                                                               \
    "s_branch mcsfa_adv_%=\n"                                                                     \
                                                                                                  \
    "mcsfa_nofit_%=:\n\t"                                                                         \
    "s_sub_u32 s76, 1, s43\n\t"                                                                   \
    "s_add_u32 s82, s82, s76\n\t"                                                                 \
    "s_mov_b32 s43, 1\n\t"                                                                        \
    "s_add_u32 s41, s47, 1\n\t"                                                                   \
    MCS_FA_CNTS_##D                                                                               \
    "s_add_u32 s78, s78, 1\n\t"                                                                   \
    "s_cmp_gt_u32 s78, s79\n\t"                                                                   \
    "s_cbranch_scc1 mcsfa_poolovf_%=\n\t"                                                         \
    "s_cmp_eq_u32 s77, -1\n\t"                                                                    \
    "s_cbranch_scc1 mcsfa_deadlock_%=\n\t"                                                        \
    "s_add_u32 s40, s40, 1\n\t"                                                                   \
    "s_cbranch_scc1 mcsfa_clkovf_%=\n\t"                                                          \
    "s_max_u32 s40, s40, s77\n"                                                                   \
    "mcsfa_adv_%=:\n\t"                                                                           \
    "s_cmp_lt_u32 s40, s77\n\t"                                                                   \
    "s_cbranch_scc1 mcsfa_loopend_%=\n\t"                                                         \
    MCS_FA_CNTR_##D                                                                               \
    "s_max_u32 s81, s81, s80\n\t"                                                                 \
    "s_mov_b32 s58, s59\n\t" /* a release: the lookahead is void */                               \
    "s_add_u32 s74, s40, 1\n\t" MCS_FL_SCAN                                                      \
    "s_cmp_lt_u32 s47, s41\n\t"                                                                   \
    "s_cbranch_scc1 mcsfl_innerF_%=\n\t"                                                          \
    "s_branch mcsfl_pend_%=\n" MCS_FA_RBODY16R                                                    \
                                                                                                  \
    "mcsfa_deadlock_%=:\n\t"                                                                      \
    "s_or_b32 s44, s44, %[fdl]\n\t"                                                               \
    "s_branch mcsfa_exit_%=\n"                                                                    \
    "mcsfa_clkovf_%=:\n\t"                                                                        \
    "s_mov_b32 s40, -1\n\t"                                                                       \
    "s_or_b32 s44, s44, %[fck]\n\t"                                                               \
    "s_branch mcsfa_exit_%=\n"                                                                    \
    "mcsfa_poolovf_%=:\n\t"                                                                       \
    "s_or_b32 s44, s44, %[fov]\n\t"                                                               \
    "s_branch mcsfa_exit_%=\n"                                                                    \
                                                                                                  \
    "mcsfa_bend_%=:\n\t"                                                                          \
    "s_max_u32 s81, s81, s80\n\t"                                                                 \
    "s_cmp_gt_u32 s81, 64*8\n\t"                                                                  \
    "s_cbranch_scc1 mcsfa_poolovf_%=\n\t"                                                         \
    "s_add_u32 s76, s57, s47\n\t"                                                                 \
    "s_cmp_ge_u32 s76, s42\n\t"                                                                   \
    "s_cbranch_scc1 mcsfa_exit_%=\n\t"                                                            \
    "s_waitcnt vmcnt(0)\n\t"                                                                      \
    "v_add_u32 v125, s57, v110\n\t"                                                               \
    "v_lshlrev_b32 v125, 2, v125\n\t" MCS_FA_NODEIDX                                              \
    "global_store_dword v125, v126, s[66:67] nt\n\t"                                              \
    "global_store_dword v125, v92, s[68:69] nt\n\t"                                               \
    "v_add_u32 v93, v92, v95\n\t"                                                                 \
    "global_store_dword v125, v93, s[70:71] nt\n\t"                                               \
    "s_add_u32 s57, s57, 64\n\t" MCS_FA_PRIO("mcsfa_") MCS_FA_TAKE16                              \
    "v_add_u32 v121, s57, v110\n\t"                                                               \
    "v_lshlrev_b32 v121, 4, v121\n\t"                                                             \
    "v_add_u32 v121, 0x400, v121\n\t"                                                             \
    "global_load_dwordx4 v[98:101], v121, s[64:65]\n\t"                                           \
    "s_sub_u32 s41, s42, s57\n\t"                                                                 \
    "s_min_u32 s41, s41, 64\n\t"                                                                  \
    "s_mov_b32 s47, 0\n\t"                                                                        \
    "s_mov_b32 s58, s59\n\t" /* new records: the lookahead is void */                            \
    MCS_FL_REC                                                                                    \
    "s_branch mcsfl_innerF_%=\n"
#define MCS_FL_LOOP(D) MCS_FL_ENTRY MCS_FL_BODY(D) MCS_FA_EXIT_S
// the lookahead loop's clobbers: W16R's plus its own (no probe build of this form: MCS_STAMPS uses
// s92-s99 for its segment clocks)
#define MCS_FL_CLOBBERS MCS_FA_CLOBBERS, "s92", "s93", "s94", "s95", "s96", "s97", "s98"

// ---- the loop with the job stream synthesised in the kernel (mcs_gen_params.fused) ---------------
// The statement runs one batch of records and ends at its batch end with s59 = 1 (or at the end of
// the cluster with s59 = 0); the kernel then generates the next batch (GenStream, mcs_gen_dev.h)
// into v[98:101] and enters again.  The loop state stays in its fixed registers between the
// statements: they are the statement's register-bound operands ({s40}, {v[32:39]}, ...), so the
// compiler keeps them there (or moves them back) across the generator's code.  Every entry sets the
// constants again; the first (s59 = 0) also loads the nodes and takes batch 0 from the operands.
#define MCS_FA_ENTRY_F(W)                                                                         \
    "s_mov_b32 s42, %[J]\n\t"                                                                     \
    "s_lshl2_add_u32 s79, s42, 0x100\n\t"                                                         \
    "s_mov_b64 s[66:67], %[onp]\n\t"                                                              \
    "s_mov_b64 s[68:69], %[osp]\n\t"                                                              \
    "s_mov_b64 s[70:71], %[ofp]\n\t"                                                              \
    "s_mov_b32 s72, %[sel0]\n\t"                                                                  \
    "s_mov_b32 s73, %[sel1]\n\t"                                                                  \
    "s_mov_b32 s49, 0x100\n\t"                                                                    \
    "v_mov_b32 v107, %[pay]\n\t"                                                                  \
    "v_mov_b32 v108, %[nb]\n\t"                                                                   \
    "v_mov_b32 v109, %[nbase]\n\t"                                                                \
    "v_mov_b32 v110, %[lane]\n\t"                                                                 \
    "v_mov_b32 v111, -1\n\t"                                                                      \
    "s_cmp_eq_u32 s59, 0\n\t"                                                                     \
    "s_mov_b32 s59, 0\n\t" /* (no SCC write) */                                                  \
    "s_cbranch_scc0 mcsfa_resume_%=\n\t" MCS_FA_INIT##W MCS_FA_RELOAD##W                         \
    "v_mov_b32 v94, %[c0]\n\t"                                                                    \
    "v_mov_b32 v95, %[c1]\n\t"                                                                    \
    "v_mov_b32 v96, %[c2]\n\t"                                                                    \
    "v_mov_b32 v97, %[c3]\n\t"                                                                    \
    "s_waitcnt lgkmcnt(0)\n\t"                                                                    \
    "s_min_u32 s41, s42, 64\n\t"                                                                  \
    "s_branch mcsfa_start_%=\n"                                                                   \
    "mcsfa_resume_%=:\n\t" MCS_FA_TAKE##W                                                        \
    "s_sub_u32 s41, s42, s57\n\t"                                                                 \
    "s_min_u32 s41, s41, 64\n\t"                                                                  \
    "s_mov_b32 s47, 0\n"                                                                          \
    "mcsfa_start_%=:\n\t" MCS_FA_REC##W                                                          \
    "s_cmp_lt_u32 s47, s41\n\t"                                                                   \
    "s_cbranch_scc0 mcsfa_bend_%=\n"
// (r05: no vmcnt wait at the exit: the batch's three result stores just issued complete while the
// generator synthesises the next batch; the compiler's code issues no store, and any wait it takes
// on its own loads only waits longer for the older stores, which complete in issue order.  The LDS
// operations of a release are waited for: the generator uses the wave's LDS scratch.)
#define MCS_FA_EXIT_F                                                                             \
    "mcsfa_exit_%=:\n\t"                                                                          \
    "s_waitcnt lgkmcnt(0)\n\t"                                                                    \
    "s_cmp_eq_u32 s47, 0\n\t" /* (as MCS_FA_EXIT_S) */                                           \
    "s_cbranch_scc1 mcsfa_xf_%=\n\t"                                                              \
    "v_add_u32 v93, v92, v95\n"                                                                   \
    "mcsfa_xf_%=:\n\t"                                                                            \
    "s_nop 1"
#define MCS_FA_LOOP_F(W, D) MCS_FA_ENTRY_F(W) MCS_FA_BODY(W, D, F) MCS_FA_EXIT_F

// The end of a run, shared by the loop kernels: the batch holding the last decision (earlier ones
// are stored in the loop), the undecided rows after a deadlock or a clock overflow, and the
// cluster's statistics.  A peak above the pool means a skipped insert: the engine re-runs the
// cluster with a larger pool.
template <int NPL, int P>
__device__ __forceinline__ void fa_finish(const FifoArgs& a, uint32_t ci, uint32_t lane, uint32_t J, uint32_t t,
                                          uint32_t r, uint32_t flags, uint32_t waited, uint32_t peak,
                                          uint32_t n_slow, uint32_t n_rel, uint32_t on, uint32_t os, uint32_t of,
                                          int32_t* o_node, uint32_t* o_start, uint32_t* o_finish) {
    if (peak > (uint32_t)(P * kWave)) flags |= MCS_FLAG_OVERFLOW;
    const uint32_t placed = r;  // FIFO places every job it decides, in order
    if (!(flags & MCS_FLAG_OVERFLOW)) {
        if (r > 0u) {  // the batch holding the last decision (earlier ones are stored)
            const uint32_t i = ((r - 1u) & ~63u) + lane;
            if (i < r) {
                o_node[i] = (int32_t)(NPL == 1 ? on : (on & 63u) * NPL + (on >> 6));
                o_start[i] = os;
                o_finish[i] = of;
            }
        }
        if (flags & (MCS_FLAG_DEADLOCK | MCS_FLAG_CLOCK_OVERFLOW)) {
            for (uint32_t i = r + lane; i < J; i += kWave) {
                o_node[i] = MCS_NODE_UNPLACED;
                o_start[i] = MCS_TIME_NONE;
                o_finish[i] = MCS_TIME_NONE;
            }
        }
    }

    if (lane == 0) {
        mcs_cluster_stats st;
        st.t_end = t;
        st.placed = placed;
        st.waited = waited;
        st.peak_running = peak;
        st.flags = flags;
        st.pool = (uint32_t)P;
        st.iterations = n_slow + r;  // passes: one per decision, plus the clock advances
        st.release_scans = n_rel;
        a.cstats[ci] = st;
        if (flags & MCS_FLAG_OVERFLOW) {
            atomicAdd(&a.totals->overflowed, 1u);
        } else {
            atomicAdd(&a.totals->placed, (unsigned long long)placed);
            atomicAdd(&a.totals->waited, (unsigned long long)waited);
            atomicAdd(&a.totals->unplaced, (unsigned long long)(J - placed));
            if (flags & MCS_FLAG_DEADLOCK) atomicAdd(&a.totals->deadlocked, 1u);
            if (flags & MCS_FLAG_CLOCK_OVERFLOW) atomicAdd(&a.totals->clock_overflowed, 1u);
        }
    }
}

// Node format W (32 or 16 bits per field); LDS: nodes [4][64] (u64 / u32 words) at 0, slot
// payloads [8][64] (u64 / u32 in a u64 stride) at 2048, slot {node address | finish << 32}
// [8][64] at 6144 (the offsets in the asm)
// (RS: the W16R form, running slots in registers; the LDS slot arrays are then unused)
// (NPL nodes per lane, P slot rows: 4/8 for 129-256 node clusters, 1/2 for at most 64 nodes)
// (DIAG: count the passes without a decision and the release scans into mcs_cluster_stats; the
// production launches skip them, 1.6 % of the C4 loop)
// (LOOK: the W16L lookahead loop, W16R's shape only)
template <int W, bool RS, int NPL, int P, bool DIAG, bool LOOK = false>
__global__ __launch_bounds__(64) void fifo_asm_kernel(FifoArgs a) {
    static_assert(W == 16 || !RS, "register slots: 16-bit node format only");
    static_assert(!LOOK || (W == 16 && RS && NPL == 4 && P == 8), "lookahead: the W16R shape");
    static_assert((NPL == 4 && P == 8) || (NPL == 1 && P == 2 && W == 16 && RS), "loop shapes");
    const uint32_t item = blockIdx.x;
    const uint32_t ci = a.cluster_list ? a.cluster_list[item] : item;
    const uint32_t lane = threadIdx.x;

    __shared__ uint64_t lds[NPL * kWave + 2 * P * kWave];
    uint64_t* const pay_nf = lds + NPL * kWave + P * kWave;

    constexpr uint32_t kGuard = W == 32 ? 0x80000000u : 0x8000u;
    constexpr uint32_t kClamp = kGuard - 1u;  // request clamp and padding value
    const uint32_t n0 = a.node_off[ci];
    const uint32_t N = a.node_off[ci + 1] - n0;
#pragma unroll
    for (int c = 0; c < NPL; ++c) {
        const uint32_t node = lane * NPL + c;
        uint2 v = make_uint2(kClamp, kClamp);  // padding: never fits
        if (node < N) {
            v = a.node_free0[n0 + node];
            v.x += kGuard;
            v.y += kGuard;
        }
        if constexpr (W == 32)
            lds[c * kWave + lane] = (uint64_t)v.x | ((uint64_t)v.y << 32);
        else
            reinterpret_cast<uint32_t*>(lds)[c * kWave + lane] = v.x | (v.y << 16);
    }
    if constexpr (!RS) {
#pragma unroll
        for (int p = 0; p < P; ++p) pay_nf[p * kWave + lane] = (uint64_t)kEmpty << 32;
    }

    const uint64_t j0 = a.job_off[ci];
    const uint32_t J = (uint32_t)(a.job_off[ci + 1] - j0);
    const uint4* jobs = a.jobs + j0;
    int32_t* o_node = a.out_node + j0;
    uint32_t* o_start = a.out_start + j0;
    uint32_t* o_finish = a.out_finish + j0;

    uint4 cur = jobs[lane];  // batch 0 (the array has kJobPad records of slack)
    cur.z = cur.z < kClamp ? cur.z : kClamp;
    cur.w = cur.w < kClamp ? cur.w : kClamp;
    if constexpr (W == 16) cur.z |= cur.w << 16;
    __syncthreads();  // (one wave: orders the LDS initialisation before the node reads in the asm)

    const uint32_t base = lds_addr(lds);
    const uint32_t v_pay = base + 2048u + lane * 8u;
    const uint32_t v_nb = base + lane * (W / 4u);
    const uint32_t v_nbase = base;
    // perm selectors: W32 gathers chunk pairs 0/1 and 2/3, W16 all four chunks at once
    const uint32_t sel0 = W == 32 ? 0x0c0c0b09u : NPL == 1 ? 0x7fffu : 0x0b0a0908u;
    const uint32_t sel1 = W == 32 ? 0x0b090c0cu : base;  // (W16R: the node array's LDS base)

    uint32_t t = 0, r = 0, flags = 0, have_w = 0;
    // free slot rows of the lane (W16 forms: plus the sentinel bit 8, so the lowest free row of a
    // full lane reads as 8, a register index still in range)
    uint32_t frm = (1u << P) - 1u + (W == 16 ? 0x100u : 0u), lmin = kEmpty;
    uint32_t used = 0, peak = 0, waited = 0, n_slow = 0, n_rel = 0;
    uint32_t on = 0, os = 0, of = 0;
#ifdef MCS_STAMPS
    uint32_t st0 = 0, st1 = 0, st2 = 0, st3 = 0;
#endif

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
#define MCS_FA_OPERANDS_IO                                                                        \
    : [t] "+s"(t), [r] "+s"(r), [flags] "+s"(flags), [hw] "+s"(have_w), [used] "+s"(used),      \
      [peak] "+s"(peak), [waited] "+s"(waited), [nslow] "+s"(n_slow), [nrel] "+s"(n_rel),       \
      [on] "+v"(on), [os] "+v"(os), [of] "+v"(of), [frm] "+v"(frm), [lmin] "+v"(lmin)            \
      MCS_FA_STAMP_OUTS                                                                           \
    : [J] "s"(J), [jobs] "s"(jobs), [onp] "s"(o_node), [osp] "s"(o_start), [ofp] "s"(o_finish), \
      [c0] "v"(cur.x), [c1] "v"(cur.y), [c2] "v"(cur.z), [c3] "v"(cur.w), [pay] "v"(v_pay),     \
      [nb] "v"(v_nb), [nbase] "v"(v_nbase), [lane] "v"(lane), [sel0] "s"(sel0),                 \
      [sel1] "s"(sel1), [fdl] "i"(MCS_FLAG_DEADLOCK), [fck] "i"(MCS_FLAG_CLOCK_OVERFLOW),        \
      [fov] "i"(MCS_FLAG_OVERFLOW)
#define MCS_FA_OPERANDS MCS_FA_OPERANDS_IO : MCS_FA_CLOBBERS
#define MCS_FL_OPERANDS MCS_FA_OPERANDS_IO : MCS_FL_CLOBBERS
    if constexpr (LOOK) {
#ifndef MCS_STAMPS
        if constexpr (DIAG) asm volatile(MCS_FL_LOOP(D1) MCS_FL_OPERANDS);
        else asm volatile(MCS_FL_LOOP(D0) MCS_FL_OPERANDS);
#endif
    } else if constexpr (W == 32)
        if constexpr (DIAG) asm volatile(MCS_FA_LOOP(32, D1) MCS_FA_OPERANDS);
        else asm volatile(MCS_FA_LOOP(32, D0) MCS_FA_OPERANDS);
    else if constexpr (NPL == 1)
        if constexpr (DIAG) asm volatile(MCS_FA_LOOP(16S, D1) MCS_FA_OPERANDS);
        else asm volatile(MCS_FA_LOOP(16S, D0) MCS_FA_OPERANDS);
    else if constexpr (RS)
        if constexpr (DIAG) asm volatile(MCS_FA_LOOP(16R, D1) MCS_FA_OPERANDS);
        else asm volatile(MCS_FA_LOOP(16R, D0) MCS_FA_OPERANDS);
    else
        if constexpr (DIAG) asm volatile(MCS_FA_LOOP(16, D1) MCS_FA_OPERANDS);
        else asm volatile(MCS_FA_LOOP(16, D0) MCS_FA_OPERANDS);
#undef MCS_FA_OPERANDS
#undef MCS_FL_OPERANDS
#undef MCS_FA_OPERANDS_IO
#pragma clang diagnostic pop

#ifdef MCS_STAMPS
    if (lane == 0) {
        atomicAdd(&g_fa_stamps[0], (unsigned long long)st0);
        atomicAdd(&g_fa_stamps[1], (unsigned long long)st1);
        atomicAdd(&g_fa_stamps[2], (unsigned long long)st2);
        atomicAdd(&g_fa_stamps[3], (unsigned long long)st3);
    }
#endif
    fa_finish<NPL, P>(a, ci, lane, J, t, r, flags, waited, peak, n_slow, n_rel, on, os, of, o_node, o_start, o_finish);
}

typedef uint32_t mcs_u32x8 __attribute__((ext_vector_type(8)));
typedef uint32_t mcs_u32x4 __attribute__((ext_vector_type(4)));

// The W16R / W16S loop on a fused job stream (MCS_FA_LOOP_F): the same decisions as
// fifo_asm_kernel, batch after batch from GenStream instead of HBM records.
template <int NPL, int P, bool DIAG>
__global__ __launch_bounds__(64) void fifo_asm_fused_kernel(FifoArgs a) {
    static_assert((NPL == 4 && P == 8) || (NPL == 1 && P == 2), "loop shapes");
    const uint32_t item = blockIdx.x;
    const uint32_t ci = a.cluster_list ? a.cluster_list[item] : item;
    const uint32_t lane = threadIdx.x;

    // LDS: the node words only (the register-slot loops keep no slot in LDS) and the generator's
    // scratch
    __shared__ uint32_t lds[NPL * kWave];
    __shared__ uint32_t gscr[kGenScratch];
    constexpr uint32_t kGuard = 0x8000u, kClamp = kGuard - 1u;
    const uint32_t n0 = a.node_off[ci];
    const uint32_t N = a.node_off[ci + 1] - n0;
#pragma unroll
    for (int c = 0; c < NPL; ++c) {
        const uint32_t node = lane * NPL + c;
        uint2 v = make_uint2(kClamp, kClamp);  // padding: never fits
        if (node < N) {
            v = a.node_free0[n0 + node];
            v.x += kGuard;
            v.y += kGuard;
        }
        lds[c * kWave + lane] = v.x | (v.y << 16);
    }

    const uint64_t j0 = a.job_off[ci];
    const uint32_t J = (uint32_t)(a.job_off[ci + 1] - j0);
    int32_t* o_node = a.out_node + j0;
    uint32_t* o_start = a.out_start + j0;
    uint32_t* o_finish = a.out_finish + j0;

    GenStream gs;
    gs.init(a.gen, ci, lane, gscr);
    uint4 cur = gs.next(0u, lane);  // batch 0
    cur.z = cur.z < kClamp ? cur.z : kClamp;
    cur.w = cur.w < kClamp ? cur.w : kClamp;
    cur.z |= cur.w << 16;
    __syncthreads();

    const uint32_t base = lds_addr(lds);
    const uint32_t v_pay = 0u;  // (no LDS slot rows)
    const uint32_t v_nb = base + lane * 4u;
    const uint32_t v_nbase = base;
    const uint32_t sel0 = NPL == 1 ? 0x7fffu : 0x0b0a0908u;
    const uint32_t sel1 = base;

    // the loop state, bound to its registers (MCS_FA_LOOP_F)
    uint32_t t = 0, have_w = 0, flags = 0, cursor = 0, cb = 0, need = 0, emin = kEmpty, fails = 0;
    uint32_t used = 0, peak = 0, waited = 0, n_slow = 0, n_rel = 0;
    uint32_t frm = (1u << P) - 1u + 0x100u, lmin = kEmpty, on = 0, os = 0, of = 0;
    mcs_u32x8 sf = kEmpty, sp = 0u, sa = 0u;  // slot rows: finish, payload, node address
    mcs_u32x4 nd = 0u;                        // node registers
    mcs_u32x4 nx = 0u;                        // the next batch's records

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
#define MCS_FF_OPERANDS                                                                           \
    : [t] "+{s40}"(t), [hw] "+{s43}"(have_w), [flags] "+{s44}"(flags), [cur] "+{s47}"(cursor),   \
      [cb] "+{s57}"(cb), [need] "+{s59}"(need), [emin] "+{s77}"(emin), [fails] "+{s78}"(fails),  \
      [used] "+{s80}"(used), [peak] "+{s81}"(peak), [waited] "+{s82}"(waited),                   \
      [nslow] "+{s83}"(n_slow), [nrel] "+{s84}"(n_rel), [sf] "+{v[32:39]}"(sf),                   \
      [sp] "+{v[40:47]}"(sp), [sa] "+{v[48:55]}"(sa), [nd] "+{v[64:67]}"(nd), [frm] "+{v89}"(frm), \
      [lmin] "+{v90}"(lmin), [on] "+{v91}"(on), [os] "+{v92}"(os), [of] "+{v93}"(of)             \
    : [nx] "{v[98:101]}"(nx), [J] "s"(J), [onp] "s"(o_node), [osp] "s"(o_start),                \
      [ofp] "s"(o_finish), [c0] "v"(cur.x), [c1] "v"(cur.y), [c2] "v"(cur.z), [c3] "v"(cur.w),   \
      [pay] "v"(v_pay), [nb] "v"(v_nb), [nbase] "v"(v_nbase), [lane] "v"(lane),                  \
      [sel0] "s"(sel0), [sel1] "s"(sel1), [fdl] "i"(MCS_FLAG_DEADLOCK),                         \
      [fck] "i"(MCS_FLAG_CLOCK_OVERFLOW), [fov] "i"(MCS_FLAG_OVERFLOW)                           \
    : MCS_FF_CLOBBERS
    for (;;) {
        if constexpr (NPL == 1)
            if constexpr (DIAG) asm volatile(MCS_FA_LOOP_F(16S, D1) MCS_FF_OPERANDS);
            else asm volatile(MCS_FA_LOOP_F(16S, D0) MCS_FF_OPERANDS);
        else
            if constexpr (DIAG) asm volatile(MCS_FA_LOOP_F(16R, D1) MCS_FF_OPERANDS);
            else asm volatile(MCS_FA_LOOP_F(16R, D0) MCS_FF_OPERANDS);
        if (!need) break;
        const uint4 b = gs.next(cb, lane);  // the next batch (bases increase)
        nx = mcs_u32x4{b.x, b.y, b.z, b.w};
    }
#undef MCS_FF_OPERANDS
#pragma clang diagnostic pop

    const uint32_t r = cb + cursor;
    peak = peak > used ? peak : used;
    fa_finish<NPL, P>(a, ci, lane, J, t, r, flags, waited, peak, n_slow, n_rel, on, os, of, o_node, o_start, o_finish);
}

// ---- the duo loop: a decision wave and a release wave per cluster (low occupancy) -----------------
// Under strong sharding a GPU holds few clusters (512 of C4's 4096 at N = 8: two waves per CU), so
// each cluster's decision chain runs alone on its SIMD and the release scans (8 slot rows, the
// payload adds, a node reload and a wave minimum: ~35 % of a lone wave's cycles) sit on that chain.
// Here a second wave of the workgroup, on an otherwise idle SIMD, holds the running slots and keeps
// the release of the next finish second ready as a packet (MCS_FH_LOOP); the decision wave
// (MCS_FA_LOOP(16D)) posts each commit to it and applies a packet with four packed adds.  Same
// decisions and results as W16R, bit for bit.
struct DuoLds {
    uint32_t ring[128][4];  // posts {kx, finish, payload, seq}
    uint32_t hdr[4];        // {e1, e2, posts taken, slots at e1 (bit 31: overflow)}
    uint32_t ack, done, pad[2];
    uint32_t delta[4 * kWave];  // the packet: released {cores | mem << 16} per node, [chunk][lane]
    uint32_t nodes[4 * kWave];  // the node words, read once by the decision wave
};

template <bool DIAG>
__global__ __launch_bounds__(2 * kWave) void fifo_duo_kernel(FifoArgs a) {
    const uint32_t item = blockIdx.x;
    const uint32_t ci = a.cluster_list ? a.cluster_list[item] : item;
    const uint32_t lane = threadIdx.x & (kWave - 1u), wave = threadIdx.x / kWave;
    __shared__ DuoLds L;

    constexpr uint32_t kGuard = 0x8000u, kClamp = kGuard - 1u;
    const uint32_t n0 = a.node_off[ci];
    const uint32_t N = a.node_off[ci + 1] - n0;
    const uint64_t j0 = a.job_off[ci];
    const uint32_t J = (uint32_t)(a.job_off[ci + 1] - j0);
    if (wave == 0) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const uint32_t node = lane * 4u + c;
            uint2 v = make_uint2(kClamp, kClamp);  // padding: never fits
            if (node < N) {
                v = a.node_free0[n0 + node];
                v.x += kGuard;
                v.y += kGuard;
            }
            L.nodes[c * kWave + lane] = v.x | (v.y << 16);
            L.delta[c * kWave + lane] = 0u;
        }
    } else {
        L.ring[lane][3] = kEmpty;  // (no post has this seq yet)
        L.ring[lane + kWave][3] = kEmpty;
        if (lane == 0) {
            L.hdr[0] = kEmpty;
            L.hdr[1] = kEmpty;
            L.hdr[2] = 0u;
            L.hdr[3] = 0u;
            L.ack = 0u;  // (finish seconds are >= 1)
            L.done = 0u;
        }
    }
    __syncthreads();
    const uint32_t rb = lds_addr(&L.ring[0][0]);
    const uint32_t hb = lds_addr(&L.hdr[0]);
    const uint32_t dl = lds_addr(&L.delta[0]) + lane * 4u;

    if (wave == 1) {
        // the release wave: polls until the decision wave is done (bounded: 64 polls per job)
        const uint64_t pb = 64ull * J + (1ull << 20);
        const uint32_t hbound = pb > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)pb;
        const uint32_t db = lds_addr(&L.delta[0]);
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
        asm volatile(MCS_FH_LOOP
                     :
                     : [hb] "s"(hbound), [db] "s"(db), [rb] "v"(rb), [dl] "v"(dl), [hdr] "v"(hb)
                     : MCS_FH_CLOBBERS);
#pragma clang diagnostic pop
        return;
    }

    const uint4* jobs = a.jobs + j0;
    int32_t* o_node = a.out_node + j0;
    uint32_t* o_start = a.out_start + j0;
    uint32_t* o_finish = a.out_finish + j0;
    uint4 cur = jobs[lane];  // batch 0 (the array has kJobPad records of slack)
    cur.z = cur.z < kClamp ? cur.z : kClamp;
    cur.w = cur.w < kClamp ? cur.w : kClamp;
    cur.z |= cur.w << 16;

    const uint32_t v_pay = 0u;  // (no LDS slot rows)
    const uint32_t v_nb = lds_addr(&L.nodes[0]) + lane * 4u;
    const uint32_t v_nbase = rb;  // (v109: the ring base)
    const uint32_t sel0 = 0x0b0a0908u, sel1 = 0u;

    uint32_t t = 0, r = 0, flags = 0, have_w = 0;
    uint32_t frm = 0u, lmin = kEmpty;
    uint32_t used = 0, peak = 0, waited = 0, n_slow = 0, n_rel = 0;
    uint32_t on = 0, os = 0, of = 0;
#ifdef MCS_STAMPS
    uint32_t st0 = 0, st1 = 0, st2 = 0, st3 = 0, spins = 0;
#define MCS_FD_STAMP_OUTS MCS_FA_STAMP_OUTS, [spins] "=s"(spins)
#define MCS_FD_SPINOUT "\n\ts_mov_b32 %[spins], s85"
#else
#define MCS_FD_STAMP_OUTS
#define MCS_FD_SPINOUT ""
#endif
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
    if constexpr (DIAG)
        asm volatile(MCS_FA_LOOP(16D, D1) MCS_FD_SPINOUT
                     : [t] "+s"(t), [r] "+s"(r), [flags] "+s"(flags), [hw] "+s"(have_w), [used] "+s"(used),
                       [peak] "+s"(peak), [waited] "+s"(waited), [nslow] "+s"(n_slow), [nrel] "+s"(n_rel),
                       [on] "+v"(on), [os] "+v"(os), [of] "+v"(of), [frm] "+v"(frm), [lmin] "+v"(lmin)
                       MCS_FD_STAMP_OUTS
                     : [J] "s"(J), [jobs] "s"(jobs), [onp] "s"(o_node), [osp] "s"(o_start), [ofp] "s"(o_finish),
                       [c0] "v"(cur.x), [c1] "v"(cur.y), [c2] "v"(cur.z), [c3] "v"(cur.w), [pay] "v"(v_pay),
                       [nb] "v"(v_nb), [nbase] "v"(v_nbase), [lane] "v"(lane), [sel0] "s"(sel0),
                       [sel1] "s"(sel1), [dl] "v"(dl), [hdr] "v"(hb), [fdl] "i"(MCS_FLAG_DEADLOCK),
                       [fck] "i"(MCS_FLAG_CLOCK_OVERFLOW), [fov] "i"(MCS_FLAG_OVERFLOW)
                     : MCS_FD_CLOBBERS);
    else
        asm volatile(MCS_FA_LOOP(16D, D0) MCS_FD_SPINOUT
                     : [t] "+s"(t), [r] "+s"(r), [flags] "+s"(flags), [hw] "+s"(have_w), [used] "+s"(used),
                       [peak] "+s"(peak), [waited] "+s"(waited), [nslow] "+s"(n_slow), [nrel] "+s"(n_rel),
                       [on] "+v"(on), [os] "+v"(os), [of] "+v"(of), [frm] "+v"(frm), [lmin] "+v"(lmin)
                       MCS_FD_STAMP_OUTS
                     : [J] "s"(J), [jobs] "s"(jobs), [onp] "s"(o_node), [osp] "s"(o_start), [ofp] "s"(o_finish),
                       [c0] "v"(cur.x), [c1] "v"(cur.y), [c2] "v"(cur.z), [c3] "v"(cur.w), [pay] "v"(v_pay),
                       [nb] "v"(v_nb), [nbase] "v"(v_nbase), [lane] "v"(lane), [sel0] "s"(sel0),
                       [sel1] "s"(sel1), [dl] "v"(dl), [hdr] "v"(hb), [fdl] "i"(MCS_FLAG_DEADLOCK),
                       [fck] "i"(MCS_FLAG_CLOCK_OVERFLOW), [fov] "i"(MCS_FLAG_OVERFLOW)
                     : MCS_FD_CLOBBERS);
#pragma clang diagnostic pop
    // the release wave stops polling
    if (lane == 0) __hip_atomic_store(&L.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#ifdef MCS_STAMPS
    if (lane == 0) {
        atomicAdd(&g_fa_stamps[0], (unsigned long long)st0);
        atomicAdd(&g_fa_stamps[1], (unsigned long long)st1);
        atomicAdd(&g_fa_stamps[2], (unsigned long long)st2);
        atomicAdd(&g_fa_stamps[3], (unsigned long long)st3);
        atomicAdd(&g_fa_stamps[4], (unsigned long long)spins);
    }
#endif
#undef MCS_FD_STAMP_OUTS
#undef MCS_FD_SPINOUT
    fa_finish<4, 8>(a, ci, lane, J, t, r, flags, waited, peak, n_slow, n_rel, on, os, of, o_node, o_start, o_finish);
}

}  // namespace

// Form codes: 22 = W16R's one-job lookahead loop (W16L), 21 = W16R's duo loop (a decision and a release wave per cluster, small grids),
// 17 = W16R and 18 = W16S (where the 16-bit format fits), 16 = W16 with LDS slots,
// 32 = W32, 19 / 20 = W16R / W16S on a fused job stream, 0 = the compiled kernel.  MCS_FIFO_ASM=0
// turns the hand-scheduled loop off, =16 / =32 force a form (A/B timing, the variant tests; neither
// has a small-cluster shape nor a fused one).
int fifo_asm_form(const FifoArgs& a, int npl, int pool, bool hor) {
    const char* env = getenv("MCS_FIFO_ASM");
    const int want = env ? atoi(env) : 1;
    // the loop's two shapes: 129-256 node clusters with 8 slot rows (C4) and at most 64 nodes with 2
    // rows (C1-C3); other shapes and pools keep the compiled kernel
    // (records and results are addressed by 32-bit offsets from the cluster's base: at most
    // kAsmMaxJobs jobs per cluster, guard_ok bit 2)
    if (want == 0 || hor || !(a.guard_ok & 4u)) return 0;
    // a fused job stream: the W16 register-slot shapes with GenStream at the batch ends
    if (a.gen.on) {
        if (want == 16 || want == 32 || !(a.guard_ok & 2u)) return 0;
        return npl == 1 && pool == 2 ? 20 : npl == 4 && pool == 8 ? 19 : 0;
    }
    if (npl == 1 && pool == 2) return (a.guard_ok & 2u) && want != 16 && want != 32 ? 18 : 0;
    if (npl != 4 || pool != 8) return 0;
    // register slots: one LDS round trip per release instead of 2 + rows; measured faster than LDS
    // slots at every occupancy from 1 to 16 cluster waves per CU
    if ((a.guard_ok & 2u) && want != 32) {
        if (want == 16) return 16;
        // small grids (a strong shard: at most 4 cluster waves per CU) run the duo loop, whose
        // release wave takes an otherwise idle SIMD; MCS_FIFO_DUO=0|1 forces either
        const char* duo = getenv("MCS_FIFO_DUO");
        const bool d = duo ? atoi(duo) != 0 : a.n_items <= kDuoMaxItems;
        if (d) return 21;
        // the one-job lookahead loop (W16L) for grids of at most kLookMaxItems clusters (one cluster
        // wave per SIMD and fewer); MCS_FIFO_LOOK=0|1 forces either
        const char* look = getenv("MCS_FIFO_LOOK");
        const bool l = look ? atoi(look) != 0 : a.n_items <= kLookMaxItems;
        return l ? 22 : 17;
    }
    return (a.guard_ok & 1u) ? 32 : 0;
}

bool fifo_asm_eligible(const FifoArgs& a, int npl, int pool, bool hor) {
    return fifo_asm_form(a, npl, pool, hor) != 0;
}

template <bool DIAG>
static hipError_t launch_form(const FifoArgs& a, int form, hipStream_t s) {
    switch (form) {
        case 20: hipLaunchKernelGGL((fifo_asm_fused_kernel<1, 2, DIAG>), dim3(a.n_items), dim3(kWave), 0, s, a); break;
        case 19: hipLaunchKernelGGL((fifo_asm_fused_kernel<4, 8, DIAG>), dim3(a.n_items), dim3(kWave), 0, s, a); break;
        case 18: hipLaunchKernelGGL((fifo_asm_kernel<16, true, 1, 2, DIAG>), dim3(a.n_items), dim3(kWave), 0, s, a); break;
        case 21: hipLaunchKernelGGL((fifo_duo_kernel<DIAG>), dim3(a.n_items), dim3(2 * kWave), 0, s, a); break;
        case 17: hipLaunchKernelGGL((fifo_asm_kernel<16, true, 4, 8, DIAG>), dim3(a.n_items), dim3(kWave), 0, s, a); break;
#ifndef MCS_STAMPS
        case 22: hipLaunchKernelGGL((fifo_asm_kernel<16, true, 4, 8, DIAG, true>), dim3(a.n_items), dim3(kWave), 0, s, a); break;
#endif
        case 16: hipLaunchKernelGGL((fifo_asm_kernel<16, false, 4, 8, DIAG>), dim3(a.n_items), dim3(kWave), 0, s, a); break;
        case 32: hipLaunchKernelGGL((fifo_asm_kernel<32, false, 4, 8, DIAG>), dim3(a.n_items), dim3(kWave), 0, s, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// MCS_FIFO_DIAG=1: the counting build (mcs_cluster_stats.iterations / release_scans); otherwise
// those two fields hold the decisions and 0
hipError_t launch_fifo_asm(const FifoArgs& a, int npl, int pool, hipStream_t s) {
    const int form = fifo_asm_form(a, npl, pool, false);
    const char* env = getenv("MCS_FIFO_DIAG");
    return env && atoi(env) != 0 ? launch_form<true>(a, form, s) : launch_form<false>(a, form, s);
}

}  // namespace mcs

#ifdef MCS_STAMPS
// the probe build's segment cycles (releases, failed fits, batch ends, whole loop), summed over the
// clusters of the launches since the last call; read and reset
extern "C" int mcs_debug_fa_stamps(unsigned long long* out) {
    unsigned long long z[5] = {0, 0, 0, 0, 0};
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(mcs::g_fa_stamps), sizeof(z)) != hipSuccess) return -1;
    return hipMemcpyToSymbol(HIP_SYMBOL(mcs::g_fa_stamps), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
