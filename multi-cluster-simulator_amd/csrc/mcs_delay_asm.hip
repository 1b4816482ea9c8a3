// mcs_delay_asm.hip — the DELAY policy's decision loop, hand-scheduled for gfx950.
//
// Scheduler.Delay (pkg/scheduler/scheduler.go:298-369, the reference's shipped default,
// scheduler.go:116) under SDELAY, one cluster of 129-256 nodes per wave64, on
// the W16R machinery of the FIFO loop (mcs_fa_macros.h): 16-bit node registers with guard bits,
// the first fit by v_pk_sub_u16 + SDWA + v_perm, the commit as one indexed move, the running slots
// in registers and the release with one LDS round trip.
//
// One Delay iteration at t:
//   * releases due at t (cluster.go:153-157, before anything else, D3);
//   * the Level1 pass (:302-329): every Level1 job in list order gets ScheduleJob; a placed job is
//     removed with append(Level1[:i], Level1[i+1:]...) and no i--, so the job sliding into slot i
//     is not examined this pass (D6, replicated);
//   * the Level0 head (:332-366): placed when it fits (ScheduleJob, :335); otherwise, once it has
//     waited MaxWaitTime (:353), it moves to the Level1 tail;
//   * time.Sleep(1 s) (:367): t + 1 after an iteration that placed or moved a job; an iteration
//     that changed nothing fast-forwards to the next release, the head's arrival or its MaxWaitTime
//     move (exact: the skipped iterations repeat the same failures).
//
// Level1 lives in the wave's LDS (r04), three SoA arrays of kL1Cap words: the request {cores |
// mem << 16} (clamped like the Level0 records), the job's row (bit 31: not examined since the D6
// skip) and its duration.  The loop has two modes with their own copies of the iteration code: mode
// 0 while Level1 is empty (the r03 loop, no pass), mode 1 while it is not.  A pass runs only when a
// node grew since the last one (a release) or a skipped job waits: every other Level1 job failed
// every node then, and nodes only shrank since.  It reads the list 64 entries per row and tests each
// row against the grown nodes alone (their current values, 3 VALU per node), gives each candidate
// the real first fit in list order, and compacts the row in place.
// The loop stops a cluster ("bail-out", kDelayBail; the engine re-runs it from t = 0 on the
// compiled delay_kernel) only when Level1 outgrows its LDS slice, when the clock leaves the u32
// range after a move, or when a runaway guard trips (more Level1 placements than jobs, or more
// failed fits than 8J + 256: a loop fault, re-run at the same pool and counted in handed_over;
// MCS_FLAG_OVERFLOW stays the real slot exhaustion, which escalates the pool).  A Level1 deadlock (nothing runs or arrives and Level1 fits no node) ends the
// cluster here, as delay_kernel does: its Level1 jobs are written unplaced.
// Same results bit for bit as delay_kernel and the oracle (tests/test_gpu_delay.py, every form).
#include "mcs_internal.h"
#include "mcs_lds.h"
#include "mcs_wave.h"

#ifdef MCS_STAMPS
#error "the DELAY loop uses s92-s101: no stamp build"
#endif

namespace mcs {

namespace {

#include "mcs_fa_macros.h"

// Level1 entries per wave in LDS (10 rows).  LDS words of a wave: the node copy [4][64], then the
// Level1 arrays cm / jw / dur [kL1Cap] each: 8704 B, so 16 cluster waves per CU (the C4 shape) take
// 136 KB of the CU's 160 KB.
constexpr uint32_t kL1Cap = 640;
constexpr uint32_t kLdsWords = 4 * kWave + 3 * kL1Cap;

// Which Level1 jobs can fit (r04).  Every job a pass leaves in Level1 failed ScheduleJob against
// every node, and a job moved in by the Level0 head failed against every node at its move; between
// passes nodes only shrink, except at releases.  So at the next pass a job can fit only a node that
// grew since the last pass ("G": some free field above the snapshot v105/v106/v116/v112 taken at
// the end of the last pass and lowered, field by field, to the nodes' values at every Level1 move,
// since the moved job was tested against those; tools/delay_g_model.py checks the rule against the
// oracle), and the exact test of a row is "fits some node of G" with G's current
// values — 3 VALU per row and per G node, no filter to build.  A job the pass skips (D6) was not
// tested: it carries bit 31 of its job-row word ("untested", s96 >> 1 of them) and is a candidate at
// the next pass whatever G holds.  More than 64 grown nodes: every job of the pass is a candidate.
// Each candidate gets the real first fit (FIT16) in list order; after a commit, node kx's new value
// replaces its G entry and the rest of the row is re-tested.
//
// Register map beyond mcs_fa_macros.h's (DELAY loop only):
//   s43 changed (this iteration placed or moved a job)   s46 (in a pass) |G|, 0xffff = every job
//   s[58:59] candidates of the row   s82 candidate lane / G cursor   s74/s75/s76 temps
//   s[88:89] live (then kept) lanes of the row   s[90:91] removed lanes of the row
//   s92 Level1 length   s93 write cursor   s94 row base   s95 the D6-skipped position
//   s96 bit 0: a release since the last pass; bits 1-31: untested Level1 jobs
//   s97 moved   s98 placed from Level1   s99 Level1 peak
//   s[100:101] sum over Level1 placements of t minus the moved jobs' arrivals
//   v56 cm  v57 job row (bit 31: untested)  v58 duration  v60-v62 temps  v63 row address
//   v88 Level1 lane address (row 0)  v102/v103 per-lane 64-bit sum of (start - arrival) of the
//   stored Level0 batches  v104 temp  v105/v106/v116/v112 the node snapshot (chunks 0-3)
//   v113 G's node values  v118 G's node indices (kx)  v123 temp   s56 MaxWaitTime
//
// probe counters of the counting build (MCS_FIFO_DIAG=1; printed by the engine with
// MCS_DELAY_PROBE=1): lane k of v119 counts event k (0 passes run, 1 passes skipped (nothing grew,
// nothing untested), 2 rows, 3 candidates, 4 candidates whose first fit failed, 5 G nodes, 6 D6
// skips, 7 compactions, 8 mode-1 iterations; 9-11 cycle sums, below)
#define MCS_FD_P_D0(k) ""
#define MCS_FD_P_D1(k) "s_mov_b64 exec, 1<<" #k "\n\tv_add_u32 v119, 1, v119\n\ts_mov_b64 exec, -1\n\t"
// cycle stamps of the counting build (s_memtime, low 32 bits of the delta, summed in v119 lanes
// 9 passes, 10 the whole loop, 11 releases): TS starts the pair R, TE(R, k) adds now - R to lane k
#define MCS_FD_TS_D0(R) ""
#define MCS_FD_TS_D1(R) "s_memtime s[" #R ":" #R "+1]\n\ts_waitcnt lgkmcnt(0)\n\t"
#define MCS_FD_TE_D0(R, k) ""
#define MCS_FD_TE_D1(R, k)                                                                        \
    "s_memtime s[38:39]\n\ts_waitcnt lgkmcnt(0)\n\ts_sub_u32 s38, s38, s" #R "\n\t"              \
    "s_mov_b64 exec, 1<<" #k "\n\tv_add_u32 v119, s38, v119\n\ts_mov_b64 exec, -1\n\t"
#define MCS_FD_PG_D0 ""
#define MCS_FD_PG_D1 "s_mov_b64 exec, 1<<5\n\tv_add_u32 v119, s46, v119\n\ts_mov_b64 exec, -1\n\t"
// (a skipped pass: straight to the Level0 head, or through its counter)
#define MCS_FD_PSK_D0 "mcsfd_head1_%="
#define MCS_FD_PSK_D1 "mcsfd_pskip_%="
#define MCS_FD_PSKB_D0 ""
#define MCS_FD_PSKB_D1 "s_branch mcsfd_head1_%=\nmcsfd_pskip_%=:\n\t" MCS_FD_P_D1(1)

// the grown nodes of chunk C (lane mask MASK, node registers V) into the G list (v113 values, v118
// kx) at cursor s82
#define MCS_FD_ENUM(C, MASK, V)                                                                   \
    "mcsfd_g" #C "_%=:\n\t"                                                                       \
    "s_ff1_i32_b64 s76, " MASK "\n\t"                                                             \
    "s_cmp_lt_i32 s76, 0\n\t"                                                                     \
    "s_cbranch_scc1 mcsfd_g" #C "e_%=\n\t"                                                        \
    "v_readlane_b32 s87, " V ", s76\n\t"                                                          \
    "s_bitset0_b64 " MASK ", s76\n\t"                                                             \
    "s_mov_b32 m0, s82\n\t"                                                                       \
    "s_add_u32 s86, s76, " #C "*64\n\t"                                                           \
    "v_writelane_b32 v113, s87, m0\n\t"                                                           \
    "v_writelane_b32 v118, s86, m0\n\t"                                                           \
    "s_add_u32 s82, s82, 1\n\t"                                                                   \
    "s_branch mcsfd_g" #C "_%=\n"                                                                 \
    "mcsfd_g" #C "e_%=:\n\t"

// G: nodes with a free field above the snapshot; |G| into s46 (0xffff past 64: every job)
#define MCS_FD_GROWN                                                                              \
    "v_pk_max_u16 v60, v64, v105\n\t"                                                             \
    "v_pk_max_u16 v61, v65, v106\n\t"                                                             \
    "v_pk_max_u16 v62, v66, v116\n\t"                                                             \
    "v_pk_max_u16 v123, v67, v112\n\t"                                                            \
    "v_cmp_ne_u32_e64 s[58:59], v60, v105\n\t"                                                    \
    "v_cmp_ne_u32_e64 s[88:89], v61, v106\n\t"                                                    \
    "v_cmp_ne_u32_e64 s[90:91], v62, v116\n\t"                                                    \
    "v_cmp_ne_u32_e64 s[74:75], v123, v112\n\t"                                                   \
    "s_bcnt1_i32_b64 s46, s[58:59]\n\t"                                                           \
    "s_bcnt1_i32_b64 s76, s[88:89]\n\t"                                                           \
    "s_add_u32 s46, s46, s76\n\t"                                                                 \
    "s_bcnt1_i32_b64 s76, s[90:91]\n\t"                                                           \
    "s_add_u32 s46, s46, s76\n\t"                                                                 \
    "s_bcnt1_i32_b64 s76, s[74:75]\n\t"                                                           \
    "s_add_u32 s46, s46, s76\n\t"                                                                 \
    "s_cmp_gt_u32 s46, 64\n\t"                                                                    \
    "s_cbranch_scc0 mcsfd_gl_%=\n\t"                                                              \
    "s_mov_b32 s46, 0xffff\n\t"                                                                   \
    "s_branch mcsfd_gdone_%=\n"                                                                   \
    "mcsfd_gl_%=:\n\t"                                                                            \
    "s_mov_b32 s82, 0\n\t" MCS_FD_ENUM(0, "s[58:59]", "v64") MCS_FD_ENUM(1, "s[88:89]", "v65")    \
    MCS_FD_ENUM(2, "s[90:91]", "v66") MCS_FD_ENUM(3, "s[74:75]", "v67")                           \
    "mcsfd_gdone_%=:\n\t"

// the row's jobs that fit some node of G (current values) or are untested, into ACC (an SGPR
// pair, zeroed here); IX is the G cursor (clobbered), s74 a temp; T names the labels
#define MCS_FD_GTEST(ACC, T, IX)                                                                  \
    "s_mov_b64 " ACC ", 0\n\t"                                                                    \
    "s_cmp_eq_u32 s46, 0xffff\n\t"                                                                \
    "s_cbranch_scc1 mcsfd_" T "all_%=\n\t"                                                        \
    "s_mov_b32 " IX ", 0\n\t"                                                                     \
    "s_cmp_eq_u32 s46, 0\n\t"                                                                     \
    "s_cbranch_scc1 mcsfd_" T "u_%=\n"                                                            \
    "mcsfd_" T "_%=:\n\t"                                                                         \
    "v_readlane_b32 s74, v113, " IX "\n\t"                                                        \
    "s_add_u32 " IX ", " IX ", 1\n\t"                                                             \
    "v_pk_sub_u16 v60, s74, v56\n\t" /* guard bits survive in both halves iff the job fits */    \
    "v_and_b32 v60, 0x80008000, v60\n\t"                                                          \
    "v_cmp_eq_u32_e32 vcc, 0x80008000, v60\n\t"                                                   \
    "s_or_b64 " ACC ", " ACC ", vcc\n\t"                                                          \
    "s_cmp_lt_u32 " IX ", s46\n\t"                                                                \
    "s_cbranch_scc1 mcsfd_" T "_%=\n"                                                             \
    "mcsfd_" T "u_%=:\n\t"                                                                        \
    "s_cmp_lt_u32 s96, 2\n\t"                                                                     \
    "s_cbranch_scc1 mcsfd_" T "e_%=\n\t"                                                          \
    "v_cmp_le_u32_e32 vcc, 0x80000000, v57\n\t" /* untested */                                  \
    "s_or_b64 " ACC ", " ACC ", vcc\n\t"                                                          \
    "s_branch mcsfd_" T "e_%=\n"                                                                  \
    "mcsfd_" T "all_%=:\n\t"                                                                      \
    "s_mov_b64 " ACC ", -1\n"                                                                     \
    "mcsfd_" T "e_%=:\n\t"

// a Level0 batch's results (the lanes placed on Level0; moved jobs are written when Level1 places
// them) and their waits; v91 = -1 marks a lane without a Level0 placement.  Result stores are plain
// (write-back): a row line stays in L2 while Level1 placements fill its holes; as nt stores every
// partial line went to HBM (127.8 -> 51.4 B/placement on the Level1-heavy stream, with the job
// records loaded nt so the stream does not evict them; profiles/r04_pmc_head, r04_pmc_plainnt)
#define MCS_FD_STORE                                                                              \
    "v_cmp_ne_u32_e32 vcc, -1, v91\n\t"                                                          \
    "s_mov_b64 exec, vcc\n\t"                                                                     \
    "v_add_u32 v125, s57, v110\n\t"                                                               \
    "v_lshlrev_b32 v125, 2, v125\n\t" MCS_FA_NODEIDX                                              \
    "global_store_dword v125, v126, s[66:67]\n\t"                                              \
    "global_store_dword v125, v92, s[68:69]\n\t"                                               \
    "v_add_u32 v93, v92, v95\n\t" /* finish = start + the batch's duration column */            \
    "global_store_dword v125, v93, s[70:71]\n\t"                                               \
    "v_sub_u32 v104, v92, v94\n\t" /* start - arrival */                                         \
    "v_add_co_u32 v102, vcc, v102, v104\n\t"                                                      \
    "v_addc_co_u32 v103, vcc, 0, v103, vcc\n\t"                                                   \
    "s_mov_b64 exec, -1\n\t"                                                                      \
    "v_mov_b32 v91, -1\n\t"

// the Level0 head (scheduler.go:332-366) of mode M: first fit; a placement commits (HD: the filter
// is dirty in mode 1), then the cursor moves (the decision is final) and the clock ticks
#define MCS_FD_HEAD(M, HD)                                                                        \
    "s_cmp_gt_u32 s45, s40\n\t" /* Level0 empty at t: the head has not arrived */                 \
    "s_cbranch_scc1 mcsfd_idle" #M "_%=\n\t" MCS_FA_FIT16 MCS_FA_ANYFIT                           \
    "s_add_u32 s55, s40, s46\n\t"                                                                 \
    "s_cbranch_vccz mcsfd_nofit" #M "_%=\n\t"                                                     \
    "s_ff1_i32_b64 s50, vcc\n\t" /* lowest lane with a fit */                                     \
    "s_cmp_eq_u32 s46, 0\n\t"                                                                     \
    "s_cbranch_scc1 mcsfd_zero" #M "_%=\n\t" MCS_FA_DECIDE16R                                     \
    "s_min_u32 s77, s77, s55\n\t" /* the wave's earliest finish */                                \
    "s_mov_b64 exec, -1\n\t"                                                                      \
    "s_mov_b32 m0, s47\n\t"                                                                       \
    "s_add_u32 s80, s80, 1\n\t" HD                                                                \
    "v_writelane_b32 v91, s54, m0\n\t"                                                            \
    "v_writelane_b32 v92, s40, m0\n"                                                              \
    "mcsfd_placed" #M "_%=:\n\t"                                                                  \
    "s_add_u32 s47, s47, 1\n\t" MCS_FA_REC16                                                      \
    "s_cmp_lt_u32 s47, s41\n\t"                                                                   \
    "s_cbranch_scc0 mcsfd_bend_%=\n"                                                              \
    /* time.Sleep(1 s) after a change (:367) */                                                   \
    "mcsfd_tick" #M "_%=:\n\t"                                                                    \
    "s_add_u32 s40, s40, 1\n\t"                                                                   \
    "s_cbranch_scc1 mcsfd_clkovf_%=\n"                                                            \
    /* the clock has advanced: releases at the new instant (cluster.go:153-157) */              \
    "mcsfd_adv" #M "_%=:\n\t"                                                                     \
    "s_cmp_lt_u32 s40, s77\n\t"                                                                   \
    "s_cbranch_scc1 mcsfd_inner" #M "_%=\n\t"

// zero-duration job: committed and released before the next ScheduleJob (D3)
#define MCS_FD_ZERO(M)                                                                            \
    "mcsfd_zero" #M "_%=:\n\t" MCS_FA_ZEROKX                                                      \
    "v_writelane_b32 v91, s54, m0\n\t"                                                            \
    "v_writelane_b32 v92, s40, m0\n\t"                                                            \
    "s_branch mcsfd_placed" #M "_%=\n"

// the Level1 pass (scheduler.go:302-329), mode 1 only; falls through to the Level0 head
#define MCS_FD_PASS(D)                                                                            \
    "s_mov_b32 s43, 0\n\t"                                                                        \
    "s_cmp_eq_u32 s96, 0\n\t" /* nothing grew, nothing untested: every job fails again */         \
    "s_cbranch_scc1 " MCS_FD_PSK_##D "\n\t"                                                       \
    "s_mov_b32 s46, 0\n\t"                                                                        \
    "s_bitcmp0_b32 s96, 0\n\t"                                                                    \
    "s_cbranch_scc1 mcsfd_rows_%=\n\t"                                                            \
    "s_and_b32 s96, s96, -2\n\t" MCS_FD_GROWN                                                     \
    "s_cmp_eq_u32 s46, 0\n\t"                                                                     \
    "s_cbranch_scc0 mcsfd_rows_%=\n\t"                                                            \
    "s_cmp_eq_u32 s96, 0\n\t"                                                                     \
    "s_cbranch_scc0 mcsfd_rows_%=\n\t"                                                            \
    "v_readlane_b32 s46, v95, s47\n\t" /* nothing grew after all: the head's duration back */   \
    "s_branch " MCS_FD_PSK_##D "\n"                                                              \
    "mcsfd_rows_%=:\n\t" MCS_FD_P_##D(0) MCS_FD_PG_##D MCS_FD_TS_##D(36)                         \
    "s_mov_b32 s93, 0\n\t"                                                                        \
    "s_mov_b32 s94, 0\n\t"                                                                        \
    "s_mov_b32 s95, -1\n"                                                                         \
    "mcsfd_row_%=:\n\t" MCS_FD_P_##D(2)                                                           \
    "s_lshl_b32 s74, s94, 2\n\t"                                                                  \
    "v_add_u32 v63, s74, v88\n\t"                                                                 \
    "ds_read_b32 v56, v63\n\t"                                                                    \
    "ds_read_b32 v57, v63 offset:%[cap4]\n\t"                                                     \
    "ds_read_b32 v58, v63 offset:%[cap8]\n\t"                                                     \
    "s_sub_u32 s74, s92, s94\n\t"                                                                 \
    "v_cmp_gt_u32_e64 s[88:89], s74, v110\n\t" /* live: the row's entries */                    \
    "s_mov_b64 s[90:91], 0\n\t"                                                                   \
    "s_waitcnt lgkmcnt(0)\n\t" MCS_FD_GTEST("s[58:59]", "rt", "s82")                                     \
    "s_and_b64 s[58:59], s[58:59], s[88:89]\n"                                                    \
    /* the candidates in list order */                                                            \
    "mcsfd_cand_%=:\n\t"                                                                          \
    "s_ff1_i32_b64 s82, s[58:59]\n\t"                                                             \
    "s_cmp_lt_i32 s82, 0\n\t"                                                                     \
    "s_cbranch_scc1 mcsfd_rowend_%=\n\t"                                                          \
    "v_readlane_b32 s48, v56, s82\n\t"                                                            \
    "v_readlane_b32 s75, v57, s82\n\t"                                                            \
    "s_bitset0_b64 s[58:59], s82\n\t"                                                             \
    "s_add_u32 s74, s94, s82\n\t"                                                                 \
    "s_cmp_eq_u32 s74, s95\n\t"                                                                   \
    "s_cbranch_scc1 mcsfd_d6_%=\n\t" MCS_FD_P_##D(3) MCS_FA_FIT16 MCS_FA_ANYFIT                   \
    "v_readlane_b32 s55, v58, s82\n\t"                                                            \
    "s_bitcmp1_b32 s75, 31\n\t"                                                                   \
    "s_cbranch_scc1 mcsfd_untested_%=\n"                                                          \
    "mcsfd_tested_%=:\n\t"                                                                        \
    "s_cbranch_vccz mcsfd_nofitc_%=\n\t" /* (an untested job that still fits no node) */         \
    "s_ff1_i32_b64 s50, vcc\n\t"                                                                  \
    "s_add_u32 s55, s55, s40\n\t" /* finish */                                                   \
    "s_cmp_eq_u32 s55, s40\n\t"                                                                   \
    "s_cbranch_scc1 mcsfd_l1zero_%=\n\t" MCS_FA_DECIDE16R                                         \
    "s_min_u32 s77, s77, s55\n\t"                                                                 \
    "s_mov_b64 exec, -1\n\t"                                                                      \
    "s_set_gpr_idx_on s53, gpr_idx(SRC0)\n\t"                                                     \
    "v_mov_b32 v123, v64\n\t" /* the committed chunk's new values */                             \
    "s_set_gpr_idx_off\n\t"                                                                       \
    "s_add_u32 s80, s80, 1\n\t"                                                                   \
    "s_cmp_eq_u32 s46, 0xffff\n\t"                                                                \
    "v_readlane_b32 s74, v123, s50\n\t" /* node kx's new value */                                \
    "s_cbranch_scc1 mcsfd_l1res_%=\n\t"                                                           \
    "v_cmp_eq_u32_e32 vcc, s54, v118\n\t" /* its G entry (if any) follows it */                \
    "v_mov_b32 v60, s74\n\t"                                                                      \
    "v_cndmask_b32 v113, v113, v60, vcc\n\t" MCS_FD_GTEST("s[60:61]", "rr", "s76")                       \
    "s_and_b64 s[58:59], s[58:59], s[60:61]\n"                                                    \
    "mcsfd_l1res_%=:\n\t" /* the job's row: node, start, finish (kx in s54) */                  \
    "s_and_b32 s74, s54, 63\n\t"                                                                  \
    "s_lshr_b32 s76, s54, 6\n\t"                                                                  \
    "s_lshl2_add_u32 s74, s74, s76\n\t" /* node = lane * 4 + chunk */                            \
    "s_sub_u32 s76, s42, 1\n\t" /* (a row inside the cluster, whatever the list holds) */       \
    "s_min_u32 s75, s75, s76\n\t"                                                                 \
    "s_lshl_b32 s75, s75, 2\n\t"                                                                  \
    "s_mov_b64 exec, 1\n\t"                                                                       \
    "v_mov_b32 v125, s75\n\t"                                                                     \
    "v_mov_b32 v126, s74\n\t"                                                                     \
    "v_mov_b32 v127, s40\n\t"                                                                     \
    "v_mov_b32 v124, s55\n\t"                                                                     \
    "global_store_dword v125, v126, s[66:67]\n\t"                                              \
    "global_store_dword v125, v127, s[68:69]\n\t"                                              \
    "global_store_dword v125, v124, s[70:71]\n\t"                                              \
    "s_mov_b64 exec, -1\n\t"                                                                      \
    "s_bitset1_b64 s[90:91], s82\n\t"                                                             \
    "s_add_u32 s95, s94, s82\n\t"                                                                 \
    "s_add_u32 s95, s95, 1\n\t" /* the entry sliding into this slot is not examined (D6) */     \
    "s_add_u32 s98, s98, 1\n\t"                                                                   \
    "s_cmp_gt_u32 s98, s42\n\t" /* more Level1 placements than jobs: a runaway, re-run */       \
    "s_cbranch_scc1 mcsfd_bail_%=\n\t"                                                         \
    "s_add_u32 s100, s100, s40\n\t"                                                               \
    "s_addc_u32 s101, s101, 0\n\t"                                                                \
    "s_mov_b32 s43, 1\n\t"                                                                        \
    "s_branch mcsfd_cand_%=\n"                                                                    \
    /* an untested job is tested now: the mark goes (in LDS too, the row may stay in place) */   \
    "mcsfd_untested_%=:\n\t"                                                                      \
    "s_sub_u32 s96, s96, 2\n\t"                                                                   \
    "s_bitset0_b32 s75, 31\n\t"                                                                   \
    "s_lshl_b64 exec, 1, s82\n\t"                                                                 \
    "v_and_b32 v57, 0x7fffffff, v57\n\t"                                                          \
    "ds_write_b32 v63, v57 offset:%[cap4]\n\t"                                                    \
    "s_mov_b64 exec, -1\n\t"                                                                      \
    "s_branch mcsfd_tested_%=\n"                                                                  \
    "mcsfd_nofitc_%=:\n\t" MCS_FD_P_##D(4)                                                        \
    "s_branch mcsfd_cand_%=\n"                                                                    \
    "mcsfd_l1zero_%=:\n\t"                                                                        \
    "v_readlane_b32 s51, v86, s50\n\t"                                                            \
    "s_ff1_i32_b32 s52, s51\n\t"                                                                  \
    "s_lshl3_add_u32 s54, s52, s50\n\t"                                                           \
    "s_branch mcsfd_l1res_%=\n"                                                                   \
    /* D6-skipped: not examined this pass; untested until the next one */                        \
    "mcsfd_d6_%=:\n\t" MCS_FD_P_##D(6)                                                            \
    "s_bitcmp1_b32 s75, 31\n\t"                                                                   \
    "s_cbranch_scc1 mcsfd_cand_%=\n\t"                                                            \
    "s_add_u32 s96, s96, 2\n\t"                                                                   \
    "s_lshl_b64 exec, 1, s82\n\t"                                                                 \
    "v_or_b32 v57, 0x80000000, v57\n\t" /* (the row is compacted: the mark reaches LDS) */      \
    "s_mov_b64 exec, -1\n\t"                                                                      \
    "s_branch mcsfd_cand_%=\n"                                                                    \
    /* compaction in the same sweep: the kept entries move down to the write cursor */           \
    "mcsfd_rowend_%=:\n\t"                                                                        \
    "s_andn2_b64 s[88:89], s[88:89], s[90:91]\n\t"                                                \
    "s_cmp_lg_u64 s[90:91], 0\n\t"                                                                \
    "s_cbranch_scc1 mcsfd_cmp_%=\n\t"                                                             \
    "s_cmp_eq_u32 s93, s94\n\t"                                                                   \
    "s_cbranch_scc1 mcsfd_rown_%=\n"                                                              \
    "mcsfd_cmp_%=:\n\t" MCS_FD_P_##D(7)                                                           \
    "s_mov_b64 exec, s[88:89]\n\t"                                                                \
    "v_mbcnt_lo_u32_b32 v62, s88, 0\n\t"                                                          \
    "v_mbcnt_hi_u32_b32 v62, s89, v62\n\t" /* rank among the kept entries */                    \
    "s_sub_u32 s74, s93, s94\n\t"                                                                 \
    "s_lshl_b32 s74, s74, 2\n\t"                                                                  \
    "v_sub_u32 v62, v62, v110\n\t"                                                                \
    "v_lshl_add_u32 v62, v62, 2, v63\n\t"                                                         \
    "v_add_u32 v62, s74, v62\n\t" /* Level1 + 4 * (wr + rank) */                                  \
    "ds_write_b32 v62, v56\n\t"                                                                   \
    "ds_write_b32 v62, v57 offset:%[cap4]\n\t"                                                    \
    "ds_write_b32 v62, v58 offset:%[cap8]\n\t"                                                    \
    "s_mov_b64 exec, -1\n"                                                                        \
    "mcsfd_rown_%=:\n\t"                                                                          \
    "s_bcnt1_i32_b64 s74, s[88:89]\n\t"                                                           \
    "s_add_u32 s93, s93, s74\n\t"                                                                 \
    "s_add_u32 s94, s94, 64\n\t"                                                                  \
    "s_cmp_lt_u32 s94, s92\n\t"                                                                   \
    "s_cbranch_scc1 mcsfd_row_%=\n\t"                                                             \
    /* the pass is over: every job left fails every node (the untested aside) */                 \
    "s_mov_b32 s92, s93\n\t"                                                                      \
    "v_readlane_b32 s46, v95, s47\n\t" /* the Level0 head's record again */                     \
    "v_readlane_b32 s48, v96, s47\n\t"                                                            \
    "v_mov_b32 v105, v64\n\t" /* the snapshot G is measured from at the next pass */             \
    "v_mov_b32 v106, v65\n\t"                                                                     \
    "v_mov_b32 v116, v66\n\t"                                                                     \
    "v_mov_b32 v112, v67\n\t" MCS_FD_TE_##D(36, 9) MCS_FD_PSKB_##D

#define MCS_FD_LOOP(D)                                                                            \
    /* ---- entry: state into the fixed registers ---- */                                        \
    "s_mov_b32 s40, 0\n\t"                                                                        \
    "s_mov_b32 s42, %[J]\n\t"                                                                     \
    "s_mov_b32 s44, 0\n\t"                                                                        \
    "s_mov_b32 s47, 0\n\t"                                                                        \
    "s_mov_b32 s56, %[mw]\n\t"                                                                    \
    "s_mov_b32 s57, 0\n\t"                                                                        \
    "s_mov_b32 s78, 0\n\t"                                                                        \
    "s_lshl3_add_u32 s79, s42, 0x100\n\t" /* failed fits bound (a runaway loop: re-run) */       \
    "s_mov_b32 s80, 0\n\t"                                                                        \
    "s_mov_b32 s81, 0\n\t"                                                                        \
    "s_mov_b32 s83, 0\n\t"                                                                        \
    "s_mov_b32 s84, 0\n\t"                                                                        \
    "s_mov_b32 s92, 0\n\t"                                                                        \
    "s_mov_b32 s96, 0\n\t"                                                                        \
    "s_mov_b32 s97, 0\n\t"                                                                        \
    "s_mov_b32 s98, 0\n\t"                                                                        \
    "s_mov_b32 s99, 0\n\t"                                                                        \
    "s_mov_b64 s[100:101], 0\n\t"                                                                 \
    "s_mov_b32 s77, -1\n\t" /* nothing running */                                                \
    "s_mov_b64 s[64:65], %[jobs]\n\t"                                                             \
    "s_mov_b64 s[66:67], %[onp]\n\t"                                                              \
    "s_mov_b64 s[68:69], %[osp]\n\t"                                                              \
    "s_mov_b64 s[70:71], %[ofp]\n\t"                                                              \
    "s_mov_b32 s72, %[sel0]\n\t"                                                                  \
    "s_mov_b32 s73, %[sel1]\n\t"                                                                  \
    "v_mov_b32 v89, 0x1ff\n\t" /* 8 free rows + the sentinel bit */                              \
    "v_mov_b32 v94, %[c0]\n\t"                                                                    \
    "v_mov_b32 v95, %[c1]\n\t"                                                                    \
    "v_mov_b32 v96, %[c2]\n\t"                                                                    \
    "v_mov_b32 v97, %[c3]\n\t"                                                                    \
    "v_mov_b32 v108, %[nb]\n\t"                                                                   \
    "v_mov_b32 v110, %[lane]\n\t"                                                                 \
    "v_mov_b32 v102, 0\n\t"                                                                       \
    "v_mov_b32 v103, 0\n\t"                                                                       \
    "v_mov_b32 v91, -1\n\t"                                                                       \
    "v_mov_b32 v119, 0\n\t"                                                                       \
    "v_add_u32 v88, 0x400, v108\n\t" /* Level1 (after the node copy) */                          \
    MCS_FA_INIT16R MCS_FA_RELOAD16 "s_waitcnt lgkmcnt(0)\n\t" MCS_FD_TS_##D(34)                   \
    /* prefetch batch 1 */                                                                        \
    "v_lshlrev_b32 v121, 4, v110\n\t"                                                             \
    "v_add_u32 v121, 0x400, v121\n\t"                                                             \
    "global_load_dwordx4 v[98:101], v121, s[64:65] nt\n\t"                                           \
    "s_min_u32 s41, s42, 64\n\t" MCS_FA_REC16                                                     \
    "s_cmp_eq_u32 s42, 0\n\t" /* no jobs: no iteration (the clock stays at 0) */                 \
    "s_cbranch_scc1 mcsfd_exit_%=\n\t"                                                            \
    "s_branch mcsfd_inner0_%=\n"                                                                  \
                                                                                                  \
    /* ======== mode 0: Level1 empty ======== */                                                 \
    "mcsfd_inner0_%=:\n\t" MCS_FA_CNTS_##D MCS_FD_HEAD(0, "")                                     \
    /* releases: shared by both modes, back to the mode's iteration */                           \
    "mcsfd_rel_%=:\n\t" MCS_FA_CNTR_##D MCS_FD_TS_##D(36)                                         \
    "s_max_u32 s81, s81, s80\n\t" /* peak: used only grows between releases */                   \
    "s_add_u32 s74, s40, 1\n\t" MCS_FA_SCAN16R                                                    \
    "v_mov_b32 v120, v90\n\t"                                                                     \
    "s_or_b32 s96, s96, 1\n\t" /* a release grew nodes: G at the next pass */                   \
    "s_nop 0\n\t"                                                                                 \
    "v_min_u32_dpp v120, v120, v120 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"                     \
    "s_nop 1\n\t"                                                                                 \
    "v_min_u32_dpp v120, v120, v120 row_shr:2 row_mask:0xf bank_mask:0xf\n\t"                     \
    "s_nop 1\n\t"                                                                                 \
    "v_min_u32_dpp v120, v120, v120 row_shr:4 row_mask:0xf bank_mask:0xf\n\t"                     \
    "s_nop 1\n\t"                                                                                 \
    "v_min_u32_dpp v120, v120, v120 row_shr:8 row_mask:0xf bank_mask:0xf\n\t"                     \
    "s_nop 1\n\t"                                                                                 \
    "v_min_u32_dpp v120, v120, v120 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"                  \
    "s_nop 1\n\t"                                                                                 \
    "v_min_u32_dpp v120, v120, v120 row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"                  \
    "s_nop 1\n\t"                                                                                 \
    "v_readlane_b32 s77, v120, 63\n\t"                                                            \
    "s_waitcnt lgkmcnt(0)\n\t" MCS_FD_TE_##D(36, 11)                                              \
    "s_cmp_lg_u32 s92, 0\n\t"                                                                     \
    "s_cbranch_scc1 mcsfd_inner1_%=\n\t"                                                          \
    "s_branch mcsfd_inner0_%=\n" MCS_FA_RBODY16R MCS_FD_ZERO(0)                                   \
    /* nothing changes at t (Level0 empty): the next iteration that can differ is a release or  */ \
    /* the head's arrival */                                                                      \
    "mcsfd_idle0_%=:\n\t"                                                                         \
    "s_min_u32 s76, s77, s45\n\t"                                                                 \
    "s_add_u32 s40, s40, 1\n\t"                                                                   \
    "s_cbranch_scc1 mcsfd_clkovf_%=\n\t"                                                          \
    "s_max_u32 s40, s40, s76\n\t"                                                                 \
    "s_branch mcsfd_adv0_%=\n"                                                                    \
    /* the head does not fit: after MaxWaitTime it moves to Level1 (:353); before, the next */    \
    /* iteration that can differ is a release or the move */                                      \
    "mcsfd_nofit0_%=:\n\t"                                                                        \
    "s_sub_u32 s76, s40, s45\n\t" /* t - arrival (the head has arrived) */                       \
    "s_cmp_ge_u32 s76, s56\n\t"                                                                   \
    "s_cbranch_scc1 mcsfd_move0_%=\n\t"                                                           \
    "s_add_u32 s78, s78, 1\n\t"                                                                   \
    "s_cmp_gt_u32 s78, s79\n\t"                                                                   \
    "s_cbranch_scc1 mcsfd_bail_%=\n\t"                                                         \
    "s_add_u32 s76, s45, s56\n\t"                                                                 \
    "s_min_u32 s76, s76, s77\n\t"                                                                 \
    "s_add_u32 s40, s40, 1\n\t"                                                                   \
    "s_cbranch_scc1 mcsfd_clkovf_%=\n\t"                                                          \
    "s_max_u32 s40, s40, s76\n\t"                                                                 \
    "s_branch mcsfd_adv0_%=\n"                                                                    \
    "mcsfd_move0_%=:\n\t" /* into mode 1: the job fails every node as they are now */           \
    "s_mov_b32 s96, 0\n\t"                                                                        \
    "v_mov_b32 v105, v64\n\t"                                                                     \
    "v_mov_b32 v106, v65\n\t"                                                                     \
    "v_mov_b32 v116, v66\n\t"                                                                     \
    "v_mov_b32 v112, v67\n\t"                                                                     \
    "s_branch mcsfd_move1_%=\n"                                                                   \
                                                                                                  \
    /* ======== mode 1: Level1 holds jobs ======== */                                            \
    "mcsfd_inner1_%=:\n\t"                                                                        \
    "s_cmp_eq_u32 s92, 0\n\t"                                                                     \
    "s_cbranch_scc1 mcsfd_inner0_%=\n\t" MCS_FA_CNTS_##D MCS_FD_P_##D(8) MCS_FD_PASS(D)            \
    "mcsfd_head1_%=:\n\t" MCS_FD_HEAD(1, "")                                                      \
    "s_branch mcsfd_rel_%=\n" MCS_FD_ZERO(1)                                                      \
    "mcsfd_idle1_%=:\n\t"                                                                         \
    "s_cmp_eq_u32 s92, 0\n\t"                                                                     \
    "s_cbranch_scc0 mcsfd_idle1b_%=\n\t"                                                          \
    "s_cmp_eq_u32 s45, -1\n\t" /* Level0 and Level1 empty for good: the run ends */              \
    "s_cbranch_scc1 mcsfd_done_%=\n"                                                              \
    "mcsfd_idle1b_%=:\n\t"                                                                        \
    "s_cmp_lg_u32 s43, 0\n\t"                                                                     \
    "s_cbranch_scc1 mcsfd_tick1_%=\n\t"                                                           \
    "s_min_u32 s76, s77, s45\n\t"                                                                 \
    "s_cmp_eq_u32 s76, -1\n\t" /* nothing runs or arrives: Level1 never fits (deadlock) */       \
    "s_cbranch_scc1 mcsfd_dead_%=\n\t"                                                            \
    "s_add_u32 s40, s40, 1\n\t"                                                                   \
    "s_cbranch_scc1 mcsfd_clkovf_%=\n\t"                                                          \
    "s_max_u32 s40, s40, s76\n\t"                                                                 \
    "s_branch mcsfd_adv1_%=\n"                                                                    \
    "mcsfd_nofit1_%=:\n\t"                                                                        \
    "s_sub_u32 s76, s40, s45\n\t"                                                                 \
    "s_cmp_ge_u32 s76, s56\n\t"                                                                   \
    "s_cbranch_scc1 mcsfd_move1_%=\n\t"                                                           \
    "s_add_u32 s78, s78, 1\n\t"                                                                   \
    "s_cmp_gt_u32 s78, s79\n\t"                                                                   \
    "s_cbranch_scc1 mcsfd_bail_%=\n\t"                                                         \
    "s_cmp_lg_u32 s43, 0\n\t"                                                                     \
    "s_cbranch_scc1 mcsfd_tick1_%=\n\t"                                                           \
    "s_add_u32 s76, s45, s56\n\t"                                                                 \
    "s_min_u32 s76, s76, s77\n\t"                                                                 \
    "s_add_u32 s40, s40, 1\n\t"                                                                   \
    "s_cbranch_scc1 mcsfd_clkovf_%=\n\t"                                                          \
    "s_max_u32 s40, s40, s76\n\t"                                                                 \
    "s_branch mcsfd_adv1_%=\n"                                                                    \
    /* the head moves to the Level1 tail (:353-360); its JobsMap value is closed-form */         \
    "mcsfd_move1_%=:\n\t"                                                                         \
    "s_cmp_ge_u32 s92, %[cap]\n\t" /* Level1 outgrew its LDS slice: re-run on delay_kernel */    \
    "s_cbranch_scc1 mcsfd_bail_%=\n\t"                                                            \
    "s_lshl_b32 s74, s92, 2\n\t"                                                                  \
    "s_add_u32 s76, s57, s47\n\t" /* the job's row */                                            \
    "s_mov_b64 exec, 1\n\t"                                                                       \
    "v_add_u32 v62, s74, v88\n\t"                                                                 \
    "v_mov_b32 v114, s48\n\t"                                                                     \
    "v_mov_b32 v115, s76\n\t"                                                                     \
    "v_mov_b32 v123, s46\n\t"                                                                     \
    "ds_write_b32 v62, v114\n\t"                                                                  \
    "ds_write_b32 v62, v115 offset:%[cap4]\n\t"                                                   \
    "ds_write_b32 v62, v123 offset:%[cap8]\n\t"                                                   \
    "s_mov_b64 exec, -1\n\t"                                                                      \
    "v_pk_min_u16 v105, v105, v64\n\t" /* it failed every node as they are now: the snapshot */ \
    "v_pk_min_u16 v106, v106, v65\n\t" /* G is measured from may not exceed them */            \
    "v_pk_min_u16 v116, v116, v66\n\t"                                                            \
    "v_pk_min_u16 v112, v112, v67\n\t"                                                            \
    "s_add_u32 s92, s92, 1\n\t"                                                                   \
    "s_max_u32 s99, s99, s92\n\t"                                                                 \
    "s_add_u32 s97, s97, 1\n\t"                                                                   \
    "s_sub_u32 s100, s100, s45\n\t"                                                               \
    "s_subb_u32 s101, s101, 0\n\t"                                                                \
    "s_branch mcsfd_placed1_%=\n"                                                                 \
                                                                                                  \
    /* ---- batch end: store the Level0 results and their waits, take the prefetched records ---- */ \
    "mcsfd_bend_%=:\n\t"                                                                          \
    "s_max_u32 s81, s81, s80\n\t"                                                                 \
    "s_cmp_gt_u32 s81, 64*8\n\t"                                                                  \
    "s_cbranch_scc1 mcsfd_poolovf_%=\n\t"                                                         \
    "s_add_u32 s76, s57, s47\n\t"                                                                 \
    "s_cmp_ge_u32 s76, s42\n\t"                                                                   \
    "s_cbranch_scc1 mcsfd_last_%=\n\t"                                                            \
    "s_waitcnt vmcnt(0)\n\t" MCS_FD_STORE                                                         \
    "s_add_u32 s57, s57, 64\n\t" MCS_FA_PRIO("mcsfd_") MCS_FA_TAKE16                              \
    "v_add_u32 v121, s57, v110\n\t"                                                               \
    "v_lshlrev_b32 v121, 4, v121\n\t"                                                             \
    "v_add_u32 v121, 0x400, v121\n\t"                                                             \
    "global_load_dwordx4 v[98:101], v121, s[64:65] nt\n\t"                                           \
    "s_sub_u32 s41, s42, s57\n\t"                                                                 \
    "s_min_u32 s41, s41, 64\n\t"                                                                  \
    "s_mov_b32 s47, 0\n\t" MCS_FA_REC16                                                           \
    "s_cmp_lg_u32 s92, 0\n\t"                                                                     \
    "s_cbranch_scc1 mcsfd_tick1_%=\n\t"                                                           \
    "s_branch mcsfd_tick0_%=\n"                                                                   \
    /* every Level0 job decided: the run ends with this iteration's sleep, unless Level1 holds */ \
    /* jobs: then the last batch is stored and Level0 stays empty (no arrival: s45 = -1) */       \
    "mcsfd_last_%=:\n\t"                                                                          \
    "s_cmp_eq_u32 s92, 0\n\t"                                                                     \
    "s_cbranch_scc1 mcsfd_done_%=\n\t"                                                            \
    "s_waitcnt vmcnt(0)\n\t" MCS_FD_STORE                                                         \
    "s_mov_b32 s57, s76\n\t"                                                                      \
    "s_mov_b32 s47, 0\n\t"                                                                        \
    "s_mov_b32 s41, 0\n\t"                                                                        \
    "s_mov_b32 s45, -1\n\t"                                                                       \
    "s_branch mcsfd_tick1_%=\n"                                                                   \
    "mcsfd_done_%=:\n\t"                                                                          \
    "s_add_u32 s40, s40, 1\n\t"                                                                   \
    "s_branch mcsfd_exit_%=\n"                                                                    \
                                                                                                  \
    /* the Level1 jobs left are retried forever: their rows are written unplaced after the loop */ \
    "mcsfd_dead_%=:\n\t"                                                                          \
    "s_or_b32 s44, s44, %[fdl]\n\t"                                                              \
    "s_branch mcsfd_exit_%=\n"                                                                    \
    /* bail-out: the cluster is re-run on delay_kernel */                                          \
    "mcsfd_bail_%=:\n\t"                                                                          \
    "s_or_b32 s44, s44, %[fbail]\n\t"                                                             \
    "s_branch mcsfd_exit_%=\n"                                                                    \
    "mcsfd_clkovf_%=:\n\t"                                                                        \
    "s_cmp_eq_u32 s97, 0\n\t" /* jobs went through Level1: delay_kernel writes their rows */     \
    "s_cbranch_scc0 mcsfd_bail_%=\n\t"                                                            \
    "s_mov_b32 s40, -1\n\t" /* the clock stays at the last second it reached */                   \
    "s_or_b32 s44, s44, %[fck]\n\t"                                                               \
    "s_branch mcsfd_exit_%=\n"                                                                    \
    "mcsfd_poolovf_%=:\n\t"                                                                       \
    "s_or_b32 s44, s44, %[fov]\n\t"                                                               \
                                                                                                  \
    /* ---- exit: state back to the compiler's registers ---- */                                 \
    "mcsfd_exit_%=:\n\t" MCS_FD_TE_##D(34, 10)                                                  \
    "s_waitcnt vmcnt(0) lgkmcnt(0)\n\t"                                                           \
    "s_mov_b64 exec, 1\n\t" /* the Level1 waits join lane 0's sum */                            \
    "v_mov_b32 v104, s101\n\t"                                                                    \
    "v_add_co_u32 v102, vcc, s100, v102\n\t"                                                      \
    "v_addc_co_u32 v103, vcc, v104, v103, vcc\n\t"                                                \
    "s_mov_b64 exec, -1\n\t"                                                                      \
    "s_mov_b32 %[t], s40\n\t"                                                                     \
    "s_add_u32 %[r], s57, s47\n\t"                                                                \
    "s_mov_b32 %[cl], s47\n\t"                                                                    \
    "s_mov_b32 %[flags], s44\n\t"                                                                 \
    "s_mov_b32 %[used], s80\n\t"                                                                  \
    "s_max_u32 %[peak], s81, s80\n\t"                                                             \
    "s_mov_b32 %[nslow], s83\n\t"                                                                 \
    "s_mov_b32 %[nrel], s84\n\t"                                                                  \
    "s_mov_b32 %[moved], s97\n\t"                                                                 \
    "s_mov_b32 %[pl1], s98\n\t"                                                                   \
    "s_mov_b32 %[pk1], s99\n\t"                                                                   \
    "s_mov_b32 %[l1n], s92\n\t"                                                                   \
    "v_mov_b32 %[on], v91\n\t"                                                                    \
    "v_mov_b32 %[os], v92\n\t"                                                                    \
    "v_mov_b32 %[arr], v94\n\t"                                                                   \
    "v_mov_b32 %[wlo], v102\n\t"                                                                  \
    "v_mov_b32 %[whi], v103\n\t"                                                                  \
    "v_add_u32 %[of], v92, v95\n\t"                                                               \
    "v_mov_b32 %[prb], v119\n\t"                                                                  \
    "s_nop 1"

template <bool DIAG>
__global__ __launch_bounds__(64) void delay_asm_kernel(DelayArgs a) {
    const uint32_t item = blockIdx.x;
    const uint32_t ci = a.cluster_list ? a.cluster_list[item] : item;
    const uint32_t lane = threadIdx.x;

    // the node copy [4][64] (releases), Level1 cm / jw / dur
    __shared__ uint32_t lds[kLdsWords];
    constexpr uint32_t kGuard = 0x8000u, kClamp = kGuard - 1u;
    const uint32_t n0 = a.node_off[ci];
    const uint32_t N = a.node_off[ci + 1] - n0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const uint32_t node = lane * 4 + c;
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
    const uint4* jobs = a.jobs + j0;
    int32_t* o_node = a.out_node + j0;
    uint32_t* o_start = a.out_start + j0;
    uint32_t* o_finish = a.out_finish + j0;

    uint4 cur = jobs[lane];  // batch 0 (the array has kJobPad records of slack)
    cur.z = cur.z < kClamp ? cur.z : kClamp;
    cur.w = cur.w < kClamp ? cur.w : kClamp;
    cur.z |= cur.w << 16;
    __syncthreads();

    const uint32_t base = lds_addr(lds);
    const uint32_t v_nb = base + lane * 4u;
    const uint32_t sel0 = 0x0b0a0908u, sel1 = base;

    uint32_t t = 0, r = 0, cl = 0, flags = 0, used = 0, peak = 0, n_slow = 0, n_rel = 0;
    uint32_t moved = 0, pl1 = 0, pk1 = 0, l1n = 0;
    uint32_t on = 0, os = 0, of = 0, arr = 0, wlo = 0, whi = 0, prb = 0;

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
#define MCS_FD_OPERANDS                                                                           \
    : [t] "=s"(t), [r] "=s"(r), [cl] "=s"(cl), [flags] "=s"(flags), [used] "=s"(used),          \
      [peak] "=s"(peak), [nslow] "=s"(n_slow), [nrel] "=s"(n_rel), [moved] "=s"(moved),          \
      [pl1] "=s"(pl1), [pk1] "=s"(pk1), [l1n] "=s"(l1n), [on] "=v"(on), [os] "=v"(os), [of] "=v"(of),             \
      [arr] "=v"(arr), [wlo] "=v"(wlo), [whi] "=v"(whi), [prb] "=v"(prb)                         \
    : [J] "s"(J), [mw] "s"(a.max_wait_s), [jobs] "s"(jobs), [onp] "s"(o_node), [osp] "s"(o_start), \
      [ofp] "s"(o_finish), [c0] "v"(cur.x), [c1] "v"(cur.y), [c2] "v"(cur.z), [c3] "v"(cur.w),    \
      [nb] "v"(v_nb), [lane] "v"(lane), [sel0] "s"(sel0), [sel1] "s"(sel1),                      \
      [fck] "i"(MCS_FLAG_CLOCK_OVERFLOW), [fov] "i"(MCS_FLAG_OVERFLOW), [fbail] "i"(kDelayBail),  \
      [fdl] "i"(MCS_FLAG_DEADLOCK),                                                             \
      [cap] "i"(kL1Cap), [cap4] "i"(kL1Cap * 4), [cap8] "i"(kL1Cap * 8)                          \
    : MCS_FA_CLOBBERS, "s92", "s93", "s94", "s95", "s96", "s97", "s98", "s99", "s100", "s101",    \
      "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v88", "v102", "v103", "v104",     \
      "v105", "v106", "v116", "v119", "s34", "s35", "s36", "s37", "s38", "s39"
    if constexpr (DIAG) asm volatile(MCS_FD_LOOP(D1) MCS_FD_OPERANDS);
    else asm volatile(MCS_FD_LOOP(D0) MCS_FD_OPERANDS);
#undef MCS_FD_OPERANDS
#pragma clang diagnostic pop

    // the Level1 layout above: Level1 at +1 KB (v88 in the loop)
    static_assert(4 * kWave * 4 == 0x400, "LDS layout: Level1 after the node copy (v88)");

    // the counting build's probe counters: into the cluster's (otherwise unused) HBM Level1 scratch
    if (DIAG && lane < 12u && 2u * J > lane) reinterpret_cast<uint32_t*>(a.l1_cm + j0)[lane] = prb;
    // a pool overflow inside Level1's last stretch (no batch end to catch it): re-run
    if (peak > 64u * 8u) flags |= MCS_FLAG_OVERFLOW;
    const bool bail = (flags & kDelayBail) != 0u;
    // WaitTime.TotalTime / 1000 (scheduler.go:309-312,338-341): the stored Level0 batches (per
    // lane), the current batch's Level0 placements (not stored yet) and, in lane 0, the Level1
    // placements' t minus the moved jobs' arrivals
    const bool mine = lane < cl && on != 0xFFFFFFFFu;
    uint64_t w = (uint64_t)wlo | ((uint64_t)whi << 32);
    if (mine) w += (uint64_t)(os - arr);
    for (int o = 32; o >= 1; o >>= 1) {
        const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)w, o);
        const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(w >> 32), o);
        w += (uint64_t)lo | ((uint64_t)hi << 32);
    }
    const uint32_t placed = r - moved + pl1;
    // a deadlock (every Level0 job decided, nothing running, Level1 fits no node): the jobs left in
    // Level1 hold 1000 * (t - arrival) in JobsMap (their arrivals are already subtracted)
    const uint32_t left = (flags & MCS_FLAG_DEADLOCK) ? l1n : 0u;
    if (lane == 0u) w += (uint64_t)left * t;

    if (!(flags & MCS_FLAG_OVERFLOW)) {
        if (mine) {  // the current batch's Level0 placements (earlier batches are stored)
            const uint32_t i = r - cl + lane;
            o_node[i] = (int32_t)((on & 63u) * 4u + (on >> 6));
            o_start[i] = os;
            o_finish[i] = of;
        }
        for (uint32_t i = lane; i < left; i += kWave) {  // never placed (scheduler.go:302-329 spins)
            const uint32_t jw = lds[4 * kWave + kL1Cap + i] & 0x7FFFFFFFu;  // (bit 31: untested)
            o_node[jw] = MCS_NODE_UNPLACED;
            o_start[jw] = MCS_TIME_NONE;
            o_finish[jw] = MCS_TIME_NONE;
        }
        if (!bail && (flags & MCS_FLAG_CLOCK_OVERFLOW)) {  // (no job went through Level1)
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
        st.waited = moved;
        st.peak_running = peak;
        st.flags = flags;  // (kBail: the engine re-runs the cluster, which rewrites these)
        st.pool = 8u;
        st.iterations = DIAG ? n_slow : r;
        st.release_scans = n_rel;
        a.cstats[ci] = st;
        if (flags & MCS_FLAG_OVERFLOW) {
            atomicAdd(&a.totals->overflowed, 1u);
        } else if (bail) {
            atomicAdd(&a.totals->bailed, 1u);
        } else {
            mcs_delay_cluster_stats ds;
            ds.total_wait_ms = (int64_t)(w * 1000ull);
            ds.jobs_count = (flags & MCS_FLAG_CLOCK_OVERFLOW) ? -1 : (int64_t)J;
            ds.moved_l1 = moved;
            ds.placed_l1 = pl1;
            ds.peak_l1 = pk1;
            ds.l1_left = left;
            a.dstats[ci] = ds;
            atomicAdd(&a.totals->placed, (unsigned long long)placed);
            atomicAdd(&a.totals->waited, (unsigned long long)moved);
            atomicAdd(&a.totals->unplaced, (unsigned long long)(J - placed));
            if (flags & MCS_FLAG_DEADLOCK) atomicAdd(&a.totals->deadlocked, 1u);
            if (flags & MCS_FLAG_CLOCK_OVERFLOW) atomicAdd(&a.totals->clock_overflowed, 1u);
        }
    }
}

}  // namespace

// The DELAY loop's one shape: clusters of 129-256 nodes (NPL 4) with 8 slot rows, the 16-bit node
// format, records in HBM, at most kAsmMaxJobs jobs per cluster (FifoArgs::guard_ok's rules);
// MCS_DELAY_ASM=0 keeps the compiled delay_kernel.
bool delay_asm_eligible(int npl, int pool, uint32_t guard_ok, bool gen_on) {
    const char* env = getenv("MCS_DELAY_ASM");
    if (env && atoi(env) == 0) return false;
    return npl == 4 && pool == 8 && (guard_ok & 2u) && (guard_ok & 4u) && !gen_on;
}

hipError_t launch_delay_asm(const DelayArgs& a, hipStream_t s) {
    if (a.n_items == 0) return hipSuccess;
    const char* env = getenv("MCS_FIFO_DIAG");
    if (env && atoi(env) != 0)
        hipLaunchKernelGGL((delay_asm_kernel<true>), dim3(a.n_items), dim3(kWave), 0, s, a);
    else
        hipLaunchKernelGGL((delay_asm_kernel<false>), dim3(a.n_items), dim3(kWave), 0, s, a);
    return hipGetLastError();
}

}  // namespace mcs
