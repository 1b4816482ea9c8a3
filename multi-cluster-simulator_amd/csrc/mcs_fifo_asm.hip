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
#include "mcs_internal.h"
#include "mcs_lds.h"
#include "mcs_wave.h"

namespace mcs {

namespace {

#ifdef MCS_STAMPS
__device__ unsigned long long g_fa_stamps[4];
#endif

// Register map of the loop (all fixed; listed as clobbers).
//   s40 t     s41 min(64, J - cb)  s42 J   s43 have_w  s44 flags  s45 arr   s46 dur
//   s47 cursor's lane in the batch (r - cb)  s48 (W16: {cores|mem<<16}) / s[48:49] cores, mem
//   s50 fl   s51 byte mask of fl   s52 8 * chunk   s53 register index of the chunk
//   s[54:55] kx, finish   s56 next clock   s57 cb   s[60:61] lanes with a free row
//   s[62:63] one-lane exec masks   s[64:65] jobs  s[66:67] out_node  s[68:69] out_start
//   s[70:71] out_finish  s72/s73 perm selectors   s74 t + 1  s75 expired  s76 tmp
//   s77 the wave's earliest finish  s78/s79 failed fits / bound 4J + 256 (a runaway loop ends as a
//   pool overflow: the engine re-runs the cluster on the compiled kernel)   s80 used  s81 peak
//   s82 waited  s83 passes without a decision  s84 release scans  s85 insert lane
//   release: row expiry masks in s[50:55], s[60:63], s[86:91]
//   v[64:71] nodes (W32: pairs {C, M} per chunk; W16: v64-v67)   v[72:79] fit-test differences
//   v80-v86 fit bits / byte mask   (release: finish rows in v[72:87])
//   v89 free rows  v90 earliest finish  v91-92 result batch (kx, start; finish = start + dur at
//   the store)
//   v[94:97] records  v[98:101] next records   v107 slot column  v108 node column  v109 node base
//   v110 lane  v111 -1   v[112:113] payload  v[114:115] {node address, fin}  v117 slot address
//   v118 frm - 1  v120 DPP min / scan temp  v121 address  v[122:123] payload  v124 lane minimum
//   v125-v127 store temps
#define MCS_FA_CLOBBERS                                                                            \
    "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53",  \
        "s54", "s55", "s56", "s57", "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s65", "s66",     \
        "s67", "s68", "s69", "s70", "s71", "s72", "s73", "s74", "s75", "s76", "s77", "s78", "s79",     \
        "s80", "s81", "s82", "s83", "s84", "s85", "s86", "s87", "s88", "s89", "s90", "s91", "v32",     \
        "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45",     \
        "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v64",                   \
        "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77",     \
        "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v89", "v90", "v91",     \
        "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v107", "v108",        \
        "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v117", "v118", "v119", "v120",        \
        "v121", "v122", "v123", "v124", "v125", "v126", "v127", "vcc", "scc", "m0", "exec", "memory"     \
        MCS_FA_STAMP_CLOBBERS

// ---- W-specific pieces ----------------------------------------------------------------------
// the insert's candidate lanes: the lanes with a free slot row (computed early, off the chain)
#define MCS_FA_FREELANES "v_cmp_ne_u32_e64 s[60:61], 0, v89\n\t"
#define MCS_FA_FREELANES32 MCS_FA_FREELANES
#define MCS_FA_FREELANES16 ""
#define MCS_FA_FREELANES16R ""

// first fit (scheduler.go:129-137): byte c of v86 is 0xff where chunk c of the lane fits
#define MCS_FA_FIT32                                                                              \
    "v_subrev_u32 v72, s48, v64\n\t"                                                              \
    "v_subrev_u32 v73, s49, v65\n\t"                                                              \
    "v_subrev_u32 v74, s48, v66\n\t"                                                              \
    "v_subrev_u32 v75, s49, v67\n\t"                                                              \
    "v_subrev_u32 v76, s48, v68\n\t"                                                              \
    "v_subrev_u32 v77, s49, v69\n\t"                                                              \
    "v_subrev_u32 v78, s48, v70\n\t"                                                              \
    "v_subrev_u32 v79, s49, v71\n\t"                                                              \
    "v_and_b32 v80, v72, v73\n\t"                                                                 \
    "v_and_b32 v81, v74, v75\n\t"                                                                 \
    "v_and_b32 v82, v76, v77\n\t"                                                                 \
    "v_and_b32 v83, v78, v79\n\t"                                                                 \
    "v_perm_b32 v84, v81, v80, s72\n\t" /* bytes 0/1 = 0xff if chunk 0/1 fits */                  \
    "v_perm_b32 v85, v83, v82, s73\n\t" /* bytes 2/3 for chunks 2/3 */                            \
    "v_or_b32 v86, v84, v85\n\t"
#define MCS_FA_FIT16                                                                              \
    "v_pk_sub_u16 v72, v64, s48\n\t"                                                              \
    "v_pk_sub_u16 v73, v65, s48\n\t"                                                              \
    "v_pk_sub_u16 v74, v66, s48\n\t"                                                              \
    "v_pk_sub_u16 v75, v67, s48\n\t"                                                              \
    "v_and_b32_sdwa v80, v72, v72 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_0\n\t" \
    "v_and_b32_sdwa v81, v74, v74 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_0\n\t" \
    "v_and_b32_sdwa v80, v73, v73 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_0\n\t" \
    "v_and_b32_sdwa v81, v75, v75 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_0\n\t" \
    /* a VALU that reads a register right after an SDWA write preserving its other word sees  */  \
    /* the old word (measured: chunk 3 never fitted): the insert's free-row lanes and rows go */  \
    /* between the last SDWA write and the v_perm */                                              \
    "v_cmp_lt_u32_e64 s[60:61], s49, v89\n\t" /* (v89 = free rows | 0x100, s49 = 0x100) */      \
    "v_ffbl_b32 v117, v89\n\t" /* lowest free row; 8 (the sentinel) when none */               \
    "v_perm_b32 v86, v81, v80, s72\n\t" /* byte c = sign of chunk c's bit 15 / 31 */

// register index of the chunk (s52 = 8 * chunk) and the commit (cluster.go:146-147)
#define MCS_FA_COMMIT32                                                                           \
    "s_lshr_b32 s53, s52, 2\n\t"                                                                  \
    "s_lshl3_add_u32 s54, s52, s50\n\t" /* kx = chunk * 64 + fl */                                \
    "s_add_u32 s55, s40, s46\n\t"       /* finish */                                              \
    "s_set_gpr_idx_on s53, gpr_idx(SRC0,DST)\n\t"                                                 \
    "v_mov_b32 v64, v72\n\t"                                                                      \
    "v_mov_b32 v65, v73\n\t"                                                                      \
    "s_set_gpr_idx_off\n\t"
#define MCS_FA_COMMIT16                                                                           \
    "s_lshr_b32 s53, s52, 3\n\t"                                                                  \
    "s_lshl3_add_u32 s54, s52, s50\n\t"                                                           \
    "s_set_gpr_idx_on s53, gpr_idx(SRC0,DST)\n\t"                                                 \
    "v_mov_b32 v64, v72\n\t"                                                                      \
    "s_set_gpr_idx_off\n\t"

// slot insert (exec = the insert lane): payload, {node address, finish}, the LDS node commit
#define MCS_FA_INSERT32                                                                           \
    "v_mov_b64 v[112:113], s[48:49]\n\t"                                                          \
    "v_lshl_add_u32 v114, s54, 3, v109\n\t"                                                       \
    "v_mov_b32 v115, s55\n\t"                                                                     \
    "v_ffbl_b32 v117, v89\n\t"                                                                    \
    "v_lshl_add_u32 v117, v117, 9, v107\n\t"                                                      \
    "v_add_u32 v118, -1, v89\n\t"                                                                 \
    "ds_sub_u64 v114, v[112:113]\n\t"                                                             \
    "ds_write_b64 v117, v[112:113]\n\t"                                                           \
    "ds_write_b64 v117, v[114:115] offset:4096\n\t"                                               \
    "v_and_b32 v89, v118, v89\n\t"
#define MCS_FA_INSERT16                                                                           \
    "v_mov_b32 v112, s48\n\t"                                                                     \
    "v_lshl_add_u32 v114, s54, 2, v109\n\t"                                                       \
    "v_mov_b32 v115, s55\n\t"                                                                     \
    "v_lshl_add_u32 v117, v117, 9, v107\n\t" /* (v117 = the lane's lowest free row, FIT16) */    \
    "v_add_u32 v118, -1, v89\n\t"                                                                 \
    "ds_sub_u32 v114, v112\n\t"                                                                   \
    "ds_write_b32 v117, v112\n\t"                                                                 \
    "ds_write_b64 v117, v[114:115] offset:4096\n\t"                                               \
    "v_and_b32 v89, v118, v89\n\t"

// the record at the cursor (s47) to the scalar unit
#define MCS_FA_REC32                                                                              \
    "v_readlane_b32 s45, v94, s47\n\t"                                                            \
    "v_readlane_b32 s46, v95, s47\n\t"                                                            \
    "v_readlane_b32 s48, v96, s47\n\t"                                                            \
    "v_readlane_b32 s49, v97, s47\n\t"
#define MCS_FA_REC16                                                                              \
    "v_readlane_b32 s45, v94, s47\n\t"                                                            \
    "v_readlane_b32 s46, v95, s47\n\t"                                                            \
    "v_readlane_b32 s48, v96, s47\n\t"

// one release row p (cluster.go:153-157): expiry lane mask MASK, node address NODE
#define MCS_FA_ROW(W, p, NODE, MASK)                                                              \
    "s_cmp_lg_u64 " MASK ", 0\n\t"                                                                \
    "s_cbranch_scc0 mcsfa_r" #p "_%=\n\t"                                                         \
    "s_bcnt1_i32_b64 s76, " MASK "\n\t"                                                           \
    "s_mov_b64 exec, " MASK "\n\t" MCS_FA_PAYREAD##W(p) "s_add_u32 s75, s75, s76\n\t"            \
    "s_waitcnt lgkmcnt(0)\n\t" MCS_FA_PAYADD##W(NODE)                                             \
    "ds_write_b32 v107, v111 offset:4096+" #p "*512+4\n\t"                                        \
    "v_or_b32 v89, 1<<" #p ", v89\n\t"                                                            \
    "s_mov_b64 exec, -1\n"                                                                        \
    "mcsfa_r" #p "_%=:\n\t"
#define MCS_FA_PAYREAD32(p) "ds_read_b64 v[122:123], v107 offset:" #p "*512\n\t"
#define MCS_FA_PAYREAD16(p) "ds_read_b32 v122, v107 offset:" #p "*512\n\t"
#define MCS_FA_PAYADD32(NODE) "ds_add_u64 " NODE ", v[122:123]\n\t"
#define MCS_FA_PAYADD16(NODE) "ds_add_u32 " NODE ", v122\n\t"

#define MCS_FA_RELEASE(W)                                                                         \
    "ds_read_b64 v[72:73], v107 offset:4096+0*512\n\t"                                            \
    "ds_read_b64 v[74:75], v107 offset:4096+1*512\n\t"                                            \
    "ds_read_b64 v[76:77], v107 offset:4096+2*512\n\t"                                            \
    "ds_read_b64 v[78:79], v107 offset:4096+3*512\n\t"                                            \
    "ds_read_b64 v[80:81], v107 offset:4096+4*512\n\t"                                            \
    "ds_read_b64 v[82:83], v107 offset:4096+5*512\n\t"                                            \
    "ds_read_b64 v[84:85], v107 offset:4096+6*512\n\t"                                            \
    "ds_read_b64 v[86:87], v107 offset:4096+7*512\n\t"                                            \
    "s_not_b32 s76, s74\n\t"                                                                      \
    "v_mov_b32 v124, s76\n\t"                                                                     \
    "s_mov_b32 s75, 0\n\t"                                                                        \
    "s_waitcnt lgkmcnt(0)\n\t"                                                                    \
    "v_cmp_ge_u32_e64 s[50:51], s40, v73\n\t"                                                     \
    "v_cmp_ge_u32_e64 s[52:53], s40, v75\n\t"                                                     \
    "v_cmp_ge_u32_e64 s[54:55], s40, v77\n\t"                                                     \
    "v_cmp_ge_u32_e64 s[60:61], s40, v79\n\t"                                                     \
    "v_cmp_ge_u32_e64 s[62:63], s40, v81\n\t"                                                     \
    "v_cmp_ge_u32_e64 s[86:87], s40, v83\n\t"                                                     \
    "v_cmp_ge_u32_e64 s[88:89], s40, v85\n\t"                                                     \
    "v_cmp_ge_u32_e64 s[90:91], s40, v87\n\t"                                                     \
    /* earliest remaining finish: d = finish - (t + 1) wraps for expired rows */                  \
    "v_subrev_u32 v73, s74, v73\n\t"                                                              \
    "v_subrev_u32 v75, s74, v75\n\t"                                                              \
    "v_subrev_u32 v77, s74, v77\n\t"                                                              \
    "v_subrev_u32 v79, s74, v79\n\t"                                                              \
    "v_subrev_u32 v81, s74, v81\n\t"                                                              \
    "v_subrev_u32 v83, s74, v83\n\t"                                                              \
    "v_subrev_u32 v85, s74, v85\n\t"                                                              \
    "v_subrev_u32 v87, s74, v87\n\t"                                                              \
    "v_min3_u32 v124, v124, v73, v75\n\t"                                                         \
    "v_min3_u32 v120, v77, v79, v81\n\t"                                                          \
    "v_min3_u32 v124, v124, v83, v85\n\t"                                                         \
    "v_min3_u32 v124, v124, v87, v120\n\t"                                                        \
    MCS_FA_ROW(W, 0, "v72", "s[50:51]") MCS_FA_ROW(W, 1, "v74", "s[52:53]")                       \
    MCS_FA_ROW(W, 2, "v76", "s[54:55]") MCS_FA_ROW(W, 3, "v78", "s[60:61]")                       \
    MCS_FA_ROW(W, 4, "v80", "s[62:63]") MCS_FA_ROW(W, 5, "v82", "s[86:87]")                       \
    MCS_FA_ROW(W, 6, "v84", "s[88:89]") MCS_FA_ROW(W, 7, "v86", "s[90:91]")                       \
    "s_sub_u32 s80, s80, s75\n\t"

// the whole clock-advance release: rows, node reload issued, earliest remaining finish in v90
#define MCS_FA_SCAN32 MCS_FA_RELEASE(32) MCS_FA_RELOAD32 "v_add_u32 v90, s74, v124\n\t"
#define MCS_FA_SCAN16 MCS_FA_RELEASE(16) MCS_FA_RELOAD16 "v_add_u32 v90, s74, v124\n\t"

// ---- W16R: the 16-bit node format with the running slots in registers ----------------------------
// Slot row r of a lane is v(32+r) finish, v(40+r) payload {cores | mem << 16}, v(48+r) the node's
// LDS address: an insert is three indexed moves (row from v_ffbl of the insert lane's free rows,
// broadcast with one v_readlane), and a release reads no slot from LDS — its only round trip is
// the node reload, issued before the earliest-finish minimum that hides it.
#define MCS_FA_FIT16R MCS_FA_FIT16
#define MCS_FA_COMMIT16R MCS_FA_COMMIT16
#define MCS_FA_REC16R MCS_FA_REC16
#define MCS_FA_TAKE16R MCS_FA_TAKE16
#define MCS_FA_RELOAD16R MCS_FA_RELOAD16
#define MCS_FA_INIT32 ""
#define MCS_FA_INIT16 "s_mov_b32 s49, 0x100\n\t"
#define MCS_FA_INIT16R                                                                            \
    "s_mov_b32 s49, 0x100\n\t"                                                                   \
    "v_mov_b32 v32, -1\n\t"                                                                      \
    "v_mov_b32 v33, -1\n\t"                                                                      \
    "v_mov_b32 v34, -1\n\t"                                                                      \
    "v_mov_b32 v35, -1\n\t"                                                                      \
    "v_mov_b32 v36, -1\n\t"                                                                      \
    "v_mov_b32 v37, -1\n\t"                                                                      \
    "v_mov_b32 v38, -1\n\t"                                                                      \
    "v_mov_b32 v39, -1\n\t"
// (exec = the insert lane, or empty when the pool is full; s73 = the node array's LDS base)
#define MCS_FA_INSERT16R                                                                          \
    "v_readlane_b32 s86, v117, s85\n\t" /* 0-7, or 8 with exec empty: in range either way */   \
    "s_lshl2_add_u32 s87, s54, s73\n\t"                                                          \
    "s_lshl_b32 s76, 1, s86\n\t"                                                                 \
    "s_set_gpr_idx_on s86, gpr_idx(DST)\n\t"                                                     \
    "v_mov_b32 v32, s55\n\t"                                                                     \
    "v_mov_b32 v40, s48\n\t"                                                                     \
    "v_mov_b32 v48, s87\n\t"                                                                     \
    "s_set_gpr_idx_off\n\t"                                                                      \
    "v_xor_b32 v89, s76, v89\n\t" /* the row is taken */
// (exec = the row's expiry mask, SCC = any: no separate test, and exec is restored to the full
// wave once after the last row)
#define MCS_FR_ROW(p, MASK, F, P, A)                                                              \
    "s_and_b64 exec, " MASK ", -1\n\t"                                                           \
    "s_cbranch_scc0 mcsfa_r" #p "_%=\n\t"                                                        \
    "s_bcnt1_i32_b64 s76, " MASK "\n\t"                                                          \
    "ds_add_u32 " A ", " P "\n\t"                                                               \
    "v_mov_b32 " F ", -1\n\t"                                                                    \
    "s_add_u32 s75, s75, s76\n\t"                                                                \
    "v_or_b32 v89, 1<<" #p ", v89\n"                                                             \
    "mcsfa_r" #p "_%=:\n\t"
#define MCS_FA_SCAN16R                                                                            \
    /* the LDS node copy is refreshed from the registers first (commits do not touch it) */       \
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
    "s_mov_b64 exec, -1\n\t"                                                                     \
    "s_sub_u32 s80, s80, s75\n\t" MCS_FA_RELOAD16                                               \
    /* the lane's earliest remaining finish (released rows now hold -1) */                     \
    "v_min3_u32 v90, v32, v33, v34\n\t"                                                          \
    "v_min3_u32 v90, v90, v35, v36\n\t"                                                          \
    "v_min3_u32 v90, v90, v37, v38\n\t"                                                          \
    "v_min_u32 v90, v90, v39\n\t"

// node registers back from the LDS copy
#define MCS_FA_RELOAD32                                                                           \
    "ds_read_b64 v[64:65], v108 offset:0\n\t"                                                     \
    "ds_read_b64 v[66:67], v108 offset:512\n\t"                                                   \
    "ds_read_b64 v[68:69], v108 offset:1024\n\t"                                                  \
    "ds_read_b64 v[70:71], v108 offset:1536\n\t"
#define MCS_FA_RELOAD16                                                                           \
    "ds_read_b32 v64, v108 offset:0\n\t"                                                          \
    "ds_read_b32 v65, v108 offset:256\n\t"                                                        \
    "ds_read_b32 v66, v108 offset:512\n\t"                                                        \
    "ds_read_b32 v67, v108 offset:768\n\t"

// the next batch's records (prefetched in v[98:101]) become current, requests clamped
#define MCS_FA_TAKE32                                                                             \
    "v_mov_b32 v94, v98\n\t"                                                                      \
    "v_mov_b32 v95, v99\n\t"                                                                      \
    "v_min_u32 v96, 0x7fffffff, v100\n\t"                                                         \
    "v_min_u32 v97, 0x7fffffff, v101\n\t"
#define MCS_FA_TAKE16                                                                             \
    "v_mov_b32 v94, v98\n\t"                                                                      \
    "v_mov_b32 v95, v99\n\t"                                                                      \
    "v_min_u32 v96, 0x7fff, v100\n\t"                                                             \
    "v_min_u32 v97, 0x7fff, v101\n\t"                                                             \
    "v_lshl_or_b32 v96, v97, 16, v96\n\t"

// ---- per-form hooks of the loop -----------------------------------------------------------------
// a decided placement: the fitting lane's chunk, the commit under exec = that lane, then the
// running-slot insert under exec = the lowest lane with a free row (none: exec empty)
#define MCS_FA_DECIDE_(W)                                                                         \
    MCS_FA_PICK1##W MCS_FA_FREELANES##W                                                           \
    "s_lshl_b64 exec, 1, s50\n\t" MCS_FA_PICK2##W MCS_FA_COMMIT##W                                \
    "s_ff1_i32_b64 s85, s[60:61]\n\t"                                                             \
    "s_lshl_b64 s[62:63], 1, s85\n\t"                                                             \
    "s_and_b64 exec, s[62:63], s[60:61]\n\t" MCS_FA_INSERT##W
#define MCS_FA_DECIDE32 MCS_FA_DECIDE_(32)
#define MCS_FA_DECIDE16 MCS_FA_DECIDE_(16)
#define MCS_FA_DECIDE16S MCS_FA_DECIDE_(16S)
// W16R: ONE register-index region for both moves (the commit's chunk, then the insert's row by
// s_set_gpr_idx_idx); the insert lane and its row are found before it (VALU reads inside the
// region would be indexed), the row is taken after it
#define MCS_FA_DECIDE16R                                                                          \
    "v_readlane_b32 s51, v86, s50\n\t"                                                            \
    "s_ff1_i32_b64 s85, s[60:61]\n\t"                                                             \
    "s_lshl_b64 exec, 1, s50\n\t"                                                                 \
    "v_readlane_b32 s86, v117, s85\n\t" /* 0-7, or 8 with exec empty: in range either way */    \
    "s_ff1_i32_b32 s52, s51\n\t"                                                                  \
    "s_lshr_b32 s53, s52, 3\n\t"                                                                  \
    "s_lshl3_add_u32 s54, s52, s50\n\t"                                                           \
    "s_set_gpr_idx_on s53, gpr_idx(SRC0,DST)\n\t"                                                 \
    "v_mov_b32 v64, v72\n\t" /* the commit (cluster.go:146-147) */                                \
    "s_lshl_b64 s[62:63], 1, s85\n\t"                                                             \
    "s_and_b64 exec, s[62:63], s[60:61]\n\t"                                                      \
    "s_lshl2_add_u32 s87, s54, s73\n\t"                                                           \
    "s_set_gpr_idx_idx s86\n\t"                                                                   \
    "v_mov_b32 v32, s55\n\t" /* the slot: finish, payload, node address (SGPR sources) */        \
    "v_mov_b32 v40, s48\n\t"                                                                      \
    "v_mov_b32 v48, s87\n\t"                                                                      \
    "s_set_gpr_idx_off\n\t"                                                                       \
    "s_lshl_b32 s76, 1, s86\n\t"                                                                  \
    "v_xor_b32 v89, s76, v89\n\t" /* the row is taken */
// lanes with a fit into vcc
#define MCS_FA_ANYFIT "v_cmp_ne_u32_e32 vcc, 0, v86\n\t"
#define MCS_FA_ANYFIT32 MCS_FA_ANYFIT
#define MCS_FA_ANYFIT16 MCS_FA_ANYFIT
#define MCS_FA_ANYFIT16R MCS_FA_ANYFIT
// the fitting lane's byte mask (PICK1, a broadcast) and its lowest fitting chunk (PICK2)
#define MCS_FA_PICK1 "v_readlane_b32 s51, v86, s50\n\t"
#define MCS_FA_PICK2 "s_ff1_i32_b32 s52, s51\n\t" /* 8 * the lane's first fitting chunk */
#define MCS_FA_PICK132 MCS_FA_PICK1
#define MCS_FA_PICK116 MCS_FA_PICK1
#define MCS_FA_PICK116R MCS_FA_PICK1
#define MCS_FA_PICK232 MCS_FA_PICK2
#define MCS_FA_PICK216 MCS_FA_PICK2
#define MCS_FA_PICK216R MCS_FA_PICK2
// a zero-duration job's node (kx into s54; m0 = the cursor for the result writes)
#define MCS_FA_ZEROKX                                                                             \
    "v_readlane_b32 s51, v86, s50\n\t"                                                           \
    "s_mov_b32 m0, s47\n\t"                                                                      \
    "s_ff1_i32_b32 s52, s51\n\t"                                                                 \
    "s_lshl3_add_u32 s54, s52, s50\n\t"
#define MCS_FA_ZEROKX32 MCS_FA_ZEROKX
#define MCS_FA_ZEROKX16 MCS_FA_ZEROKX
#define MCS_FA_ZEROKX16R MCS_FA_ZEROKX
// slots of the pool (64 lanes x P rows)
#define MCS_FA_POOLMAX32 "64*8"
#define MCS_FA_POOLMAX16 "64*8"
#define MCS_FA_POOLMAX16R "64*8"
// the result batch's node index from kx = chunk * 64 + lane
#define MCS_FA_NODEIDX                                                                            \
    "v_and_b32 v126, 63, v91\n\t"                                                                \
    "v_lshrrev_b32 v127, 6, v91\n\t"                                                             \
    "v_lshl_add_u32 v126, v126, 2, v127\n\t" /* node = lane * 4 + chunk */
#define MCS_FA_NODEIDX32 MCS_FA_NODEIDX
#define MCS_FA_NODEIDX16 MCS_FA_NODEIDX
#define MCS_FA_NODEIDX16R MCS_FA_NODEIDX

// ---- W16S: W16R for clusters of at most 64 nodes (one chunk, node = lane) and 2 slot rows --------
// (cluster_small / cluster_big: C1-C3).  The fit bit is bit 15 of one SDWA AND; no chunk pick, and
// the commit is a plain move under exec = the fitting lane.  s72 = 0x7fff.
#define MCS_FA_FIT16S                                                                             \
    "v_pk_sub_u16 v72, v64, s48\n\t"                                                             \
    "v_and_b32_sdwa v80, v72, v72 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_0\n\t" \
    "v_cmp_lt_u32_e64 s[60:61], s49, v89\n\t"                                                    \
    "v_ffbl_b32 v117, v89\n\t"
#define MCS_FA_ANYFIT16S "v_cmp_lt_u32_e32 vcc, s72, v80\n\t"
#define MCS_FA_PICK116S ""
#define MCS_FA_PICK216S ""
#define MCS_FA_FREELANES16S ""
#define MCS_FA_COMMIT16S                                                                          \
    "s_mov_b32 s54, s50\n\t"                                                                     \
    "v_mov_b32 v64, v72\n\t"
#define MCS_FA_ZEROKX16S                                                                          \
    "s_mov_b32 m0, s47\n\t"                                                                      \
    "s_mov_b32 s54, s50\n\t"
#define MCS_FA_POOLMAX16S "64*2"
#define MCS_FA_NODEIDX16S "v_mov_b32 v126, v91\n\t"
#define MCS_FA_REC16S MCS_FA_REC16
#define MCS_FA_TAKE16S MCS_FA_TAKE16
#define MCS_FA_RELOAD16S "ds_read_b32 v64, v108 offset:0\n\t"
#define MCS_FA_INIT16S                                                                            \
    "s_mov_b32 s49, 0x100\n\t"                                                                   \
    "v_mov_b32 v32, -1\n\t"                                                                      \
    "v_mov_b32 v33, -1\n\t"
#define MCS_FA_INSERT16S MCS_FA_INSERT16R
#define MCS_FA_SCAN16S                                                                            \
    "ds_write_b32 v108, v64 offset:0\n\t"                                                        \
    "s_mov_b32 s75, 0\n\t"                                                                       \
    "v_cmp_ge_u32_e64 s[50:51], s40, v32\n\t"                                                    \
    "v_cmp_ge_u32_e64 s[52:53], s40, v33\n\t"                                                    \
    MCS_FR_ROW(0, "s[50:51]", "v32", "v40", "v48") MCS_FR_ROW(1, "s[52:53]", "v33", "v41", "v49")  \
    "s_mov_b64 exec, -1\n\t"                                                                     \
    "s_sub_u32 s80, s80, s75\n\t" MCS_FA_RELOAD16S                                              \
    "v_min_u32 v90, v32, v33\n\t"

// ---- MCS_STAMPS probe build (tools/stamp_fa.py): s_memtime cycles per loop segment ------------------
// s[92:93] segment start, s94 releases, s95 failed fits, s96 batch ends, s97 the whole loop; each
// stamp waits for its own SMEM read (lgkmcnt, which also drains LDS): read the shares, not the time
#ifdef MCS_STAMPS
#define MCS_FA_T0 "s_memtime s[92:93]\n\ts_waitcnt lgkmcnt(0)\n\t"
#define MCS_FA_T1(acc)                                                                            \
    "s_memtime s[98:99]\n\ts_waitcnt lgkmcnt(0)\n\ts_sub_u32 s98, s98, s92\n\ts_add_u32 " acc ", " acc \
    ", s98\n\t"
#define MCS_FA_TSTART MCS_FA_T0 "s_sub_u32 s97, 0, s92\n\ts_mov_b32 s94, 0\n\ts_mov_b32 s95, 0\n\ts_mov_b32 s96, 0\n\t"
#define MCS_FA_TEND                                                                               \
    "s_memtime s[98:99]\n\ts_waitcnt lgkmcnt(0)\n\ts_add_u32 s97, s97, s98\n\t"                  \
    "s_mov_b32 %[st0], s94\n\ts_mov_b32 %[st1], s95\n\ts_mov_b32 %[st2], s96\n\ts_mov_b32 %[st3], s97\n\t"
#define MCS_FA_STAMP_CLOBBERS , "s92", "s93", "s94", "s95", "s96", "s97", "s98", "s99"
#define MCS_FA_STAMP_OUTS , [st0] "=s"(st0), [st1] "=s"(st1), [st2] "=s"(st2), [st3] "=s"(st3)
#else
#define MCS_FA_T0 ""
#define MCS_FA_T1(acc) ""
#define MCS_FA_TSTART ""
#define MCS_FA_TEND ""
#define MCS_FA_STAMP_CLOBBERS
#define MCS_FA_STAMP_OUTS
#endif

// ---- the decision loop ------------------------------------------------------------------------
// diagnostic counters (passes without a decision, release scans): DIAG launches only
#define MCS_FA_CNTS_D1 "s_add_u32 s83, s83, 1\n\t"
#define MCS_FA_CNTR_D1 "s_add_u32 s84, s84, 1\n\t"
#define MCS_FA_CNTS_D0 ""
#define MCS_FA_CNTR_D0 ""
#define MCS_FA_LOOP(W, D)                                                                         \
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
    "s_cbranch_scc0 mcsfa_bend_%=\n"                                                              \
                                                                                                  \
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
    "s_branch mcsfa_hwadv_%=\n"                                                                   \
                                                                                                  \
    /* zero-duration job: committed and released before the next decision (D3) */               \
    "mcsfa_zero_%=:\n\t" MCS_FA_ZEROKX##W                                                        \
    "v_writelane_b32 v91, s54, m0\n\t"                                                            \
    "v_writelane_b32 v92, s40, m0\n\t"                                                            \
    "s_branch mcsfa_placed_%=\n"                                                                  \
                                                                                                  \
    /* (the clock moves by t + 1 here and on a failed fit: the carry is the u32 clock's overflow) */ \
    "mcsfa_hwadv_%=:\n\t"                                                                         \
    "s_mov_b32 s43, 0\n\t"                                                                        \
    "s_add_u32 s40, s40, 1\n\t"                                                                   \
    "s_cbranch_scc1 mcsfa_clkovf_%=\n\t"                                                          \
    "s_branch mcsfa_adv_%=\n"                                                                     \
                                                                                                  \
    /* no node fits: WaitQueue append (:264-268), sleep to the next completion (A.3) */          \
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
    MCS_FA_T1("s95") "s_branch mcsfa_adv_%=\n"                                                    \
                                                                                                  \
    "mcsfa_arrive_%=:\n\t"                                                                        \
    "s_mov_b32 s40, s45\n\t" /* (> t) */                                                         \
    MCS_FA_CNTS_##D "\n"                                                                          \
    /* the clock has advanced: releases at the new instant (A.2 step 1) */                       \
    "mcsfa_adv_%=:\n\t"                                                                           \
    "s_cmp_lt_u32 s40, s77\n\t" /* nothing finishes by t: no release */                          \
    "s_cbranch_scc1 mcsfa_loopend_%=\n\t"                                                         \
    /* release every running job with finish <= t (cluster.go:153-157) */                        \
    MCS_FA_CNTR_##D MCS_FA_T0                                                                     \
    "s_max_u32 s81, s81, s80\n\t" /* peak: used only grows between releases */                   \
    "s_add_u32 s74, s40, 1\n\t" MCS_FA_SCAN##W                                                   \
    /* the wave's earliest remaining finish (DPP minimum of v90) under the reload's latency */   \
    "v_mov_b32 v120, v90\n\t"                                                                     \
    "s_nop 1\n\t"                                                                                 \
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
    "s_waitcnt lgkmcnt(0)\n\t" MCS_FA_T1("s94")                                                   \
    "s_branch mcsfa_loopend_%=\n"                                                                 \
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
    "s_cbranch_scc1 mcsfa_poolovf_%=\n\t"                                                         \
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
    "s_add_u32 s57, s57, 64\n\t" MCS_FA_TAKE##W                                                   \
    "v_add_u32 v121, s57, v110\n\t"                                                               \
    "v_lshlrev_b32 v121, 4, v121\n\t"                                                             \
    "v_add_u32 v121, 0x400, v121\n\t"                                                             \
    "global_load_dwordx4 v[98:101], v121, s[64:65]\n\t"                                           \
    "s_sub_u32 s41, s42, s57\n\t"                                                                 \
    "s_min_u32 s41, s41, 64\n\t"                                                                  \
    "s_mov_b32 s47, 0\n\t" MCS_FA_REC##W MCS_FA_T1("s96")                                         \
    "s_branch mcsfa_inner_%=\n"                                                                   \
                                                                                                  \
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

// Node format W (32 or 16 bits per field); LDS: nodes [4][64] (u64 / u32 words) at 0, slot
// payloads [8][64] (u64 / u32 in a u64 stride) at 2048, slot {node address | finish << 32}
// [8][64] at 6144 (the offsets in the asm)
// (RS: the W16R form, running slots in registers; the LDS slot arrays are then unused)
// (NPL nodes per lane, P slot rows: 4/8 for 129-256 node clusters, 1/2 for at most 64 nodes)
// (DIAG: count the passes without a decision and the release scans into mcs_cluster_stats; the
// production launches skip them, 1.6 % of the C4 loop)
template <int W, bool RS, int NPL, int P, bool DIAG>
__global__ __launch_bounds__(64) void fifo_asm_kernel(FifoArgs a) {
    static_assert(W == 16 || !RS, "register slots: 16-bit node format only");
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
#define MCS_FA_OPERANDS                                                                           \
    : [t] "+s"(t), [r] "+s"(r), [flags] "+s"(flags), [hw] "+s"(have_w), [used] "+s"(used),      \
      [peak] "+s"(peak), [waited] "+s"(waited), [nslow] "+s"(n_slow), [nrel] "+s"(n_rel),       \
      [on] "+v"(on), [os] "+v"(os), [of] "+v"(of), [frm] "+v"(frm), [lmin] "+v"(lmin)            \
      MCS_FA_STAMP_OUTS                                                                           \
    : [J] "s"(J), [jobs] "s"(jobs), [onp] "s"(o_node), [osp] "s"(o_start), [ofp] "s"(o_finish), \
      [c0] "v"(cur.x), [c1] "v"(cur.y), [c2] "v"(cur.z), [c3] "v"(cur.w), [pay] "v"(v_pay),     \
      [nb] "v"(v_nb), [nbase] "v"(v_nbase), [lane] "v"(lane), [sel0] "s"(sel0),                 \
      [sel1] "s"(sel1), [fdl] "i"(MCS_FLAG_DEADLOCK), [fck] "i"(MCS_FLAG_CLOCK_OVERFLOW),        \
      [fov] "i"(MCS_FLAG_OVERFLOW)                                                              \
    : MCS_FA_CLOBBERS
    if constexpr (W == 32)
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
#pragma clang diagnostic pop

    if (peak > (uint32_t)(P * kWave)) flags |= MCS_FLAG_OVERFLOW;  // a skipped insert
#ifdef MCS_STAMPS
    if (lane == 0) {
        atomicAdd(&g_fa_stamps[0], (unsigned long long)st0);
        atomicAdd(&g_fa_stamps[1], (unsigned long long)st1);
        atomicAdd(&g_fa_stamps[2], (unsigned long long)st2);
        atomicAdd(&g_fa_stamps[3], (unsigned long long)st3);
    }
#endif
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

}  // namespace

// Form codes: 17 = W16R and 18 = W16S (where the 16-bit format fits), 16 = W16 with LDS slots,
// 32 = W32, 0 = the compiled kernel.  MCS_FIFO_ASM=0 turns the hand-scheduled loop off, =16 / =32
// force a form (A/B timing, the variant tests; neither has a small-cluster shape).
int fifo_asm_form(const FifoArgs& a, int npl, int pool, bool hor) {
    const char* env = getenv("MCS_FIFO_ASM");
    const int want = env ? atoi(env) : 1;
    // the loop's two shapes: 129-256 node clusters with 8 slot rows (C4) and at most 64 nodes with 2
    // rows (C1-C3); other shapes and pools keep the compiled kernel
    // (records and results are addressed by 32-bit offsets from the cluster's base: at most
    // kAsmMaxJobs jobs per cluster, guard_ok bit 2)
    if (want == 0 || hor || a.gen.on || !(a.guard_ok & 4u)) return 0;
    if (npl == 1 && pool == 2) return (a.guard_ok & 2u) && want != 16 && want != 32 ? 18 : 0;
    if (npl != 4 || pool != 8) return 0;
    // register slots: one LDS round trip per release instead of 2 + rows; measured faster than LDS
    // slots at every occupancy from 1 to 16 cluster waves per CU
    if ((a.guard_ok & 2u) && want != 32) return want == 16 ? 16 : 17;
    return (a.guard_ok & 1u) ? 32 : 0;
}

bool fifo_asm_eligible(const FifoArgs& a, int npl, int pool, bool hor) {
    return fifo_asm_form(a, npl, pool, hor) != 0;
}

template <bool DIAG>
static hipError_t launch_form(const FifoArgs& a, int form, hipStream_t s) {
    switch (form) {
        case 18: hipLaunchKernelGGL((fifo_asm_kernel<16, true, 1, 2, DIAG>), dim3(a.n_items), dim3(kWave), 0, s, a); break;
        case 17: hipLaunchKernelGGL((fifo_asm_kernel<16, true, 4, 8, DIAG>), dim3(a.n_items), dim3(kWave), 0, s, a); break;
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
    unsigned long long z[4] = {0, 0, 0, 0};
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(mcs::g_fa_stamps), sizeof(z)) != hipSuccess) return -1;
    return hipMemcpyToSymbol(HIP_SYMBOL(mcs::g_fa_stamps), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
