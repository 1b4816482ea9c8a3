// mcs_fa_macros.h — the hand-scheduled gfx950 pieces shared by the FIFO decision loop
// (mcs_fifo_asm.hip) and the DELAY loop (mcs_delay_asm.hip): the fixed register map, the node
// formats' fit tests, commits, slot inserts, releases and record handling.  Included by .hip files
// only (inline-asm text).
#pragma once

// ---- gfx950 hazard audit of the hand-scheduled loops (FIFO W16R/W16S/fused, duo, DELAY) -----------
// LLVM's hazard recognizer does not look inside inline asm, so every producer -> consumer pair the
// hardware does not interlock is covered here by instruction distance or an explicit s_nop.  A
// "wait state" is one issued instruction of this wave (s_nop N = N + 1 of them).
//
//  hazard (CDNA3/gfx950)                           needs  where it occurs                     covered by
//  VALU writes VGPR -> DPP reads it                  2     every DPP min/max chain (SCANEND,   s_nop 1 between the steps; before
//                                                          the DELAY filter, the duo e2 scan)  the first: s_nop 1, or (DELAY rel)
//                                                                                              s_mov s96 + s_nop 0
//  SDWA / op_sel write preserving the other word     1     MCS_FA_FIT16: v80/v81 (WORD_1,      v_cmp_lt s[60:61] + v_ffbl v117
//    -> VALU reads that VGPR (DstSelForwarding)            UNUSED_PRESERVE) -> v_perm          between (found by measurement,
//                                                                                              tools/asm_debug.py); FIT16D: s_nop 1
//  VALU writes SGPR -> v_readlane / v_writelane      4     none: every lane select is SALU-    (s50/s85/s82 from s_ff1, s47/m0
//    uses it as the lane select                            written                             from s_add/s_mov)
//  SALU writes M0 -> v_writelane with an M0 lane     1*    result writes at a Level0 decision  >= 1 other instruction between
//    select (*not in the ISA table; kept anyway)           (HEAD, ZEROKX)                      (s_add s80 / s_ff1, s_lshl3_add)
//                                                          DELAY G list (MCS_FD_ENUM: m0 =     s_add s86 between
//                                                          cursor -> v_writelane v113/v118)
//  VALU writes VGPR -> v_readlane / v_readfirstlane  1     DECIDE16R / ZEROKX read v86, v117;  >= 3 instructions between every
//    reads it (gfx950)                                     REC16 after TAKE16; SCANEND v120     pair; SCANEND: s_nop 1
//                                                          DELAY G pass (r04): v_cndmask v113  >= 6 (GTEST's scalar prologue)
//                                                          -> GTEST's v_readlane v113; v123
//                                                          (indexed move) -> v_readlane s74     >= 3 (s_set_gpr_idx_off, s_add,
//                                                                                              s_cmp)
//  VALU writes VCC -> s_cbranch_vccz/vccnz           0     ANYFIT -> the fit branch             (interlocked on gfx9; SALU
//                                                                                              instructions between anyway)
//  VALU writes EXEC -> DPP (5) / v_readlane (4)      5/4   none: exec is written by SALU only   (no v_cmpx in any loop)
//  VMEM store of > 64 bits -> its data VGPRs         1     none: every store is one dword       -
//    rewritten
//  VALU writes SGPR -> VMEM reads it (address/      5     none: the store/load bases s[64:71]   -
//    soffset)                                              are SALU-written
//  s_set_gpr_idx_on -> indexed VALU, _off -> plain   0     DECIDE16R / COMMIT16 / INSERT16R     (the indexed moves sit between
//                                                                                              on and off; no non-indexed VALU
//                                                                                              read inside a region)
// A reorder that moves a consumer next to its producer in the table must add the s_nop.

// progress-based wave priority at each batch end: the fewer of its jobs a wave has decided, the higher
// its issue priority (s_setprio 3 while more than J/2 of the wave's jobs remain, 2 while more than J/4,
// 1 while more than J/8, else 0).  The waves sharing a SIMD then keep pace, instead of the oldest racing
// ahead under age-ordered issue and the youngest finishing alone, latency-bound, after the others have
// left.  r04 A/B (profiles/r04_prio_*, r04_geo*): quarters of J against no priority, C4 FIFO 8.08 ->
// 7.25 ms, C4 DELAY 7.58 -> 6.80, Level1-heavy DELAY 29.6 -> 26.3; these halving thresholds, which
// tighten the pack towards the end, a further 7.28 -> 7.08 and 26.45 -> 26.02 (1/4, 1/8, 1/16 lost;
// 1/2, 1/4, 1/16 tied).  s76 scratch (SCC from the subtraction: 0 remaining once the cursor passed J);
// P prefixes the labels.
#define MCS_FA_PRIO(P)                                                                            \
    "s_sub_u32 s76, s42, s57\n\t"                                                                 \
    "s_cselect_b32 s76, 0, s76\n\t"                                                               \
    "s_lshl_b32 s76, s76, 1\n\t"                                                                  \
    "s_cmp_gt_u32 s76, s42\n\t"                                                                   \
    "s_cbranch_scc0 " P "p2_%=\n\t"                                                              \
    "s_setprio 3\n\t"                                                                            \
    "s_branch " P "pe_%=\n"                                                                       \
    P "p2_%=:\n\t"                                                                               \
    "s_lshl_b32 s76, s76, 1\n\t"                                                                  \
    "s_cmp_gt_u32 s76, s42\n\t"                                                                   \
    "s_cbranch_scc0 " P "p1_%=\n\t"                                                              \
    "s_setprio 2\n\t"                                                                            \
    "s_branch " P "pe_%=\n"                                                                       \
    P "p1_%=:\n\t"                                                                               \
    "s_lshl_b32 s76, s76, 1\n\t"                                                                  \
    "s_cmp_gt_u32 s76, s42\n\t"                                                                   \
    "s_cbranch_scc0 " P "p0_%=\n\t"                                                              \
    "s_setprio 1\n\t"                                                                            \
    "s_branch " P "pe_%=\n"                                                                       \
    P "p0_%=:\n\t"                                                                               \
    "s_setprio 0\n"                                                                               \
    P "pe_%=:\n\t"

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

// the fused loop's clobbers: MCS_FA_CLOBBERS less the state it keeps in register-bound operands
// (MCS_FA_LOOP_F: s40 s43 s44 s47 s57 s59 s77 s78 s80-s84, v32-v55, v64-v67, v89-v93, v98-v101)
#define MCS_FF_CLOBBERS \
    "s41", "s42", "s45", "s46", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55", "s56", \
        "s58", "s60", "s61", "s62", "s63", "s64", "s65", "s66", "s67", "s68", "s69", "s70", \
        "s71", "s72", "s73", "s74", "s75", "s76", "s79", "s85", "s86", "s87", "s88", "s89", \
        "s90", "s91", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", \
        "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v94", "v95", \
        "v96", "v97", "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", \
        "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127", \
        "vcc", "scc", "m0", "exec", "memory" \
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
// wave once after the last row).  r05: a row with an expiry branches to its body out of line
// (MCS_FR_BODY, placed by the loop after an unconditional branch) and returns; a row without one
// falls through.  ~1.5 of the 8 rows expire per scan, so a scan takes ~3 taken branches instead of
// ~6.5: at one wave per SIMD a taken branch costs ~20 cycles, the row test ~8.
#define MCS_FR_ROW(p, MASK, F, P, A)                                                              \
    "s_and_b64 exec, " MASK ", -1\n\t"                                                           \
    "s_cbranch_scc1 mcsfa_rb" #p "_%=\n"                                                         \
    "mcsfa_r" #p "_%=:\n\t"
#define MCS_FR_BODY(p, MASK, F, P, A)                                                             \
    "mcsfa_rb" #p "_%=:\n\t"                                                                     \
    "s_bcnt1_i32_b64 s76, " MASK "\n\t"                                                          \
    "ds_add_u32 " A ", " P "\n\t"                                                               \
    "v_mov_b32 " F ", -1\n\t"                                                                    \
    "s_add_u32 s75, s75, s76\n\t"                                                                \
    "v_or_b32 v89, 1<<" #p ", v89\n\t"                                                           \
    "s_branch mcsfa_r" #p "_%=\n"
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
// the expiring rows' bodies of MCS_FA_SCAN16R (out of line: after an unconditional branch)
#define MCS_FA_RBODY16R                                                                           \
    MCS_FR_BODY(0, "s[50:51]", "v32", "v40", "v48") MCS_FR_BODY(1, "s[52:53]", "v33", "v41", "v49") \
    MCS_FR_BODY(2, "s[54:55]", "v34", "v42", "v50") MCS_FR_BODY(3, "s[60:61]", "v35", "v43", "v51") \
    MCS_FR_BODY(4, "s[62:63]", "v36", "v44", "v52") MCS_FR_BODY(5, "s[86:87]", "v37", "v45", "v53") \
    MCS_FR_BODY(6, "s[88:89]", "v38", "v46", "v54") MCS_FR_BODY(7, "s[90:91]", "v39", "v47", "v55")
#define MCS_FA_RBODY16S                                                                           \
    MCS_FR_BODY(0, "s[50:51]", "v32", "v40", "v48") MCS_FR_BODY(1, "s[52:53]", "v33", "v41", "v49")
#define MCS_FA_RBODY32 ""
#define MCS_FA_RBODY16 ""
#define MCS_FA_RBODY16D ""

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

// the end of a release scan: the wave's earliest remaining finish (DPP minimum of v90) under the
// node reload's latency, then the reload's wait
#define MCS_FA_SCANEND                                                                            \
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
    "s_waitcnt lgkmcnt(0)\n\t"
#define MCS_FA_SCANEND32 MCS_FA_SCANEND
#define MCS_FA_SCANEND16 MCS_FA_SCANEND
#define MCS_FA_SCANEND16R MCS_FA_SCANEND
#define MCS_FA_SCANEND16S MCS_FA_SCANEND
// batch-end hook (the duo loop's ring check); nothing for the one-wave forms
#define MCS_FA_BENDCHK32 ""
#define MCS_FA_BENDCHK16 ""
#define MCS_FA_BENDCHK16R ""
#define MCS_FA_BENDCHK16S ""

// ---- W16D: the duo loop's decision wave (fifo_duo_kernel, mcs_fifo_asm.hip) --------------------
// W16R's node format and first fit, with the running slots held by a second wave of the workgroup
// (the release wave, MCS_FH_LOOP below): a commit posts the slot {kx, finish, payload, seq} to an LDS
// ring instead of inserting it, and a clock advance past the earliest finish applies the release
// packet the release wave keeps ready for it (the payloads of the slots finishing at that second,
// summed per node in the node registers' layout) with four v_pk_add_u16 — no slot scan, no LDS
// node round trip and no wave minimum on this wave's chain.
//   s49 slots posted   s60 ring offset of the next post   s62 finish of the last post   s63 waits
//   v102-v106 the post   v109 ring base   v118 the packet's delta words of this lane (+256 per chunk)
//   v119 packet header {e1, e2, posts taken, slots} (+16: ack, +20: done)
// Header check: the packet is for this wave's earliest finish s77 and the release wave has taken
// every post, or every post but the last one whose finish lies after the packet's second (its own
// second then becomes the next candidate).  Otherwise the wave re-reads the header (bounded: past
// 4096 reads the cluster stops as a pool overflow and the engine re-runs it on the compiled kernel).
#define MCS_FA_FIT16D                                                                             \
    "v_pk_sub_u16 v72, v64, s48\n\t"                                                              \
    "v_pk_sub_u16 v73, v65, s48\n\t"                                                              \
    "v_pk_sub_u16 v74, v66, s48\n\t"                                                              \
    "v_pk_sub_u16 v75, v67, s48\n\t"                                                              \
    "v_and_b32_sdwa v80, v72, v72 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_0\n\t" \
    "v_and_b32_sdwa v81, v74, v74 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_0\n\t" \
    "v_and_b32_sdwa v80, v73, v73 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_0\n\t" \
    "v_and_b32_sdwa v81, v75, v75 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_0\n\t" \
    "s_nop 1\n\t" /* (the SDWA hazard of MCS_FA_FIT16) */                                       \
    "v_perm_b32 v86, v81, v80, s72\n\t"
#define MCS_FA_ANYFIT16D MCS_FA_ANYFIT
#define MCS_FA_DECIDE16D                                                                          \
    "v_readlane_b32 s51, v86, s50\n\t"                                                            \
    "s_lshl_b64 exec, 1, s50\n\t"                                                                 \
    "s_ff1_i32_b32 s52, s51\n\t"                                                                  \
    "s_lshr_b32 s53, s52, 3\n\t"                                                                  \
    "s_lshl3_add_u32 s54, s52, s50\n\t"                                                           \
    "s_set_gpr_idx_on s53, gpr_idx(SRC0,DST)\n\t"                                                 \
    "v_mov_b32 v64, v72\n\t" /* the commit (cluster.go:146-147) */                                \
    "s_set_gpr_idx_off\n\t"                                                                       \
    /* the post, seq written last (the release wave takes an entry by its seq) */                \
    "v_mov_b64 v[102:103], s[54:55]\n\t"                                                          \
    "v_mov_b32 v104, s48\n\t"                                                                     \
    "v_mov_b32 v105, s49\n\t"                                                                     \
    "v_add_u32 v106, s60, v109\n\t"                                                               \
    "ds_write_b96 v106, v[102:104]\n\t"                                                           \
    "ds_write_b32 v106, v105 offset:12\n\t"                                                       \
    "s_add_u32 s49, s49, 1\n\t"                                                                   \
    "s_add_u32 s60, s60, 16\n\t"                                                                  \
    "s_and_b32 s60, s60, 0x7f0\n\t"                                                               \
    "s_mov_b32 s62, s55\n\t"
#define MCS_FA_REC16D MCS_FA_REC16
#define MCS_FA_ZEROKX16D MCS_FA_ZEROKX
#define MCS_FA_POOLMAX16D "64*8"
#define MCS_FA_NODEIDX16D MCS_FA_NODEIDX
#define MCS_FA_TAKE16D MCS_FA_TAKE16
#define MCS_FA_RELOAD16D MCS_FA_RELOAD16
#define MCS_FA_INIT16D                                                                            \
    "s_mov_b32 s49, 0\n\t" MCS_FD_SPIN0                                                          \
    "s_mov_b32 s60, 0\n\t"                                                                        \
    "s_mov_b32 s62, 0\n\t"                                                                        \
    "s_mov_b32 s63, 0\n\t"                                                                        \
    "v_mov_b32 v118, %[dl]\n\t"                                                                   \
    "v_mov_b32 v119, %[hdr]\n\t"
#define MCS_FA_SCAN16D                                                                            \
    "mcsfd_rd_%=:\n\t"                                                                            \
    "ds_read_b128 v[120:123], v119\n\t"                                                           \
    "ds_read2st64_b32 v[124:125], v118 offset1:1\n\t"                                             \
    "ds_read2st64_b32 v[126:127], v118 offset0:2 offset1:3\n\t"                                   \
    "s_waitcnt lgkmcnt(0)\n\t"                                                                    \
    "v_readfirstlane_b32 s86, v120\n\t" /* e1 */                                                 \
    "v_readfirstlane_b32 s87, v121\n\t" /* e2 */                                                 \
    "v_readfirstlane_b32 s88, v122\n\t" /* posts taken */                                        \
    "v_readfirstlane_b32 s75, v123\n\t" /* slots finishing at e1 */                              \
    "s_sub_u32 s89, s49, s88\n\t"                                                                 \
    "s_cmp_eq_u32 s89, 0\n\t"                                                                     \
    "s_cbranch_scc1 mcsfd_all_%=\n\t"                                                             \
    "s_cmp_eq_u32 s89, 1\n\t"                                                                     \
    "s_cbranch_scc0 mcsfd_wait_%=\n\t"                                                            \
    "s_cmp_gt_u32 s62, s86\n\t"                                                                   \
    "s_cbranch_scc0 mcsfd_wait_%=\n\t"                                                            \
    "s_min_u32 s87, s87, s62\n"                                                                   \
    "mcsfd_all_%=:\n\t"                                                                           \
    "s_cmp_eq_u32 s86, s77\n\t"                                                                   \
    "s_cbranch_scc0 mcsfd_wait_%=\n\t"                                                            \
    "v_pk_add_u16 v64, v64, v124\n\t" /* the releases (cluster.go:153-157) */                   \
    "v_pk_add_u16 v65, v65, v125\n\t"                                                             \
    "v_pk_add_u16 v66, v66, v126\n\t"                                                             \
    "v_pk_add_u16 v67, v67, v127\n\t"                                                             \
    "v_mov_b32 v120, s86\n\t"                                                                     \
    "s_mov_b64 exec, 1\n\t"                                                                       \
    "ds_write_b32 v119, v120 offset:16\n\t" /* ack: the release wave retires e1 */             \
    "s_mov_b64 exec, -1\n\t"                                                                      \
    "s_sub_u32 s80, s80, s75\n\t"                                                                 \
    "s_mov_b32 s77, s87\n\t"                                                                      \
    "s_mov_b32 s63, 0\n\t"                                                                        \
    "s_cmp_lt_u32 s40, s77\n\t"                                                                   \
    "s_cbranch_scc1 mcsfd_done_%=\n\t"                                                            \
    "s_branch mcsfd_rd_%=\n" /* a second finish second is due too (rare) */                      \
    "mcsfd_wait_%=:\n\t" MCS_FD_SPIN                                                              \
    "s_bitcmp1_b32 s75, 31\n\t" /* the release wave's slots overflowed */                       \
    "s_cbranch_scc1 mcsfa_poolovf_%=\n\t"                                                         \
    "s_add_u32 s63, s63, 1\n\t"                                                                   \
    "s_cmp_gt_u32 s63, 0x1000\n\t"                                                                \
    "s_cbranch_scc1 mcsfa_poolovf_%=\n\t"                                                         \
    "s_branch mcsfd_rd_%=\n"                                                                      \
    "mcsfd_done_%=:\n\t"
#define MCS_FA_SCANEND16D ""
// the ring holds 128 posts: at a batch end at most 64 may be untaken, so the batch's <= 64 posts
// cannot overwrite one
#define MCS_FA_BENDCHK16D                                                                         \
    "mcsfd_bc_%=:\n\t"                                                                            \
    "ds_read_b32 v120, v119 offset:8\n\t"                                                         \
    "s_waitcnt lgkmcnt(0)\n\t"                                                                    \
    "v_readfirstlane_b32 s88, v120\n\t"                                                           \
    "s_sub_u32 s89, s49, s88\n\t"                                                                 \
    "s_cmp_le_u32 s89, 64\n\t"                                                                    \
    "s_cbranch_scc1 mcsfd_bcok_%=\n\t"                                                            \
    "s_add_u32 s63, s63, 1\n\t"                                                                   \
    "s_cmp_gt_u32 s63, 0x1000\n\t"                                                                \
    "s_cbranch_scc1 mcsfa_poolovf_%=\n\t"                                                         \
    "s_branch mcsfd_bc_%=\n"                                                                      \
    "mcsfd_bcok_%=:\n\t"                                                                          \
    "s_mov_b32 s63, 0\n\t"
#define MCS_FD_CLOBBERS MCS_FA_CLOBBERS, "v102", "v103", "v104", "v105", "v106"

// ---- the duo loop's release wave: the running slots and the release packet ------------------------
// Rows as W16R (row r of a lane: v(32+r) finish, v(40+r) payload, v(48+r) the node's delta word
// address), free rows in v89 (+ the 0x100 sentinel).  The wave polls the ack word, the done word and
// the ring entry of its next post; a post is inserted (and added to the packet when it finishes at
// e1, or starts a new packet when it finishes earlier), an ack of e1 frees e1's slots and builds the
// packet of the next finish second.  Every change publishes the header {e1, e2, posts taken, slots
// at e1} after the delta words it covers (one wave's LDS operations complete in order).
//   s40 e1  s41 e2  s42 posts taken  s43 slots at e1 (bit 31: a post found no free slot)
//   s44 ring offset  s45-s55 temps  s56 polls  s57 poll bound  s58 delta base  s59 0x100
//   v109 ring base  v111 -1  v112 0  v113 ring entry address  v114 this lane's delta words
//   v115 header address  v117 lowest free row  v120-v127 reads / temps
#define MCS_FH_FREE(p, MASK, F)                                                                   \
    "s_and_b64 exec, " MASK ", -1\n\t"                                                            \
    "s_cbranch_scc0 mcsfh_f" #p "_%=\n\t"                                                         \
    "v_mov_b32 " F ", -1\n\t"                                                                     \
    "v_or_b32 v89, 1<<" #p ", v89\n"                                                              \
    "mcsfh_f" #p "_%=:\n\t"
#define MCS_FH_ADD(p, MASK, P, A)                                                                 \
    "s_and_b64 exec, " MASK ", -1\n\t"                                                            \
    "s_cbranch_scc0 mcsfh_a" #p "_%=\n\t"                                                         \
    "s_bcnt1_i32_b64 s54, " MASK "\n\t"                                                           \
    "ds_add_u32 " A ", " P "\n\t"                                                                 \
    "s_add_u32 s43, s43, s54\n"                                                                   \
    "mcsfh_a" #p "_%=:\n\t"
#define MCS_FH_CMP(s0)                                                                            \
    "v_cmp_eq_u32_e64 s[60:61], " s0 ", v32\n\t"                                                  \
    "v_cmp_eq_u32_e64 s[62:63], " s0 ", v33\n\t"                                                  \
    "v_cmp_eq_u32_e64 s[64:65], " s0 ", v34\n\t"                                                  \
    "v_cmp_eq_u32_e64 s[66:67], " s0 ", v35\n\t"                                                  \
    "v_cmp_eq_u32_e64 s[68:69], " s0 ", v36\n\t"                                                  \
    "v_cmp_eq_u32_e64 s[70:71], " s0 ", v37\n\t"                                                  \
    "v_cmp_eq_u32_e64 s[72:73], " s0 ", v38\n\t"                                                  \
    "v_cmp_eq_u32_e64 s[74:75], " s0 ", v39\n\t"
#define MCS_FH_LOOP                                                                               \
    "s_mov_b32 s40, -1\n\t"                                                                       \
    "s_mov_b32 s41, -1\n\t"                                                                       \
    "s_mov_b32 s42, 0\n\t"                                                                        \
    "s_mov_b32 s43, 0\n\t"                                                                        \
    "s_mov_b32 s44, 0\n\t"                                                                        \
    "s_mov_b32 s56, 0\n\t"                                                                        \
    "s_mov_b32 s57, %[hb]\n\t"                                                                    \
    "s_mov_b32 s58, %[db]\n\t"                                                                    \
    "s_mov_b32 s59, 0x100\n\t"                                                                    \
    "v_mov_b32 v109, %[rb]\n\t"                                                                   \
    "v_mov_b32 v111, -1\n\t"                                                                      \
    "v_mov_b32 v112, 0\n\t"                                                                       \
    "v_mov_b32 v113, %[rb]\n\t"                                                                   \
    "v_mov_b32 v114, %[dl]\n\t"                                                                   \
    "v_mov_b32 v115, %[hdr]\n\t"                                                                  \
    "v_mov_b32 v89, 0x1ff\n\t"                                                                    \
    "v_mov_b32 v32, -1\n\t"                                                                       \
    "v_mov_b32 v33, -1\n\t"                                                                       \
    "v_mov_b32 v34, -1\n\t"                                                                       \
    "v_mov_b32 v35, -1\n\t"                                                                       \
    "v_mov_b32 v36, -1\n\t"                                                                       \
    "v_mov_b32 v37, -1\n\t"                                                                       \
    "v_mov_b32 v38, -1\n\t"                                                                       \
    "v_mov_b32 v39, -1\n"                                                                         \
    "mcsfh_poll_%=:\n\t"                                                                          \
    /* the ack and done words before the ring entry: a post precedes any later ack of the   */    \
    /* decision wave, so an ack seen here comes with every post before it                   */    \
    "ds_read_b32 v120, v115 offset:16\n\t"                                                        \
    "ds_read_b32 v121, v115 offset:20\n\t"                                                        \
    "ds_read_b128 v[124:127], v113\n\t"                                                           \
    "s_waitcnt lgkmcnt(0)\n\t"                                                                    \
    "v_readfirstlane_b32 s45, v127\n\t"                                                           \
    "s_cmp_eq_u32 s45, s42\n\t"                                                                   \
    "s_cbranch_scc1 mcsfh_ins_%=\n\t"                                                             \
    "v_readfirstlane_b32 s45, v120\n\t"                                                           \
    "s_cmp_eq_u32 s45, s40\n\t"                                                                   \
    "s_cbranch_scc1 mcsfh_rel_%=\n\t"                                                             \
    "v_readfirstlane_b32 s45, v121\n\t"                                                           \
    "s_cmp_lg_u32 s45, 0\n\t"                                                                     \
    "s_cbranch_scc1 mcsfh_exit_%=\n\t"                                                            \
    "s_add_u32 s56, s56, 1\n\t"                                                                   \
    "s_cmp_gt_u32 s56, s57\n\t"                                                                   \
    "s_cbranch_scc1 mcsfh_exit_%=\n\t" MCS_FH_IDLE                                                \
    "s_branch mcsfh_poll_%=\n"                                                                    \
                                                                                                  \
    /* ---- a post: insert the slot ---- */                                                       \
    "mcsfh_ins_%=:\n\t"                                                                           \
    "v_readfirstlane_b32 s48, v124\n\t" /* kx */                                                 \
    "v_readfirstlane_b32 s46, v125\n\t" /* finish */                                             \
    "v_readfirstlane_b32 s47, v126\n\t" /* payload */                                            \
    "s_add_u32 s42, s42, 1\n\t"                                                                   \
    "s_add_u32 s44, s44, 16\n\t"                                                                  \
    "s_and_b32 s44, s44, 0x7f0\n\t"                                                               \
    "v_add_u32 v113, s44, v109\n\t"                                                               \
    "s_lshl2_add_u32 s49, s48, s58\n\t" /* the node's delta word */                              \
    "v_cmp_lt_u32_e64 s[50:51], s59, v89\n\t" /* lanes with a free row */                       \
    "v_ffbl_b32 v117, v89\n\t"                                                                    \
    "s_ff1_i32_b64 s52, s[50:51]\n\t"                                                             \
    "s_cmp_eq_u32 s52, -1\n\t"                                                                    \
    "s_cbranch_scc1 mcsfh_full_%=\n\t"                                                            \
    "v_readlane_b32 s53, v117, s52\n\t"                                                           \
    "s_lshl_b64 exec, 1, s52\n\t"                                                                 \
    "s_set_gpr_idx_on s53, gpr_idx(DST)\n\t"                                                      \
    "v_mov_b32 v32, s46\n\t"                                                                      \
    "v_mov_b32 v40, s47\n\t"                                                                      \
    "v_mov_b32 v48, s49\n\t"                                                                      \
    "s_set_gpr_idx_off\n\t"                                                                       \
    "s_lshl_b32 s54, 1, s53\n\t"                                                                  \
    "v_xor_b32 v89, s54, v89\n\t"                                                                 \
    /* the packet: a slot at e1 joins it, an earlier one starts a new one (e1 becomes e2) */      \
    "s_cmp_eq_u32 s46, s40\n\t"                                                                   \
    "s_cbranch_scc1 mcsfh_add_%=\n\t"                                                             \
    "s_cmp_lt_u32 s46, s40\n\t"                                                                   \
    "s_cbranch_scc1 mcsfh_new_%=\n\t"                                                             \
    "s_min_u32 s41, s41, s46\n\t"                                                                 \
    "s_branch mcsfh_pub_%=\n"                                                                     \
    "mcsfh_new_%=:\n\t"                                                                           \
    "s_mov_b32 s41, s40\n\t"                                                                      \
    "s_mov_b32 s40, s46\n\t"                                                                      \
    "s_and_b32 s43, s43, 0x80000000\n\t"                                                          \
    "s_mov_b64 exec, -1\n\t"                                                                      \
    "ds_write2st64_b32 v114, v112, v112 offset1:1\n\t"                                            \
    "ds_write2st64_b32 v114, v112, v112 offset0:2 offset1:3\n\t"                                  \
    "s_lshl_b64 exec, 1, s52\n"                                                                   \
    "mcsfh_add_%=:\n\t" /* (exec = the slot's lane) */                                           \
    "v_mov_b32 v120, s49\n\t"                                                                     \
    "v_mov_b32 v121, s47\n\t"                                                                     \
    "ds_add_u32 v120, v121\n\t"                                                                   \
    "s_add_u32 s43, s43, 1\n"                                                                     \
    "mcsfh_pub_%=:\n\t"                                                                           \
    "s_mov_b64 exec, 1\n\t"                                                                       \
    "v_mov_b32 v120, s40\n\t"                                                                     \
    "v_mov_b32 v121, s41\n\t"                                                                     \
    "v_mov_b32 v122, s42\n\t"                                                                     \
    "v_mov_b32 v123, s43\n\t"                                                                     \
    "ds_write_b128 v115, v[120:123]\n\t"                                                          \
    "s_mov_b64 exec, -1\n\t"                                                                      \
    "s_branch mcsfh_poll_%=\n"                                                                    \
    "mcsfh_full_%=:\n\t" /* no free slot: the decision wave stops as a pool overflow */          \
    "s_bitset1_b32 s43, 31\n\t"                                                                   \
    "s_branch mcsfh_pub_%=\n"                                                                     \
                                                                                                  \
    /* ---- an ack of e1: free e1's slots, build the packet of the next finish second ---- */     \
    "mcsfh_rel_%=:\n\t"                                                                           \
    "ds_write2st64_b32 v114, v112, v112 offset1:1\n\t"                                            \
    "ds_write2st64_b32 v114, v112, v112 offset0:2 offset1:3\n\t" MCS_FH_CMP("s40")                \
    MCS_FH_FREE(0, "s[60:61]", "v32") MCS_FH_FREE(1, "s[62:63]", "v33")                           \
    MCS_FH_FREE(2, "s[64:65]", "v34") MCS_FH_FREE(3, "s[66:67]", "v35")                           \
    MCS_FH_FREE(4, "s[68:69]", "v36") MCS_FH_FREE(5, "s[70:71]", "v37")                           \
    MCS_FH_FREE(6, "s[72:73]", "v38") MCS_FH_FREE(7, "s[74:75]", "v39")                           \
    "s_mov_b64 exec, -1\n\t"                                                                      \
    "s_mov_b32 s40, s41\n\t"                                                                      \
    "s_and_b32 s43, s43, 0x80000000\n\t"                                                          \
    "s_mov_b32 s41, -1\n\t"                                                                       \
    "s_cmp_eq_u32 s40, -1\n\t"                                                                    \
    "s_cbranch_scc1 mcsfh_pub_%=\n\t" MCS_FH_CMP("s40")                                           \
    MCS_FH_ADD(0, "s[60:61]", "v40", "v48") MCS_FH_ADD(1, "s[62:63]", "v41", "v49")               \
    MCS_FH_ADD(2, "s[64:65]", "v42", "v50") MCS_FH_ADD(3, "s[66:67]", "v43", "v51")               \
    MCS_FH_ADD(4, "s[68:69]", "v44", "v52") MCS_FH_ADD(5, "s[70:71]", "v45", "v53")               \
    MCS_FH_ADD(6, "s[72:73]", "v46", "v54") MCS_FH_ADD(7, "s[74:75]", "v47", "v55")               \
    "s_mov_b64 exec, -1\n\t"                                                                      \
    /* e2: the earliest finish after e1 (f - (e1 + 1) wraps for e1's own slots and free rows) */  \
    "s_add_u32 s55, s40, 1\n\t"                                                                   \
    "v_subrev_u32 v120, s55, v32\n\t"                                                             \
    "v_subrev_u32 v121, s55, v33\n\t"                                                             \
    "v_subrev_u32 v122, s55, v34\n\t"                                                             \
    "v_subrev_u32 v123, s55, v35\n\t"                                                             \
    "v_subrev_u32 v124, s55, v36\n\t"                                                             \
    "v_subrev_u32 v125, s55, v37\n\t"                                                             \
    "v_subrev_u32 v126, s55, v38\n\t"                                                             \
    "v_subrev_u32 v127, s55, v39\n\t"                                                             \
    "v_min3_u32 v120, v120, v121, v122\n\t"                                                       \
    "v_min3_u32 v123, v123, v124, v125\n\t"                                                       \
    "v_min3_u32 v120, v120, v126, v127\n\t"                                                       \
    "v_min_u32 v120, v120, v123\n\t"                                                              \
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
    "v_readlane_b32 s41, v120, 63\n\t"                                                            \
    "s_add_u32 s41, s41, s55\n\t"                                                                 \
    "s_branch mcsfh_pub_%=\n"                                                                     \
    "mcsfh_exit_%=:\n\t"                                                                          \
    "s_waitcnt lgkmcnt(0)"
#define MCS_FH_CLOBBERS                                                                           \
    "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53",  \
        "s54", "s55", "s56", "s57", "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s65", "s66",     \
        "s67", "s68", "s69", "s70", "s71", "s72", "s73", "s74", "s75", "v32", "v33", "v34", "v35",     \
        "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48",     \
        "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v89", "v109", "v111", "v112", "v113",        \
        "v114", "v115", "v117", "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127", "vcc", \
        "scc", "exec", "memory"

// (probe builds: the decision wave's header re-reads in s85 (MCS_STAMPS); an idle poll of the
// release wave sleeps (MCS_FH_SLEEP, an A/B of its issue pressure))
#ifdef MCS_STAMPS
#define MCS_FD_SPIN "s_add_u32 s85, s85, 1\n\t"
#define MCS_FD_SPIN0 "s_mov_b32 s85, 0\n\t"
#else
#define MCS_FD_SPIN ""
#define MCS_FD_SPIN0 ""
#endif
#ifdef MCS_FH_SLEEP
#define MCS_FH_IDLE "s_sleep " MCS_FH_SLEEP "\n\t"
#else
#define MCS_FH_IDLE ""
#endif

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

// diagnostic counters (passes without a decision, release scans): DIAG launches only
#define MCS_FA_CNTS_D1 "s_add_u32 s83, s83, 1\n\t"
#define MCS_FA_CNTR_D1 "s_add_u32 s84, s84, 1\n\t"
#define MCS_FA_CNTS_D0 ""
#define MCS_FA_CNTR_D0 ""
