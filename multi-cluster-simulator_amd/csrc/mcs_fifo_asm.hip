// mcs_fifo_asm.hip — the batched FIFO decision loop, hand-scheduled for gfx950.
//
// Same algorithm, layout and results as fifo_kernel<4, 8, false, false, false> (mcs_kernels.hip):
// Scheduler.Fifo (pkg/scheduler/scheduler.go:216-296) over ScheduleJob's first fit (:127-139) and
// Node.RunJob's commit/release (pkg/scheduler/cluster.go:141-161), one cluster (up to 256 nodes)
// per wave64, SFIFO semantics with the exact fast-forward of SURVEY Appendix A.3.  The whole
// decision loop (batches, passes, releases, waits) is one asm statement on fixed registers, so
// the shape of each pass is chosen here instead of by the CFG structurizer:
//
//   * Fit test in VALU, no scalar mask algebra.  Node free vectors live in registers with a guard
//     bit: C = 2^31 + free_c, M = 2^31 + free_m (free < 2^31 - 1, checked on the host; requests
//     are clamped to 2^31 - 1 when a batch is loaded, which cannot change a fit).  a = C - cores
//     and b = M - mem keep bit 31 exactly when the node fits, so (a & b) >> 31 is the fit bit; two
//     v_perm (sign-replicating selectors) gather the four chunks' bits into one byte mask per lane
//     and one v_cmp gives the lanes with a fit.  Padding nodes hold 2^31 - 1 (no guard, and no
//     clamped request wraps it): they never fit, not even a zero job.
//   * Commit without branches: the lowest set byte of lane fl's mask is its first fitting chunk
//     c; under exec = lane fl, one indexed move pair (s_set_gpr_idx_on 2c) copies the already
//     computed a/b into that chunk's registers.
//   * Slot insert under exec = the lowest lane with a free row (s_ff1 of the free-row lanes,
//     ANDed back with them); a full pool leaves exec empty and is caught by peak > 64*P at the
//     batch end (the cluster is re-run with a bigger pool by the engine, as for the compiled
//     kernel).  The counters (used, peak, waited, passes) are scalar.
//   * The cursor's lane in the batch lives in m0: the record broadcasts (v_readlane) and the
//     result batch writes (v_writelane) select their lane with it directly.
//   * The ready head's arrival/clock checks, the WaitQueue bookkeeping and the releases follow
//     fifo_kernel line by line (see the comments there); the result batch keeps the node's LDS
//     index (chunk * 64 + lane) and converts it to the node index when it is stored.
//
// Hazards (wait states are not inserted by the compiler inside asm): DPP reads a VGPR 2 states
// after its write (s_nop 1), v_readlane reads a VGPR at least 1 instruction after its write, m0
// is read by v_writelane at least 1 state after an SALU write.  Loads and stores issued here are waited for before the statement ends.
#include "mcs_internal.h"
#include "mcs_lds.h"
#include "mcs_wave.h"

namespace mcs {

namespace {

constexpr int kAsmNpl = 4;
constexpr int kAsmPool = 8;
constexpr uint32_t kGuard = 0x80000000u;
constexpr uint32_t kClamp = 0x7FFFFFFFu;  // request clamp and padding value

// Register map of the loop (all fixed; listed as clobbers).
//   s40 t     s41 min(64, J - cb)  s42 J   s43 have_w  s44 flags  s45 arr   s46 dur
//   s47 cursor's lane in the batch (r - cb)  s[48:49] cores, mem   s50 fl   s51 byte mask of fl
//   s52 8 * chunk   s53 2 * chunk   s[54:55] kx, finish   s56 next clock   s57 cb
//   s[58:59] exec save   s[60:61] lanes with a free row   s[62:63] one-lane exec masks
//   s[64:65] jobs  s[66:67] out_node  s[68:69] out_start  s[70:71] out_finish  s72/s73 perm selectors
//   s74 t + 1  s75 expired  s76 tmp  s77 next completion  s78/s79 clock advances / bound 4J + 256
//   (a runaway loop ends as a pool overflow: the engine re-runs the cluster on the compiled kernel)
//   s80 used  s81 peak  s82 waited  s83 passes without a decision  s84 release scans  s85 insert lane
//   v[64:71] node pairs {C, M} per chunk    v[72:79] a/b per chunk (release: finish rows 0-3)
//   v[80:83] a&b   v84/v85 half masks   v86 byte mask (release: rows 4-7 in v[80:87])
//   v89 free rows  v90 earliest finish  v91-93 result batch (kx, start, finish)
//   v[94:97] records  v[98:101] next records   v107 slot column  v108 node column  v109 node base
//   v110 lane  v111 -1   v[112:113] need  v[114:115] {kx, fin}  v117 slot address  v118 frm - 1
//   v119 node address  v120 DPP min  v121 d / address  v[122:123] payload  v124 lane minimum
//   v125-v127 store temps
#define MCS_FA_CLOBBERS                                                                            \
    "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53",  \
        "s54", "s55", "s56", "s57", "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s65", "s66",     \
        "s67", "s68", "s69", "s70", "s71", "s72", "s73", "s74", "s75", "s76", "s77", "s78", "s79",     \
        "s80", "s81", "s82", "s83", "s84", "s85", "v64", "v65", "v66", "v67", "v68", "v69", "v70",     \
        "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83",     \
        "v84", "v85", "v86", "v87", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97",     \
        "v98", "v99", "v100", "v101", "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114",  \
        "v115", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125", "v126",        \
        "v127", "vcc", "scc", "m0", "exec", "memory"

// one release row p (cluster.go:153-157): node / finish words of the row in NODE / FIN
#define MCS_FA_ROW(p, NODE, FIN)                                                              \
    "v_cmp_ge_u32_e32 vcc, s40, " FIN "\n\t"                                                  \
    "v_subrev_u32 v121, s74, " FIN "\n\t"                                                     \
    "v_min_u32 v124, v121, v124\n\t"                                                          \
    "s_cbranch_vccz mcsfa_r" #p "_%=\n\t"                                                     \
    "s_bcnt1_i32_b64 s76, vcc\n\t"                                                            \
    "s_add_u32 s75, s75, s76\n\t"                                                             \
    "s_mov_b64 s[58:59], exec\n\t"                                                            \
    "s_mov_b64 exec, vcc\n\t"                                                                 \
    "ds_read_b64 v[122:123], v107 offset:" #p "*512\n\t"                                      \
    "v_lshl_add_u32 v121, " NODE ", 3, v109\n\t"                                              \
    "s_waitcnt lgkmcnt(0)\n\t"                                                                \
    "ds_add_u64 v121, v[122:123]\n\t"                                                         \
    "ds_write_b32 v107, v111 offset:4096+" #p "*512+4\n\t"                                    \
    "v_or_b32 v89, 1<<" #p ", v89\n\t"                                                        \
    "s_mov_b64 exec, s[58:59]\n"                                                              \
    "mcsfa_r" #p "_%=:\n\t"

__global__ __launch_bounds__(64) void fifo_asm_kernel(FifoArgs a) {
    const uint32_t item = blockIdx.x;
    const uint32_t ci = a.cluster_list ? a.cluster_list[item] : item;
    const uint32_t lane = threadIdx.x;

    // nodes [4][64] u64 at 0, slot payloads {cores | mem << 32} [8][64] at 2048, slot
    // {node | finish << 32} [8][64] at 6144 (the offsets in the asm below)
    __shared__ uint64_t lds[kAsmNpl * kWave + 2 * kAsmPool * kWave];
    uint64_t* const nodes = lds;
    uint64_t* const pay_nf = lds + kAsmNpl * kWave + kAsmPool * kWave;

    const uint32_t n0 = a.node_off[ci];
    const uint32_t N = a.node_off[ci + 1] - n0;
#pragma unroll
    for (int c = 0; c < kAsmNpl; ++c) {
        const uint32_t node = lane * kAsmNpl + c;
        uint64_t w = (uint64_t)kClamp | ((uint64_t)kClamp << 32);  // padding: never fits
        if (node < N) {
            const uint2 v = a.node_free0[n0 + node];
            w = (uint64_t)(v.x + kGuard) | ((uint64_t)(v.y + kGuard) << 32);
        }
        nodes[c * kWave + lane] = w;
    }
#pragma unroll
    for (int p = 0; p < kAsmPool; ++p) pay_nf[p * kWave + lane] = (uint64_t)kEmpty << 32;

    const uint64_t j0 = a.job_off[ci];
    const uint32_t J = (uint32_t)(a.job_off[ci + 1] - j0);
    const uint4* jobs = a.jobs + j0;
    int32_t* o_node = a.out_node + j0;
    uint32_t* o_start = a.out_start + j0;
    uint32_t* o_finish = a.out_finish + j0;

    uint4 cur = jobs[lane];  // batch 0 (the array has kJobPad records of slack)
    cur.z = cur.z < kClamp ? cur.z : kClamp;
    cur.w = cur.w < kClamp ? cur.w : kClamp;
    uint64_t nv[kAsmNpl];
    __syncthreads();  // (one wave: orders the LDS initialisation before the reads)
#pragma unroll
    for (int c = 0; c < kAsmNpl; ++c) nv[c] = nodes[c * kWave + lane];

    const uint32_t base = lds_addr(lds);
    const uint32_t v_pay = base + 2048u + lane * 8u;
    const uint32_t v_nb = base + lane * 8u;
    const uint32_t v_nbase = base;

    uint32_t t = 0, r = 0, flags = 0, have_w = 0;
    uint32_t frm = (1u << kAsmPool) - 1u, lmin = kEmpty;
    uint32_t used = 0, peak = 0, waited = 0, n_slow = 0, n_rel = 0;
    uint32_t on = 0, os = 0, of = 0;

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
    asm volatile(
        // ---- entry: state into the fixed registers ----
        "s_mov_b32 s40, %[t]\n\t"
        "s_mov_b32 s42, %[J]\n\t"
        "s_mov_b32 s43, 0\n\t"
        "s_mov_b32 s44, 0\n\t"
        "s_mov_b32 s47, 0\n\t"
        "s_mov_b32 s57, 0\n\t"
        "s_mov_b32 s78, 0\n\t"
        "s_lshl2_add_u32 s79, s42, 0x100\n\t"
        "s_mov_b32 s80, 0\n\t"
        "s_mov_b32 s81, 0\n\t"
        "s_mov_b32 s82, 0\n\t"
        "s_mov_b32 s83, 0\n\t"
        "s_mov_b32 s84, 0\n\t"
        "s_mov_b64 s[64:65], %[jobs]\n\t"
        "s_mov_b64 s[66:67], %[onp]\n\t"
        "s_mov_b64 s[68:69], %[osp]\n\t"
        "s_mov_b64 s[70:71], %[ofp]\n\t"
        "s_mov_b32 s72, 0x0c0c0b09\n\t"
        "s_mov_b32 s73, 0x0b090c0c\n\t"
        "v_mov_b64 v[64:65], %[n0]\n\t"
        "v_mov_b64 v[66:67], %[n1]\n\t"
        "v_mov_b64 v[68:69], %[n2]\n\t"
        "v_mov_b64 v[70:71], %[n3]\n\t"
        "v_mov_b32 v89, %[frm]\n\t"
        "v_mov_b32 v90, %[lmin]\n\t"
        "v_mov_b32 v94, %[c0]\n\t"
        "v_mov_b32 v95, %[c1]\n\t"
        "v_mov_b32 v96, %[c2]\n\t"
        "v_mov_b32 v97, %[c3]\n\t"
        "v_mov_b32 v107, %[pay]\n\t"
        "v_mov_b32 v108, %[nb]\n\t"
        "v_mov_b32 v109, %[nbase]\n\t"
        "v_mov_b32 v110, %[lane]\n\t"
        "v_mov_b32 v111, -1\n\t"
        // prefetch batch 1
        "v_lshlrev_b32 v121, 4, v110\n\t"
        "v_add_u32 v121, 0x400, v121\n\t"
        "global_load_dwordx4 v[98:101], v121, s[64:65]\n\t"
        "s_min_u32 s41, s42, 64\n\t"
        "v_readlane_b32 s45, v94, s47\n\t"
        "v_readlane_b32 s46, v95, s47\n\t"
        "v_readlane_b32 s48, v96, s47\n\t"
        "v_readlane_b32 s49, v97, s47\n\t"
        "s_cmp_lt_u32 s47, s41\n\t"
        "s_cbranch_scc0 mcsfa_bend_%=\n"

        // ---- one pass = one decision (scheduler.go:216-296) ----
        "mcsfa_inner_%=:\n\t"
        "s_cmp_gt_u32 s45, s40\n\t"  // ready head not arrived: sleep to it
        "s_cbranch_scc1 mcsfa_arrive_%=\n\t"
        // first fit (:129-137): a, b per chunk; fit bit = bit 31 of a & b
        "v_subrev_u32 v72, s48, v64\n\t"
        "v_subrev_u32 v73, s49, v65\n\t"
        "v_subrev_u32 v74, s48, v66\n\t"
        "v_subrev_u32 v75, s49, v67\n\t"
        "v_subrev_u32 v76, s48, v68\n\t"
        "v_subrev_u32 v77, s49, v69\n\t"
        "v_subrev_u32 v78, s48, v70\n\t"
        "v_subrev_u32 v79, s49, v71\n\t"
        "v_and_b32 v80, v72, v73\n\t"
        "v_and_b32 v81, v74, v75\n\t"
        "v_and_b32 v82, v76, v77\n\t"
        "v_and_b32 v83, v78, v79\n\t"
        "v_perm_b32 v84, v81, v80, s72\n\t"  // bytes 0/1 = 0xff if chunk 0/1 fits
        "v_perm_b32 v85, v83, v82, s73\n\t"  // bytes 2/3 for chunks 2/3
        "v_or_b32 v86, v84, v85\n\t"
        "v_cmp_ne_u32_e32 vcc, 0, v86\n\t"
        "s_cbranch_vccz mcsfa_nofit_%=\n\t"
        "s_ff1_i32_b64 s50, vcc\n\t"  // lowest lane with a fit
        "s_cmp_eq_u32 s46, 0\n\t"
        "s_cbranch_scc1 mcsfa_zero_%=\n\t"
        "v_readlane_b32 s51, v86, s50\n\t"
        "v_cmp_ne_u32_e64 s[60:61], 0, v89\n\t"
        "s_lshl_b64 s[62:63], 1, s50\n\t"
        "s_mov_b64 s[58:59], exec\n\t"
        "s_ff1_i32_b32 s52, s51\n\t"         // 8 * its first fitting chunk
        "s_lshr_b32 s53, s52, 2\n\t"
        "s_lshl3_add_u32 s54, s52, s50\n\t"  // kx = chunk * 64 + fl
        "s_add_u32 s55, s40, s46\n\t"        // finish
        // commit in registers (cluster.go:146-147): lane fl, chunk pair a/b -> C/M (indexed)
        "s_mov_b64 exec, s[62:63]\n\t"
        "s_set_gpr_idx_on s53, gpr_idx(SRC0,DST)\n\t"
        "v_mov_b32 v64, v72\n\t"
        "v_mov_b32 v65, v73\n\t"
        "s_set_gpr_idx_off\n\t"
        // running-slot insert: lowest lane with a free row (none: exec empty), its lowest free row
        "s_ff1_i32_b64 s85, s[60:61]\n\t"
        "s_lshl_b64 s[62:63], 1, s85\n\t"
        "s_and_b64 exec, s[62:63], s[60:61]\n\t"
        "v_mov_b64 v[112:113], s[48:49]\n\t"
        "v_mov_b64 v[114:115], s[54:55]\n\t"
        "v_lshl_add_u32 v119, s54, 3, v109\n\t"
        "v_ffbl_b32 v117, v89\n\t"
        "v_lshl_add_u32 v117, v117, 9, v107\n\t"
        "v_add_u32 v118, -1, v89\n\t"
        "ds_sub_u64 v119, v[112:113]\n\t"
        "ds_write_b64 v117, v[112:113]\n\t"
        "ds_write_b64 v117, v[114:115] offset:4096\n\t"
        "v_and_b32 v89, v118, v89\n\t"
        "v_min_u32 v90, s55, v90\n\t"
        "s_mov_b64 exec, s[58:59]\n\t"
        "s_mov_b32 m0, s47\n\t"
        "s_add_u32 s80, s80, 1\n\t"
        "s_max_u32 s81, s81, s80\n\t"
        "v_writelane_b32 v91, s54, m0\n\t"
        "v_writelane_b32 v92, s40, m0\n\t"
        "v_writelane_b32 v93, s55, m0\n"
        // next ready job; a WaitQueue head placed sleeps 1 s (:250)
        "mcsfa_placed_%=:\n\t"
        "s_add_u32 s47, s47, 1\n\t"
        "s_cmp_lg_u32 s43, 0\n\t"
        "v_readlane_b32 s45, v94, s47\n\t"
        "v_readlane_b32 s46, v95, s47\n\t"
        "v_readlane_b32 s48, v96, s47\n\t"
        "v_readlane_b32 s49, v97, s47\n\t"
        "s_cbranch_scc1 mcsfa_hwadv_%=\n"
        "mcsfa_loopend_%=:\n\t"
        "s_cmp_lt_u32 s47, s41\n\t"
        "s_cbranch_scc1 mcsfa_inner_%=\n\t"
        "s_branch mcsfa_bend_%=\n"

        // zero-duration job: committed and released before the next decision (D3)
        "mcsfa_zero_%=:\n\t"
        "v_readlane_b32 s51, v86, s50\n\t"
        "s_mov_b32 m0, s47\n\t"
        "s_ff1_i32_b32 s52, s51\n\t"
        "s_lshl3_add_u32 s54, s52, s50\n\t"
        "v_writelane_b32 v91, s54, m0\n\t"
        "v_writelane_b32 v92, s40, m0\n\t"
        "v_writelane_b32 v93, s40, m0\n\t"
        "s_branch mcsfa_placed_%=\n"

        "mcsfa_hwadv_%=:\n\t"
        "s_mov_b32 s43, 0\n\t"
        "s_add_u32 s56, s40, 1\n\t"
        "s_branch mcsfa_adv_%=\n"

        // no node fits: WaitQueue append (:264-268), sleep to the next completion (A.3)
        "mcsfa_nofit_%=:\n\t"
        "s_sub_u32 s76, 1, s43\n\t"
        "s_add_u32 s82, s82, s76\n\t"
        "s_mov_b32 s43, 1\n\t"
        "s_add_u32 s83, s83, 1\n\t"
        "v_mov_b32 v120, v90\n\t"
        "s_nop 1\n\t"
        "v_min_u32_dpp v120, v120, v120 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_min_u32_dpp v120, v120, v120 row_shr:2 row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_min_u32_dpp v120, v120, v120 row_shr:4 row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_min_u32_dpp v120, v120, v120 row_shr:8 row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_min_u32_dpp v120, v120, v120 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_min_u32_dpp v120, v120, v120 row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_readlane_b32 s77, v120, 63\n\t"
        "s_cmp_eq_u32 s77, -1\n\t"
        "s_cbranch_scc1 mcsfa_deadlock_%=\n\t"
        "s_add_u32 s56, s40, 1\n\t"
        "s_max_u32 s56, s56, s77\n\t"
        "s_branch mcsfa_adv_%=\n"

        "mcsfa_arrive_%=:\n\t"
        "s_mov_b32 s56, s45\n\t"
        "s_add_u32 s83, s83, 1\n"
        // advance the clock to s56: releases at the new instant (A.2 step 1)
        "mcsfa_adv_%=:\n\t"
        "s_add_u32 s78, s78, 1\n\t"  // runaway guard: at most 3 advances per job (arrival,
        "s_cmp_gt_u32 s78, s79\n\t"  // a completion that frees >= 1 job, a placed wait head)
        "s_cbranch_scc1 mcsfa_poolovf_%=\n\t"
        "s_cmp_lt_u32 s56, s40\n\t"
        "s_cbranch_scc1 mcsfa_clkovf_%=\n\t"
        "s_mov_b32 s40, s56\n\t"
        "v_cmp_ge_u32_e32 vcc, s40, v90\n\t"
        "s_cbranch_vccz mcsfa_loopend_%=\n\t"
        // release every running job with finish <= t (cluster.go:153-157)
        "s_add_u32 s84, s84, 1\n\t"
        "s_add_u32 s74, s40, 1\n\t"
        "ds_read_b64 v[72:73], v107 offset:4096+0*512\n\t"
        "ds_read_b64 v[74:75], v107 offset:4096+1*512\n\t"
        "ds_read_b64 v[76:77], v107 offset:4096+2*512\n\t"
        "ds_read_b64 v[78:79], v107 offset:4096+3*512\n\t"
        "ds_read_b64 v[80:81], v107 offset:4096+4*512\n\t"
        "ds_read_b64 v[82:83], v107 offset:4096+5*512\n\t"
        "ds_read_b64 v[84:85], v107 offset:4096+6*512\n\t"
        "ds_read_b64 v[86:87], v107 offset:4096+7*512\n\t"
        "s_not_b32 s76, s74\n\t"
        "v_mov_b32 v124, s76\n\t"
        "s_mov_b32 s75, 0\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        MCS_FA_ROW(0, "v72", "v73")
        MCS_FA_ROW(1, "v74", "v75")
        MCS_FA_ROW(2, "v76", "v77")
        MCS_FA_ROW(3, "v78", "v79")
        MCS_FA_ROW(4, "v80", "v81")
        MCS_FA_ROW(5, "v82", "v83")
        MCS_FA_ROW(6, "v84", "v85")
        MCS_FA_ROW(7, "v86", "v87")
        "s_sub_u32 s80, s80, s75\n\t"
        "ds_read_b64 v[64:65], v108 offset:0\n\t"
        "ds_read_b64 v[66:67], v108 offset:512\n\t"
        "ds_read_b64 v[68:69], v108 offset:1024\n\t"
        "ds_read_b64 v[70:71], v108 offset:1536\n\t"
        "v_add_u32 v90, s74, v124\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "s_branch mcsfa_loopend_%=\n"

        "mcsfa_deadlock_%=:\n\t"
        "s_or_b32 s44, s44, %[fdl]\n\t"
        "s_branch mcsfa_exit_%=\n"
        "mcsfa_clkovf_%=:\n\t"
        "s_or_b32 s44, s44, %[fck]\n\t"
        "s_branch mcsfa_exit_%=\n"
        "mcsfa_poolovf_%=:\n\t"
        "s_or_b32 s44, s44, %[fov]\n\t"
        "s_branch mcsfa_exit_%=\n"

        // ---- batch end: store the 64 results, take the prefetched records, prefetch the next ----
        "mcsfa_bend_%=:\n\t"
        "s_cmp_gt_u32 s81, 64*8\n\t"
        "s_cbranch_scc1 mcsfa_poolovf_%=\n\t"
        "s_add_u32 s76, s57, s47\n\t"
        "s_cmp_ge_u32 s76, s42\n\t"
        "s_cbranch_scc1 mcsfa_exit_%=\n\t"
        "s_waitcnt vmcnt(0)\n\t"
        "v_add_u32 v125, s57, v110\n\t"
        "v_lshlrev_b32 v125, 2, v125\n\t"
        "v_and_b32 v126, 63, v91\n\t"
        "v_lshrrev_b32 v127, 6, v91\n\t"
        "v_lshl_add_u32 v126, v126, 2, v127\n\t"  // node = lane * 4 + chunk
        "global_store_dword v125, v126, s[66:67] nt\n\t"
        "global_store_dword v125, v92, s[68:69] nt\n\t"
        "global_store_dword v125, v93, s[70:71] nt\n\t"
        "s_add_u32 s57, s57, 64\n\t"
        "v_mov_b32 v94, v98\n\t"
        "v_mov_b32 v95, v99\n\t"
        "v_min_u32 v96, 0x7fffffff, v100\n\t"
        "v_min_u32 v97, 0x7fffffff, v101\n\t"
        "v_add_u32 v121, s57, v110\n\t"
        "v_lshlrev_b32 v121, 4, v121\n\t"
        "v_add_u32 v121, 0x400, v121\n\t"
        "global_load_dwordx4 v[98:101], v121, s[64:65]\n\t"
        "s_sub_u32 s41, s42, s57\n\t"
        "s_min_u32 s41, s41, 64\n\t"
        "s_mov_b32 s47, 0\n\t"
        "v_readlane_b32 s45, v94, s47\n\t"
        "v_readlane_b32 s46, v95, s47\n\t"
        "v_readlane_b32 s48, v96, s47\n\t"
        "v_readlane_b32 s49, v97, s47\n\t"
        "s_branch mcsfa_inner_%=\n"

        // ---- exit: state back to the compiler's registers ----
        "mcsfa_exit_%=:\n\t"
        "s_waitcnt vmcnt(0) lgkmcnt(0)\n\t"
        "s_mov_b32 %[t], s40\n\t"
        "s_add_u32 %[r], s57, s47\n\t"
        "s_mov_b32 %[flags], s44\n\t"
        "s_mov_b32 %[hw], s43\n\t"
        "s_mov_b32 %[used], s80\n\t"
        "s_mov_b32 %[peak], s81\n\t"
        "s_mov_b32 %[waited], s82\n\t"
        "s_mov_b32 %[nslow], s83\n\t"
        "s_mov_b32 %[nrel], s84\n\t"
        "v_mov_b32 %[on], v91\n\t"
        "v_mov_b32 %[os], v92\n\t"
        "v_mov_b32 %[of], v93\n\t"
        "v_mov_b32 %[frm], v89\n\t"
        "v_mov_b32 %[lmin], v90\n\t"
        "s_nop 1"
        : [t] "+s"(t), [r] "+s"(r), [flags] "+s"(flags), [hw] "+s"(have_w), [used] "+s"(used),
          [peak] "+s"(peak), [waited] "+s"(waited), [nslow] "+s"(n_slow), [nrel] "+s"(n_rel),
          [on] "+v"(on), [os] "+v"(os), [of] "+v"(of), [frm] "+v"(frm), [lmin] "+v"(lmin)
        : [J] "s"(J), [jobs] "s"(jobs), [onp] "s"(o_node), [osp] "s"(o_start), [ofp] "s"(o_finish),
          [n0] "v"(nv[0]), [n1] "v"(nv[1]), [n2] "v"(nv[2]), [n3] "v"(nv[3]), [c0] "v"(cur.x),
          [c1] "v"(cur.y), [c2] "v"(cur.z), [c3] "v"(cur.w), [pay] "v"(v_pay), [nb] "v"(v_nb),
          [nbase] "v"(v_nbase), [lane] "v"(lane), [fdl] "i"(MCS_FLAG_DEADLOCK),
          [fck] "i"(MCS_FLAG_CLOCK_OVERFLOW), [fov] "i"(MCS_FLAG_OVERFLOW)
        : MCS_FA_CLOBBERS);
#pragma clang diagnostic pop

    if (peak > (uint32_t)(kAsmPool * kWave)) flags |= MCS_FLAG_OVERFLOW;  // a skipped insert
    const uint32_t placed = r;  // FIFO places every job it decides, in order
    if (!(flags & MCS_FLAG_OVERFLOW)) {
        if (r > 0u) {  // the batch holding the last decision (earlier ones are stored)
            const uint32_t i = ((r - 1u) & ~63u) + lane;
            if (i < r) {
                o_node[i] = (int32_t)((on & 63u) * kAsmNpl + (on >> 6));
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
        st.pool = (uint32_t)kAsmPool;
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

bool fifo_asm_eligible(const FifoArgs& a, int npl, int pool, bool hor) {
    const char* env = getenv("MCS_FIFO_ASM");
    if (env && atoi(env) == 0) return false;
    return !hor && !a.gen.on && a.guard_ok && npl <= kAsmNpl && pool <= kAsmPool;  // (a larger pool
    // than asked for changes no result)
}

hipError_t launch_fifo_asm(const FifoArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(fifo_asm_kernel, dim3(a.n_items), dim3(kWave), 0, s, a);
    return hipGetLastError();
}

}  // namespace mcs
