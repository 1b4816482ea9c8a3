// mcs_delay_asm.hip — the DELAY policy's decision loop, hand-scheduled for gfx950.
//
// Scheduler.Delay (pkg/scheduler/scheduler.go:298-369, the reference's shipped default,
// scheduler.go:116) under SDELAY, one cluster of 129-256 nodes per wave64, on
// the W16R machinery of the FIFO loop (mcs_fa_macros.h): 16-bit node registers with guard bits,
// the first fit by v_pk_sub_u16 + SDWA + v_perm, the commit as one indexed move, the running slots
// in registers and the release with one LDS round trip.
//
// The loop is DELAY's fast path: every iteration while Level1 is empty.  One iteration at t:
//   * releases due at t (cluster.go:153-157, before anything else, D3);
//   * the Level1 pass (:302-329) has nothing to examine;
//   * the Level0 head (:332-366): placed when it fits (ScheduleJob, :335); otherwise, once it has
//     waited MaxWaitTime (:353), it would move to Level1: the loop stops there ("bail-out", flag
//     kDelayBail) and the engine re-runs that cluster from t = 0 on the compiled delay_kernel, which has
//     the Level1 list.  A cluster that bails does so at its first Level1 move;
//   * time.Sleep(1 s) (:367): t + 1 after a placement; an iteration that changes nothing
//     fast-forwards to the next release, the head's arrival or its MaxWaitTime move (exact, the
//     skipped iterations repeat the same failures).
// Same results bit for bit as delay_kernel (tests/test_gpu_delay.py, every form).
#include "mcs_internal.h"
#include "mcs_lds.h"
#include "mcs_wave.h"

namespace mcs {

namespace {

#include "mcs_fa_macros.h"


// v102/v103: per-lane 64-bit sum of (start - arrival) of the stored Level0 batches (WaitTime,
// scheduler.go:338-341, at whole seconds); v104 temp.  s56 MaxWaitTime.
#define MCS_FD_LOOP(D)                                                                            \
    /* ---- entry: state into the fixed registers ---- */                                        \
    "s_mov_b32 s40, 0\n\t"                                                                        \
    "s_mov_b32 s42, %[J]\n\t"                                                                     \
    "s_mov_b32 s44, 0\n\t"                                                                        \
    "s_mov_b32 s47, 0\n\t"                                                                        \
    "s_mov_b32 s56, %[mw]\n\t"                                                                    \
    "s_mov_b32 s57, 0\n\t"                                                                        \
    "s_mov_b32 s78, 0\n\t"                                                                        \
    "s_lshl2_add_u32 s79, s42, 0x100\n\t"                                                         \
    "s_mov_b32 s80, 0\n\t"                                                                        \
    "s_mov_b32 s81, 0\n\t"                                                                        \
    "s_mov_b32 s83, 0\n\t"                                                                        \
    "s_mov_b32 s84, 0\n\t"                                                                        \
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
    "v_mov_b32 v103, 0\n\t" MCS_FA_INIT16R MCS_FA_RELOAD16 "s_waitcnt lgkmcnt(0)\n\t"             \
    /* prefetch batch 1 */                                                                        \
    "v_lshlrev_b32 v121, 4, v110\n\t"                                                             \
    "v_add_u32 v121, 0x400, v121\n\t"                                                             \
    "global_load_dwordx4 v[98:101], v121, s[64:65]\n\t"                                           \
    "s_min_u32 s41, s42, 64\n\t" MCS_FA_REC16                                                     \
    "s_cmp_eq_u32 s42, 0\n\t" /* no jobs: no iteration (the clock stays at 0) */                 \
    "s_cbranch_scc1 mcsfd_exit_%=\n"                                                              \
                                                                                                  \
    /* ---- one iteration at t with Level1 empty: the Level0 head (scheduler.go:332-366) ---- */   \
    "mcsfd_inner_%=:\n\t" MCS_FA_CNTS_##D                                                         \
    "s_cmp_gt_u32 s45, s40\n\t" /* Level0 empty at t: the head has not arrived */                 \
    "s_cbranch_scc1 mcsfd_idle_%=\n\t" MCS_FA_FIT16 MCS_FA_ANYFIT                                 \
    "s_add_u32 s55, s40, s46\n\t"                                                                 \
    "s_cbranch_vccz mcsfd_nofit_%=\n\t"                                                           \
    "s_ff1_i32_b64 s50, vcc\n\t" /* lowest lane with a fit */                                     \
    "s_cmp_eq_u32 s46, 0\n\t"                                                                     \
    "s_cbranch_scc1 mcsfd_zero_%=\n\t" MCS_FA_DECIDE16R                                           \
    "s_min_u32 s77, s77, s55\n\t" /* the wave's earliest finish */                                \
    "s_mov_b64 exec, -1\n\t"                                                                      \
    "s_mov_b32 m0, s47\n\t"                                                                       \
    "s_add_u32 s80, s80, 1\n\t"                                                                   \
    "v_writelane_b32 v91, s54, m0\n\t"                                                            \
    "v_writelane_b32 v92, s40, m0\n"                                                              \
    "mcsfd_placed_%=:\n\t"                                                                        \
    "s_add_u32 s47, s47, 1\n\t" MCS_FA_REC16                                                      \
    "s_cmp_lt_u32 s47, s41\n\t"                                                                   \
    "s_cbranch_scc0 mcsfd_bend_%=\n"                                                              \
    /* time.Sleep(1 s) after a placement (:367) */                                                \
    "mcsfd_tick_%=:\n\t"                                                                          \
    "s_add_u32 s40, s40, 1\n\t"                                                                   \
    "s_cbranch_scc1 mcsfd_clkovf_%=\n"                                                            \
    /* the clock has advanced: releases at the new instant (cluster.go:153-157) */              \
    "mcsfd_adv_%=:\n\t"                                                                           \
    "s_cmp_lt_u32 s40, s77\n\t"                                                                   \
    "s_cbranch_scc1 mcsfd_inner_%=\n\t" MCS_FA_CNTR_##D                                           \
    "s_max_u32 s81, s81, s80\n\t" /* peak: used only grows between releases */                   \
    "s_add_u32 s74, s40, 1\n\t" MCS_FA_SCAN16R                                                    \
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
    "s_waitcnt lgkmcnt(0)\n\t"                                                                    \
    "s_branch mcsfd_inner_%=\n"                                                                   \
                                                                                                  \
    /* zero-duration job: committed and released before the next ScheduleJob (D3) */             \
    "mcsfd_zero_%=:\n\t" MCS_FA_ZEROKX                                                           \
    "v_writelane_b32 v91, s54, m0\n\t"                                                            \
    "v_writelane_b32 v92, s40, m0\n\t"                                                            \
    "s_branch mcsfd_placed_%=\n"                                                                  \
                                                                                                  \
    /* nothing changes at t (Level0 empty): the next iteration that can differ is a release or  */ \
    /* the head's arrival */                                                                      \
    "mcsfd_idle_%=:\n\t"                                                                          \
    "s_min_u32 s76, s77, s45\n\t"                                                                 \
    "s_add_u32 s40, s40, 1\n\t"                                                                   \
    "s_cbranch_scc1 mcsfd_clkovf_%=\n\t"                                                          \
    "s_max_u32 s40, s40, s76\n\t"                                                                 \
    "s_branch mcsfd_adv_%=\n"                                                                     \
                                                                                                  \
    /* the head does not fit: after MaxWaitTime it moves to Level1 (:353): the compiled kernel */  \
    /* continues from here; before, the next iteration that can differ is a release or the move */ \
    "mcsfd_nofit_%=:\n\t"                                                                         \
    "s_sub_u32 s76, s40, s45\n\t" /* t - arrival (the head has arrived) */                       \
    "s_cmp_ge_u32 s76, s56\n\t"                                                                   \
    "s_cbranch_scc1 mcsfd_bail_%=\n\t"                                                            \
    "s_add_u32 s78, s78, 1\n\t" /* runaway guard (a pool overflow: re-run on delay_kernel) */     \
    "s_cmp_gt_u32 s78, s79\n\t"                                                                   \
    "s_cbranch_scc1 mcsfd_poolovf_%=\n\t"                                                         \
    "s_add_u32 s76, s45, s56\n\t"                                                                 \
    "s_min_u32 s76, s76, s77\n\t"                                                                 \
    "s_add_u32 s40, s40, 1\n\t"                                                                   \
    "s_cbranch_scc1 mcsfd_clkovf_%=\n\t"                                                          \
    "s_max_u32 s40, s40, s76\n\t"                                                                 \
    "s_branch mcsfd_adv_%=\n"                                                                     \
                                                                                                  \
    /* bail-out: the cluster is re-run on delay_kernel (it has the Level1 list) */                \
    "mcsfd_bail_%=:\n\t"                                                                          \
    "s_or_b32 s44, s44, %[fbail]\n\t"                                                             \
    "s_branch mcsfd_exit_%=\n"                                                                    \
                                                                                                  \
    "mcsfd_clkovf_%=:\n\t"                                                                        \
    "s_mov_b32 s40, -1\n\t" /* the clock stays at the last second it reached */                   \
    "s_or_b32 s44, s44, %[fck]\n\t"                                                               \
    "s_branch mcsfd_exit_%=\n"                                                                    \
    "mcsfd_poolovf_%=:\n\t"                                                                       \
    "s_or_b32 s44, s44, %[fov]\n\t"                                                               \
    "s_branch mcsfd_exit_%=\n"                                                                    \
                                                                                                  \
    /* ---- batch end: store the 64 results and their waits, take the prefetched records ---- */ \
    "mcsfd_bend_%=:\n\t"                                                                          \
    "s_max_u32 s81, s81, s80\n\t"                                                                 \
    "s_cmp_gt_u32 s81, 64*8\n\t"                                                                  \
    "s_cbranch_scc1 mcsfd_poolovf_%=\n\t"                                                         \
    "s_add_u32 s76, s57, s47\n\t"                                                                 \
    "s_cmp_ge_u32 s76, s42\n\t"                                                                   \
    "s_cbranch_scc1 mcsfd_done_%=\n\t"                                                            \
    "s_waitcnt vmcnt(0)\n\t"                                                                      \
    "v_add_u32 v125, s57, v110\n\t"                                                               \
    "v_lshlrev_b32 v125, 2, v125\n\t" MCS_FA_NODEIDX                                              \
    "global_store_dword v125, v126, s[66:67] nt\n\t"                                              \
    "global_store_dword v125, v92, s[68:69] nt\n\t"                                               \
    "v_add_u32 v93, v92, v95\n\t" /* finish = start + the batch's duration column */            \
    "global_store_dword v125, v93, s[70:71] nt\n\t"                                               \
    "v_sub_u32 v104, v92, v94\n\t" /* start - arrival */                                         \
    "v_add_co_u32 v102, vcc, v102, v104\n\t"                                                      \
    "v_addc_co_u32 v103, vcc, 0, v103, vcc\n\t"                                                   \
    "s_add_u32 s57, s57, 64\n\t" MCS_FA_TAKE16                                                    \
    "v_add_u32 v121, s57, v110\n\t"                                                               \
    "v_lshlrev_b32 v121, 4, v121\n\t"                                                             \
    "v_add_u32 v121, 0x400, v121\n\t"                                                             \
    "global_load_dwordx4 v[98:101], v121, s[64:65]\n\t"                                           \
    "s_sub_u32 s41, s42, s57\n\t"                                                                 \
    "s_min_u32 s41, s41, 64\n\t"                                                                  \
    "s_mov_b32 s47, 0\n\t" MCS_FA_REC16                                                           \
    "s_branch mcsfd_tick_%=\n"                                                                    \
    /* every job placed: the run ends with this iteration's sleep */                             \
    "mcsfd_done_%=:\n\t"                                                                          \
    "s_add_u32 s40, s40, 1\n"                                                                     \
                                                                                                  \
    /* ---- exit: state back to the compiler's registers ---- */                                 \
    "mcsfd_exit_%=:\n\t"                                                                          \
    "s_waitcnt vmcnt(0) lgkmcnt(0)\n\t"                                                           \
    "s_mov_b32 %[t], s40\n\t"                                                                     \
    "s_add_u32 %[r], s57, s47\n\t"                                                                \
    "s_mov_b32 %[cl], s47\n\t"                                                                    \
    "s_mov_b32 %[flags], s44\n\t"                                                                 \
    "s_mov_b32 %[used], s80\n\t"                                                                  \
    "s_max_u32 %[peak], s81, s80\n\t"                                                             \
    "s_mov_b32 %[nslow], s83\n\t"                                                                 \
    "s_mov_b32 %[nrel], s84\n\t"                                                                  \
    "v_mov_b32 %[on], v91\n\t"                                                                    \
    "v_mov_b32 %[os], v92\n\t"                                                                    \
    "v_mov_b32 %[arr], v94\n\t"                                                                   \
    "v_mov_b32 %[wlo], v102\n\t"                                                                  \
    "v_mov_b32 %[whi], v103\n\t"                                                                  \
    "s_cmp_eq_u32 s47, 0\n\t"                                                                     \
    "s_cbranch_scc1 mcsfd_xf_%=\n\t"                                                              \
    "v_add_u32 v93, v92, v95\n"                                                                   \
    "mcsfd_xf_%=:\n\t"                                                                            \
    "v_mov_b32 %[of], v93\n\t"                                                                    \
    "s_nop 1"

template <bool DIAG>
__global__ __launch_bounds__(64) void delay_asm_kernel(DelayArgs a) {
    const uint32_t item = blockIdx.x;
    const uint32_t ci = a.cluster_list ? a.cluster_list[item] : item;
    const uint32_t lane = threadIdx.x;

    __shared__ uint32_t lds[4 * kWave];  // the node copy [4][64] (releases)
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
    uint32_t on = 0, os = 0, of = 0, arr = 0, wlo = 0, whi = 0;

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
#define MCS_FD_OPERANDS                                                                           \
    : [t] "=s"(t), [r] "=s"(r), [cl] "=s"(cl), [flags] "=s"(flags), [used] "=s"(used),          \
      [peak] "=s"(peak), [nslow] "=s"(n_slow), [nrel] "=s"(n_rel), [on] "=v"(on), [os] "=v"(os), \
      [of] "=v"(of), [arr] "=v"(arr), [wlo] "=v"(wlo), [whi] "=v"(whi)                           \
    : [J] "s"(J), [mw] "s"(a.max_wait_s), [jobs] "s"(jobs), [onp] "s"(o_node), [osp] "s"(o_start), \
      [ofp] "s"(o_finish), [c0] "v"(cur.x), [c1] "v"(cur.y), [c2] "v"(cur.z), [c3] "v"(cur.w),    \
      [nb] "v"(v_nb), [lane] "v"(lane), [sel0] "s"(sel0), [sel1] "s"(sel1),                      \
      [fck] "i"(MCS_FLAG_CLOCK_OVERFLOW), [fov] "i"(MCS_FLAG_OVERFLOW), [fbail] "i"(kDelayBail)        \
    : MCS_FA_CLOBBERS, "v102", "v103", "v104"
    if constexpr (DIAG) asm volatile(MCS_FD_LOOP(D1) MCS_FD_OPERANDS);
    else asm volatile(MCS_FD_LOOP(D0) MCS_FD_OPERANDS);
#undef MCS_FD_OPERANDS
#pragma clang diagnostic pop

    const bool bail = (flags & kDelayBail) != 0u;
    // WaitTime.TotalTime / 1000 over the placed Level0 jobs: the stored batches (per lane) and the
    // current batch's first cl rows (not stored yet)
    uint64_t w = (uint64_t)wlo | ((uint64_t)whi << 32);
    if (lane < cl) w += (uint64_t)(os - arr);
    for (int o = 32; o >= 1; o >>= 1) {
        const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)w, o);
        const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(w >> 32), o);
        w += (uint64_t)lo | ((uint64_t)hi << 32);
    }

    if (!(flags & MCS_FLAG_OVERFLOW)) {
        if (r > 0u) {  // the batch holding the last decision (earlier ones are stored)
            const uint32_t i = ((r - 1u) & ~63u) + lane;
            if (i < r) {
                o_node[i] = (int32_t)((on & 63u) * 4u + (on >> 6));
                o_start[i] = os;
                o_finish[i] = of;
            }
        }
        if (!bail && (flags & MCS_FLAG_CLOCK_OVERFLOW)) {
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
        st.placed = r;
        st.waited = 0u;  // (moved to Level1: none on this path)
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
            ds.moved_l1 = 0u;
            ds.placed_l1 = 0u;
            ds.peak_l1 = 0u;
            ds.l1_left = 0u;
            a.dstats[ci] = ds;
            atomicAdd(&a.totals->placed, (unsigned long long)r);
            atomicAdd(&a.totals->unplaced, (unsigned long long)(J - r));
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
