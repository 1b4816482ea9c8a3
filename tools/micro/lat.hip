// lat.hip — latency/issue microbenchmarks of the instruction patterns in fifo_kernel's pass loop
// (one wave64 on one SIMD; s_memtime around N iterations of an asm body).  Diagnostic tool only.
//   build: hipcc --offload-arch=gfx950 -O2 -o tools/micro/lat tools/micro/lat.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#define N_IT 2000
#define REP4(x) x x x x
#define REP8(x) REP4(x) REP4(x)

#define BODY(name, setup, body)                                                          \
    if (test == id) {                                                                     \
        unsigned long long t0, t1;                                                        \
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory"); \
        asm volatile(setup "s_mov_b32 s90, 2000\n"                                        \
                     "1:\n" body "9:\n s_sub_u32 s90, s90, 1\n\ts_cmp_lg_u32 s90, 0\n\ts_cbranch_scc1 1b\n" \
                     ::: "s90", "s91", "s92", "s93", "s94", "s95", "s96", "s97", "v40", "v41", \
                     "v42", "v43", "v44", "v45", "vcc", "m0", "scc", "memory");           \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");      \
        if (threadIdx.x == 0) { out[id] = t1 - t0; }                                      \
    }                                                                                     \
    ++id;

__global__ void lat(unsigned long long* out, int test) {
    __shared__ unsigned long long lds[512];
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
    int id = 0;
    BODY("loop", "", "")
    BODY("salu_indep8", "", REP8("s_add_u32 s91, s92, 1\n"))
    BODY("salu_dep8", "", REP8("s_add_u32 s91, s91, 1\n"))
    BODY("valu_indep8", "", REP8("v_add_u32 v41, v42, 1\n"))
    BODY("valu_dep8", "", REP8("v_add_u32 v41, v41, 1\n"))
    BODY("vcmp_sand_cnd x4", "v_mov_b32 v41, 5\n",
         REP4("v_cmp_le_u32 s[92:93], 3, v41\n s_and_b64 s[94:95], s[92:93], exec\n v_cndmask_b32 v41, 7, v41, s[94:95]\n"))
    BODY("vcmp_sand x4 (to salu)", "v_mov_b32 v41, 5\n s_mov_b64 s[94:95], -1\n",
         REP4("v_cmp_le_u32 s[92:93], 3, v41\n s_and_b64 s[94:95], s[92:93], s[94:95]\n"))
    BODY("readlane->salu x4", "v_mov_b32 v41, 1\n s_mov_b32 s92, 0\n",
         REP4("v_readlane_b32 s92, v41, s92\n s_add_u32 s92, s92, 0\n"))
    BODY("readlane indep x4", "v_mov_b32 v41, 1\n s_mov_b32 s92, 0\n",
         REP4("v_readlane_b32 s93, v41, s92\n"))
    BODY("salu->valu x4", "s_mov_b32 s92, 1\n",
         REP4("s_add_u32 s92, s92, 1\n v_add_u32 v41, s92, v41\n"))
    BODY("s_branch taken x4", "",
         "s_branch 2f\n2:\n s_branch 3f\n3:\n s_branch 4f\n4:\n s_branch 5f\n5:\n")
    BODY("s_cbranch not taken x4 (+1 salu)", "",
         "s_cmp_eq_u32 0, 1\n" REP4("s_cbranch_scc1 9f\n") )
    BODY("s_cbranch taken x4", "s_cmp_eq_u32 0, 0\n",
         "s_cbranch_scc1 2f\n2:\n s_cbranch_scc1 3f\n3:\n s_cbranch_scc1 4f\n4:\n s_cbranch_scc1 5f\n5:\n")
    BODY("vcmp->cbranch_vccz x4", "v_mov_b32 v41, 5\n",
         REP4("v_cmp_le_u32 vcc, 3, v41\n s_cbranch_vccz 9f\n"))
    BODY("ds_read+wait x4 (dep)", "v_mov_b32 v41, 0\n",
         REP4("ds_read_b32 v41, v41\n s_waitcnt lgkmcnt(0)\n"))
    BODY("ds_write+wait x4", "v_mbcnt_lo_u32_b32 v41, -1, 0\n v_mbcnt_hi_u32_b32 v41, -1, v41\n v_lshlrev_b32 v41, 3, v41\n",
         REP4("ds_write_b64 v41, v[42:43]\n s_waitcnt lgkmcnt(0)\n"))
    BODY("ds_add_u64+read+wait x4", "v_mbcnt_lo_u32_b32 v41, -1, 0\n v_mbcnt_hi_u32_b32 v41, -1, v41\n v_lshlrev_b32 v41, 3, v41\n",
         REP4("ds_add_u64 v41, v[42:43]\n ds_read_b64 v[44:45], v41\n s_waitcnt lgkmcnt(0)\n"))
    BODY("writelane m0 x4", "s_mov_b32 s92, 3\n",
         REP4("s_mov_b32 m0, s92\n s_nop 0\n v_writelane_b32 v41, s92, m0\n"))
    BODY("ff1 chain x4", "s_mov_b64 s[92:93], 8\n",
         REP4("s_ff1_i32_b64 s94, s[92:93]\n s_lshl_b64 s[92:93], 8, s94\n"))
    BODY("saveexec pattern x4", "v_mov_b32 v41, 0\n",
         REP4("v_cmp_eq_u32 vcc, 0, v41\n s_and_saveexec_b64 s[92:93], vcc\n v_add_u32 v42, 1, v42\n s_or_b64 exec, exec, s[92:93]\n"))
    BODY("dpp min chain (6)", "",
         "v_min_u32_dpp v41, v41, v41 row_shr:1 row_mask:0xf bank_mask:0xf\n s_nop 1\n"
         "v_min_u32_dpp v41, v41, v41 row_shr:2 row_mask:0xf bank_mask:0xf\n s_nop 1\n"
         "v_min_u32_dpp v41, v41, v41 row_shr:4 row_mask:0xf bank_mask:0xf\n s_nop 1\n"
         "v_min_u32_dpp v41, v41, v41 row_shr:8 row_mask:0xf bank_mask:0xf\n s_nop 1\n"
         "v_min_u32_dpp v41, v41, v41 row_bcast:15 row_mask:0xa bank_mask:0xf\n s_nop 1\n"
         "v_min_u32_dpp v41, v41, v41 row_bcast:31 row_mask:0xc bank_mask:0xf\n s_nop 0\n"
         "v_readlane_b32 s92, v41, 63\n s_add_u32 s92, s92, 0\n")
    BODY("global_load+wait (L2)", "v_mov_b32 v41, 0\n v_mov_b32 v42, 0\n",
         "")
}

int main() {
    unsigned long long* d;
    unsigned long long h[64] = {};
    hipMalloc(&d, sizeof(h));
    const char* names[] = {"loop", "salu_indep8", "salu_dep8", "valu_indep8", "valu_dep8", "vcmp_sand_cnd x4",
                           "vcmp_sand x4", "readlane->salu x4", "readlane indep x4", "salu->valu x4",
                           "s_branch taken x4", "s_cbranch not taken x4", "s_cbranch taken x4",
                           "vcmp->cbranch_vccz x4", "ds_read+wait x4 (dep)", "ds_write+wait x4",
                           "ds_add_u64+read+wait x4", "writelane m0 x4", "ff1 chain x4", "saveexec pattern x4",
                           "dpp min chain (6)", "nothing"};
    const int n = 22;
    for (int rep = 0; rep < 2; ++rep)
        for (int t = 0; t < n; ++t) {
            hipMemset(d, 0, sizeof(h));
            hipLaunchKernelGGL(lat, dim3(1), dim3(64), 0, 0, d, t);
            hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
            if (rep == 1) printf("%-28s %8.2f cyc/iter\n", names[t], (double)h[t] / N_IT);
        }
    return 0;
}
