// mcs_lds.h — single-address LDS access helpers shared by the placement kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mcs {

// LDS costs on gfx950 (tools/micro/ldsbw.hip, 16 waves per CU): the LDS pipe spends about 2 CU
// cycles on a ds_read_b64 or _b32, 4 on a read2 / read_b128, 8 on a read2st64_b64, 6 on a
// ds_write_b64 or ds_add_u64 and 13.5 on a write2st64_b64 — per instruction, whatever the number
// of active lanes.  At 16 cluster waves per CU the LDS pipe is the shared resource, so every LDS
// access below is a single-address b64 instruction (LLVM would pair neighbouring loads into
// read2st64, so they are written in asm).
//
// nvr[c] = nodes[c * 64 + lane] for every chunk, and one wait, in one asm statement (LLVM then
// tracks no LDS load of its own, and no copy of a register still being loaded can slip between
// the reads and the wait; base = this lane's byte address of chunk 0)
#define MCS_R1(i) "ds_read_b64 %" #i ", %[b] offset:" #i "*512\n\t"
#define MCS_R4(i0, i1, i2, i3) MCS_R1(i0) MCS_R1(i1) MCS_R1(i2) MCS_R1(i3)
#define MCS_O4(a, i) "=&v"(a[i]), "=&v"(a[i + 1]), "=&v"(a[i + 2]), "=&v"(a[i + 3])
template <int NPL>
__device__ __forceinline__ void reload_nodes(uint64_t (&nvr)[NPL], uint32_t base) {
    if constexpr (NPL == 1) {
        asm volatile(MCS_R1(0) "s_waitcnt lgkmcnt(0)" : "=&v"(nvr[0]) : [b] "v"(base) : "memory");
    } else if constexpr (NPL == 2) {
        asm volatile(MCS_R1(0) MCS_R1(1) "s_waitcnt lgkmcnt(0)" : "=&v"(nvr[0]), "=&v"(nvr[1]) : [b] "v"(base) : "memory");
    } else if constexpr (NPL == 4) {
        asm volatile(MCS_R4(0, 1, 2, 3) "s_waitcnt lgkmcnt(0)" : MCS_O4(nvr, 0) : [b] "v"(base) : "memory");
    } else if constexpr (NPL == 8) {
        asm volatile(MCS_R4(0, 1, 2, 3) MCS_R4(4, 5, 6, 7) "s_waitcnt lgkmcnt(0)"
                     : MCS_O4(nvr, 0), MCS_O4(nvr, 4) : [b] "v"(base) : "memory");
    } else {
        static_assert(NPL == 16, "chunks per lane");
        asm volatile(MCS_R4(0, 1, 2, 3) MCS_R4(4, 5, 6, 7) MCS_R4(8, 9, 10, 11) MCS_R4(12, 13, 14, 15)
                     "s_waitcnt lgkmcnt(0)"
                     : MCS_O4(nvr, 0), MCS_O4(nvr, 4), MCS_O4(nvr, 8), MCS_O4(nvr, 12) : [b] "v"(base) : "memory");
    }
}

// nf[p] = row p of the {node | finish << 32} slot words (base: this lane's address of row 0),
// 16 rows per asm statement with its wait
template <int P>
__device__ __forceinline__ void read_finish_rows(uint64_t (&nf)[P], uint32_t base) {
    if constexpr (P == 2) {
        asm volatile(MCS_R1(0) MCS_R1(1) "s_waitcnt lgkmcnt(0)" : "=&v"(nf[0]), "=&v"(nf[1]) : [b] "v"(base) : "memory");
    } else if constexpr (P == 4) {
        asm volatile(MCS_R4(0, 1, 2, 3) "s_waitcnt lgkmcnt(0)" : MCS_O4(nf, 0) : [b] "v"(base) : "memory");
    } else if constexpr (P == 8) {
        asm volatile(MCS_R4(0, 1, 2, 3) MCS_R4(4, 5, 6, 7) "s_waitcnt lgkmcnt(0)"
                     : MCS_O4(nf, 0), MCS_O4(nf, 4) : [b] "v"(base) : "memory");
    } else {
        static_assert(P % 16 == 0, "slot rows");
#pragma unroll
        for (int h = 0; h < P; h += 16) {
            uint64_t* q = nf + h;
            asm volatile(MCS_R4(0, 1, 2, 3) MCS_R4(4, 5, 6, 7) MCS_R4(8, 9, 10, 11) MCS_R4(12, 13, 14, 15)
                         "s_waitcnt lgkmcnt(0)"
                         : "=&v"(q[0]), "=&v"(q[1]), "=&v"(q[2]), "=&v"(q[3]), "=&v"(q[4]), "=&v"(q[5]),
                           "=&v"(q[6]), "=&v"(q[7]), "=&v"(q[8]), "=&v"(q[9]), "=&v"(q[10]), "=&v"(q[11]),
                           "=&v"(q[12]), "=&v"(q[13]), "=&v"(q[14]), "=&v"(q[15])
                         : [b] "v"(base + (uint32_t)h * 512u)
                         : "memory");
        }
    }
}
#undef MCS_R1
#undef MCS_R4
#undef MCS_O4

}  // namespace mcs
