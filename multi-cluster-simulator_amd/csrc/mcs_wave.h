// mcs_wave.h — wave64 helpers shared by the gfx950 kernels (DPP reductions, lane broadcast).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mcs_internal.h"

namespace mcs {

// Copies of n elements between HBM and LDS by one wave, U elements per lane per round with all
// of a round's reads issued before its writes.  The plain `for (i = lane; i < n; i += 64)
// dst[i] = src[i]` compiles to one read, one wait and one write per iteration: a serialized HBM
// (or LDS) round trip per 64 elements, which dominated the lock-step tick kernels' staging.
template <int U, typename T>
__device__ __forceinline__ void copy_rounds(T* __restrict__ dst, const T* __restrict__ src, uint32_t n,
                                            uint32_t lane) {
    for (uint32_t b = 0; b < n; b += (uint32_t)U * kWave) {
        T v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t i = b + (uint32_t)u * kWave + lane;
            v[u] = i < n ? src[i] : T{};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t i = b + (uint32_t)u * kWave + lane;
            if (i < n) dst[i] = v[u];
        }
    }
}

// lane mask of a >= b (unsigned): one v_cmp into a scalar register pair (a __ballot of a
// combined bool re-materialises the mask through a VGPR)
__device__ __forceinline__ uint64_t lanes_ge(uint32_t a, uint32_t b) {
    return __builtin_amdgcn_uicmp(a, b, 35 /* ICMP_UGE */);
}

__device__ __forceinline__ uint64_t lanes_ne(uint32_t a, uint32_t b) {
    return __builtin_amdgcn_uicmp(a, b, 33 /* ICMP_NE */);
}

// the byte offset of a __shared__ object in LDS (for inline-asm ds_* operands)
template <typename T>
__device__ __forceinline__ uint32_t lds_addr(T* p) {
    return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) T*)p;
}

// Progress-based issue priority at a batch boundary, the compiled kernels' form of the hand-scheduled
// loops' MCS_FA_PRIO (mcs_fa_macros.h): 3 while more than half of the wave's J jobs
// remain past the cursor, 2 while more than a quarter, 1 while more than an eighth, else 0.  Both
// arguments are wave-uniform; only the issue order among a SIMD's waves changes.
__device__ __forceinline__ void wave_progress_prio(uint32_t cursor, uint32_t J) {
    const uint32_t rem = cursor < J ? J - cursor : 0u;
    if (2u * rem > J) __builtin_amdgcn_s_setprio(3);
    else if (4u * rem > J) __builtin_amdgcn_s_setprio(2);
    else if (8u * rem > J) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
}

__device__ __forceinline__ uint32_t readlane(uint32_t v, uint32_t l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}

// a wave-uniform value pinned to an SGPR (an "s" asm operand may otherwise get a VGPR where the
// divergence analysis cannot prove uniformity); free when the value already lives in an SGPR
__device__ __forceinline__ uint32_t sgpr(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

// unsigned min over the wave with DPP row shifts and row broadcasts (no LDS round trip):
// rows of 16 lanes are scanned with row_shr 1/2/4/8, then row_bcast:15 / row_bcast:31 carry the
// row minima upward; lane 63 ends with the wave minimum.  Lanes with no DPP source keep `old` =
// kEmpty, the identity of min.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint32_t dpp_min_step(uint32_t v) {
    const uint32_t w =
        (uint32_t)__builtin_amdgcn_update_dpp((int)kEmpty, (int)v, CTRL, ROW_MASK, 0xf, false);
    return w < v ? w : v;
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    v = dpp_min_step<0x111, 0xf>(v);  // row_shr:1
    v = dpp_min_step<0x112, 0xf>(v);  // row_shr:2
    v = dpp_min_step<0x114, 0xf>(v);  // row_shr:4
    v = dpp_min_step<0x118, 0xf>(v);  // row_shr:8
    v = dpp_min_step<0x142, 0xa>(v);  // row_bcast:15 into rows 1 and 3
    v = dpp_min_step<0x143, 0xc>(v);  // row_bcast:31 into rows 2 and 3
    return readlane(v, 63);
}

// inclusive prefix scans over the wave with the same DPP steps (lane l ends with the lanes 0..l):
// lanes with no DPP source take `old` = 0, the identity of max and of add
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint32_t dpp_src0(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROW_MASK, 0xf, false);
}
__device__ __forceinline__ uint32_t wave_scan_max_u32(uint32_t v) {
    uint32_t w;
    w = dpp_src0<0x111, 0xf>(v); v = w > v ? w : v;
    w = dpp_src0<0x112, 0xf>(v); v = w > v ? w : v;
    w = dpp_src0<0x114, 0xf>(v); v = w > v ? w : v;
    w = dpp_src0<0x118, 0xf>(v); v = w > v ? w : v;
    w = dpp_src0<0x142, 0xa>(v); v = w > v ? w : v;
    w = dpp_src0<0x143, 0xc>(v); v = w > v ? w : v;
    return v;
}
__device__ __forceinline__ uint32_t wave_scan_or_u32(uint32_t v) {
    v |= dpp_src0<0x111, 0xf>(v);
    v |= dpp_src0<0x112, 0xf>(v);
    v |= dpp_src0<0x114, 0xf>(v);
    v |= dpp_src0<0x118, 0xf>(v);
    v |= dpp_src0<0x142, 0xa>(v);
    v |= dpp_src0<0x143, 0xc>(v);
    return v;
}
__device__ __forceinline__ uint32_t wave_scan_add_u32(uint32_t v) {
    v += dpp_src0<0x111, 0xf>(v);
    v += dpp_src0<0x112, 0xf>(v);
    v += dpp_src0<0x114, 0xf>(v);
    v += dpp_src0<0x118, 0xf>(v);
    v += dpp_src0<0x142, 0xa>(v);
    v += dpp_src0<0x143, 0xc>(v);
    return v;
}

}  // namespace mcs
