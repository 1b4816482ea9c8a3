// ldsbw.hip — LDS pipe cost per instruction under full occupancy (16 waves per CU, every CU busy):
// each wave issues N LDS instructions of one kind back to back; prints CU cycles per instruction.
// Diagnostic tool only.  build: hipcc --offload-arch=gfx950 -O2 -o tools/micro/ldsbw tools/micro/ldsbw.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#define N 4096
#define R8(x) x x x x x x x x

__global__ __launch_bounds__(64) void k(unsigned long long* out, int test) {
    __shared__ unsigned long long lds[1280];
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
    const unsigned a = threadIdx.x * 8u;
    unsigned long long t0, t1;
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    if (test == 0) {
        for (int i = 0; i < N / 8; ++i)
            asm volatile(R8("ds_read2st64_b64 v[40:43], %0 offset0:1 offset1:2\n") "s_waitcnt lgkmcnt(0)" ::"v"(a) : "v40", "v41", "v42", "v43", "memory");
    } else if (test == 1) {
        for (int i = 0; i < N / 8; ++i)
            asm volatile("s_mov_b64 s[40:41], exec\n s_mov_b64 exec, 1\n" R8("ds_read2st64_b64 v[40:43], %0 offset0:1 offset1:2\n") "s_waitcnt lgkmcnt(0)\n s_mov_b64 exec, s[40:41]" ::"v"(a) : "v40", "v41", "v42", "v43", "s40", "s41", "memory");
    } else if (test == 2) {
        for (int i = 0; i < N / 8; ++i)
            asm volatile(R8("ds_read_b64 v[40:41], %0 offset:512\n") "s_waitcnt lgkmcnt(0)" ::"v"(a) : "v40", "v41", "memory");
    } else if (test == 3) {
        for (int i = 0; i < N / 8; ++i)
            asm volatile("s_mov_b64 s[40:41], exec\n s_mov_b64 exec, 1\n v_mov_b32 v40, 1\n v_mov_b32 v41, 0\n" R8("ds_write2st64_b64 %0, v[40:41], v[40:41] offset0:3 offset1:4\n") "s_waitcnt lgkmcnt(0)\n s_mov_b64 exec, s[40:41]" ::"v"(a) : "v40", "v41", "s40", "s41", "memory");
    } else if (test == 4) {
        for (int i = 0; i < N / 8; ++i)
            asm volatile("s_mov_b64 s[40:41], exec\n s_mov_b64 exec, 1\n v_mov_b32 v40, 1\n v_mov_b32 v41, 0\n" R8("ds_add_u64 %0, v[40:41] offset:1024\n") "s_waitcnt lgkmcnt(0)\n s_mov_b64 exec, s[40:41]" ::"v"(a) : "v40", "v41", "s40", "s41", "memory");
    } else if (test == 5) {
        for (int i = 0; i < N / 8; ++i)
            asm volatile("v_mov_b32 v40, 1\n v_mov_b32 v41, 0\n" R8("ds_write2st64_b64 %0, v[40:41], v[40:41] offset0:3 offset1:4\n") "s_waitcnt lgkmcnt(0)" ::"v"(a) : "v40", "v41", "memory");
    } else if (test == 6) {
        for (int i = 0; i < N / 8; ++i)
            asm volatile("v_mov_b32 v40, 1\n v_mov_b32 v41, 0\n" R8("ds_write_b64 %0, v[40:41] offset:1536\n") "s_waitcnt lgkmcnt(0)" ::"v"(a) : "v40", "v41", "memory");
    } else if (test == 7) {
        for (int i = 0; i < N / 8; ++i)
            asm volatile("v_mov_b32 v40, 1\n" R8("ds_write_b32 %0, v40 offset:1536\n") "s_waitcnt lgkmcnt(0)" ::"v"(a) : "v40", "memory");
    } else if (test == 8) {
        for (int i = 0; i < N / 8; ++i)
            asm volatile(R8("ds_read_b32 v40, %0 offset:512\n") "s_waitcnt lgkmcnt(0)" ::"v"(a) : "v40", "memory");
    } else if (test == 9) {
        const unsigned a16 = threadIdx.x * 16u;
        for (int i = 0; i < N / 8; ++i)
            asm volatile(R8("ds_read_b128 v[40:43], %0\n") "s_waitcnt lgkmcnt(0)" ::"v"(a16) : "v40", "v41", "v42", "v43", "memory");
    } else if (test == 10) {
        for (int i = 0; i < N / 8; ++i)
            asm volatile("s_mov_b64 s[40:41], exec\n s_mov_b64 exec, 1\n v_mov_b32 v40, 1\n v_mov_b32 v41, 0\n" R8("ds_write_b64 %0, v[40:41] offset:1536\n") "s_waitcnt lgkmcnt(0)\n s_mov_b64 exec, s[40:41]" ::"v"(a) : "v40", "v41", "s40", "s41", "memory");
    } else if (test == 11) {
        for (int i = 0; i < N / 8; ++i)
            asm volatile(R8("ds_read2_b32 v[40:41], %0 offset0:1 offset1:65\n") "s_waitcnt lgkmcnt(0)" ::"v"(a) : "v40", "v41", "memory");
    } else if (test == 12) {
        for (int i = 0; i < N / 8; ++i)
            asm volatile(R8("ds_read_b64 v[40:41], %0 offset:512\n") ::"v"(a) : "v40", "v41", "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    } else if (test == 13) {
        for (int i = 0; i < N / 8; ++i)
            asm volatile("v_mov_b32 v40, 1\n v_mov_b32 v41, 0\n" R8("ds_add_u64 %0, v[40:41] offset:1024\n") "s_waitcnt lgkmcnt(0)" ::"v"(a) : "v40", "v41", "memory");
    }
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    if (threadIdx.x == 0) atomicMax(&out[test], t1 - t0);
}

int main() {
    unsigned long long* d;
    unsigned long long h[16];
    hipMalloc(&d, sizeof(h));
    const char* names[] = {"read2st64_b64 64 lanes", "read2st64_b64 1 lane", "read_b64 64 lanes",
                           "write2st64_b64 1 lane", "add_u64 1 lane", "write2st64_b64 64 lanes",
                           "write_b64 64 lanes", "write_b32 64 lanes", "read_b32 64 lanes", "read_b128 64 lanes",
                           "write_b64 1 lane", "read2_b32 64 lanes", "read_b64 no per-8 wait", "add_u64 64 lanes"};
    for (int waves : {1, 16}) {
        for (int t = 0; t < 14; ++t) {
            hipMemset(d, 0, sizeof(h));
            hipLaunchKernelGGL(k, dim3(256 * waves), dim3(64), 0, 0, d, t);
            hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
            printf("waves/CU %2d  %-26s %7.2f cycles per instruction per wave (max wave)\n", waves, names[t],
                   (double)h[t] / N);
        }
    }
    return 0;
}
