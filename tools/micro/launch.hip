// launch.hip — the floor under a one-launch-per-tick loop: a hipGraph of N dependent launches of a
// kernel shaped like tr_rk_kernel's grid (16 workgroups x 256 threads, dynamic LDS), timed with
// events.  Variants: empty body; one load of the previous launch's store (the cross-launch round
// trip); that plus 16 KB of stores per workgroup (L2 write-back at the launch end).
// Diagnostic tool only.  build: hipcc --offload-arch=gfx950 -O2 -o tools/micro/launch tools/micro/launch.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CHK(x)                                                                    \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                             \
        }                                                                         \
    } while (0)

__global__ __launch_bounds__(256) void k_empty(unsigned* p, int n) {}

__global__ __launch_bounds__(256) void k_chain(unsigned* p, int nstore) {
    extern __shared__ unsigned lds[];
    const unsigned v = p[blockIdx.x * 256 + threadIdx.x];  // the previous launch's value
    lds[threadIdx.x] = v + 1u;
    __syncthreads();
    unsigned* q = p + 65536 + blockIdx.x * 4096;
    for (int i = threadIdx.x; i < nstore; i += 256) q[i] = lds[i & 255];
    p[blockIdx.x * 256 + threadIdx.x] = lds[threadIdx.x];
}

static int run(const char* name, int which, int nstore, size_t lds, unsigned* d, hipStream_t s) {
    const int N = 2000;
    hipGraph_t g;
    hipGraphExec_t ge;
    CHK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < N; ++i) {
        if (which == 0)
            hipLaunchKernelGGL(k_empty, dim3(16), dim3(256), lds, s, d, 0);
        else
            hipLaunchKernelGGL(k_chain, dim3(16), dim3(256), lds, s, d, nstore);
    }
    CHK(hipStreamEndCapture(s, &g));
    CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    CHK(hipGraphLaunch(ge, s));  // warm
    CHK(hipStreamSynchronize(s));
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        CHK(hipEventRecord(a, s));
        CHK(hipGraphLaunch(ge, s));
        CHK(hipEventRecord(b, s));
        CHK(hipEventSynchronize(b));
        float ms;
        CHK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
    }
    printf("{\"variant\": \"%s\", \"lds\": %zu, \"stores_per_wg\": %d, \"us_per_launch\": %.3f}\n", name, lds,
           nstore, best * 1e3 / N);
    CHK(hipGraphExecDestroy(ge));
    CHK(hipGraphDestroy(g));
    CHK(hipEventDestroy(a));
    CHK(hipEventDestroy(b));
    return 0;
}

int main() {
    unsigned* d;
    CHK(hipMalloc(&d, 16u << 20));
    CHK(hipMemset(d, 0, 16u << 20));
    hipStream_t s;
    CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CHK(hipFuncSetAttribute((const void*)k_chain, hipFuncAttributeMaxDynamicSharedMemorySize, 65536));
    CHK(hipFuncSetAttribute((const void*)k_empty, hipFuncAttributeMaxDynamicSharedMemorySize, 65536));
    if (run("empty", 0, 0, 0, d, s) || run("empty_lds16k", 0, 0, 16384, d, s) || run("chain", 1, 0, 1024, d, s) ||
        run("chain_lds16k", 1, 0, 16384, d, s) || run("chain_store16k", 1, 4096, 16384, d, s))
        return 1;
    CHK(hipFree(d));
    return 0;
}
