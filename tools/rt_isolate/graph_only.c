/* graph_only.c — rocprofv3 --runtime-trace exit-fault isolation: a hipGraph of 64
 * memset nodes captured from a stream, instantiated, replayed 10 times and destroyed, then a normal
 * exit.  No RCCL, no engine, no torch, no kernels of ours (the r06 legs showed the fault without
 * RCCL: the graph-replayed C5-DELAY bench run faults, a world-1 RCCL run of the engine does not). */
#include <hip/hip_runtime_api.h>
#include <stdio.h>

int main(void) {
    if (hipSetDevice(0) != hipSuccess) return 2;
    void* buf = NULL;
    if (hipMalloc(&buf, 1 << 16) != hipSuccess) return 3;
    hipStream_t s;
    if (hipStreamCreate(&s) != hipSuccess) return 4;
    hipGraph_t g = NULL;
    if (hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal) != hipSuccess) return 5;
    for (int i = 0; i < 64; ++i)
        if (hipMemsetAsync((char*)buf + 1024 * i, i, 1024, s) != hipSuccess) return 6;
    if (hipStreamEndCapture(s, &g) != hipSuccess) return 7;
    hipGraphExec_t ge = NULL;
    if (hipGraphInstantiate(&ge, g, NULL, NULL, 0) != hipSuccess) return 8;
    for (int k = 0; k < 10; ++k)
        if (hipGraphLaunch(ge, s) != hipSuccess) return 9;
    if (hipStreamSynchronize(s) != hipSuccess) return 10;
    (void)hipGraphExecDestroy(ge);
    (void)hipGraphDestroy(g);
    (void)hipStreamDestroy(s);
    (void)hipFree(buf);
    printf("GRAPH-ONLY OK\n");
    return 0;
}
