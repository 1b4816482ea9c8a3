/* comm_only.c — the smallest program of the rocprofv3 --runtime-trace exit-fault isolation
 * (VERDICT r05 item 6): one world-1 RCCL communicator, created, finalized and
 * destroyed, then a normal exit.  No engine, no torch, no kernels of ours.  Built by
 * tools/rt_isolate/Makefile against /opt/rocm's RCCL and HIP runtime. */
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>
#include <stdio.h>

int main(void) {
    if (hipSetDevice(0) != hipSuccess) return 2;
    ncclUniqueId id;
    ncclComm_t comm;
    if (ncclGetUniqueId(&id) != ncclSuccess) return 3;
    if (ncclCommInitRank(&comm, 1, id, 0) != ncclSuccess) return 4;
    /* one collective so the proxy and the communicator's device resources are live */
    void* buf = NULL;
    if (hipMalloc(&buf, 4096) != hipSuccess) return 5;
    hipStream_t s;
    if (hipStreamCreate(&s) != hipSuccess) return 6;
    if (ncclAllGather(buf, buf, 4096, ncclUint8, comm, s) != ncclSuccess) return 7;
    if (hipStreamSynchronize(s) != hipSuccess) return 8;
    if (ncclCommFinalize(comm) != ncclSuccess) return 9;
    if (ncclCommDestroy(comm) != ncclSuccess) return 10;
    (void)hipStreamDestroy(s);
    (void)hipFree(buf);
    printf("COMM-ONLY OK\n");
    return 0;
}
