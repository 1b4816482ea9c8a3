// mcs_state.hip — the ClusterState telemetry record as a batched reduction.
//
// state_kernel rebuilds, for every cluster of the last FIFO/DELAY run and one simulated second t,
// the record the scheduler's Start stream sends (pkg/scheduler/trader_server.go:24-47):
//   cores/memory utilization = GetResourceUtilization (cluster.go:46-63) over the counters after
//   second t: sum_i (float32(Cores_i) - float32(CoresAvailable_i)) in node order, / float32(total);
//   totals = SetTotalResources (cluster.go:26-40), uint32 sums of the physical nodes.
// A job holds its node at t iff it was placed with start <= t < finish (releases precede decisions,
// D3; a zero-duration job never holds it).
//
// Layout: one 256-thread workgroup (4 waves) per cluster.  The results SoA (node, start, finish)
// is scanned with coalesced 4 B loads; only the jobs running at t load their record's cores and
// memory.  Per-node usage accumulates in LDS with u32 atomics; the float32 sum is serial in node
// order (lane 0), as Go's loop is.  HBM-bound: 12 B per job scanned plus 8 B per running job.
#include "mcs_internal.h"
#include "mcs_wave.h"

namespace mcs {

namespace {

constexpr int kStateThreads = 256;

__global__ __launch_bounds__(kStateThreads) void state_kernel(StateArgs a) {
    extern __shared__ uint32_t used[];  // [2 * max_n]: cores then memory per node
    const uint32_t c = blockIdx.x;
    const uint32_t tid = threadIdx.x;
    const uint32_t n0 = a.node_off[c], N = a.node_off[c + 1] - n0;
    for (uint32_t i = tid; i < 2u * N; i += kStateThreads) used[i] = 0u;
    __syncthreads();

    const uint64_t j0 = a.job_off[c];
    const uint32_t J = (uint32_t)(a.job_off[c + 1] - j0);
    const int32_t* __restrict__ node = a.out_node + j0;
    const uint32_t* __restrict__ start = a.out_start + j0;
    const uint32_t* __restrict__ finish = a.out_finish + j0;
    const uint4* __restrict__ jobs = a.jobs + j0;
    const uint32_t t = a.t;
    uint32_t nrun = 0;
#pragma unroll 4
    for (uint32_t i = tid; i < J; i += kStateThreads) {
        const int32_t k = __builtin_nontemporal_load(node + i);
        const uint32_t s = __builtin_nontemporal_load(start + i);
        const uint32_t f = __builtin_nontemporal_load(finish + i);
        if (k >= 0 && (uint32_t)k < N && s <= t && t < f) {
            const uint2 cm = *reinterpret_cast<const uint2*>(&jobs[i].z);
            atomicAdd(&used[k], cm.x);
            atomicAdd(&used[N + k], cm.y);
            ++nrun;
        }
    }
    // running-job count: wave sums, then one LDS add per wave
    for (int o = 32; o > 0; o >>= 1) nrun += (uint32_t)__shfl_xor((int)nrun, o);
    __shared__ uint32_t run_total;
    if (tid == 0) run_total = 0u;
    __syncthreads();
    if ((tid & 63u) == 0u) atomicAdd(&run_total, nrun);
    __syncthreads();

    if (tid == 0) {
        float cu = 0.0f, mu = 0.0f;
        uint32_t tc = 0, tm = 0;
        for (uint32_t i = 0; i < N; ++i) {
            const uint2 cap = a.cap[n0 + i];
            const uint2 fr0 = a.free0[n0 + i];
            // live counters (Go uint64; no trading here, so they never wrap)
            const uint32_t fc = fr0.x - used[i], fm = fr0.y - used[N + i];
            cu = __fadd_rn(cu, __fsub_rn((float)cap.x, (float)fc));
            mu = __fadd_rn(mu, __fsub_rn((float)cap.y, (float)fm));
            tc += cap.x;
            tm += cap.y;
        }
        mcs_cluster_state st;
        st.cores_utilization = __fdiv_rn(cu, (float)tc);
        st.memory_utilization = __fdiv_rn(mu, (float)tm);
        st.total_cpu = tc;
        st.total_memory = tm;
        st.running = run_total;
        st.t_s = t;
        a.out[c] = st;
    }
}

}  // namespace

hipError_t launch_state(const StateArgs& a, uint32_t max_n, hipStream_t s) {
    if (a.n_clusters == 0) return hipSuccess;
    hipLaunchKernelGGL(state_kernel, dim3(a.n_clusters), dim3(kStateThreads), 2 * max_n * sizeof(uint32_t), s, a);
    return hipGetLastError();
}

}  // namespace mcs
