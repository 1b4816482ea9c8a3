// mcs_trader_dev.h — Trader.ApproveTrade (pkg/trader/trader.go:141-167) as ONE device function, used
// by both lock-step trader kernels (mcs_trade.hip: the FIFO zero contract; mcs_dtrade.hip: real
// contracts) and by the mcs_approve_trade mirror that pins its float32/float64 boundaries (KAT6).
// The library is built with -ffp-contract=off and every operation is an explicit _rn intrinsic, so
// the arithmetic rounds exactly like Go on amd64 (GOAMD64=v1 emits no FMA).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mcs {

// approvePolicy{CoreUtilization 0.8, MemoryUtilization 0.8, MinCoreIncentive -1, MinMemoryIncentive -1}
// (trader.go:47-52) on the responder's sample {cu, mu} and totals {tc, tm} (SetTotalResources,
// uint32), for the contract {kc cores, km memory, ksec whole seconds, price 0}.
__device__ __forceinline__ bool approve_trade_dev(uint32_t tc, uint32_t tm, float cu, float mu, uint32_t kc,
                                                  uint32_t km, uint32_t ksec) {
    if (!(cu < 0.8f && mu < 0.8f)) return false;  // :147 (a NaN utilization denies, as in Go)
    const float ftm = (float)tm, ftc = (float)tc;
    const float avail_mem = __fsub_rn(ftm, __fmul_rn(ftm, mu));   // :148, T - (T*u)
    const float avail_core = __fsub_rn(ftc, __fmul_rn(ftc, cu));  // :149
    if (!(avail_core >= (float)kc && avail_mem >= (float)km)) return false;  // :151
    const double secs = (double)ksec;  // Duration.Seconds() of whole seconds
    const double b = __dmul_rn(__dmul_rn(-1.0, (double)kc), secs);
    const double d = __dmul_rn(__dmul_rn(-1.0, (double)km), secs);
    const double incentive = __dadd_rn(b, d);  // :154, left to right
    return 0.0 >= incentive;                   // float64(price 0) >= incentive (:155)
}

}  // namespace mcs
