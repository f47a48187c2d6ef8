// Specialised Adam kernels, in a translation unit of their own so the general kernel's code
// generation is untouched: rounds without an in-kernel exchange (one client, or FedAvg outside
// the kernel) -- the body of fl_adam_kernel (fl_adam_body.inc) with the peer paths compiled out
// -- and rounds whose exchange uses LL chunks (below).  Fewer live
// registers (92 VGPRs / 180 SGPR spills vs 123 / 405): the one-client round 23.0 -> 22.6 us
// (tools/ab_bench.sh, profiles/ab_adam_local_r2.log).
#include "fl_common.h"
#include "fl_device.h"
#include "peer_device.h"
#include "fl_adam.h"

__global__ void __launch_bounds__(ADAM_WAVES * 64)
fl_adam_local_kernel(MLPDesc d, FLConfig c, FLBuffers b, const float* __restrict__ pin,
                     const float* __restrict__ anchor, float* __restrict__ comm, const FLState* __restrict__ st,
                     int local_step, MLPDescB e, int pack, FLState* __restrict__ st_out, int fold, int tail_a,
                     int fold_mask) {
    const PeerArgs pa = {};
    const int xchg = 0, afold = 0;
#define ADAM_PA_LL false
#include "fl_adam_body.inc"
#undef ADAM_PA_LL
}

// Rounds whose exchange runs on LL chunks (peer_device.h, the default data plane of several
// clients): the general body with the publish / wait / pull paths compiled out.
__global__ void __launch_bounds__(ADAM_WAVES * 64)
fl_adam_ll_kernel(MLPDesc d, FLConfig c, FLBuffers b, const float* __restrict__ pin,
                  const float* __restrict__ anchor, float* __restrict__ comm, const FLState* __restrict__ st,
                  int local_step, MLPDescB e, int pack, FLState* __restrict__ st_out, int fold, int tail_a,
                  int fold_mask, PeerArgs pa, int xchg, int afold) {
#define ADAM_PA_LL true
#include "fl_adam_body.inc"
#undef ADAM_PA_LL
}

hipError_t fl_launch_adam_ll(const MLPDesc& d, const FLConfig& c, const FLBuffers& b, const float* pin,
                             const float* anchor, float* comm, const FLState* st, int local_step, const MLPDescB& e,
                             int pack, FLState* st_out, int fold, int tail_a, int fold_mask, const PeerArgs& pa,
                             int xchg, int afold, hipStream_t s) {
    if (pa.ll == nullptr) return hipErrorInvalidValue;
    const int blocks = (d.P + 63) / 64 + 1;
    hipLaunchKernelGGL(fl_adam_ll_kernel, dim3(blocks), dim3(ADAM_WAVES * 64), 0, s, d, c, b, pin, anchor, comm, st,
                       local_step, e, pack, st_out, fold, tail_a, fold_mask, pa, xchg, afold);
    return hipGetLastError();
}

hipError_t fl_launch_adam_local(const MLPDesc& d, const FLConfig& c, const FLBuffers& b, const float* pin,
                                const float* anchor, float* comm, const FLState* st, int local_step,
                                const MLPDescB& e, int pack, FLState* st_out, int fold, int tail_a, int fold_mask,
                                hipStream_t s) {
    const int blocks = (d.P + 63) / 64 + 1;
    hipLaunchKernelGGL(fl_adam_local_kernel, dim3(blocks), dim3(ADAM_WAVES * 64), 0, s, d, c, b, pin, anchor, comm, st,
                       local_step, e, pack, st_out, fold, tail_a, fold_mask);
    return hipGetLastError();
}
