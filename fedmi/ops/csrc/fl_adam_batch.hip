// Adam kernel of the trial batches (fl_engine.cpp TrialBatch; BASELINE config 5): the body of
// fl_adam_kernel (fl_adam_body.inc) for K trials at once (blockIdx.y = trial), in blocks of 4
// waves instead of 16.  A packed group round is bound by workgroup slots x latency: a 1024-thread
// Adam block (92 VGPRs x 4 waves per SIMD) holds a whole CU and cannot sit beside a train
// workgroup of another trial batch, a 256-thread block can (one wave per SIMD), and 4-5 of them
// fit a CU.  Every wave runs 4 of the canonical 16 waves' slab rows, so the gradient sums -- and
// every trial's weights and history -- stay bit-identical to its standalone engine's
// (tests/test_fed_sweep.py).  At most 128 VGPRs (4 waves per SIMD): a train workgroup holds 4 waves x 96
// of the SIMD's 512.
#define ADAM_WAVES 4
#define ADAM_WDEPTH 1
#include "fl_common.h"
#include "fl_device.h"
#include "peer_device.h"
#include "fl_adam.h"

// Trial batch (no peer exchange: the trials' FedAvg is one shared collective outside).
__global__ void __launch_bounds__(ADAM_WAVES * 64) __attribute__((amdgpu_waves_per_eu(4)))
fl_adam_batch_kernel(MLPDesc d, const FLTrialDesc* __restrict__ T, FLSel pin_sel, FLSel anchor_sel, FLSel comm_sel,
                     FLSel st_sel, int local_step, MLPDescB e, int pack, FLSel st_out_sel, int fold, int tail_a,
                     int fold_mask) {
    const FLTrialDesc& t = T[blockIdx.y];
    const FLConfig c = t.c;
    const FLBuffers b = t.b;
    const float* __restrict__ pin = reinterpret_cast<const float*>(fl_sel(t, pin_sel));
    const float* __restrict__ anchor = reinterpret_cast<const float*>(fl_sel(t, anchor_sel));
    float* __restrict__ comm = reinterpret_cast<float*>(fl_sel(t, comm_sel));
    const FLState* __restrict__ st = reinterpret_cast<const FLState*>(fl_sel(t, st_sel));
    FLState* __restrict__ st_out = reinterpret_cast<FLState*>(fl_sel(t, st_out_sel));
    const PeerArgs pa = {};
    const int xchg = 0, afold = 0;
#define ADAM_PA_LL false
#include "fl_adam_body.inc"
#undef ADAM_PA_LL
}

hipError_t fl_launch_adam_batch(const MLPDesc& d, const MLPDescB* e, const FLTrialDesc* T, int K, FLSel pin,
                                FLSel anchor, FLSel comm, FLSel st, int local_step, FLSel st_out, int fold, int tail_a,
                                int fold_mask, hipStream_t s) {
    if (K < 1 || (fold && st_out.base < 0)) return hipErrorInvalidValue;
    const int blocks = (d.P + 63) / 64 + 1;
    MLPDescB ee = {};
    if (e != nullptr) ee = *e;
    hipLaunchKernelGGL(fl_adam_batch_kernel, dim3(blocks, K), dim3(ADAM_WAVES * 64), 0, s, d, T, pin, anchor, comm,
                       st, local_step, ee, e != nullptr ? 1 : 0, st_out, fold, tail_a, fold_mask);
    return hipGetLastError();
}
