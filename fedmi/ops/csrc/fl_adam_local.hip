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

// The same LL-exchange body on a VIRTUAL grid: `gridDim.x` physical blocks walk the
// (P + 63) / 64 + 1 Adam blocks in block order (block b runs virtual blocks b, b + G, ...).
// Every value is the same computation as fl_adam_ll_kernel's (bit-identical); only the number
// of workgroups that spin in the exchange at once changes.  Needed where the exchanging ranks
// SHARE a GPU (tests, `bench.py --share-gpu`): each Adam block waits for its chunk from every
// rank, so all ranks' blocks of a chunk must be resident at once -- 8 ranks x 179 blocks of
// 1024 threads (reference MLP) do not fit one GPU, 8 x 16 do.  On separate GPUs (one rank per
// GPU) the full grid is always resident and this kernel is not used.  Deadlock freedom: every
// rank walks the virtual blocks in the same order with the same G, so with all G x world
// physical blocks resident, physical block b of every rank reaches virtual block v together.
__device__ __forceinline__ void fl_adam_ll_vblock(const int adam_blk, const MLPDesc& d, const FLConfig& c,
                                                  const FLBuffers& b, const float* __restrict__ pin,
                                                  const float* __restrict__ anchor, float* __restrict__ comm,
                                                  const FLState* __restrict__ st, int local_step, const MLPDescB& e,
                                                  int pack, FLState* __restrict__ st_out, int fold, int tail_a,
                                                  int fold_mask, const PeerArgs& pa, int xchg, int afold) {
#define ADAM_PA_LL true
#define ADAM_BLK adam_blk
#include "fl_adam_body.inc"
#undef ADAM_BLK
#undef ADAM_PA_LL
}

__global__ void __launch_bounds__(ADAM_WAVES * 64)
fl_adam_ll_grid_kernel(MLPDesc d, FLConfig c, FLBuffers b, const float* __restrict__ pin,
                       const float* __restrict__ anchor, float* __restrict__ comm, const FLState* __restrict__ st,
                       int local_step, MLPDescB e, int pack, FLState* __restrict__ st_out, int fold, int tail_a,
                       int fold_mask, PeerArgs pa, int xchg, int afold, int n_vblocks) {
    for (int vb = blockIdx.x; vb < n_vblocks; vb += gridDim.x) {
        fl_adam_ll_vblock(vb, d, c, b, pin, anchor, comm, st, local_step, e, pack, st_out, fold, tail_a, fold_mask,
                          pa, xchg, afold);
        __syncthreads();  // the block's LDS (partials, state) is free before the next virtual block
    }
}

// Reduce-scatter + all-gather weight chunks (FEDMI_PEER_RSAG=1, PeerArgs::rsag): the LL kernels'
// body with peer_rsag in place of the all-to-all push (bit-identical sums), full and virtual grid.
__global__ void __launch_bounds__(ADAM_WAVES * 64)
fl_adam_rsag_kernel(MLPDesc d, FLConfig c, FLBuffers b, const float* __restrict__ pin,
                    const float* __restrict__ anchor, float* __restrict__ comm, const FLState* __restrict__ st,
                    int local_step, MLPDescB e, int pack, FLState* __restrict__ st_out, int fold, int tail_a,
                    int fold_mask, PeerArgs pa, int xchg, int afold) {
#define ADAM_PA_LL true
#define ADAM_PA_RSAG true
#include "fl_adam_body.inc"
#undef ADAM_PA_RSAG
#undef ADAM_PA_LL
}

__device__ __forceinline__ void fl_adam_rsag_vblock(const int adam_blk, const MLPDesc& d, const FLConfig& c,
                                                    const FLBuffers& b, const float* __restrict__ pin,
                                                    const float* __restrict__ anchor, float* __restrict__ comm,
                                                    const FLState* __restrict__ st, int local_step,
                                                    const MLPDescB& e, int pack, FLState* __restrict__ st_out,
                                                    int fold, int tail_a, int fold_mask, const PeerArgs& pa, int xchg,
                                                    int afold) {
#define ADAM_PA_LL true
#define ADAM_PA_RSAG true
#define ADAM_BLK adam_blk
#include "fl_adam_body.inc"
#undef ADAM_BLK
#undef ADAM_PA_RSAG
#undef ADAM_PA_LL
}

__global__ void __launch_bounds__(ADAM_WAVES * 64)
fl_adam_rsag_grid_kernel(MLPDesc d, FLConfig c, FLBuffers b, const float* __restrict__ pin,
                         const float* __restrict__ anchor, float* __restrict__ comm, const FLState* __restrict__ st,
                         int local_step, MLPDescB e, int pack, FLState* __restrict__ st_out, int fold, int tail_a,
                         int fold_mask, PeerArgs pa, int xchg, int afold, int n_vblocks) {
    for (int vb = blockIdx.x; vb < n_vblocks; vb += gridDim.x) {
        fl_adam_rsag_vblock(vb, d, c, b, pin, anchor, comm, st, local_step, e, pack, st_out, fold, tail_a, fold_mask,
                            pa, xchg, afold);
        __syncthreads();
    }
}

hipError_t fl_launch_adam_ll(const MLPDesc& d, const FLConfig& c, const FLBuffers& b, const float* pin,
                             const float* anchor, float* comm, const FLState* st, int local_step, const MLPDescB& e,
                             int pack, FLState* st_out, int fold, int tail_a, int fold_mask, const PeerArgs& pa,
                             int xchg, int afold, hipStream_t s) {
    if (pa.ll == nullptr) return hipErrorInvalidValue;
    const int blocks = (d.P + 63) / 64 + 1;
    if (pa.rsag) {
        if (pa.adam_grid > 0 && pa.adam_grid < blocks)
            hipLaunchKernelGGL(fl_adam_rsag_grid_kernel, dim3(pa.adam_grid), dim3(ADAM_WAVES * 64), 0, s, d, c, b, pin,
                               anchor, comm, st, local_step, e, pack, st_out, fold, tail_a, fold_mask, pa, xchg, afold,
                               blocks);
        else
            hipLaunchKernelGGL(fl_adam_rsag_kernel, dim3(blocks), dim3(ADAM_WAVES * 64), 0, s, d, c, b, pin, anchor,
                               comm, st, local_step, e, pack, st_out, fold, tail_a, fold_mask, pa, xchg, afold);
        return hipGetLastError();
    }
    if (pa.adam_grid > 0 && pa.adam_grid < blocks) {
        hipLaunchKernelGGL(fl_adam_ll_grid_kernel, dim3(pa.adam_grid), dim3(ADAM_WAVES * 64), 0, s, d, c, b, pin,
                           anchor, comm, st, local_step, e, pack, st_out, fold, tail_a, fold_mask, pa, xchg, afold,
                           blocks);
        return hipGetLastError();
    }
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
