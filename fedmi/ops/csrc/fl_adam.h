// Adam-kernel helpers shared by the translation units that instantiate the Adam body
// (fl_adam_body.inc): fl_kernels.hip (general kernel with the in-kernel xGMI exchange, trial
// batches) and fl_adam_local.hip (rounds without an in-kernel exchange).
#pragma once
#include "fl_common.h"
#include "fl_device.h"

// Slab reduction + Adam + StepLR + FedAvg pre-scale.  Block = 16 waves x 64 DENSE
// parameters: wave w sums slab rows w, w+16, ... of its 64 columns with 16 rows in flight
// per lane (one 4-byte load per row would leave ~1 KB in flight per wave: latency bound);
// the 16 partials are combined in a fixed order (deterministic), then wave 0 applies Adam
// and writes the result at the parameter's image position.  Image padding is never
// written (it stays 0 in every buffer).  The last block writes this rank's metric tail.
#ifndef ADAM_WAVES
#define ADAM_WAVES 16
#endif
// the canonical wave count of the reduction order (fl_adam_body.inc): blocks of ADAM_WAVES < 16
// waves emulate 16 / ADAM_WAVES canonical waves each and give bit-identical sums
#define ADAM_CANON 16
static_assert(ADAM_CANON % ADAM_WAVES == 0, "ADAM_WAVES must divide 16");
#ifndef ADAM_DEPTH
#define ADAM_DEPTH 16
#endif
// 16-byte slab loads in flight per lane (fl_adam_body.inc): 2 x 16 waves x 8 rows = 256 fp16 slab
// rows (the 8000-row shard's 250 workgroups) in ONE round of loads
#ifndef ADAM_WDEPTH
#define ADAM_WDEPTH 2
#endif
typedef _Float16 fl_half8 __attribute__((ext_vector_type(8)));
#ifdef FL_SLAB_AUX
// A/B builds: a 16-byte slab load with the cache-policy bits FL_SLAB_AUX (fl_adam_body.inc)
template <typename VT>
__device__ __forceinline__ VT fl_slab_ld_aux(const float* slab, const VT* p) {
    // uniform resource (the slab base), per-lane byte offset
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(slab), (short)0, 0x7fffffff, 0x00020000);
    const int off = (int)(reinterpret_cast<const char*>(p) - reinterpret_cast<const char*>(slab));
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, FL_SLAB_AUX);
    VT out;
    __builtin_memcpy(&out, &v, 16);
    return out;
}
#endif
typedef float fl_float4v __attribute__((ext_vector_type(4)));
// bf16 mode: parameter -> packed LDS-layout image(s).  A weight is stored as its bf16 hi part
// and, `wlo_delta` bytes further, its lo part bf16(p - hi) (split-bf16 forward, fl_common.h);
// a bias stays fp32.
#ifdef FL_PACK_SC1  // (A/B builds: the packed image written through)
template <typename T>
__device__ __forceinline__ void pk_st(T* p, T v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
#else
template <typename T>
__device__ __forceinline__ void pk_st(T* p, T v) { *p = v; }
#endif
__device__ __forceinline__ void pack_store(char* img, int pk, bool is_bias, int wlo_delta, float p) {
    if (is_bias) {
        pk_st(reinterpret_cast<float*>(img + pk), p);
        return;
    }
    const uint32_t u = __float_as_uint(p);
    const uint32_t h = (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
    const uint32_t r = __float_as_uint(p - __uint_as_float(h << 16));
    pk_st(reinterpret_cast<uint16_t*>(img + pk), (uint16_t)h);
    pk_st(reinterpret_cast<uint16_t*>(img + pk + wlo_delta), (uint16_t)((r + 0x7fffu + ((r >> 16) & 1u)) >> 16));
}

// Adam step of one parameter (wave 0 lane of fl_adam_kernel) from the block's partial sums.
// `p`, `m`, `v`, `anc`: the parameter, its Adam moments and its anchor value, loaded by the
// caller at the start of the kernel (their latency hides behind the slab loads).  Returns the
// FedAvg contribution p * scale (also stored into `comm` on the last local step).
__device__ __forceinline__ float adam_update(const FLConfig& c, const FLBuffers& b, float* __restrict__ comm,
                                            const FLState& S, int local_step, int last_local_step, int pack, int j,
                                            int pk, bool is_bias, int wlo_delta, float (*part)[64], int lane, float p,
                                            float m, float v, float anc, float scale) {
    if (b.undo != nullptr && local_step == 0) {
        // a late fold may discard this round: keep the parameter's pre-round state (FLBuffers::undo)
        b.undo[j] = p;
        b.undo[c.tail_off + j] = m;
        b.undo[2 * c.tail_off + j] = v;
        if (pack) pack_store(reinterpret_cast<char*>(b.undo + 3 * c.tail_off), pk, is_bias, wlo_delta, p);
    }
    // `scale`: this round's FedAvg weight (rtab); 0 = the client is not sampled this round: no
    // update, its local model stays the round's input (global) model and it contributes nothing
    if (scale != 0.f) {
        float g = 0.f;
#pragma unroll
        for (int w = 0; w < ADAM_CANON; ++w) g += part[w][lane];
        if (c.slab_f16) g *= c.inv_n;  // fp16 slab: partial sums of the unscaled gradient
        if (c.weight_decay != 0.f) g += c.weight_decay * p;
        if (c.prox_mu != 0.f) g += c.prox_mu * (p - anc);
        // torch.optim.Adam single-tensor path: scalars in double, rounded to fp32 once;
        // exp_avg.lerp_(g, 1-b1); exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2);
        // p.addcdiv_(m, sqrt(v)/sqrt(bc2) + eps, -lr/bc1).  StepLR steps once per round.
        const int t = S.cur_round * c.local_steps + local_step + 1;
        const float step_size = b.sched[2 * (t - 1)];
        const float bc2_sqrt = b.sched[2 * (t - 1) + 1];
        m = m + c.omb1 * (g - m);
        v = v * c.beta2f + c.omb2 * g * g;
        const float denom = sqrtf(v) / bc2_sqrt + c.eps;
        p = p + (-step_size) * (m / denom);
        b.m[j] = m;
        b.v[j] = v;
    }
    b.local[j] = p;
    if (pack) pack_store(b.pk_local, pk, is_bias, wlo_delta, p);
    if (last_local_step) comm[j] = p * scale;
    return p * scale;
}

// A late fold found that the round before this one ran past the stop (FLState::late): put the
// parameter's local value, Adam moments and packed local image back to their pre-round state.
__device__ __forceinline__ void undo_restore(const FLConfig& c, const FLBuffers& b, int pack, int j, int pk,
                                             bool is_bias, int wlo_delta) {
    const float p = b.undo[j];
    b.local[j] = p;
    b.m[j] = b.undo[c.tail_off + j];
    b.v[j] = b.undo[2 * c.tail_off + j];
    if (pack) pack_store(b.pk_local, pk, is_bias, wlo_delta, p);
}

// Chunk ids of the Adam-fused exchange (peer_device.h): the final metric tails, the early lag
// region A (in-kernel fold of a lagged predecessor), then one per block of 64 parameters.
#define ADAM_CHUNK_TAIL 0
#define ADAM_CHUNK_LAG 1
#define ADAM_CHUNK_W0 2
