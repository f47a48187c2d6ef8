// Device side of the one-shot xGMI peer all-reduce (peer_allreduce.hip): control block,
// kernel arguments and the publish / wait / pull-reduce building blocks.  Shared by the
// standalone all-reduce kernel and the fused "local evaluation + FedAvg" kernels of the round
// engine (fl_kernels.hip, fl_kernels_bf16.hip), which overlap the weight all-reduce with the
// evaluation of the post-step local model.
//
// A call reduces [0, n) = [weights | metric tails].  Every rank publishes the two parts with
// separate monotonic flags, so the weights can be pulled while the tails are still being
// computed:
//   * flags[j]  = last call whose WEIGHTS rank j has published to this rank;
//   * tflags[j] = last call whose TAILS rank j has published (the standalone kernel publishes
//     both at once; the fused kernel publishes tflags when its last evaluation block is done).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fl_common.h"

#define PEER_MAX_WORLD 8  // one node: every GPU has a direct xGMI link to each of its 7 peers


// Optional epilogue of the reduction: also write the reduced fp32 parameter image as the
// packed bf16 LDS image the bf16 train kernel stages (fl_kernels_bf16.hip, MLPDescB), so the
// separate pack kernel after FedAvg disappears.  Offsets are in float4 units of the fp32
// image (fl_common.h layout) and bytes of the packed region.
struct PeerPack {
    char* pk;                       // packed region (nullptr: no packing)
    int wlo_delta;                  // split-bf16: lo image of W_l at pk_w[l] + wlo_delta (MLPDescB)
    int L;
    int img4_w[FL_MAX_LAYERS];      // first float4 of W_l in the image
    int img4_b[FL_MAX_LAYERS];      // first float4 of b_l
    int img4_end[FL_MAX_LAYERS];    // one past the last float4 of b_l
    int ldw4[FL_MAX_LAYERS];        // float4s per image row of W_l
    int k4[FL_MAX_LAYERS];          // packed float4 columns per row: roundup16(K_l) / 4
    int pk_w[FL_MAX_LAYERS];        // byte offset of W_l in the packed region
    int pk_lda[FL_MAX_LAYERS];      // packed W row stride (bf16 elements, MLPDescB::ldw)
    int pk_wgap, pk_wxor;           // packed W row gaps / chunk swizzle (fl_common.h)
    int pk_b[FL_MAX_LAYERS];        // byte offset of b_l in the packed region
};


struct PeerCtl {
    unsigned flags[PEER_MAX_WORLD];   // weights published, per source rank
    unsigned tflags[PEER_MAX_WORLD];  // tails published, per source rank
    unsigned seq;                     // calls this rank has completed
    unsigned done;                    // blocks of the running call that have finished
    unsigned err;                     // sticky failure word (PEER_ERR_*), 0 = healthy
    unsigned pad[64 - 2 * PEER_MAX_WORLD - 3];
};
static_assert(sizeof(PeerCtl) == 256, "PeerCtl is one 256-byte block");

// The sticky failure word PeerCtl::err = (kind << 16) | (reporting rank << 8) | missing rank.
// A failure is written into EVERY rank's word (PeerArgs::err_dst), so the whole job drains in
// one timeout: each later wait of every rank sees the word and returns instead of waiting its
// own full timeout (the reference's contract is "any failure -> comm.Abort()",
// FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py:129,203-205).
#define PEER_ERR_TIMEOUT 1u        // a wait of the reporting rank timed out on `missing`
#define PEER_ERR_ABORT 2u          // the reporting rank's host aborted the job (Comm.Abort / watchdog)
#define PEER_MISSING_EVAL 0xfeu    // missing: one of the reporting rank's own evaluation blocks
#define PEER_MISSING_NONE 0xffu
// Waits look at the failure words only once they have waited this long (100 MHz ticks: 20 us).
// A healthy round's waits end sooner, so the polling loop of the fast path is unchanged.
#define PEER_SLOW_TICKS 2000

struct PeerArgs {
    const float* src[PEER_MAX_WORLD];    // every rank's send buffer of this parity (mapped)
    unsigned* flag_dst[PEER_MAX_WORLD];  // &ctl_j->flags[rank]
    unsigned* tflag_dst[PEER_MAX_WORLD]; // &ctl_j->tflags[rank]
    PeerCtl* ctl;                        // this rank's control block
    float* out;
    long long n;                         // floats in the call
    long long n_w;                       // floats of the weights part (multiple of 4); tails = [n_w, n)
    long long timeout;                   // s_memrealtime ticks
    unsigned* eflags;                    // fused calls: per evaluation block, last call it finished
    int n_eval;                          // evaluation blocks of a fused call
    int world;
    int uc;                              // send buffers are uncached memory (see peer_flag_store)
    // Adam-fused exchange (chunked flags, call index = FLState::calls): chunk k of call t
    // published by rank j  <=>  cflags_j... row of rank j in MY chunk-flag table >= t
    unsigned* cflag_dst[PEER_MAX_WORLD]; // &chunk_flags_j[rank * n_chunks]: my row in rank j's table
    unsigned* cflags;                    // my table: [world][n_chunks]
    int n_chunks;
    int rank;
    // Low-latency (LL) weight chunks of the Adam-fused exchange: 8-byte slots {value, call index}
    // in a ring [2 parities][PEER_MAX_WORLD source ranks][n_chunks * 64] in every rank's
    // allocation.  nullptr: the chunks go through the publish / wait / pull protocol.
    unsigned long long* ll_dst[PEER_MAX_WORLD];  // rank j's ring (mapped)
    unsigned long long* ll;                      // my ring
    // > 0: the LL Adam kernel runs on this many workgroups, each walking several Adam blocks
    // (fl_adam_local.hip fl_adam_ll_grid_kernel) -- for ranks that share one GPU
    int adam_grid;
    // Fail-fast: every rank's failure word (mapped; [rank] = &ctl->err) and this rank's host
    // abort word (pinned host memory, written by PeerAllReduce::abort; nullptr: none)
    unsigned* err_dst[PEER_MAX_WORLD];
    const unsigned* host_abort;
    // 1: the Adam-fused weight chunks go through reduce-scatter + all-gather on the LL ring
    // (peer_rsag below) instead of every rank pushing every value to every rank
    int rsag;
};

// All-reduce blocks of a fused evaluation + FedAvg kernel (FL_THREADS = 512 threads each):
// one float4 of the weights per thread, at most 32 blocks.
static inline int fl_fedavg_blocks(long long n_w) {
    const long long n4 = n_w >> 2;
    const long long nb = (n4 + 511) / 512;
    return (int)(nb < 1 ? 1 : (nb > 32 ? 32 : nb));
}

__device__ __forceinline__ uint32_t peer_bf16_rne(float x) {
    const uint32_t u = __float_as_uint(x);
    return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}

// System-coherent (sc0 sc1: aux 17) buffer loads: they bypass this GPU's L1 and L2, so a
// peer's buffer is read from its memory as published, with no stale local copy.
__device__ __forceinline__ float4 peer_load16(const float* base, int bytes, int off) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, bytes,
                                                                         0x00020000);
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 17);
    return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
}
__device__ __forceinline__ float peer_load4(const float* base, int bytes, int off) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, bytes,
                                                                         0x00020000);
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 17));
}

// Image float4 i (fp32 parameter image) -> packed bf16 LDS image (PeerPack).
__device__ __forceinline__ void peer_pack_store(const PeerPack& p, int i, float4 s) {
#pragma unroll
    for (int l = 0; l < FL_MAX_LAYERS; ++l) {
        if (l >= p.L || i < p.img4_w[l] || i >= p.img4_end[l]) continue;
        if (i < p.img4_b[l]) {
            const int q = i - p.img4_w[l];
            const int n = q / p.ldw4[l], c4s = q - n * p.ldw4[l];
            if (c4s < p.k4[l]) {  // columns [roundup16(K), ldw) are the image's zero pad
                const int c4 = c4s ^ (fl_swz(n) >> 2);  // logical chunk (swizzled image, fl_common.h)
                const uint32_t hx = peer_bf16_rne(s.x), hy = peer_bf16_rne(s.y), hz = peer_bf16_rne(s.z),
                               hw = peer_bf16_rne(s.w);
                char* dst = p.pk + p.pk_w[l] + fl_wrow(n, p.pk_lda[l], p.pk_wgap) + 16 * ((c4 >> 1) ^ fl_wswz(n, p.pk_wxor)) +
                            8 * (c4 & 1);
                *reinterpret_cast<uint2*>(dst) = make_uint2(hx | (hy << 16), hz | (hw << 16));
                // lo parts: bf16(x - hi) (split-bf16 forward, fl_common.h)
                *reinterpret_cast<uint2*>(dst + p.wlo_delta) =
                    make_uint2(peer_bf16_rne(s.x - __uint_as_float(hx << 16)) |
                                   (peer_bf16_rne(s.y - __uint_as_float(hy << 16)) << 16),
                               peer_bf16_rne(s.z - __uint_as_float(hz << 16)) |
                                   (peer_bf16_rne(s.w - __uint_as_float(hw << 16)) << 16));
            }
        } else {
            *reinterpret_cast<float4*>(p.pk + p.pk_b[l] + (i - p.img4_b[l]) * 16) = s;
        }
    }
}

// The call this kernel performs: one more than the calls completed (written by the last
// block of the previous call, which finished before this kernel started).
__device__ __forceinline__ unsigned peer_target(const PeerArgs& a) {
    __shared__ unsigned target_s;
    if (threadIdx.x == 0) target_s = __hip_atomic_load(&a.ctl->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    __syncthreads();
    return target_s;
}

// Lanes 0..world-1: store `target` into every rank's flag slot for this rank.
__device__ __forceinline__ void peer_flag_store(unsigned* dst, unsigned v, int uc);
__device__ __forceinline__ void peer_publish(unsigned* const* dst, int world, unsigned target, int uc) {
    if (threadIdx.x < (unsigned)world) peer_flag_store(dst[threadIdx.x], target, uc);
}

// Memory ordering of the protocol (publisher on GPU j, reader on GPU i):
//   publisher: data stores (uncached send buffer) -> RELEASE store of the flag at system scope
//              (the release waits for every earlier store of the wave to be acknowledged and
//              writes back this GPU's dirty L2 lines), so the data is in j's memory before
//              the flag can be seen over xGMI;
//   reader:    relaxed polling of the flag (cheap loop), then ONE system-scope ACQUIRE fence
//              (invalidates i's non-coherent cache lines) before any read of the data, which
//              in addition uses cache-bypassing (sc0 sc1) loads.
// Release / acquire pair at system scope: correct across GPUs by construction, not only on
// one device where the tests run.
// Fence strength.  Reader: an acquire fence (system scope) after every wait.  Writer: when the
// send buffers are UNCACHED memory (the normal case, PeerArgs::uc), a data store is complete once
// acknowledged, so `s_waitcnt vmcnt(0)` before the flag store is the release; if the uncached
// allocation was refused and the buffers are ordinary (cacheable) memory, the flag store is a
// system-scope RELEASE (which also writes this GPU's dirty L2 lines back).  A/B on the emulated
// multi-client round (profiles/peer_fences_r2.log): release stores on every Adam block cost
// 1.0-1.6 us per round, the acquire fences 0.6 us.
__device__ __forceinline__ void peer_acquire() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, ""); }
// flag publish of a value whose data this wave stored into the send buffer
__device__ __forceinline__ void peer_flag_store(unsigned* dst, unsigned v, int uc) {
    if (uc) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(dst, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else {
        __hip_atomic_store(dst, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Report a failure to every rank (this lane's vector stores; any lane may call it).
__device__ __forceinline__ void peer_fail(const PeerArgs& a, unsigned word) {
    __hip_atomic_store(&a.ctl->err, word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    for (int j = 0; j < a.world; ++j)
        if (j != a.rank && a.err_dst[j] != nullptr)
            __hip_atomic_store(a.err_dst[j], word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Called by a lane whose awaited value has not arrived (after a poll): true when its wait must
// end.  After PEER_SLOW_TICKS it ends as soon as any rank has reported a failure (the sticky
// word is set) or this rank's host aborted; at the timeout it reports `missing` to every rank.
__device__ __forceinline__ bool peer_give_up(const PeerArgs& a, unsigned long long t0, unsigned missing) {
    const long long dt = (long long)(__builtin_amdgcn_s_memrealtime() - t0);
    if (dt < PEER_SLOW_TICKS) return false;
    if (__hip_atomic_load(&a.ctl->err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) return true;
    if (a.host_abort != nullptr && __hip_atomic_load(a.host_abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) {
        peer_fail(a, (PEER_ERR_ABORT << 16) | ((unsigned)a.rank << 8) | PEER_MISSING_NONE);
        return true;
    }
    if (dt > a.timeout) {
        peer_fail(a, (PEER_ERR_TIMEOUT << 16) | ((unsigned)a.rank << 8) | (missing & 0xffu));
        return true;
    }
    return false;
}

// Wait until every rank has published `target` in `flags` (one polling lane per rank; ends
// early on a reported failure, PEER_ERR_*).
__device__ __forceinline__ void peer_wait(const PeerArgs& a, unsigned* flags, unsigned target) {
    if (threadIdx.x < (unsigned)a.world) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while ((int)(__hip_atomic_load(&flags[threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - target) < 0) {
            if (peer_give_up(a, t0, threadIdx.x)) break;
            __builtin_amdgcn_s_sleep(2);
        }
    }
    peer_acquire();
    __syncthreads();
}

// out[4*i0 .. 4*i1) = sum over ranks, rank order (bit-identical on every rank); block `bid`
// of `nb` blocks takes a grid-stride share.  Optional bf16 pack of the weights.
// BATCH = ranks whose float4 is in flight at once per thread: all 8 in the standalone kernel;
// 2 in the fused evaluation kernel, which must stay within 64 VGPRs (two 1024-thread
// workgroups per CU) -- there the extra round trips hide behind the evaluation.
template <int BATCH>
__device__ __forceinline__ void peer_reduce4(const PeerArgs& a, const PeerPack& pk, long long i0, long long i1,
                                             int bid, int nb) {
    const int bytes = (int)(a.n * 4);
    for (long long i = i0 + (long long)bid * blockDim.x + threadIdx.x; i < i1; i += (long long)nb * blockDim.x) {
        // the sum is the same left fold in rank order for any BATCH
        float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int j0 = 0; j0 < PEER_MAX_WORLD; j0 += BATCH) {
            float4 v[BATCH];
#pragma unroll
            for (int j = 0; j < BATCH; ++j)
                if (j0 + j < a.world) v[j] = peer_load16(a.src[j0 + j], bytes, (int)(i * 16));
#pragma unroll
            for (int j = 0; j < BATCH; ++j)
                if (j0 + j < a.world) {
                    if (j0 + j == 0) {
                        s = v[j];
                    } else {
                        s.x += v[j].x;
                        s.y += v[j].y;
                        s.z += v[j].z;
                        s.w += v[j].w;
                    }
                }
        }
        reinterpret_cast<float4*>(a.out)[i] = s;
        if (pk.pk != nullptr) peer_pack_store(pk, (int)i, s);
    }
}

// Scalar reduce of floats [e0, e1) by one block.
__device__ __forceinline__ void peer_reduce1(const PeerArgs& a, long long e0, long long e1) {
    const int bytes = (int)(a.n * 4);
    for (long long e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
        float s = peer_load4(a.src[0], bytes, (int)(e * 4));
#pragma unroll
        for (int j = 1; j < PEER_MAX_WORLD; ++j)
            if (j < a.world) s += peer_load4(a.src[j], bytes, (int)(e * 4));
        a.out[e] = s;
    }
}

// The `n_count` blocks that read the call's data call this last: the last of them to finish
// advances the call counter.  (Blocks that only read `seq` at their start need not count if
// some counting block waits for them, as the fused kernel's tail block does.)
__device__ __forceinline__ void peer_finish(const PeerArgs& a, unsigned target, unsigned n_count) {
    __syncthreads();
    if (threadIdx.x == 0) {
        // relaxed: seq is read only by the next call, after the kernel boundary
        const unsigned prev = __hip_atomic_fetch_add(&a.ctl->done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == n_count - 1) {
            __hip_atomic_store(&a.ctl->done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&a.ctl->seq, target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// Wait (bounded) until every evaluation block of this call has stored `target` in its flag:
// plain per-block stores into uncached memory, so no block serialises on a shared counter.
// Thread 0 alone decides to give up (waves read different clocks; the block leaves together).
__device__ __forceinline__ void peer_wait_eval(const PeerArgs& a, unsigned target) {
    __shared__ int state_s;  // 0: all done, 1: pending, 2: give up
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        int pend = 0;
        for (int i = threadIdx.x; i < a.n_eval; i += blockDim.x)
            pend |= (int)(__hip_atomic_load(&a.eflags[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) < 0;
        if (threadIdx.x == 0) state_s = 0;
        __syncthreads();
        if (pend) state_s = 1;
        __syncthreads();
        if (threadIdx.x == 0 && state_s != 0 && peer_give_up(a, t0, PEER_MISSING_EVAL)) state_s = 2;
        __syncthreads();
        const int st = state_s;
        __syncthreads();
        if (st == 0) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // pairs with peer_eval_done's release
            break;
        }
        if (st == 2) break;
        __builtin_amdgcn_s_sleep(2);
    }
}

// Fused evaluation + FedAvg call, role of the all-reduce blocks (bid < nb): pull and reduce
// the weights as soon as every rank published them, then the tails once every rank's
// evaluation is done.  The tails are a few dozen floats: block 0 alone publishes and
// reduces them.
__device__ __forceinline__ void peer_fused_reduce(const PeerArgs& a, const PeerPack& pk, unsigned target, int bid,
                                                  int nb) {
    if (bid == 0) peer_publish(a.flag_dst, a.world, target, a.uc);
    peer_wait(a, a.ctl->flags, target);
    peer_reduce4<2>(a, pk, 0, a.n_w >> 2, bid, nb);
    if (bid == 0) {
        peer_wait_eval(a, target);
        peer_publish(a.tflag_dst, a.world, target, a.uc);
        peer_wait(a, a.ctl->tflags, target);
        peer_reduce1(a, a.n_w, a.n);
    }
}

// Fused call, evaluation block `blk`: once its confusion counts are in the send buffer
// (device-scope atomics into uncached memory, complete when acknowledged: vmcnt 0), it
// stores the call index in its flag.
__device__ __forceinline__ void peer_eval_done(const PeerArgs& a, unsigned target, int blk) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(&a.eflags[blk], target, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------------------
// Adam-fused exchange: the FedAvg all-reduce inside the Adam kernel (fl_kernels.hip).  The
// block that updated a chunk of parameters publishes it (its values are in the uncached send
// buffer once acknowledged), waits for the same chunk from every rank and pulls + sums it:
// no separate all-reduce kernel, no kernel boundary between the update and the reduction.
// Executed by one wave; `target` = the call index (device round state, same on every rank).
// ---------------------------------------------------------------------------------------
// (the caller's stores of the chunk are this wave's: the release store waits for all of them)
__device__ __forceinline__ void peer_chunk_publish(const PeerArgs& a, int chunk, unsigned target) {
    const int lane = threadIdx.x & 63;
    if (lane < a.world) peer_flag_store(a.cflag_dst[lane] + chunk, target, a.uc);
}
__device__ __forceinline__ void peer_chunk_wait(const PeerArgs& a, int chunk, unsigned target) {
    const int lane = threadIdx.x & 63;
    if (lane < a.world) {
        const unsigned* f = a.cflags + lane * a.n_chunks + chunk;
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while ((int)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - target) < 0) {
            if (peer_give_up(a, t0, lane)) break;
            __builtin_amdgcn_s_sleep(2);
        }
    }
    __builtin_amdgcn_wave_barrier();
    peer_acquire();  // whole wave: every lane reads the chunk next
}
__device__ __forceinline__ void peer_chunk_exchange_wait(const PeerArgs& a, int chunk, unsigned target) {
    peer_chunk_publish(a, chunk, target);
    peer_chunk_wait(a, chunk, target);
}

// Sum over ranks (rank order) of the send buffers at float position `pos`.
__device__ __forceinline__ float peer_pull_sum(const PeerArgs& a, int pos) {
    const int bytes = (int)(a.n * 4);
    float v[PEER_MAX_WORLD];
#pragma unroll
    for (int k = 0; k < PEER_MAX_WORLD; ++k)
        if (k < a.world) v[k] = peer_load4(a.src[k], bytes, pos * 4);
    float s = v[0];
#pragma unroll
    for (int k = 1; k < PEER_MAX_WORLD; ++k)
        if (k < a.world) s += v[k];
    return s;
}

// ---------------------------------------------------------------------------------------
// LL (low-latency) chunk exchange: the sender PUSHES each value, together with the call index,
// as ONE 8-byte store into every rank's ring slot for (call parity, sender, position); the
// receiver polls its own ring until every sender's slot carries this call's index, then sums
// in rank order.  An aligned 8-byte store is single-copy atomic, so a slot showing the index
// also shows the value: no fence, no flag store after an acknowledged data store, no remote
// read round trip -- one one-way xGMI write per value instead of write + flag + pull.
// Slots alternate by call parity: a sender writes call t + 2 into a slot only after every
// rank joined call t + 1, which each does after finishing its reads of call t (kernel order).
// The value of an inactive lane is never polled (same positions on every rank).
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ size_t peer_ll_slot(const PeerArgs& a, unsigned target, int src, int pos) {
    return ((size_t)((target & 1u) * PEER_MAX_WORLD + src) * a.n_chunks) * 64 + pos;
}
// this lane's value at ring position `pos` (= chunk * 64 + lane) into every rank's ring
__device__ __forceinline__ void peer_ll_push(const PeerArgs& a, int pos, unsigned target, float v) {
    const unsigned long long w = ((unsigned long long)target << 32) | __float_as_uint(v);
    const size_t slot = peer_ll_slot(a, target, a.rank, pos);
#pragma unroll
    for (int k = 0; k < PEER_MAX_WORLD; ++k)
        if (k < a.world) __hip_atomic_store(a.ll_dst[k] + slot, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// Sum over ranks (rank order) of ring position `pos` for call `target`, polling (ends early on a
// reported failure, PEER_ERR_*: then missing values count 0 and the host discards the round).
// Called by the whole wave; lanes with `active` false (no value at their position) return 0.
__device__ __forceinline__ float peer_ll_sum(const PeerArgs& a, int pos, unsigned target, bool active) {
    if (!active) return 0.f;
    float v[PEER_MAX_WORLD];
    unsigned pend = 0;
#pragma unroll
    for (int k = 0; k < PEER_MAX_WORLD; ++k) {
        v[k] = 0.f;
        if (k < a.world) pend |= 1u << k;
    }
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
#pragma unroll
        for (int k = 0; k < PEER_MAX_WORLD; ++k)
            if (pend & (1u << k)) {
                const unsigned long long w =
                    __hip_atomic_load(a.ll + peer_ll_slot(a, target, k, pos), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if ((unsigned)(w >> 32) == target) {
                    v[k] = __uint_as_float((unsigned)w);
                    pend &= ~(1u << k);
                }
            }
        if (pend == 0) break;
        if (peer_give_up(a, t0, (unsigned)__builtin_ctz(pend))) break;
        __builtin_amdgcn_s_sleep(1);
    }
    float s = v[0];
#pragma unroll
    for (int k = 1; k < PEER_MAX_WORLD; ++k)
        if (k < a.world) s += v[k];
    return s;
}

// ---------------------------------------------------------------------------------------
// Reduce-scatter + all-gather (RS+AG) exchange of one LL chunk (FEDMI_PEER_RSAG=1).  Chunk c is
// OWNED by rank c % world: every other rank pushes its value to the owner only (one 8-byte slot,
// the same ring position as the LL exchange); the owner sums all ranks' values in rank order --
// the LL exchange's sum, bit for bit -- and pushes the sum, with the call index, into every
// other rank's slot of source `owner` (unused by the reduce-scatter there: only the owner
// receives contributions for its chunks).  Per link and round the bytes drop from P slots to
// 2 P / world (1/4 at world 8), for one more one-way hop: the design the bench's N > 1 runs
// measure against the LL ring on real xGMI links (bench.py plane_companions).
// Slot reuse is the LL ring's argument: a rank writes call t + 2 into a slot only after it
// finished call t + 1, which needs the owner's call t + 1 sum, sent after the owner read call t.
// ---------------------------------------------------------------------------------------
// Poll ring slot (source `src`, `pos`) for call `target` (ends early on a reported failure).
__device__ __forceinline__ float peer_ll_wait1(const PeerArgs& a, int src, int pos, unsigned target, bool active) {
    if (!active) return 0.f;
    const unsigned long long* slot = a.ll + peer_ll_slot(a, target, src, pos);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        const unsigned long long w = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if ((unsigned)(w >> 32) == target) return __uint_as_float((unsigned)w);
        if (peer_give_up(a, t0, (unsigned)src)) return 0.f;
        __builtin_amdgcn_s_sleep(1);
    }
}
__device__ __forceinline__ float peer_rsag(const PeerArgs& a, int chunk, int pos, unsigned target, bool active,
                                           float v) {
    const int owner = chunk % a.world;
    const size_t slot = peer_ll_slot(a, target, a.rank, pos);
    if (a.rank != owner) {
        if (active)
            __hip_atomic_store(a.ll_dst[owner] + slot, ((unsigned long long)target << 32) | __float_as_uint(v),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return peer_ll_wait1(a, owner, pos, target, active);
    }
    if (active)
        __hip_atomic_store(a.ll + slot, ((unsigned long long)target << 32) | __float_as_uint(v), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    const float s = peer_ll_sum(a, pos, target, active);
    if (active) {
        const unsigned long long w = ((unsigned long long)target << 32) | __float_as_uint(s);
        for (int k = 0; k < a.world; ++k)
            if (k != owner) __hip_atomic_store(a.ll_dst[k] + slot, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    return s;
}
