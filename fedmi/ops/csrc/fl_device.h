// Device helpers shared by the fp32 (fl_kernels.hip) and bf16 (fl_kernels_bf16.hip) fused
// round kernels: LDS-only barrier, phase stamps, wave reductions, the sklearn-semantics
// metrics of a confusion matrix and the device-side early-stopping state machine.
#pragma once
#include "fl_common.h"
#include <math.h>


// In-kernel phase stamps (100 MHz s_memrealtime) for profiling; off unless b.dbg is set.
#define FL_STAMP(i)                                                                            \
    do {                                                                                       \
        if (b.dbg != nullptr && threadIdx.x == 0)                                              \
            b.dbg[blockIdx.x * 16 + (i)] = __builtin_amdgcn_s_memrealtime();                   \
    } while (0)

// Workgroup barrier that orders LDS only.  __syncthreads() also waits vmcnt(0), which puts
// every in-flight global store (the per-block gradient slab) and load on the critical path
// of each phase; the phases here only hand data to each other through LDS.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Partial barrier through an LDS counter: a wave's LDS stores are complete (lgkmcnt) before
// its lane 0 counts it in; waiting waves re-read the counter (s_sleep between reads) and may
// then read what the counted waves stored.  Only waves that arrive are waited for.
__device__ __forceinline__ void lds_count_arrive(int* cnt) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if ((threadIdx.x & 63) == 0) atomicAdd(cnt, 1);
}
__device__ __forceinline__ void lds_count_wait(int* cnt, int target) {
    while (*reinterpret_cast<volatile int*>(cnt) < target) __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");
}

// Gradient-slab stores.  The slab (n_blocks x P fp32, ~11 MB for the reference MLP) is read
// once, by the next kernel: non-temporal stores stream it past the L2, so the train kernel's
// end no longer writes back 11 MB of dirty lines (measured: fl_train 19.5 -> 14.8 us per
// round, rocprofv3; FL_SLAB_CACHED restores plain stores for comparison).
// write-through (`sc1`), as the fp16 slab (slab_store_h): fp32 round 27.65 -> 26.78 us steady
// against nontemporal stores (profiles/slab_store_policy_r5.log)
__device__ __forceinline__ void slab_store(float* p, float v) {
#if defined(FL_SLAB_CACHED)
    *p = v;
#elif defined(FL_SLAB_NT)
    __builtin_nontemporal_store(v, p);
#else
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
}

// fp16 slab of the bf16 kernels: per-workgroup partial sums of the UNscaled gradient (deltas
// p - onehot, not (p - onehot) / n: |partial| <= rows x max|activation|, far inside fp16's range
// for these models; clamped so an outlier saturates instead of becoming inf, while a NaN stays
// NaN -- fmaxf would turn it into the clamp bound -- so the debug mode's non-finite check still
// sees it), rounded to fp16 (11 significant bits -- finer than the bf16 operands the partials
// are computed from) and summed in fp32 by the Adam kernel, which applies the 1/n.  Half the
// bytes of the fp32 slab, which is written and read back once per round.
__device__ __forceinline__ void slab_store_h(uint16_t* p, float v) {
    const float c = v == v ? fminf(fmaxf(v, -65504.f), 65504.f) : v;
    const _Float16 h = (_Float16)c;
    // write-through (`sc1`: the line leaves the XCD's L2 at once, so the next kernel's reads from
    // other XCDs need no write-back at the kernel boundary): -0.4 us per one-client round in the
    // driver's shape and -0.8 to -0.9 us per emulated N > 1 round against nontemporal stores
    // (profiles/slab_store_policy_r5.log); FL_SLAB_NT / FL_SLAB_CACHED for A/B builds
#if defined(FL_SLAB_CACHED)
    *p = *reinterpret_cast<const uint16_t*>(&h);
#elif defined(FL_SLAB_NT)
    __builtin_nontemporal_store(*reinterpret_cast<const uint16_t*>(&h), p);
#else
    __hip_atomic_store(p, *reinterpret_cast<const uint16_t*>(&h), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// ---------------------------------------------------------------------------------------
// Metrics + early stopping on the device (reference C:85-90, C:165-195).
// ---------------------------------------------------------------------------------------

// Accuracy + weighted precision / recall / F1 (zero_division=0) of a confusion matrix given
// by an accessor cmv(t, p) (sklearn semantics, fedmi/fl/metrics.py).  No local arrays: the
// accessor is re-read per class so nothing spills to scratch.
template <typename CM>
__device__ void metrics_from_cm(CM cmv, int C, double out[4]) {
    double total = 0, tp_sum = 0;
    for (int t = 0; t < C; ++t)
        for (int p = 0; p < C; ++p) {
            const double x = cmv(t, p);
            total += x;
            if (t == p) tp_sum += x;
        }
    if (total <= 0) { out[0] = out[1] = out[2] = out[3] = 0; return; }
    double prec = 0, rec = 0, f1 = 0;
    for (int t = 0; t < C; ++t) {
        double support = 0, pred = 0;
        for (int p = 0; p < C; ++p) { support += cmv(t, p); pred += cmv(p, t); }
        const double tp = cmv(t, t);
        const double w = support / total;
        const double pc = pred > 0 ? tp / pred : 0.0;
        const double rc = support > 0 ? tp / support : 0.0;
        const double den = 2 * tp + (pred - tp) + (support - tp);
        const double fc = den > 0 ? 2 * tp / den : 0.0;
        prec += w * pc; rec += w * rc; f1 += w * fc;
    }
    out[0] = tp_sum / total; out[1] = prec; out[2] = rec; out[3] = f1;
}

// Fold round k's all-reduced tails (`tails` = per-rank slots of C*C counts + loss) into the
// state, if k is the next round to finalize.  Executed by one full wave: lane j computes
// client j's metrics, lane 0 combines them in rank order (the reference's np.mean order)
// and applies the early-stop rule.  Returns the new state in lane 0.
static __device__ FLState fold_round(const MLPDesc& d, const FLConfig& c, const FLBuffers& b,
                                     const float* tails, int r, FLState S, bool write_hist) {
    const int lane = threadIdx.x & 63;
    if (S.stopped || r < 0 || r < S.finalized) return S;
    {
        const int C = d.dim[d.L];
        double mk[4] = {0, 0, 0, 0};
        double lk = 0;
        if (lane < c.world) {
            const float* cm = tails + lane * c.tail_stride;
            metrics_from_cm([&](int t, int p) { return (double)cm[t * C + p]; }, C, mk);
            lk = (double)cm[C * C];
            if (write_hist && r < c.max_rounds)
                for (int q = 0; q < 4; ++q) b.hist_rank[((size_t)r * c.world + lane) * 4 + q] = mk[q];
        }
        // the round's sampled clients (all of them without client sampling): the global
        // metrics and loss are theirs (fl_common.h FLBuffers::rtab)
        const float* rt = b.rtab + 4 * (size_t)r;
        const uint32_t m_lo = __float_as_uint(rt[2]), m_hi = __float_as_uint(rt[3]);
        const double n_act = (double)rt[1];
        auto sampled = [&](int k) { return ((k < 32 ? (m_lo >> k) : (m_hi >> (k - 32))) & 1u) != 0; };
        double mean[4] = {0, 0, 0, 0};
        double loss = 0;
        for (int k = 0; k < c.world; ++k) {
            const bool in = sampled(k);
            for (int q = 0; q < 4; ++q) {
                const double v = __shfl(mk[q], k, 64);
                if (in) mean[q] += v;
            }
            const double lv = __shfl(lk, k, 64);
            if (in) loss += lv;
        }
        if (lane != 0) return S;
        if (c.metric_mode == 0) {
            for (int q = 0; q < 4; ++q) mean[q] /= n_act;
        } else {
            metrics_from_cm(
                [&](int t, int p) {
                    double x = 0;
                    for (int k = 0; k < c.world; ++k)
                        if (sampled(k)) x += (double)tails[k * c.tail_stride + t * C + p];
                    return x;
                },
                C, mean);
        }
        if (write_hist && r < c.max_rounds) {
            for (int q = 0; q < 4; ++q) b.hist_global[(size_t)r * 4 + q] = mean[q];
            b.hist_loss[r] = (float)(loss / n_act);
        }
        if (c.es_enabled) {
            bool close = S.has_prev != 0;
            if (close)
                for (int q = 0; q < 4; ++q)
                    close = close && (fabs(mean[q] - S.prev[q]) <= c.atol + c.rtol * fabs(S.prev[q]));
            if (close) {
                S.count -= 1;
                if (S.count == 0) { S.stopped = 1; S.stop_round = r + 1; }
            } else {
                for (int q = 0; q < 4; ++q) S.prev[q] = mean[q];
                S.has_prev = 1;
                S.count = c.patience;
            }
        }
        S.finalized = r + 1;
    }
    return S;
}

// Can folding the pending rounds (at most two: regions A and B below) stop training?  Only
// then does a block other than the history block need the fold itself: otherwise the round's
// liveness -- all such a block takes from the fold -- is decided by the state on entry (the
// patience counter is >= 1 after any fold that starts above 2: a "close" round decrements it,
// any other resets it to the patience).  The history block (write_hist) always folds.
__device__ __forceinline__ bool fold_may_stop(const FLConfig& c, const FLState& S) {
    return c.es_enabled && !S.stopped && S.count <= 2;
}

// Regions of the all-reduced comm buffer `pg` that hold metrics (fl_common.h FL_FOLD_*):
//   B (tail_off): the previous round's (next_round - 1) own evaluation;
//   A (lag_off) : lagged rounds -- the round before it (next_round - 2), scored inside the
//                 previous round's train kernel.  Folded first: rounds finalize in order.
static __device__ FLState finalize_state(const MLPDesc& d, const FLConfig& c, const FLBuffers& b,
                                         const float* pg, FLState S, bool write_hist, int mask = FL_FOLD_B) {
    if ((mask & FL_FOLD_A) && c.lag_off > 0) {
        S = fold_round(d, c, b, pg + c.lag_off, S.next_round - 2, S, write_hist);
        // only lane 0 holds the folded state: every lane must take the same branch below
        S.finalized = __shfl(S.finalized, 0, 64);
        S.stopped = __shfl(S.stopped, 0, 64);
    }
    if (mask & FL_FOLD_B) S = fold_round(d, c, b, pg + c.tail_off, S.next_round - 1, S, write_hist);
    return S;
}

