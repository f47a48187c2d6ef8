// Fused float64 minibatch step of the sklearn-compatible trainer: TWO kernels per minibatch
// instead of the layered path's ~15 (gather, 3 forward GEMMs, loss head, per layer wgrad +
// bias column sum + dgrad, step counter, Adam -- mlp_trainer.cpp MLPTrainerT::step).
//
// What the reference runs is sklearn's MLPClassifier._fit_stochastic: per minibatch of 200 rows
// a forward pass, the loss head, backprop and an Adam update, all in float64
// (FL_SkLearn_MLPClassifier_Limitation.py:77-101, hyperparameters_tuning.py:90-91).  Everything
// in one minibatch step is ROW-LOCAL except the weight gradient, which sums over the rows:
//
//   skf_rowpass  (grid: ceil(rows/16) row blocks x T trials, 16 waves)
//       gather the block's 16 rows through the epoch permutation -> every layer's forward
//       (bias + ReLU; v_mfma_f64_16x16x4_f64, weights streamed from L2; a narrow output layer
//       on the VALU) -> loss head (logistic + sklearn's clipped binary log-loss, or softmax)
//       -> the backward deltas of every layer (ReLU mask), each written IN PLACE over the
//       activation it masks.  Activations (the wgrad operands) and deltas go to global memory.
//   skf_wgrad_adam (grid: 16x16 gradient tiles of all layers x T trials, 4 waves)
//       dW = delta^T . act over the minibatch rows -- the bias gradient is the extra column of a
//       constant-1 input -- the 4 waves split the rows and their partial tiles are summed in a
//       fixed order, then sklearn's Adam (+ the L2 term alpha/m W) updates p, m, v in the
//       epilogue and adds 0.5 alpha sum W^2 (pre-update) to the epoch loss.
//
// The Adam step counter of a trial is advanced by row block 0 of skf_rowpass (its other blocks
// never read it); skf_wgrad_adam, ordered after it on the stream, uses it.  Summation orders
// differ from the layered path and from BLAS, so results agree with the float64 numpy oracle
// to ~1e-12 per step, not bitwise (tests/test_sklearn_estimator.py: loss curve rtol 1e-9).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <mutex>
#include <math.h>
#include <stdint.h>

#include "mlp_f64.h"

typedef double skf_f64x4 __attribute__((ext_vector_type(4)));

#define SKF_RB 16          // rows per row block (the MFMA's M)
#define SKF_WAVES 16       // waves of a row block
#define SKF_KB 16          // k-steps (of 4) whose weight operands one wave loads at once
#define SKF_NARROW 4       // output layers at most this wide run on the VALU
static_assert(SKF_WAVES == SKF_RB, "skf_fwd_narrow: one wave per row");

__host__ __device__ __forceinline__ int skf_np(int n) { return (n + 15) & ~15; }
// LDS row stride (doubles) of a buffer with np (multiple of 16) columns: np = 2 (mod 32), so the
// MFMA operand reads (16 rows x 4 consecutive columns per wave) hit distinct banks
__host__ __device__ __forceinline__ int skf_ld(int np) { return np + 2 + ((np & 16) ? 16 : 0); }

#define SKF_RED_DOUBLES (SKF_WAVES * 64 * 4)   // partial tiles of a k-split layer (skf_layer)
// LDS of a row block (doubles): the layer buffers, the k-split partials, and the narrow output
// layer's weights + bias when it runs on the VALU
__host__ __device__ __forceinline__ int skf_narrow_doubles(const SkfArgs& a) {
    const int C = a.dims[a.L];
    return C <= SKF_NARROW ? C * a.dims[a.L - 1] + C : 0;
}
size_t skf_lds_bytes(const SkfArgs& a) {
    size_t d = (size_t)skf_ld((a.dims[0] + 15) & ~15);
    for (int l = 0; l < a.L; ++l) d += (size_t)skf_ld((a.dims[l + 1] + 15) & ~15);
    return (d * SKF_RB + SKF_RED_DOUBLES + skf_narrow_doubles(a)) * sizeof(double);
}

// Workgroup barrier that orders LDS only: __syncthreads() also waits for every outstanding
// global store (vmcnt 0), i.e. for the activations / deltas streaming out to memory
// The row pass's outputs for the wgrad kernel (gathered rows, activations, deltas).  SkfArgs::wthru
// (FEDMI_SK_WTHRU=1) writes them through (`sc1`) so no XCD's L2 holds them dirty at the kernel
// boundary: (400, 200) x 9 172-191 -> 159 us per step, but (50, 400) x 1 49 -> 58 and (50, 400) x 9
// 66 -> 76 (profiles/sk_store_policy_r5.log); default-policy stores by default.
__device__ __forceinline__ void skf_st(double* p, double v, bool wthru) {
    if (wthru) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
}

__device__ __forceinline__ void skf_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ double skf_wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// One layer of the row pass on the matrix cores (v_mfma_f64_16x16x4_f64):
//   FWD  out[16][N] = act(src[16][K] . W^T + b)       tiles over n, k-steps over K
//   BWD  dst[16][K] = (src[16][N] . W) * (dst > 0)     tiles over k, k-steps over N; dst holds the
//        activation it masks and is overwritten in place (the lane that reads an activation for
//        its mask is the lane that writes its delta)
// The weight operands stream from L2 (8-byte loads, SKF_KB k-steps per chunk).  The row pass is
// latency-bound, so the work is cut so that every wave holds at most ~2 chunks: a product with
// fewer 16-wide tiles than waves is split along k into G groups (units = tile x group), whose
// partial tiles meet in `red` (LDS) and are summed in group order; each wave walks its chunks
// with the next chunk's loads in flight while the current one multiplies.
// Branch-free by construction: every operand load is unconditional (clamped address, zero
// selected after the load) and every MFMA runs (a zero weight operand, an in-range activation
// column), so the compiler keeps the next chunk's loads in flight across the current chunk's
// MFMAs -- with predicated loads / MFMAs it waited for ALL loads before every MFMA.
// Split row pass (skf_cs_* below) extras: `ldwt` = row stride of WT (FWD) / of W (BWD) when W / WT /
// bias point at a slice of the layer's output columns (0: the layer's own N / K); `raw` (BWD) = store
// the product itself instead of masking the activation in dst; `gmax` caps the k-groups (a slice
// keeps the whole product's); skf_layer's `kb_steps` keeps the whole product's chunk length.
template <bool FWD, int KB>
__device__ __forceinline__ void skf_layer_kb(const double* __restrict__ src, int ld_s, double* __restrict__ dst,
                                             int ld_d, const double* __restrict__ W, const double* __restrict__ bias,
                                             int K, int N, bool relu, double* __restrict__ red, int wave, int lane,
                                             const double* __restrict__ zero, const double* __restrict__ WT,
                                             unsigned long long* dbg = nullptr, int ldwt = 0, bool raw = false,
                                             int gmax = SKF_WAVES) {
    if (ldwt <= 0) ldwt = FWD ? N : K;   // FWD: row stride of WT [K][N]; BWD: row stride of W [N][K]
    const int lr = lane & 15, lg = lane >> 4;
    if (dbg != nullptr && threadIdx.x == 0) dbg[0] = __builtin_amdgcn_s_memrealtime();
    const int ntiles = FWD ? (N + 15) >> 4 : (K + 15) >> 4;
    const int steps = FWD ? (K + 3) >> 2 : (N + 3) >> 2;
    const int nb = (steps + KB - 1) / KB;           // chunks per tile
    const int G = min(gmax, ntiles < SKF_WAVES ? max(1, min(nb, SKF_WAVES / ntiles)) : 1);
    const int units = ntiles * G;
    const int bpg = (nb + G - 1) / G;               // chunks per unit
    const int my_units = wave < units ? (units - 1 - wave) / SKF_WAVES + 1 : 0;
    const int nchunks = my_units * bpg;
    // chunk c of this wave: unit u = wave + 16 (c / bpg), its batch b = g bpg + c % bpg
    auto load = [&](int c, double (&bw)[KB]) {
        const int u = wave + SKF_WAVES * (c / bpg);
        const int tile = u / G, b = (u - tile * G) * bpg + c % bpg;
        const int col = tile * 16 + lr;   // output column of this lane
#pragma unroll
        for (int i = 0; i < KB; ++i) {
            const int kk = 4 * (b * KB + i) + lg;   // contraction index of this lane
            const bool ok = FWD ? (col < N && kk < K) : (col < K && kk < N);
            // out of range: read a zero from `zero` instead of selecting 0 after the load (a
            // select would wait for the load right here, prefetch included)
            // FWD reads the transposed copy WT [K][N] when there is one (SkfArgs::wt): 16 consecutive
            // output columns per k-row -- whole cache lines -- instead of 16 rows x 32 bytes
            const double* q = ok ? (FWD ? (WT != nullptr ? WT + (size_t)kk * ldwt + col : W + (size_t)col * K + kk)
                                        : W + (size_t)kk * ldwt + col)
                                 : zero;
            bw[i] = *q;
        }
    };
    auto mult = [&](int c, const double (&bw)[KB], skf_f64x4& acc) {
        const int u = wave + SKF_WAVES * (c / bpg);
        const int tile = u / G, b = (u - tile * G) * bpg + c % bpg;
        double av[KB];   // every activation operand read from LDS before the first MFMA
#pragma unroll
        for (int i = 0; i < KB; ++i) {
            const int st = b * KB + i;
            const int col = st < steps ? 4 * st + lg : lg;   // past the end: any finite column, times 0
            av[i] = src[lr * ld_s + col];
        }
        // keep the reads ahead of the MFMAs (the scheduler otherwise sinks each read next to its
        // MFMA and exposes the LDS latency per step)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < KB; ++i) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[i], bw[i], acc, 0, 0, 0);
    };
    // D reg j of lane l = D[(l >> 4) + 4j][l & 15]
    auto epilogue = [&](int tile, const skf_f64x4& acc) {
        const int col = tile * 16 + lr;
        if (FWD) {
            const double bv = col < N ? bias[col] : 0.0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                double v = acc[j] + bv;
                if (relu) v = v > 0.0 ? v : 0.0;
                dst[(lg + 4 * j) * ld_d + col] = col < N ? v : 0.0;
            }
        } else if (raw) {
#pragma unroll
            for (int j = 0; j < 4; ++j) dst[(lg + 4 * j) * ld_d + col] = col < K ? acc[j] : 0.0;
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                double* p = dst + (lg + 4 * j) * ld_d + col;
                const double m = *p;
                *p = (col < K && m > 0.0) ? acc[j] : 0.0;
            }
        }
    };
    auto finish = [&](int c, const skf_f64x4& acc) {
        const int u = wave + SKF_WAVES * (c / bpg);
        if (G == 1) {
            epilogue(u, acc);
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) red[(u * 64 + lane) * 4 + j] = acc[j];
        }
    };
    double b0[KB], b1[KB];
    skf_f64x4 acc = {0.0, 0.0, 0.0, 0.0};
    if (nchunks > 0) load(0, b0);
    for (int c = 0; c < nchunks; c += 2) {
        if (c + 1 < nchunks) load(c + 1, b1);
        mult(c, b0, acc);
        if (dbg != nullptr && threadIdx.x == 0 && c == 0) {
            asm volatile("s_nop 0" ::"v"(acc[0]));   // after the first chunk's MFMAs issued
            dbg[1] = __builtin_amdgcn_s_memrealtime();
        }
        if (c % bpg == bpg - 1) {
            finish(c, acc);
            acc = (skf_f64x4){0.0, 0.0, 0.0, 0.0};
        }
        if (c + 1 < nchunks) {
            if (c + 2 < nchunks) load(c + 2, b0);
            mult(c + 1, b1, acc);
            if ((c + 1) % bpg == bpg - 1) {
                finish(c + 1, acc);
                acc = (skf_f64x4){0.0, 0.0, 0.0, 0.0};
            }
        }
    }
    if (dbg != nullptr && threadIdx.x == 0) dbg[2] = __builtin_amdgcn_s_memrealtime();
    if (G > 1) {
        skf_lds_barrier();
        for (int tile = wave; tile < ntiles; tile += SKF_WAVES) {
            skf_f64x4 s = {0.0, 0.0, 0.0, 0.0};
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int j = 0; j < 4; ++j) s[j] += red[((tile * G + g) * 64 + lane) * 4 + j];
            epilogue(tile, s);
        }
    }
}

// chunk length by contraction depth: short products waste no MFMAs on padding
template <bool FWD>
__device__ __forceinline__ void skf_layer(const double* __restrict__ src, int ld_s, double* __restrict__ dst, int ld_d,
                                          const double* __restrict__ W, const double* __restrict__ bias, int K, int N,
                                          bool relu, double* __restrict__ red, int wave, int lane,
                                          const double* __restrict__ zero, const double* __restrict__ WT,
                                          unsigned long long* dbg = nullptr, int ldwt = 0, bool raw = false,
                                          int gmax = SKF_WAVES, int kb_steps = 0) {
    // kb_steps > 0: pick the chunk length of a product this many k-steps deep (a slice of a wider
    // product keeps the whole product's chunking, so its sums are the same)
    const int steps = kb_steps > 0 ? kb_steps : (FWD ? (K + 3) >> 2 : (N + 3) >> 2);
    if (steps <= 4)
        skf_layer_kb<FWD, 4>(src, ld_s, dst, ld_d, W, bias, K, N, relu, red, wave, lane, zero, WT, dbg, ldwt, raw, gmax);
    else if (steps <= 8)
        skf_layer_kb<FWD, 8>(src, ld_s, dst, ld_d, W, bias, K, N, relu, red, wave, lane, zero, WT, dbg, ldwt, raw, gmax);
    else
        skf_layer_kb<FWD, SKF_KB>(src, ld_s, dst, ld_d, W, bias, K, N, relu, red, wave, lane, zero, WT, dbg, ldwt, raw,
                                  gmax);
}

// Narrow output layer (N <= SKF_NARROW) on the VALU, weights staged in LDS (Ws [N][K], bias at
// Ws[N * K + c]): wave w = row w, lanes split k, one deterministic xor-tree sum per output.
__device__ __forceinline__ void skf_fwd_narrow(const double* __restrict__ in, int ld_i, double* __restrict__ out,
                                               int ld_o, const double* __restrict__ Ws, int K, int N, int wave,
                                               int lane) {
    const int r = wave;  // SKF_WAVES == SKF_RB
    for (int c = 0; c < N; ++c) {
        double s = 0.0;
        for (int k = lane; k < K; k += 64) s += in[r * ld_i + k] * Ws[c * K + k];
        s = skf_wave_sum(s);
        if (lane == 0) out[r * ld_o + c] = s + Ws[N * K + c];
    }
    if (lane < skf_np(N) && lane >= N) out[r * ld_o + lane] = 0.0;
}

// Backward through the narrow output layer (N <= SKF_NARROW; weights staged in LDS): every
// thread owns (row, k) elements.
__device__ __forceinline__ void skf_bwd_narrow(const double* __restrict__ d, int ld_d, double* __restrict__ a, int ld_a,
                                               const double* __restrict__ W, int K, int N) {
    const int kp = skf_np(K);
    for (int e = threadIdx.x; e < SKF_RB * kp; e += blockDim.x) {
        const int r = e / kp, k = e - r * kp;
        double s = 0.0;
        for (int n = 0; n < N; ++n) s += d[r * ld_d + n] * (k < K ? W[(size_t)n * K + k] : 0.0);
        double* p = a + r * ld_a + k;
        *p = (k < K && *p > 0.0) ? s : 0.0;
    }
}

// phase stamps (profiling, SkfArgs::dbg): thread 0 of row block (0, 0), 100 MHz clock; the tile split's
// skf_cs_fwd writes 0-4, skf_cs_bwd 5-10 (a stamp's store makes later code wait for it: they perturb)
#define SKF_STAMP(i)                                                                              \
    do {                                                                                          \
        if (a.dbg != nullptr && threadIdx.x == 0 && rb == 0 && blockIdx.y == 0)                   \
            a.dbg[i] = __builtin_amdgcn_s_memrealtime();                                          \
    } while (0)

__global__ void __launch_bounds__(SKF_WAVES * 64) skf_rowpass_kernel(SkfArgs a) {
    extern __shared__ double lds[];
    __shared__ int ys[SKF_RB];
    const int t = blockIdx.y;
    if (a.active[t] == 0) return;
    // (the wave index in a scalar register: the layer loops' control flow stays scalar)
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    // (measured: placing a trial's row blocks and wgrad tiles on one XCD, so the weights its Adam
    // wrote are L2-resident, changed nothing -- profiles/sk_step_bench_r5e.jsonl; the row pass is
    // bound per CU, the same with 1 or 9 trials)
    const int rb = blockIdx.x;
    const int r0 = rb * SKF_RB;
    const int nr = min(SKF_RB, a.rows - r0);
    SKF_STAMP(0);
    if (rb == 0 && threadIdx.x == 0) a.step[t] += 1;  // this minibatch's Adam step t
    const double* P = a.params + (size_t)t * a.P;
    // LDS: buffer 0 = the rows' inputs, buffer l + 1 = layer l's output (then its delta); offsets
    // recomputed from the (uniform) dims instead of a dynamically indexed array (scratch)
    auto ldof = [&](int l) { return skf_ld(skf_np(a.dims[l])); };
    auto bufp = [&](int l) {
        int o = 0;
        for (int i = 0; i < l; ++i) o += ldof(i) * SKF_RB;
        return lds + o;
    };
    double* red = bufp(a.L + 1);
    double* wnar = red + SKF_RED_DOUBLES;
    const bool narrow = a.dims[a.L] <= SKF_NARROW;
    if (narrow) {
        // the narrow output layer's weights + bias -> LDS, in flight with the gather
        const int nw = skf_narrow_doubles(a), C = a.dims[a.L], Kl = a.dims[a.L - 1];
        for (int e = threadIdx.x; e < nw; e += blockDim.x)
            wnar[e] = e < C * Kl ? P[a.w_off[a.L - 1] + e] : P[a.b_off[a.L - 1] + e - C * Kl];
    }
    // gather through the epoch permutation (sklearn: X[sample_idx[batch_slice]])
    const int F = a.dims[0], fp = skf_np(F);
    const int* perm = a.perms + (size_t)(*a.epoch_ctr) * a.n_perm + a.off + r0;
    double* xg = a.xg + ((size_t)t * a.Bmax + r0) * F;
    for (int e = threadIdx.x; e < SKF_RB * fp; e += blockDim.x) {
        const int r = e / fp, f = e - r * fp;
        double v = 0.0;
        if (r < nr && f < F) {
            v = a.X[(size_t)perm[r] * F + f];
            skf_st(&xg[(size_t)r * F + f], v, a.wthru);
        }
        bufp(0)[r * ldof(0) + f] = v;
    }
    if (threadIdx.x < SKF_RB) ys[threadIdx.x] = threadIdx.x < nr ? a.y[perm[threadIdx.x]] : 0;
    skf_lds_barrier();
    SKF_STAMP(1);
    // forward
    for (int l = 0; l < a.L; ++l) {
        const int K = a.dims[l], N = a.dims[l + 1];
        const double* W = P + a.w_off[l];
        const double* b = P + a.b_off[l];
        if (l == a.L - 1 && narrow)
            skf_fwd_narrow(bufp(l), ldof(l), bufp(l + 1), ldof(l + 1), wnar, K, N, wave, lane);
        else
            skf_layer<true>(bufp(l), ldof(l), bufp(l + 1), ldof(l + 1), W, b, K, N, l + 1 < a.L, red, wave, lane, a.zero,
                            a.wt != nullptr ? a.wt + (size_t)t * a.P + a.w_off[l] : nullptr,
                            (a.dbg != nullptr && l == 1 && rb == 0 && t == 0) ? a.dbg + 13 : nullptr);
        skf_lds_barrier();
        SKF_STAMP(2 + l);
        if (l + 1 < a.L) {  // hidden activation: the next layer's wgrad operand (kernel 2)
            double* ag = a.acts + (((size_t)l * a.T + t) * a.Bmax + r0) * a.maxw;
            for (int e = threadIdx.x; e < nr * N; e += blockDim.x) {
                const int r = e / N, c = e - r * N;
                skf_st(&ag[(size_t)r * a.maxw + c], bufp(l + 1)[r * ldof(l + 1) + c], a.wthru);
            }
        }
    }
    // loss head: delta = (p - onehot) / m, written over the logits; row losses summed
    {
        const int C = a.dims[a.L];
        double* z = bufp(a.L);
        const int ldz = ldof(a.L);
        double lrow = 0.0;
        const double eps = 2.220446049250313e-16;
        if (threadIdx.x < SKF_RB) {
            const int r = threadIdx.x, yy = ys[r];
            double* zr = z + r * ldz;
            if (r >= nr) {
                for (int c = 0; c < C; ++c) zr[c] = 0.0;
            } else if (a.head == 1) {
                const double p = 1.0 / (1.0 + exp(-zr[0]));
                const double pc = fmin(fmax(p, eps), 1.0 - eps);
                lrow = yy ? -log(pc) : -log(1.0 - pc);
                zr[0] = (p - (double)yy) * a.inv_rows;
            } else {
                double mx = zr[0];
                for (int c = 1; c < C; ++c) mx = fmax(mx, zr[c]);
                double se = 0.0;
                for (int c = 0; c < C; ++c) se += exp(zr[c] - mx);
                const double py = fmin(fmax(exp(zr[yy] - mx) / se, eps), 1.0 - eps);
                lrow = -log(py);
                for (int c = 0; c < C; ++c) zr[c] = (exp(zr[c] - mx) / se - (c == yy ? 1.0 : 0.0)) * a.inv_rows;
            }
        }
        if (wave == 0) {
            lrow = skf_wave_sum(lrow);
            if (lane == 0) atomicAdd(&a.loss_acc[t], lrow);
        }
        skf_lds_barrier();
        SKF_STAMP(7);
        double* dg = a.deltas + (((size_t)(a.L - 1) * a.T + t) * a.Bmax + r0) * a.maxw;
        for (int e = threadIdx.x; e < nr * C; e += blockDim.x) {
            const int r = e / C, c = e - r * C;
            skf_st(&dg[(size_t)r * a.maxw + c], z[r * ldz + c], a.wthru);
        }
    }
    // backward: delta of layer l - 1 from layer l's, over the activation it masks
    for (int l = a.L - 1; l >= 1; --l) {
        const int K = a.dims[l], N = a.dims[l + 1];
        const double* W = P + a.w_off[l];
        if (l == a.L - 1 && narrow)
            skf_bwd_narrow(bufp(l + 1), ldof(l + 1), bufp(l), ldof(l), wnar, K, N);
        else
            skf_layer<false>(bufp(l + 1), ldof(l + 1), bufp(l), ldof(l), W, nullptr, K, N, false, red, wave, lane, a.zero, nullptr);
        skf_lds_barrier();
        SKF_STAMP(8 + (a.L - 1 - l));
        double* dg = a.deltas + (((size_t)(l - 1) * a.T + t) * a.Bmax + r0) * a.maxw;
        for (int e = threadIdx.x; e < nr * K; e += blockDim.x) {
            const int r = e / K, c = e - r * K;
            skf_st(&dg[(size_t)r * a.maxw + c], bufp(l)[r * ldof(l) + c], a.wthru);
        }
    }
    if (a.dbg != nullptr) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    SKF_STAMP(12);
}

// ---------------------------------------------------------------------------------------
// Tile-split row pass (SkfArgs::split = S > 1), BIT-IDENTICAL to skf_rowpass.  skf_rowpass runs one
// 16-row block on ONE CU and is bound by that CU's float64 MFMA pipes (MFMA busy 67 %): every row
// block streams and multiplies the whole weight set alone, so a 200-row minibatch uses 13 CUs.  For
// two hidden layers and a narrow head (sklearn's [S] net (50, 400) and the [H] grid's two-layer
// nets) the two products of hidden layer 1 -- its forward (output tiles over its N columns) and its
// input gradient (output tiles over its K inputs) -- are split by OUTPUT TILES over S workgroups per
// row block.  Every output tile is a complete sum in one workgroup, with skf_rowpass's chunk length
// and k-groups for the whole product (kb_steps, gmax), so nothing is re-associated:
//   skf_cs_fwd  (row block x slice x trial)  gather, hidden layer 0 (every slice recomputes it, slice
//               0 stores it), the slice's forward tiles of hidden layer 1 -> acts
//   skf_cs_bwd  (row block x slice x trial)  the logits from ALL of layer 1's activations in
//               skf_fwd_narrow's order, the loss head, layer 1's delta (skf_bwd_narrow's sums; every
//               slice, slice 0 stores it), the slice's tiles of layer 1's input gradient masked by
//               layer 0's activations -> layer 0's delta
// The weights are therefore those of skf_rowpass bit for bit, and the float64 estimator keeps
// tracking scikit-learn epoch by epoch (tools/sklearn_parity.py).
// ---------------------------------------------------------------------------------------
struct SkfGroups { int KB, nb, G, bpg; };
// skf_layer_kb's cut of a product: chunk length KB (k-steps), nb chunks per tile, G k-groups of
// bpg chunks (the same arithmetic as skf_layer / skf_layer_kb)
__host__ __device__ __forceinline__ SkfGroups skf_groups(int steps, int ntiles) {
    SkfGroups g;
    g.KB = steps <= 4 ? 4 : (steps <= 8 ? 8 : SKF_KB);
    g.nb = (steps + g.KB - 1) / g.KB;
    const int Gm = ntiles < SKF_WAVES ? (SKF_WAVES / ntiles < g.nb ? SKF_WAVES / ntiles : g.nb) : 1;
    g.G = Gm < 1 ? 1 : Gm;
    g.bpg = (g.nb + g.G - 1) / g.G;
    return g;
}
// Tiles of slice `sl` of a product with `ntiles` output tiles cut into `S` slices: [t0, t0 + n)
__host__ __device__ __forceinline__ void skf_slice_tiles(int ntiles, int S, int sl, int* t0, int* n) {
    const int per = (ntiles + S - 1) / S;
    *t0 = sl * per;
    const int e = *t0 + per < ntiles ? *t0 + per : ntiles;
    *n = e > *t0 ? e - *t0 : 0;
}

int skf_pick_split(const SkfArgs& a, int want, int cus) {
    if (a.L != 3 || a.dims[a.L] > SKF_NARROW || want == 1) return 1;
    const int K = a.dims[1], N = a.dims[2];   // hidden layer 1: K -> N
    const int nt_f = (N + 15) >> 4, nt_b = (K + 15) >> 4;
    int S = nt_f < nt_b ? nt_f : nt_b;        // every slice owns >= 1 tile of both products
    if (S > 8) S = 8;
    if (want > 1) {
        S = want < S ? want : S;
    } else {
        // about one workgroup per CU over all row blocks and trials (more queue behind each other:
        // profiles/sk_tile_split_ab_r6.log)
        const int nrb = (a.Bmax + SKF_RB - 1) / SKF_RB;
        const int by_cus = std::max(1, cus) / std::max(1, nrb * a.T);
        S = S < by_cus ? S : by_cus;
    }
    // every slice must own tiles of both products (the last slice of a ceil-cut can be empty)
    for (; S >= 2; --S) {
        int t0, nf, nb;
        skf_slice_tiles(nt_f, S, S - 1, &t0, &nf);
        skf_slice_tiles(nt_b, S, S - 1, &t0, &nb);
        if (nf >= 1 && nb >= 1) break;
    }
    return S < 2 ? 1 : S;
}

// LDS of skf_cs_bwd (doubles): layer 1's activations -> its delta [16][ld(N)], layer 0's activations
// of the slice's input-gradient tiles -> layer 0's delta [16][ld(K)], the k-split partials, the head
// weights + bias
static size_t skf_cs_bwd_lds(const SkfArgs& a) {
    const size_t d = (size_t)SKF_RB * skf_ld(skf_np(a.dims[2])) + (size_t)SKF_RB * skf_ld(skf_np(a.dims[1])) +
                     SKF_RED_DOUBLES + (size_t)a.dims[3] * (a.dims[2] + 1);
    return d * sizeof(double);
}

__global__ void __launch_bounds__(SKF_WAVES * 64) skf_cs_fwd_kernel(SkfArgs a) {
    extern __shared__ double lds[];
    const int t = blockIdx.z, sl = blockIdx.y, rb = blockIdx.x;
    if (a.active[t] == 0) return;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int r0 = rb * SKF_RB, nr = min(SKF_RB, a.rows - r0);
    const int K1 = a.dims[1], N1 = a.dims[2];
    int tf0, ntf;
    skf_slice_tiles((N1 + 15) >> 4, a.split, sl, &tf0, &ntf);
    const int c0 = tf0 * 16, nc = min(ntf * 16, N1 - c0);   // this slice's output columns of layer 1
    SKF_STAMP(0);
    if (rb == 0 && sl == 0 && threadIdx.x == 0) a.step[t] += 1;  // this minibatch's Adam step
    const double* P = a.params + (size_t)t * a.P;
    auto ldof = [&](int l) { return skf_ld(skf_np(a.dims[l])); };
    double* b0 = lds;                               // inputs [16][ld(F)]
    double* b1 = b0 + ldof(0) * SKF_RB;             // hidden 0 [16][ld(K1)]
    double* b2 = b1 + ldof(1) * SKF_RB;             // hidden 1 [16][ld(N1)] (this slice's columns)
    double* red = b2 + ldof(2) * SKF_RB;
    const int F = a.dims[0], fp = skf_np(F);
    const int* perm = a.perms + (size_t)(*a.epoch_ctr) * a.n_perm + a.off + r0;
    double* xg = a.xg + ((size_t)t * a.Bmax + r0) * F;
    for (int e = threadIdx.x; e < SKF_RB * fp; e += blockDim.x) {
        const int r = e / fp, f = e - r * fp;
        double v = 0.0;
        if (r < nr && f < F) {
            v = a.X[(size_t)perm[r] * F + f];
            if (sl == 0) skf_st(&xg[(size_t)r * F + f], v, a.wthru);
        }
        b0[r * ldof(0) + f] = v;
    }
    skf_lds_barrier();
    SKF_STAMP(1);
    // hidden layer 0, whole (the same call as skf_rowpass); slice 0 stores it
    skf_layer<true>(b0, ldof(0), b1, ldof(1), P + a.w_off[0], P + a.b_off[0], F, K1, true, red, wave, lane, a.zero,
                    a.wt != nullptr ? a.wt + (size_t)t * a.P + a.w_off[0] : nullptr);
    skf_lds_barrier();
    SKF_STAMP(2);
    if (sl == 0 && wave < nr) {   // (a row per wave)
        double* ag = a.acts + ((size_t)t * a.Bmax + r0 + wave) * a.maxw;
        for (int c = lane; c < K1; c += 64) skf_st(&ag[c], b1[wave * ldof(1) + c], a.wthru);
    }
    // the slice's output tiles of hidden layer 1's forward, with skf_rowpass's chunking and k-groups
    const SkfGroups gf = skf_groups((K1 + 3) >> 2, (N1 + 15) >> 4);
    skf_layer<true>(b1, ldof(1), b2 + c0, ldof(2), P + a.w_off[1] + (size_t)c0 * K1, P + a.b_off[1] + c0, K1, nc, true,
                    red, wave, lane, a.zero, a.wt != nullptr ? a.wt + (size_t)t * a.P + a.w_off[1] + c0 : nullptr,
                    nullptr, N1, false, gf.G, (K1 + 3) >> 2);
    skf_lds_barrier();
    SKF_STAMP(3);
    if (wave < nr) {   // (a row per wave)
        double* ag = a.acts + (((size_t)a.T + t) * a.Bmax + r0 + wave) * a.maxw + c0;
        for (int j = lane; j < nc; j += 64) skf_st(&ag[j], b2[wave * ldof(2) + c0 + j], a.wthru);
    }
    if (a.dbg != nullptr) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    SKF_STAMP(4);
}

__global__ void __launch_bounds__(SKF_WAVES * 64) skf_cs_bwd_kernel(SkfArgs a) {
    extern __shared__ double lds[];
    __shared__ double dz_s[SKF_RB * SKF_NARROW];
    const int t = blockIdx.z, sl = blockIdx.y, rb = blockIdx.x;
    if (a.active[t] == 0) return;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int r0 = rb * SKF_RB, nr = min(SKF_RB, a.rows - r0);
    const int K1 = a.dims[1], N1 = a.dims[2], C = a.dims[3];
    int tb0, ntb;
    skf_slice_tiles((K1 + 15) >> 4, a.split, sl, &tb0, &ntb);
    const int k0 = tb0 * 16, nk = min(ntb * 16, K1 - k0);   // this slice's input-gradient columns
    SKF_STAMP(5);
    const double* P = a.params + (size_t)t * a.P;
    const int np2 = skf_np(N1), ld2 = skf_ld(np2), ldk = skf_ld(skf_np(K1));
    double* h = lds;                       // [16][ld2]: layer 1's activations, then its delta
    double* a0s = h + SKF_RB * ld2;        // [16][ldk]: layer 0's activations of the slice -> its delta
    double* red = a0s + SKF_RB * ldk;
    double* wh = red + SKF_RED_DOUBLES;    // head weights [C][N1], then its bias [C]
    const double* Wh = P + a.w_off[2];
    for (int e = threadIdx.x; e < C * N1; e += blockDim.x) wh[e] = Wh[e];
    if (threadIdx.x < C) wh[C * N1 + threadIdx.x] = P[a.b_off[2] + threadIdx.x];
    const double* ag = a.acts + (((size_t)a.T + t) * a.Bmax + r0) * a.maxw;
#ifdef SKF_HLOAD_FLAT   // (A/B: the round-6 first version)
    for (int e = threadIdx.x; e < SKF_RB * np2; e += blockDim.x) {
        const int r = e / np2, j = e - r * np2;
        h[r * ld2 + j] = (r < nr && j < N1) ? ag[(size_t)r * a.maxw + j] : 0.0;
    }
#else
    {   // wave w = row w, 4 loads in flight per lane before the first LDS store (-1 us per [S] step,
        // profiles/sk_step_marginal_r6.log)
        const double* agr = ag + (size_t)wave * a.maxw;
        double* hr = h + wave * ld2;
        for (int k0 = lane; k0 < np2; k0 += 256) {
            double v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int k = k0 + 64 * u;
                v[u] = *((wave < nr && k < N1) ? agr + k : a.zero);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (k0 + 64 * u < np2) hr[k0 + 64 * u] = v[u];
        }
    }
#endif
    const double* a0g = a.acts + ((size_t)t * a.Bmax + r0) * a.maxw;
    const int npk = skf_np(nk);
    for (int e = threadIdx.x; e < SKF_RB * npk; e += blockDim.x) {
        const int r = e / npk, j = e - r * npk;
        a0s[r * ldk + j] = (r < nr && j < nk) ? a0g[(size_t)r * a.maxw + k0 + j] : 0.0;
    }
    skf_lds_barrier();
    SKF_STAMP(6);
    // logits: skf_fwd_narrow's sums (wave w = row w, lanes over k, xor tree, + bias)
    {
        const int r = wave;
        for (int c = 0; c < C; ++c) {
            double sum = 0.0;
            for (int k = lane; k < N1; k += 64) sum += h[r * ld2 + k] * wh[c * N1 + k];
            sum = skf_wave_sum(sum);
            if (lane == 0) dz_s[r * C + c] = sum + wh[C * N1 + c];
        }
    }
    skf_lds_barrier();
    SKF_STAMP(7);
    // loss head (skf_rowpass's): the logits become the head delta in place
    double lrow = 0.0;
    if (threadIdx.x < SKF_RB) {
        const int r = threadIdx.x;
        const double eps = 2.220446049250313e-16;
        double* zr = dz_s + r * C;
        if (r >= nr) {
            for (int c = 0; c < C; ++c) zr[c] = 0.0;
        } else {
            const int* perm = a.perms + (size_t)(*a.epoch_ctr) * a.n_perm + a.off + r0;
            const int yy = a.y[perm[r]];
            if (a.head == 1) {
                const double p = 1.0 / (1.0 + exp(-zr[0]));
                const double pc = fmin(fmax(p, eps), 1.0 - eps);
                lrow = yy ? -log(pc) : -log(1.0 - pc);
                zr[0] = (p - (double)yy) * a.inv_rows;
            } else {
                double mx = zr[0];
                for (int c = 1; c < C; ++c) mx = fmax(mx, zr[c]);
                double se = 0.0;
                for (int c = 0; c < C; ++c) se += exp(zr[c] - mx);
                const double py = fmin(fmax(exp(zr[yy] - mx) / se, eps), 1.0 - eps);
                lrow = -log(py);
                for (int c = 0; c < C; ++c) zr[c] = (exp(zr[c] - mx) / se - (c == yy ? 1.0 : 0.0)) * a.inv_rows;
            }
        }
    }
    if (sl == 0 && wave == 0) {
        lrow = skf_wave_sum(lrow);
        if (lane == 0) atomicAdd(&a.loss_acc[t], lrow);
    }
    skf_lds_barrier();
    if (sl == 0) {  // the head delta: the head's wgrad operand
        double* dg = a.deltas + (((size_t)2 * a.T + t) * a.Bmax + r0) * a.maxw;
        for (int e = threadIdx.x; e < nr * C; e += blockDim.x) {
            const int r = e / C, c = e - r * C;
            skf_st(&dg[(size_t)r * a.maxw + c], dz_s[r * C + c], a.wthru);
        }
    }
    // layer 1's delta, every column (skf_bwd_narrow's sums, ReLU mask), in place
#ifdef SKF_DELTA_FLAT   // (A/B: the round-6 first version)
    for (int e = threadIdx.x; e < SKF_RB * np2; e += blockDim.x) {
        const int r = e / np2, k = e - r * np2;
        double sum = 0.0;
        for (int n = 0; n < C; ++n) sum += dz_s[r * C + n] * (k < N1 ? wh[n * N1 + k] : 0.0);
        double* p = h + r * ld2 + k;
        *p = (k < N1 && *p > 0.0) ? sum : 0.0;
    }
#else
    {   // wave w = row w, lanes over the columns (no index division), the same sums (-1.6 us per [S]
        // step, profiles/sk_step_marginal_r6.log)
        static_assert(SKF_RB == SKF_WAVES, "one row per wave");
        const int r = wave;
        double dzr[SKF_NARROW];
#pragma unroll
        for (int n = 0; n < SKF_NARROW; ++n) dzr[n] = n < C ? dz_s[r * C + n] : 0.0;
        double* hr = h + r * ld2;
        for (int k = lane; k < np2; k += 64) {
            double sum = 0.0;
#pragma unroll
            for (int n = 0; n < SKF_NARROW; ++n)
                if (n < C) sum += dzr[n] * (k < N1 ? wh[n * N1 + k] : 0.0);
            const double m = hr[k];
            hr[k] = (k < N1 && m > 0.0) ? sum : 0.0;
        }
    }
#endif
    skf_lds_barrier();
    SKF_STAMP(8);
    if (sl == 0 && wave < nr) {  // layer 1's delta: the wgrad operand of layer 1 (a row per wave)
        double* dg = a.deltas + (((size_t)a.T + t) * a.Bmax + r0 + wave) * a.maxw;
        for (int c = lane; c < N1; c += 64) skf_st(&dg[c], h[wave * ld2 + c], a.wthru);
    }
    // the slice's tiles of layer 1's input gradient, masked in place over layer 0's activations:
    // skf_rowpass's chunk length and k-groups for the whole product (each tile a complete sum)
    const SkfGroups gb = skf_groups((N1 + 3) >> 2, (K1 + 15) >> 4);
    skf_layer<false>(h, ld2, a0s, ldk, P + a.w_off[1] + k0, nullptr, nk, N1, false, red, wave, lane, a.zero, nullptr,
                     nullptr, K1, false, gb.G, (N1 + 3) >> 2);
    skf_lds_barrier();
    SKF_STAMP(9);
    if (wave < nr) {   // (a row per wave)
        double* dg = a.deltas + ((size_t)t * a.Bmax + r0 + wave) * a.maxw + k0;
        for (int j = lane; j < nk; j += 64) skf_st(&dg[j], a0s[wave * ldk + j], a.wthru);
    }
    if (a.dbg != nullptr) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    SKF_STAMP(10);
}

// One 16 x 16 tile of one layer's gradient [N][K + 1] (column K = bias) per workgroup; the 4
// waves split the minibatch rows, partial tiles summed in wave order, Adam in the epilogue.
__global__ void __launch_bounds__(256) skf_wgrad_adam_kernel(SkfArgs a) {
    __shared__ double part[4][64][4];
    __shared__ double sq_s;
#ifdef SKF_WG_XCD
    // (A/B) XCD-grouped tiles: the dispatcher deals linear workgroup ids round-robin over the 8
    // XCDs; remap so each XCD gets a contiguous trial-major range (one trial's tiles share their
    // activation / delta columns in that XCD's L2).  Only the workgroup -> tile map changes.
    // Not the default: -2.5 % per step with every trial active, +7 % on the [H] sweep, where converged
    // trials' workgroups exit at once and leave their XCDs idle (profiles/sk_wgrad_xcd_r6_rejected.log).
    const int gx = gridDim.x, nwg = gx * gridDim.y, hw = blockIdx.x + blockIdx.y * gx;
    const int q = nwg / 8, r = nwg % 8, xcd = hw % 8;
    const int lin = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + hw / 8;
    const int t = lin / gx;
#else
    const int t = blockIdx.y;
#endif
    if (a.active[t] == 0) return;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int lr = lane & 15, lg = lane >> 4;
    // which layer / tile
#ifdef SKF_WG_XCD
    int id = lin % gx, l = 0;
#else
    int id = blockIdx.x, l = 0;
#endif
    for (; l < a.L - 1; ++l) {
        const int n_t = ((a.dims[l + 1] + 15) >> 4) * ((a.dims[l] + 1 + 15) >> 4);
        if (id < n_t) break;
        id -= n_t;
    }
    const int K = a.dims[l], N = a.dims[l + 1];
    const int kts = (K + 1 + 15) >> 4;
    const int n0 = (id / kts) * 16, k0 = (id % kts) * 16;
    const double* dl = a.deltas + ((size_t)l * a.T + t) * a.Bmax * a.maxw;
    const double* in = l == 0 ? a.xg + (size_t)t * a.Bmax * K : a.acts + ((size_t)(l - 1) * a.T + t) * a.Bmax * a.maxw;
    const int ldi = l == 0 ? K : a.maxw;
    // rows of this wave
    const int rw = (((a.rows + 3) / 4) + 3) & ~3;
    const int rb = wave * rw, re = min(a.rows, rb + rw);
    // wave 0 runs the Adam epilogue: its parameters' p, m, v are loaded now, in flight with the
    // operand loads (D reg j of lane l = D[(l >> 4) + 4j][l & 15])
    double* P = a.params + (size_t)t * a.P;
    double* M = a.m + (size_t)t * a.P;
    double* V = a.v + (size_t)t * a.P;
    double pp[4], pm[4], pv[4];
    size_t pidx[4];
    bool pok[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int nn = n0 + lg + 4 * j, kk = k0 + lr;
        pok[j] = wave == 0 && nn < N && kk <= K;
        pidx[j] = kk < K ? (size_t)a.w_off[l] + (size_t)nn * K + kk : (size_t)a.b_off[l] + nn;
        pp[j] = pok[j] ? P[pidx[j]] : 0.0;
        pm[j] = pok[j] ? M[pidx[j]] : 0.0;
        pv[j] = pok[j] ? V[pidx[j]] : 0.0;
    }
    skf_f64x4 acc = {0.0, 0.0, 0.0, 0.0};
    const int n = n0 + lr, k = k0 + lr;
    constexpr int SB = 13;  // k-steps (4 rows each) whose operands are in flight together
    // sklearn AdamOptimizer: lr_t = lr sqrt(1 - b2^t) / (1 - b1^t) -- two float64 pow()s, computed
    // by wave 0 while its first operand loads are in flight (after the products they were on the
    // epilogue's critical path)
    double lr_t = 0.0;
    bool have_lr = false;
    for (int s0 = rb; s0 < re; s0 += 4 * SB) {
        double av[SB], bv[SB];
#pragma unroll
        for (int u = 0; u < SB; ++u) {
            const int r = s0 + 4 * u + lg;
            const bool okr = r < re;
            // A(i = n, kk = r) = delta[r][n];  B(kk = r, j = k) = in[r][k] (k == K: the bias's 1)
            av[u] = (okr && n < N) ? dl[(size_t)r * a.maxw + n] : 0.0;
            bv[u] = (okr && k < K) ? in[(size_t)r * ldi + k] : ((okr && k == K) ? 1.0 : 0.0);
        }
        if (!have_lr) {
            have_lr = true;
            if (wave == 0) {
                const double step = (double)a.step[t];
                lr_t = a.lr[t] * sqrt(1.0 - pow(a.beta2, step)) / (1.0 - pow(a.beta1, step));
            }
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int u = 0; u < SB; ++u) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[u], bv[u], acc, 0, 0, 0);
    }
    if (!have_lr && wave == 0) {  // (a wave without rows)
        const double step = (double)a.step[t];
        lr_t = a.lr[t] * sqrt(1.0 - pow(a.beta2, step)) / (1.0 - pow(a.beta1, step));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) part[wave][lane][j] = acc[j];
    __syncthreads();
    if (wave != 0) return;
    double g4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) g4[j] = ((part[0][lane][j] + part[1][lane][j]) + part[2][lane][j]) + part[3][lane][j];
    const double wdec = a.alpha * a.inv_rows;
    const bool coef = k0 + lr < K;   // a coefficient (not a bias): L2 term, and its loss
    double sq = 0.0;
    // every update computed before the first store, the stores back to back (computed between the
    // stores, each update waited for the previous one's: 0.4-0.7 us per step, profiles/sk_tile_split_ab_r6.log)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        double p = pp[j], g = g4[j];
        if (coef && pok[j]) {
            sq += p * p;
            g += wdec * p;
        }
        const double m = a.beta1 * pm[j] + (1.0 - a.beta1) * g;
        const double v = a.beta2 * pv[j] + (1.0 - a.beta2) * g * g;
        pm[j] = m;
        pv[j] = v;
        pp[j] = p - lr_t * m / (sqrt(v) + a.eps);
    }
    sq = skf_wave_sum(sq);
    double* wtl = a.wt != nullptr && coef ? a.wt + (size_t)t * a.P + a.w_off[l] + (size_t)(k0 + lr) * N + n0 + lg : nullptr;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (!pok[j]) continue;
        M[pidx[j]] = pm[j];
        V[pidx[j]] = pv[j];
        P[pidx[j]] = pp[j];
        if (wtl != nullptr) wtl[4 * j] = pp[j];   // the transposed copy the forward reads
    }
    if (lane == 0 && a.l2_coef != 0.0) atomicAdd(&a.loss_acc[t], a.l2_coef * sq);
}

int skf_wgrad_tiles(const SkfArgs& a) {
    int n = 0;
    for (int l = 0; l < a.L; ++l) n += ((a.dims[l + 1] + 15) / 16) * ((a.dims[l] + 1 + 15) / 16);
    return n;
}

bool skf_supported(const SkfArgs& a) {
    if (a.L < 1 || a.L > SKF_MAXL) return false;
    if (a.dims[a.L] > 16) return false;                // one head tile
    if (skf_lds_bytes(a) > 160 * 1024) return false;   // CDNA4 LDS per workgroup
    if (a.split > 1) {                                 // tile split: two hidden layers, narrow head
        if (a.L != 3 || a.dims[a.L] > SKF_NARROW) return false;
        if (skf_cs_bwd_lds(a) > 160 * 1024) return false;
    }
    return true;
}

// The dynamic-LDS limit is a per-device attribute of the row-pass kernel, raised to the largest
// size any trainer on the device needs.  Called by every fused trainer at construction -- not from
// inside a stream capture, where the attribute call would invalidate the capture -- and guarded:
// the [H] sweep builds and runs trainers from several host threads at once.
hipError_t skf_prepare(const SkfArgs& a) {
    static std::mutex mu;
    static size_t lds_set[64] = {};
    const size_t lds = std::max(skf_lds_bytes(a), a.split > 1 ? skf_cs_bwd_lds(a) : (size_t)0);
    if (lds <= 64 * 1024) return hipSuccess;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    std::lock_guard<std::mutex> g(mu);
    if (lds <= lds_set[dev]) return hipSuccess;
    const void* ks[] = {reinterpret_cast<const void*>(skf_rowpass_kernel), reinterpret_cast<const void*>(skf_cs_fwd_kernel),
                        reinterpret_cast<const void*>(skf_cs_bwd_kernel)};
    for (const void* k : ks) {
        const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    lds_set[dev] = lds;
    return hipSuccess;
}

hipError_t skf_step_launch(const SkfArgs& a, hipStream_t s) {
    if (!skf_supported(a) || a.rows < 1 || a.rows > a.Bmax) return hipErrorInvalidValue;
    const size_t lds = skf_lds_bytes(a);
    // normally a no-op: the trainer raised the limit when it was built (skf_prepare), outside
    // any stream capture
    if (lds > 64 * 1024) {
        const hipError_t e = skf_prepare(a);
        if (e != hipSuccess) return e;
    }
    const int nrb = (a.rows + SKF_RB - 1) / SKF_RB;
    if (a.split > 1) {
        if (skf_cs_bwd_lds(a) > 64 * 1024) {
            const hipError_t e = skf_prepare(a);
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL(skf_cs_fwd_kernel, dim3(nrb, a.split, a.T), dim3(SKF_WAVES * 64), lds, s, a);
        hipLaunchKernelGGL(skf_cs_bwd_kernel, dim3(nrb, a.split, a.T), dim3(SKF_WAVES * 64), skf_cs_bwd_lds(a), s, a);
    } else {
        hipLaunchKernelGGL(skf_rowpass_kernel, dim3(nrb, a.T), dim3(SKF_WAVES * 64), lds, s, a);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(skf_wgrad_adam_kernel, dim3(skf_wgrad_tiles(a), a.T), dim3(256), 0, s, a);
    return hipGetLastError();
}
