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
#include <math.h>
#include <stdint.h>

#include "mlp_f64.h"

typedef double skf_f64x4 __attribute__((ext_vector_type(4)));

#define SKF_RB 16          // rows per row block (the MFMA's M)
#define SKF_WAVES 16       // waves of a row block
#define SKF_KB 16          // k-steps (of 4) whose weight operands one wave loads at once
#define SKF_NARROW 4       // output layers at most this wide run on the VALU
static_assert(SKF_WAVES == SKF_RB, "skf_fwd_narrow: one wave per row");

__device__ __forceinline__ int skf_np(int n) { return (n + 15) & ~15; }
// LDS row stride (doubles) of a buffer with np (multiple of 16) columns: np = 2 (mod 32), so the
// MFMA operand reads (16 rows x 4 consecutive columns per wave) hit distinct banks
__host__ __device__ __forceinline__ int skf_ld(int np) { return np + 2 + ((np & 16) ? 16 : 0); }

size_t skf_lds_bytes(const SkfArgs& a) {
    size_t d = (size_t)skf_ld((a.dims[0] + 15) & ~15);
    for (int l = 0; l < a.L; ++l) d += (size_t)skf_ld((a.dims[l + 1] + 15) & ~15);
    return d * SKF_RB * sizeof(double);
}

__device__ __forceinline__ double skf_wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// out[16][N] (ld_o) = act(in[16][K] (ld_i) . W^T + b): 16-column tiles round-robin over the
// waves, k-steps in batches of SKF_KB whose 8-byte weight loads are all in flight together.
__device__ __forceinline__ void skf_fwd_mfma(const double* __restrict__ in, int ld_i, double* __restrict__ out,
                                             int ld_o, const double* __restrict__ W, const double* __restrict__ bias,
                                             int K, int N, bool relu, int wave, int lane) {
    const int steps = (K + 3) >> 2, nt_all = (N + 15) >> 4;
    const int lr = lane & 15, lg = lane >> 4;
    for (int nt = wave; nt < nt_all; nt += SKF_WAVES) {
        const int n = nt * 16 + lr;
        skf_f64x4 acc = {0.0, 0.0, 0.0, 0.0};
        for (int s0 = 0; s0 < steps; s0 += SKF_KB) {
            double bw[SKF_KB];
#pragma unroll
            for (int u = 0; u < SKF_KB; ++u) {
                const int k = 4 * (s0 + u) + lg;
                const bool ok = n < N && k < K;
                bw[u] = ok ? W[(size_t)n * K + k] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < SKF_KB; ++u)
                if (s0 + u < steps) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(in[lr * ld_i + 4 * (s0 + u) + lg], bw[u], acc, 0, 0, 0);
        }
        // D reg j of lane l = D[(l >> 4) + 4j][l & 15]
        const double bv = n < N ? bias[n] : 0.0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            double v = acc[j] + bv;
            if (relu) v = v > 0.0 ? v : 0.0;
            out[(lg + 4 * j) * ld_o + n] = n < N ? v : 0.0;
        }
    }
}

// Narrow output layer (N <= SKF_NARROW) on the VALU: wave w = row w, lanes split k, one
// deterministic xor-tree sum per output.
__device__ __forceinline__ void skf_fwd_narrow(const double* __restrict__ in, int ld_i, double* __restrict__ out,
                                               int ld_o, const double* __restrict__ W, const double* __restrict__ bias,
                                               int K, int N, int wave, int lane) {
    const int r = wave;  // SKF_WAVES == SKF_RB
    for (int c = 0; c < N; ++c) {
        double s = 0.0;
        for (int k = lane; k < K; k += 64) s += in[r * ld_i + k] * W[(size_t)c * K + k];
        s = skf_wave_sum(s);
        if (lane == 0) out[r * ld_o + c] = s + bias[c];
    }
    if (lane < skf_np(N) && lane >= N) out[r * ld_o + lane] = 0.0;
}

// dIn[16][K] = (d[16][N] . W[N][K]) * (a[16][K] > 0), written over a (in place: the lane that
// reads an activation for its mask is the lane that overwrites it).
__device__ __forceinline__ void skf_bwd_mfma(const double* __restrict__ d, int ld_d, double* __restrict__ a, int ld_a,
                                             const double* __restrict__ W, int K, int N, int wave, int lane) {
    const int steps = (N + 3) >> 2, kt_all = (K + 15) >> 4;
    const int lr = lane & 15, lg = lane >> 4;
    for (int kt = wave; kt < kt_all; kt += SKF_WAVES) {
        const int k = kt * 16 + lr;
        skf_f64x4 acc = {0.0, 0.0, 0.0, 0.0};
        for (int s0 = 0; s0 < steps; s0 += SKF_KB) {
            double bw[SKF_KB];
#pragma unroll
            for (int u = 0; u < SKF_KB; ++u) {
                const int n = 4 * (s0 + u) + lg;
                const bool ok = n < N && k < K;
                bw[u] = ok ? W[(size_t)n * K + k] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < SKF_KB; ++u)
                if (s0 + u < steps) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(d[lr * ld_d + 4 * (s0 + u) + lg], bw[u], acc, 0, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            double* p = a + (lg + 4 * j) * ld_a + k;
            const double m = *p;
            *p = (k < K && m > 0.0) ? acc[j] : 0.0;
        }
    }
}

// Backward through a narrow layer (N <= SKF_NARROW): every thread owns (row, k) elements.
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

__global__ void __launch_bounds__(SKF_WAVES * 64) skf_rowpass_kernel(SkfArgs a) {
    extern __shared__ double lds[];
    __shared__ int ys[SKF_RB];
    const int t = blockIdx.y;
    if (a.active[t] == 0) return;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int r0 = blockIdx.x * SKF_RB;
    const int nr = min(SKF_RB, a.rows - r0);
    if (blockIdx.x == 0 && threadIdx.x == 0) a.step[t] += 1;  // this minibatch's Adam step t
    const double* P = a.params + (size_t)t * a.P;
    // LDS: buffer 0 = the rows' inputs, buffer l + 1 = layer l's output (then its delta); offsets
    // recomputed from the (uniform) dims instead of a dynamically indexed array (scratch)
    auto ldof = [&](int l) { return skf_ld(skf_np(a.dims[l])); };
    auto bufp = [&](int l) {
        int o = 0;
        for (int i = 0; i < l; ++i) o += ldof(i) * SKF_RB;
        return lds + o;
    };
    // gather through the epoch permutation (sklearn: X[sample_idx[batch_slice]])
    const int F = a.dims[0], fp = skf_np(F);
    const int* perm = a.perms + (size_t)(*a.epoch_ctr) * a.n_perm + a.off + r0;
    double* xg = a.xg + ((size_t)t * a.Bmax + r0) * F;
    for (int e = threadIdx.x; e < SKF_RB * fp; e += blockDim.x) {
        const int r = e / fp, f = e - r * fp;
        double v = 0.0;
        if (r < nr && f < F) {
            v = a.X[(size_t)perm[r] * F + f];
            xg[(size_t)r * F + f] = v;
        }
        bufp(0)[r * ldof(0) + f] = v;
    }
    if (threadIdx.x < SKF_RB) ys[threadIdx.x] = threadIdx.x < nr ? a.y[perm[threadIdx.x]] : 0;
    __syncthreads();
    // forward
    for (int l = 0; l < a.L; ++l) {
        const int K = a.dims[l], N = a.dims[l + 1];
        const double* W = P + a.w_off[l];
        const double* b = P + a.b_off[l];
        if (l == a.L - 1 && N <= SKF_NARROW)
            skf_fwd_narrow(bufp(l), ldof(l), bufp(l + 1), ldof(l + 1), W, b, K, N, wave, lane);
        else
            skf_fwd_mfma(bufp(l), ldof(l), bufp(l + 1), ldof(l + 1), W, b, K, N, l + 1 < a.L, wave, lane);
        __syncthreads();
        if (l + 1 < a.L) {  // hidden activation: the next layer's wgrad operand (kernel 2)
            double* ag = a.acts + (((size_t)l * a.T + t) * a.Bmax + r0) * a.maxw;
            for (int e = threadIdx.x; e < nr * N; e += blockDim.x) {
                const int r = e / N, c = e - r * N;
                ag[(size_t)r * a.maxw + c] = bufp(l + 1)[r * ldof(l + 1) + c];
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
        __syncthreads();
        double* dg = a.deltas + (((size_t)(a.L - 1) * a.T + t) * a.Bmax + r0) * a.maxw;
        for (int e = threadIdx.x; e < nr * C; e += blockDim.x) {
            const int r = e / C, c = e - r * C;
            dg[(size_t)r * a.maxw + c] = z[r * ldz + c];
        }
    }
    // backward: delta of layer l - 1 from layer l's, over the activation it masks
    for (int l = a.L - 1; l >= 1; --l) {
        const int K = a.dims[l], N = a.dims[l + 1];
        const double* W = P + a.w_off[l];
        if (N <= SKF_NARROW)
            skf_bwd_narrow(bufp(l + 1), ldof(l + 1), bufp(l), ldof(l), W, K, N);
        else
            skf_bwd_mfma(bufp(l + 1), ldof(l + 1), bufp(l), ldof(l), W, K, N, wave, lane);
        __syncthreads();
        double* dg = a.deltas + (((size_t)(l - 1) * a.T + t) * a.Bmax + r0) * a.maxw;
        for (int e = threadIdx.x; e < nr * K; e += blockDim.x) {
            const int r = e / K, c = e - r * K;
            dg[(size_t)r * a.maxw + c] = bufp(l)[r * ldof(l) + c];
        }
    }
}

// One 16 x 16 tile of one layer's gradient [N][K + 1] (column K = bias) per workgroup; the 4
// waves split the minibatch rows, partial tiles summed in wave order, Adam in the epilogue.
__global__ void __launch_bounds__(256) skf_wgrad_adam_kernel(SkfArgs a) {
    __shared__ double part[4][64][4];
    __shared__ double sq_s;
    const int t = blockIdx.y;
    if (a.active[t] == 0) return;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int lr = lane & 15, lg = lane >> 4;
    // which layer / tile
    int id = blockIdx.x, l = 0;
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
    skf_f64x4 acc = {0.0, 0.0, 0.0, 0.0};
    const int n = n0 + lr, k = k0 + lr;
    constexpr int SB = 13;  // k-steps (4 rows each) whose operands are in flight together
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
#pragma unroll
        for (int u = 0; u < SB; ++u) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[u], bv[u], acc, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) part[wave][lane][j] = acc[j];
    __syncthreads();
    if (wave != 0) return;
    double g4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) g4[j] = ((part[0][lane][j] + part[1][lane][j]) + part[2][lane][j]) + part[3][lane][j];
    // sklearn AdamOptimizer: lr_t = lr sqrt(1 - b2^t) / (1 - b1^t)
    const double step = (double)a.step[t];
    const double lr_t = a.lr[t] * sqrt(1.0 - pow(a.beta2, step)) / (1.0 - pow(a.beta1, step));
    const double wdec = a.alpha * a.inv_rows;
    double sq = 0.0;
    double* P = a.params + (size_t)t * a.P;
    double* M = a.m + (size_t)t * a.P;
    double* V = a.v + (size_t)t * a.P;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int nn = n0 + lg + 4 * j, kk = k0 + lr;  // D reg j of lane l = D[(l >> 4) + 4j][l & 15]
        if (nn >= N || kk > K) continue;
        const size_t i = kk < K ? (size_t)a.w_off[l] + (size_t)nn * K + kk : (size_t)a.b_off[l] + nn;
        double p = P[i];
        double g = g4[j];
        if (kk < K) {  // coefficient: L2 term, and its loss
            sq += p * p;
            g += wdec * p;
        }
        double m = M[i], v = V[i];
        m = a.beta1 * m + (1.0 - a.beta1) * g;
        v = a.beta2 * v + (1.0 - a.beta2) * g * g;
        p = p - lr_t * m / (sqrt(v) + a.eps);
        M[i] = m;
        V[i] = v;
        P[i] = p;
    }
    sq = skf_wave_sum(sq);
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
    return true;
}

hipError_t skf_step_launch(const SkfArgs& a, hipStream_t s) {
    if (!skf_supported(a) || a.rows < 1 || a.rows > a.Bmax) return hipErrorInvalidValue;
    const size_t lds = skf_lds_bytes(a);
    static size_t lds_set = 0;
    if (lds > 64 * 1024 && lds > lds_set) {
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(skf_rowpass_kernel),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        lds_set = lds;
    }
    hipLaunchKernelGGL(skf_rowpass_kernel, dim3((a.rows + SKF_RB - 1) / SKF_RB, a.T), dim3(SKF_WAVES * 64), lds, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(skf_wgrad_adam_kernel, dim3(skf_wgrad_tiles(a), a.T), dim3(256), 0, s, a);
    return hipGetLastError();
}
