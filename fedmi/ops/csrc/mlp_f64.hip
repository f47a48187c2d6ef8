// float64 kernels of the layered minibatch trainer (sklearn numerics on the GPU).
//
// The [S] / [H] reference estimators are scikit-learn MLPClassifiers, which train in float64
// (FL_SkLearn_MLPClassifier_Limitation.py:77-84, hyperparameters_tuning.py:90-91; sklearn's
// _multilayer_perceptron.py keeps X, the coefficients and the Adam state in float64).  These
// kernels give MLPTrainer (mlp_trainer.cpp) a dtype=float64 mode so the HIP backend follows
// sklearn to ~1e-12 instead of fp32's ~1e-4 drift over hundreds of epochs:
//   * GEMMs on v_mfma_f64_16x16x4_f64 (64x64 tile, 4 waves of 32x32, BK 16, double-buffered
//     LDS, the fp32/bf16 kernel's operand staging and epilogues: bias, bias+ReLU, ReLU mask);
//   * minibatch gather, loss heads (softmax / sklearn binary log-loss), bias column sums and
//     sklearn / torch Adam in double.
// Batched over packed trials (blockIdx.z / y = trial) exactly like the fp32 kernels.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "gemm_mfma.h"
#include "mlp_f64.h"

typedef double f64x4 __attribute__((ext_vector_type(4)));

#define G64_BM 64
#define G64_BK 16
#define G64_LD (G64_BK + 2)   // 16-byte pad per staged row
#define G64_THREADS 256

// 64 x BK tile of operand `src` -> registers (4 doubles per thread), zero outside [rows, kdim).
template <bool KCONTIG>
__device__ __forceinline__ void load_tile64(const double* __restrict__ src, int ld, int rows, int kdim, int row0,
                                            int k0, double (&reg)[4]) {
    const int t = threadIdx.x;
    if (KCONTIG) {
        const int row = t >> 2, kq = (t & 3) * 4;
        const int gr = row0 + row;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int gk = k0 + kq + e;
            const bool ok = gr < rows && gk < kdim;
            const double v = src[(size_t)(ok ? gr : 0) * ld + (ok ? gk : 0)];
            reg[e] = ok ? v : 0.0;
        }
    } else {
        const int k = t >> 4, rq = (t & 15) * 4;
        const int gk = k0 + k;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int gr = row0 + rq + e;
            const bool ok = gr < rows && gk < kdim;
            const double v = src[(size_t)(ok ? gk : 0) * ld + (ok ? gr : 0)];
            reg[e] = ok ? v : 0.0;
        }
    }
}

template <bool KCONTIG>
__device__ __forceinline__ void store_tile64(double* lds, const double (&reg)[4]) {
    const int t = threadIdx.x;
    if (KCONTIG) {
        const int row = t >> 2, kq = (t & 3) * 4;
#pragma unroll
        for (int e = 0; e < 4; ++e) lds[row * G64_LD + kq + e] = reg[e];
    } else {
        const int k = t >> 4, rq = (t & 15) * 4;
#pragma unroll
        for (int e = 0; e < 4; ++e) lds[(rq + e) * G64_LD + k] = reg[e];
    }
}

__device__ __forceinline__ int xcd_remap64(int bid, int nwg) {
    const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

// C[M][N] = epi(alpha * sum_k A(m,k) B(k,n)) (+ beta * C); A/B k-contiguous or not (AK / BK_).
// v_mfma_f64_16x16x4_f64: A lane l = A[l&15][k0 + (l>>4)], B lane l = B[k0 + (l>>4)][l&15];
// D reg j of lane l = D[(l>>4) + 4j][l&15] (the f64 form's own C/D map).
template <bool AK, bool BK_, int EPI>
__global__ void __launch_bounds__(G64_THREADS) gemm_f64_kernel(Gemm64Args g) {
    __shared__ double As[2][G64_BM * G64_LD];
    __shared__ double Bs[2][G64_BM * G64_LD];
    const int mt = (g.M + G64_BM - 1) / G64_BM, nt = (g.N + G64_BM - 1) / G64_BM;
    const int bid = xcd_remap64(blockIdx.x, mt * nt);
    const int m0 = (bid % mt) * G64_BM, n0 = (bid / mt) * G64_BM;
    const int z = blockIdx.z;
    if (g.active != nullptr && g.active[z] == 0) return;
    const double* A = g.A + z * g.sA;
    const double* B = g.B + z * g.sB;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
    const int lr = lane & 15, lg = lane >> 4;
    f64x4 acc[2][2];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) acc[x][y] = (f64x4){0.0, 0.0, 0.0, 0.0};
    double ra[4], rb[4];
    int cur = 0;
    load_tile64<AK>(A, g.lda, g.M, g.K, m0, 0, ra);
    load_tile64<BK_>(B, g.ldb, g.N, g.K, n0, 0, rb);
    store_tile64<AK>(As[0], ra);
    store_tile64<BK_>(Bs[0], rb);
    __syncthreads();
    for (int k0 = 0; k0 < g.K; k0 += G64_BK) {
        const bool more = k0 + G64_BK < g.K;
        if (more) {  // next slab's loads in flight during this slab's MFMAs
            load_tile64<AK>(A, g.lda, g.M, g.K, m0, k0 + G64_BK, ra);
            load_tile64<BK_>(B, g.ldb, g.N, g.K, n0, k0 + G64_BK, rb);
        }
        const double* as = As[cur];
        const double* bs = Bs[cur];
#pragma unroll
        for (int s = 0; s < G64_BK / 4; ++s) {
            double a[2], b[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                a[i] = as[(wm + 16 * i + lr) * G64_LD + 4 * s + lg];
                b[i] = bs[(wn + 16 * i + lr) * G64_LD + 4 * s + lg];
            }
#pragma unroll
            for (int x = 0; x < 2; ++x)
#pragma unroll
                for (int y = 0; y < 2; ++y) acc[x][y] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[x], b[y], acc[x][y], 0, 0, 0);
        }
        if (more) {
            store_tile64<AK>(As[cur ^ 1], ra);
            store_tile64<BK_>(Bs[cur ^ 1], rb);
        }
        __syncthreads();
        cur ^= 1;
    }
    double* C = g.C + z * g.sC;
    const double* bias = g.bias != nullptr ? g.bias + z * g.sBias : nullptr;
    const double* mask = g.mask != nullptr ? g.mask + z * g.sMask : nullptr;
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) {
            const int n = n0 + wn + 16 * y + lr;
            if (n >= g.N) continue;
            const double bv = (EPI == GEMM_EPI_BIAS || EPI == GEMM_EPI_BIAS_RELU) ? bias[n] : 0.0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int m = m0 + wm + 16 * x + lg + 4 * j;
                if (m >= g.M) continue;
                double v = acc[x][y][j] * g.alpha;
                if (EPI == GEMM_EPI_BIAS || EPI == GEMM_EPI_BIAS_RELU) v += bv;
                if (EPI == GEMM_EPI_BIAS_RELU) v = v > 0.0 ? v : 0.0;
                if (EPI == GEMM_EPI_MASK) v = mask[(size_t)m * g.ldmask + n] > 0.0 ? v : 0.0;
                const size_t off = (size_t)m * g.ldc + n;
                if (g.beta != 0.0) v += g.beta * C[off];
                C[off] = v;
            }
        }
}

template <bool AK, bool BK_>
static hipError_t launch64(const Gemm64Args& g, int epi, int batch, hipStream_t s) {
    const int mt = (g.M + G64_BM - 1) / G64_BM, nt = (g.N + G64_BM - 1) / G64_BM;
    const dim3 grid(mt * nt, 1, batch);
    switch (epi) {
        case GEMM_EPI_NONE: hipLaunchKernelGGL((gemm_f64_kernel<AK, BK_, GEMM_EPI_NONE>), grid, dim3(G64_THREADS), 0, s, g); break;
        case GEMM_EPI_BIAS: hipLaunchKernelGGL((gemm_f64_kernel<AK, BK_, GEMM_EPI_BIAS>), grid, dim3(G64_THREADS), 0, s, g); break;
        case GEMM_EPI_BIAS_RELU:
            hipLaunchKernelGGL((gemm_f64_kernel<AK, BK_, GEMM_EPI_BIAS_RELU>), grid, dim3(G64_THREADS), 0, s, g);
            break;
        case GEMM_EPI_MASK: hipLaunchKernelGGL((gemm_f64_kernel<AK, BK_, GEMM_EPI_MASK>), grid, dim3(G64_THREADS), 0, s, g); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t gemm_f64_launch(const Gemm64Args& g, int a_kcontig, int b_kcontig, int epi, int batch, hipStream_t s) {
    if (g.M <= 0 || g.N <= 0 || g.K <= 0 || batch < 1) return hipErrorInvalidValue;
    if (a_kcontig && b_kcontig) return launch64<true, true>(g, epi, batch, s);
    if (a_kcontig && !b_kcontig) return launch64<true, false>(g, epi, batch, s);
    if (!a_kcontig && !b_kcontig) return launch64<false, false>(g, epi, batch, s);
    return launch64<false, true>(g, epi, batch, s);
}

// ---------------------------------------------------------------------------------------
// Minibatch gather (rows perm[epoch][off + i] -> out[i][:F], zero padded to ldo; labels).
__global__ void gather_rows_f64_kernel(const double* __restrict__ X, int ld, const int* __restrict__ y,
                                       const int* __restrict__ perms, const int* __restrict__ epoch_ctr,
                                       long long n_perm, int off, int M, int F, double* __restrict__ out, int ldo,
                                       int* __restrict__ yb) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= M * ldo) return;
    const int i = e / ldo, f = e - i * ldo;
    const int* perm = perms + (epoch_ctr != nullptr ? (long long)(*epoch_ctr) * n_perm : 0);
    const int src = perms != nullptr ? perm[off + i] : off + i;
    out[e] = f < F ? X[(size_t)src * ld + f] : 0.0;
    if (f == 0 && yb != nullptr) yb[i] = y[src];
}

hipError_t gather_rows_f64_launch(const double* X, int ld, const int* y, const int* perms, const int* epoch_ctr,
                                  long long n_perm, int off, int M, int F, double* out, int ldo, int* yb,
                                  hipStream_t s) {
    const int n = M * ldo;
    hipLaunchKernelGGL(gather_rows_f64_kernel, dim3((n + 255) / 256), dim3(256), 0, s, X, ld, y, perms, epoch_ctr,
                       n_perm, off, M, F, out, ldo, yb);
    return hipGetLastError();
}

// Output head in double: mode 0 softmax + log-loss; mode 1 sklearn binary head (logistic,
// probabilities clipped to [eps, 1 - eps] with eps = float64 machine epsilon, as sklearn
// clips them in the dtype of the data).  dz = (p - onehot) * scale; loss_acc[t] += row losses.
__global__ void __launch_bounds__(256)
xent_f64_kernel(const double* __restrict__ z, int ldz, long long sZ, const int* __restrict__ y, int M, int C, int mode,
                double scale, double* __restrict__ dz, int lddz, long long sDz, double* __restrict__ loss_acc,
                const int* __restrict__ active) {
    __shared__ double red[256];
    const int t = blockIdx.y;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    double lrow = 0.0;
    const bool run = active == nullptr || active[t] != 0;
    if (run && i < M) {
        const double* zr = z + t * sZ + (size_t)i * ldz;
        double* dr = dz + t * sDz + (size_t)i * lddz;
        const int yy = y[i];
        if (mode == 1) {
            const double p = 1.0 / (1.0 + exp(-zr[0]));
            const double eps = 2.220446049250313e-16;
            const double pc = fmin(fmax(p, eps), 1.0 - eps);
            lrow = yy ? -log(pc) : -log(1.0 - pc);
            dr[0] = (p - (double)yy) * scale;
        } else {
            double mx = zr[0];
            for (int k = 1; k < C; ++k) mx = fmax(mx, zr[k]);
            double se = 0.0;
            for (int k = 0; k < C; ++k) se += exp(zr[k] - mx);
            // sklearn multinomial log-loss on the clipped softmax probability of the true class
            const double eps = 2.220446049250313e-16;
            const double py = fmin(fmax(exp(zr[yy] - mx) / se, eps), 1.0 - eps);
            lrow = -log(py);
            for (int k = 0; k < C; ++k) dr[k] = (exp(zr[k] - mx) / se - (k == yy ? 1.0 : 0.0)) * scale;
        }
    }
    red[threadIdx.x] = lrow;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0 && run && loss_acc != nullptr) atomicAdd(&loss_acc[t], red[0]);
}

hipError_t xent_f64_launch(const double* z, int ldz, long long sZ, const int* y, int M, int C, int mode, double scale,
                           double* dz, int lddz, long long sDz, double* loss_acc, const int* active, int T,
                           hipStream_t s) {
    hipLaunchKernelGGL(xent_f64_kernel, dim3((M + 255) / 256, T), dim3(256), 0, s, z, ldz, sZ, y, M, C, mode, scale,
                       dz, lddz, sDz, loss_acc, active);
    return hipGetLastError();
}

// Bias gradient: out[n] = beta*out[n] + sum_m X[m][n] (16 waves split the rows, fixed-order fold).
__global__ void __launch_bounds__(1024) colsum_f64_kernel(const double* __restrict__ X, int M, int N, int ld,
                                                          double* __restrict__ out, double beta, long long sX,
                                                          long long sOut, const int* __restrict__ active) {
    __shared__ double part[16][64];
    const int t = blockIdx.y;
    if (active != nullptr && active[t] == 0) return;
    X += t * sX;
    out += t * sOut;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int n = blockIdx.x * 64 + lane;
    double s = 0.0;
    if (n < N)
        for (int m = wave; m < M; m += 16) s += X[(size_t)m * ld + n];
    part[wave][lane] = s;
    __syncthreads();
    if (wave == 0 && n < N) {
        double v = 0.0;
#pragma unroll
        for (int w = 0; w < 16; ++w) v += part[w][lane];
        out[n] = (beta != 0.0 ? beta * out[n] : 0.0) + v;
    }
}

hipError_t colsum_f64_launch(const double* X, int M, int N, int ld, double* out, double beta, int batch, long long sX,
                             long long sOut, const int* active, hipStream_t s) {
    hipLaunchKernelGGL(colsum_f64_kernel, dim3((N + 63) / 64, batch), dim3(1024), 0, s, X, M, N, ld, out, beta, sX,
                       sOut, active);
    return hipGetLastError();
}

// Adam over [T][n] float64 parameters: style 1 sklearn AdamOptimizer (lr_t = lr sqrt(1-b2^t) /
// (1-b1^t), p -= lr_t m / (sqrt(v) + eps)); style 0 torch.optim.Adam.  L2 (sklearn: alpha/batch
// on the coefficients, wd_mask) and its loss term 0.5*alpha*sum(coef^2) of the pre-update weights.
__global__ void __launch_bounds__(256) adam_f64_kernel(Adam64Args a) {
    __shared__ double red[256];
    __shared__ double coef[2];
    const int t = blockIdx.y;
    const bool run = a.active == nullptr || a.active[t] != 0;
    if (threadIdx.x == 0) {
        const long long step = a.step[t];
        const double lr = a.lr[t];
        if (a.style == 0) {
            coef[0] = lr / (1.0 - pow(a.beta1, (double)step));
            coef[1] = sqrt(1.0 - pow(a.beta2, (double)step));
        } else {
            coef[0] = lr * sqrt(1.0 - pow(a.beta2, (double)step)) / (1.0 - pow(a.beta1, (double)step));
            coef[1] = 0.0;
        }
    }
    __syncthreads();
    const double c0 = coef[0], c1 = coef[1];
    double sq = 0.0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; run && i < a.n; i += (size_t)gridDim.x * blockDim.x) {
        const size_t j = (size_t)t * a.n + i;
        double p = a.p[j], g = a.g[j];
        if (a.wd_mask == nullptr || a.wd_mask[i] != 0) {
            sq += p * p;
            if (a.wd != 0.0) g += a.wd * p;
        }
        if (a.mu != 0.0) g += a.mu * (p - a.anchor[j]);
        double m = a.m[j], v = a.v[j];
        m = a.beta1 * m + (1.0 - a.beta1) * g;
        v = a.beta2 * v + (1.0 - a.beta2) * g * g;
        if (a.style == 0) p = p - c0 * m / (sqrt(v) / c1 + a.eps);
        else p = p - c0 * m / (sqrt(v) + a.eps);
        a.m[j] = m;
        a.v[j] = v;
        a.p[j] = p;
    }
    if (a.loss_acc == nullptr || a.l2_coef == 0.0) return;
    red[threadIdx.x] = sq;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0 && run) atomicAdd(&a.loss_acc[t], a.l2_coef * red[0]);
}

hipError_t adam_f64_launch(const Adam64Args& a, int T, hipStream_t s) {
    const unsigned blocks = (unsigned)std::min<size_t>(1024, (a.n + 255) / 256);
    hipLaunchKernelGGL(adam_f64_kernel, dim3(blocks, T), dim3(256), 0, s, a);
    return hipGetLastError();
}
