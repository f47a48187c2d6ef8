// Grid-level MFMA GEMMs with fused MLP epilogues for gfx950 (the "layered" path).
//
// The fused round engine (fl_kernels.hip) keeps a whole small MLP in one workgroup's LDS.
// Wider models (sklearn configs up to 400 units, the north-star 4096-wide MLP) and
// minibatch training run layer by layer on these kernels:
//
//   fwd   : Y[M,N]  = act(X[M,K] . W[N,K]^T + b)          bias (+ReLU) epilogue
//   dgrad : dX[M,K] = (dY[M,N] . W[N,K]) * (A[M,K] > 0)    ReLU-mask epilogue
//   wgrad : dW[N,K] = dY^T . X  (split-K over M into fp32 slabs, fixed-order reduce)
//
// One templated kernel: C[M][N] = sum_k A(m,k) B(k,n), where each operand is read either
// k-contiguous or m/n-contiguous from global memory and always staged into LDS
// k-contiguous, so MFMA fragments are 16-byte LDS reads.  Tile 64x64, 4 waves of 32x32
// (2x2 16x16 MFMA tiles), double-buffered LDS with the next k-slab's global loads issued
// before the current slab's MFMAs.  Inputs are fp32 (v_mfma_f32_16x16x4_f32, exact fp32)
// or bf16 (v_mfma_f32_16x16x32_bf16, fp32 accumulate).  Grid blocks are remapped so the
// tiles of one 8-block group share an XCD (L2 locality, T1 in the CDNA guide).
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#include "gemm_mfma.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

#define GT_BM 64
#define GT_BN 64
#define GT_THREADS 256

template <typename T> struct KStep;
template <> struct KStep<float> { static constexpr int BK = 16; };
template <> struct KStep<__hip_bfloat16> { static constexpr int BK = 32; };

__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(__hip_bfloat16 x) { return __bfloat162float(x); }
__device__ __forceinline__ short bf_bits(float x) {
    __hip_bfloat16 h = __float2bfloat16(x);
    return *reinterpret_cast<short*>(&h);
}

// LDS row stride (elements) of a k-contiguous staged tile: BK + one 16-byte pad.
template <typename T> __host__ __device__ constexpr int lds_ld() { return KStep<T>::BK + 16 / (int)sizeof(T); }

// Stage a 64 x BK tile of operand `src` into LDS as [row][k] (k contiguous).
// KCONTIG: element (row, k) at src[row*ld + k]; else at src[k*ld + row].
template <typename T, bool KCONTIG>
__device__ __forceinline__ void load_tile(const T* __restrict__ src, int ld, int rows, int kdim, int row0, int k0,
                                          T (&reg)[KStep<T>::BK * 64 / GT_THREADS]) {
    constexpr int BK = KStep<T>::BK;
    constexpr int PER = BK * 64 / GT_THREADS;  // elements per thread: 4 (f32) / 8 (bf16)
    const int t = threadIdx.x;
    if (KCONTIG) {
        // thread -> (row, k-group of PER)
        const int row = t / (BK / PER), kq = (t % (BK / PER)) * PER;
        const int gr = row0 + row;
#pragma unroll
        for (int e = 0; e < PER; ++e) {
            const int gk = k0 + kq + e;
            const bool ok = gr < rows && gk < kdim;
            const T v = src[(size_t)(ok ? gr : 0) * ld + (ok ? gk : 0)];
            reg[e] = ok ? v : T(0.f);
        }
    } else {
        // thread -> (k, row-group of PER): coalesced along rows
        const int k = t / (64 / PER), rq = (t % (64 / PER)) * PER;
        const int gk = k0 + k;
#pragma unroll
        for (int e = 0; e < PER; ++e) {
            const int gr = row0 + rq + e;
            const bool ok = gr < rows && gk < kdim;
            const T v = src[(size_t)(ok ? gk : 0) * ld + (ok ? gr : 0)];
            reg[e] = ok ? v : T(0.f);
        }
    }
}

template <typename T, bool KCONTIG>
__device__ __forceinline__ void store_tile(T* lds, const T (&reg)[KStep<T>::BK * 64 / GT_THREADS]) {
    constexpr int BK = KStep<T>::BK;
    constexpr int PER = BK * 64 / GT_THREADS;
    constexpr int LD = lds_ld<T>();
    const int t = threadIdx.x;
    if (KCONTIG) {
        const int row = t / (BK / PER), kq = (t % (BK / PER)) * PER;
#pragma unroll
        for (int e = 0; e < PER; ++e) lds[row * LD + kq + e] = reg[e];
    } else {
        const int k = t / (64 / PER), rq = (t % (64 / PER)) * PER;
#pragma unroll
        for (int e = 0; e < PER; ++e) lds[(rq + e) * LD + k] = reg[e];
    }
}

// MFMA over one staged BK slab for the wave's 32x32 sub-tile (2x2 16x16 tiles).
__device__ __forceinline__ void mma_slab(const float* As, const float* Bs, int wm, int wn, f32x4 (&acc)[2][2]) {
    constexpr int LD = lds_ld<float>();
    const int lane = threadIdx.x & 63, lr = lane & 15, lg = lane >> 4;
    float4 a[2], b[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) a[i] = *reinterpret_cast<const float4*>(As + (wm + 16 * i + lr) * LD + 4 * lg);
#pragma unroll
    for (int i = 0; i < 2; ++i) b[i] = *reinterpret_cast<const float4*>(Bs + (wn + 16 * i + lr) * LD + 4 * lg);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int y = 0; y < 2; ++y) {
                const float av = j == 0 ? a[x].x : j == 1 ? a[x].y : j == 2 ? a[x].z : a[x].w;
                const float bv = j == 0 ? b[y].x : j == 1 ? b[y].y : j == 2 ? b[y].z : b[y].w;
                acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[x][y], 0, 0, 0);
            }
}

__device__ __forceinline__ void mma_slab(const __hip_bfloat16* As, const __hip_bfloat16* Bs, int wm, int wn,
                                         f32x4 (&acc)[2][2]) {
    constexpr int LD = lds_ld<__hip_bfloat16>();
    const int lane = threadIdx.x & 63, lr = lane & 15, lg = lane >> 4;
    bf16x8 a[2], b[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) a[i] = *reinterpret_cast<const bf16x8*>(As + (wm + 16 * i + lr) * LD + 8 * lg);
#pragma unroll
    for (int i = 0; i < 2; ++i) b[i] = *reinterpret_cast<const bf16x8*>(Bs + (wn + 16 * i + lr) * LD + 8 * lg);
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[x], b[y], acc[x][y], 0, 0, 0);
}

// Bijective XCD-aware remap of the linear block id (CDNA guide §5 "XCD swizzle").
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
    const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

template <typename T, bool AK, bool BK_, int EPI>
__global__ void __launch_bounds__(GT_THREADS)
gemm_kernel(GemmArgs g) {
    constexpr int BK = KStep<T>::BK;
    constexpr int LD = lds_ld<T>();
    constexpr int PER = BK * 64 / GT_THREADS;
    __shared__ __attribute__((aligned(16))) T As[2][GT_BM * LD];
    __shared__ __attribute__((aligned(16))) T Bs[2][GT_BN * LD];
    const int mt = (g.M + GT_BM - 1) / GT_BM, nt = (g.N + GT_BN - 1) / GT_BN;
    const int nwg = mt * nt;
    const int bid = xcd_remap(blockIdx.x, nwg);
    const int tm = bid % mt, tn = bid / mt;
    const int m0 = tm * GT_BM, n0 = tn * GT_BN;
    // split-K range (blockIdx.y)
    const int ksplit = gridDim.y;
    const int kper = ((g.K + ksplit * BK - 1) / (ksplit * BK)) * BK;
    const int kbeg = blockIdx.y * kper;
    const int kend = min(g.K, kbeg + kper);
    const int z = blockIdx.z;
    if (g.active != nullptr && g.active[z] == 0) return;
    const T* A = reinterpret_cast<const T*>(g.A) + z * g.sA;
    const T* B = reinterpret_cast<const T*>(g.B) + z * g.sB;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
    f32x4 acc[2][2];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) acc[x][y] = (f32x4){0.f, 0.f, 0.f, 0.f};
    T ra[PER], rb[PER];
    int cur = 0;
    if (kbeg < kend) {
        load_tile<T, AK>(A, g.lda, g.M, kend, m0, kbeg, ra);
        load_tile<T, BK_>(B, g.ldb, g.N, kend, n0, kbeg, rb);
        store_tile<T, AK>(As[0], ra);
        store_tile<T, BK_>(Bs[0], rb);
        __syncthreads();
        for (int k0 = kbeg; k0 < kend; k0 += BK) {
            const bool more = k0 + BK < kend;
            if (more) {  // next slab's global loads in flight during this slab's MFMAs
                load_tile<T, AK>(A, g.lda, g.M, kend, m0, k0 + BK, ra);
                load_tile<T, BK_>(B, g.ldb, g.N, kend, n0, k0 + BK, rb);
            }
            mma_slab(As[cur], Bs[cur], wm, wn, acc);
            if (more) {
                store_tile<T, AK>(As[cur ^ 1], ra);
                store_tile<T, BK_>(Bs[cur ^ 1], rb);
            }
            __syncthreads();
            cur ^= 1;
        }
    }
    // epilogue: C/D map col = lane&15, row = 4*(lane>>4) + j
    const int lr = lane & 15, lg = lane >> 4;
    float* C = g.C + (size_t)blockIdx.y * g.slab_stride + z * g.sC;
    const float* bias = g.bias != nullptr ? g.bias + z * g.sBias : nullptr;
    const size_t moff = (size_t)(z * g.sMask);
    __hip_bfloat16* Cb = g.Cbf16 != nullptr ? reinterpret_cast<__hip_bfloat16*>(g.Cbf16) + z * g.sC : nullptr;
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) {
            const int n = n0 + wn + 16 * y + lr;
            if (n >= g.N) continue;
            float bv = 0.f;
            if (EPI == GEMM_EPI_BIAS || EPI == GEMM_EPI_BIAS_RELU) bv = bias[n];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int m = m0 + wm + 16 * x + 4 * lg + j;
                if (m >= g.M) continue;
                float v = acc[x][y][j] * g.alpha;
                if (EPI == GEMM_EPI_BIAS || EPI == GEMM_EPI_BIAS_RELU) v += bv;
                if (EPI == GEMM_EPI_BIAS_RELU) v = fmaxf(v, 0.f);
                if (EPI == GEMM_EPI_MASK) {
                    const size_t mi = moff + (size_t)m * g.ldmask + n;
                    const float a = g.mask_bf16 ? __bfloat162float(reinterpret_cast<const __hip_bfloat16*>(g.mask)[mi])
                                                : reinterpret_cast<const float*>(g.mask)[mi];
                    v = a > 0.f ? v : 0.f;
                }
                const size_t off = (size_t)m * g.ldc + n;
                if (g.beta != 0.f) v += g.beta * C[off];
                C[off] = v;
                if (Cb) Cb[off] = __float2bfloat16(v);
            }
        }
}

// Fixed-order split-K reduction: out[i] = beta*out[i] + sum_s slab[s][i].
__global__ void splitk_reduce_kernel(const float* __restrict__ slab, size_t stride, int splits, float* __restrict__ out,
                                     size_t n, float beta) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float s = 0.f;
    for (int k = 0; k < splits; ++k) s += slab[k * stride + i];
    out[i] = (beta != 0.f ? beta * out[i] : 0.f) + s;
}

// Column sums (bias gradient): out[n] = beta*out[n] + sum_m X[m][n], one wave per 64 columns
// x 16 waves splitting the rows, fixed-order combine.
// Batched over blockIdx.y (problem t: X + t*sX, out + t*sOut, skipped when !active[t]).
__global__ void __launch_bounds__(1024) colsum_kernel(const float* __restrict__ X, int M, int N, int ld,
                                                      float* __restrict__ out, float beta, long long sX,
                                                      long long sOut, const int* __restrict__ active) {
    __shared__ float part[16][64];
    const int t = blockIdx.y;
    if (active != nullptr && active[t] == 0) return;
    X += t * sX;
    out += t * sOut;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int n = blockIdx.x * 64 + lane;
    float s = 0.f;
    if (n < N)
        for (int m = wave; m < M; m += 16) s += X[(size_t)m * ld + n];
    part[wave][lane] = s;
    __syncthreads();
    if (wave == 0 && n < N) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < 16; ++w) t += part[w][lane];
        out[n] = (beta != 0.f ? beta * out[n] : 0.f) + t;
    }
}

// y = bf16(scale * x) (scale 1: plain rounding; the wide FedAvg's bf16 buckets carry the
// n_i / N weight in the same pass)
__global__ void f32_to_bf16_kernel(const float* __restrict__ x, __hip_bfloat16* __restrict__ y, size_t n, float scale) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = __float2bfloat16(x[i] * scale);
}

// bf16 FedAvg buckets that keep the fp32 master (wide client, allreduce_dtype="bf16"): the wire
// carries the scaled DELTA d = bf16(scale * (w_local - w_global_prev)), whose bf16 rounding is
// relative to one round's update instead of to the weight, and the reduced sum is added back
// to the fp32 previous global model: w = g = g + sum_i d_i.  VEC: 4 elements per thread
// (float4 loads, one 8-byte bf16 store; 16/8-byte aligned operands), else one per thread.
template <bool VEC>
__global__ void fedavg_delta_bf16_kernel(const float* __restrict__ w, const float* __restrict__ g,
                                         __hip_bfloat16* __restrict__ d, size_t n, float scale) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t i = VEC ? t * 4 : t;
    if (VEC && i + 4 <= n) {
        const float4 a = *reinterpret_cast<const float4*>(w + i);
        const float4 b = *reinterpret_cast<const float4*>(g + i);
        __hip_bfloat16 o[4] = {__float2bfloat16(scale * (a.x - b.x)), __float2bfloat16(scale * (a.y - b.y)),
                               __float2bfloat16(scale * (a.z - b.z)), __float2bfloat16(scale * (a.w - b.w))};
        *reinterpret_cast<uint2*>(d + i) = *reinterpret_cast<const uint2*>(o);
    } else {
        for (size_t j = i; j < n && j < i + (VEC ? 4 : 1); ++j) d[j] = __float2bfloat16(scale * (w[j] - g[j]));
    }
}

template <bool VEC>
__global__ void fedavg_apply_delta_kernel(float* __restrict__ w, float* __restrict__ g,
                                          const __hip_bfloat16* __restrict__ d, size_t n) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t i = VEC ? t * 4 : t;
    if (VEC && i + 4 <= n) {
        float4 b = *reinterpret_cast<const float4*>(g + i);
        const uint2 raw = *reinterpret_cast<const uint2*>(d + i);
        const __hip_bfloat16* q = reinterpret_cast<const __hip_bfloat16*>(&raw);
        b.x += __bfloat162float(q[0]); b.y += __bfloat162float(q[1]);
        b.z += __bfloat162float(q[2]); b.w += __bfloat162float(q[3]);
        *reinterpret_cast<float4*>(g + i) = b;
        *reinterpret_cast<float4*>(w + i) = b;
    } else {
        for (size_t j = i; j < n && j < i + (VEC ? 4 : 1); ++j) {
            const float v = g[j] + __bfloat162float(d[j]);
            g[j] = v;
            w[j] = v;
        }
    }
}

static bool fedavg_vec_ok(const void* w, const void* g, const void* d) {
    return !((((uintptr_t)w | (uintptr_t)g) & 15) || ((uintptr_t)d & 7));
}

hipError_t fedavg_delta_bf16_launch(const float* w, const float* g, void* d, size_t n, float scale, hipStream_t s) {
    auto* o = reinterpret_cast<__hip_bfloat16*>(d);
    if (fedavg_vec_ok(w, g, d)) {
        const size_t th = (n + 3) / 4;
        hipLaunchKernelGGL(fedavg_delta_bf16_kernel<true>, dim3((unsigned)((th + 255) / 256)), dim3(256), 0, s, w, g,
                           o, n, scale);
    } else {
        hipLaunchKernelGGL(fedavg_delta_bf16_kernel<false>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, w, g,
                           o, n, scale);
    }
    return hipGetLastError();
}

hipError_t fedavg_apply_delta_launch(float* w, float* g, const void* d, size_t n, hipStream_t s) {
    auto* q = reinterpret_cast<const __hip_bfloat16*>(d);
    if (fedavg_vec_ok(w, g, d)) {
        const size_t th = (n + 3) / 4;
        hipLaunchKernelGGL(fedavg_apply_delta_kernel<true>, dim3((unsigned)((th + 255) / 256)), dim3(256), 0, s, w, g,
                           q, n);
    } else {
        hipLaunchKernelGGL(fedavg_apply_delta_kernel<false>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, w, g,
                           q, n);
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
template <typename T, bool AK, bool BK_>
static hipError_t launch_t(const GemmArgs& g, int epi, int splits, int batch, hipStream_t s) {
    const int mt = (g.M + GT_BM - 1) / GT_BM, nt = (g.N + GT_BN - 1) / GT_BN;
    dim3 grid(mt * nt, splits, batch);
    switch (epi) {
        case GEMM_EPI_NONE: hipLaunchKernelGGL((gemm_kernel<T, AK, BK_, GEMM_EPI_NONE>), grid, dim3(GT_THREADS), 0, s, g); break;
        case GEMM_EPI_BIAS: hipLaunchKernelGGL((gemm_kernel<T, AK, BK_, GEMM_EPI_BIAS>), grid, dim3(GT_THREADS), 0, s, g); break;
        case GEMM_EPI_BIAS_RELU: hipLaunchKernelGGL((gemm_kernel<T, AK, BK_, GEMM_EPI_BIAS_RELU>), grid, dim3(GT_THREADS), 0, s, g); break;
        case GEMM_EPI_MASK: hipLaunchKernelGGL((gemm_kernel<T, AK, BK_, GEMM_EPI_MASK>), grid, dim3(GT_THREADS), 0, s, g); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t gemm_launch(const GemmArgs& g, int dtype, int a_kcontig, int b_kcontig, int epi, int splits, int batch,
                       hipStream_t s) {
    if (g.M <= 0 || g.N <= 0 || g.K <= 0 || splits < 1 || batch < 1) return hipErrorInvalidValue;
    if (splits > 1 && (epi != GEMM_EPI_NONE || g.beta != 0.f || g.Cbf16 != nullptr)) return hipErrorInvalidValue;
    if (dtype == 0) {
        if (a_kcontig && b_kcontig) return launch_t<float, true, true>(g, epi, splits, batch, s);
        if (a_kcontig && !b_kcontig) return launch_t<float, true, false>(g, epi, splits, batch, s);
        if (!a_kcontig && !b_kcontig) return launch_t<float, false, false>(g, epi, splits, batch, s);
        return launch_t<float, false, true>(g, epi, splits, batch, s);
    }
    if (a_kcontig && b_kcontig) return launch_t<__hip_bfloat16, true, true>(g, epi, splits, batch, s);
    if (a_kcontig && !b_kcontig) return launch_t<__hip_bfloat16, true, false>(g, epi, splits, batch, s);
    if (!a_kcontig && !b_kcontig) return launch_t<__hip_bfloat16, false, false>(g, epi, splits, batch, s);
    return launch_t<__hip_bfloat16, false, true>(g, epi, splits, batch, s);
}

hipError_t splitk_reduce_launch(const float* slab, size_t stride, int splits, float* out, size_t n, float beta,
                                hipStream_t s) {
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, slab, stride, splits,
                       out, n, beta);
    return hipGetLastError();
}

// Column sums of a contiguous [M][N] matrix with few columns (N <= 64, e.g. the logits-head
// bias gradient): thread t < S = 1024 - 1024 % N reads the flat elements t, t + S, ... (all in
// column t % N, coalesced across the block), then column n folds the partials t = n, n + N, ...
// in fixed order.
__global__ void __launch_bounds__(1024) colsum_flat_kernel(const float* __restrict__ X, size_t total, int N,
                                                           float* __restrict__ out, float beta) {
    __shared__ float part[1024];
    const int t = threadIdx.x, S = 1024 - 1024 % N;
    float acc = 0.f;
    if (t < S)
        for (size_t e = t; e < total; e += S) acc += X[e];
    part[t] = acc;
    __syncthreads();
    if (t < N) {
        float v = 0.f;
        for (int i = t; i < S; i += N) v += part[i];
        out[t] = (beta != 0.f ? beta * out[t] : 0.f) + v;
    }
}

// The same few-column sums split over row ranges: block z folds rows [z*rc, (z+1)*rc) into
// slab[z][N] (rc*N is a multiple of N, so element e of the range is still in column e % N), and
// splitk_reduce folds the slabs in fixed order.  One block streaming 1 MiB alone took 130 us.
__global__ void __launch_bounds__(1024) colsum_split_kernel(const float* __restrict__ X, int M, int N, int rc,
                                                            float* __restrict__ slab) {
    __shared__ float part[1024];
    const int t = threadIdx.x, S = 1024 - 1024 % N, z = blockIdx.x;
    const size_t e0 = (size_t)z * rc * N;
    const size_t e1 = (size_t)min(M, (z + 1) * rc) * N;
    float acc = 0.f;
    if (t < S)
        for (size_t e = e0 + t; e < e1; e += S) acc += X[e];
    part[t] = acc;
    __syncthreads();
    if (t < N) {
        float v = 0.f;
        for (int i = t; i < S; i += N) v += part[i];
        slab[(size_t)z * N + t] = v;
    }
}

hipError_t colsum_split_launch(const float* X, int M, int N, int splits, float* slab, float* out, float beta,
                               hipStream_t s) {
    if (N < 1 || N > 64 || splits < 1 || M < 1) return hipErrorInvalidValue;
    const int rc = (M + splits - 1) / splits;
    splits = (M + rc - 1) / rc;
    hipLaunchKernelGGL(colsum_split_kernel, dim3((unsigned)splits), dim3(1024), 0, s, X, M, N, rc, slab);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return splitk_reduce_launch(slab, (size_t)N, splits, out, (size_t)N, beta, s);
}

hipError_t colsum_launch(const float* X, int M, int N, int ld, float* out, float beta, int batch, long long sX,
                         long long sOut, const int* active, hipStream_t s) {
    if (N <= 64 && ld == N && batch == 1 && active == nullptr && (size_t)M * N >= 4096) {
        hipLaunchKernelGGL(colsum_flat_kernel, dim3(1), dim3(1024), 0, s, X, (size_t)M * N, N, out, beta);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(colsum_kernel, dim3((N + 63) / 64, batch), dim3(1024), 0, s, X, M, N, ld, out, beta, sX, sOut,
                       active);
    return hipGetLastError();
}

hipError_t f32_to_bf16_launch(const float* x, void* y, size_t n, hipStream_t s, float scale) {
    hipLaunchKernelGGL(f32_to_bf16_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x,
                       reinterpret_cast<__hip_bfloat16*>(y), n, scale);
    return hipGetLastError();
}
