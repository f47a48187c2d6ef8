// Layered-path GEMM interface (gemm_mfma.hip) and loss / optimizer kernels (mlp_ops.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

enum { GEMM_EPI_NONE = 0, GEMM_EPI_BIAS = 1, GEMM_EPI_BIAS_RELU = 2, GEMM_EPI_MASK = 3 };

struct GemmArgs {
    int M, N, K;
    const void* A;       // fp32 or bf16 (dtype)
    int lda;
    const void* B;
    int ldb;
    float* C;            // fp32 [M][ldc] (or split-K slabs, slab_stride apart)
    int ldc;
    void* Cbf16;         // optional bf16 copy of C (same ldc), for the next bf16 GEMM
    const float* bias;   // [N] for BIAS epilogues
    const void* mask;    // [M][ldmask] for MASK (ReLU derivative from the layer input)
    int ldmask;
    int mask_bf16;
    float alpha;
    float beta;          // C = alpha*acc (+ bias ...) + beta*C
    size_t slab_stride;  // floats between split-K partial outputs
    // batched (packed trials): blockIdx.z selects the problem; element strides per problem
    // (0 = shared operand, e.g. one minibatch feeding every trial's first layer)
    long long sA, sB, sC, sBias, sMask;
    const int* active;   // optional per-problem flag: 0 = skip (stopped trial)
};

hipError_t gemm_launch(const GemmArgs& g, int dtype /*0 f32, 1 bf16*/, int a_kcontig, int b_kcontig, int epi,
                       int splits, int batch, hipStream_t s);
// out[n] = beta*out[n] + sum_m X[m][n] for contiguous X [M][N], N <= 64, rows split `splits` ways
// into slab[splits][N] and folded in fixed order.
hipError_t colsum_split_launch(const float* X, int M, int N, int splits, float* slab, float* out, float beta,
                               hipStream_t s);
hipError_t splitk_reduce_launch(const float* slab, size_t stride, int splits, float* out, size_t n, float beta,
                                hipStream_t s);
hipError_t colsum_launch(const float* X, int M, int N, int ld, float* out, float beta, int batch, long long sX,
                         long long sOut, const int* active, hipStream_t s);
hipError_t fedavg_delta_bf16_launch(const float* w, const float* g, void* d, size_t n, float scale, hipStream_t s);
hipError_t fedavg_apply_delta_launch(float* w, float* g, const void* d, size_t n, hipStream_t s);
hipError_t f32_to_bf16_launch(const float* x, void* y, size_t n, hipStream_t s, float scale = 1.f);
