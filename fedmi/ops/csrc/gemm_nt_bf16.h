// bf16 NT GEMM (gemm_nt_bf16.hip): C = alpha * A[M][K] . B[N][K]^T (+bias, ReLU, mask, +beta*C).
#pragma once
#include <hip/hip_runtime.h>

struct NTArgs {
    int M, N, K;
    const void* A; int lda;     // bf16 [M][lda]
    const void* B; int ldb;     // bf16 [N][ldb]
    float* C; int ldc;          // optional fp32 output
    void* Cbf16; int ldcb;      // optional bf16 row-major output
    void* CbT; int ldct;        // optional bf16 transposed output [N][ldct]
    const float* bias;          // optional [N]
    const void* mask; int ldmask;  // optional bf16 [M][ldmask]: out = mask > 0 ? v : 0
    int relu;
    float alpha, beta;
    unsigned long long* dbg;    // optional [blocks][8] s_memrealtime phase stamps (profiling; full-line loop)
    float* csum; int ldcs;      // optional column sums of the bf16 output (bias gradient of a dgrad):
                                // csum[m / 128][n] = sum of the tile half's 128 rows (256x256 loops only)
};

hipError_t gemm_nt_bf16_launch(const NTArgs& g, hipStream_t s);
hipError_t transpose_bf16_launch(const float* in, int R, int C, int ldi, void* out, int ldo, hipStream_t s);
// out[n] = sum_r dT[n][r] (+ beta * out[n]); dT bf16 [Nrows][ld], M % 8 == 0.
hipError_t pad_bf16_launch(const float* in, int R, int C, long long rs, long long cs, void* out, int ldo,
                           hipStream_t s);
hipError_t rowsum_bf16_launch(const void* dT, int Nrows, int M, int ld, float* out, float beta, hipStream_t s);
// Skinny weight gradient, out = beta*out + sum_r S[r][c] W[r][n] (C = 2 with trans = 0: out[c][n];
// C = 14 with trans = 1: out[n][c]), split over `splits` row ranges into slab[splits][(C + b) * Nw];
// bias_out (C = 14 only; b = 1) also gets beta*bias_out + the column sums of W.
hipError_t skinny_wgrad_launch(const void* W, int ldw, int Nw, const void* S, int lds, int C, int rows, int trans,
                               int splits, float* slab, float* out, float beta, float* bias_out, hipStream_t s);
// 0 = single-buffered two-barrier main loop, 1 = double-buffered (default)
void gemm_nt_set_variant(int v);
// phase stamps of the next launches (tools/nt_stamps.py); nullptr = off
void gemm_nt_set_debug(unsigned long long* dbg);
