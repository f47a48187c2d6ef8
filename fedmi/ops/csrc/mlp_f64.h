// float64 layered-path kernels (mlp_f64.hip): the sklearn estimator's dtype=float64 HIP mode.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

#include <algorithm>

struct Gemm64Args {
    int M, N, K;
    const double* A;
    int lda;
    const double* B;
    int ldb;
    double* C;
    int ldc;
    const double* bias;
    const double* mask;
    int ldmask;
    double alpha, beta;
    long long sA, sB, sC, sBias, sMask;   // per-trial strides (0 = shared operand)
    const int* active;
};

struct Adam64Args {
    double* p; double* m; double* v;
    const double* g;
    const double* anchor;
    const unsigned char* wd_mask;
    size_t n;
    int style;              // 0 torch Adam, 1 sklearn AdamOptimizer
    const double* lr;       // [T]
    double beta1, beta2, eps, wd, mu;
    const long long* step;  // [T]
    double* loss_acc;
    double l2_coef;
    const int* active;
};

hipError_t gemm_f64_launch(const Gemm64Args& g, int a_kcontig, int b_kcontig, int epi, int batch, hipStream_t s);
hipError_t gather_rows_f64_launch(const double* X, int ld, const int* y, const int* perms, const int* epoch_ctr,
                                  long long n_perm, int off, int M, int F, double* out, int ldo, int* yb,
                                  hipStream_t s);
hipError_t xent_f64_launch(const double* z, int ldz, long long sZ, const int* y, int M, int C, int mode, double scale,
                           double* dz, int lddz, long long sDz, double* loss_acc, const int* active, int T,
                           hipStream_t s);
hipError_t colsum_f64_launch(const double* X, int M, int N, int ld, double* out, double beta, int batch, long long sX,
                             long long sOut, const int* active, hipStream_t s);
hipError_t adam_f64_launch(const Adam64Args& a, int T, hipStream_t s);
