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

// Fused float64 minibatch step (mlp_fused_f64.hip): two kernels per minibatch for sklearn's
// Adam / binary-logistic or softmax head / L2 (style 1), no FedProx, at most SKF_MAXL layers.
#define SKF_MAXL 4
struct SkfArgs {
    int L, T, P;
    int dims[SKF_MAXL + 1];
    int w_off[SKF_MAXL], b_off[SKF_MAXL];   // dense [N][K] weights, then the bias, per layer
    const double* X;                        // [n][dims[0]]
    const int* y;
    const int* perms;                       // [epochs][n_perm]
    const int* epoch_ctr;
    long long n_perm;
    int off, rows, Bmax, maxw, head;        // minibatch rows perm[off : off + rows]; head 1 = logistic
    int wthru;                              // row pass writes acts / deltas / rows through (sc1): large jobs
    double inv_rows, alpha, beta1, beta2, eps, l2_coef;
    double *params, *m, *v;                 // [T][P]
    const double* lr;                       // [T]
    long long* step;                        // [T] Adam step counter
    double* loss_acc;                       // [T] epoch loss sum
    const int* active;                      // [T]
    double* xg;                             // [T][Bmax][dims[0]] gathered rows
    double* acts;                           // [L][T][Bmax][maxw] hidden activations
    double* deltas;                         // [L][T][Bmax][maxw]
    unsigned long long* dbg;                // optional: s_memrealtime phase stamps of row block (0, 0)
    const double* zero;                     // one 0.0 in device memory (branch-free masked loads)
    double* wt;                             // optional [T][P]: each layer's weights transposed [K][N] (kept by
                                            // the Adam epilogue; read by the forward), nullptr: none
    // Tile-split row pass (mlp_fused_f64.hip skf_cs_*, two hidden layers): split > 1 cuts hidden layer
    // 1's forward and input-gradient products by output tiles over `split` workgroups per row block
    int split;
};
// Slices of the tile-split row pass for a fused job (1: none) on a device with `cus` CUs; `want`:
// 0 = the rule, 1 = off, > 1 = at most that many.
int skf_pick_split(const SkfArgs& a, int want, int cus);
bool skf_supported(const SkfArgs& a);
size_t skf_lds_bytes(const SkfArgs& a);
hipError_t skf_prepare(const SkfArgs& a);
hipError_t skf_step_launch(const SkfArgs& a, hipStream_t s);
