// Loss heads, optimizer and minibatch plumbing of the layered path (mlp_ops.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

struct GatherArgs {
    const float* X; int ld;        // shard [n][ld]
    const int* y;                  // shard labels
    const int* perms;              // [epochs][n_perm] row permutations (nullptr: identity)
    const int* epoch_ctr;          // device epoch counter selecting the permutation
    long long n_perm;
    int off, M, F;                 // minibatch = perm[off : off+M]
    float* out; int ldo; void* outb;
    int* yb;                       // gathered labels [M]
};

struct XentArgs {
    const float* z;      // logits [T][M][ldz] (stride sZ between trials)
    int ldz;
    long long sZ;
    const int* y;        // labels of the shard
    const int* idx;      // minibatch row -> shard row (nullptr: identity)
    int M, C, mode;      // mode 0: softmax CE; 1: sklearn binary logistic head
    float scale;         // dz multiplier (1 / batch)
    float* dz;           // [T][M][lddz]
    int lddz;
    long long sDz;
    double* loss_acc;    // [T] running sum of per-row losses (nullptr: skip)
    int* pred;           // [T][M] predictions (nullptr: skip)
    const int* active;   // [T] or nullptr
};

struct AdamArgs {
    float* p; float* m; float* v;  // [T][n]
    const float* g;                // [T][n]
    const float* anchor;           // FedProx anchor [T][n] (if mu != 0)
    const unsigned char* wd_mask;  // [n] 1 = decayed entry (coefs), nullptr = all
    size_t n;
    int style;                     // 0 torch Adam, 1 sklearn AdamOptimizer
    const double* lr;              // [T] learning rate per trial
    double beta1, beta2, eps;
    double wd;                     // gradient L2 coefficient (sklearn: alpha / batch)
    double mu;                     // FedProx
    const long long* step;         // [T] 1-based step of this update
    double* loss_acc;              // [T] (+= l2_coef * sum p^2 over decayed entries)
    double l2_coef;                // sklearn: 0.5 * alpha
    const int* active;
    void* p_bf16;                  // optional bf16 shadow [T][n]
    double lr_scalar;              // used when lr == nullptr
    long long step_scalar;         // used when step == nullptr
};

struct EpochArgs {
    int T;
    int* epoch_ctr;
    double* loss_acc; double* best; int* count; int* n_iter; int* active; double* curve;
    long long n_samples;
    double tol;
    int n_iter_no_change, max_iter, tol_stop;
};

hipError_t gather_rows_launch(const GatherArgs& a, hipStream_t s);
hipError_t xent_launch(const XentArgs& a, int T, hipStream_t s);
hipError_t adam_launch(const AdamArgs& a, int T, hipStream_t s);
hipError_t step_count_launch(long long* step, const int* active, int T, hipStream_t s);
hipError_t epoch_end_launch(const EpochArgs& a, hipStream_t s);
hipError_t logits_confusion_launch(const float* z, int ldz, const int* y, int M, int C, float* cm, hipStream_t s);
hipError_t confusion_launch(const int* pred, const int* y, const int* idx, int M, int C, int T, float* cm,
                            hipStream_t s);
