// Loss heads, optimizer and minibatch plumbing of the layered path (packed trials).
//
// Everything is batched over T "problems" (blockIdx.y / z = trial): the hyperparameter
// sweep of hyperparameters_tuning.py:73-124 trains 9 learning rates of one hidden-layer
// config at once, sharing each minibatch (same random_state -> same init and shuffles as
// sklearn), with per-trial learning rate, loss accumulators and stop flags on the device.
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <math.h>
#include <stdint.h>

#include <algorithm>

#include "mlp_ops.h"

// ---------------------------------------------------------------------------------------
// Minibatch assembly: rows perm[epoch][off + i] of the shard -> out[i][:F] (zero padded to
// ldo) and their labels -> yb[i].  The epoch is read from a device counter (advanced by
// epoch_end_kernel), so one captured epoch graph is replayed for every epoch.
__global__ void gather_rows_kernel(GatherArgs a) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= a.M * a.ldo) return;
    const int i = e / a.ldo, f = e - i * a.ldo;
    const int* perm = a.perms + (a.epoch_ctr != nullptr ? (long long)(*a.epoch_ctr) * a.n_perm : 0);
    const int src = a.perms != nullptr ? perm[a.off + i] : a.off + i;
    const float v = f < a.F ? a.X[(size_t)src * a.ld + f] : 0.f;
    a.out[e] = v;
    if (a.outb) reinterpret_cast<__hip_bfloat16*>(a.outb)[e] = __float2bfloat16(v);
    if (f == 0 && a.yb != nullptr) a.yb[i] = a.y[src];
}

// ---------------------------------------------------------------------------------------
// Output head.  mode 0: softmax cross-entropy over C logits (torch CrossEntropyLoss / sklearn
// multinomial log_loss); mode 1: sklearn binary head -- one logit, logistic output,
// binary log-loss with probabilities clipped to [eps, 1-eps] (sklearn binary_log_loss).
// dz = (p - onehot) * scale.  Per-row losses are summed per block and added in double to
// loss_acc[t] (sum, not mean: the caller divides by its sample count like sklearn).
__global__ void __launch_bounds__(256)
xent_kernel(XentArgs a) {
    __shared__ double red[256];
    const int t = blockIdx.y;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    double lrow = 0.0;
    const bool run = a.active == nullptr || a.active[t] != 0;
    if (run && i < a.M) {
        const float* z = a.z + t * a.sZ + (size_t)i * a.ldz;
        float* dz = a.dz + t * a.sDz + (size_t)i * a.lddz;
        const int y = a.y[a.idx != nullptr ? a.idx[i] : i];
        if (a.mode == 1) {
            const float p = 1.f / (1.f + expf(-z[0]));
            const float eps = 1.1920929e-07f;
            const float pc = fminf(fmaxf(p, eps), 1.f - eps);
            lrow = y ? -log((double)pc) : -log(1.0 - (double)pc);
            dz[0] = (p - (float)y) * a.scale;
            if (a.pred) a.pred[t * a.M + i] = p > 0.5f ? 1 : 0;
        } else {
            float mx = z[0];
            int am = 0;
            for (int k = 1; k < a.C; ++k)
                if (z[k] > mx) { mx = z[k]; am = k; }
            float se = 0.f;
            for (int k = 0; k < a.C; ++k) se += expf(z[k] - mx);
            lrow = (double)(mx + logf(se) - z[y]);
            for (int k = 0; k < a.C; ++k) dz[k] = (expf(z[k] - mx) / se - (k == y ? 1.f : 0.f)) * a.scale;
            if (a.pred) a.pred[t * a.M + i] = am;
        }
    }
    red[threadIdx.x] = lrow;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0 && run && a.loss_acc != nullptr) atomicAdd(&a.loss_acc[t], red[0]);
}

// ---------------------------------------------------------------------------------------
// Adam over [T][P] flat parameters.  style 0: torch.optim.Adam (bias-corrected sqrt(v) + eps);
// style 1: sklearn AdamOptimizer (lr_t = lr sqrt(1-b2^t)/(1-b1^t), update -lr_t m/(sqrt(v)+eps)).
// L2: g += wd * p on entries with wd_mask (sklearn: alpha/batch on coefs only), and the
// sklearn loss term 0.5*alpha*sum(coef^2) (of the pre-update weights) is added to loss_acc.
#define ADAM_EPT 4

__global__ void __launch_bounds__(256)
adam_kernel(AdamArgs a) {
    __shared__ double red[256];
    __shared__ float coef[2];
    const int t = blockIdx.y;
    const bool run = a.active == nullptr || a.active[t] != 0;
    // the trial's bias-corrected step factors, once per block (fp64 pow/sqrt per element made
    // this kernel compute-bound: 454 us for the 33.6 M-parameter wide MLP)
    if (threadIdx.x == 0) {
        const long long step = a.step != nullptr ? a.step[t] : a.step_scalar;
        const double lr = a.lr != nullptr ? a.lr[t] : a.lr_scalar;
        if (a.style == 0) {
            coef[0] = (float)(lr / (1.0 - pow(a.beta1, (double)step)));
            coef[1] = (float)sqrt(1.0 - pow(a.beta2, (double)step));
        } else {
            coef[0] = (float)(lr * sqrt(1.0 - pow(a.beta2, (double)step)) / (1.0 - pow(a.beta1, (double)step)));
            coef[1] = 0.f;
        }
    }
    __syncthreads();
    const float c0 = coef[0], c1 = coef[1];
    const float omb1 = (float)(1.0 - a.beta1), b1 = (float)a.beta1;
    const float omb2 = (float)(1.0 - a.beta2), b2 = (float)a.beta2;
    const float eps = (float)a.eps, wd = (float)a.wd, mu = (float)a.mu;
    double sq = 0.0;
    // ADAM_EPT elements per thread, strided by the block size (coalesced, independent chains)
#pragma unroll
    for (int e = 0; e < ADAM_EPT; ++e) {
        const size_t i = ((size_t)blockIdx.x * ADAM_EPT + e) * blockDim.x + threadIdx.x;
        if (!run || i >= a.n) continue;
        const size_t j = (size_t)t * a.n + i;
        float p = a.p[j];
        float g = a.g[j];
        const bool decay = a.wd_mask == nullptr || a.wd_mask[i] != 0;
        if (decay) {
            sq += (double)p * (double)p;
            if (a.wd != 0.0) g += wd * p;
        }
        if (a.mu != 0.0) g += mu * (p - a.anchor[j]);
        float m = a.m[j], v = a.v[j];
        if (a.style == 0) {
            m = m + omb1 * (g - m);
            v = v * b2 + omb2 * g * g;
            p = p + (-c0) * (m / (sqrtf(v) / c1 + eps));
        } else {
            m = b1 * m + omb1 * g;
            v = b2 * v + omb2 * g * g;
            p = p - c0 * m / (sqrtf(v) + eps);
        }
        a.m[j] = m;
        a.v[j] = v;
        a.p[j] = p;
        if (a.p_bf16) reinterpret_cast<__hip_bfloat16*>(a.p_bf16)[j] = __float2bfloat16(p);
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

// One optimizer step done for every active trial: bump its step counter.
__global__ void step_count_kernel(long long* step, const int* active, int T) {
    const int t = threadIdx.x;
    if (t < T && (active == nullptr || active[t])) step[t] += 1;
}

// ---------------------------------------------------------------------------------------
// End of epoch, per trial (sklearn _fit_stochastic + _update_no_improvement_count):
// loss_ = acc / n; curve append; count += (loss_ > best - tol) ? 1 : reset; best = min;
// n_iter += 1; stop when count > n_iter_no_change or n_iter == max_iter.
__global__ void epoch_end_kernel(EpochArgs a) {
    const int t = threadIdx.x;
    if (t == 0 && a.epoch_ctr != nullptr) *a.epoch_ctr += 1;
    if (t >= a.T || !a.active[t]) return;
    const double loss = a.loss_acc[t] / (double)a.n_samples;
    a.loss_acc[t] = 0.0;
    const int it = a.n_iter[t];
    if (it < a.max_iter) a.curve[(size_t)t * a.max_iter + it] = loss;
    if (loss > a.best[t] - a.tol) a.count[t] += 1;
    else a.count[t] = 0;
    if (loss < a.best[t]) a.best[t] = loss;
    a.n_iter[t] = it + 1;
    if ((a.tol_stop && a.count[t] > a.n_iter_no_change) || it + 1 >= a.max_iter) a.active[t] = 0;
}

// Confusion counts from predictions: cm[t][y][p] += 1 (float, exact below 2^24).
__global__ void confusion_kernel(const int* __restrict__ pred, const int* __restrict__ y, const int* __restrict__ idx,
                                 int M, int C, int T, float* __restrict__ cm) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int t = blockIdx.y;
    if (i >= M || t >= T) return;
    const int yy = y[idx != nullptr ? idx[i] : i];
    atomicAdd(&cm[(size_t)t * C * C + yy * C + pred[(size_t)t * M + i]], 1.f);
}

// Argmax of fp32 logits rows + confusion counts (local evaluation of the wide client, C:75-91):
// cm[y][argmax] += 1 over M rows, counts accumulated per block in LDS then added to the float
// counters (exact below 2^24 per cell per call).
__global__ void __launch_bounds__(256)
logits_confusion_kernel(const float* __restrict__ z, int ldz, const int* __restrict__ y, int M, int C,
                        float* __restrict__ cm) {
    __shared__ int cnt[16 * 16];
    for (int i = threadIdx.x; i < C * C; i += blockDim.x) cnt[i] = 0;
    __syncthreads();
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < M; i += gridDim.x * blockDim.x) {
        const float* zr = z + (size_t)i * ldz;
        int best = 0;
        float bv = zr[0];
        for (int k = 1; k < C; ++k)
            if (zr[k] > bv) { bv = zr[k]; best = k; }   // torch.max(dim=1): first maximum
        atomicAdd(&cnt[y[i] * C + best], 1);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < C * C; i += blockDim.x)
        if (cnt[i]) atomicAdd(&cm[i], (float)cnt[i]);
}

// ---------------------------------------------------------------------------------------
hipError_t logits_confusion_launch(const float* z, int ldz, const int* y, int M, int C, float* cm, hipStream_t s) {
    if (C < 1 || C > 16 || M < 0) return hipErrorInvalidValue;
    if (M == 0) return hipSuccess;
    const int blocks = (int)std::min<long long>(1024, ((long long)M + 255) / 256);
    hipLaunchKernelGGL(logits_confusion_kernel, dim3(blocks), dim3(256), 0, s, z, ldz, y, M, C, cm);
    return hipGetLastError();
}

hipError_t gather_rows_launch(const GatherArgs& a, hipStream_t s) {
    const int n = a.M * a.ldo;
    hipLaunchKernelGGL(gather_rows_kernel, dim3((n + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t xent_launch(const XentArgs& a, int T, hipStream_t s) {
    hipLaunchKernelGGL(xent_kernel, dim3((a.M + 255) / 256, T), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t adam_launch(const AdamArgs& a, int T, hipStream_t s) {
    hipLaunchKernelGGL(adam_kernel, dim3((unsigned)((a.n + 256 * ADAM_EPT - 1) / (256 * ADAM_EPT)), T), dim3(256), 0, s, a);
    if (hipGetLastError() != hipSuccess) return hipErrorLaunchFailure;
    return hipSuccess;
}

hipError_t step_count_launch(long long* step, const int* active, int T, hipStream_t s) {
    hipLaunchKernelGGL(step_count_kernel, dim3(1), dim3(64), 0, s, step, active, T);
    return hipGetLastError();
}

hipError_t epoch_end_launch(const EpochArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(epoch_end_kernel, dim3(1), dim3(64), 0, s, a);
    return hipGetLastError();
}

hipError_t confusion_launch(const int* pred, const int* y, const int* idx, int M, int C, int T, float* cm,
                            hipStream_t s) {
    hipLaunchKernelGGL(confusion_kernel, dim3((M + 255) / 256, T), dim3(256), 0, s, pred, y, idx, M, C, T, cm);
    return hipGetLastError();
}
