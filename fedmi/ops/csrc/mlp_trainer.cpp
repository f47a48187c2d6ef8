// Native minibatch trainer for T packed MLPs of one architecture (layered path), in fp32
// (exact-fp32 MFMA) or float64 (f64 MFMA: sklearn's precision, mlp_f64.hip).
//
// Serves the scikit-learn-compatible estimator (FL_SkLearn_MLPClassifier_Limitation.py:77-101,
// hyperparameters_tuning.py:90-91) and the hyperparameter sweep with trial packing: the 9
// learning rates of one hidden-layer config train together, sharing every minibatch.  One
// epoch = ceil(n/B) minibatch steps; each step is
//   gather -> L fused fwd GEMMs (bias+ReLU) -> loss head -> per layer: wgrad GEMM + bias
//   colsum + dgrad GEMM (ReLU mask) -> step counter -> Adam (+L2 loss term)
// and the epoch ends with the sklearn tol / n_iter_no_change rule evaluated on the device
// per trial.  An epoch is captured once into a hipGraph and replayed (the epoch's row
// permutation is selected by a device counter), so the host issues one launch per epoch.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/numpy.h>
#include <pybind11/stl.h>

#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

#include "gemm_mfma.h"

void sk_epoch_perms(uint32_t* key, int* pos, int n, int epochs, int32_t* perms);  // sk_perms.cpp
#include "gemm_nt_bf16.h"
#include "mlp_f64.h"
#include "mlp_ops.h"

namespace py = pybind11;

#define TR_CHECK(expr)                                                                         \
    do {                                                                                       \
        hipError_t _e = (expr);                                                                \
        if (_e != hipSuccess)                                                                  \
            throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) +      \
                                     " at " #expr);                                            \
    } while (0)

template <typename T>
static inline T* ptr_of(py::dict& d, const char* k) {
    return reinterpret_cast<T*>(d[k].cast<uintptr_t>());
}

// Kernel dispatch of the trainer by element type: fp32 (gemm_mfma.hip / mlp_ops.hip: exact-fp32
// MFMA) or float64 (mlp_f64.hip: v_mfma_f64_16x16x4_f64, sklearn's own precision).
template <typename T> struct TrainerOps;

template <> struct TrainerOps<float> {
    static void gather(const float* X, int ld, const int* y, const int* perms, int* epoch_ctr, long long n_perm,
                       int off, int M, int F, float* out, int ldo, int* yb, hipStream_t s) {
        GatherArgs ga{X, ld, y, perms, epoch_ctr, n_perm, off, M, F, out, ldo, nullptr, yb};
        TR_CHECK(gather_rows_launch(ga, s));
    }
    static void gemm(int M, int N, int K, const float* A, int lda, long long sA, int akc, const float* B, int ldb,
                     long long sB, int bkc, float* C, int ldc, long long sC, const float* bias, long long sBias,
                     const float* mask, int ldmask, long long sMask, int epi, const int* active, int T, hipStream_t s) {
        GemmArgs g{};
        g.M = M; g.N = N; g.K = K;
        g.A = A; g.lda = lda; g.sA = sA;
        g.B = B; g.ldb = ldb; g.sB = sB;
        g.C = C; g.ldc = ldc; g.sC = sC;
        g.bias = bias; g.sBias = sBias;
        g.mask = mask; g.ldmask = ldmask; g.sMask = sMask;
        g.alpha = 1.f; g.beta = 0.f; g.active = active;
        TR_CHECK(gemm_launch(g, 0, akc, bkc, epi, 1, T, s));
    }
    static void xent(const float* z, int ldz, long long sZ, const int* y, int M, int C, int mode, double scale,
                     float* dz, int lddz, long long sDz, double* loss_acc, const int* active, int T, hipStream_t s) {
        XentArgs xa{};
        xa.z = z; xa.ldz = ldz; xa.sZ = sZ; xa.y = y; xa.idx = nullptr; xa.M = M; xa.C = C; xa.mode = mode;
        xa.scale = (float)scale; xa.dz = dz; xa.lddz = lddz; xa.sDz = sDz; xa.loss_acc = loss_acc; xa.pred = nullptr;
        xa.active = active;
        TR_CHECK(xent_launch(xa, T, s));
    }
    static void colsum(const float* X, int M, int N, int ld, float* out, int T, long long sX, long long sOut,
                       const int* active, hipStream_t s) {
        TR_CHECK(colsum_launch(X, M, N, ld, out, 0.f, T, sX, sOut, active, s));
    }
    static void adam(float* p, float* m, float* v, const float* g, const float* anchor, const unsigned char* wd_mask,
                     size_t n, int style, const double* lr, double b1, double b2, double eps, double wd, double mu,
                     const long long* step, double* loss_acc, double l2, const int* active, int T, hipStream_t s) {
        AdamArgs aa{};
        aa.p = p; aa.m = m; aa.v = v; aa.g = g; aa.anchor = anchor; aa.wd_mask = wd_mask; aa.n = n; aa.style = style;
        aa.lr = lr; aa.beta1 = b1; aa.beta2 = b2; aa.eps = eps; aa.wd = wd; aa.mu = mu; aa.step = step;
        aa.loss_acc = loss_acc; aa.l2_coef = l2; aa.active = active; aa.p_bf16 = nullptr;
        TR_CHECK(adam_launch(aa, T, s));
    }
};

template <> struct TrainerOps<double> {
    static void gather(const double* X, int ld, const int* y, const int* perms, int* epoch_ctr, long long n_perm,
                       int off, int M, int F, double* out, int ldo, int* yb, hipStream_t s) {
        TR_CHECK(gather_rows_f64_launch(X, ld, y, perms, epoch_ctr, n_perm, off, M, F, out, ldo, yb, s));
    }
    static void gemm(int M, int N, int K, const double* A, int lda, long long sA, int akc, const double* B, int ldb,
                     long long sB, int bkc, double* C, int ldc, long long sC, const double* bias, long long sBias,
                     const double* mask, int ldmask, long long sMask, int epi, const int* active, int T,
                     hipStream_t s) {
        Gemm64Args g{};
        g.M = M; g.N = N; g.K = K;
        g.A = A; g.lda = lda; g.sA = sA;
        g.B = B; g.ldb = ldb; g.sB = sB;
        g.C = C; g.ldc = ldc; g.sC = sC;
        g.bias = bias; g.sBias = sBias;
        g.mask = mask; g.ldmask = ldmask; g.sMask = sMask;
        g.alpha = 1.0; g.beta = 0.0; g.active = active;
        TR_CHECK(gemm_f64_launch(g, akc, bkc, epi, T, s));
    }
    static void xent(const double* z, int ldz, long long sZ, const int* y, int M, int C, int mode, double scale,
                     double* dz, int lddz, long long sDz, double* loss_acc, const int* active, int T, hipStream_t s) {
        TR_CHECK(xent_f64_launch(z, ldz, sZ, y, M, C, mode, scale, dz, lddz, sDz, loss_acc, active, T, s));
    }
    static void colsum(const double* X, int M, int N, int ld, double* out, int T, long long sX, long long sOut,
                       const int* active, hipStream_t s) {
        TR_CHECK(colsum_f64_launch(X, M, N, ld, out, 0.0, T, sX, sOut, active, s));
    }
    static void adam(double* p, double* m, double* v, const double* g, const double* anchor,
                     const unsigned char* wd_mask, size_t n, int style, const double* lr, double b1, double b2,
                     double eps, double wd, double mu, const long long* step, double* loss_acc, double l2,
                     const int* active, int T, hipStream_t s) {
        Adam64Args a{};
        a.p = p; a.m = m; a.v = v; a.g = g; a.anchor = anchor; a.wd_mask = wd_mask; a.n = n; a.style = style;
        a.lr = lr; a.beta1 = b1; a.beta2 = b2; a.eps = eps; a.wd = wd; a.mu = mu; a.step = step;
        a.loss_acc = loss_acc; a.l2_coef = l2; a.active = active;
        TR_CHECK(adam_f64_launch(a, T, s));
    }
};

template <typename T>
class MLPTrainerT {
  public:
    using Ops = TrainerOps<T>;
    MLPTrainerT(std::vector<int> dims, int Tr, py::dict cfg, py::dict bufs) : dims_(dims), T_(Tr) {
        L_ = (int)dims.size() - 1;
        if (L_ < 1) throw std::runtime_error("MLPTrainer: need >= 1 layer");
        int off = 0;
        for (int l = 0; l < L_; ++l) {
            w_off_.push_back(off);
            off += dims[l] * dims[l + 1];
            b_off_.push_back(off);
            off += dims[l + 1];
        }
        P_ = off;
        n_ = cfg["n_rows"].cast<int>();
        B_ = cfg["batch"].cast<int>();
        head_ = cfg["head"].cast<int>();
        style_ = cfg["style"].cast<int>();
        beta1_ = cfg["beta1"].cast<double>();
        beta2_ = cfg["beta2"].cast<double>();
        eps_ = cfg["eps"].cast<double>();
        alpha_ = cfg["alpha"].cast<double>();
        wd_ = cfg["weight_decay"].cast<double>();
        mu_ = cfg["mu"].cast<double>();
        tol_ = cfg["tol"].cast<double>();
        nic_ = cfg["n_iter_no_change"].cast<int>();
        max_iter_ = cfg["max_iter"].cast<int>();
        tol_stop_ = cfg["tol_stop"].cast<int>();
        X_ = ptr_of<const T>(bufs, "X");
        y_ = ptr_of<const int>(bufs, "y");
        perms_ = ptr_of<const int>(bufs, "perms");
        epoch_ctr_ = ptr_of<int>(bufs, "epoch_ctr");
        params_ = ptr_of<T>(bufs, "params");
        grads_ = ptr_of<T>(bufs, "grads");
        m_ = ptr_of<T>(bufs, "m");
        v_ = ptr_of<T>(bufs, "v");
        anchor_ = ptr_of<const T>(bufs, "anchor");
        wd_mask_ = ptr_of<const unsigned char>(bufs, "wd_mask");
        lr_ = ptr_of<const double>(bufs, "lr");
        step_ = ptr_of<long long>(bufs, "step");
        loss_acc_ = ptr_of<double>(bufs, "loss_acc");
        best_ = ptr_of<double>(bufs, "best");
        count_ = ptr_of<int>(bufs, "count");
        n_iter_ = ptr_of<int>(bufs, "n_iter");
        active_ = ptr_of<int>(bufs, "active");
        curve_ = ptr_of<double>(bufs, "curve");
        xb_ = ptr_of<T>(bufs, "xb");
        yb_ = ptr_of<int>(bufs, "yb");
        acts_ = ptr_of<T>(bufs, "acts");    // [L][T][B][maxw]
        deltas_ = ptr_of<T>(bufs, "deltas");
        maxw_ = cfg["maxw"].cast<int>();
        if constexpr (std::is_same<T, double>::value) {
            // fused two-kernel minibatch step (mlp_fused_f64.hip) where it applies; the layered
            // path otherwise, or with FEDMI_SK_FUSED=0 (A/B)
            const char* env = std::getenv("FEDMI_SK_FUSED");
            const bool want = !(env != nullptr && env[0] == '0') &&
                              (!cfg.contains("fused") || cfg["fused"].cast<bool>());
            if (want && style_ == 1 && mu_ == 0.0 && wd_ == 0.0 && L_ <= SKF_MAXL) {
                SkfArgs a = fused_args(0, 1);
                fused_ = skf_supported(a);
                // tile-split row pass (mlp_fused_f64.hip skf_cs_*, bit-identical to the one-workgroup
                // row pass): FEDMI_SK_SPLIT=1 turns it off, S > 1 asks for S slices, default:
                // skf_pick_split's rule
                if (fused_) {
                    const char* sp = std::getenv("FEDMI_SK_SPLIT");
                    int cus = 0, dev = 0;
                    if (hipGetDevice(&dev) != hipSuccess ||
                        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
                        cus = 0;
                    const int S = skf_pick_split(a, sp != nullptr && *sp ? std::atoi(sp) : 0, cus);
                    if (S > 1) {
                        split_ = S;
                        if (!skf_supported(fused_args(0, 1))) split_ = 1;   // (LDS of the split kernels): no split
                    }
                }
            }
            if (fused_ && bufs.contains("wt")) wt_ = ptr_of<double>(bufs, "wt");
            if (fused_) TR_CHECK(skf_prepare(fused_args(0, 1)));
            if (fused_) {
                TR_CHECK(hipMalloc(&zero_, 64));
                TR_CHECK(hipMemset(zero_, 0, 64));
            }
            const char* st = std::getenv("FEDMI_SK_STAMPS");
            if (fused_ && st != nullptr && st[0] == '1') {
                TR_CHECK(hipMalloc(&dbg_, 16 * sizeof(unsigned long long)));
                TR_CHECK(hipMemset(dbg_, 0, 16 * sizeof(unsigned long long)));
            }
        }
    }
    ~MLPTrainerT() {
        drop_graph();
        if (dbg_) (void)hipFree(dbg_);
        if (zero_) (void)hipFree(zero_);
    }
    int split() const { return split_; }
    // Last fused row pass's phase stamps (FEDMI_SK_STAMPS=1), microseconds since its start.
    std::vector<double> stamps() const {
        std::vector<double> out;
        if (!dbg_) return out;
        unsigned long long h[16];
        TR_CHECK(hipDeviceSynchronize());
        TR_CHECK(hipMemcpy(h, dbg_, sizeof(h), hipMemcpyDeviceToHost));
        for (int i = 0; i < 16; ++i) out.push_back(h[i] ? (double)(h[i] - h[0]) / 100.0 : -1.0);
        return out;
    }

    int P() const { return P_; }
    bool fused() const { return fused_; }

    // One minibatch step on rows perm[epoch][off : off+rows].
    void step(int off, int rows, hipStream_t s) {
        if constexpr (std::is_same<T, double>::value) {
            if (fused_) {
                TR_CHECK(skf_step_launch(fused_args(off, rows), s));
                return;
            }
        }
        Ops::gather(X_, dims_[0], y_, perms_, epoch_ctr_, (long long)n_, off, rows, dims_[0], xb_, dims_[0], yb_, s);
        forward(xb_, rows, s, acts_, /*Bstride*/ B_);
        const long long sAct = (long long)B_ * maxw_;
        // loss head
        Ops::xent(act(L_ - 1), maxw_, sAct, yb_, rows, dims_[L_], head_, 1.0 / (double)rows, delta(L_ - 1), maxw_,
                  sAct, loss_acc_, active_, T_, s);
        // backward
        for (int l = L_ - 1; l >= 0; --l) {
            const int K = dims_[l], N = dims_[l + 1];
            const T* in = l == 0 ? xb_ : act(l - 1);
            const long long s_in = l == 0 ? 0 : sAct;
            const int ld_in = l == 0 ? dims_[0] : maxw_;
            // wgrad: dW[N][K] = dZ^T (rows x N) . in (rows x K)
            Ops::gemm(N, K, rows, delta(l), maxw_, sAct, 0, in, ld_in, s_in, 0, grads_ + w_off_[l], K, P_, nullptr, 0,
                      nullptr, 0, 0, GEMM_EPI_NONE, active_, T_, s);
            Ops::colsum(delta(l), rows, N, maxw_, grads_ + b_off_[l], T_, sAct, P_, active_, s);
            if (l > 0)  // dgrad: dIn[rows][K] = dZ . W[N][K], masked by in > 0 (ReLU)
                Ops::gemm(rows, K, N, delta(l), maxw_, sAct, 1, params_ + w_off_[l], K, P_, 0, delta(l - 1), maxw_, sAct,
                          nullptr, 0, act(l - 1), maxw_, sAct, GEMM_EPI_MASK, active_, T_, s);
        }
        TR_CHECK(step_count_launch(step_, active_, T_, s));
        // sklearn: coef grads (dW + alpha*W)/batch; torch: weight_decay * p
        Ops::adam(params_, m_, v_, grads_, anchor_, wd_mask_, (size_t)P_, style_, lr_, beta1_, beta2_, eps_,
                  style_ == 1 ? alpha_ / (double)rows : wd_, mu_, step_, loss_acc_, style_ == 1 ? 0.5 * alpha_ : 0.0,
                  active_, T_, s);
    }

    void epoch(hipStream_t s) {
        for (int off = 0; off < n_; off += B_) step(off, std::min(B_, n_ - off), s);
        EpochArgs ea{T_, epoch_ctr_, loss_acc_, best_, count_, n_iter_, active_, curve_, (long long)n_, tol_, nic_,
                     max_iter_, tol_stop_};
        TR_CHECK(epoch_end_launch(ea, s));
    }

    // Run up to n_epochs epochs (graph-replayed), polling the active flags every
    // `check_every` epochs; returns epochs issued.
    int run(int n_epochs, uintptr_t stream, int check_every, bool use_graph) {
        hipStream_t s = reinterpret_cast<hipStream_t>(stream);
        std::vector<int> act(T_);
        int done = 0;
        while (done < n_epochs) {
            const int chunk = std::min(check_every, n_epochs - done);
            for (int e = 0; e < chunk; ++e) {
                if (use_graph) {
                    if (!exec_) capture(s);
                    TR_CHECK(hipGraphLaunch(exec_, s));
                } else {
                    epoch(s);
                }
            }
            done += chunk;
            TR_CHECK(hipMemcpyAsync(act.data(), active_, sizeof(int) * T_, hipMemcpyDeviceToHost, s));
            TR_CHECK(hipStreamSynchronize(s));
            bool any = false;
            for (int t = 0; t < T_; ++t) any = any || act[t] != 0;
            if (!any) break;
        }
        return done;
    }

    // Capture the epoch graph now (no launch): callers that run several trainers from several host
    // threads capture them all first, from one thread, so no capture overlaps another thread's
    // HIP calls (fedmi/hpo/sweep.py).
    void prepare(uintptr_t stream) {
        if (!exec_) capture(reinterpret_cast<hipStream_t>(stream));
    }

    // Forward pass of all trials over an arbitrary row block (evaluation / predict):
    // logits of the last layer land in out [T][rows][ld = maxw].
    void predict_logits(uintptr_t Xp, int rows, uintptr_t ws, uintptr_t stream) {
        hipStream_t s = reinterpret_cast<hipStream_t>(stream);
        forward(reinterpret_cast<const T*>(Xp), rows, s, reinterpret_cast<T*>(ws), rows, /*gated*/ false);
    }

  private:
    // Arguments of the fused float64 step (mlp_fused_f64.hip); xb_ holds [T][B][dims[0]] there.
    SkfArgs fused_args(int off, int rows) const {
        SkfArgs a{};
        a.L = L_; a.T = T_; a.P = P_;
        for (int l = 0; l <= L_ && l <= SKF_MAXL; ++l) a.dims[l] = dims_[l];
        for (int l = 0; l < L_ && l < SKF_MAXL; ++l) { a.w_off[l] = w_off_[l]; a.b_off[l] = b_off_[l]; }
        a.X = reinterpret_cast<const double*>(X_); a.y = y_; a.perms = perms_; a.epoch_ctr = epoch_ctr_;
        a.n_perm = n_; a.off = off; a.rows = rows; a.Bmax = B_; a.maxw = maxw_; a.head = head_;
        // write the row pass's hand-off buffers through (sc1): FEDMI_SK_WTHRU=1; off by default --
        // it helped (400, 200) x 9 and hurt (50, 400) x 1 / x 9 (profiles/sk_store_policy_r5.log)
        const char* wt_env = std::getenv("FEDMI_SK_WTHRU");
        a.wthru = wt_env != nullptr && wt_env[0] == '1';
        a.inv_rows = 1.0 / (double)rows; a.alpha = alpha_; a.beta1 = beta1_; a.beta2 = beta2_; a.eps = eps_;
        a.l2_coef = 0.5 * alpha_;
        a.params = reinterpret_cast<double*>(params_); a.m = reinterpret_cast<double*>(m_);
        a.v = reinterpret_cast<double*>(v_); a.lr = lr_; a.step = step_; a.loss_acc = loss_acc_;
        a.active = active_;
        a.xg = reinterpret_cast<double*>(xb_); a.acts = reinterpret_cast<double*>(acts_);
        a.deltas = reinterpret_cast<double*>(deltas_);
        a.dbg = dbg_;
        a.zero = zero_;
        a.wt = wt_;
        a.split = split_;
        return a;
    }
    int split_ = 1;                      // tile-split row pass (SkfArgs::split)
    unsigned long long* dbg_ = nullptr;  // FEDMI_SK_STAMPS=1: phase stamps of the fused row pass
    double* zero_ = nullptr;             // SkfArgs::zero
    double* wt_ = nullptr;               // SkfArgs::wt (bufs["wt"], optional)
    bool fused_ = false;
    T* act(int l) const { return acts_ + (size_t)l * T_ * B_ * maxw_; }
    T* delta(int l) const { return deltas_ + (size_t)l * T_ * B_ * maxw_; }

    // acts layout [L][T][Bs][maxw]; x shared by all trials (row stride dims[0]).
    void forward(const T* x, int rows, hipStream_t s, T* acts, int Bs, bool gated = true) {
        for (int l = 0; l < L_; ++l) {
            const int K = dims_[l], N = dims_[l + 1];
            const T* A = l == 0 ? x : acts + (size_t)(l - 1) * T_ * Bs * maxw_;
            Ops::gemm(rows, N, K, A, l == 0 ? dims_[0] : maxw_, l == 0 ? 0 : (long long)Bs * maxw_, 1,
                      params_ + w_off_[l], K, P_, 1, acts + (size_t)l * T_ * Bs * maxw_, maxw_, (long long)Bs * maxw_,
                      params_ + b_off_[l], P_, nullptr, 0, 0, l + 1 < L_ ? GEMM_EPI_BIAS_RELU : GEMM_EPI_BIAS,
                      gated ? active_ : nullptr, T_, s);
        }
    }

    void capture(hipStream_t s) {
        drop_graph();
        TR_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        try {
            epoch(s);
        } catch (...) {
            hipGraph_t g;
            hipStreamEndCapture(s, &g);
            if (g) hipGraphDestroy(g);
            throw;
        }
        TR_CHECK(hipStreamEndCapture(s, &graph_));
        TR_CHECK(hipGraphInstantiate(&exec_, graph_, nullptr, nullptr, 0));
    }
    void drop_graph() {
        if (exec_) { hipGraphExecDestroy(exec_); exec_ = nullptr; }
        if (graph_) { hipGraphDestroy(graph_); graph_ = nullptr; }
    }

    std::vector<int> dims_, w_off_, b_off_;
    int T_, L_, P_, n_, B_, head_, style_, nic_, max_iter_, tol_stop_, maxw_;
    double beta1_, beta2_, eps_, alpha_, wd_, mu_, tol_;
    const T* X_;
    const int* y_;
    const int* perms_;
    int* epoch_ctr_;
    T *params_, *grads_, *m_, *v_;
    const T* anchor_;
    const unsigned char* wd_mask_;
    const double* lr_;
    long long* step_;
    double *loss_acc_, *best_, *curve_;
    int *count_, *n_iter_, *active_;
    T* xb_;
    int* yb_;
    T *acts_, *deltas_;
    hipGraph_t graph_ = nullptr;
    hipGraphExec_t exec_ = nullptr;
};

// Standalone layered GEMM entry (tests, wide-MLP path): dtype 0 f32 / 1 bf16.
static void gemm_py(int M, int N, int K, uintptr_t A, int lda, int a_kc, uintptr_t B, int ldb, int b_kc, uintptr_t C,
                    int ldc, int epi, uintptr_t bias, uintptr_t mask, int ldmask, int mask_bf16, float alpha,
                    float beta, int dtype, int splits, uintptr_t slab, uintptr_t Cbf16, uintptr_t stream) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    GemmArgs g{};
    g.M = M; g.N = N; g.K = K;
    g.A = reinterpret_cast<const void*>(A); g.lda = lda;
    g.B = reinterpret_cast<const void*>(B); g.ldb = ldb;
    g.bias = reinterpret_cast<const float*>(bias);
    g.mask = reinterpret_cast<const void*>(mask); g.ldmask = ldmask; g.mask_bf16 = mask_bf16;
    g.alpha = alpha;
    if (splits > 1) {
        g.C = reinterpret_cast<float*>(slab); g.ldc = ldc; g.beta = 0.f;
        g.slab_stride = (size_t)M * ldc;
        TR_CHECK(gemm_launch(g, dtype, a_kc, b_kc, GEMM_EPI_NONE, splits, 1, s));
        TR_CHECK(splitk_reduce_launch(reinterpret_cast<float*>(slab), (size_t)M * ldc, splits,
                                      reinterpret_cast<float*>(C), (size_t)M * ldc, beta, s));
    } else {
        g.C = reinterpret_cast<float*>(C); g.ldc = ldc; g.beta = beta;
        g.Cbf16 = reinterpret_cast<void*>(Cbf16);
        TR_CHECK(gemm_launch(g, dtype, a_kc, b_kc, epi, 1, 1, s));
    }
}

static void colsum_py(uintptr_t X, int M, int N, int ld, uintptr_t out, float beta, uintptr_t stream) {
    TR_CHECK(colsum_launch(reinterpret_cast<const float*>(X), M, N, ld, reinterpret_cast<float*>(out), beta, 1, 0, 0,
                           nullptr, reinterpret_cast<hipStream_t>(stream)));
}

static void to_bf16_py(uintptr_t x, uintptr_t y, size_t n, uintptr_t stream, float scale) {
    TR_CHECK(f32_to_bf16_launch(reinterpret_cast<const float*>(x), reinterpret_cast<void*>(y), n,
                                reinterpret_cast<hipStream_t>(stream), scale));
}

static void fedavg_delta_bf16_py(uintptr_t w, uintptr_t g, uintptr_t d, size_t n, float scale, uintptr_t stream) {
    TR_CHECK(fedavg_delta_bf16_launch(reinterpret_cast<const float*>(w), reinterpret_cast<const float*>(g),
                                      reinterpret_cast<void*>(d), n, scale, reinterpret_cast<hipStream_t>(stream)));
}

static void fedavg_apply_delta_py(uintptr_t w, uintptr_t g, uintptr_t d, size_t n, uintptr_t stream) {
    TR_CHECK(fedavg_apply_delta_launch(reinterpret_cast<float*>(w), reinterpret_cast<float*>(g),
                                       reinterpret_cast<const void*>(d), n, reinterpret_cast<hipStream_t>(stream)));
}

// Single-problem loss head (wide path): softmax CE (mode 0) / sklearn binary (mode 1).
static void xent_py(uintptr_t z, int ldz, uintptr_t y, int M, int C, int mode, float scale, uintptr_t dz, int lddz,
                    uintptr_t loss_acc, uintptr_t stream) {
    XentArgs a{};
    a.z = reinterpret_cast<const float*>(z); a.ldz = ldz; a.y = reinterpret_cast<const int*>(y);
    a.M = M; a.C = C; a.mode = mode; a.scale = scale;
    a.dz = reinterpret_cast<float*>(dz); a.lddz = lddz; a.loss_acc = reinterpret_cast<double*>(loss_acc);
    TR_CHECK(xent_launch(a, 1, reinterpret_cast<hipStream_t>(stream)));
}

// Single-problem torch-style Adam over a flat fp32 vector (host-side lr / step).
static void adam_flat_py(uintptr_t p, uintptr_t m, uintptr_t v, uintptr_t g, size_t n, double lr, double b1, double b2,
                         double eps, long long t, uintptr_t stream) {
    AdamArgs a{};
    a.p = reinterpret_cast<float*>(p); a.m = reinterpret_cast<float*>(m); a.v = reinterpret_cast<float*>(v);
    a.g = reinterpret_cast<const float*>(g); a.n = n; a.style = 0; a.beta1 = b1; a.beta2 = b2; a.eps = eps;
    a.lr_scalar = lr; a.step_scalar = t;
    TR_CHECK(adam_launch(a, 1, reinterpret_cast<hipStream_t>(stream)));
}

// bf16 NT GEMM (gemm_nt_bf16.hip): C = alpha * A[M][K] . B[N][K]^T with fused epilogue.
static void gemm_nt_py(int M, int N, int K, uintptr_t A, int lda, uintptr_t B, int ldb, uintptr_t C, int ldc,
                       uintptr_t Cbf16, int ldcb, uintptr_t CbT, int ldct, uintptr_t bias, uintptr_t mask, int ldmask,
                       int relu, float alpha, float beta, uintptr_t stream, uintptr_t csum, int ldcs) {
    NTArgs g{};
    g.csum = reinterpret_cast<float*>(csum); g.ldcs = ldcs;
    g.M = M; g.N = N; g.K = K;
    g.A = reinterpret_cast<const void*>(A); g.lda = lda;
    g.B = reinterpret_cast<const void*>(B); g.ldb = ldb;
    g.C = reinterpret_cast<float*>(C); g.ldc = ldc;
    g.Cbf16 = reinterpret_cast<void*>(Cbf16); g.ldcb = ldcb;
    g.CbT = reinterpret_cast<void*>(CbT); g.ldct = ldct;
    g.bias = reinterpret_cast<const float*>(bias);
    g.mask = reinterpret_cast<const void*>(mask); g.ldmask = ldmask;
    g.relu = relu; g.alpha = alpha; g.beta = beta;
    TR_CHECK(gemm_nt_bf16_launch(g, reinterpret_cast<hipStream_t>(stream)));
}

static void transpose_bf16_py(uintptr_t in, int R, int C, int ldi, uintptr_t out, int ldo, uintptr_t stream) {
    TR_CHECK(transpose_bf16_launch(reinterpret_cast<const float*>(in), R, C, ldi, reinterpret_cast<void*>(out), ldo,
                                   reinterpret_cast<hipStream_t>(stream)));
}

static void pad_bf16_py(uintptr_t in, int R, int C, long long rs, long long cs, uintptr_t out, int ldo,
                        uintptr_t stream) {
    TR_CHECK(pad_bf16_launch(reinterpret_cast<const float*>(in), R, C, rs, cs, reinterpret_cast<void*>(out), ldo,
                             reinterpret_cast<hipStream_t>(stream)));
}

static void rowsum_bf16_py(uintptr_t dT, int Nrows, int M, int ld, uintptr_t out, float beta, uintptr_t stream) {
    TR_CHECK(rowsum_bf16_launch(reinterpret_cast<const void*>(dT), Nrows, M, ld, reinterpret_cast<float*>(out), beta,
                                reinterpret_cast<hipStream_t>(stream)));
}

static void skinny_wgrad_py(uintptr_t W, int ldw, int Nw, uintptr_t S, int lds, int C, int rows, int trans,
                            int splits, uintptr_t slab, uintptr_t out, float beta, uintptr_t bias_out,
                            uintptr_t stream) {
    TR_CHECK(skinny_wgrad_launch(reinterpret_cast<const void*>(W), ldw, Nw, reinterpret_cast<const void*>(S), lds, C,
                                 rows, trans, splits, reinterpret_cast<float*>(slab), reinterpret_cast<float*>(out),
                                 beta, reinterpret_cast<float*>(bias_out), reinterpret_cast<hipStream_t>(stream)));
}

static void colsum_split_py(uintptr_t X, int M, int N, int splits, uintptr_t slab, uintptr_t out, float beta,
                            uintptr_t stream) {
    TR_CHECK(colsum_split_launch(reinterpret_cast<const float*>(X), M, N, splits, reinterpret_cast<float*>(slab),
                                 reinterpret_cast<float*>(out), beta, reinterpret_cast<hipStream_t>(stream)));
}

static void logits_confusion_py(uintptr_t z, int ldz, uintptr_t y, int M, int C, uintptr_t cm, uintptr_t stream) {
    TR_CHECK(logits_confusion_launch(reinterpret_cast<const float*>(z), ldz, reinterpret_cast<const int*>(y), M, C,
                                     reinterpret_cast<float*>(cm), reinterpret_cast<hipStream_t>(stream)));
}

void register_trainer(py::module_& m) {
    m.def("logits_confusion", &logits_confusion_py);
    // sklearn's per-epoch shuffles (sk_perms.cpp): (key uint32[624], pos, n, epochs) -> (perms int32
    // [epochs][n], key, pos) -- numpy's MT19937 stream, state in / state out
    m.def("sk_epoch_perms", [](py::array_t<uint32_t, py::array::c_style | py::array::forcecast> key, int pos, int n,
                               int epochs) {
        if (key.size() != 624 || n < 1 || epochs < 0 || pos < 0 || pos > 624)
            throw std::runtime_error("sk_epoch_perms: bad MT19937 state or sizes");
        std::vector<uint32_t> k(key.data(), key.data() + 624);
        py::array_t<int32_t> perms({(py::ssize_t)epochs, (py::ssize_t)n});
        {
            py::gil_scoped_release nogil;
            sk_epoch_perms(k.data(), &pos, n, epochs, perms.mutable_data());
        }
        py::array_t<uint32_t> kout(624);
        std::copy(k.begin(), k.end(), kout.mutable_data());
        return py::make_tuple(perms, kout, pos);
    });
    // the tile-split row pass's slice rule (host arithmetic, CPU-testable): dims = [F, h0, h1, C]
    m.def("sk_pick_split", [](std::vector<int> dims, int T, int Bmax, int want, int cus) {
        SkfArgs a;
        std::memset(&a, 0, sizeof(a));
        if (dims.size() < 2 || (int)dims.size() > SKF_MAXL + 1) throw std::runtime_error("sk_pick_split: bad dims");
        a.L = (int)dims.size() - 1;
        for (size_t i = 0; i < dims.size(); ++i) a.dims[i] = dims[i];
        a.T = T;
        a.Bmax = Bmax;
        return skf_pick_split(a, want, cus);
    });
    m.def("colsum_split", &colsum_split_py);
    m.def("skinny_wgrad", &skinny_wgrad_py);
    m.def("gemm_nt", &gemm_nt_py, py::arg("M"), py::arg("N"), py::arg("K"), py::arg("A"), py::arg("lda"), py::arg("B"),
          py::arg("ldb"), py::arg("C"), py::arg("ldc"), py::arg("Cbf16"), py::arg("ldcb"), py::arg("CbT"), py::arg("ldct"),
          py::arg("bias"), py::arg("mask"), py::arg("ldmask"), py::arg("relu"), py::arg("alpha"), py::arg("beta"),
          py::arg("stream"), py::arg("csum") = 0, py::arg("ldcs") = 0);
    m.def("gemm_nt_set_variant", &gemm_nt_set_variant);
    m.def("gemm_nt_set_debug", [](uintptr_t p) { gemm_nt_set_debug(reinterpret_cast<unsigned long long*>(p)); });
    m.def("transpose_bf16", &transpose_bf16_py);
    m.def("rowsum_bf16", &rowsum_bf16_py);
    m.def("pad_bf16", &pad_bf16_py);
    m.def("xent", &xent_py);
    m.def("fedavg_delta_bf16", &fedavg_delta_bf16_py);
    m.def("fedavg_apply_delta", &fedavg_apply_delta_py);
    m.def("adam_flat", &adam_flat_py);
    py::class_<MLPTrainerT<float>>(m, "MLPTrainer")
        .def(py::init<std::vector<int>, int, py::dict, py::dict>())
        .def("run", &MLPTrainerT<float>::run, py::arg("n_epochs"), py::arg("stream"), py::arg("check_every") = 8,
             py::arg("use_graph") = true, py::call_guard<py::gil_scoped_release>())
        .def("prepare", &MLPTrainerT<float>::prepare)
        .def("predict_logits", &MLPTrainerT<float>::predict_logits)
        .def_property_readonly("fused", &MLPTrainerT<float>::fused)
        .def_property_readonly("P", &MLPTrainerT<float>::P);
    py::class_<MLPTrainerT<double>>(m, "MLPTrainer64")
        .def(py::init<std::vector<int>, int, py::dict, py::dict>())
        .def("run", &MLPTrainerT<double>::run, py::arg("n_epochs"), py::arg("stream"), py::arg("check_every") = 8,
             py::arg("use_graph") = true, py::call_guard<py::gil_scoped_release>())
        .def("prepare", &MLPTrainerT<double>::prepare)
        .def("predict_logits", &MLPTrainerT<double>::predict_logits)
        .def_property_readonly("fused", &MLPTrainerT<double>::fused)
        .def_property_readonly("split", &MLPTrainerT<double>::split)
        .def("stamps", &MLPTrainerT<double>::stamps)
        .def_property_readonly("P", &MLPTrainerT<double>::P);
    m.def("gemm", &gemm_py);
    m.def("colsum", &colsum_py);
    m.def("to_bf16", &to_bf16_py, py::arg("x"), py::arg("y"), py::arg("n"), py::arg("stream"), py::arg("scale") = 1.f);
}
