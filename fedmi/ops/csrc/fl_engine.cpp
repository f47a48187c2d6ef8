// Native runtime of the federated round engine: kernel sequencing, HIP-graph capture of
// whole rounds, and an RCCL communicator owned by the engine (no torch / pickle in the
// round loop).  Exposed to Python as module `fedmi.ops._fedmi_hip` (pybind11).
//
// The reference runs the round loop in Python with 3 gathers + 3 bcasts + (2 + 2k)
// barriers per round (FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py:130-201,
// SURVEY §2.4).  Here `FLEngine::run` issues, per round, three kernels and one
// ncclAllReduce on the caller's stream; `capture` records an even number of rounds into a
// hipGraph that is replayed with one host call.  Early stopping is decided on the device,
// so nothing in the loop waits on the host.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <cmath>
#include <thread>
#include <vector>

#include "fl_common.h"
#include "fl_layout.h"
#include "peer_allreduce.h"

namespace py = pybind11;

#define HIP_CHECK(expr)                                                                       \
    do {                                                                                      \
        hipError_t _e = (expr);                                                               \
        if (_e != hipSuccess)                                                                 \
            throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) +     \
                                     " at " #expr);                                           \
    } while (0)

#define NCCL_CHECK(expr)                                                                      \
    do {                                                                                      \
        ncclResult_t _r = (expr);                                                             \
        if (_r != ncclSuccess)                                                                \
            throw std::runtime_error(std::string("RCCL error ") + ncclGetErrorString(_r) +   \
                                     " at " #expr);                                           \
    } while (0)

hipError_t fl_set_lds_limit(size_t bytes);  // fl_kernels.hip
void register_trainer(pybind11::module_& m);  // mlp_trainer.cpp

static inline hipStream_t as_stream(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }
template <typename T>
static inline T* as_ptr(uintptr_t p) { return reinterpret_cast<T*>(p); }

// ---------------------------------------------------------------------------------------
// RCCL communicator: one per process (= one per GPU / federated client).
// ---------------------------------------------------------------------------------------
//
// The communicator is NON-BLOCKING (ncclConfig_t::blocking = 0): ncclCommInitRankConfig returns at
// once and the bootstrap (unique-id rendezvous, topology, rings) runs inside RCCL while this thread
// polls ncclCommGetAsyncError against a deadline with the GIL released.  A peer that never calls
// init (died before it, stuck elsewhere) therefore ends in ncclCommAbort and a Python exception
// naming the deadline, not in a process blocked forever inside ncclCommInitRank -- the reference's
// contract is "any failure -> comm.Abort()" (C:203-205).  Every later call on a non-blocking
// communicator may also return ncclInProgress (e.g. the lazy connection set-up of the first
// collective); `settle` waits those out under the same deadline.
class RcclComm {
  public:
    RcclComm(int nranks, int rank, py::bytes uid, int device, double timeout_s)
        : nranks_(nranks), rank_(rank), timeout_s_(timeout_s) {
        std::string s = uid;
        if (s.size() != sizeof(ncclUniqueId)) throw std::runtime_error("bad RCCL unique id size");
        ncclUniqueId id;
        std::memcpy(&id, s.data(), sizeof(id));
        HIP_CHECK(hipSetDevice(device));
        ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
        cfg.blocking = 0;
        ncclResult_t r;
        {
            py::gil_scoped_release nogil;
            r = ncclCommInitRankConfig(&comm_, nranks, id, rank, &cfg);
            if (r == ncclSuccess || r == ncclInProgress) r = wait_settled();
        }
        if (r != ncclSuccess) {
            if (comm_) {
                py::gil_scoped_release nogil;
                ncclCommAbort(comm_);
            }
            comm_ = nullptr;
            if (r == ncclInProgress)
                throw std::runtime_error("RCCL bootstrap timed out after " + std::to_string(timeout_s_) +
                                         " s (rank " + std::to_string(rank) + " of " + std::to_string(nranks) +
                                         "): a peer never joined ncclCommInitRankConfig; communicator aborted");
            throw std::runtime_error(std::string("RCCL bootstrap failed: ") + ncclGetErrorString(r));
        }
    }
    ~RcclComm() { destroy(); }

    static py::bytes unique_id() {
        ncclUniqueId id;
        NCCL_CHECK(ncclGetUniqueId(&id));
        return py::bytes(reinterpret_cast<const char*>(&id), sizeof(id));
    }

    void allreduce_f32(uintptr_t buf, size_t count, uintptr_t stream) {
        settle(ncclAllReduce(as_ptr<float>(buf), as_ptr<float>(buf), count, ncclFloat32, ncclSum, live(),
                             as_stream(stream)), "ncclAllReduce(f32)");
    }
    void allreduce_bf16(uintptr_t buf, size_t count, uintptr_t stream) {
        settle(ncclAllReduce(as_ptr<void>(buf), as_ptr<void>(buf), count, ncclBfloat16, ncclSum, live(),
                             as_stream(stream)), "ncclAllReduce(bf16)");
    }
    void allreduce_f64(uintptr_t buf, size_t count, uintptr_t stream) {
        settle(ncclAllReduce(as_ptr<double>(buf), as_ptr<double>(buf), count, ncclFloat64, ncclSum, live(),
                             as_stream(stream)), "ncclAllReduce(f64)");
    }
    void broadcast_bytes(uintptr_t buf, size_t nbytes, int root, uintptr_t stream) {
        settle(ncclBroadcast(as_ptr<void>(buf), as_ptr<void>(buf), nbytes, ncclUint8, root, live(),
                             as_stream(stream)), "ncclBroadcast");
    }
    void allgather_f32(uintptr_t send, uintptr_t recv, size_t count, uintptr_t stream) {
        settle(ncclAllGather(as_ptr<float>(send), as_ptr<float>(recv), count, ncclFloat32, live(),
                             as_stream(stream)), "ncclAllGather");
    }
    // ncclCommGetAsyncError of a live communicator (0 = ncclSuccess); lets a watchdog see an
    // asynchronous RCCL failure without issuing a collective.
    int async_error() const {
        if (!comm_) return (int)ncclInvalidArgument;
        ncclResult_t st = ncclSuccess;
        ncclCommGetAsyncError(comm_, &st);
        return (int)st;
    }
    void abort() {
        if (comm_) {
            ncclCommAbort(comm_);
            comm_ = nullptr;
        }
    }
    void destroy() {
        if (comm_) {
            ncclCommDestroy(comm_);
            comm_ = nullptr;
        }
    }
    int rank() const { return rank_; }
    int size() const { return nranks_; }
    ncclComm_t handle() const { return comm_; }

  private:
    ncclComm_t live() const {
        if (!comm_) throw std::runtime_error("RCCL communicator used after abort/destroy");
        return comm_;
    }
    // Poll the communicator's state until it leaves ncclInProgress or the deadline passes
    // (returns ncclInProgress then).  Called without the GIL.
    ncclResult_t wait_settled() const {
        const auto t_end = std::chrono::steady_clock::now() +
                           std::chrono::microseconds((long long)(timeout_s_ * 1e6));
        ncclResult_t st = ncclInProgress;
        for (;;) {
            if (ncclCommGetAsyncError(comm_, &st) != ncclSuccess) return ncclInternalError;
            if (st != ncclInProgress) return st;
            if (std::chrono::steady_clock::now() >= t_end) return ncclInProgress;
            std::this_thread::sleep_for(std::chrono::microseconds(200));
        }
    }
    void settle(ncclResult_t r, const char* what) {
        if (r == ncclInProgress) {
            if (PyGILState_Check()) {
                py::gil_scoped_release nogil;
                r = wait_settled();
            } else {
                r = wait_settled();
            }
        }
        if (r != ncclSuccess)
            throw std::runtime_error(std::string("RCCL error ") +
                                     (r == ncclInProgress ? "timeout" : ncclGetErrorString(r)) + " in " + what);
    }
    int nranks_, rank_;
    double timeout_s_;
    ncclComm_t comm_ = nullptr;
};

// ---------------------------------------------------------------------------------------
// Engine
// ---------------------------------------------------------------------------------------
class TrialBatch;

// One launch of a round, as recorded for a trial batch (TrialBatch below) instead of issued.
struct FLLaunchRec {
    enum Kind { PACK, TRAIN, ADAM, EVAL, FINALIZE };
    int kind;
    int i[4];           // TRAIN: ls, stage_local, mode, fold_mask | ADAM: ls, fold, tail_a, fold_mask |
                        // FINALIZE: mask
    const void* p[5];   // pointer arguments in launcher order
};

class FLEngine {
    friend class TrialBatch;

  public:
    FLEngine(std::vector<int> dims, py::dict cfg, py::dict bufs) {
        const int L = (int)dims.size() - 1;
        if (L < 1 || L > FL_MAX_LAYERS) throw std::runtime_error("FLEngine: 1..4 Linear layers supported");
        std::memset(&d_, 0, sizeof(d_));
        std::memset(&c_, 0, sizeof(c_));
        std::memset(&b_, 0, sizeof(b_));
        c_.R = cfg["R"].cast<int>();
        if (c_.R != 16 && c_.R != 32 && c_.R != 64) throw std::runtime_error("FLEngine: R must be 16, 32 or 64");
        const int C = dims[L];
        if (C > FL_MAX_CLASSES) throw std::runtime_error("FLEngine: at most 16 classes");
        if (dims[0] > 4096) throw std::runtime_error("FLEngine: too many features");
        fl_build_fp32_layout(dims.data(), L, c_.R, &d_);   // fl_layout.h (host-tested with sanitizers)
        const int lds = d_.lds_floats;
        dtype_ = cfg.contains("dtype") ? cfg["dtype"].cast<int>() : 0;
        if (dtype_ == 0) {
            if (c_.R == 64) throw std::runtime_error("FLEngine: R = 64 needs the bf16 kernels");
            if ((size_t)lds * 4 > FL_LDS_DYNAMIC_MAX)
                throw std::runtime_error("FLEngine: activations exceed LDS; use a smaller R or the layered path");
            HIP_CHECK(fl_set_lds_limit((size_t)lds * 4));
        } else {
            fl_build_bf16_layout(d_, c_.R, &e_, &ev_);
            // FEDMI_LAG_REG=0: lagged rounds score before the training pass instead of beside it (A/B)
            const char* lreg_env = std::getenv("FEDMI_LAG_REG");
            if (lreg_env != nullptr && lreg_env[0] == '0') e_.lag_reg = ev_.lag_reg = 0;
            const size_t need = (size_t)std::max(e_.lds_bytes, ev_.lds_bytes);
            if (need > FL_LDS_DYNAMIC_MAX)
                throw std::runtime_error("FLEngine(bf16): model exceeds LDS; use a smaller R or the layered path");
            HIP_CHECK(fl_set_lds_limit_bf16(need));
        }

        c_.n_rows = cfg["n_rows"].cast<int>();
        c_.inv_n = 1.0f / (float)c_.n_rows;
        c_.world = cfg["world"].cast<int>();
        c_.rank = cfg["rank"].cast<int>();
        if (c_.world > FL_MAX_WORLD) throw std::runtime_error("FLEngine: world too large");
        c_.agg_scale = cfg["agg_scale"].cast<float>();
        c_.slab_stride = ((d_.P + 1) + 3) & ~3;
        c_.n_slabs = (c_.n_rows + c_.R - 1) / c_.R;
        // bf16 kernels: fp16 gradient partials unless the caller asks for fp32 (engine.py grad_slab)
        c_.slab_f16 = dtype_ == 1 && (cfg.contains("slab_f16") ? cfg["slab_f16"].cast<bool>() : true) ? 1 : 0;
        c_.tail_off = d_.Pimg;
        c_.tail_stride = C * C + 1;
        c_.tail_len = c_.world * c_.tail_stride;
        c_.local_steps = cfg["local_steps"].cast<int>();
        c_.lr0 = cfg["lr"].cast<double>();
        c_.gamma = cfg["gamma"].cast<double>();
        c_.step_size = cfg["step_size"].cast<int>();
        c_.beta1 = cfg["beta1"].cast<double>();
        c_.beta2 = cfg["beta2"].cast<double>();
        c_.omb1 = (float)(1.0 - c_.beta1);
        c_.omb2 = (float)(1.0 - c_.beta2);
        c_.beta2f = (float)c_.beta2;
        c_.eps = (float)cfg["eps"].cast<double>();
        c_.weight_decay = (float)cfg["weight_decay"].cast<double>();
        c_.prox_mu = (float)cfg["prox_mu"].cast<double>();
        c_.es_enabled = cfg["early_stop"].cast<bool>() ? 1 : 0;
        c_.patience = cfg["patience"].cast<int>();
        c_.atol = cfg["atol"].cast<double>();
        c_.rtol = cfg["rtol"].cast<double>();
        c_.max_rounds = cfg["max_rounds"].cast<int>();
        c_.metric_mode = cfg["metric_mode"].cast<int>();
        // Fused evaluation needs the round's input weights to BE the previous round's
        // post-step local model: one client (FedAvg of one is the identity, agg_scale 1).
        fused_ = cfg.contains("fused_eval") && cfg["fused_eval"].cast<bool>() && c_.world == 1 &&
                 c_.agg_scale == 1.0f;
        eval_fedavg_ = !cfg.contains("eval_fedavg") || cfg["eval_fedavg"].cast<bool>();
        // Lagged evaluation (fl_common.h FL_EVAL_LAGGED): several clients, early stopping off,
        // bf16 kernels, and room in LDS for the second parameter image.  The comm buffer then
        // carries the lag region A after the tails (the caller sized it: comm_len).
        const bool lag_req = cfg.contains("lagged_eval") && cfg["lagged_eval"].cast<bool>();
        if (lag_req) c_.lag_off = d_.Pimg + c_.tail_len;
        comm_len_ = d_.Pimg + c_.tail_len * (lag_req ? 2 : 1);
        const bool emulate = cfg.contains("emulate_clients") && cfg["emulate_clients"].cast<bool>();
        emulate_ = emulate;
        // (with early stopping the rounds are lagged when the FedAvg runs inside the Adam kernel,
        // which folds the metrics in time, or rides RCCL, folded one round late: see lagged())
        // (the lagged train kernel scores the previous local model in the train layout itself)
        lag_ok_ = lag_req && dtype_ == 1 && (c_.world > 1 || emulate) && !fused_;
        // several clients + register scoring: the training forward pass is plain bf16 (no round
        // scores from it), in every round kind of the engine alike (lagged, classic, step API).
        // cfg["plain_fwd"] (EngineConfig.plain_fwd): -1 auto, 0 off, 1 on wherever valid;
        // FEDMI_PLAIN_FWD=0 forces the split forward (A/B builds)
        {
            const int req = cfg.contains("plain_fwd") ? cfg["plain_fwd"].cast<int>() : -1;
            const char* pf = std::getenv("FEDMI_PLAIN_FWD");
            const bool valid = dtype_ == 1 && e_.lag_reg && !fused_;
            const bool want = req < 0 ? (c_.world > 1 || emulate) : req > 0;
            c_.plain_fwd = (valid && want && !(pf != nullptr && pf[0] == '0')) ? 1 : 0;
        }
        // split scoring: with register scoring (e_.lag_reg) and a train grid that leaves at least as
        // many CUs idle as it occupies, lagged rounds score on workgroups of their own (the shards
        // of 4-8 clients); FEDMI_SPLIT_SCORE=0 / 1 forces it off / on (A/B)
        {
            int cus = 0, dev = 0;
            if (hipGetDevice(&dev) != hipSuccess ||
                hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
                cus = 0;
            const char* ss = std::getenv("FEDMI_SPLIT_SCORE");
            const bool force_on = ss != nullptr && ss[0] == '1', force_off = ss != nullptr && ss[0] == '0';
            c_.split_score = (lag_ok_ && dtype_ == 1 && e_.lag_reg && !force_off &&
                              (force_on || 2 * c_.n_slabs <= cus)) ? 1 : 0;
        }

        b_.X = as_ptr<const float>(bufs["X"].cast<uintptr_t>());
        b_.y = as_ptr<const int>(bufs["y"].cast<uintptr_t>());
        b_.slab = as_ptr<float>(bufs["slab"].cast<uintptr_t>());
        b_.local = as_ptr<float>(bufs["local"].cast<uintptr_t>());
        b_.m = as_ptr<float>(bufs["m"].cast<uintptr_t>());
        b_.v = as_ptr<float>(bufs["v"].cast<uintptr_t>());
        b_.hist_global = as_ptr<double>(bufs["hist_global"].cast<uintptr_t>());
        b_.hist_rank = as_ptr<double>(bufs["hist_rank"].cast<uintptr_t>());
        b_.hist_loss = as_ptr<float>(bufs["hist_loss"].cast<uintptr_t>());
        pbuf_[0] = as_ptr<float>(bufs["params0"].cast<uintptr_t>());
        pbuf_[1] = as_ptr<float>(bufs["params1"].cast<uintptr_t>());
        st_[0] = as_ptr<FLState>(bufs["state0"].cast<uintptr_t>());
        st_[1] = as_ptr<FLState>(bufs["state1"].cast<uintptr_t>());
        // Adam/StepLR schedule and per-round FedAvg table (fl_common.h FLBuffers::sched / rtab):
        // host-built device tables owned by the caller
        b_.sched = as_ptr<const float>(bufs["sched"].cast<uintptr_t>());
        b_.rtab = as_ptr<const float>(bufs["rtab"].cast<uintptr_t>());
        b_.sat = bufs.contains("sat") ? as_ptr<int>(bufs["sat"].cast<uintptr_t>()) : nullptr;
        {
            // FL_EVAL_LAGGED: previous round's counts + loss (zero)
            const size_t nlag = FL_MAX_CLASSES * FL_MAX_CLASSES + 4;
            HIP_CHECK(hipMalloc(&lagbuf_, nlag * sizeof(float)));
            HIP_CHECK(hipMemset(lagbuf_, 0, nlag * sizeof(float)));
            b_.cnt = lagbuf_;
            b_.lbuf = lagbuf_ + FL_MAX_CLASSES * FL_MAX_CLASSES;
        }
        if (dtype_ == 1) {
            // packed bf16 parameter regions; padding stays zero forever
            HIP_CHECK(hipMalloc(&pk_, 2 * (size_t)e_.param_bytes));
            HIP_CHECK(hipMemset(pk_, 0, 2 * (size_t)e_.param_bytes));
            b_.pk_global = pk_;
            b_.pk_local = pk_ + e_.param_bytes;
        }
        if (lag_ok_ && c_.es_enabled) {
            // pre-round [local | m | v | packed local image] for a round a late fold discards
            // (FLBuffers::undo); used only while late_fold() (refresh_undo)
            if ((e_.param_bytes & 3) != 0 || (d_.Pimg & 3) != 0)
                throw std::runtime_error("undo buffer: image sizes must be multiples of 4");
            const size_t bytes = 3 * (size_t)d_.Pimg * sizeof(float) + (dtype_ == 1 ? (size_t)e_.param_bytes : 0);
            HIP_CHECK(hipMalloc(&undo_, bytes));
            HIP_CHECK(hipMemset(undo_, 0, bytes));
            b_.undo_pk_bytes = dtype_ == 1 ? e_.param_bytes : 0;
        }
        refresh_undo();
    }

    ~FLEngine() {
        drop_graph();
        if (undo_) (void)hipFree(undo_);
        if (pk_) (void)hipFree(pk_);
        if (lagbuf_) (void)hipFree(lagbuf_);
    }

    // Issue rounds [r0, r0 + n): per round the train/Adam pair (one per local step), the
    // evaluation (classic rounds) and, when world > 1, one all-reduce.
    // Lagged engines (several clients, no early stop) issue every round lagged except, with
    // `close`, the last, which evaluates itself: after it every metric is in the buffers.
    void run(int r0, int n, uintptr_t stream, RcclComm* comm, bool close = true) {
        hipStream_t s = as_stream(stream);
        for (int r = r0; r < r0 + n; ++r) issue_round(r, s, comm, true, lagged() && !(close && r == r0 + n - 1));
    }

    // Local part of round r (no all-reduce; the caller reduces a shared buffer).
    void run_local(int r, uintptr_t stream) { issue_round(r, as_stream(stream), nullptr, false); }

    // One phase of round r: 0 = local training (all local steps), 1 = local evaluation,
    // 2 = FedAvg all-reduce.  Used by the step-by-step reference API
    // (train_one_epoch / evaluate_local / federated_averaging); always classic rounds.
    void phase(int r, int which, uintptr_t stream, RcclComm* comm) {
        hipStream_t s = as_stream(stream);
        if (which == 0) {
            flush_pending_eval(r, s);
            issue_train(r, s, false);
            prev_lagged_ = false;
        } else if (which == 1) {
            issue_eval(r, s);
            cm_in_tail_ = true;
        } else if (which == 2) {
            issue_allreduce(r, s, comm);
        } else {
            throw std::runtime_error("phase: 0, 1 or 2");
        }
    }

    // Fold every pending metric into the state / history (host synchronisation point); `r`
    // = rounds issued.  A fused last round is evaluated first.
    void finalize(int r, uintptr_t stream) {
        hipStream_t s = as_stream(stream);
        flush_pending_eval(r, s);
        if (prev_lagged_)
            throw std::runtime_error("finalize: the last round is lagged (its metrics need one more round)");
        const int mask = (prev_scored_ && !prev_afold_ ? FL_FOLD_A : 0) | FL_FOLD_B;
        if (rec_ != nullptr)
            rec_->push_back({FLLaunchRec::FINALIZE, {mask, 0, 0, 0}, {pbuf_[r & 1], st_[r & 1], st_[(r + 1) & 1]}});
        else
            HIP_CHECK(fl_launch_finalize(d_, c_, b_, pbuf_[r & 1], st_[r & 1], st_[(r + 1) & 1], s, mask,
                                         late_fold() ? pbuf_[(r + 1) & 1] : nullptr));
        cm_in_tail_ = false;
    }

    // Record `n` rounds (n even, starting at an even round) into one hipGraph.  Round
    // indices live on the device, so the same graph is replayed for every chunk.  A graph
    // always starts from the steady state (see needs_eager_round).
    //
    // Captured graphs are cached by round count (up to kMaxGraphs): callers that alternate
    // between graph lengths (run() at cfg.graph_rounds, the streaming console's shorter chunks
    // of lagged engines) select the instantiated graph again instead of re-capturing it (ADVICE
    // r4).  A graph is a pure function of the engine's configuration and buffers -- every change
    // of those drops the cache (drop_graph) -- except a pending repack of host-written weights
    // (need_pack_), which is captured into the graph's first round: with one pending the graph is
    // captured afresh.
    void capture(int n, uintptr_t stream, RcclComm* comm) {
        if (n <= 0 || (n & 1)) throw std::runtime_error("capture: n must be a positive even number");
        if (needs_eager_round()) throw std::runtime_error("capture: issue one eager round first");
        for (size_t i = 0; i < graphs_.size(); ++i)
            if (graphs_[i].n == n) {
                if (!need_pack_ && graphs_[i].comm == comm) {
                    select_graph((int)i);
                    return;
                }
                destroy_rec(graphs_[i]);
                graphs_.erase(graphs_.begin() + i);
                break;
            }
        if ((int)graphs_.size() >= kMaxGraphs) {
            destroy_rec(graphs_.front());
            graphs_.erase(graphs_.begin());
        }
        graph_ = nullptr;
        exec_ = nullptr;
        hipStream_t s = as_stream(stream);
        const bool pend = pending_cm_, tail = cm_in_tail_, plag = prev_lagged_, pscore = prev_scored_,
                   pafold = prev_afold_;
        const long long ev0 = eval_launches_;
        HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        try {
            for (int r = 0; r < n; ++r) issue_round(r, s, comm, true, lagged());
        } catch (...) {
            hipGraph_t g;
            hipStreamEndCapture(s, &g);
            if (g) hipGraphDestroy(g);
            pending_cm_ = pend;
            cm_in_tail_ = tail;
            prev_lagged_ = plag;
            prev_scored_ = pscore;
            prev_afold_ = pafold;
            eval_launches_ = ev0;
            throw;
        }
        GraphRec rec{n, nullptr, nullptr, eval_launches_ - ev0 /* counted per replay, not at capture */, comm};
        HIP_CHECK(hipStreamEndCapture(s, &rec.g));
        if (hipGraphInstantiate(&rec.e, rec.g, nullptr, nullptr, 0) != hipSuccess) {
            hipGraphDestroy(rec.g);
            throw std::runtime_error("capture: hipGraphInstantiate failed");
        }
        graphs_.push_back(rec);
        ++captures_;
        select_graph((int)graphs_.size() - 1);
        eval_launches_ = ev0;
        pending_cm_ = pend;  // nothing ran yet: replay() applies the rounds' effect
        cm_in_tail_ = tail;
        prev_lagged_ = plag;
        prev_scored_ = pscore;
        prev_afold_ = pafold;
    }

    void replay(uintptr_t stream) {
        if (!exec_) throw std::runtime_error("replay: no captured graph");
        if (needs_eager_round()) throw std::runtime_error("replay: issue one eager round first");
        HIP_CHECK(hipGraphLaunch(exec_, as_stream(stream)));
        eval_launches_ += graph_evals_;
        pending_cm_ = fused_;
        cm_in_tail_ = !fused_;
        prev_lagged_ = lagged();
        prev_scored_ = lagged();
        prev_afold_ = lagged() && xchg_;
    }

    int graph_rounds() const { return graph_rounds_; }
    long long graph_captures() const { return captures_; }
    // Stand-alone evaluation kernels issued so far (eager launches + every graph replay's):
    // a one-client fused run launches one per host-side weight change / run end, not per round.
    long long eval_launches() const { return eval_launches_; }

    // Host-side round bookkeeping (which metrics the last issued round left pending) as a bit
    // set.  A caller that captures rounds of this engine into its own graph (a trial group)
    // reads it after the capture and restores it after every replay of that graph.
    int flags() const {
        return (pending_cm_ ? 1 : 0) | (cm_in_tail_ ? 2 : 0) | (prev_lagged_ ? 4 : 0) | (prev_scored_ ? 8 : 0) |
               (prev_afold_ ? 16 : 0) | (need_pack_ ? 32 : 0);
    }
    void set_flags(int f) {
        pending_cm_ = f & 1;
        cm_in_tail_ = f & 2;
        prev_lagged_ = f & 4;
        prev_scored_ = f & 8;
        prev_afold_ = f & 16;
        need_pack_ = f & 32;
    }

    // The captured rounds assume the steady state of their kind: a fused graph must not
    // start behind a classic round (whose counts already sit in the tail), a classic graph
    // not behind a fused one (whose counts were never computed).
    // A lagged graph must start behind a lagged round that scored ITS predecessor: the first
    // captured round's fold mask (region A of the round before) is fixed at capture, and every
    // replay after the first starts behind such a round.  (Captured behind a lagged round that
    // followed a self-evaluating one -- e.g. a warm-up that closed on an odd round count -- every
    // replay's first round skipped the region-A fold: that round's metrics never reached the
    // history or the early-stop rule.  The Adam-fused exchange folds in time and was unaffected.)
    bool needs_eager_round() const {
        if (lagged()) return !prev_lagged_ || !prev_scored_;
        return fused_ ? cm_in_tail_ : pending_cm_;
    }
    // Lagged rounds: allowed by the layout, and either no early stopping (metrics may be
    // folded one round late), the Adam-fused exchange (which folds them in time) or an
    // external all-reduce (RCCL: folded one round late, a round run past a stop is discarded
    // bit-exactly -- late_fold()).  A peer all-reduce kernel without the in-kernel exchange
    // (several local steps) keeps classic rounds with early stopping: its send buffer is not the
    // output buffer a late stop republishes from.
    bool lagged() const { return lag_ok_ && (!c_.es_enabled || xchg_ || peer_ == nullptr); }
    bool late_fold() const { return lagged() && c_.es_enabled && !xchg_; }
    // The kernels keep / restore the pre-round state only where a round can be discarded.
    void refresh_undo() { b_.undo = (late_fold() && undo_ != nullptr) ? undo_ : nullptr; }
    bool adam_exchange() const { return xchg_; }
    bool fused() const { return fused_; }

    // Early-stop parameters (train_and_evaluate(termination_patience, tolerance), C:122): the
    // kernels take FLConfig by value, so a captured graph is dropped; the caller rewrites the
    // round state's patience counter before the first round.
    void set_early_stop(int patience, double atol, double rtol) {
        if (patience < 1) throw std::runtime_error("set_early_stop: patience must be >= 1");
        c_.patience = patience;
        c_.atol = atol;
        c_.rtol = rtol;
        drop_graph();
    }

    // The host wrote the global weights (set_weights / resume): the next round repacks them.
    void invalidate() { need_pack_ = true; }

    // The host loaded a complete round state (resume): no metrics are pending.
    void reset_pending() {
        pending_cm_ = false;
        cm_in_tail_ = false;
        prev_lagged_ = false;
        prev_scored_ = false;
        prev_afold_ = false;
    }

    // Aggregate with the one-shot xGMI all-reduce (peer_allreduce.hip) instead of RCCL: every
    // round publishes into the peer object's send buffers, and its kernel writes the reduced
    // image into this engine's parameter buffer (plus, in bf16 mode, the packed bf16 image).
    void attach_peer(PeerAllReduce& p) {
        // (world 1 is accepted: a one-rank "all-reduce" emulates the multi-client round on
        // one GPU for measurements, tools/round_emulate.py)
        if (fused_ || p.world() != c_.world || p.rank() != c_.rank || !p.is_open())
            throw std::runtime_error("attach_peer: communicator does not match this engine");
        if (p.n_floats() != comm_len_)
            throw std::runtime_error("attach_peer: buffer length != parameter image + tails");
        drop_graph();
        peer_ = &p;
        p.prepare_eval((c_.n_rows + c_.R - 1) / c_.R);
        // lagged rounds reduce inside the Adam kernel when the communicator has a chunk-flag
        // table for every Adam block (+ the tail block); one local step per round
        // (chunks: every Adam block, the tail block and the early lag-region chunk)
        xchg_ = lag_ok_ && c_.local_steps == 1 && p.n_chunks() >= (d_.P + 63) / 64 + 2;
        refresh_undo();
        std::memset(&pp_, 0, sizeof(pp_));
        if (dtype_ == 1) {
            pp_.pk = b_.pk_global;
            pp_.wlo_delta = e_.wlo_delta;
            pp_.pk_wgap = e_.wgap;
            pp_.pk_wxor = e_.wxor;
            pp_.L = d_.L;
            for (int l = 0; l < d_.L; ++l) {
                const int K = d_.dim[l], N = d_.dim[l + 1];
                pp_.img4_w[l] = d_.iw_off[l] / 4;
                pp_.img4_b[l] = d_.ib_off[l] / 4;
                pp_.img4_end[l] = (d_.ib_off[l] + ((N + 15) & ~15)) / 4;
                pp_.ldw4[l] = fl_ldw(K) / 4;
                pp_.k4[l] = ((K + 15) & ~15) / 4;
                pp_.pk_w[l] = e_.w_off[l] - e_.param_off;
                pp_.pk_lda[l] = e_.ldw[l];
                pp_.pk_b[l] = e_.bias_off[l] - e_.param_off;
            }
        }
    }
    bool has_peer() const { return peer_ != nullptr; }

    // Enable (ptr != 0) / disable in-kernel phase stamps: [blocks, 16] uint64 buffer.
    // (a configuration change like any other: cached graphs hold the old stamp buffer)
    void set_debug(uintptr_t ptr) {
        b_.dbg = as_ptr<unsigned long long>(ptr);
        drop_graph();
    }

    // Launch one kernel of round r on its live state (0 = train, 1 = adam, 2 = eval).
    void launch_one(int r, int which, uintptr_t stream) {
        hipStream_t s = as_stream(stream);
        float* pg = pbuf_[r & 1];
        float* cb = comm_buf(r);
        FLState* so = st_[(r + 1) & 1];
        if (which == 0) launch_train(pg, so, so, 1, s);
        else if (which == 1) launch_adam(b_.local, pg, cb, so, 1, s);
        else if (which == 3 && dtype_ == 1) launch_train(pg, so, so, 0, s, FL_EVAL_LAGGED, b_.cnt, 0);  // advances so
        else launch_eval(b_.local, cb, so, s);
    }

    // Per-kernel device time (us, averaged over `iters` back-to-back launches, hipEvents)
    // re-running the kernels of the last issued round `r` on its (live) state.  Training
    // launches use local_step=1 semantics so the round state is not advanced.
    py::dict time_kernels(int r, int iters, uintptr_t stream) {
        hipStream_t s = as_stream(stream);
        float* pg = pbuf_[r & 1];
        float* cb = comm_buf(r);
        FLState* so = st_[(r + 1) & 1];
        hipEvent_t e0, e1;
        HIP_CHECK(hipEventCreate(&e0));
        HIP_CHECK(hipEventCreate(&e1));
        py::dict out;
        auto timeit = [&](const char* name, auto&& launch) {
            launch();
            HIP_CHECK(hipEventRecord(e0, s));
            for (int i = 0; i < iters; ++i) launch();
            HIP_CHECK(hipEventRecord(e1, s));
            HIP_CHECK(hipEventSynchronize(e1));
            float ms = 0.f;
            HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
            out[name] = 1e3 * ms / iters;
        };
        const int ls = 1;
        timeit("train", [&] { launch_train(pg, so, so, ls, s); });
        timeit("adam", [&] { launch_adam(b_.local, pg, cb, so, ls, s); });
        timeit("eval", [&] { launch_eval(b_.local, cb, so, s); });
        HIP_CHECK(hipEventDestroy(e0));
        HIP_CHECK(hipEventDestroy(e1));
        return out;
    }

    // Per-kernel device time of the REAL round design (us per round, by kernel kind): rounds
    // [r0, r0 + n) are issued eagerly exactly as run() issues them, with a hipEvent after every
    // launch; a sleeping gate kernel holds the stream until the whole sequence is enqueued, so
    // the kernels run back to back (host launch pace does not leak into the intervals).  The
    // interval before a kernel's event is charged to that kernel: launch gaps on the device
    // are included (that is what a graph replay pays too, minus the graph's own launch cost).
    // With the Adam-fused peer exchange, waiting for slower ranks shows up under "adam".
    // `warm` untraced rounds run first behind the gate (they absorb the ranks' start skew: the
    // first in-kernel exchange waits for the last rank to arrive).
    py::dict trace(int r0, int n, uintptr_t stream, RcclComm* comm, bool close, double gate_us, int warm) {
        if (rec_ != nullptr) throw std::runtime_error("trace: not inside a trial batch");
        if (n < 1 || warm < 0) throw std::runtime_error("trace: n >= 1, warm >= 0");
        hipStream_t s = as_stream(stream);
        std::vector<std::pair<int, hipEvent_t>> ev;
        hipEvent_t e0;
        HIP_CHECK(hipEventCreateWithFlags(&e0, trace_event_flags()));
        HIP_CHECK(fl_launch_gate(gate_us, s));
        if (warm > 0) run(r0, warm, stream, comm, false);
        HIP_CHECK(hipEventRecord(e0, s));
        tev_ = &ev;
        try {
            run(r0 + warm, n, stream, comm, close);
        } catch (...) {
            tev_ = nullptr;
            throw;
        }
        tev_ = nullptr;
        HIP_CHECK(hipStreamSynchronize(s));
        static const char* names[TR_N] = {"pack", "train", "adam", "eval", "allreduce", "eval_fedavg"};
        double us[TR_N] = {0};
        int cnt[TR_N] = {0};
        hipEvent_t prev = e0;
        for (auto& [what, e] : ev) {
            float ms = 0.f;
            HIP_CHECK(hipEventElapsedTime(&ms, prev, e));
            us[what] += 1e3 * ms;
            ++cnt[what];
            prev = e;
        }
        float total = 0.f;
        HIP_CHECK(hipEventElapsedTime(&total, e0, prev));
        py::dict out, launches;
        for (int k = 0; k < TR_N; ++k)
            if (cnt[k]) {
                out[names[k]] = us[k] / n;
                launches[names[k]] = cnt[k];
            }
        out["round"] = 1e3 * total / n;
        out["launches"] = launches;
        out["rounds"] = n;
        for (auto& pe : ev) hipEventDestroy(pe.second);
        hipEventDestroy(e0);
        return out;
    }

    // held-out evaluation: confusion matrix of `params` on (X, y) accumulated into cm_out
    void confusion(uintptr_t X, uintptr_t y, int n_rows, uintptr_t params, uintptr_t cm_out, uintptr_t stream) {
        HIP_CHECK(fl_launch_confusion(d_, c_.R, as_ptr<const float>(X), as_ptr<const int>(y), n_rows,
                                      as_ptr<const float>(params), as_ptr<float>(cm_out), as_stream(stream)));
    }

    py::dict layout() const {
        py::dict o;
        std::vector<int> w, bb, iw, ib, ld, dims;
        for (int l = 0; l < d_.L; ++l) {
            w.push_back(d_.w_off[l]); bb.push_back(d_.b_off[l]);
            iw.push_back(d_.iw_off[l]); ib.push_back(d_.ib_off[l]);
        }
        for (int l = 0; l <= d_.L; ++l) { ld.push_back(d_.ld[l]); dims.push_back(d_.dim[l]); }
        o["P"] = d_.P;
        o["Pimg"] = d_.Pimg;
        o["w_off"] = w;
        o["b_off"] = bb;
        o["iw_off"] = iw;
        o["ib_off"] = ib;
        o["ld"] = ld;
        o["dims"] = dims;
        o["lds_bytes"] = dtype_ == 0 ? d_.lds_floats * 4 : e_.lds_bytes;
        o["bank_level"] = dtype_ == 0 ? -1 : e_.level;
        o["eval_lds_bytes"] = dtype_ == 0 ? d_.lds_floats * 4 : ev_.lds_bytes;
        o["lag_reg"] = dtype_ == 1 && e_.lag_reg != 0;  // lagged rounds score in registers (fl_layout.h)
        o["plain_fwd"] = c_.plain_fwd != 0;              // plain-bf16 training forward (several clients)
        o["split_score"] = c_.split_score != 0;          // lagged scoring on workgroups of its own
        o["eval_fedavg"] = peer_ != nullptr && !fused_ && eval_fedavg_fits();
        o["dtype"] = dtype_;
        o["slab_stride"] = c_.slab_stride;
        o["n_slabs"] = c_.n_slabs;
        o["slab_f16"] = c_.slab_f16;
        o["tail_off"] = c_.tail_off;
        o["tail_stride"] = c_.tail_stride;
        o["tail_len"] = c_.tail_len;
        o["comm_len"] = comm_len_;
        o["lagged_eval"] = lagged();
        o["state_bytes"] = (int)sizeof(FLState);
        return o;
    }

  private:
    void launch_train(const float* pg, const FLState* si, FLState* so, int ls, hipStream_t s,
                      int mode = FL_EVAL_CLASSIC, float* cm_out = nullptr, int fold_mask = FL_FOLD_B) {
        if (dtype_ == 0) {
            if (rec_ != nullptr)
                rec_->push_back({FLLaunchRec::TRAIN, {ls, 0, mode, fold_mask}, {pg, si, so, cm_out}});
            else
                HIP_CHECK(fl_launch_train(d_, c_, b_, pg, si, so, ls, s, mode, cm_out, fold_mask));
            mark(TR_TRAIN, s);
            // (the fp32 kernels read the fp32 image directly: nothing to repack, but the flag
            // also tells issue_train that the host replaced the weights -- consumed here, or
            // every fused round would flush a separate evaluation)
            need_pack_ = false;
        } else {
            // the round's input weights -> packed bf16 image.  With one client the FedAvg
            // output IS the local model (agg_scale = 1), which the Adam kernel already packed,
            // so the pack is needed only after host-side weight changes; later local steps
            // stage the Adam-packed local image too.
            const bool solo = c_.world == 1 && c_.agg_scale == 1.0f && !need_pack_;
            // the peer all-reduce already wrote the packed image of its output
            const bool packed = solo || (peer_ != nullptr && !need_pack_);
            if (rec_ != nullptr) {
                if (ls == 0 && !packed) rec_->push_back({FLLaunchRec::PACK, {0, 0, 0, 0}, {pg, b_.pk_global}});
                rec_->push_back({FLLaunchRec::TRAIN, {ls, solo ? 1 : 0, mode, fold_mask}, {pg, si, so, cm_out}});
                need_pack_ = false;
                return;
            }
            if (ls == 0 && !packed) {
                HIP_CHECK(fl_launch_pack_bf16(d_, e_, pg, b_.pk_global, s));
                mark(TR_PACK, s);
            }
            need_pack_ = false;
            HIP_CHECK(fl_launch_train_bf16(d_, e_, c_, b_, pg, si, so, ls, s, solo, mode, cm_out, fold_mask));
            mark(TR_TRAIN, s);
        }
    }
    void launch_adam(const float* pin, const float* anchor, float* comm, const FLState* st, int ls,
                     hipStream_t s, FLState* st_out = nullptr, int fold = 0, int tail_a = 0,
                     int fold_mask = FL_FOLD_B, const PeerArgs* peer = nullptr, int wx = 0, int afold = 0) {
        if (rec_ != nullptr) {
            if (peer != nullptr || wx || afold) throw std::runtime_error("trial batch: no in-kernel exchange");
            rec_->push_back({FLLaunchRec::ADAM, {ls, fold, tail_a, fold_mask}, {pin, anchor, comm, st, st_out}});
            return;
        }
        HIP_CHECK(fl_launch_adam(d_, c_, b_, pin, anchor, comm, st, ls, s, dtype_ == 1 ? &e_ : nullptr, st_out,
                                 fold, tail_a, fold_mask, peer, wx, afold));
        mark(TR_ADAM, s);
    }
    void launch_eval(const float* params, float* comm, const FLState* st, hipStream_t s) {
        ++eval_launches_;
        if (rec_ != nullptr) {
            rec_->push_back({FLLaunchRec::EVAL, {0, 0, 0, 0}, {params, comm, st}});
            return;
        }
        if (dtype_ == 0) HIP_CHECK(fl_launch_eval(d_, c_, b_, params, comm, st, s));
        else HIP_CHECK(fl_launch_eval_bf16(d_, ev_, c_, b_, params, comm, st, s));
        mark(TR_EVAL, s);
    }
    // Train/Adam pairs of round r.  Fused rounds (fl_common.h FL_EVAL_FUSED): the first train
    // kernel also scores the previous round's model from its own forward pass, and the first
    // Adam kernel folds those counts and makes the round's live / stop decision.
    // Lagged rounds (FL_EVAL_LAGGED): the train kernel scores the previous round's local model
    // iff that round had no evaluation of its own; its fold consumes region A when the previous
    // round scored ITS predecessor and region B when the previous round was evaluated.
    // `xchg`: this round's FedAvg runs inside its Adam kernel (peer_device.h chunk exchange).
    void issue_train(int r, hipStream_t s, bool fused, bool xchg = false) {
        float* pg = pbuf_[r & 1];
        float* cb = comm_buf(r);
        FLState* si = st_[r & 1];
        FLState* so = st_[(r + 1) & 1];
        if (fused && need_pack_) flush_pending_eval(r, s);  // host replaced the weights: score the old model
        // Every round's metric fold runs in its first Adam kernel (overlapped with the slab
        // loads; measured: folding at the start of the train kernel cost ~3 us per round), the
        // train kernel trains on the tentative live decision.
        const bool score = !fused && prev_lagged_;
        int mode = (fused && !cm_in_tail_) ? FL_EVAL_FUSED : FL_EVAL_FUSED_SKIP;
        if (score) mode = FL_EVAL_LAGGED;
        // metrics of the previous round: region B of its all-reduce (it evaluated itself), or
        // region A one round later (lagged, FedAvg outside Adam); with the Adam-fused exchange
        // a lagged predecessor is folded inside this Adam kernel from the exchanged region A
        const bool afold = score && xchg_;  // fold the lagged predecessor in this Adam kernel
        const int mask = fused ? FL_FOLD_B
                               : ((prev_scored_ && !prev_afold_ ? FL_FOLD_A : 0) | (prev_lagged_ ? 0 : FL_FOLD_B));
        float* cm_out = score ? b_.cnt : pg + c_.tail_off + c_.rank * c_.tail_stride;
        for (int ls = 0; ls < c_.local_steps; ++ls) {
            const bool first = ls == 0;
            launch_train(pg, first ? si : so, so, ls, s, first ? mode : FL_EVAL_CLASSIC, cm_out, mask);
            if (first && (xchg || afold)) {
                const PeerArgs pa = peer_->args((r + 1) & 1, pbuf_[(r + 1) & 1]);
                launch_adam(pg, pg, cb, si, ls, s, so, 1, score ? 1 : 0, mask, &pa, xchg ? 1 : 0, afold ? 1 : 0);
            } else if (first) {
                launch_adam(pg, pg, cb, si, ls, s, so, 1, score ? 1 : 0, mask);
            }
            else launch_adam(b_.local, pg, cb, so, ls, s);
        }
        pending_cm_ = fused;
        cm_in_tail_ = false;
        prev_scored_ = score;
        prev_afold_ = afold;
    }
    void issue_eval(int r, hipStream_t s) {
        launch_eval(b_.local, comm_buf(r), st_[(r + 1) & 1], s);
    }
    // A fused round r-1 left its metrics pending (they are normally scored by round r's
    // train kernel): score them with the eval kernel before anything that needs them.
    void flush_pending_eval(int r, hipStream_t s) {
        if (!pending_cm_) return;
        issue_eval(r - 1, s);
        pending_cm_ = false;
        cm_in_tail_ = true;
    }
    // Buffer round r publishes into (FedAvg contribution + metric tails): the peer
    // all-reduce's send buffer, or, for RCCL, the parameter buffer it reduces in place.
    float* comm_buf(int r) const { return peer_ != nullptr ? peer_->send((r + 1) & 1) : pbuf_[(r + 1) & 1]; }
    void issue_allreduce(int r, hipStream_t s, RcclComm* comm) {
        // (one client: FedAvg is the identity; an emulating engine still issues the collective,
        // e.g. a one-rank RCCL all-reduce, so the multi-client round shape runs on one GPU)
        if (c_.world < 2 && peer_ == nullptr && !(emulate_ && comm != nullptr)) return;
        if (peer_ != nullptr)
            HIP_CHECK(peer_->launch((r + 1) & 1, pbuf_[(r + 1) & 1], dtype_ == 1 ? &pp_ : nullptr, s));
        else if (comm != nullptr)
            comm->allreduce_f32((uintptr_t)pbuf_[(r + 1) & 1], (size_t)comm_len_, (uintptr_t)s);
        else
            return;
        mark(TR_ALLREDUCE, s);
    }
    // `lag`: a lagged round -- no evaluation; the next round's train kernel scores it.
    void issue_round(int r, hipStream_t s, RcclComm* comm, bool allow_fused, bool lag = false) {
        const bool fused = fused_ && allow_fused;
        lag = lag && lagged() && !fused;
        if (!fused) flush_pending_eval(r, s);
        const bool xchg = lag && xchg_;
        issue_train(r, s, fused, xchg);
        prev_lagged_ = lag;
        if (lag) {
            if (!xchg) issue_allreduce(r, s, comm);
            return;
        }
        if (!fused && peer_ != nullptr && eval_fedavg_fits()) {
            // evaluation and the one-shot all-reduce in one kernel (peer_device.h)
            issue_eval_fedavg(r, s);
            cm_in_tail_ = true;
            return;
        }
        if (!fused) {
            issue_eval(r, s);
            cm_in_tail_ = true;
        }
        issue_allreduce(r, s, comm);
    }
    // The fused evaluation + FedAvg grid (evaluation blocks + all-reduce blocks) must be
    // resident in one wave, which needs two evaluation workgroups per CU (measured: with one
    // per CU the extra blocks spill into a second wave and the fused kernel loses to the
    // separate kernels, tools/round_emulate.py).
    bool eval_fedavg_fits() const {
        const size_t lds = dtype_ == 0 ? (size_t)d_.lds_floats * 4 : (size_t)ev_.lds_bytes;
        return eval_fedavg_ && 2 * lds <= (size_t)160 * 1024;
    }
    void issue_eval_fedavg(int r, hipStream_t s) {
        if (rec_ != nullptr) throw std::runtime_error("trial batch: no peer all-reduce");
        const int p = (r + 1) & 1;
        const PeerArgs a = peer_->args(p, pbuf_[p], d_.Pimg);
        PeerPack pk;
        std::memset(&pk, 0, sizeof(pk));
        if (dtype_ == 1) pk = pp_;
        if (dtype_ == 0)
            HIP_CHECK(fl_launch_eval_fedavg(d_, c_, b_, b_.local, comm_buf(r), st_[(r + 1) & 1], a, pk, s));
        else
            HIP_CHECK(fl_launch_eval_fedavg_bf16(d_, ev_, c_, b_, b_.local, comm_buf(r), st_[(r + 1) & 1], a, pk, s));
        mark(TR_EVAL_FEDAVG, s);
    }

    struct GraphRec {
        int n;                 // rounds
        hipGraph_t g;
        hipGraphExec_t e;
        long long evals;       // evaluation kernels per replay
        RcclComm* comm;        // communicator the rounds were captured with
    };
    static constexpr int kMaxGraphs = 4;
    static void destroy_rec(GraphRec& r) {
        if (r.e) hipGraphExecDestroy(r.e);
        if (r.g) hipGraphDestroy(r.g);
        r.e = nullptr;
        r.g = nullptr;
    }
    void select_graph(int i) {
        graph_ = graphs_[i].g;
        exec_ = graphs_[i].e;
        graph_rounds_ = graphs_[i].n;
        graph_evals_ = graphs_[i].evals;
    }
    void drop_graph() {
        for (auto& r : graphs_) destroy_rec(r);
        graphs_.clear();
        exec_ = nullptr;
        graph_ = nullptr;
        graph_rounds_ = 0;
    }
    std::vector<GraphRec> graphs_;
    long long captures_ = 0;   // graphs captured + instantiated (not counting cache hits)

    MLPDesc d_;
    MLPDescB e_;
    MLPDescB ev_;  // evaluation-only layout of e_ (no delta buffers)
    int dtype_ = 0;  // 0 = fp32 MFMA, 1 = bf16 MFMA (fp32 accumulate / master weights)
    char* pk_ = nullptr;
    float* lagbuf_ = nullptr;  // FL_EVAL_LAGGED count + loss carry-over
    long long comm_len_ = 0;   // floats of a comm buffer: image + tails (+ lag region)
    bool lag_ok_ = false;      // lagged rounds possible (layout, clients, bf16): see lagged()
    bool emulate_ = false;     // one process stands in for a multi-client round (measurements, tests)
    bool xchg_ = false;        // lagged rounds: FedAvg inside the Adam kernel (no all-reduce kernel)
    bool prev_lagged_ = false; // the last issued round had no evaluation of its own
    bool prev_scored_ = false; // the last issued round's train kernel scored its predecessor
    bool prev_afold_ = false;  // ... and its Adam kernel folded that predecessor (exchanged in-kernel)
    bool need_pack_ = true;  // host changed the global weights: repack before the next round
    PeerAllReduce* peer_ = nullptr;  // one-shot xGMI all-reduce (nullptr: RCCL)
    float* undo_ = nullptr;          // FLBuffers::undo storage (lagged engines with early stopping)
    PeerPack pp_;                    // its bf16 pack epilogue (bf16 mode)
    bool eval_fedavg_ = true;  // world > 1 with peer: evaluation + all-reduce in one kernel
    bool fused_ = false;       // rounds evaluate the previous round inside the train kernel
    bool pending_cm_ = false;  // the last issued round was fused: its metrics are not scored yet
    bool cm_in_tail_ = false;  // the last round's counts sit in the tail, not yet folded
    FLConfig c_;
    FLBuffers b_;
    float* pbuf_[2];
    FLState* st_[2];
    hipGraph_t graph_ = nullptr;
    hipGraphExec_t exec_ = nullptr;
    int graph_rounds_ = 0;
    long long eval_launches_ = 0;  // see eval_launches()
    long long graph_evals_ = 0;    // evaluation kernels inside the captured graph
    std::vector<FLLaunchRec>* rec_ = nullptr;  // TrialBatch: record launches instead of issuing them
    // trace(): an event after every launch, tagged with what was launched
    enum { TR_PACK, TR_TRAIN, TR_ADAM, TR_EVAL, TR_ALLREDUCE, TR_EVAL_FEDAVG, TR_N };
    std::vector<std::pair<int, hipEvent_t>>* tev_ = nullptr;
    // trace markers without the system-scope release/acquire (device-side timing only needs the
    // marker's timestamp); FEDMI_TRACE_SYSFENCE=1 restores default events (A/B)
    static unsigned trace_event_flags() {
        const char* v = std::getenv("FEDMI_TRACE_SYSFENCE");
        return (v != nullptr && v[0] == '1') ? hipEventDefault : hipEventDisableSystemFence;
    }
    void mark(int what, hipStream_t s) {
        if (tev_ == nullptr) return;
        hipEvent_t e;
        HIP_CHECK(hipEventCreateWithFlags(&e, trace_event_flags()));
        tev_->emplace_back(what, e);
        HIP_CHECK(hipEventRecord(e, s));
    }
};

// ---------------------------------------------------------------------------------------
// Trial batch (fl_common.h FLTrialDesc): K engines of one shape run every kernel of a round as
// ONE launch with a trial grid dimension.  Each engine's round logic (state machine, modes,
// buffer parities) runs unchanged in recording mode; the recorded launches of the K engines
// are matched launch by launch and issued batched.  Engines are ordered by local steps,
// descending, so the trials taking part in a later local step are a prefix of the table.
// ---------------------------------------------------------------------------------------
class TrialBatch {
  public:
    explicit TrialBatch(std::vector<FLEngine*> engs) : engs_(std::move(engs)) {
        K_ = (int)engs_.size();
        if (K_ < 1) throw std::runtime_error("TrialBatch: no engines");
        const FLEngine& a = *engs_[0];
        for (int k = 0; k < K_; ++k) {
            const FLEngine& e = *engs_[k];
            if (e.peer_ != nullptr) throw std::runtime_error("TrialBatch: engines must not use the peer all-reduce");
            if (e.dtype_ != a.dtype_ || std::memcmp(&e.d_, &a.d_, sizeof(MLPDesc)) != 0 ||
                (a.dtype_ == 1 && (std::memcmp(&e.e_, &a.e_, sizeof(MLPDescB)) != 0 ||
                                   std::memcmp(&e.ev_, &a.ev_, sizeof(MLPDescB)) != 0)))
                throw std::runtime_error("TrialBatch: engines differ in shape or dtype");
            if (e.c_.R != a.c_.R || e.c_.n_rows != a.c_.n_rows || e.c_.world != a.c_.world ||
                e.c_.plain_fwd != a.c_.plain_fwd ||
                e.c_.rank != a.c_.rank || e.c_.slab_f16 != a.c_.slab_f16 || e.c_.lag_off != a.c_.lag_off ||
                e.fused_ != a.fused_ || e.lagged() != a.lagged() || e.emulate_ != a.emulate_)
                throw std::runtime_error("TrialBatch: engines differ in rows, clients or round kind");
            if (k > 0 && e.c_.local_steps > engs_[k - 1]->c_.local_steps)
                throw std::runtime_error("TrialBatch: order the engines by local steps, descending");
        }
        HIP_CHECK(hipMalloc(&dT_, sizeof(FLTrialDesc) * K_));
        upload(nullptr);
    }
    ~TrialBatch() {
        if (dT_) (void)hipFree(dT_);
    }
    int size() const { return K_; }

    // Rounds [r0, r0 + n) of every trial (FLEngine::run without a communicator).
    void run(int r0, int n, uintptr_t stream, bool close) {
        for (int r = r0; r < r0 + n; ++r) {
            const bool last = close && r == r0 + n - 1;
            issue([&](FLEngine* e) { e->run(r, 1, stream, nullptr, last); }, as_stream(stream));
        }
    }
    // Local part of round r of every trial (the caller reduces the trials' shared buffer).
    void run_local(int r, uintptr_t stream) {
        issue([&](FLEngine* e) { e->run_local(r, stream); }, as_stream(stream));
    }
    void finalize(int r, uintptr_t stream) {
        issue([&](FLEngine* e) { e->finalize(r, stream); }, as_stream(stream));
    }
    bool needs_eager_round() const {
        for (auto* e : engs_)
            if (e->needs_eager_round()) return true;
        return false;
    }

  private:
    void build_table(std::vector<FLTrialDesc>& T) const {
        T.assign(K_, FLTrialDesc{});
        for (int k = 0; k < K_; ++k) {
            const FLEngine& e = *engs_[k];
            T[k].c = e.c_;
            T[k].b = e.b_;
            char* const bases[FL_TB_BASES] = {(char*)e.pbuf_[0], (char*)e.pbuf_[1], (char*)e.st_[0], (char*)e.st_[1],
                                              (char*)e.b_.local, (char*)e.lagbuf_, e.b_.pk_global, e.b_.pk_local};
            std::memcpy(T[k].base, bases, sizeof(bases));
        }
    }
    // (re)upload the table when an engine's configuration changed (e.g. set_early_stop);
    // never inside a stream capture
    void upload(hipStream_t s) {
        std::vector<FLTrialDesc> T;
        build_table(T);
        if (!host_.empty() && std::memcmp(T.data(), host_.data(), sizeof(FLTrialDesc) * K_) == 0) return;
        if (s != nullptr) {
            hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
            HIP_CHECK(hipStreamIsCapturing(s, &cs));
            if (cs != hipStreamCaptureStatusNone)
                throw std::runtime_error("TrialBatch: a trial's configuration changed during a graph capture");
            HIP_CHECK(hipStreamSynchronize(s));  // kernels still reading the old table
        }
        HIP_CHECK(hipMemcpy(dT_, T.data(), sizeof(FLTrialDesc) * K_, hipMemcpyHostToDevice));
        host_ = std::move(T);
    }
    size_t base_bytes(const FLEngine& e, int i) const {
        switch (i) {
            case FL_TB_PBUF0: case FL_TB_PBUF1: return (size_t)e.comm_len_ * sizeof(float);
            case FL_TB_ST0: case FL_TB_ST1: return sizeof(FLState);
            case FL_TB_LOCAL: return (size_t)e.d_.Pimg * sizeof(float);
            case FL_TB_LAG: return (FL_MAX_CLASSES * FL_MAX_CLASSES + 4) * sizeof(float);
            default: return e.dtype_ == 1 ? (size_t)e.e_.param_bytes : 0;
        }
    }
    FLSel resolve(int k, const void* p) const {
        FLSel sel = {-1, 0, 0};
        if (p == nullptr) return sel;
        const char* q = static_cast<const char*>(p);
        for (int i = 0; i < FL_TB_BASES; ++i) {
            const char* b0 = host_[k].base[i];
            if (b0 != nullptr && q >= b0 && q < b0 + base_bytes(*engs_[k], i)) {
                sel.base = i;
                sel.off = (long long)(q - b0);
                return sel;
            }
        }
        throw std::runtime_error("TrialBatch: launch argument outside the trial's buffers");
    }
    static bool same_launch(const FLLaunchRec& a, const FLLaunchRec& b) {
        return a.kind == b.kind && std::memcmp(a.i, b.i, sizeof(a.i)) == 0;
    }

    // Record every engine's launches, match them into batched launches (all checks done before
    // anything is issued: on a mismatch the engines' round bookkeeping is rolled back and
    // nothing ran), then issue them.
    template <class F>
    void issue(F&& per_engine, hipStream_t s) {
        upload(s);
        std::vector<int> flags0(K_);
        for (int k = 0; k < K_; ++k) flags0[k] = engs_[k]->flags();
        auto rollback = [&]() {
            for (int k = 0; k < K_; ++k) {
                engs_[k]->rec_ = nullptr;
                engs_[k]->set_flags(flags0[k]);
            }
        };
        struct Planned {
            const FLLaunchRec* m;
            FLSel sel[5];
            int cnt;
        };
        std::vector<std::vector<FLLaunchRec>> recs(K_);
        std::vector<Planned> plan;
        try {
            for (int k = 0; k < K_; ++k) {
                engs_[k]->rec_ = &recs[k];
                per_engine(engs_[k]);
                engs_[k]->rec_ = nullptr;
            }
            std::vector<size_t> pos(K_, 0);
            for (const FLLaunchRec& m : recs[0]) {
                // trials whose next recorded launch is this one: a prefix of the table
                Planned pl;
                pl.m = &m;
                pl.cnt = 0;
                for (int k = 0; k < K_; ++k) {
                    const bool match = pos[k] < recs[k].size() && same_launch(recs[k][pos[k]], m);
                    if (match && k != pl.cnt) throw std::runtime_error("TrialBatch: launch sequences do not align");
                    if (match) ++pl.cnt;
                }
                for (int a = 0; a < 5; ++a) {
                    pl.sel[a] = resolve(0, m.p[a]);
                    for (int k = 1; k < pl.cnt; ++k) {
                        const FLSel o = resolve(k, recs[k][pos[k]].p[a]);
                        if (o.base != pl.sel[a].base || o.off != pl.sel[a].off)
                            throw std::runtime_error("TrialBatch: trials disagree on a launch argument");
                    }
                }
                for (int k = 0; k < pl.cnt; ++k) ++pos[k];
                plan.push_back(pl);
            }
            for (int k = 0; k < K_; ++k)
                if (pos[k] != recs[k].size()) throw std::runtime_error("TrialBatch: launch sequences do not align");
        } catch (...) {
            rollback();
            throw;
        }
        const FLEngine& e0 = *engs_[0];
        for (const Planned& pl : plan) launch(e0, *pl.m, pl.sel, pl.cnt, s);
    }
    void launch(const FLEngine& e, const FLLaunchRec& m, const FLSel* sel, int cnt, hipStream_t s) {
        const FLConfig& c = e.c_;
        switch (m.kind) {
            case FLLaunchRec::PACK:
                HIP_CHECK(fl_launch_pack_bf16_batch(e.d_, e.e_, dT_, cnt, sel[0], sel[1], s));
                break;
            case FLLaunchRec::TRAIN:
                if (e.dtype_ == 0)
                    HIP_CHECK(fl_launch_train_batch(e.d_, c.R, c.n_slabs, dT_, cnt, sel[0], sel[1], sel[2], m.i[0],
                                                    m.i[2], sel[3], m.i[3], s));
                else
                    HIP_CHECK(fl_launch_train_bf16_batch(e.d_, e.e_, c.R, c.n_slabs, dT_, cnt, sel[0], sel[1], sel[2],
                                                         m.i[0], m.i[1], m.i[2], sel[3], m.i[3], s, c.plain_fwd));
                break;
            case FLLaunchRec::ADAM:
                HIP_CHECK(fl_launch_adam_batch(e.d_, e.dtype_ == 1 ? &e.e_ : nullptr, dT_, cnt, sel[0], sel[1], sel[2],
                                               sel[3], m.i[0], sel[4], m.i[1], m.i[2], m.i[3], s));
                break;
            case FLLaunchRec::EVAL:
                if (e.dtype_ == 0)
                    HIP_CHECK(fl_launch_eval_batch(e.d_, c.R, c.n_rows, dT_, cnt, sel[0], sel[1], sel[2], s));
                else
                    HIP_CHECK(fl_launch_eval_bf16_batch(e.d_, e.ev_, c.R, c.n_rows, dT_, cnt, sel[0], sel[1], sel[2],
                                                        s));
                break;
            case FLLaunchRec::FINALIZE:
                HIP_CHECK(fl_launch_finalize_batch(e.d_, dT_, cnt, sel[0], sel[1], sel[2], m.i[0], s));
                break;
            default: throw std::runtime_error("TrialBatch: unknown launch");
        }
    }

    std::vector<FLEngine*> engs_;
    int K_ = 0;
    FLTrialDesc* dT_ = nullptr;
    std::vector<FLTrialDesc> host_;
};

// Thin wrappers used by tests and the synthetic-data path.
static void synth(uintptr_t X, uintptr_t y, long long n, int F, unsigned long long seed, unsigned long long off,
                  uintptr_t w1, uintptr_t w2, int H, uintptr_t stream, float label_noise) {
    HIP_CHECK(fl_launch_synth(as_ptr<float>(X), as_ptr<int>(y), n, F, seed, off, as_ptr<const float>(w1),
                              as_ptr<const float>(w2), H, as_stream(stream), label_noise));
}

#ifndef FEDMI_SRC_DIGEST
#define FEDMI_SRC_DIGEST "unknown"
#endif
// found by fedmi/ops/build.py:so_digest in the file bytes (no load needed)
__attribute__((used)) static const char kSrcDigestMarker[] = "FEDMI_SRC_DIGEST:" FEDMI_SRC_DIGEST;

static py::dict device_info(int dev) {
    hipDeviceProp_t p;
    HIP_CHECK(hipGetDeviceProperties(&p, dev));
    py::dict o;
    o["name"] = std::string(p.name);
    o["arch"] = std::string(p.gcnArchName);
    o["cus"] = p.multiProcessorCount;
    o["lds_per_block"] = (long long)p.sharedMemPerBlock;
    o["hbm_bytes"] = (long long)p.totalGlobalMem;
    return o;
}

PYBIND11_MODULE(_fedmi_hip, m) {
    m.doc() = "fedmi native runtime: fused FL round kernels (gfx950), HIP graphs, RCCL";
    py::class_<RcclComm>(m, "RcclComm")
        .def(py::init<int, int, py::bytes, int, double>(), py::arg("nranks"), py::arg("rank"), py::arg("uid"),
             py::arg("device"), py::arg("timeout_s") = 120.0)
        .def_static("unique_id", &RcclComm::unique_id)
        .def("async_error", &RcclComm::async_error)
        .def("allreduce_f32", &RcclComm::allreduce_f32)
        .def("allreduce_f64", &RcclComm::allreduce_f64)
        .def("allreduce_bf16", &RcclComm::allreduce_bf16)
        .def("allgather_f32", &RcclComm::allgather_f32)
        .def("broadcast_bytes", &RcclComm::broadcast_bytes)
        .def("abort", &RcclComm::abort)
        .def("destroy", &RcclComm::destroy)
        .def_property_readonly("rank", &RcclComm::rank)
        .def_property_readonly("size", &RcclComm::size);
    py::class_<FLEngine>(m, "FLEngine")
        .def(py::init<std::vector<int>, py::dict, py::dict>())
        .def("run", &FLEngine::run, py::arg("r0"), py::arg("n"), py::arg("stream"), py::arg("comm") = nullptr,
             py::arg("close") = true)
        .def("run_local", &FLEngine::run_local)
        .def("phase", &FLEngine::phase, py::arg("r"), py::arg("which"), py::arg("stream"), py::arg("comm") = nullptr)
        .def("finalize", &FLEngine::finalize)
        .def("capture", &FLEngine::capture, py::arg("n"), py::arg("stream"), py::arg("comm") = nullptr)
        .def("replay", &FLEngine::replay)
        .def("flags", &FLEngine::flags)
        .def("set_flags", &FLEngine::set_flags)
        .def("graph_rounds", &FLEngine::graph_rounds)
        .def_property_readonly("graph_captures", &FLEngine::graph_captures)
        .def_property_readonly("eval_launches", &FLEngine::eval_launches)
        .def("time_kernels", &FLEngine::time_kernels)
        .def("trace", &FLEngine::trace, py::arg("r0"), py::arg("n"), py::arg("stream"), py::arg("comm") = nullptr,
             py::arg("close") = true, py::arg("gate_us") = 5000.0, py::arg("warm") = 0)
        .def("set_debug", &FLEngine::set_debug)
        .def("invalidate", &FLEngine::invalidate)
        .def("set_early_stop", &FLEngine::set_early_stop)
        .def("reset_pending", &FLEngine::reset_pending)
        .def("attach_peer", &FLEngine::attach_peer, py::keep_alive<1, 2>())
        .def_property_readonly("has_peer", &FLEngine::has_peer)
        .def("needs_eager_round", &FLEngine::needs_eager_round)
        .def_property_readonly("fused", &FLEngine::fused)
        .def_property_readonly("lagged", &FLEngine::lagged)
        .def_property_readonly("adam_exchange", &FLEngine::adam_exchange)
        .def_property_readonly("late_fold", &FLEngine::late_fold)
        .def("launch_one", &FLEngine::launch_one)
        .def("confusion", &FLEngine::confusion)
        .def("layout", &FLEngine::layout);
    py::class_<TrialBatch>(m, "TrialBatch")
        .def(py::init<std::vector<FLEngine*>>(), py::keep_alive<1, 2>())
        .def("run", &TrialBatch::run, py::arg("r0"), py::arg("n"), py::arg("stream"), py::arg("close") = true)
        .def("run_local", &TrialBatch::run_local)
        .def("finalize", &TrialBatch::finalize)
        .def("needs_eager_round", &TrialBatch::needs_eager_round)
        .def_property_readonly("size", &TrialBatch::size);
    m.def("synth", &synth, py::arg("X"), py::arg("y"), py::arg("n"), py::arg("F"), py::arg("seed"), py::arg("off"),
          py::arg("w1"), py::arg("w2"), py::arg("H"), py::arg("stream"), py::arg("label_noise") = 0.f);
    m.def("device_info", &device_info);
    m.attr("STATE_BYTES") = (int)sizeof(FLState);
    m.attr("SRC_DIGEST") = std::string(kSrcDigestMarker + sizeof("FEDMI_SRC_DIGEST:") - 1);
    register_trainer(m);
    register_peer(m);
}
