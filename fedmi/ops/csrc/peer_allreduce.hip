// One-shot all-reduce over xGMI peer memory, for the latency-bound FedAvg message of the fused
// round engine.
//
// The reference aggregates with gather -> numpy average on rank 0 -> bcast of pickled weights
// (FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py:101-120).  The fused engine reduces
// [parameter image * n_i/N | per-rank metric tails] every round: ~50 KB for the reference MLP,
// a purely latency-bound message.  A ring all-reduce over 8 GPUs is 2 x 7 dependent steps; an
// MI355X node has a direct xGMI link between every pair of its 8 GPUs, so one step suffices:
//
//   * every rank exports one allocation -- two send buffers (round parity) and a 256-byte
//     control block -- through a HIP IPC handle and maps every peer's allocation once;
//   * the all-reduce is ONE kernel: block 0 publishes "my send buffer for call s is complete"
//     with one system-scope store into each peer's control block; every block waits (one
//     polling lane per peer) until all ranks published s, then pulls its slice of all send
//     buffers over the 7 links at once with system-coherent 16-byte loads, sums them in rank
//     order (so every rank gets bit-identical weights) and writes the result; in bf16 mode it
//     also writes the packed bf16 LDS image the next round's train kernel stages, which
//     removes the pack kernel from the round;
//   * the data a rank publishes were written by earlier kernels on its stream; their kernel
//     boundary wrote the L2s back, so the flag store may follow them directly;
//   * send buffers alternate by round parity and flags are monotonic call counters, so no
//     second barrier is needed: a rank rewrites buffer p (call s + 2) only after every peer
//     entered call s + 1, i.e. finished reading call s;
//   * every wait is bounded (s_memrealtime): on a timeout the kernel writes a sticky failure
//     word into EVERY rank's control block instead of hanging the GPU, so every later wait of
//     every rank ends at once and the job drains in one timeout; the host checks the word after
//     every chunk of rounds and aborts (fedmi/parallel/peer.py check_peer_error).  A host abort
//     word in pinned memory lets Comm.Abort / a watchdog release this rank's spinning kernels.
//
// The same allocation carries a chunk-flag table and an LL ring for the round engine's
// Adam-fused exchange (peer_device.h): there the call index comes from the device round state;
// every Adam block PUSHES its 64 parameters' contributions, each with the call index in one
// 8-byte store, into every rank's ring and polls its own ring (the metric chunks use the
// chunk flags: publish / wait / pull).  Start-up self-tests all three protocols on a known
// payload (fedmi/parallel/peer.py) before the engine may use them.
#include "peer_allreduce.h"

#include <pybind11/stl.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <thread>
#include <cstring>
#include <stdexcept>
#include <stdint.h>

namespace py = pybind11;

#define PEER_THREADS 256
#define PEER_MAX_BLOCKS 64

static void phip(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e) + " at " + what);
}
#define PHIP(expr) phip((expr), #expr)

// Standalone call: both parts were written by earlier kernels on this stream, so both flags
// are published at once; then every block pulls its share of all send buffers.
__global__ void __launch_bounds__(PEER_THREADS) peer_allreduce_kernel(PeerArgs a, PeerPack pk) {
    const unsigned target = peer_target(a);
    if (blockIdx.x == 0) {
        peer_publish(a.flag_dst, a.world, target, a.uc);
        peer_publish(a.tflag_dst, a.world, target, a.uc);
    }
    peer_wait(a, a.ctl->flags, target);
    peer_reduce4<PEER_MAX_WORLD>(a, pk, 0, a.n >> 2, blockIdx.x, gridDim.x);
    if (blockIdx.x == 0) peer_reduce1(a, a.n & ~3ll, a.n);
    peer_finish(a, target, gridDim.x);
}

// Self-test of the Adam-fused chunk exchange (peer_device.h): block c exchanges chunk c
// (floats [64c, 64c + 64)) of the send buffers with call index `target`.
__global__ void __launch_bounds__(64) peer_chunk_test_kernel(PeerArgs a, unsigned target, float* out) {
    const int c = blockIdx.x;
    peer_chunk_exchange_wait(a, c, target);
    const int pos = c * 64 + (int)threadIdx.x;
    if (pos < a.n) out[pos] = peer_pull_sum(a, pos);
}

// Self-test of the LL chunk exchange (peer_device.h): block c pushes floats [64c, 64c + 64) of
// this rank's send buffer with call index `target` and sums every rank's values.
__global__ void __launch_bounds__(64) peer_ll_test_kernel(PeerArgs a, unsigned target, float* out) {
    const int pos = blockIdx.x * 64 + (int)threadIdx.x;
    const bool valid = pos < a.n;
    peer_ll_push(a, pos, target, valid ? a.src[a.rank][pos] : 0.f);
    const float v = peer_ll_sum(a, pos, target, valid);
    if (valid) out[pos] = v;
}

// Self-test of the RS+AG chunk exchange (peer_device.h peer_rsag): block c reduces chunk c
// (owner c % world) of this rank's send buffer with call index `target`.
__global__ void __launch_bounds__(64) peer_rsag_test_kernel(PeerArgs a, unsigned target, float* out) {
    const int pos = blockIdx.x * 64 + (int)threadIdx.x;
    const bool valid = pos < a.n;
    const float v = peer_rsag(a, blockIdx.x, pos, target, valid, valid ? a.src[a.rank][pos] : 0.f);
    if (valid) out[pos] = v;
}

// Self-test payload: exact in fp32 for any summation order (multiples of 1/4 in [-256, 256)).
__global__ void peer_fill_kernel(float* dst, long long n, int rank, unsigned salt) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned h = (unsigned)i * 2654435761u + (unsigned)rank * 40503u + salt * 97u;
    dst[i] = (float)(h % 2048u) * 0.25f - 256.f;
}

PeerAllReduce::PeerAllReduce(int world, int rank, int device, long long n, double timeout_s, int n_chunks)
    : world_(world), rank_(rank), device_(device), n_(n), n_chunks_(n_chunks < 0 ? 0 : n_chunks) {
    if (world < 1 || world > PEER_MAX_WORLD) throw std::runtime_error("PeerAllReduce: world must be 1..8");
    if (rank < 0 || rank >= world) throw std::runtime_error("PeerAllReduce: bad rank");
    if (n <= 0 || n * 4 > (1ll << 30)) throw std::runtime_error("PeerAllReduce: 1..2^28 floats");
    PHIP(hipSetDevice(device));
    buf_bytes_ = ((size_t)n * 4 + 255) & ~(size_t)255;
    // [send 0 | send 1 | control block | chunk flags: PEER_MAX_WORLD x n_chunks | LL ring:
    //  2 x PEER_MAX_WORLD x n_chunks x 64 slots of 8 bytes]
    cf_off_ = 2 * buf_bytes_ + sizeof(PeerCtl);
    ll_off_ = cf_off_ + (((size_t)PEER_MAX_WORLD * n_chunks_ * 4 + 255) & ~(size_t)255);
    ll_bytes_ = (size_t)2 * PEER_MAX_WORLD * n_chunks_ * 64 * 8;
    total_ = ll_off_ + ll_bytes_;
    // FEDMI_PEER_LL=0: weight chunks through publish / wait / pull instead (A/B)
    const char* ll_env = std::getenv("FEDMI_PEER_LL");
    use_ll_ = n_chunks_ > 0 && !(ll_env != nullptr && std::strcmp(ll_env, "0") == 0);
    // FEDMI_PEER_RSAG=1: LL weight chunks by reduce-scatter + all-gather (peer_device.h peer_rsag)
    const char* rsag_env = std::getenv("FEDMI_PEER_RSAG");
    use_rsag_ = use_ll_ && rsag_env != nullptr && std::strcmp(rsag_env, "1") == 0;
    // FEDMI_ADAM_GRID=G: the LL Adam kernel on G workgroups (ranks sharing one GPU; PeerArgs)
    const char* ag_env = std::getenv("FEDMI_ADAM_GRID");
    if (ag_env != nullptr && *ag_env) adam_grid_ = std::max(0, std::atoi(ag_env));
    // Uncached device memory (MTYPE UC, what RCCL uses for its xGMI buffers): peers write the
    // flags and read the send buffers over xGMI, and no L2 -- this GPU's or a peer's -- may
    // hold a stale copy of either.  The send buffers are written once per round (~50 KB),
    // so bypassing the L2 costs nothing measurable.
    uncached_ = true;
    if (hipExtMallocWithFlags(reinterpret_cast<void**>(&base_), total_, hipDeviceMallocUncached) != hipSuccess) {
        (void)hipGetLastError();
        base_ = nullptr;
        uncached_ = false;  // cacheable fallback: flag publishes become system-scope releases
        PHIP(hipMalloc(reinterpret_cast<void**>(&base_), total_));
    }
    PHIP(hipMemset(base_, 0, total_));
    PHIP(hipHostMalloc(reinterpret_cast<void**>(&host_abort_), 2 * sizeof(unsigned),
                       hipHostMallocMapped | hipHostMallocCoherent));
    host_abort_[0] = 0u;
    host_abort_[1] = 0u;
    abort_word_ = host_abort_ + 1;
    PHIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&host_abort_dev_), host_abort_, 0));
    PHIP(hipDeviceSynchronize());
    set_timeout(timeout_s);
}

PeerAllReduce::~PeerAllReduce() {
    try {
        close();
    } catch (...) {
    }
}

void PeerAllReduce::close() {
    for (char* p : mapped_) (void)hipIpcCloseMemHandle(p);
    mapped_.clear();
    open_ = false;
    if (eflags_) {
        (void)hipFree(eflags_);
        eflags_ = nullptr;
        n_eval_ = 0;
    }
    if (base_) {
        (void)hipFree(base_);
        base_ = nullptr;
    }
    if (host_abort_) {
        (void)hipHostFree(host_abort_);
        host_abort_ = host_abort_dev_ = abort_word_ = nullptr;
    }
}

bool PeerAllReduce::abort(double wait_s) {
    if (host_abort_ == nullptr || base_ == nullptr) return false;
    const unsigned word = (PEER_ERR_ABORT << 16) | ((unsigned)rank_ << 8) | PEER_MISSING_NONE;
    // 1. this rank's kernels: they poll the pinned word (no GPU operation needed, cannot block)
    __atomic_store_n(&host_abort_[0], 1u, __ATOMIC_SEQ_CST);
    *abort_word_ = word;
    if (!open_) return false;
    // 2. every rank's failure word, copied from pinned memory on a private stream (best effort,
    //    bounded: the caller is tearing the process down)
    if (hipSetDevice(device_) != hipSuccess) return false;
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return false;
    for (int j = 0; j < world_; ++j) {
        unsigned* dst = &reinterpret_cast<PeerCtl*>(peer_base_[j] + 2 * buf_bytes_)->err;
        (void)hipMemcpyAsync(dst, abort_word_, sizeof(unsigned), hipMemcpyHostToDevice, s);
    }
    const auto t_end = std::chrono::steady_clock::now() + std::chrono::microseconds((long long)(wait_s * 1e6));
    bool done = false;
    for (;;) {
        const hipError_t q = hipStreamQuery(s);
        if (q == hipSuccess) {
            done = true;
            break;
        }
        if (q != hipErrorNotReady || std::chrono::steady_clock::now() >= t_end) break;
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    (void)hipGetLastError();
    // (a stream still busy is leaked on purpose: destroying it would wait for the copies)
    if (done) (void)hipStreamDestroy(s);
    return done;
}

py::bytes PeerAllReduce::handle() const {
    hipIpcMemHandle_t h;
    PHIP(hipIpcGetMemHandle(&h, base_));
    return py::bytes(reinterpret_cast<const char*>(&h), sizeof(h));
}

void PeerAllReduce::open(const std::vector<py::bytes>& handles) {
    if (open_) throw std::runtime_error("PeerAllReduce: already open");
    if ((int)handles.size() != world_) throw std::runtime_error("PeerAllReduce: need one handle per rank");
    PHIP(hipSetDevice(device_));
    // Peer mappings of every other visible GPU (one process per GPU sees the whole node): the
    // kernels read the peers' send buffers and write their flags directly over xGMI.  The IPC
    // open below enables access lazily for the handle's device; enabling it up front for all
    // peers makes the mapping independent of how the handle's device is resolved.
    int n_dev = 0;
    PHIP(hipGetDeviceCount(&n_dev));
    for (int d = 0; d < n_dev; ++d) {
        int can = 0;
        if (d == device_ || hipDeviceCanAccessPeer(&can, device_, d) != hipSuccess || !can) continue;
        const hipError_t e = hipDeviceEnablePeerAccess(d, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
            throw std::runtime_error(std::string("PeerAllReduce: peer access to device ") + std::to_string(d) +
                                     ": " + hipGetErrorString(e));
        (void)hipGetLastError();
    }
    for (int j = 0; j < world_; ++j) {
        if (j == rank_) {
            peer_base_[j] = base_;
            continue;
        }
        const std::string s = handles[j];
        if (s.size() != sizeof(hipIpcMemHandle_t)) throw std::runtime_error("PeerAllReduce: bad IPC handle");
        hipIpcMemHandle_t h;
        std::memcpy(&h, s.data(), sizeof(h));
        void* p = nullptr;
        PHIP(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
        peer_base_[j] = static_cast<char*>(p);
        mapped_.push_back(static_cast<char*>(p));
    }
    open_ = true;
}

float* PeerAllReduce::send(int parity) const { return reinterpret_cast<float*>(base_ + (parity & 1) * buf_bytes_); }

void PeerAllReduce::prepare_eval(int n_eval) {
    if (n_eval == n_eval_) return;
    PHIP(hipSetDevice(device_));
    if (eflags_ != nullptr) (void)hipFree(eflags_);
    eflags_ = nullptr;
    n_eval_ = 0;
    const size_t bytes = (size_t)std::max(n_eval, 1) * sizeof(unsigned);
    if (hipExtMallocWithFlags(reinterpret_cast<void**>(&eflags_), bytes, hipDeviceMallocUncached) != hipSuccess) {
        (void)hipGetLastError();
        eflags_ = nullptr;
        PHIP(hipMalloc(reinterpret_cast<void**>(&eflags_), bytes));
    }
    // call indices are monotonic and start at 1: 0 = "no call finished yet"
    PHIP(hipMemset(eflags_, 0, bytes));
    PHIP(hipDeviceSynchronize());
    n_eval_ = n_eval;
}

void PeerAllReduce::clear() {
    PHIP(hipSetDevice(device_));
    PHIP(hipMemset(base_, 0, 2 * buf_bytes_));
    // chunk flags restart at 0: the engine's call index starts at 1 (self-test calls used it)
    // (and the LL ring's call indices: every slot reads "no call yet")
    if (n_chunks_ > 0) PHIP(hipMemset(base_ + cf_off_, 0, total_ - cf_off_));
    PHIP(hipDeviceSynchronize());
}

void PeerAllReduce::set_timeout(double seconds) { timeout_ticks_ = (long long)(seconds * 1e8); }

int PeerAllReduce::error() const {
    unsigned e = 0;
    PHIP(hipMemcpy(&e, &reinterpret_cast<PeerCtl*>(base_ + 2 * buf_bytes_)->err, sizeof(e), hipMemcpyDeviceToHost));
    return (int)e;
}

PeerArgs PeerAllReduce::args(int parity, float* out, long long n_w) const {
    PeerArgs a;
    std::memset(&a, 0, sizeof(a));
    for (int j = 0; j < world_; ++j) {
        a.src[j] = reinterpret_cast<const float*>(peer_base_[j] + (parity & 1) * buf_bytes_);
        PeerCtl* cj = reinterpret_cast<PeerCtl*>(peer_base_[j] + 2 * buf_bytes_);
        a.flag_dst[j] = &cj->flags[rank_];
        a.tflag_dst[j] = &cj->tflags[rank_];
    }
    a.ctl = reinterpret_cast<PeerCtl*>(base_ + 2 * buf_bytes_);
    a.out = out;
    a.n = n_;
    a.n_w = n_w < 0 ? (n_ & ~3ll) : n_w;
    a.timeout = timeout_ticks_;
    a.eflags = eflags_;
    a.n_eval = n_eval_;
    a.world = world_;
    a.uc = uncached_ ? 1 : 0;
    a.n_chunks = n_chunks_;
    if (n_chunks_ > 0) {
        for (int j = 0; j < world_; ++j)
            a.cflag_dst[j] = reinterpret_cast<unsigned*>(peer_base_[j] + 2 * buf_bytes_ + sizeof(PeerCtl)) +
                             (size_t)rank_ * n_chunks_;
        a.cflags = reinterpret_cast<unsigned*>(base_ + 2 * buf_bytes_ + sizeof(PeerCtl));
        if (use_ll_) {
            for (int j = 0; j < world_; ++j) a.ll_dst[j] = reinterpret_cast<unsigned long long*>(peer_base_[j] + ll_off_);
            a.ll = reinterpret_cast<unsigned long long*>(base_ + ll_off_);
        }
    }
    a.rank = rank_;
    a.adam_grid = adam_grid_;
    if (open_)
        for (int j = 0; j < world_; ++j) a.err_dst[j] = &reinterpret_cast<PeerCtl*>(peer_base_[j] + 2 * buf_bytes_)->err;
    a.host_abort = host_abort_dev_;
    a.rsag = use_rsag_ ? 1 : 0;
    return a;
}

hipError_t PeerAllReduce::launch(int parity, float* out, const PeerPack* pack, hipStream_t s) const {
    if (!open_) return hipErrorNotInitialized;
    const PeerArgs a = args(parity, out);
    PeerPack p;
    std::memset(&p, 0, sizeof(p));
    if (pack != nullptr) p = *pack;
    const long long n4 = n_ / 4;
    const int blocks = (int)std::min<long long>(PEER_MAX_BLOCKS, std::max<long long>(1, (n4 + PEER_THREADS - 1) / PEER_THREADS));
    hipLaunchKernelGGL(peer_allreduce_kernel, dim3(blocks), dim3(PEER_THREADS), 0, s, a, p);
    return hipGetLastError();
}

void register_peer(py::module_& m) {
    py::class_<PeerAllReduce>(m, "PeerAllReduce")
        .def(py::init<int, int, int, long long, double, int>(), py::arg("world"), py::arg("rank"), py::arg("device"),
             py::arg("n_floats"), py::arg("timeout_s") = 60.0, py::arg("n_chunks") = 0)
        .def_property_readonly("n_chunks", &PeerAllReduce::n_chunks)
        .def("handle", &PeerAllReduce::handle)
        .def("open", &PeerAllReduce::open)
        .def("send_ptr", [](const PeerAllReduce& p, int parity) { return reinterpret_cast<uintptr_t>(p.send(parity)); })
        .def("allreduce",
             [](const PeerAllReduce& p, int parity, uintptr_t out, uintptr_t stream) {
                 PHIP(p.launch(parity, reinterpret_cast<float*>(out), nullptr, reinterpret_cast<hipStream_t>(stream)));
             })
        .def("chunk_test",
             [](const PeerAllReduce& p, int parity, unsigned target, uintptr_t out, uintptr_t stream) {
                 if (p.n_chunks() <= 0) throw std::runtime_error("chunk_test: no chunk-flag table");
                 const PeerArgs a = p.args(parity, reinterpret_cast<float*>(out));
                 hipLaunchKernelGGL(peer_chunk_test_kernel, dim3(p.n_chunks()), dim3(64), 0,
                                    reinterpret_cast<hipStream_t>(stream), a, target, reinterpret_cast<float*>(out));
                 PHIP(hipGetLastError());
             })
        .def("ll_test",
             [](const PeerAllReduce& p, unsigned target, uintptr_t out, uintptr_t stream) {
                 if (!p.uses_ll()) throw std::runtime_error("ll_test: no LL ring");
                 const PeerArgs a = p.args((int)(target & 1), reinterpret_cast<float*>(out));
                 const int blocks = (int)std::min<long long>(p.n_chunks(), (p.n_floats() + 63) / 64);
                 hipLaunchKernelGGL(peer_ll_test_kernel, dim3(blocks), dim3(64), 0,
                                    reinterpret_cast<hipStream_t>(stream), a, target, reinterpret_cast<float*>(out));
                 PHIP(hipGetLastError());
             })
        .def("rsag_test",
             [](const PeerAllReduce& p, unsigned target, uintptr_t out, uintptr_t stream) {
                 if (!p.uses_ll()) throw std::runtime_error("rsag_test: no LL ring");
                 const PeerArgs a = p.args((int)(target & 1), reinterpret_cast<float*>(out));
                 const int blocks = (int)std::min<long long>(p.n_chunks(), (p.n_floats() + 63) / 64);
                 hipLaunchKernelGGL(peer_rsag_test_kernel, dim3(blocks), dim3(64), 0,
                                    reinterpret_cast<hipStream_t>(stream), a, target, reinterpret_cast<float*>(out));
                 PHIP(hipGetLastError());
             })
        .def_property_readonly("uses_ll", &PeerAllReduce::uses_ll)
        .def_property_readonly("uses_rsag", &PeerAllReduce::uses_rsag)
        .def_property("adam_grid", &PeerAllReduce::adam_grid, &PeerAllReduce::set_adam_grid)
        .def("fill_test",
             [](const PeerAllReduce& p, int parity, unsigned salt, uintptr_t stream) {
                 const long long n = p.n_floats();
                 hipLaunchKernelGGL(peer_fill_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                                    reinterpret_cast<hipStream_t>(stream), p.send(parity), n, p.rank(), salt);
                 PHIP(hipGetLastError());
             })
        .def("read",
             [](const PeerAllReduce& p, int parity, long long off, long long n) {
                 if (off < 0 || n < 0 || off + n > p.n_floats()) throw std::runtime_error("read: out of range");
                 std::vector<float> v((size_t)n);
                 if (n) PHIP(hipMemcpy(v.data(), p.send(parity) + off, n * sizeof(float), hipMemcpyDeviceToHost));
                 return v;
             })
        .def("clear", &PeerAllReduce::clear)
        .def("set_timeout", &PeerAllReduce::set_timeout)
        .def_property_readonly("timeout_s", [](const PeerAllReduce& p) { return p.timeout_s(); })
        .def("error", &PeerAllReduce::error)
        .def("abort", &PeerAllReduce::abort, py::arg("wait_s") = 1.0, py::call_guard<py::gil_scoped_release>())
        .def("close", &PeerAllReduce::close)
        .def_property_readonly("world", &PeerAllReduce::world)
        .def_property_readonly("rank", &PeerAllReduce::rank)
        .def_property_readonly("n_floats", &PeerAllReduce::n_floats)
        .def_property_readonly("is_open", &PeerAllReduce::is_open)
        .def_property_readonly("uncached", &PeerAllReduce::uncached);
}
