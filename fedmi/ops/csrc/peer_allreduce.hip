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
//   * every wait is bounded (s_memrealtime): on a timeout the kernel sets a sticky error word
//     instead of hanging the GPU, and the host checks it at each synchronisation point.
#include "peer_allreduce.h"

#include <pybind11/stl.h>

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <stdint.h>

namespace py = pybind11;

#define PEER_THREADS 256
#define PEER_MAX_BLOCKS 64

struct PeerCtl {
    unsigned flags[PEER_MAX_WORLD];  // flags[j]: last call rank j has published to this rank
    unsigned seq;                    // calls this rank has completed
    unsigned done;                   // blocks of the running call that have finished
    unsigned err;                    // sticky: a wait timed out
    unsigned pad[64 - PEER_MAX_WORLD - 3];
};
static_assert(sizeof(PeerCtl) == 256, "PeerCtl is one 256-byte block");

struct PeerArgs {
    const float* src[PEER_MAX_WORLD];  // every rank's send buffer of this parity (mapped)
    unsigned* flag_dst[PEER_MAX_WORLD];  // &ctl_j->flags[rank]
    PeerCtl* ctl;                      // this rank's control block
    float* out;
    long long n;                       // floats
    long long timeout;                 // s_memrealtime ticks
};

static void phip(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e) + " at " + what);
}
#define PHIP(expr) phip((expr), #expr)

__device__ __forceinline__ uint32_t bf16_rne(float x) {
    const uint32_t u = __float_as_uint(x);
    return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}

// System-coherent (sc0 sc1: aux 17) buffer loads: they bypass this GPU's L1 and L2, so a
// peer's buffer is read from its memory as published, with no stale local copy.
__device__ __forceinline__ float4 load_sys16(const float* base, int bytes, int off) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, bytes,
                                                                         0x00020000);
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 17);
    return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
}
__device__ __forceinline__ float load_sys4(const float* base, int bytes, int off) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, bytes,
                                                                         0x00020000);
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 17));
}

// Image float4 i (fp32 parameter image) -> packed bf16 LDS image (PeerPack).
__device__ __forceinline__ void pack_store(const PeerPack& p, int i, float4 s) {
#pragma unroll
    for (int l = 0; l < FL_MAX_LAYERS; ++l) {
        if (l >= p.L || i < p.img4_w[l] || i >= p.img4_end[l]) continue;
        if (i < p.img4_b[l]) {
            const int q = i - p.img4_w[l];
            const int n = q / p.ldw4[l], c4 = q - n * p.ldw4[l];
            if (c4 < p.k4[l])  // columns [roundup16(K), ldw) are the image's zero pad
                *reinterpret_cast<uint2*>(p.pk + p.pk_w[l] + (n * p.pk_lda[l] + 4 * c4) * 2) =
                    make_uint2(bf16_rne(s.x) | (bf16_rne(s.y) << 16), bf16_rne(s.z) | (bf16_rne(s.w) << 16));
        } else {
            *reinterpret_cast<float4*>(p.pk + p.pk_b[l] + (i - p.img4_b[l]) * 16) = s;
        }
    }
}

template <int W>
__global__ void __launch_bounds__(PEER_THREADS) peer_allreduce_kernel(PeerArgs a, PeerPack pk) {
    __shared__ unsigned target_s;
    const int tid = threadIdx.x;
    if (tid == 0) target_s = __hip_atomic_load(&a.ctl->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    __syncthreads();
    const unsigned target = target_s;
    // publish this rank's send buffer for call `target` to every rank (itself included)
    if (blockIdx.x == 0 && tid < W)
        __hip_atomic_store(a.flag_dst[tid], target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    // wait until every rank has published call `target`: one polling lane per rank, bounded
    if (tid < W) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while ((int)(__hip_atomic_load(&a.ctl->flags[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - target) < 0) {
            if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > a.timeout) {
                __hip_atomic_store(&a.ctl->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
    __syncthreads();
    // pull + reduce in rank order: every rank computes the same bits
    const int bytes = (int)(a.n * 4);
    const long long n4 = a.n >> 2;
    for (long long i = (long long)blockIdx.x * PEER_THREADS + tid; i < n4; i += (long long)gridDim.x * PEER_THREADS) {
        float4 v[W];
#pragma unroll
        for (int j = 0; j < W; ++j) v[j] = load_sys16(a.src[j], bytes, (int)(i * 16));
        float4 s = v[0];
#pragma unroll
        for (int j = 1; j < W; ++j) {
            s.x += v[j].x;
            s.y += v[j].y;
            s.z += v[j].z;
            s.w += v[j].w;
        }
        reinterpret_cast<float4*>(a.out)[i] = s;
        if (pk.pk != nullptr) pack_store(pk, (int)i, s);
    }
    if (blockIdx.x == 0)
        for (long long e = n4 * 4 + tid; e < a.n; e += PEER_THREADS) {
            float s = load_sys4(a.src[0], bytes, (int)(e * 4));
#pragma unroll
            for (int j = 1; j < W; ++j) s += load_sys4(a.src[j], bytes, (int)(e * 4));
            a.out[e] = s;
        }
    // the last block to finish advances the call counter (every block has read it by then)
    __syncthreads();
    if (tid == 0) {
        const unsigned prev = __hip_atomic_fetch_add(&a.ctl->done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == gridDim.x - 1) {
            __hip_atomic_store(&a.ctl->done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&a.ctl->seq, target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// Self-test payload: exact in fp32 for any summation order (multiples of 1/4 in [-256, 256)).
__global__ void peer_fill_kernel(float* dst, long long n, int rank, unsigned salt) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned h = (unsigned)i * 2654435761u + (unsigned)rank * 40503u + salt * 97u;
    dst[i] = (float)(h % 2048u) * 0.25f - 256.f;
}

PeerAllReduce::PeerAllReduce(int world, int rank, int device, long long n, double timeout_s)
    : world_(world), rank_(rank), device_(device), n_(n) {
    if (world < 2 || world > PEER_MAX_WORLD) throw std::runtime_error("PeerAllReduce: world must be 2..8");
    if (rank < 0 || rank >= world) throw std::runtime_error("PeerAllReduce: bad rank");
    if (n <= 0 || n * 4 > (1ll << 30)) throw std::runtime_error("PeerAllReduce: 1..2^28 floats");
    PHIP(hipSetDevice(device));
    buf_bytes_ = ((size_t)n * 4 + 255) & ~(size_t)255;
    total_ = 2 * buf_bytes_ + sizeof(PeerCtl);
    // Uncached device memory (MTYPE UC, what RCCL uses for its xGMI buffers): peers write the
    // flags and read the send buffers over xGMI, and no L2 -- this GPU's or a peer's -- may
    // hold a stale copy of either.  The send buffers are written once per round (~50 KB),
    // so bypassing the L2 costs nothing measurable.
    if (hipExtMallocWithFlags(reinterpret_cast<void**>(&base_), total_, hipDeviceMallocUncached) != hipSuccess) {
        (void)hipGetLastError();
        base_ = nullptr;
        PHIP(hipMalloc(reinterpret_cast<void**>(&base_), total_));
    }
    PHIP(hipMemset(base_, 0, total_));
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
    for (char* p : mapped_) hipIpcCloseMemHandle(p);
    mapped_.clear();
    open_ = false;
    if (base_) {
        hipFree(base_);
        base_ = nullptr;
    }
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

void PeerAllReduce::clear() {
    PHIP(hipSetDevice(device_));
    PHIP(hipMemset(base_, 0, 2 * buf_bytes_));
    PHIP(hipDeviceSynchronize());
}

void PeerAllReduce::set_timeout(double seconds) { timeout_ticks_ = (long long)(seconds * 1e8); }

int PeerAllReduce::error() const {
    unsigned e = 0;
    PHIP(hipMemcpy(&e, &reinterpret_cast<PeerCtl*>(base_ + 2 * buf_bytes_)->err, sizeof(e), hipMemcpyDeviceToHost));
    return (int)e;
}

hipError_t PeerAllReduce::launch(int parity, float* out, const PeerPack* pack, hipStream_t s) const {
    if (!open_) return hipErrorNotInitialized;
    PeerArgs a;
    std::memset(&a, 0, sizeof(a));
    for (int j = 0; j < world_; ++j) {
        a.src[j] = reinterpret_cast<const float*>(peer_base_[j] + (parity & 1) * buf_bytes_);
        a.flag_dst[j] = &reinterpret_cast<PeerCtl*>(peer_base_[j] + 2 * buf_bytes_)->flags[rank_];
    }
    a.ctl = reinterpret_cast<PeerCtl*>(base_ + 2 * buf_bytes_);
    a.out = out;
    a.n = n_;
    a.timeout = timeout_ticks_;
    PeerPack p;
    std::memset(&p, 0, sizeof(p));
    if (pack != nullptr) p = *pack;
    const long long n4 = n_ / 4;
    const int blocks = (int)std::min<long long>(PEER_MAX_BLOCKS, std::max<long long>(1, (n4 + PEER_THREADS - 1) / PEER_THREADS));
    switch (world_) {
#define PEER_CASE(W)                                                                                  \
    case W:                                                                                           \
        hipLaunchKernelGGL(peer_allreduce_kernel<W>, dim3(blocks), dim3(PEER_THREADS), 0, s, a, p);  \
        break;
        PEER_CASE(2) PEER_CASE(3) PEER_CASE(4) PEER_CASE(5) PEER_CASE(6) PEER_CASE(7) PEER_CASE(8)
#undef PEER_CASE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

void register_peer(py::module_& m) {
    py::class_<PeerAllReduce>(m, "PeerAllReduce")
        .def(py::init<int, int, int, long long, double>(), py::arg("world"), py::arg("rank"), py::arg("device"),
             py::arg("n_floats"), py::arg("timeout_s") = 60.0)
        .def("handle", &PeerAllReduce::handle)
        .def("open", &PeerAllReduce::open)
        .def("send_ptr", [](const PeerAllReduce& p, int parity) { return reinterpret_cast<uintptr_t>(p.send(parity)); })
        .def("allreduce",
             [](const PeerAllReduce& p, int parity, uintptr_t out, uintptr_t stream) {
                 PHIP(p.launch(parity, reinterpret_cast<float*>(out), nullptr, reinterpret_cast<hipStream_t>(stream)));
             })
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
        .def("error", &PeerAllReduce::error)
        .def("close", &PeerAllReduce::close)
        .def_property_readonly("world", &PeerAllReduce::world)
        .def_property_readonly("rank", &PeerAllReduce::rank)
        .def_property_readonly("n_floats", &PeerAllReduce::n_floats)
        .def_property_readonly("is_open", &PeerAllReduce::is_open);
}
