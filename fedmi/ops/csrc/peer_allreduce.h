// One-shot all-reduce over xGMI peer memory (peer_allreduce.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>

#include <string>
#include <vector>

#include "fl_common.h"

#define PEER_MAX_WORLD 8  // one node: every GPU has a direct xGMI link to each of its 7 peers

// Optional epilogue of the reduction: also write the reduced fp32 parameter image as the
// packed bf16 LDS image the bf16 train kernel stages (fl_kernels_bf16.hip, MLPDescB), so the
// separate pack kernel after FedAvg disappears.  Offsets are in float4 units of the fp32
// image (fl_common.h layout) and bytes of the packed region.
struct PeerPack {
    char* pk;                       // packed region (nullptr: no packing)
    int L;
    int img4_w[FL_MAX_LAYERS];      // first float4 of W_l in the image
    int img4_b[FL_MAX_LAYERS];      // first float4 of b_l
    int img4_end[FL_MAX_LAYERS];    // one past the last float4 of b_l
    int ldw4[FL_MAX_LAYERS];        // float4s per image row of W_l
    int k4[FL_MAX_LAYERS];          // packed float4 columns per row: roundup16(K_l) / 4
    int pk_w[FL_MAX_LAYERS];        // byte offset of W_l in the packed region
    int pk_lda[FL_MAX_LAYERS];      // packed row stride (bf16 elements)
    int pk_b[FL_MAX_LAYERS];        // byte offset of b_l in the packed region
};

struct PeerCtl;

class PeerAllReduce {
  public:
    PeerAllReduce(int world, int rank, int device, long long n_floats, double timeout_s);
    ~PeerAllReduce();
    PeerAllReduce(const PeerAllReduce&) = delete;
    PeerAllReduce& operator=(const PeerAllReduce&) = delete;

    pybind11::bytes handle() const;                     // IPC handle of this rank's allocation
    void open(const std::vector<pybind11::bytes>& handles);  // all ranks' handles, rank order
    float* send(int parity) const;                      // this rank's send buffer of a parity
    // out[0:n] = sum over ranks (rank order) of send(parity); optional bf16 pack epilogue
    hipError_t launch(int parity, float* out, const PeerPack* pack, hipStream_t s) const;
    // Zero both send buffers (image padding is never written by the engine's kernels and
    // must read as 0).  Call only while no peer is reading: after a host barrier.
    void clear();
    void set_timeout(double seconds);
    int error() const;                                  // sticky: a wait timed out
    long long n_floats() const { return n_; }
    int world() const { return world_; }
    int rank() const { return rank_; }
    bool is_open() const { return open_; }
    void close();

  private:
    int world_, rank_, device_;
    long long n_;
    size_t buf_bytes_ = 0, total_ = 0;
    char* base_ = nullptr;
    std::vector<char*> mapped_;        // peers' allocations, opened from their IPC handles
    char* peer_base_[PEER_MAX_WORLD] = {};
    long long timeout_ticks_ = 0;      // s_memrealtime ticks (100 MHz)
    bool open_ = false;
};

void register_peer(pybind11::module_& m);
