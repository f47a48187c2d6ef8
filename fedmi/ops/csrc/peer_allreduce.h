// One-shot all-reduce over xGMI peer memory (peer_allreduce.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>

#include <string>
#include <vector>

#include "fl_common.h"
#include "peer_device.h"


class PeerAllReduce {
  public:
    // n_chunks > 0: chunk-flag table for the Adam-fused exchange (peer_device.h)
    PeerAllReduce(int world, int rank, int device, long long n_floats, double timeout_s, int n_chunks = 0);
    ~PeerAllReduce();
    PeerAllReduce(const PeerAllReduce&) = delete;
    PeerAllReduce& operator=(const PeerAllReduce&) = delete;

    pybind11::bytes handle() const;                     // IPC handle of this rank's allocation
    void open(const std::vector<pybind11::bytes>& handles);  // all ranks' handles, rank order
    float* send(int parity) const;                      // this rank's send buffer of a parity
    // out[0:n] = sum over ranks (rank order) of send(parity); optional bf16 pack epilogue
    hipError_t launch(int parity, float* out, const PeerPack* pack, hipStream_t s) const;
    // Kernel arguments of a call on `parity` writing `out` (peer_device.h), for kernels that
    // fuse the all-reduce with other work; `n_w` = floats of the weights part (default: all
    // whole float4s).
    PeerArgs args(int parity, float* out, long long n_w = -1) const;
    // Per-block completion flags for fused calls with `n_eval` evaluation blocks.
    void prepare_eval(int n_eval);
    // Zero both send buffers (image padding is never written by the engine's kernels and
    // must read as 0).  Call only while no peer is reading: after a host barrier.
    void clear();
    void set_timeout(double seconds);
    double timeout_s() const { return (double)timeout_ticks_ * 1e-8; }
    int error() const;                                  // sticky failure word (PEER_ERR_*, peer_device.h)
    // Fail-fast abort of the job from the host (Comm.Abort, watchdogs): sets the host abort word
    // this rank's spinning kernels poll, and (bounded) writes the failure word of every rank, so
    // the peers' waits end too.  Returns true when the peers' words were written in time.
    bool abort(double wait_s);
    long long n_floats() const { return n_; }
    int world() const { return world_; }
    int rank() const { return rank_; }
    int n_chunks() const { return n_chunks_; }
    bool is_open() const { return open_; }
    bool uncached() const { return uncached_; }         // send buffers in uncached memory
    bool uses_ll() const { return use_ll_; }            // LL weight chunks (peer_device.h)
    bool uses_rsag() const { return use_rsag_; }        // ... by reduce-scatter + all-gather (peer_rsag)
    int adam_grid() const { return adam_grid_; }        // PeerArgs::adam_grid (0 = full Adam grid)
    void set_adam_grid(int g) { adam_grid_ = g < 0 ? 0 : g; }
    void close();

  private:
    int world_, rank_, device_;
    long long n_;
    int n_chunks_ = 0;
    size_t buf_bytes_ = 0, total_ = 0;
    size_t cf_off_ = 0, ll_off_ = 0, ll_bytes_ = 0;  // chunk-flag table, LL ring (byte offsets)
    bool use_ll_ = false;
    bool use_rsag_ = false;
    int adam_grid_ = 0;
    char* base_ = nullptr;
    std::vector<char*> mapped_;        // peers' allocations, opened from their IPC handles
    char* peer_base_[PEER_MAX_WORLD] = {};
    long long timeout_ticks_ = 0;      // s_memrealtime ticks (100 MHz)
    bool open_ = false;
    bool uncached_ = true;
    unsigned* eflags_ = nullptr;       // fused calls: one completion flag per evaluation block
    int n_eval_ = 0;
    unsigned* host_abort_ = nullptr;   // pinned host word (PeerArgs::host_abort) + its device address
    unsigned* host_abort_dev_ = nullptr;
    unsigned* abort_word_ = nullptr;   // pinned source of the failure word abort() writes
};

void register_peer(pybind11::module_& m);
