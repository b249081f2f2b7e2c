// Device-resident gather-to-root (gather!, src/gather.jl:25-65).
//
// Reference: non-root ranks Isend their whole local array; root Irecv's each
// block into a cached grow-only flat buffer, copies its own block, Waitall's,
// then scatters the blocks into the global layout with a host triple loop
// (gather.jl:60-63). Here: one RCCL group receives all blocks straight into a
// grow-only device buffer and a HIP reorder kernel writes the global layout
// (block from coords (c0,c1,c2) -> A_global[c0*s0:(c0+1)*s0, ...]).
#pragma once

#include <cstdint>
#include <functional>
#include <string>
#include <utility>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "igg/comm.hpp"
#include "igg/halo.hpp"

namespace igg {

// Reorder `nprocs` contiguous blocks of extent `s` (rank order = row-major
// Cartesian coords over `dims`) from `src` into the C-contiguous global array
// `dst` of extent dims*s.
void launch_gather_reorder(const void* src, void* dst, const Int3& s, const Int3& dims,
                           int elem_bytes, hipStream_t stream);

class Gatherer {
 public:
  ~Gatherer() { free(); }
  // `a` must be a C-contiguous device field; `dst` (device, C-contiguous
  // dims*size) is only used on `root`.
  void gather(const Field& a, void* dst, int root, const Int3& dims, RcclComm& comm,
              hipStream_t stream);
  size_t capacity() const { return bytes_; }
  void free();

 private:
  char* buf_ = nullptr;
  size_t bytes_ = 0;
};

// Non-blocking gather by root pull (MI355X copy engines). start(): every rank
// drains its stream (so `a` is final), publishes the IPC handle + offset of the
// allocation holding `a`; the root enqueues one hipMemcpyAsync per peer
// (peer -> root staging buffer: a P2P copy over xGMI executed by the SDMA
// engines, no compute units) plus its own block on a private stream, and
// returns immediately: the application keeps computing while the data moves.
// wait(): the root orders the caller's stream after the pulls and reorders
// into the global layout; every rank then passes a barrier, after which the
// peers may modify `a` again (MPI_Igather semantics: `a` is read-only until
// wait() returns). Peer mappings live from start() to wait() only.
class PullGatherer {
 public:
  using AllGather = std::function<std::vector<std::string>(const std::string&)>;
  PullGatherer(int rank, int nranks, AllGather allgather);
  ~PullGatherer();
  PullGatherer(const PullGatherer&) = delete;
  PullGatherer& operator=(const PullGatherer&) = delete;
  void start(const Field& a, int root, const Int3& dims);
  void wait(void* dst, hipStream_t stream);
  bool pending() const { return pending_; }
  void free();

 private:
  int rank_, nranks_;
  AllGather allgather_;
  hipStream_t side_ = nullptr;
  hipEvent_t done_ = nullptr;
  char* buf_ = nullptr;
  size_t bytes_ = 0;
  bool pending_ = false;
  int root_ = 0;
  Field field_{};
  Int3 dims_{1, 1, 1};
  std::vector<std::pair<std::string, void*>> opened_;  // peer mappings of the pending gather
};

}  // namespace igg
