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

}  // namespace igg
