// Batched strided 2-D copies: the single primitive behind halo pack, unpack,
// in-place self-periodic exchange and gather reorder.
//
// Reference equivalents: write_d2x!/read_x2d! GPU kernels
// (src/update_halo.jl:655-678), write_h2h!/read_h2h! + memcopy! host copies
// (src/update_halo.jl:569-596, 755-784) and gpumemcopy! (:796-798). Unlike the
// reference (one 32-lane launch per field and side), one launch here moves every
// face of every field of a dimension.
#pragma once

#include <cstdint>
#include <functional>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "igg/common.hpp"

namespace igg {

// One strided 2-D copy of n_outer x n_inner elements; strides are in elements.
struct Copy2D {
  const char* src;
  char* dst;
  int64_t n_outer, n_inner;
  int64_t src_so, src_si;
  int64_t dst_so, dst_si;
};

// Optional wait at the start of a copy launch (the z unpack of FusedHalo with
// the in-kernel step synchronisation: no sync kernel runs between the stencil
// and the unpack): one thread per workgroup spins until ARRIVED[rank] >= EPOCH
// in `flags` (this GPU's flag block, put.hpp) for every listed rank, then a
// system acquire orders the workgroup's loads after the senders' stores.
struct CopyWait {
  uint64_t* flags = nullptr;  // own flag block (EPOCH, ERROR, ARRIVED[])
  int rank[2] = {0, 0};
  int n = 0;
  int64_t timeout_ticks = 0;
};

constexpr int MAX_BATCH = 32;  // all 26 one-phase directions in one launch; kernarg < 4 KiB

struct CopyBatch {
  Copy2D c[MAX_BATCH];
  int64_t block_start[MAX_BATCH + 1];
  int n;
  uint32_t flat_mask = 0;    // bit c: copy c has short rows -> one element per lane
  uint32_t gather_mask = 0;  // bit c: long rows with a strided side (z faces of a C-ordered field)
  // Put transport: a device-resident exchange epoch selects the arena half;
  // parity_side 1 shifts every dst, 2 every src by parity_bytes when odd.
  const uint64_t* epoch = nullptr;
  int64_t parity_bytes = 0;
  int parity_side = 0;
  int parity_add = 0;  // half = ((*epoch + parity_add) & 1)
  CopyWait wait;       // n > 0: wait for the senders' arrival first
};

struct ParityShift {
  const uint64_t* epoch = nullptr;
  int64_t bytes = 0;
  int side = 0;  // 0 none, 1 dst, 2 src
  int add = 0;   // the half is ((*epoch + add) & 1)
};

// Device: enqueue all copies (any count, split in MAX_BATCH chunks) on `stream`.
// system_fence: every wave ends by waiting for its stores and writing its
// XCD's L2 back at system scope (put transport: stores into a peer's
// fine-grained arena reach the owner before the following sync kernel
// publishes them; docs/COHERENCE.md).
void launch_copy2d(const std::vector<Copy2D>& copies, int elem_bytes, hipStream_t stream,
                   bool system_fence = false, const ParityShift& parity = ParityShift{},
                   const CopyWait& wait = CopyWait{});

// Host: perform all copies now (threaded above THREADCOPY_THRESHOLD bytes).
void host_copy2d(const std::vector<Copy2D>& copies, int elem_bytes);

// Host parallel-for on the runtime's persistent worker pool.
void host_parallel_for(int64_t n, int64_t grain, const std::function<void(int64_t, int64_t)>& fn);

}  // namespace igg
