// Batched strided 2-D copy kernel for gfx950 (pack / unpack / self-periodic /
// gather reorder). One launch covers every face of every field of one
// dimension, both sides: the reference launches one (1,32,1)/(32,1,1)-thread
// kernel per field and side (src/update_halo.jl:497-501), i.e. 32-lane groups
// that waste half of every 64-lane CDNA wavefront. Here: 256-thread blocks
// (4 full waves), 4 elements per thread, block->copy mapping by prefix sums.
#include <hip/hip_runtime.h>

#include "igg/copy.hpp"

namespace igg {
namespace {

constexpr int BLOCK = 256;
constexpr int EPT = 4;  // elements per thread
constexpr int64_t ELEMS_PER_BLOCK = BLOCK * EPT;

struct alignas(16) B16 { uint64_t x, y; };

template <typename T>
__global__ void __launch_bounds__(BLOCK) copy2d_batch_kernel(const CopyBatch batch) {
  const int64_t b = blockIdx.x;
  int c = 0;
  // Wave-uniform scan over <= MAX_BATCH prefix sums (scalar loads from kernarg).
  while (c + 1 < batch.n && b >= batch.block_start[c + 1]) ++c;
  const Copy2D& cp = batch.c[c];
  const int64_t total = cp.n_outer * cp.n_inner;
  const int64_t base = (b - batch.block_start[c]) * ELEMS_PER_BLOCK + threadIdx.x;
  const T* __restrict__ src = reinterpret_cast<const T*>(cp.src);
  T* __restrict__ dst = reinterpret_cast<T*>(cp.dst);
  T v[EPT];
  int64_t doff[EPT];
  bool ok[EPT];
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int64_t e = base + k * BLOCK;
    ok[k] = e < total;
    const int64_t o = ok[k] ? e / cp.n_inner : 0;
    const int64_t i = ok[k] ? e - o * cp.n_inner : 0;
    if (ok[k]) v[k] = src[o * cp.src_so + i * cp.src_si];
    doff[k] = o * cp.dst_so + i * cp.dst_si;
  }
#pragma unroll
  for (int k = 0; k < EPT; ++k)
    if (ok[k]) dst[doff[k]] = v[k];
}

template <typename T>
void launch_typed(const std::vector<Copy2D>& copies, hipStream_t stream) {
  size_t pos = 0;
  while (pos < copies.size()) {
    CopyBatch batch{};
    batch.n = 0;
    int64_t blocks = 0;
    while (pos < copies.size() && batch.n < MAX_BATCH) {
      const Copy2D& c = copies[pos++];
      const int64_t total = c.n_outer * c.n_inner;
      if (total <= 0) continue;
      batch.c[batch.n] = c;
      batch.block_start[batch.n] = blocks;
      blocks += (total + ELEMS_PER_BLOCK - 1) / ELEMS_PER_BLOCK;
      ++batch.n;
    }
    if (batch.n == 0) continue;
    batch.block_start[batch.n] = blocks;
    if (blocks > 0x7fffffffLL) fail("launch_copy2d: too many blocks (", blocks, ")");
    hipLaunchKernelGGL(copy2d_batch_kernel<T>, dim3(static_cast<unsigned>(blocks)), dim3(BLOCK), 0,
                       stream, batch);
    IGG_HIP_CHECK(hipGetLastError());
  }
}

}  // namespace

void launch_copy2d(const std::vector<Copy2D>& copies, int elem_bytes, hipStream_t stream) {
  if (copies.empty()) return;
  switch (elem_bytes) {
    case 1: launch_typed<uint8_t>(copies, stream); break;
    case 2: launch_typed<uint16_t>(copies, stream); break;
    case 4: launch_typed<uint32_t>(copies, stream); break;
    case 8: launch_typed<uint64_t>(copies, stream); break;
    case 16: launch_typed<B16>(copies, stream); break;
    default: fail("launch_copy2d: unsupported element size ", elem_bytes, " bytes");
  }
}

}  // namespace igg
