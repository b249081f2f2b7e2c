// Batched strided 2-D copy kernel for gfx950 (pack / unpack / self-periodic /
// one-phase messages). One launch covers every face (and edge/corner message)
// of every field: the reference launches one (1,32,1)/(32,1,1)-thread kernel per
// field and side (src/update_halo.jl:497-501), i.e. 32-lane groups that waste
// half of every 64-lane CDNA wavefront. Here: 256-thread workgroups (4 full
// waves); a workgroup copies one CHUNK of one row (the inner, fastest-varying
// extent of the region), so the per-element index math is a single multiply-add
// and the block->(copy, row, chunk) decode is scalar (once per workgroup).
// Rows with unit stride on both sides move 4 elements per lane in flight.
#include <hip/hip_runtime.h>

#include "igg/copy.hpp"

namespace igg {
namespace {

constexpr int BLOCK = 256;
constexpr int EPT = 4;                         // elements per thread per chunk
constexpr int64_t CHUNK = BLOCK * EPT;         // elements of a row per workgroup

struct alignas(16) B16 { uint64_t x, y; };

template <typename T, bool FENCE>
__global__ void __launch_bounds__(BLOCK) copy2d_batch_kernel(const CopyBatch batch) {
  const int64_t b = blockIdx.x;
  int c = 0;
  // Wave-uniform scan over <= MAX_BATCH prefix sums (scalar loads from kernarg).
  while (c + 1 < batch.n && b >= batch.block_start[c + 1]) ++c;
  const Copy2D& cp = batch.c[c];
  const int64_t local = b - batch.block_start[c];
  const int64_t nchunks = (cp.n_inner + CHUNK - 1) / CHUNK;
  const int64_t o = local / nchunks;              // row (outer index)
  const int64_t i0 = (local - o * nchunks) * CHUNK;
  const T* __restrict__ src = reinterpret_cast<const T*>(cp.src) + o * cp.src_so;
  T* __restrict__ dst = reinterpret_cast<T*>(cp.dst) + o * cp.dst_so;
  const int64_t n = cp.n_inner;
  T v[EPT];
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int64_t i = i0 + k * BLOCK + threadIdx.x;
    if (i < n) v[k] = src[i * cp.src_si];
  }
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int64_t i = i0 + k * BLOCK + threadIdx.x;
    if (i < n) dst[i * cp.dst_si] = v[k];
  }
  if (FENCE) __threadfence_system();
}

// Copies whose rows are short (n_inner < 64, e.g. a face whose inner extent is
// tiny or an edge/corner message) are flattened: one element per lane.
template <typename T, bool FENCE>
__global__ void __launch_bounds__(BLOCK) copy2d_flat_kernel(const CopyBatch batch) {
  const int64_t b = blockIdx.x;
  int c = 0;
  while (c + 1 < batch.n && b >= batch.block_start[c + 1]) ++c;
  const Copy2D& cp = batch.c[c];
  const int64_t e = (b - batch.block_start[c]) * BLOCK + threadIdx.x;
  if (e < cp.n_outer * cp.n_inner) {
    const int64_t o = e / cp.n_inner, i = e - o * cp.n_inner;
    reinterpret_cast<T*>(cp.dst)[o * cp.dst_so + i * cp.dst_si] =
        reinterpret_cast<const T*>(cp.src)[o * cp.src_so + i * cp.src_si];
  }
  if (FENCE) __threadfence_system();
}

template <typename T, bool FENCE>
void launch_typed(const std::vector<Copy2D>& copies, hipStream_t stream) {
  for (int flat = 0; flat < 2; ++flat) {
    size_t pos = 0;
    while (pos < copies.size()) {
      CopyBatch batch{};
      batch.n = 0;
      int64_t blocks = 0;
      while (pos < copies.size() && batch.n < MAX_BATCH) {
        const Copy2D& c = copies[pos++];
        const int64_t total = c.n_outer * c.n_inner;
        if (total <= 0) continue;
        const bool is_flat = c.n_inner < 64;
        if (is_flat != (flat == 1)) continue;
        batch.c[batch.n] = c;
        batch.block_start[batch.n] = blocks;
        blocks += is_flat ? (total + BLOCK - 1) / BLOCK
                          : c.n_outer * ((c.n_inner + CHUNK - 1) / CHUNK);
        ++batch.n;
      }
      if (batch.n == 0) continue;
      batch.block_start[batch.n] = blocks;
      if (blocks > 0x7fffffffLL) fail("launch_copy2d: too many blocks (", blocks, ")");
      if (flat)
        hipLaunchKernelGGL((copy2d_flat_kernel<T, FENCE>), dim3(static_cast<unsigned>(blocks)), dim3(BLOCK), 0,
                           stream, batch);
      else
        hipLaunchKernelGGL((copy2d_batch_kernel<T, FENCE>), dim3(static_cast<unsigned>(blocks)), dim3(BLOCK), 0,
                           stream, batch);
      IGG_HIP_CHECK(hipGetLastError());
    }
  }
}

}  // namespace

template <bool FENCE>
void launch_sized(const std::vector<Copy2D>& copies, int elem_bytes, hipStream_t stream) {
  switch (elem_bytes) {
    case 1: launch_typed<uint8_t, FENCE>(copies, stream); break;
    case 2: launch_typed<uint16_t, FENCE>(copies, stream); break;
    case 4: launch_typed<uint32_t, FENCE>(copies, stream); break;
    case 8: launch_typed<uint64_t, FENCE>(copies, stream); break;
    case 16: launch_typed<B16, FENCE>(copies, stream); break;
    default: fail("launch_copy2d: unsupported element size ", elem_bytes, " bytes");
  }
}

void launch_copy2d(const std::vector<Copy2D>& copies, int elem_bytes, hipStream_t stream,
                   bool system_fence) {
  if (copies.empty()) return;
  if (system_fence) launch_sized<true>(copies, elem_bytes, stream);
  else launch_sized<false>(copies, elem_bytes, stream);
}

}  // namespace igg
