// Gather block-reorder kernel (root side of gather!): replaces the host triple
// loop of src/gather.jl:60-63. Reads the rank-ordered flat receive buffer
// linearly (coalesced) and writes each block row contiguously into the global
// array.
#include <hip/hip_runtime.h>

#include "igg/gather.hpp"

namespace igg {
namespace {

constexpr int BLOCK = 256;
struct alignas(16) B16 { uint64_t x, y; };

template <typename T>
__global__ void __launch_bounds__(BLOCK)
gather_reorder_kernel(const T* __restrict__ src, T* __restrict__ dst, int64_t s0, int64_t s1,
                      int64_t s2, int64_t d0, int64_t d1, int64_t d2, int64_t total) {
  const int64_t blk = s0 * s1 * s2;
  const int64_t g1 = d1 * s1, g2 = d2 * s2;
  for (int64_t e = static_cast<int64_t>(blockIdx.x) * BLOCK + threadIdx.x; e < total;
       e += static_cast<int64_t>(gridDim.x) * BLOCK) {
    const int64_t p = e / blk;
    int64_t r = e - p * blk;
    const int64_t i2 = r % s2; r /= s2;
    const int64_t i1 = r % s1;
    const int64_t i0 = r / s1;
    const int64_t c2 = p % d2;
    const int64_t c1 = (p / d2) % d1;
    const int64_t c0 = p / (d1 * d2);
    dst[((c0 * s0 + i0) * g1 + c1 * s1 + i1) * g2 + c2 * s2 + i2] = src[e];
  }
}

template <typename T>
void launch(const void* src, void* dst, const Int3& s, const Int3& d, hipStream_t stream) {
  const int64_t total = s[0] * s[1] * s[2] * d[0] * d[1] * d[2];
  if (total == 0) return;
  const int64_t blocks = std::min<int64_t>((total + BLOCK - 1) / BLOCK, 256 * 16);
  hipLaunchKernelGGL(gather_reorder_kernel<T>, dim3(static_cast<unsigned>(blocks)), dim3(BLOCK), 0,
                     stream, static_cast<const T*>(src), static_cast<T*>(dst), s[0], s[1], s[2],
                     d[0], d[1], d[2], total);
  IGG_HIP_CHECK(hipGetLastError());
}

}  // namespace

void launch_gather_reorder(const void* src, void* dst, const Int3& s, const Int3& dims,
                           int elem_bytes, hipStream_t stream) {
  switch (elem_bytes) {
    case 1: launch<uint8_t>(src, dst, s, dims, stream); break;
    case 2: launch<uint16_t>(src, dst, s, dims, stream); break;
    case 4: launch<uint32_t>(src, dst, s, dims, stream); break;
    case 8: launch<uint64_t>(src, dst, s, dims, stream); break;
    case 16: launch<B16>(src, dst, s, dims, stream); break;
    default: fail("gather: unsupported element size ", elem_bytes);
  }
}

}  // namespace igg
