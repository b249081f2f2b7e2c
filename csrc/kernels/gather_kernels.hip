// Gather block-reorder kernel (root side of gather!): replaces the host triple
// loop of src/gather.jl:60-63. The rank-ordered flat receive buffer is a
// sequence of rows (s2 contiguous elements each: nprocs * s0 * s1 rows); every
// row lands contiguously in the global array. One wave per row: the row's
// (rank, i0, i1) -> destination decode is wave-uniform scalar math (once per
// row, not per element), and the lanes stream the row with 16-byte accesses
// when its byte length allows, else element by element.
#include <hip/hip_runtime.h>

#include "igg/gather.hpp"

namespace igg {
namespace {

constexpr int BLOCK = 256;
constexpr int WAVES = BLOCK / 64;
struct alignas(16) B16 { uint64_t x, y; };

struct RowGeom {
  int64_t s0, s1, s2;   // block extent (elements)
  int64_t d0, d1, d2;   // process grid
  int64_t nrows;        // nprocs * s0 * s1
};

template <typename U>
__global__ void __launch_bounds__(BLOCK)
gather_rows_kernel(const char* __restrict__ src, char* __restrict__ dst, const RowGeom g, int64_t units) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = static_cast<int64_t>(blockIdx.x) * WAVES + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * WAVES;
  const int64_t rows_per_block = g.s0 * g.s1;
  const int64_t g1 = g.d1 * g.s1;
  for (int64_t row = wave; row < g.nrows; row += nwaves) {
    const int64_t p = row / rows_per_block;
    const int64_t rem = row - p * rows_per_block;
    const int64_t i0 = rem / g.s1, i1 = rem - i0 * g.s1;
    const int64_t c2 = p % g.d2, c1 = (p / g.d2) % g.d1, c0 = p / (g.d1 * g.d2);
    const U* s = reinterpret_cast<const U*>(src) + row * units;
    // destination row (in units of s2 elements) of the global array
    const int64_t drow = ((c0 * g.s0 + i0) * g1 + c1 * g.s1 + i1) * g.d2 + c2;
    U* d = reinterpret_cast<U*>(dst) + drow * units;
    int64_t u = lane;
    for (; u + 192 < units; u += 256) {  // 4 independent loads in flight per lane
      const U a0 = s[u], a1 = s[u + 64], a2 = s[u + 128], a3 = s[u + 192];
      d[u] = a0;
      d[u + 64] = a1;
      d[u + 128] = a2;
      d[u + 192] = a3;
    }
    for (; u < units; u += 64) d[u] = s[u];
  }
}

template <typename U>
void launch_rows(const void* src, void* dst, const RowGeom& g, int64_t units, hipStream_t stream) {
  // a few waves per CU in flight; rows are grid-strided
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((g.nrows + WAVES - 1) / WAVES, 256 * 32));
  hipLaunchKernelGGL(gather_rows_kernel<U>, dim3(static_cast<unsigned>(blocks)), dim3(BLOCK), 0, stream,
                     static_cast<const char*>(src), static_cast<char*>(dst), g, units);
  IGG_HIP_CHECK(hipGetLastError());
}

}  // namespace

void launch_gather_reorder(const void* src, void* dst, const Int3& s, const Int3& dims,
                           int elem_bytes, hipStream_t stream) {
  RowGeom g{s[0], s[1], s[2], dims[0], dims[1], dims[2], dims[0] * dims[1] * dims[2] * s[0] * s[1]};
  if (g.nrows == 0 || s[2] == 0) return;
  if (elem_bytes != 1 && elem_bytes != 2 && elem_bytes != 4 && elem_bytes != 8 && elem_bytes != 16)
    fail("gather: unsupported element size ", elem_bytes);
  const int64_t row_bytes = s[2] * elem_bytes;
  // 16-byte units when every row (source and destination) is 16-byte aligned:
  // rows are row_bytes apart in the source and start at multiples of
  // s2*elem_bytes in the destination (both allocations are 256-byte aligned).
  const bool v16 = row_bytes % 16 == 0 && reinterpret_cast<uintptr_t>(src) % 16 == 0 &&
                   reinterpret_cast<uintptr_t>(dst) % 16 == 0;
  if (v16) {
    launch_rows<B16>(src, dst, g, row_bytes / 16, stream);
    return;
  }
  switch (elem_bytes) {
    case 1: launch_rows<uint8_t>(src, dst, g, s[2], stream); break;
    case 2: launch_rows<uint16_t>(src, dst, g, s[2], stream); break;
    case 4: launch_rows<uint32_t>(src, dst, g, s[2], stream); break;
    case 8: launch_rows<uint64_t>(src, dst, g, s[2], stream); break;
    default: launch_rows<B16>(src, dst, g, s[2], stream); break;
  }
}

}  // namespace igg
