// Bandwidth roofline probes for gfx950 (diagnostics; benchmarks/roofline.py).
// triad: out = a + s*b over n doubles — the same traffic mix as the diffusion
// stencil (2 streams read, 1 written); copy: out = a. 16 B per lane per access,
// grid-stride over a fixed grid, optional non-temporal stores.
#include <hip/hip_runtime.h>

#include "igg/common.hpp"

namespace igg {
namespace {

typedef double d2 __attribute__((ext_vector_type(2)));

template <bool NT, bool TRIAD, int UNROLL>
__global__ void __launch_bounds__(256) stream_kernel(d2* __restrict__ out, const d2* __restrict__ a,
                                                     const d2* __restrict__ b, double s, int64_t n2) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256 * UNROLL;
  for (int64_t base = static_cast<int64_t>(blockIdx.x) * 256 * UNROLL + threadIdx.x; base < n2; base += stride) {
    d2 va[UNROLL], vb[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int64_t i = base + u * 256;
      if (i < n2) {
        va[u] = a[i];
        if (TRIAD) vb[u] = b[i];
      }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int64_t i = base + u * 256;
      if (i < n2) {
        const d2 r = TRIAD ? va[u] + s * vb[u] : va[u];
        if (NT) __builtin_nontemporal_store(r, out + i);
        else out[i] = r;
      }
    }
  }
}

// read-only: sum of a + b per thread, one store per thread at the end (the
// streamed bytes are the 2 reads); write-only: out = s (fill).
template <int UNROLL>
__global__ void __launch_bounds__(256) read_kernel(double* __restrict__ out, const d2* __restrict__ a,
                                                   const d2* __restrict__ b, int64_t n2) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256 * UNROLL;
  d2 acc = {0.0, 0.0};
  for (int64_t base = static_cast<int64_t>(blockIdx.x) * 256 * UNROLL + threadIdx.x; base < n2; base += stride) {
    d2 va[UNROLL], vb[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int64_t i = base + u * 256;
      if (i < n2) {
        va[u] = __builtin_nontemporal_load(a + i);
        vb[u] = __builtin_nontemporal_load(b + i);
      } else {
        va[u] = d2{0.0, 0.0};
        vb[u] = d2{0.0, 0.0};
      }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) acc += va[u] + vb[u];
  }
  out[static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x] = acc.x + acc.y;
}

template <int UNROLL>
__global__ void __launch_bounds__(256) write_kernel(d2* __restrict__ out, double s, int64_t n2) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256 * UNROLL;
  for (int64_t base = static_cast<int64_t>(blockIdx.x) * 256 * UNROLL + threadIdx.x; base < n2; base += stride) {
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int64_t i = base + u * 256;
      if (i < n2) __builtin_nontemporal_store(d2{s, s}, out + i);
    }
  }
}

}  // namespace

void launch_stream_probe(int kind, double* out, const double* a, const double* b, int64_t n, int blocks,
                         hipStream_t stream) {
  const int64_t n2 = n / 2;
  auto* o = reinterpret_cast<d2*>(out);
  auto* pa = reinterpret_cast<const d2*>(a);
  auto* pb = reinterpret_cast<const d2*>(b);
  switch (kind) {
    case 0: hipLaunchKernelGGL((stream_kernel<true, true, 4>), dim3(blocks), dim3(256), 0, stream, o, pa, pb, 0.5, n2); break;
    case 1: hipLaunchKernelGGL((stream_kernel<false, true, 4>), dim3(blocks), dim3(256), 0, stream, o, pa, pb, 0.5, n2); break;
    case 2: hipLaunchKernelGGL((stream_kernel<true, false, 4>), dim3(blocks), dim3(256), 0, stream, o, pa, pb, 0.5, n2); break;
    case 3: hipLaunchKernelGGL((stream_kernel<false, false, 4>), dim3(blocks), dim3(256), 0, stream, o, pa, pb, 0.5, n2); break;
    case 4: hipLaunchKernelGGL((stream_kernel<true, true, 8>), dim3(blocks), dim3(256), 0, stream, o, pa, pb, 0.5, n2); break;
    // read-only (2 streams; `out` must hold blocks*256 doubles) / write-only (1 stream)
    case 5: hipLaunchKernelGGL((read_kernel<4>), dim3(blocks), dim3(256), 0, stream, out, pa, pb, n2); break;
    case 6: hipLaunchKernelGGL((write_kernel<4>), dim3(blocks), dim3(256), 0, stream, o, 0.5, n2); break;
    default: fail("stream probe: bad kind ", kind);
  }
  IGG_HIP_CHECK(hipGetLastError());
}

}  // namespace igg
