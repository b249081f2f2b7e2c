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

// z-face column probe (benchmarks/zface_counters.py): one 8-B element per
// row of `pitch` elements - the z face of a C-ordered field, one element per
// 4 KiB row at 512^3 f64. DIR 0 (pack): dst[r] = src[r * pitch]; DIR 1
// (unpack): dst[r * pitch] = src[r]. The strided side goes through a buffer
// access with cache-policy bits `aux` (gfx950: 1 sc0, 2 nt, 16 sc1), the
// contiguous side is plain. Each lane keeps ZROWS independent requests in
// flight (like the copy kernel's gather path).
constexpr int ZROWS = 8;
typedef unsigned int U2 __attribute__((ext_vector_type(2)));

template <int DIR>
__global__ void __launch_bounds__(256) zcol_kernel(const U2* __restrict__ src, U2* __restrict__ dst,
                                                  int64_t rows, int64_t pitch, int aux) {
  const int64_t nthr = static_cast<int64_t>(gridDim.x) * 256;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  const void* strided = DIR == 0 ? static_cast<const void*>(src) : static_cast<const void*>(dst);
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(strided), static_cast<short>(0), 0x7fffffff, 0x00020000);
  U2 v[ZROWS];
#pragma unroll
  for (int k = 0; k < ZROWS; ++k) {
    const int64_t r = r0 + k * nthr;
    v[k] = U2{0, 0};
    if (r < rows) {
      if (DIR == 0) {
        const int off = static_cast<int>(r * pitch * 8);
        switch (aux) {  // the policy operand must be a constant
          case 1: v[k] = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 1); break;
          case 2: v[k] = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 2); break;
          case 3: v[k] = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 3); break;
          case 16: v[k] = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 16); break;
          case 17: v[k] = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 17); break;
          case 18: v[k] = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 18); break;
          default: v[k] = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0); break;
        }
      } else {
        v[k] = src[r];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < ZROWS; ++k) {
    const int64_t r = r0 + k * nthr;
    if (r < rows) {
      if (DIR == 0) {
        dst[r] = v[k];
      } else {
        const int off = static_cast<int>(r * pitch * 8);
        switch (aux) {
          case 1: __builtin_amdgcn_raw_buffer_store_b64(v[k], rs, off, 0, 1); break;
          case 2: __builtin_amdgcn_raw_buffer_store_b64(v[k], rs, off, 0, 2); break;
          case 3: __builtin_amdgcn_raw_buffer_store_b64(v[k], rs, off, 0, 3); break;
          case 16: __builtin_amdgcn_raw_buffer_store_b64(v[k], rs, off, 0, 16); break;
          case 17: __builtin_amdgcn_raw_buffer_store_b64(v[k], rs, off, 0, 17); break;
          case 18: __builtin_amdgcn_raw_buffer_store_b64(v[k], rs, off, 0, 18); break;
          default: __builtin_amdgcn_raw_buffer_store_b64(v[k], rs, off, 0, 0); break;
        }
      }
    }
  }
}

}  // namespace

void launch_zcol_probe(int dir, const void* src, void* dst, int64_t rows, int64_t pitch, int aux,
                       hipStream_t stream) {
  if (rows <= 0 || pitch <= 0 || rows * pitch * 8 > 0x7fffffffLL) fail("zcol probe: the strided side must span < 2 GiB");
  if (aux != 0 && aux != 1 && aux != 2 && aux != 3 && aux != 16 && aux != 17 && aux != 18)
    fail("zcol probe: aux in {0, 1, 2, 3, 16, 17, 18}");
  const int64_t threads = (rows + ZROWS - 1) / ZROWS;
  const unsigned blocks = static_cast<unsigned>((threads + 255) / 256);
  auto* s = static_cast<const U2*>(src);
  auto* d = static_cast<U2*>(dst);
  if (dir == 0) hipLaunchKernelGGL(zcol_kernel<0>, dim3(blocks), dim3(256), 0, stream, s, d, rows, pitch, aux);
  else hipLaunchKernelGGL(zcol_kernel<1>, dim3(blocks), dim3(256), 0, stream, s, d, rows, pitch, aux);
  IGG_HIP_CHECK(hipGetLastError());
}

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
