// Fused 2-D staggered acoustic step (see include/igg/acoustic.hpp).
//
// Thread (i, j) owns cell (i, j) plus the x-face and y-face on its lower sides,
// for i in [0, nx], j in [0, ny] (the extra row/column covers the last faces).
// Workgroup = 64 consecutive j (one wave along the contiguous dimension) x 4 i;
// every global access of a wave is one contiguous 64-element segment, and the
// neighbour values a thread re-reads (P and V of cells i-1 / j-1) were just
// loaded by the adjacent lane or wave, so they come from L1/L2, not HBM.
#include <hip/hip_runtime.h>

#include "igg/acoustic.hpp"
#include "igg/common.hpp"
#include "igg/copy.hpp"

namespace igg {
namespace {

constexpr int BJ = 64, BI = 4;

template <typename T>
struct Acc {
  const T* __restrict__ p;
  const T* __restrict__ vx;
  const T* __restrict__ vy;
  int64_t nx, ny;
  T dtk, rdx, rdy;
  // P2 of cell (i, j); callers guarantee 0 <= i < nx, 0 <= j < ny.
  __device__ __forceinline__ T p2(int64_t i, int64_t j) const {
    const T div = (vx[(i + 1) * ny + j] - vx[i * ny + j]) * rdx +
                  (vy[i * (ny + 1) + j + 1] - vy[i * (ny + 1) + j]) * rdy;
    return p[i * ny + j] - dtk * div;
  }
};

template <typename T>
__global__ void __launch_bounds__(BJ * BI) acoustic2d_kernel(AcousticArgs a) {
  const int64_t j = static_cast<int64_t>(blockIdx.x) * BJ + (threadIdx.x % BJ);
  const int64_t i = static_cast<int64_t>(blockIdx.y) * BI + (threadIdx.x / BJ);
  const int64_t nx = a.nx, ny = a.ny;
  if (i > nx || j > ny) return;
  Acc<T> c{reinterpret_cast<const T*>(a.p), reinterpret_cast<const T*>(a.vx), reinterpret_cast<const T*>(a.vy),
           nx, ny, static_cast<T>(a.dtk), static_cast<T>(a.rdx), static_cast<T>(a.rdy)};
  const T dt_rho = static_cast<T>(a.dt_rho);
  T* p2 = reinterpret_cast<T*>(a.p2);
  T* vx2 = reinterpret_cast<T*>(a.vx2);
  T* vy2 = reinterpret_cast<T*>(a.vy2);
  const bool cell = i < nx && j < ny;
  const T pc = cell ? c.p2(i, j) : T(0);
  if (cell) p2[i * ny + j] = pc;
  if (j < ny) {  // x-face (i, j), i in [0, nx]
    const int64_t k = i * ny + j;
    vx2[k] = (i >= 1 && i <= nx - 1) ? c.vx[k] - dt_rho * (pc - c.p2(i - 1, j)) * c.rdx : c.vx[k];
  }
  if (i < nx) {  // y-face (i, j), j in [0, ny]
    const int64_t k = i * (ny + 1) + j;
    vy2[k] = (j >= 1 && j <= ny - 1) ? c.vy[k] - dt_rho * (pc - c.p2(i, j - 1)) * c.rdy : c.vy[k];
  }
}

template <typename T>
void host_typed(const AcousticArgs& a) {
  const int64_t nx = a.nx, ny = a.ny;
  Acc<T> c{reinterpret_cast<const T*>(a.p), reinterpret_cast<const T*>(a.vx), reinterpret_cast<const T*>(a.vy),
           nx, ny, static_cast<T>(a.dtk), static_cast<T>(a.rdx), static_cast<T>(a.rdy)};
  auto p2f = [&](int64_t i, int64_t j) {
    const T div = (c.vx[(i + 1) * ny + j] - c.vx[i * ny + j]) * c.rdx +
                  (c.vy[i * (ny + 1) + j + 1] - c.vy[i * (ny + 1) + j]) * c.rdy;
    return c.p[i * ny + j] - c.dtk * div;
  };
  const T dt_rho = static_cast<T>(a.dt_rho);
  T* p2 = reinterpret_cast<T*>(a.p2);
  T* vx2 = reinterpret_cast<T*>(a.vx2);
  T* vy2 = reinterpret_cast<T*>(a.vy2);
  host_parallel_for(nx + 1, 16, [&](int64_t i0, int64_t i1) {
    for (int64_t i = i0; i < i1; ++i)
      for (int64_t j = 0; j <= ny; ++j) {
        const bool cell = i < nx && j < ny;
        const T pc = cell ? p2f(i, j) : T(0);
        if (cell) p2[i * ny + j] = pc;
        if (j < ny) {
          const int64_t k = i * ny + j;
          vx2[k] = (i >= 1 && i <= nx - 1) ? c.vx[k] - dt_rho * (pc - p2f(i - 1, j)) * c.rdx : c.vx[k];
        }
        if (i < nx) {
          const int64_t k = i * (ny + 1) + j;
          vy2[k] = (j >= 1 && j <= ny - 1) ? c.vy[k] - dt_rho * (pc - p2f(i, j - 1)) * c.rdy : c.vy[k];
        }
      }
  });
}

}  // namespace

void launch_acoustic2d(const AcousticArgs& a, hipStream_t stream) {
  if (a.nx < 1 || a.ny < 1) fail("acoustic2d: empty grid");
  const dim3 grid(static_cast<unsigned>((a.ny + 1 + BJ - 1) / BJ), static_cast<unsigned>((a.nx + 1 + BI - 1) / BI));
  if (a.elem_bytes == 8)
    hipLaunchKernelGGL(acoustic2d_kernel<double>, grid, dim3(BJ * BI), 0, stream, a);
  else if (a.elem_bytes == 4)
    hipLaunchKernelGGL(acoustic2d_kernel<float>, grid, dim3(BJ * BI), 0, stream, a);
  else
    fail("acoustic2d: element size must be 4 or 8 bytes (got ", a.elem_bytes, ")");
  IGG_HIP_CHECK(hipGetLastError());
}

void host_acoustic2d(const AcousticArgs& a) {
  if (a.elem_bytes == 8) host_typed<double>(a);
  else if (a.elem_bytes == 4) host_typed<float>(a);
  else fail("acoustic2d: element size must be 4 or 8 bytes (got ", a.elem_bytes, ")");
}

}  // namespace igg
