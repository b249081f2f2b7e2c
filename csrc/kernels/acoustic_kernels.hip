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
constexpr int WAVES = 4;       // waves per workgroup of the marching kernel
constexpr int64_t MARCH_CH = 8;  // rows of i per wave (short chunks = more waves in flight; swept: benchmarks/acoustic_sweep.py)

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

// Marching version: a wave walks CH rows of i over 64 lanes = 62 owned
// columns plus one halo column on each side (lane 0: j0-1, lane 63: j0+62), so
// every neighbour value comes from a lane shuffle (ds_bpermute) and no lane
// takes a divergent extra load. Vx(i, j) and P2(i-1, j) are carried in
// registers from the previous row; the next row's loads are issued before the
// current row is computed. Per row each array is read once (+2/62 halo
// columns) and each output written once.
constexpr int OWN = 62;

template <typename T>
__global__ void __launch_bounds__(64 * WAVES) acoustic2d_march_kernel(AcousticArgs a, int64_t ch) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = static_cast<int64_t>(blockIdx.x) * WAVES + (threadIdx.x >> 6);
  const int64_t nx = a.nx, ny = a.ny;
  const int64_t nseg = (ny + 1 + OWN - 1) / OWN;
  const int64_t seg = wave % nseg, chunk = wave / nseg;
  const int64_t i0 = chunk * ch;
  if (i0 > nx) return;  // wave-uniform
  const int64_t i1 = min(i0 + ch, nx + 1);
  const int64_t j = seg * OWN + lane - 1;                // column of this lane
  const bool own = lane >= 1 && lane <= OWN && j <= ny;  // stores column j
  const bool jc = j >= 0 && j < ny;                      // column has cells / x-faces
  const int64_t jv = min<int64_t>(max<int64_t>(j, 0), ny);      // clamped face column
  const int64_t jcc = min<int64_t>(max<int64_t>(j, 0), ny - 1);  // clamped cell column
  const T* __restrict__ p = reinterpret_cast<const T*>(a.p);
  const T* __restrict__ vx = reinterpret_cast<const T*>(a.vx);
  const T* __restrict__ vy = reinterpret_cast<const T*>(a.vy);
  T* __restrict__ p2 = reinterpret_cast<T*>(a.p2);
  T* __restrict__ vx2 = reinterpret_cast<T*>(a.vx2);
  T* __restrict__ vy2 = reinterpret_cast<T*>(a.vy2);
  const T dtk = static_cast<T>(a.dtk), dt_rho = static_cast<T>(a.dt_rho);
  const T rdx = static_cast<T>(a.rdx), rdy = static_cast<T>(a.rdy);
  const int64_t sy = ny + 1;
  // Row state: Vx(i, j) (carried) and P2(i-1, j) (carried).
  T vx_i = vx[i0 * ny + jcc];
  T p2_prev = T(0);
  if (i0 >= 1) {
    const int64_t r = i0 - 1;
    const T vyh = vy[r * sy + jv];
    const T vyn = __shfl_down(vyh, 1);
    p2_prev = p[r * ny + jcc] - dtk * ((vx_i - vx[r * ny + jcc]) * rdx + (vyn - vyh) * rdy);
  }
  // Prefetched loads of row i.
  T vy_h = T(0), vx_n = T(0), pp = T(0);
  if (i0 < nx) {
    vy_h = vy[i0 * sy + jv];
    vx_n = vx[(i0 + 1) * ny + jcc];
    pp = p[i0 * ny + jcc];
  }
  for (int64_t i = i0; i < i1; ++i) {
    if (i < nx) {
      T vy_h1 = T(0), vx_n1 = T(0), pp1 = T(0);
      if (i + 1 < nx && i + 1 < i1) {  // prefetch row i+1
        vy_h1 = vy[(i + 1) * sy + jv];
        vx_n1 = vx[(i + 2) * ny + jcc];
        pp1 = p[(i + 1) * ny + jcc];
      }
      const T vy_n = __shfl_down(vy_h, 1);
      const T pc = pp - dtk * ((vx_n - vx_i) * rdx + (vy_n - vy_h) * rdy);
      const T pl = __shfl_up(pc, 1);
      if (own) {
        if (jc) {
          p2[i * ny + j] = pc;
          vx2[i * ny + j] = (i >= 1) ? vx_i - dt_rho * (pc - p2_prev) * rdx : vx_i;
        }
        vy2[i * sy + j] = (j >= 1 && j <= ny - 1) ? vy_h - dt_rho * (pc - pl) * rdy : vy_h;
      }
      vx_i = vx_n;
      p2_prev = pc;
      vy_h = vy_h1;
      vx_n = vx_n1;
      pp = pp1;
    } else if (own && jc) {  // i == nx: the last x-face is a boundary face
      vx2[i * ny + j] = vx_i;
    }
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

static int g_acoustic_variant = 1;  // 0: one thread per cell (recompute), 1: marching
static int64_t g_march_ch = MARCH_CH;
void acoustic2d_set_variant(int v) { g_acoustic_variant = v; }
void acoustic2d_set_chunk(int64_t ch) { g_march_ch = ch > 0 ? ch : MARCH_CH; }

void launch_acoustic2d(const AcousticArgs& a, hipStream_t stream) {
  if (a.nx < 1 || a.ny < 1) fail("acoustic2d: empty grid");
  if (a.elem_bytes != 4 && a.elem_bytes != 8)
    fail("acoustic2d: element size must be 4 or 8 bytes (got ", a.elem_bytes, ")");
  if (g_acoustic_variant == 1) {
    const int64_t ch = g_march_ch;
    const int64_t nseg = (a.ny + 1 + OWN - 1) / OWN, nch = (a.nx + 1 + ch - 1) / ch;
    const int64_t waves = nseg * nch;
    const dim3 grid(static_cast<unsigned>((waves + WAVES - 1) / WAVES));
    if (a.elem_bytes == 8)
      hipLaunchKernelGGL(acoustic2d_march_kernel<double>, grid, dim3(64 * WAVES), 0, stream, a, ch);
    else
      hipLaunchKernelGGL(acoustic2d_march_kernel<float>, grid, dim3(64 * WAVES), 0, stream, a, ch);
  } else {
    const dim3 grid(static_cast<unsigned>((a.ny + 1 + BJ - 1) / BJ), static_cast<unsigned>((a.nx + 1 + BI - 1) / BI));
    if (a.elem_bytes == 8)
      hipLaunchKernelGGL(acoustic2d_kernel<double>, grid, dim3(BJ * BI), 0, stream, a);
    else
      hipLaunchKernelGGL(acoustic2d_kernel<float>, grid, dim3(BJ * BI), 0, stream, a);
  }
  IGG_HIP_CHECK(hipGetLastError());
}

void host_acoustic2d(const AcousticArgs& a) {
  if (a.elem_bytes == 8) host_typed<double>(a);
  else if (a.elem_bytes == 4) host_typed<float>(a);
  else fail("acoustic2d: element size must be 4 or 8 bytes (got ", a.elem_bytes, ")");
}

}  // namespace igg
