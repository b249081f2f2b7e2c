// Fused 2-D staggered acoustic step (see include/igg/acoustic.hpp).
//
// Thread (i, j) owns cell (i, j) plus the x-face and y-face on its lower sides,
// for i in [0, nx], j in [0, ny] (the extra row/column covers the last faces).
// Workgroup = 64 consecutive j (one wave along the contiguous dimension) x 4 i;
// every global access of a wave is one contiguous 64-element segment, and the
// neighbour values a thread re-reads (P and V of cells i-1 / j-1) were just
// loaded by the adjacent lane or wave, so they come from L1/L2, not HBM.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "igg/acoustic.hpp"
#include "igg/common.hpp"
#include "igg/copy.hpp"
#include "igg/devsync.hpp"
#include "igg/sysstore.hpp"

namespace igg {
namespace {

constexpr int BJ = 64, BI = 4;
constexpr int WAVES = 4;       // waves per workgroup of the marching kernel
constexpr int64_t MARCH_CH = 8;   // rows of i per wave, scalar march (short chunks = more waves in flight)
constexpr int64_t VMARCH_CH = 2;  // rows of i per wave, vector march (swept 2..12: profiles/r1_configs/acoustic_sweep_vmarch.log)

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

// Vectorised marching version: each lane owns VJ consecutive columns (16 B
// per lane and array for f32 VJ=4), a wave = 62 owned vectors + one halo
// vector on each side (lanes 0 and 63), so each load/store instruction moves
// 1 KiB instead of 256 B. Neighbour columns come from the lane's own vector or
// one lane shuffle. P/Vx rows (pitch ny, ny % VJ == 0) are vector aligned; Vy
// rows have pitch ny+1, so Vy uses element-aligned vector accesses (gfx950
// global memory accepts dword-aligned dwordx4), and the lane that starts at
// column ny handles the last Vy face column with a scalar access. Same
// arithmetic per element as acoustic2d_march_kernel (bitwise equal).
//
// FUSED (FusedAcoustic, acoustic.hpp): the staggered boundary faces travel to
// the neighbours inside this sweep. Row i = 2 of Vx2 goes to the x-low
// neighbour's row nx, row nx-2 to the x-high neighbour's row 0; column 2 of
// Vy2 to the y-low neighbour's column ny, column ny-2 to the y-high
// neighbour's column 0 - system-scope stores (st_sys, igg/sysstore.hpp:
// written through this XCD's L2, acknowledged by the owner's memory before
// the wave retires); and
// this rank's own faces on a side with a neighbour are not written here (the
// neighbour stores them).
template <typename T>
__device__ __forceinline__ void st_remote(T* p, const T& v, int plain) {
  if (plain) *p = v;  // debug knob (IGG_FUSED_PLAIN_STORES=1), single device only
  else st_sys(p, v);
}

// The rows [i0, i1) of one wave's segment. FEAT: the exchange features of the
// fused step (sends, faces left to the neighbours) are compiled in; a wave runs
// that form only if its tile touches them (acoustic2d_vmarch_kernel).
template <typename T, int VJ, bool FEAT>
__device__ __forceinline__ void vmarch_rows(const AcousticArgs& a, const AcousticHalo& h, int64_t seg,
                                            int64_t i0, int64_t i1) {
  // No FMA contraction: every value is rounded per operation, so a point gets
  // bitwise the same result wherever it is computed - in the march loop or in
  // a chunk's first-row recomputation of P2(i-1), on this rank or on the
  // neighbour that owns it (the fused exchange recomputes halo values locally
  // instead of receiving them: acoustic.hpp FusedAcoustic). Memory-bound
  // kernel: the extra VALU operations are free.
#pragma clang fp contract(off)
  typedef T V __attribute__((ext_vector_type(VJ)));
  typedef T VU __attribute__((ext_vector_type(VJ), aligned(sizeof(T))));
  constexpr int64_t OWNV = 62 * VJ;
  const int lane = threadIdx.x & 63;
  const int64_t nx = a.nx, ny = a.ny, sy = ny + 1;
  const int64_t j0 = seg * OWNV + static_cast<int64_t>(lane - 1) * VJ;  // first column of this lane
  const bool own = lane >= 1 && lane <= 62 && j0 <= ny;
  const bool cells = j0 + VJ <= ny && j0 >= 0;   // VJ cell / x-face columns
  const bool last = j0 == ny;                    // only the boundary y-face column ny
  const int64_t jl = min<int64_t>(max<int64_t>(j0, 0), ny - VJ);  // clamped vector start
  const T* __restrict__ p = reinterpret_cast<const T*>(a.p);
  const T* __restrict__ vx = reinterpret_cast<const T*>(a.vx);
  const T* __restrict__ vy = reinterpret_cast<const T*>(a.vy);
  T* __restrict__ p2 = reinterpret_cast<T*>(a.p2);
  T* __restrict__ vx2 = reinterpret_cast<T*>(a.vx2);
  T* __restrict__ vy2 = reinterpret_cast<T*>(a.vy2);
  const T dtk = static_cast<T>(a.dtk), dt_rho = static_cast<T>(a.dt_rho);
  const T rdx = static_cast<T>(a.rdx), rdy = static_cast<T>(a.rdy);
  auto ldv = [&](const T* base, int64_t row) { return *reinterpret_cast<const V*>(base + row * ny + jl); };
  auto ldy = [&](int64_t row) {  // Vy(row, j0..j0+VJ-1); the column-ny lane holds Vy(row, ny) in element 0
    V v = *reinterpret_cast<const VU*>(vy + row * sy + jl);
    if (last) {
      v = V(T(0));
      v[0] = vy[row * sy + ny];
    }
    return v;
  };
  auto vy_next = [&](const V& h) {  // Vy(row, j+1) per element
    V n;
    const T up = __shfl_down(h[0], 1);
#pragma unroll
    for (int e = 0; e < VJ; ++e) n[e] = e + 1 < VJ ? h[e + 1 < VJ ? e + 1 : e] : up;
    return n;
  };
  V vx_i = ldv(vx, i0);
  V p2_prev = V(T(0));
  if (i0 >= 1) {
    const V vyh = ldy(i0 - 1), vxp = ldv(vx, i0 - 1), pp0 = ldv(p, i0 - 1);
    const V vyn = vy_next(vyh);
#pragma unroll
    for (int e = 0; e < VJ; ++e) p2_prev[e] = pp0[e] - dtk * ((vx_i[e] - vxp[e]) * rdx + (vyn[e] - vyh[e]) * rdy);
  }
  V vy_h = V(T(0)), vx_n = V(T(0)), pp = V(T(0));
  if (i0 < nx) {
    vy_h = ldy(i0);
    vx_n = ldv(vx, i0 + 1);
    pp = ldv(p, i0);
  }
  for (int64_t i = i0; i < i1; ++i) {
    if (i < nx) {
      V vy_h1 = V(T(0)), vx_n1 = V(T(0)), pp1 = V(T(0));
      if (i + 1 < nx && i + 1 < i1) {  // prefetch row i+1
        vy_h1 = ldy(i + 1);
        vx_n1 = ldv(vx, i + 2);
        pp1 = ldv(p, i + 1);
      }
      const V vy_n = vy_next(vy_h);
      V pc;
#pragma unroll
      for (int e = 0; e < VJ; ++e) pc[e] = pp[e] - dtk * ((vx_n[e] - vx_i[e]) * rdx + (vy_n[e] - vy_h[e]) * rdy);
      const T pl_lane = __shfl_up(pc[VJ - 1], 1);
      if (own) {
        V vyo;
#pragma unroll
        for (int e = 0; e < VJ; ++e) {
          const T pl = e == 0 ? pl_lane : pc[e > 0 ? e - 1 : 0];
          const int64_t j = j0 + e;
          vyo[e] = (j >= 1 && j <= ny - 1) ? vy_h[e] - dt_rho * (pc[e] - pl) * rdy : vy_h[e];
        }
        if (cells) {
          V vxo;
#pragma unroll
          for (int e = 0; e < VJ; ++e) vxo[e] = (i >= 1) ? vx_i[e] - dt_rho * (pc[e] - p2_prev[e]) * rdx : vx_i[e];
          __builtin_nontemporal_store(pc, reinterpret_cast<V*>(p2 + i * ny + j0));
          if constexpr (FEAT) {
            // face 0 of a side with a neighbour: the neighbour stores it
            if (!(i == 0 && h.nb_x[0])) __builtin_nontemporal_store(vxo, reinterpret_cast<V*>(vx2 + i * ny + j0));
            if (i == 2 && h.send_x[0]) st_remote(reinterpret_cast<V*>(h.send_x[0]) + j0 / VJ, vxo, h.plain_stores);
            if (i == nx - 2 && h.send_x[1]) st_remote(reinterpret_cast<V*>(h.send_x[1]) + j0 / VJ, vxo, h.plain_stores);
            if (j0 == 0 && h.nb_y[0]) {  // column 0 is the y-low neighbour's to store
#pragma unroll
              for (int e = 1; e < VJ; ++e) vy2[i * sy + e] = vyo[e];
            } else {
              *reinterpret_cast<VU*>(vy2 + i * sy + j0) = vyo;
            }
            const int64_t r2 = 2 - j0, rn = ny - 2 - j0;  // element of column 2 / ny-2 in this lane
            if (h.send_y[0] && r2 >= 0 && r2 < VJ) st_remote(reinterpret_cast<T*>(h.send_y[0]) + i * sy, vyo[r2], h.plain_stores);
            if (h.send_y[1] && rn >= 0 && rn < VJ) st_remote(reinterpret_cast<T*>(h.send_y[1]) + i * sy, vyo[rn], h.plain_stores);
          } else {
            __builtin_nontemporal_store(vxo, reinterpret_cast<V*>(vx2 + i * ny + j0));
            *reinterpret_cast<VU*>(vy2 + i * sy + j0) = vyo;
          }
        } else if (last) {
          if (!FEAT || !h.nb_y[1]) vy2[i * sy + ny] = vy_h[0];
        }
      }
      vx_i = vx_n;
      p2_prev = pc;
      vy_h = vy_h1;
      vx_n = vx_n1;
      pp = pp1;
    } else if (own && cells) {  // i == nx: the last x-faces are boundary faces
      if (!FEAT || !h.nb_x[1]) *reinterpret_cast<V*>(vx2 + i * ny + j0) = vx_i;
    }
  }
}

// Does the wave of segment `seg` / rows [i0, i1) run the exchange form? Rows
// 0..2 and nx-2..nx (x faces and sends), segment 0 (columns 0..2) and the
// segments holding columns ny-2..ny (they may straddle the last two). Host
// and device use the same rule (the in-kernel step sync counts these waves).
__host__ __device__ inline bool vmarch_feature_rows(int64_t i0, int64_t i1, int64_t nx) {
  return i0 <= 2 || i1 > nx - 2;
}
__host__ __device__ inline bool vmarch_feature_seg(int64_t seg, int64_t ny, int64_t ownv) {
  return seg == 0 || seg >= (ny - 2) / ownv;
}
__host__ __device__ inline bool vmarch_feature(int64_t seg, int64_t i0, int64_t i1, int64_t nx, int64_t ny,
                                               int64_t ownv) {
  return vmarch_feature_seg(seg, ny, ownv) || vmarch_feature_rows(i0, i1, nx);
}

template <typename T, int VJ, bool FUSED>
__global__ void __launch_bounds__(64 * WAVES) acoustic2d_vmarch_kernel(AcousticArgs a, int64_t ch,
                                                                     AcousticHalo h) {
  constexpr int64_t OWNV = 62 * VJ;
  const int64_t wave = static_cast<int64_t>(blockIdx.x) * WAVES + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t nx = a.nx, ny = a.ny;
  const int64_t nseg = (ny + 1 + OWNV - 1) / OWNV;
  const int64_t seg = wave % nseg, chunk = wave / nseg;
  const int64_t i0 = chunk * ch;
  if (i0 > nx) return;  // wave-uniform
  const int64_t i1 = min(i0 + ch, nx + 1);
  if constexpr (FUSED) {
    // Only the tiles at the exchanged faces carry the exchange code; the
    // others run the plain sweep (wave-uniform branch). Exchange code merely
    // present in the hot loop costs every wave (the diffusion kernel's
    // measurement: profiles/r2_fused_spec/).
    if (vmarch_feature(seg, i0, i1, nx, ny, OWNV)) {
      const int lane = threadIdx.x & 63;
      const uint64_t c = h.sync.my_flags ? step_sync_enter(h.sync, lane) : 0;
      vmarch_rows<T, VJ, true>(a, h, seg, i0, i1);
      // System-scope remote stores acknowledged (they reached the owner's
      // memory) before the wave retires: the sync kernel that publishes the
      // arrival flags runs next on this stream, or the last exchanging wave
      // publishes them (step_sync_exit).
      if (h.sync.my_flags) step_sync_exit(h.sync, lane, c);
      else __builtin_amdgcn_s_waitcnt(0);
      return;
    }
  }
  vmarch_rows<T, VJ, false>(a, h, seg, i0, i1);
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

static int g_acoustic_variant = 2;  // 0: one thread per cell (recompute), 1: marching, 2: vector marching
static int64_t g_march_ch = 0;  // 0: the variant's default
void acoustic2d_set_variant(int v) { g_acoustic_variant = v; }
void acoustic2d_set_chunk(int64_t ch) { g_march_ch = ch > 0 ? ch : 0; }

void launch_acoustic2d(const AcousticArgs& a, hipStream_t stream) {
  if (a.nx < 1 || a.ny < 1) fail("acoustic2d: empty grid");
  if (a.elem_bytes != 4 && a.elem_bytes != 8)
    fail("acoustic2d: element size must be 4 or 8 bytes (got ", a.elem_bytes, ")");
  constexpr int VJ4 = 4, VJ8 = 2;  // 16 B per lane (f32 / f64)
  const int vj = a.elem_bytes == 4 ? VJ4 : VJ8;
  if (g_acoustic_variant == 2 && a.ny % vj == 0 && a.ny >= 2 * vj) {
    const int64_t ch = g_march_ch > 0 ? g_march_ch : VMARCH_CH;
    const int64_t nseg = (a.ny + 1 + 62 * vj - 1) / (62 * vj), nch = (a.nx + 1 + ch - 1) / ch;
    const int64_t waves = nseg * nch;
    const dim3 grid(static_cast<unsigned>((waves + WAVES - 1) / WAVES));
    const AcousticHalo none{};
    if (a.elem_bytes == 8)
      hipLaunchKernelGGL((acoustic2d_vmarch_kernel<double, VJ8, false>), grid, dim3(64 * WAVES), 0, stream, a, ch,
                         none);
    else
      hipLaunchKernelGGL((acoustic2d_vmarch_kernel<float, VJ4, false>), grid, dim3(64 * WAVES), 0, stream, a, ch,
                         none);
  } else if (g_acoustic_variant >= 1) {
    const int64_t ch = g_march_ch > 0 ? g_march_ch : MARCH_CH;
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

void launch_acoustic2d_fused(const AcousticArgs& a, const AcousticHalo& h, hipStream_t stream) {
  if (a.elem_bytes != 4 && a.elem_bytes != 8)
    fail("acoustic2d (fused halo): element size must be 4 or 8 bytes (got ", a.elem_bytes, ")");
  const int vj = a.elem_bytes == 4 ? 4 : 2;
  if (a.ny % vj != 0 || a.ny < 2 * vj || a.nx < 5 || a.ny < 5)
    fail("acoustic2d (fused halo): needs ny % ", vj, " == 0 and nx, ny >= 5");
  if (h.sync.my_flags && (h.sync.n_peers < 1 || h.sync.n_peers > 4))
    fail("acoustic2d (fused halo): in-kernel sync needs 1..4 peers (got ", h.sync.n_peers, ")");
  const int64_t ch = g_march_ch > 0 ? g_march_ch : VMARCH_CH;
  const int64_t ownv = 62 * vj;
  const int64_t nseg = (a.ny + 1 + ownv - 1) / ownv, nch = (a.nx + 1 + ch - 1) / ch;
  // exchanging waves (the in-kernel step sync waits for this many to count)
  int64_t fseg = 0, feat = 0;
  for (int64_t sg = 0; sg < nseg; ++sg) fseg += vmarch_feature_seg(sg, a.ny, ownv) ? 1 : 0;
  for (int64_t c = 0; c < nch; ++c)
    feat += vmarch_feature_rows(c * ch, std::min(c * ch + ch, a.nx + 1), a.nx) ? nseg : fseg;
  AcousticHalo hh = h;
  hh.sync.feat_waves = feat;
  if (feat < 1) hh.sync.my_flags = nullptr;  // unreachable (rows 0..2 always exchange); keep the sync kernel form
  const dim3 grid(static_cast<unsigned>((nseg * nch + WAVES - 1) / WAVES));
  if (a.elem_bytes == 8)
    hipLaunchKernelGGL((acoustic2d_vmarch_kernel<double, 2, true>), grid, dim3(64 * WAVES), 0, stream, a, ch, hh);
  else
    hipLaunchKernelGGL((acoustic2d_vmarch_kernel<float, 4, true>), grid, dim3(64 * WAVES), 0, stream, a, ch, hh);
  IGG_HIP_CHECK(hipGetLastError());
}

void host_acoustic2d(const AcousticArgs& a) {
  if (a.elem_bytes == 8) host_typed<double>(a);
  else if (a.elem_bytes == 4) host_typed<float>(a);
  else fail("acoustic2d: element size must be 4 or 8 bytes (got ", a.elem_bytes, ")");
}

}  // namespace igg
