#pragma once
// The plain x-march of one wave (2.5-D blocking, vector lanes) for the waves
// of the restrict-form / fused kernels that exchange nothing (fused_impl.hpp
// hx_sweep). It is the loop of the plain vector kernel
// (stencil_kernels.hip diffusion3d_vkernel), kept as a separate copy on
// purpose: compiled through this function the vector kernel itself got a
// different schedule (f32 tiling 14 1.2 % slower, f64 tiling 14 with whole-line
// z stores spilling 8 VGPRs), so it keeps its own loop.
//
// Round 6: the restrict form's own plain loop ran 15 % more VALU than this one
// for the same tiling. Its addresses were 64-bit per lane (v_lshl_add_u64,
// v_mov_b64), where this loop uses a uniform base + 32-bit lane offset.
// Memory traffic was the same (TCC_EA0_RDREQ 18.0 vs 18.2 M per launch).
// That cost tiling 11 2 % per step on fast pages (profiles/r6_vsweep/), so
// the restrict-form plain waves now run this loop.
//
// Each lane owns VZ consecutive z points, so a wave covers a 64*VZ-point
// contiguous row segment with one vector load per array. Tiles are aligned to
// row starts, so every vector access is naturally aligned (n2 % VZ == 0). The
// z neighbours come from the lane's own vector and its two lane neighbours
// (__shfl up/down); only the two segment-edge values are loaded (uniform
// address). Row bases are wave-uniform, so the per-lane address is a 32-bit
// offset. PF: prefetch plane x+2 of T and x+1 of Cp while computing plane x.
// NT: non-temporal stores of T2 (streamed once).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "igg/devmath.hpp"

namespace igg {

template <typename T, int VZ>
struct SweepVec {
  typedef T type __attribute__((ext_vector_type(VZ)));
};

template <typename T, int VZ>
__device__ __forceinline__ typename SweepVec<T, VZ>::type sweep_load(const T* p) {
  return *reinterpret_cast<const typename SweepVec<T, VZ>::type*>(p);
}

// One wave's sweep of rows y0 .. y0+nv-1 (nv <= RY) of the z segment starting
// at zt, planes xs .. xe-1, over the box z range [lo2, hi2).
// HZ: the whole-line z-edge store form (DiffusionArgs::halo_z). A z-edge lane
// stores its whole vector, with t's value in the halo element, instead of a
// partial line. That is only for a box spanning the whole inner z range. With
// SIDES, zh_lo / zh_hi allow it per z side (the fused kernel: a side whose halo
// column a neighbour writes keeps partial stores); without, both sides.
template <typename T, int RY, int VZ, bool PF, bool NT, bool HZ, bool SIDES = false>
__device__ __forceinline__ void v_sweep(T* __restrict__ t2, const T* __restrict__ t, const T* __restrict__ cpp,
                                        int64_t n0, int64_t n1, int64_t n2, int64_t xs, int64_t xe, int64_t y0,
                                        int nv, int64_t zt, int64_t lo2, int64_t hi2, T rdx2, T rdy2, T rdz2,
                                        T dtlam, bool zh_lo = true, bool zh_hi = true) {
  using V = typename SweepVec<T, VZ>::type;
  const int lane = threadIdx.x & 63;
  const int64_t s1 = n2, s0 = n1 * n2;
  const int64_t z0 = zt + lane * VZ;
  // Lanes whose vector holds no box point alias the first/last vector that does,
  // so a thin box (a single send plane) touches only the lines it needs.
  const int64_t zlo_v = (lo2 / VZ) * VZ, zhi_v = ((hi2 - 1) / VZ) * VZ;
  const int64_t zc = min(max(z0, zlo_v), zhi_v);
  const int zl = static_cast<int>(zc - zt);  // per-lane offset in the tile
  const bool lane_full = z0 >= lo2 && z0 + VZ <= hi2;
  bool zfull = HZ && lo2 == 1 && hi2 == n2 - 1 && zc == z0 && z0 + VZ <= n2;
  if constexpr (HZ && SIDES) zfull = zfull && ((z0 < lo2 && zh_lo) || (z0 + VZ > hi2 && zh_hi));
  // z-neighbours come from lane neighbours except where that neighbour lane is
  // clamped (or outside the wave): those lanes load their edge value directly.
  const bool load_prev = lane == 0 || z0 - VZ < zlo_v;
  const bool load_next = lane == 63 || z0 + VZ > zhi_v;
  const int zpi = static_cast<int>(max<int64_t>(zc - 1, 0) - zt);
  const int zni = static_cast<int>(min<int64_t>(zc + VZ, n2 - 1) - zt);

  int64_t rowb[RY];  // wave-uniform row bases (element index of the tile origin)
#pragma unroll
  for (int r = 0; r < RY; ++r) rowb[r] = (y0 + min(r, nv - 1)) * s1 + zt;
  const int64_t rowm = (y0 - 1) * s1 + zt, rowp = (y0 + nv) * s1 + zt;

  V tm[RY], tc[RY], tp[RY], cp[RY];
#pragma unroll
  for (int r = 0; r < RY; ++r) {
    tm[r] = sweep_load<T, VZ>(t + (xs - 1) * s0 + rowb[r] + zl);
    tc[r] = sweep_load<T, VZ>(t + xs * s0 + rowb[r] + zl);
    tp[r] = sweep_load<T, VZ>(t + (xs + 1) * s0 + rowb[r] + zl);
    cp[r] = sweep_load<T, VZ>(cpp + xs * s0 + rowb[r] + zl);
  }
  for (int64_t x = xs; x < xe; ++x) {
    const int64_t off = x * s0;
    V tn[RY], cpn[RY];
    if (PF) {
      const int64_t xn = min(x + 2, n0 - 1), xc = min(x + 1, xe - 1);
#pragma unroll
      for (int r = 0; r < RY; ++r) {
        tn[r] = sweep_load<T, VZ>(t + xn * s0 + rowb[r] + zl);
        cpn[r] = sweep_load<T, VZ>(cpp + xc * s0 + rowb[r] + zl);
      }
    }
    const V ym = sweep_load<T, VZ>(t + off + rowm + zl);
    const V yp = sweep_load<T, VZ>(t + off + rowp + zl);
    T em[RY], ep[RY];
#pragma unroll
    for (int r = 0; r < RY; ++r) {
      em[r] = load_prev ? t[off + rowb[r] + zpi] : T(0);
      ep[r] = load_next ? t[off + rowb[r] + zni] : T(0);
    }
#pragma unroll
    for (int r = 0; r < RY; ++r) {
      const V& c = tc[r];
      const V& yv = (r == 0) ? ym : tc[r > 0 ? r - 1 : 0];
      const V& yn = (r + 1 < nv) ? tc[(r + 1 < RY) ? r + 1 : r] : yp;
      T prev = __shfl_up(c[VZ - 1], 1);
      T next = __shfl_down(c[0], 1);
      if (load_prev) prev = em[r];
      if (load_next) next = ep[r];
      V out;
#pragma unroll
      for (int e = 0; e < VZ; ++e) {
        const T zm = e == 0 ? prev : c[e > 0 ? e - 1 : 0];
        const T zp = e == VZ - 1 ? next : c[e + 1 < VZ ? e + 1 : e];
        out[e] = diffusion_point(c[e], tm[r][e], tp[r][e], yv[e], yn[e], zm, zp, cp[r][e], rdx2, rdy2, rdz2, dtlam);
      }
      if (r < nv) {
        T* dst = t2 + off + rowb[r] + zl;
        if (lane_full) {
          if (NT) __builtin_nontemporal_store(out, reinterpret_cast<V*>(dst));
          else *reinterpret_cast<V*>(dst) = out;
        } else if (HZ && zfull) {
          // the z-edge lane of a full-z box: the halo element (z = 0 or n2-1)
          // is written with t's value, so the whole vector - and its cache
          // line - is stored instead of a partial line
          V o = out;
#pragma unroll
          for (int e = 0; e < VZ; ++e)
            if (z0 + e < lo2 || z0 + e >= hi2) o[e] = c[e];
          if (NT) __builtin_nontemporal_store(o, reinterpret_cast<V*>(dst));
          else *reinterpret_cast<V*>(dst) = o;
        } else {
#pragma unroll
          for (int e = 0; e < VZ; ++e)
            if (z0 + e >= lo2 && z0 + e < hi2 && zc == z0) dst[e] = out[e];
        }
      }
    }
#pragma unroll
    for (int r = 0; r < RY; ++r) {
      tm[r] = tc[r];
      tc[r] = tp[r];
      if (PF) {
        tp[r] = tn[r];
        cp[r] = cpn[r];
      }
    }
    if (!PF && x + 1 < xe) {
#pragma unroll
      for (int r = 0; r < RY; ++r) {
        tp[r] = sweep_load<T, VZ>(t + (x + 2) * s0 + rowb[r] + zl);
        cp[r] = sweep_load<T, VZ>(cpp + (x + 1) * s0 + rowb[r] + zl);
      }
    }
  }
}

}  // namespace igg
