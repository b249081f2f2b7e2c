#pragma once
// Fused halo-exchange diffusion kernel templates for gfx950 (included by the
// csrc/kernels/fused_*.hip translation units; see igg/fused.hpp).
//
// Same 2.5-D blocked, vectorised sweep as diffusion3d_vkernel (stencil_kernels.hip)
// over the inner box [1, n-1)^3, plus the exchange of the update_halo! step
// (reference: src/update_halo.jl:32-78 after examples/diffusion3D_*:42-46):
//   * receive: the face halos are read from this rank's arena regions (written
//     by the neighbours' previous step) instead of the field's halo planes -
//     dim 0 by redirecting the plane base of x=0 / n0-1, dim 1 by redirecting
//     the base of the y=0 / n1-1 rows, dim 2 element-wise (below);
//   * send: the values of the planes x=1/n0-2, rows y=1/n1-2 and elements
//     z=1/n2-2 are stored into the receivers' arenas (IPC-mapped
//     peer memory: the stores travel over xGMI while the sweep goes on).
// Every pointer is a separate __restrict__ kernel argument so the compiler
// knows the remote stores never alias the T/Cp loads and keeps the plain
// kernel's load schedule. The z edge (one element per row, in lane 0 of the
// first segment and lane zh of the last) moves lane-distributed: the halo
// values of the RY rows are fetched one x step ahead by lanes r / 32+r with
// ONE load instruction and patched into the edge lane with readlane; the
// send values are gathered the same way and leave with ONE store per step.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <vector>

#include "igg/devmath.hpp"
#include "igg/devsync.hpp"
#include "igg/stencil.hpp"
#include "igg/sysstore.hpp"
#include "igg/vsweep.hpp"


namespace igg {

// Diagnostics state set by fused_debug() and copied into the next launches
// (defined in fused_kernels.hip).
extern int64_t* g_hx_stamps;
extern int g_hx_force_sel;

// Fused launches by tiling family and element type, one translation unit each
// so they compile in parallel (the tiling-9 family with its side-only z forms
// alone took 7.7 min as one unit of both types): fused_t0_<dt>.hip (variants
// 0, 50), fused_t11_<dt>.hip (40, 42), fused_t9_<dt>.hip (9),
// fused_t14_<dt>.hip (14, 44); the bodies are in igg/fused_families.hpp, each
// unit instantiates one (family, type). Return false for a variant not in the
// family.
template <typename T>
bool fused_family_t0(const DiffusionArgs& d, const HaloIOArgs& io, int v, int mode, hipStream_t s);
template <typename T>
bool fused_family_t11(const DiffusionArgs& d, const HaloIOArgs& io, int v, int mode, hipStream_t s);
template <typename T>
bool fused_family_t9(const DiffusionArgs& d, const HaloIOArgs& io, int v, int mode, hipStream_t s);
template <typename T>
bool fused_family_t14(const DiffusionArgs& d, const HaloIOArgs& io, int v, int mode, hipStream_t s);

namespace {

template <typename T, int VZ>
struct Vec {
  typedef T type __attribute__((ext_vector_type(VZ)));
};

template <typename T, int VZ>
__device__ __forceinline__ typename Vec<T, VZ>::type vld(const T* p) {
  return *reinterpret_cast<const typename Vec<T, VZ>::type*>(p);
}

template <typename T>
__device__ __forceinline__ T lane_read(T v, int l) {
  if constexpr (sizeof(T) == 8) {
    const int2 p = __builtin_bit_cast(int2, v);
    return __builtin_bit_cast(T, make_int2(__builtin_amdgcn_readlane(p.x, l), __builtin_amdgcn_readlane(p.y, l)));
  } else {
    return __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
  }
}

// DPP lane moves inside a 16-lane row (gfx9 row_shl / row_shr; ZDPP below):
// lane i takes lane i + r (shl) or i - r (shr) of its own 16-lane row; lanes
// whose source lies outside the row read 0 (bound_ctrl). r is a constant after
// the row loop is unrolled (the switch folds); r = 0 is the identity.
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, true);
}

template <typename T, int CTRL>
__device__ __forceinline__ T dpp_t(T v) {
  if constexpr (sizeof(T) == 8) {
    const int2 p = __builtin_bit_cast(int2, v);
    return __builtin_bit_cast(T, make_int2(dpp_i<CTRL>(p.x), dpp_i<CTRL>(p.y)));
  } else {
    return __builtin_bit_cast(T, dpp_i<CTRL>(__builtin_bit_cast(int, v)));
  }
}

#define IGG_DPP_ROW_CASES(BASE)                                                                                    \
  case 1: return dpp_t<T, BASE + 1>(v);   case 2: return dpp_t<T, BASE + 2>(v);   case 3: return dpp_t<T, BASE + 3>(v);   \
  case 4: return dpp_t<T, BASE + 4>(v);   case 5: return dpp_t<T, BASE + 5>(v);   case 6: return dpp_t<T, BASE + 6>(v);   \
  case 7: return dpp_t<T, BASE + 7>(v);   case 8: return dpp_t<T, BASE + 8>(v);   case 9: return dpp_t<T, BASE + 9>(v);   \
  case 10: return dpp_t<T, BASE + 10>(v); case 11: return dpp_t<T, BASE + 11>(v); case 12: return dpp_t<T, BASE + 12>(v); \
  case 13: return dpp_t<T, BASE + 13>(v); case 14: return dpp_t<T, BASE + 14>(v); case 15: return dpp_t<T, BASE + 15>(v);

template <typename T>
__device__ __forceinline__ T row_shl(T v, int r) {  // lane i <- lane i + r
  switch (r) {
    IGG_DPP_ROW_CASES(0x100)
    default: return v;
  }
}

template <typename T>
__device__ __forceinline__ T row_shr(T v, int r) {  // lane i <- lane i - r
  switch (r) {
    IGG_DPP_ROW_CASES(0x110)
    default: return v;
  }
}
#undef IGG_DPP_ROW_CASES

__device__ __forceinline__ int64_t xcd_remap(int64_t b, int64_t nb) {
  const int64_t q = nb / 8, r = nb % 8, xcd = b % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
}

// Block chunk index in march order (chunks holding the x send planes first).
__device__ __forceinline__ int64_t hx_chunk(int64_t cxr, int64_t nch) {
  return (cxr == 0 || nch < 2) ? cxr : (cxr == 1 ? nch - 1 : cxr - 1);
}

template <typename T>
struct HxScal {
  int64_t n0, n1, n2, zp, zrow;  // z sends: x*zp + (y-1)*zrow (arena: zrow 1; direct: n1*n2, n2)
  int64_t ntz, nty, ch;  // z tiles, y tiles, planes per chunk
  T rdx2, rdy2, rdz2, dtlam;
  // Diagnostics (fused_debug): per-wave {class, start, end, cu} stamps
  // (wall_clock64 ticks) into `stamps` (4 int64 per wave) when non-null;
  // force_sel >= 0 runs every wave with that feature class.
  int64_t* stamps;
  int force_sel;
  int peel;  // send mode bit 8: sweep the exchanged x planes of a chunk separately (kernel below)
  // Send mode bit 32: dispatch the exchanging z-edge tiles first (hx_tile).
  // order_lo: z tile 0 exchanges; order_hi: the z tile holding n2-VZ (index
  // tz_hi) exchanges.
  int order, order_lo, order_hi;
  int64_t tz_hi;
  // DiffusionArgs::halo_z per z side: the z-edge lane stores its whole vector
  // (its halo element - t's value, or the received one - into t2's halo) as
  // one full-line store (launch_hx decides per side).
  int zh_lo, zh_hi;
  StepSync sync;  // in-kernel step synchronisation (put.hpp; my_flags null: a sync kernel follows)
};

// Tile (z tile, y tile, x chunk) of block `bid` of `nblk`. Default: z tiles
// fastest, so the z tiles of one row-chunk are neighbours in dispatch order
// and (xcd_remap) on one XCD's L2; the x chunks holding the exchanged planes
// come first (hx_chunk). With a.order (send mode bit 32) the z-EDGE tiles of an
// exchanging z side are dispatched first - longest work first. The z-edge
// waves carry the z sends (+8-11 % per wave, profiles/r3_waves/); with the
// default order they are spread evenly over the launch, so at 2 residency
// rounds every other slot runs one heavy and one light wave and the kernel
// takes (1 + 0.106)/1 of the plain time however few of them there are (a
// 2x2x2 corner rank: a quarter). Dispatched first, they run in the first
// round(s) while later rounds' light waves fill the slots they leave: with
// enough rounds the kernel approaches the average instead of the maximum.
// Scheduling only: the results are unchanged.
template <typename T>
struct HxTile {
  int64_t tz, ty, cx;
};

template <typename T>
__device__ __forceinline__ HxTile<T> hx_tile(const HxScal<T>& a, int64_t bid, int64_t nblk) {
  const int64_t nch = (a.n0 - 2 + a.ch - 1) / a.ch;
  if (a.order && (a.order_lo || a.order_hi)) {
    const int64_t R = a.nty * nch;  // row-chunks per z tile
    const int64_t tzi = bid / R;
    const int64_t rc = xcd_remap(bid - tzi * R, R);
    const int nh = (a.order_lo ? 1 : 0) + ((a.order_hi && !(a.order_lo && a.tz_hi == 0)) ? 1 : 0);
    int64_t tz;
    if (tzi < nh) {
      tz = (tzi == 0 && a.order_lo) ? 0 : a.tz_hi;
    } else {
      tz = tzi - nh + (a.order_lo ? 1 : 0);  // the light tiles in ascending order
      if (a.order_hi && a.tz_hi != 0 && tz >= a.tz_hi) ++tz;
    }
    return {tz, rc % a.nty, hx_chunk(rc / a.nty, nch)};
  }
  const int64_t b = xcd_remap(bid, nblk);
  const int64_t rest = b / a.ntz;
  return {b % a.ntz, rest % a.nty, hx_chunk(rest / a.nty, nch)};
}

// Writer side of the cross-device hand-off: every store into peer memory
// (arena regions, or the neighbour's field with direct z) is a system-scope
// store, st_sys (igg/sysstore.hpp). (A plain store + per-wave buffer_wbl2
// sc0 sc1 also works but writes back the XCD's whole L2 from every storing
// wave: +14 % per step, profiles/r3_coherence/.)

// FEAT bits (compile-time exchange features): 1 x-in, 2 y-in, 4 z-in, 8 z-out,
// 64 x-out, 128 y-out; 256 = non-temporal Cp loads (plain variants); 512 =
// lane-distributed z-segment edge loads (plain variants, below); 1024 = one
// workgroup per CU (launch); 2048 = no per-wave specialisation (kernel below);
// 4096 = z edge values staged through LDS instead of v_readlane; HZ (262144) =
// the whole-line z-edge store form (DiffusionArgs::halo_z). 207 = the full
// exchange, 0 = the plain update (variants 21+); other subsets served the cost
// bisect (profiles/r1_fused/feature_bisect_*).
constexpr int HZ = 262144;
// Side-only z forms (chosen per wave by diffusion3d_hx_kernel when the tiling
// has ZSIDES): a z-edge wave holds one z edge unless a row fits in one wave,
// so the other side's per-row readlanes and selects are compiled out (ZLO:
// only z = 0 / 1 exchange code, ZHI: only z = n2-1 / n2-2). Opt-in per tiling:
// the extra sweep instantiations made tilings 11/14 (fused 40/42/44) 4 %
// slower in every shape, tiling 9 1.2 % faster at a 2x2x2 corner
// (profiles/r4_shapes/, pass 4).
constexpr int ZLO = 524288, ZHI = 1048576, ZSIDES = 2097152;
// ZDPP (round 6): the z-edge lane moves as DPP row shifts
// instead of v_readlane + select. The lane-distributed rows sit where one
// shift reaches the edge lane within its 16-lane DPP row: low edge row r in
// lane r (lane 0 <- lane r: row_shl r; send: lane r <- lane 0: row_shr r),
// high edge row r in lane zh - r (lane zh <- lane zh - r: row_shr r; send:
// lane zh - r <- lane zh: row_shl r). No SGPR round trip per row. Needs
// RY <= 16, one z edge per wave, and zh % 16 >= RY - 1 (launch_mode checks;
// otherwise the readlane form runs).
constexpr int ZDPP = 4194304;
// OCC2 (round 6, launch only): at most 2 workgroups per CU, enforced with an
// unused dynamic LDS allocation as FEAT 1024 does for one; the grid's chunks are
// sized for that residency. f32 tiling 0 gains 2.5 % (plain variant 44).
constexpr int OCC2 = 8388608;

template <typename T, int BY, int RY, int VZ, bool PF, int BZ, bool DF, int FEAT>
__device__ __forceinline__ void
hx_sweep(T* __restrict__ t2, const T* __restrict__ t, const T* __restrict__ cpp,
         const T* __restrict__ xi0, const T* __restrict__ xi1, const T* __restrict__ yi0,
         const T* __restrict__ yi1, const T* __restrict__ zi0, const T* __restrict__ zi1,
         T* __restrict__ xo0, T* __restrict__ xo1, T* __restrict__ yo0, T* __restrict__ yo1,
         T* __restrict__ zo0, T* __restrict__ zo1, const HxScal<T>& a, int64_t clip_lo = 0,
         int64_t clip_hi = INT64_MAX) {
  using V = typename Vec<T, VZ>::type;
  constexpr int W = 64 * VZ * BZ;
  // FEAT 16384 / 32768 / 65536 / 131072 are measurement-only forms (rounds
  // 1-2, not adopted): compiled only with build.py --probes (IGG_PROBES).
#ifndef IGG_PROBES
  static_assert((FEAT & (16384 | 32768 | 65536 | 131072)) == 0, "measurement-only FEAT bits need IGG_PROBES");
#endif
  // FEAT 65536 (RV, plain sweeps only): reversed march - chunks from the top x
  // down and each chunk's planes from high x to low - for every other step of
  // the ping-pong loop, so a step starts on the planes the previous (forward)
  // step touched last, which may still sit in the memory-side Infinity Cache.
  // The x term is summed in the forward order: results are bitwise identical.
  constexpr bool RV = (FEAT & 65536) != 0;
  static_assert(!RV || (FEAT & (1 | 2 | 4 | 8 | 64 | 128 | 4096 | 8192)) == 0, "RV: plain sweeps only");
  constexpr int64_t DX = RV ? -1 : 1;
  // Chunks holding the x send planes run first (order 0, last, 1, 2, ...): the
  // plane x=n0-2 is computed in the last step of the last chunk, so with >= 2
  // residency rounds its remote stores drain while later rounds compute
  // instead of at the kernel's tail. Scheduling only: results are unchanged.
  // (hx_tile; send mode bit 32 also puts the z-edge tiles first.)
  const int64_t nch = (a.n0 - 2 + a.ch - 1) / a.ch;
  const HxTile<T> tile = hx_tile(a, blockIdx.x, gridDim.x);
  const int64_t tz = tile.tz, ty = tile.ty;
  int64_t cx = tile.cx;
  if constexpr (RV) {  // reversed march (probe form): chunks from the top, default order
    const int64_t b = xcd_remap(blockIdx.x, gridDim.x);
    cx = nch - 1 - (b / a.ntz) / a.nty;
  }
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wz = wid % BZ, wy = wid / BZ;
  const int64_t n0 = a.n0, n1 = a.n1, n2 = a.n2, s0 = n1 * n2;
  const int64_t zt = tz * W + wz * (64 * VZ);
  const int64_t y0 = 1 + ty * (BY * RY) + wy * RY;
  // [clip_lo, clip_hi): the part of the chunk this call sweeps (the kernel
  // peels the exchanged x planes off a chunk: see diffusion3d_hx_kernel)
  const int64_t xs = max<int64_t>(1 + cx * a.ch, clip_lo);
  const int64_t xe = min(min<int64_t>(1 + cx * a.ch + a.ch, n0 - 1), clip_hi);
  const int nv = static_cast<int>(min<int64_t>(RY, n1 - 1 - y0));
  if (nv <= 0 || xs >= xe) return;
  const int64_t hi2 = n2 - 1;
  if (zt >= hi2) return;
  // A wave that exchanges nothing runs the plain vector march (igg/vsweep.hpp):
  // 15 % less VALU than this loop's plain form, 2 % per step for tiling 11
  // (profiles/r6_vsweep/). FEAT 512 (lane-distributed edge loads) only chose
  // how this loop's plain form fetched the segment edges: ignored there. Not
  // for 8-wave workgroups (tiling 43's full-row tiles): at <= 256 VGPRs the
  // vector march spills (4 VGPRs, 20 B scratch) and ran 4.5 % slower. Not for
  // the side-only z forms (tiling 9, ZSIDES): there the 2x2x2 corner step got
  // 0.6 % slower (same-box A/B, profiles/r6_vsweep/). f64 only: the f32
  // restrict-form plain variants ran 2.5-6 % slower relative to the vector
  // kernel with it (1024^3).
  constexpr int NOT_PLAIN =
      1 | 2 | 4 | 8 | 64 | 128 | 256 | 4096 | 8192 | 16384 | 32768 | 65536 | 131072 | ZSIDES;
  if constexpr ((FEAT & NOT_PLAIN) == 0 && BY * BZ <= 4 && sizeof(T) == 8) {
    v_sweep<T, RY, VZ, PF, true, (FEAT & HZ) != 0, true>(t2, t, cpp, n0, n1, n2, xs, xe, y0, nv, zt, 1, hi2, a.rdx2,
                                                         a.rdy2, a.rdz2, a.dtlam, a.zh_lo != 0, a.zh_hi != 0);
    return;
  }
  const int64_t z0 = zt + lane * VZ;
  const int64_t zhi_v = ((hi2 - 1) / VZ) * VZ;
  const int64_t zc = min(z0, zhi_v);
  const int zl = static_cast<int>(zc - zt);
  const bool lane_full = z0 >= 1 && z0 + VZ <= hi2;
  // Lanes past the box alias the last valid vector (zc < z0) and compute
  // garbage there: they must not store (remote whole-vector stores included).
  const bool zown = zc == z0;
  const bool zfull = (FEAT & HZ) != 0 && zown && ((z0 == 0 && a.zh_lo) || (z0 + VZ == n2 && a.zh_hi));
  const bool load_prev = lane == 0;
  const bool load_next = lane == 63 || z0 + VZ > zhi_v;
  const int zpi = static_cast<int>(max<int64_t>(zc - 1, 0) - zt);
  const int zni = static_cast<int>(min<int64_t>(zc + VZ, n2 - 1) - zt);
  // FEAT 512: the z neighbours across the segment's ends (lane 0's prev, the
  // load_next lanes' next: one uniform element per row each) are fetched by
  // lanes r / 32+r with ONE load per x step, one step ahead, and moved with
  // readlane - instead of 2*RY single-lane loads held in 2*RY registers.
  static_assert(!(FEAT & 512) || RY <= 32, "FEAT 512: at most 32 rows per wave");
  const int64_t zc63 = min<int64_t>(zt + 63 * VZ, zhi_v);
  const int zedge = lane < 32 ? static_cast<int>(max<int64_t>(zt - 1, 0) - zt)
                              : static_cast<int>(min<int64_t>(zc63 + VZ, n2 - 1) - zt);
  const int64_t rowe = (y0 + min(lane & 31, nv - 1)) * n2 + zt + zedge;

  int64_t rowb[RY];
#pragma unroll
  for (int r = 0; r < RY; ++r) rowb[r] = (y0 + min(r, nv - 1)) * n2 + zt;
  // y-neighbour rows outside the wave (dim-1 halo rows come from the arena).
  const T* ymb = t + (y0 - 1) * n2 + zt;
  const T* ypb = t + (y0 + nv) * n2 + zt;
  int64_t yms = s0, yps = s0;
  if ((FEAT & 2) && y0 == 1 && yi0) { ymb = yi0 + zt; yms = n2; }
  if ((FEAT & 2) && y0 + nv == n1 - 1 && yi1) { ypb = yi1 + zt; yps = n2; }
  // y send rows of this wave.
  T* const yrow0 = ((FEAT & 128) && y0 == 1 && yo0) ? yo0 + zt : nullptr;
  int ry1 = static_cast<int>(n1 - 2 - y0);
  T* const yrow1 = ((FEAT & 128) && ry1 >= 0 && ry1 < nv && yo1) ? yo1 + zt : nullptr;
  if (!yrow1) ry1 = -1;
  // z edges of this wave: low edge in lane 0 (element 0 = halo z=0, element
  // 1 = send z=1), high edge in lane zh (element VZ-1 = halo, VZ-2 = send).
  const bool has_lo = zt == 0, has_hi = zt <= n2 - VZ && n2 - VZ < zt + 64 * VZ;
  // readfirstlane: the compiler must see zh as uniform, or every readlane
  // with it becomes a waterfall loop draining vmcnt (measured +27 % per step).
  const int zh = __builtin_amdgcn_readfirstlane(static_cast<int>((n2 - VZ - zt) / VZ));
  constexpr bool SLO = (FEAT & ZHI) == 0, SHI = (FEAT & ZLO) == 0;  // z sides this form handles
  constexpr bool ZD = (FEAT & ZDPP) != 0;
  static_assert(!ZD || (RY <= 16 && (FEAT & (4096 | 8192)) == 0), "ZDPP: RY <= 16, not with the LDS / edge-lane forms");
  const bool zin_lo = SLO && (FEAT & 4) && has_lo && zi0, zin_hi = SHI && (FEAT & 4) && has_hi && zi1;
  const bool zout_lo = SLO && (FEAT & 8) && has_lo && zo0, zout_hi = SHI && (FEAT & 8) && has_hi && zo1;
  const bool zin = zin_lo || zin_hi, zout = zout_lo || zout_hi;
  // halo_z (FEAT HZ): this wave holds a z edge whose halo element it may write
  const bool hz_wave = (FEAT & HZ) != 0 && ((has_lo && a.zh_lo) || (has_hi && a.zh_hi));
  const int rl = lane & 31;
  // Lane-distributed z values: row r of the low edge in lane r, of the high
  // edge in lane 32+r (rows < nv); ZDPP: in lane zh - r.
  const int rh = ZD ? zh - lane : rl;  // row of a high-edge lane
  const bool lo_l = lane < 32 && rl < nv, hi_l = ZD ? (rh >= 0 && rh < nv) : (lane >= 32 && rl < nv);
  // Every lane loads (lanes without a row of their own read a valid dummy in
  // the same region): a load under a per-lane condition would be a divergent
  // branch around a load in the hot loop, which costs the loop its prefetch.
  const T* zsrc = lo_l && zin_lo ? zi0 + (y0 - 1) + rl
                                 : (hi_l && zin_hi ? zi1 + (y0 - 1) + rh
                                                   : (zin_lo ? zi0 : zi1) + (y0 - 1));
  const int64_t zro = ((y0 - 1) + (hi_l && !lo_l ? rh : rl)) * a.zrow;
  T* zdst = lo_l && zout_lo ? zo0 + zro : (hi_l && zout_hi ? zo1 + zro : nullptr);
  const bool remote = zout || yrow0 || yrow1 || (xs == 1 && xo0) || (xe == n0 - 1 && xo1);
  T znext = T(0), zv = T(0);
  if (zin) znext = zsrc[xs * a.zp];
  // FEAT 4096: the z edge values move between the edge lane and the
  // lane-distributed row layout through 4*RY LDS slots of this wave (in/out x
  // lo/hi) instead of v_readlane (whose SGPR result feeds VALU with wait states
  // that one wave per SIMD cannot hide: profiles/r2_fused_spec/).
  T* zs = nullptr;
  if constexpr ((FEAT & 4096) != 0) {
    __shared__ T zslots[BY * BZ * 4 * RY];
    zs = zslots + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * (4 * RY);
  }
  // FEAT 8192 (ZE): the z edge without per-row cross-lane operations. The
  // halo values of the wave's rows are read by uniform-address loads (every
  // lane the same address: one request per row, or scalar loads), one x step
  // ahead, and selected into the edge lane; the edge lane's send values are
  // kept in registers over the row loop and transposed once per step through
  // RY LDS slots of this wave to the lane-distributed layout of the (single,
  // coalesced) remote store. A wave with both z edges (n2 <= 64*VZ + VZ) is
  // not supported by this form (launch_mode falls back).
  constexpr bool ZE = (FEAT & 8192) != 0;
  const T* zi_base = zin_lo ? zi0 : zi1;
  T zi_cur[ZE ? RY : 1], zi_nxt[ZE ? RY : 1];
  T* zo_lds = nullptr;
  if constexpr (ZE) {
    __shared__ T zo_slots[BY * BZ * RY];
    zo_lds = zo_slots + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * RY;
#pragma unroll
    for (int r = 0; r < RY; ++r) {
      zi_cur[r] = T(0);
      zi_nxt[r] = zin ? zi_base[xs * a.zp + (y0 - 1) + min(r, nv - 1)] : T(0);
    }
  }
  const bool ze_lo = zin_lo && lane == 0, ze_hi = zin_hi && lane == zh;
  // Deferred sends (DF): the y row / z values of step x leave after the loads
  // of step x+1 were issued, so their acknowledgement never gates those loads.
  V ysend;
  T* ysend_dst = nullptr;
  T* zsend_dst = nullptr;

  auto plane = [&](int64_t X) -> const T* {
    if constexpr ((FEAT & 1) != 0) {
      if (X == 0 && xi0) return xi0;
      if (X == n0 - 1 && xi1) return xi1;
    }
    return t + X * s0;
  };
  // Cp is streamed once (no reuse): FEAT bit 256 loads it non-temporally so it
  // does not displace the T lines that neighbouring waves re-read (y/z halos).
  auto ldc = [&](const T* p) -> V {
    if constexpr ((FEAT & 256) != 0) return __builtin_nontemporal_load(reinterpret_cast<const V*>(p));
    return vld<T, VZ>(p);
  };
  // tm / tp: the planes behind / ahead of the march (x - DX / x + DX)
  const int64_t xf = RV ? xe - 1 : xs, len = xe - xs;
  V tm[RY], tc[RY], tp[RY], cp[RY];
#pragma unroll
  for (int r = 0; r < RY; ++r) {
    tm[r] = vld<T, VZ>(plane(xf - DX) + rowb[r] + zl);
    tc[r] = vld<T, VZ>(plane(xf) + rowb[r] + zl);
    tp[r] = vld<T, VZ>(plane(xf + DX) + rowb[r] + zl);
    cp[r] = ldc(cpp + xf * s0 + rowb[r] + zl);
  }
  T evn = T(0);
  if constexpr ((FEAT & 512) != 0 && (FEAT & 16384) == 0) evn = t[xf * s0 + rowe];
  int64_t x = xf;
  for (int64_t i = 0; i < len; ++i, x += DX) {
    const int64_t off = x * s0;
    T evc = T(0);
    if constexpr ((FEAT & 512) != 0) {
      evc = evn;
      if constexpr ((FEAT & 16384) == 0) {
        if (i + 1 < len) evn = t[off + DX * s0 + rowe];
      }
#ifdef IGG_PROBES
      // FEAT 16384 / 32768: timing probes (results WRONG): skip the z-segment
      // edge loads / the y-halo row loads, to price the tile-edge re-fetch.
      if constexpr ((FEAT & 16384) != 0) evn = evn * T(0.5);
#endif
    }
    // z halo of plane x (fetched one step ahead), prefetch plane x+1's. (The
    // alternative of substituting it at its use measured slower for every
    // tiling: profiles/r1_fused/feature_bisect_v11_zin_alt.log.)
    T zcur = T(0);
    bool pl = false, ph = false;  // this lane patches its z=0 / z=n2-1 halo element (per row, below)
    if constexpr (ZE) {
#pragma unroll
      for (int r = 0; r < RY; ++r) zi_cur[r] = zi_nxt[r];
      if (zin && x + 1 < xe) {
#pragma unroll
        for (int r = 0; r < RY; ++r) zi_nxt[r] = zi_base[(x + 1) * a.zp + (y0 - 1) + min(r, nv - 1)];
      }
    } else if (zin) {
      zcur = znext;
      if (x + 1 < xe) znext = zsrc[(x + 1) * a.zp];
      if constexpr ((FEAT & 4096) != 0) {
        // through the wave's LDS slots: no v_readlane -> SGPR -> VALU chain
        if (lo_l || hi_l) zs[(lane < 32 ? 0 : RY) + rl] = zcur;
#pragma unroll
        for (int r = 0; r < RY; ++r) {
          if (zin_lo) {
            const T v = zs[r];
            if (lane == 0) tc[r][0] = v;
          }
          if (zin_hi) {
            const T v = zs[RY + r];
            if (lane == zh) tc[r][VZ - 1] = v;
          }
        }
      } else {
        pl = zin_lo && lane == 0;
        ph = zin_hi && lane == zh;
      }
    }
    T* const xd0 = (FEAT & 64) && x == 1 ? xo0 : nullptr;
    T* const xd1 = (FEAT & 64) && x == n0 - 2 ? xo1 : nullptr;
    V tn[RY], cpn[RY];
    if (PF) {
      const int64_t xn = RV ? max<int64_t>(x - 2, 0) : min(x + 2, n0 - 1);
      const int64_t xc = RV ? max<int64_t>(x - 1, xs) : min(x + 1, xe - 1);
      const T* pn = ((FEAT & 1) && xn == n0 - 1 && xi1) ? xi1 : t + xn * s0;
#pragma unroll
      for (int r = 0; r < RY; ++r) {
        tn[r] = vld<T, VZ>(pn + rowb[r] + zl);
        cpn[r] = ldc(cpp + xc * s0 + rowb[r] + zl);
      }
    }
    V ym, yp;
    if constexpr ((FEAT & 32768) == 0) {
      ym = vld<T, VZ>(ymb + x * yms + zl);
      yp = vld<T, VZ>(ypb + x * yps + zl);
    }
#ifdef IGG_PROBES
    if constexpr ((FEAT & 32768) != 0) {  // timing probe (results WRONG)
      ym = tc[0];
      yp = tc[RY - 1];
    }
#endif
    T em[RY], ep[RY];
    if constexpr ((FEAT & 512) == 0) {
#pragma unroll
      for (int r = 0; r < RY; ++r) {
        em[r] = load_prev ? t[off + rowb[r] + zpi] : T(0);
        ep[r] = load_next ? t[off + rowb[r] + zni] : T(0);
      }
    }
    if constexpr (DF) {
      if (ysend_dst) st_sys(reinterpret_cast<V*>(ysend_dst), ysend);
      if (zsend_dst) st_sys(zsend_dst, zv);
      ysend_dst = nullptr;
      zsend_dst = nullptr;
    }
    T zo_buf[ZE ? RY : 1];
#pragma unroll
    for (int r = 0; r < RY; ++r) {
      if constexpr (ZE && (FEAT & 4) != 0) {
        tc[r][0] = ze_lo ? zi_cur[r] : tc[r][0];
        tc[r][VZ - 1] = ze_hi ? zi_cur[r] : tc[r][VZ - 1];
      } else if constexpr (ZD && (FEAT & 4) != 0) {
        if constexpr (SLO) {
          const T vl = row_shl(zcur, r);  // lane 0 <- lane r
          tc[r][0] = pl ? vl : tc[r][0];
        }
        if constexpr (SHI) {
          const T vh = row_shr(zcur, r);  // lane zh <- lane zh - r
          tc[r][VZ - 1] = ph ? vh : tc[r][VZ - 1];
        }
      } else if constexpr ((FEAT & 4) != 0 && (FEAT & 4096) == 0) {
        // z halo patch of row r right before its update, branch-free: patching
        // every row up front made the step wait for all of this plane's loads
        // at once (and per-row branches split the body into blocks the
        // scheduler cannot interleave: profiles/r2_fused_spec/).
        if constexpr (SLO) {
          const T vl = lane_read(zcur, r);
          tc[r][0] = pl ? vl : tc[r][0];
        }
        if constexpr (SHI) {
          const T vh = lane_read(zcur, 32 + r);
          tc[r][VZ - 1] = ph ? vh : tc[r][VZ - 1];
        }
      }
      const V& c = tc[r];
      const V& yv = (r == 0) ? ym : tc[r > 0 ? r - 1 : 0];
      const V& yn = (r + 1 < nv) ? tc[(r + 1 < RY) ? r + 1 : r] : yp;
      T prev = __shfl_up(c[VZ - 1], 1);
      T next = __shfl_down(c[0], 1);
      if constexpr ((FEAT & 512) != 0) {
        const T pv = lane_read(evc, r), nx = lane_read(evc, 32 + r);
        if (load_prev) prev = pv;
        if (load_next) next = nx;
      } else {
        if (load_prev) prev = em[r];
        if (load_next) next = ep[r];
      }
      V out;
#pragma unroll
      for (int e = 0; e < VZ; ++e) {
        const T zm = e == 0 ? prev : c[e > 0 ? e - 1 : 0];
        const T zp = e == VZ - 1 ? next : c[e + 1 < VZ ? e + 1 : e];
        const T xpv = RV ? tm[r][e] : tp[r][e], xmv = RV ? tp[r][e] : tm[r][e];  // planes x+1, x-1
        out[e] = diffusion_point(c[e], xmv, xpv, yv[e], yn[e], zm, zp, cp[r][e], a.rdx2, a.rdy2, a.rdz2, a.dtlam);
      }
      if (r < nv) {
        T* dst = t2 + off + rowb[r] + zl;
        if constexpr ((FEAT & HZ) != 0) {
          // a z-edge lane (halo_z): its halo element takes t's value (or the
          // received one), in place, so the whole vector - one full line - is
          // stored below instead of a partial line; a wave-uniform branch, so
          // waves away from the z edges run none of it
          if (hz_wave && zfull) {
#pragma unroll
            for (int e = 0; e < VZ; ++e)
              if (z0 + e == 0 || z0 + e == hi2) out[e] = c[e];
          }
        }
        if (lane_full || ((FEAT & HZ) != 0 && zfull)) {
#ifdef IGG_PROBES
          // FEAT 131072: plain (temporal) stores, to measure what the
          // non-temporal hint costs or saves in the Infinity Cache
          if constexpr ((FEAT & 131072) != 0) *reinterpret_cast<V*>(dst) = out;
          else
#endif
          __builtin_nontemporal_store(out, reinterpret_cast<V*>(dst));
        } else {
#pragma unroll
          for (int e = 0; e < VZ; ++e)
            if (z0 + e >= 1 && z0 + e < hi2 && zc == z0) dst[e] = out[e];
        }
        // Send planes / rows (whole vectors of the lanes that own them: the
        // halo elements they carry are never read by the receiver).
        if (xd0 && zown) st_sys_at(xd0, static_cast<uint32_t>((rowb[r] + zl) * sizeof(T)), out);
        if (xd1 && zown) st_sys_at(xd1, static_cast<uint32_t>((rowb[r] + zl) * sizeof(T)), out);
        if (r == 0 && yrow0) {
          if (DF) { ysend = out; ysend_dst = zown ? yrow0 + x * n2 + zl : nullptr; }
          else if (zown) st_sys_at(yrow0, static_cast<uint32_t>((x * n2 + zl) * sizeof(T)), out);
        }
        if (r == ry1) {
          // one deferral slot: taken by row 0 if this wave also sends that row
          if (DF && !yrow0) { ysend = out; ysend_dst = zown ? yrow1 + x * n2 + zl : nullptr; }
          else if (zown) st_sys_at(yrow1, static_cast<uint32_t>((x * n2 + zl) * sizeof(T)), out);
        }
        if constexpr (ZE && (FEAT & 8) != 0) {
          zo_buf[r] = has_lo ? out[1] : out[VZ - 2];  // the send element of the edge lane
        } else if constexpr ((FEAT & 4096) != 0) {
          if (zout_lo && lane == 0) zs[2 * RY + r] = out[1];
          if (zout_hi && lane == zh) zs[3 * RY + r] = out[VZ - 2];
        } else if constexpr (ZD && (FEAT & 8) != 0) {
          if constexpr (SLO) {
            const T vl = row_shr(out[1], r);  // lane r <- lane 0
            zv = (zout_lo && lane == r) ? vl : zv;
          }
          if constexpr (SHI) {
            const T vh = row_shl(out[VZ - 2], r);  // lane zh - r <- lane zh
            zv = (zout_hi && lane == zh - r) ? vh : zv;
          }
        } else if constexpr ((FEAT & 8) != 0) {
          // branch-free (see the z-in patch): unconditional readlanes + selects
          if constexpr (SLO) {
            const T vl = lane_read(out[1], 0);
            zv = (zout_lo && lane == r) ? vl : zv;
          }
          if constexpr (SHI) {
            const T vh = lane_read(out[VZ - 2], zh);
            zv = (zout_hi && lane == 32 + r) ? vh : zv;
          }
        }
      }
    }
    if constexpr ((FEAT & 4096) != 0) {
      if (zdst) zv = zs[(lane < 32 ? 2 * RY : 3 * RY) + rl];
    }
    if constexpr (ZE && (FEAT & 8) != 0) {
      if (zout) {  // uniform: one transpose through LDS per step
        if (lane == (zout_lo ? 0 : zh)) {
#pragma unroll
          for (int r = 0; r < RY; ++r) zo_lds[r] = zo_buf[r];
        }
        zv = zo_lds[rl < RY ? rl : 0];
      }
    }
    if (zdst) {
      if (DF) zsend_dst = zdst + x * a.zp;
      else st_sys(zdst + x * a.zp, zv);
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
    if (!PF && i + 1 < len) {
      const T* pn = ((FEAT & 1) && x + 2 == n0 - 1 && xi1) ? xi1 : t + (x + 2 * DX) * s0;
#pragma unroll
      for (int r = 0; r < RY; ++r) {
        tp[r] = vld<T, VZ>(pn + rowb[r] + zl);
        cp[r] = ldc(cpp + (x + DX) * s0 + rowb[r] + zl);
      }
    }
  }
  if constexpr (DF) {  // sends of the last step
    if (ysend_dst) st_sys(reinterpret_cast<V*>(ysend_dst), ysend);
    if (zsend_dst) st_sys(zsend_dst, zv);
  }
  // Remote stores (system scope, st_sys) acknowledged before the wave retires:
  // the sync kernel that publishes the arrival flags runs after this kernel
  // on the same stream.
  if (remote) __builtin_amdgcn_s_waitcnt(0);
}

// The kernel: each wave runs the sweep specialised to the exchange features its
// tile actually touches. A wave away from every exchanged face (most of them:
// not in the first/last x chunk, not in the first/last y row of tiles, not in a
// z-edge tile) runs the plain sweep (FEAT without exchange bits): the exchange
// code only present in the same loop, with its pointers null at run time,
// measured +60-70 us per step for tilings 11/40 (profiles/r2_fused_spec/),
// because it changes the hot loop's schedule. The test is wave-uniform, so the
// dispatch is a scalar branch; results are unchanged (the skipped features are
// no-ops for such a wave).
#ifdef IGG_WAVES_PER_EU  // measurement builds (build.py IGG_EXTRA_FLAGS)
#define IGG_HX_OCC_ATTR __attribute__((amdgpu_waves_per_eu(IGG_WAVES_PER_EU)))
#else
#define IGG_HX_OCC_ATTR
#endif
template <typename T, int BY, int RY, int VZ, bool PF, int BZ, bool DF, int FEAT = 207>
__global__ void __launch_bounds__(64 * BY * BZ) IGG_HX_OCC_ATTR
diffusion3d_hx_kernel(T* __restrict__ t2, const T* __restrict__ t, const T* __restrict__ cpp,
                      const T* __restrict__ xi0, const T* __restrict__ xi1, const T* __restrict__ yi0,
                      const T* __restrict__ yi1, const T* __restrict__ zi0, const T* __restrict__ zi1,
                      T* __restrict__ xo0, T* __restrict__ xo1, T* __restrict__ yo0, T* __restrict__ yo1,
                      T* __restrict__ zo0, T* __restrict__ zo1, const HxScal<T> a) {
  constexpr int FX = FEAT & (1 | 64), FY = FEAT & (2 | 128), FZ = FEAT & (4 | 8);
  constexpr int FK = FEAT & ~(1 | 2 | 4 | 8 | 64 | 128);
#define IGG_HX_SWEEP(F)                                                                                  \
  hx_sweep<T, BY, RY, VZ, PF, BZ, DF, (F)>(t2, t, cpp, xi0, xi1, yi0, yi1, zi0, zi1, xo0, xo1, yo0, yo1, \
                                           zo0, zo1, a)
#define IGG_HX_SWEEP_ZS(F)                                                    \
  do {                                                                        \
    if constexpr (FZ != 0 && (FEAT & ZSIDES) != 0) {                          \
      if (zs == 1) IGG_HX_SWEEP_R((F) | ZLO);                                 \
      else if (zs == 2) IGG_HX_SWEEP_R((F) | ZHI);                            \
      else IGG_HX_SWEEP_R(F);                                                 \
    } else {                                                                  \
      IGG_HX_SWEEP_R(F);                                                      \
    }                                                                         \
  } while (0)
#define IGG_HX_SWEEP_R(F)                                                                                \
  hx_sweep<T, BY, RY, VZ, PF, BZ, DF, (F)>(t2, t, cpp, xi0, xi1, yi0, yi1, zi0, zi1, xo0, xo1, yo0, yo1, \
                                           zo0, zo1, a, clo, chi)
  if constexpr ((FX | FY | FZ) == 0 || (FEAT & 2048) != 0) {
    IGG_HX_SWEEP(FEAT);  // nothing to specialise, or specialisation disabled (FEAT 2048)
  } else {
    constexpr int W = 64 * VZ * BZ;
    const HxTile<T> tile = hx_tile(a, blockIdx.x, gridDim.x);
    const int64_t tz = tile.tz, ty = tile.ty, cx = tile.cx;
    const int64_t n0 = a.n0, n1 = a.n1, n2 = a.n2;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wz = wid % BZ, wy = wid / BZ;
    const int64_t zt = tz * W + wz * (64 * VZ);
    const int64_t y0 = 1 + ty * (BY * RY) + wy * RY;
    const int64_t xs = 1 + cx * a.ch;
    const int64_t xe = min(xs + a.ch, n0 - 1);
    const int64_t nv = min<int64_t>(RY, n1 - 1 - y0);
    // conservative: a chunk that reads plane 0 / n0-1 or computes plane 1 / n0-2
    // Per side, and only sides with a neighbour count (a 2x1x1 rank runs no
    // y/z code at all; a 2x2x2 corner rank only the z-edge tiles of one side).
    const bool wx = FX != 0 && ((xs <= 1 && (xi0 || xo0)) || (xe >= n0 - 2 && (xi1 || xo1)));
    const bool wyy = FY != 0 && ((y0 <= 1 && (yi0 || yo0)) || (y0 + nv >= n1 - 1 && (yi1 || yo1)));
    const bool wz_lo = zt == 0 && (zi0 || zo0);
    const bool wz_hi = zt <= n2 - VZ && n2 - VZ < zt + 64 * VZ && (zi1 || zo1);
    const bool wzz = FZ != 0 && (wz_lo || wz_hi);
    int sel = __builtin_amdgcn_readfirstlane((wx ? 1 : 0) | (wyy ? 2 : 0) | (wzz ? 4 : 0));
    // which z side(s) a z wave holds: 1 low only, 2 high only, 0 both
    const int zs = __builtin_amdgcn_readfirstlane((wz_lo && !wz_hi) ? 1 : ((wz_hi && !wz_lo) ? 2 : 0));
    if (a.force_sel >= 0) sel = a.force_sel;
    const int64_t t_start = a.stamps ? wall_clock64() : 0;
    // The exchanging waves (sel != 0) synchronise the step with the
    // neighbours (StepSync, put.hpp); the others never touch memory a
    // neighbour reads or writes. Per workgroup: its first exchanging wave
    // polls the flags (one system acquire for the CU's L1) and hands the step
    // number to the others through LDS; its last one counts the workgroup
    // (hx_feature_wgs on the host) - a 2x2x2 corner has ~1,100 exchanging
    // waves, whose per-wave uncached polls and counts slowed every wave.
    const bool ks = a.sync.my_flags != nullptr && sel != 0;
    __shared__ uint64_t wsync[4];  // entered, go, step number c, retired
    if (a.sync.my_flags != nullptr) {  // launch-uniform: every wave of the workgroup
      if (threadIdx.x < 4) wsync[threadIdx.x] = 0;
      __syncthreads();
    }
    int n_ex = 0;  // exchanging waves of this workgroup (same rule as sel, every wave computes it)
    if (ks) {
      int qy = 0, qz = 0;
      for (int j = 0; j < BY; ++j) {
        const int64_t yj = 1 + ty * (BY * RY) + j * RY, nvj = min<int64_t>(RY, n1 - 1 - yj);
        qy += (FY != 0 && ((yj <= 1 && (yi0 || yo0)) || (yj + nvj >= n1 - 1 && (yi1 || yo1)))) ? 0 : 1;
      }
      for (int k = 0; k < BZ; ++k) {
        const int64_t zk = tz * W + k * (64 * VZ);
        const bool lo = zk == 0 && (zi0 || zo0), hi = zk <= n2 - VZ && n2 - VZ < zk + 64 * VZ && (zi1 || zo1);
        qz += (FZ != 0 && (lo || hi)) ? 0 : 1;
      }
      n_ex = __builtin_amdgcn_readfirstlane(wx ? BY * BZ : BY * BZ - qy * qz);
    }
    const uint64_t kc = ks ? step_sync_enter_wg(a.sync, threadIdx.x & 63, wsync) : 0;
    // Peel (a.peel): an x-chunk wave needs the x exchange only at x = 1 (reads
    // plane 0 from the arena, sends plane 1) and x = n0-2 (sends it, reads
    // plane n0-1); the planes in between are swept with the x features
    // compiled out (up to 3 parts; each part reloads its first 3 planes).
    int64_t plo_[3], phi_[3];
    int psel[3], np = 1;
    plo_[0] = 0;
    phi_[0] = INT64_MAX;
    psel[0] = sel;
    if (a.peel && (sel & 1) && a.force_sel < 0) {
      const bool lo = xs == 1 && (xi0 || xo0), hi = xe == n0 - 1 && (xi1 || xo1);
      int64_t a0 = xs;
      np = 0;
      if (lo) { plo_[np] = xs; phi_[np] = xs + 1; psel[np++] = sel; a0 = xs + 1; }
      const int64_t b0 = hi ? n0 - 2 : xe;
      if (b0 > a0) { plo_[np] = a0; phi_[np] = b0; psel[np++] = sel & ~1; }
      if (hi && n0 - 2 >= a0) { plo_[np] = n0 - 2; phi_[np] = n0 - 1; psel[np++] = sel; }
    }
    for (int p = 0; p < np; ++p) {
      const int64_t clo = plo_[p], chi = phi_[p];
      switch (__builtin_amdgcn_readfirstlane(psel[p])) {
        case 0: IGG_HX_SWEEP_R(FK); break;
        case 1: IGG_HX_SWEEP_R(FK | FX); break;
        case 2: IGG_HX_SWEEP_R(FK | FY); break;
        case 3: IGG_HX_SWEEP_R(FK | FX | FY); break;
        case 4: IGG_HX_SWEEP_ZS(FK | FZ); break;
        case 5: IGG_HX_SWEEP_ZS(FK | FX | FZ); break;
        case 6: IGG_HX_SWEEP_ZS(FK | FY | FZ); break;
        default: IGG_HX_SWEEP_ZS(FEAT); break;
      }
    }
    if (ks) step_sync_exit_wg(a.sync, threadIdx.x & 63, kc, wsync, n_ex);
    if (a.stamps) {
      // one vector store per wave (lane 0; lane-dependent address -> VGPR store)
      const int lane = threadIdx.x & 63;
      const int64_t w = (static_cast<int64_t>(blockIdx.x) * (BY * BZ) + wid) * 4;
      if (lane < 4) {
        int cu = 0;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(cu));
        const int64_t v[4] = {sel, t_start, wall_clock64(), static_cast<int64_t>(cu)};
        a.stamps[w + lane] = v[lane];
      }
    }
  }
#undef IGG_HX_SWEEP
#undef IGG_HX_SWEEP_R
#undef IGG_HX_SWEEP_ZS
}

int resident(const void* kernel, int block, size_t lds = 0) {
  static std::vector<std::pair<const void*, int>> cache;
  for (const auto& c : cache)
    if (c.first == kernel) return c.second;
  int dev = 0, cus = 0, occ = 0;
  IGG_HIP_CHECK(hipGetDevice(&dev));
  IGG_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  IGG_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel, block, lds));
  const int r = std::max(1, occ) * std::max(1, cus);
  cache.emplace_back(kernel, r);
  return r;
}

// Workgroups of the launch with at least one exchanging wave (sel != 0 in
// diffusion3d_hx_kernel, the same per-wave rule on the host): the units the
// in-kernel step sync counts (step_sync_exit_wg). The rule is separable - the
// x part depends on the chunk, the y part on the wave's rows, the z part on
// its z tile - and the waves of a workgroup share its chunk, so a workgroup
// has none if its chunk, all its wave rows and all its z columns are
// feature-free: a product.
template <int BY, int RY, int VZ, int BZ, int FEAT>
int64_t hx_feature_wgs(int64_t n0, int64_t n1, int64_t n2, int64_t ch, int64_t nty, int64_t ntz,
                       const HaloIOArgs& io) {
  constexpr int FX = FEAT & (1 | 64), FY = FEAT & (2 | 128), FZ = FEAT & (4 | 8);
  constexpr int W = 64 * VZ * BZ;
  auto on = [&](int d, int s) { return io.in[d][s] != 0 || io.out[d][s] != 0; };
  const int64_t nch = (n0 - 2 + ch - 1) / ch;
  int64_t qx = 0, qy = 0, qz = 0;  // chunks / y tiles / z tiles WITHOUT the feature in any wave
  for (int64_t cx = 0; cx < nch; ++cx) {
    const int64_t xs = 1 + cx * ch, xe = std::min(xs + ch, n0 - 1);
    qx += !(FX != 0 && ((xs <= 1 && on(0, 0)) || (xe >= n0 - 2 && on(0, 1))));
  }
  for (int64_t ty = 0; ty < nty; ++ty) {
    bool none = true;
    for (int wy = 0; wy < BY; ++wy) {
      const int64_t y0 = 1 + ty * (BY * RY) + wy * RY, nv = std::min<int64_t>(RY, n1 - 1 - y0);
      if (FY != 0 && ((y0 <= 1 && on(1, 0)) || (y0 + nv >= n1 - 1 && on(1, 1)))) none = false;
    }
    qy += none;
  }
  for (int64_t tz = 0; tz < ntz; ++tz) {
    bool none = true;
    for (int wz = 0; wz < BZ; ++wz) {
      const int64_t zt = tz * W + wz * (64 * VZ);
      if (FZ != 0 && ((zt == 0 && on(2, 0)) || (zt <= n2 - VZ && n2 - VZ < zt + 64 * VZ && on(2, 1)))) none = false;
    }
    qz += none;
  }
  return nch * nty * ntz - qx * qy * qz;
}

// Whole-line z-edge stores allowed at z side s (HaloIOArgs::zh; -1: no
// neighbour or an arena z input there).
inline bool zh_side(const HaloIOArgs& io, int s) {
  return io.zh[s] >= 0 ? io.zh[s] != 0 : (io.in[2][s] != 0 || io.out[2][s] == 0);
}

template <typename T, int BY, int RY, int VZ, bool PF, int BZ, bool DF, int FEAT = 207>
void launch_hx(const DiffusionArgs& d, const HaloIOArgs& io, hipStream_t stream, bool peel = false,
               bool order = false) {
  const int64_t n0 = d.n[0], n1 = d.n[1], n2 = d.n[2];
  if (n2 % VZ != 0 || n2 < 2 * VZ)
    fail("diffusion3d (fused halo): n2 must be a multiple of ", VZ, " and >= ", 2 * VZ);
  auto kern = &diffusion3d_hx_kernel<T, BY, RY, VZ, PF, BZ, DF, FEAT>;
  const int block = 64 * BY * BZ;
  constexpr int W = 64 * VZ * BZ, TY = BY * RY;
  HxScal<T> a;
  a.n0 = n0; a.n1 = n1; a.n2 = n2; a.zp = io.zpitch; a.zrow = io.zrow > 0 ? io.zrow : 1;
  a.ntz = (n2 - 1 + W - 1) / W;
  a.nty = (n1 - 2 + TY - 1) / TY;
  const int64_t len0 = n0 - 2, tiles = a.ntz * a.nty;
  const int rounds = d.rounds > 0 ? d.rounds : 1;
  // FEAT 1024: one workgroup per CU, enforced with an unused dynamic LDS
  // allocation (isolates the occupancy effect of the lower-VGPR FEAT 512 form).
  size_t lds = (FEAT & 1024) ? 96 * 1024 : ((FEAT & OCC2) ? 79 * 1024 : 0);
  // Measurement knob: IGG_HX_WG_PER_CU=k caps the resident workgroups per CU at
  // k (dynamic LDS of 160 KiB / k), which also sizes the chunks of the grid.
  if (const char* e = std::getenv("IGG_HX_WG_PER_CU"); e && (FEAT & 1024) == 0) {
    const int k = std::atoi(e);
    if (k > 0) lds = std::max<size_t>(lds, (160 * 1024) / static_cast<size_t>(k) - 1024);
  }
  const int64_t target = static_cast<int64_t>(rounds) * resident(reinterpret_cast<const void*>(kern), block, lds);
  const int64_t ch_all = std::max<int64_t>(1, (len0 * tiles + target - 1) / target);
  const int64_t nch = std::max<int64_t>(1, (len0 + ch_all - 1) / ch_all);
  a.ch = (len0 + nch - 1) / nch;
  const int64_t blocks = tiles * ((len0 + a.ch - 1) / a.ch);
  if (blocks > 0x7fffffffLL) fail("diffusion3d (fused halo): grid too large");
  a.rdx2 = static_cast<T>(d.rd2[0]);
  a.rdy2 = static_cast<T>(d.rd2[1]);
  a.rdz2 = static_cast<T>(d.rd2[2]);
  a.dtlam = static_cast<T>(d.dt_lam);
  a.stamps = g_hx_stamps;
  a.force_sel = g_hx_force_sel;
  a.peel = peel ? 1 : 0;
  constexpr int FZ_ = FEAT & (4 | 8);
  a.order = order ? 1 : 0;
  a.order_lo = (FZ_ != 0 && (io.in[2][0] || io.out[2][0])) ? 1 : 0;
  a.order_hi = (FZ_ != 0 && (io.in[2][1] || io.out[2][1])) ? 1 : 0;
  a.tz_hi = (n2 - VZ) / W;
  // halo_z per z side: without a neighbour (fixed boundary: T2's halo equals
  // T's), or with the arena z exchange (the edge lane holds the received halo
  // value: T2's halo planes are stale by design in fused mode and rewritten by
  // sync_halo; nobody else writes them). Not with direct z: the neighbour
  // stores into exactly that element while this kernel runs.
  a.zh_lo = (d.halo_z && zh_side(io, 0)) ? 1 : 0;
  a.zh_hi = (d.halo_z && zh_side(io, 1)) ? 1 : 0;
  a.sync = StepSync{};
  // In-kernel step sync: the specialised kernel only (per-wave feature
  // classes), and not under the diagnostics that override the classes.
  constexpr int FXYZ = FEAT & (1 | 2 | 4 | 8 | 64 | 128);
  if (io.sync.my_flags && FXYZ != 0 && (FEAT & 2048) == 0 && !a.stamps && a.force_sel < 0) {
    a.sync = io.sync;
    // counted per workgroup (step_sync_exit_wg)
    a.sync.feat_waves = hx_feature_wgs<BY, RY, VZ, BZ, FEAT>(n0, n1, n2, a.ch, a.nty, a.ntz, io);
    if (a.sync.feat_waves < 1) a.sync.my_flags = nullptr;
  }
  if (io.sync_used) *io.sync_used = a.sync.my_flags != nullptr;
  auto in = [&](int k, int s) { return reinterpret_cast<const T*>(io.in[k][s]); };
  auto out = [&](int k, int s) { return reinterpret_cast<T*>(io.out[k][s]); };
  hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(blocks)), dim3(block), lds, stream,
                     reinterpret_cast<T*>(d.t2), reinterpret_cast<const T*>(d.t), reinterpret_cast<const T*>(d.cp),
                     in(0, 0), in(0, 1), in(1, 0), in(1, 1), in(2, 0), in(2, 1), out(0, 0), out(0, 1), out(1, 0),
                     out(1, 1), out(2, 0), out(2, 1), a);
  IGG_HIP_CHECK(hipGetLastError());
}

// Send ordering (FusedHalo mode): 0 = remote stores right after the values
// are computed (fastest when stores are acknowledged quickly, e.g. loopback),
// 1 = deferred by one x step (their acknowledgement latency over xGMI can
// never gate the next step's loads). The z edge is lane-distributed in both
// (a per-row direct variant measured 5-100 us slower: profiles/fused/).
//
// Mode bit 2 (modes 2/3 = 0/1 + 2): without a z neighbour (dims[2] == 1 and
// not periodic: the 2x1x1 and 2x2x1 topologies of 2 and 4 ranks) the z-edge
// exchange is compiled out (FEAT 195 = x/y in/out). Results are identical (207
// skips the null z sides at run time). It pays for the 255-VGPR tiling 11
// (loopback 2x2x1 interior rank: 0.632 vs 0.651 ms for the best 207 form) but
// the other tilings' 195 forms measured slower than their 207 forms
// (profiles/r1_noz/), so it is an A/B choice, not automatic.
//
// Mode bit 4 (direct z, FusedHalo with registered field buffers): the z-face
// values are stored straight into the halo column of the neighbour's next
// field (one element per row, the row's own 64-B line) instead of a packed
// arena region, so no wave patches a received z halo into its rows (the cost
// of the z-edge waves of tilings 11/40: profiles/r2_fused_spec/).
//
// Mode bit 32 (order): the z-edge tiles of an exchanging z side are dispatched
// first (hx_tile: longest work first), so with several residency rounds their
// extra time is spread over the slots instead of setting the tail.
//
// Mode bit 8 (peel): a wave of an x-exchange chunk sweeps x = 1 and x = n0-2
// with the x features and the planes in between without them (the x code in
// the loop slows the whole chunk's march: profiles/r2_f32_fused/ class 1).
// XF: extra FEAT bits of the tiling (512 | 1024 for fused variant 40).
template <typename T, int BY, int RY, int VZ, bool PF, int BZ, int XF = 0>
void launch_mode(const DiffusionArgs& d, const HaloIOArgs& io, int mode, hipStream_t s) {
  if constexpr ((XF & ZDPP) != 0) {
    // the DPP z form: one z edge per wave, and the high edge's rows (lanes
    // zh - r) inside the edge lane's 16-lane DPP row
    const int64_t zh = ((d.n[2] - VZ) % (64 * VZ)) / VZ;
    if (d.n[2] <= 64 * VZ + VZ || zh % 16 < RY - 1) {
      launch_mode<T, BY, RY, VZ, PF, BZ, (XF & ~ZDPP)>(d, io, mode, s);
      return;
    }
  }
  if constexpr ((XF & 8192) != 0) {
    // the edge-lane z form needs every wave to hold at most one z edge
    if (d.n[2] <= 64 * VZ + VZ) {
      launch_mode<T, BY, RY, VZ, PF, BZ, (XF & ~8192)>(d, io, mode, s);
      return;
    }
  }
  const bool zx = io.in[2][0] || io.in[2][1] || io.out[2][0] || io.out[2][1];
  const bool pk = (mode & 8) != 0;  // peel the exchanged x planes (kernel)
  const bool ord = (mode & 32) != 0;  // z-edge tiles first (hx_tile)
  mode &= 7;
  if ((mode & 4) && zx) {
    // Direct z (FEAT 203 = 207 without z-in): the z sends land in the
    // receivers' field halo elements, so the z-edge waves read their halo
    // from the field like every other wave and carry only the send code.
    if (io.in[2][0] || io.in[2][1]) fail("diffusion3d (fused halo): direct z mode with z arena input");
    // halo_z contract (HaloIOArgs::zh): a side whose halo column a neighbour
    // writes during this kernel (direct z) never takes whole-line edge stores
    for (int sd = 0; sd < 2; ++sd)
      if (d.halo_z && io.out[2][sd] && !io.z_out_arena && zh_side(io, sd))
        fail("diffusion3d (fused halo): whole-line z-edge stores on a direct-z side (HaloIOArgs::zh)");
    if (mode & 1) launch_hx<T, BY, RY, VZ, PF, BZ, true, 203 | XF | HZ>(d, io, s, pk, ord);
    else launch_hx<T, BY, RY, VZ, PF, BZ, false, 203 | XF | HZ>(d, io, s, pk, ord);
  } else if (zx || !(mode & 2)) {
    mode &= 1;
    if (mode == 0) launch_hx<T, BY, RY, VZ, PF, BZ, false, 207 | XF | HZ>(d, io, s, pk, ord);
    else launch_hx<T, BY, RY, VZ, PF, BZ, true, 207 | XF | HZ>(d, io, s, pk, ord);
  } else {
    mode &= 1;
    if (mode == 0) launch_hx<T, BY, RY, VZ, PF, BZ, false, 195 | XF | HZ>(d, io, s, pk, ord);
    else launch_hx<T, BY, RY, VZ, PF, BZ, true, 195 | XF | HZ>(d, io, s, pk, ord);
  }
}

}  // namespace
}  // namespace igg
