// Fused 3-D heat-diffusion stencil for gfx950 (CDNA4).
// Computes the update of examples/diffusion3D_multigpu_CuArrays_novis.jl:42-46
// (five broadcasts and four temporaries there) in one kernel.
//
// Regime: 7-point update, ~15 flop per cell against >= 24 B (f64) of compulsory
// HBM traffic -> < 1 flop/B: HBM-bandwidth bound, so MFMA buys nothing here
// (SURVEY.md §7.4 item 3). What matters:
//   * exactly 3 compulsory streams (T in, Cp in, T2 out), fused, no temporaries;
//   * 2.5-D blocking: a workgroup owns a (64 x BY*RY) tile of the (dim2, dim1)
//     plane and marches along dim 0, keeping the previous/current/next planes of
//     its RY rows in registers (x-neighbours never re-read from memory) and
//     taking y-neighbours of interior rows from its own registers;
//   * one wavefront = one 64-point contiguous row (512 B for f64): full-width
//     coalesced loads/stores, z-neighbours hit the same/adjacent lines in L1;
//   * XCD-aware block remap: consecutive tiles (which share halo rows) land on
//     the same XCD so halo rows are served by that XCD's L2;
//   * a box list lets one launch compute the 6 boundary slabs (overlap path).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "igg/devmath.hpp"
#include "igg/stencil.hpp"

namespace igg {
namespace {

constexpr int MAX_BOXES = 8;

struct BoxTable {
  int64_t lo[MAX_BOXES][3];
  int64_t hi[MAX_BOXES][3];
  int64_t ntz[MAX_BOXES], nty[MAX_BOXES], ch[MAX_BOXES];
  int64_t zt0[MAX_BOXES];  // first z tile origin (vector kernel: aligned to 64*VZ)
  int64_t start[MAX_BOXES + 1];
  int n;
};

template <typename T>
struct KArgs {
  T* __restrict__ t2;
  const T* __restrict__ t;
  const T* __restrict__ cp;
  int64_t n0, n1, n2;
  T rdx2, rdy2, rdz2, dtlam;
  int halo_z;  // DiffusionArgs::halo_z: z-edge lanes store whole vectors (halo elements copied from t)
};

__device__ __forceinline__ int64_t xcd_remap(int64_t b, int64_t nb) {
  // Bijective round-robin inversion (cdna_hip_programming.md §5 'XCD swizzle
  // must be bijective'): blocks dealt to XCD k get the contiguous id range k*q..
  const int64_t q = nb / 8, r = nb % 8, xcd = b % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
}

template <typename T, int BY, int RY, bool XCD>
__global__ void __launch_bounds__(64 * BY)
diffusion3d_kernel(const KArgs<T> a, const BoxTable bt) {
  const int64_t nb = bt.start[bt.n];
  int64_t b = blockIdx.x;
  if (XCD) b = xcd_remap(b, nb);
  int k = 0;
  while (k + 1 < bt.n && b >= bt.start[k + 1]) ++k;
  int64_t local = b - bt.start[k];
  const int64_t tz = local % bt.ntz[k];
  local /= bt.ntz[k];
  const int64_t ty = local % bt.nty[k];
  const int64_t cx = local / bt.nty[k];

  const int lane = threadIdx.x & 63;
  const int wy = threadIdx.x >> 6;
  const int64_t z = bt.lo[k][2] + tz * 64 + lane;
  const int64_t y0 = bt.lo[k][1] + ty * (BY * RY) + wy * RY;
  const int64_t xs = bt.lo[k][0] + cx * bt.ch[k];
  const int64_t xe = min(xs + bt.ch[k], bt.hi[k][0]);
  // Rows of this wave inside the box (wave-uniform). Rows/lanes past the box
  // alias the last valid row/lane: their loads hit lines already being read
  // (no extra HBM traffic for thin boundary slabs) and their stores are masked.
  const int nv = static_cast<int>(min<int64_t>(RY, bt.hi[k][1] - y0));
  if (nv <= 0) return;
  const bool zvalid = z < bt.hi[k][2];
  const int64_t zc = min(z, bt.hi[k][2] - 1);  // z+1 <= hi <= n2-1 stays in bounds
  const int64_t s1 = a.n2, s0 = a.n1 * a.n2;

  int64_t row[RY];
  bool valid[RY];
#pragma unroll
  for (int r = 0; r < RY; ++r) {
    valid[r] = zvalid && r < nv;
    row[r] = (y0 + min(r, nv - 1)) * s1 + zc;
  }
  const int64_t row_m = (y0 - 1) * s1 + zc;   // y0-1 >= lo-1 >= 0
  const int64_t row_p = (y0 + nv) * s1 + zc;  // y0+nv <= hi <= n1-1

  const T* __restrict__ t = a.t;
  T tm[RY], tc[RY];
#pragma unroll
  for (int r = 0; r < RY; ++r) {
    tm[r] = t[(xs - 1) * s0 + row[r]];
    tc[r] = t[xs * s0 + row[r]];
  }
  for (int64_t x = xs; x < xe; ++x) {
    const int64_t off = x * s0;
    T tp[RY], zm[RY], zp[RY], cp[RY];
#pragma unroll
    for (int r = 0; r < RY; ++r) {
      tp[r] = t[off + s0 + row[r]];
      zm[r] = t[off + row[r] - 1];
      zp[r] = t[off + row[r] + 1];
      cp[r] = a.cp[off + row[r]];
    }
    const T ym = t[off + row_m];
    const T yp = t[off + row_p];
#pragma unroll
    for (int r = 0; r < RY; ++r) {
      const T yprev = (r == 0) ? ym : tc[r - 1];
      const T ynext = (r + 1 < nv) ? tc[(r + 1 < RY) ? r + 1 : r] : yp;
      const T out = diffusion_point(tc[r], tm[r], tp[r], yprev, ynext, zm[r], zp[r], cp[r], a.rdx2, a.rdy2, a.rdz2,
                                    a.dtlam);
      if (valid[r]) a.t2[off + row[r]] = out;
    }
#pragma unroll
    for (int r = 0; r < RY; ++r) {
      tm[r] = tc[r];
      tc[r] = tp[r];
    }
  }
}

// Vectorised variant: each lane owns VZ consecutive z points (16 B per lane for
// f64 VZ=2), so one wave covers a 64*VZ-point (1 KiB) contiguous row segment
// with one global_load_dwordx4 per array. Tiles are aligned to row starts, so
// every vector access is naturally aligned (requires n2 % VZ == 0). The z
// neighbours come from the lane's own vector and its two lane neighbours
// (__shfl up/down = ds_bpermute); only the two tile-edge values are loaded
// (wave-uniform address). Row bases are wave-uniform (readfirstlane) so the
// per-lane address is a 32-bit offset. PF: prefetch plane x+2 of T and x+1 of
// Cp while computing plane x. NT: non-temporal stores of T2 (streamed once).
template <typename T, int VZ>
struct VecOf {
  typedef T type __attribute__((ext_vector_type(VZ)));
};

template <typename T, int VZ>
__device__ __forceinline__ typename VecOf<T, VZ>::type vload(const T* p) {
  return *reinterpret_cast<const typename VecOf<T, VZ>::type*>(p);
}

// HZ: the whole-line z-edge store form (DiffusionArgs::halo_z), a separate
// instantiation - its extra branches cost tiling 11 2.7 % where the partial
// edge stores cost it nothing, so the autotune times both forms.
// IGG_WAVES_PER_EU (measurement builds, build.py IGG_EXTRA_FLAGS): a minimum
// occupancy for the register allocator (profiles/r6_vsweep/).
#ifdef IGG_WAVES_PER_EU
#define IGG_OCC_ATTR __attribute__((amdgpu_waves_per_eu(IGG_WAVES_PER_EU)))
#else
#define IGG_OCC_ATTR
#endif
template <typename T, int BY, int RY, int VZ, bool PF, bool NT, int BZ, bool HZ>
__global__ void __launch_bounds__(64 * BY * BZ) IGG_OCC_ATTR
diffusion3d_vkernel(const KArgs<T> a, const BoxTable bt) {
  using V = typename VecOf<T, VZ>::type;
  constexpr int W = 64 * VZ * BZ;  // block tile width along z
  const int64_t nb = bt.start[bt.n];
  const int64_t b = xcd_remap(blockIdx.x, nb);
  int k = 0;
  while (k + 1 < bt.n && b >= bt.start[k + 1]) ++k;
  int64_t local = b - bt.start[k];
  const int64_t tz = local % bt.ntz[k];
  local /= bt.ntz[k];
  const int64_t ty = local % bt.nty[k];
  const int64_t cx = local / bt.nty[k];

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wz = wid % BZ, wy = wid / BZ;
  const int64_t zt = bt.zt0[k] + tz * W + wz * (64 * VZ);    // wave-uniform segment origin
  const int64_t y0 = bt.lo[k][1] + ty * (BY * RY) + wy * RY;
  const int64_t xs = bt.lo[k][0] + cx * bt.ch[k];
  const int64_t xe = min(xs + bt.ch[k], bt.hi[k][0]);
  const int nv = static_cast<int>(min<int64_t>(RY, bt.hi[k][1] - y0));
  if (nv <= 0) return;
  const int64_t lo2 = bt.lo[k][2], hi2 = bt.hi[k][2];
  const int64_t n2 = a.n2, s1 = a.n2, s0 = a.n1 * a.n2;
  const int64_t z0 = zt + lane * VZ;
  if (zt >= hi2) return;  // whole wave segment past the box (partial last tile)
  // Lanes whose vector holds no box point alias the first/last vector that does,
  // so a thin box (a single send plane) touches only the lines it needs.
  const int64_t zlo_v = (lo2 / VZ) * VZ, zhi_v = ((hi2 - 1) / VZ) * VZ;
  const int64_t zc = min(max(z0, zlo_v), zhi_v);
  const int zl = static_cast<int>(zc - zt);                  // per-lane offset in the tile
  const bool lane_full = z0 >= lo2 && z0 + VZ <= hi2;
  const bool zfull = HZ && lo2 == 1 && hi2 == n2 - 1 && zc == z0 && z0 + VZ <= n2;
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

  const T* __restrict__ t = a.t;
  const T* __restrict__ cpp = a.cp;
  V tm[RY], tc[RY], tp[RY], cp[RY];
#pragma unroll
  for (int r = 0; r < RY; ++r) {
    tm[r] = vload<T, VZ>(t + (xs - 1) * s0 + rowb[r] + zl);
    tc[r] = vload<T, VZ>(t + xs * s0 + rowb[r] + zl);
    tp[r] = vload<T, VZ>(t + (xs + 1) * s0 + rowb[r] + zl);
    cp[r] = vload<T, VZ>(cpp + xs * s0 + rowb[r] + zl);
  }
  for (int64_t x = xs; x < xe; ++x) {
    const int64_t off = x * s0;
    V tn[RY], cpn[RY];
    if (PF) {
      const int64_t xn = min(x + 2, a.n0 - 1), xc = min(x + 1, xe - 1);
#pragma unroll
      for (int r = 0; r < RY; ++r) {
        tn[r] = vload<T, VZ>(t + xn * s0 + rowb[r] + zl);
        cpn[r] = vload<T, VZ>(cpp + xc * s0 + rowb[r] + zl);
      }
    }
    const V ym = vload<T, VZ>(t + off + rowm + zl);
    const V yp = vload<T, VZ>(t + off + rowp + zl);
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
        out[e] = diffusion_point(c[e], tm[r][e], tp[r][e], yv[e], yn[e], zm, zp, cp[r][e], a.rdx2, a.rdy2, a.rdz2,
                                 a.dtlam);
      }
      if (r < nv) {
        T* dst = a.t2 + off + rowb[r] + zl;
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
        tp[r] = vload<T, VZ>(t + (x + 2) * s0 + rowb[r] + zl);
        cp[r] = vload<T, VZ>(cpp + (x + 1) * s0 + rowb[r] + zl);
      }
    }
  }
}

struct Variant {
  const char* name;
  int by, ry, vz;  // vz = 1: scalar kernel
  bool pf, nt;
};

// Tuned variants; keep in sync with dispatch() below. Default (0) is the best
// measured on MI355X for 512^3 f64 (benchmarks/stencil_sweep.py).
constexpr Variant VARIANTS[] = {
    {"v4_by4_ry4_nt", 4, 4, 4, false, true},     // 0
    {"s_by4_ry8", 4, 8, 1, false, false},        // 1 (scalar fallback family)
    {"v2_by4_ry4_pf_nt", 4, 4, 2, true, true},   // 2
    {"v4_by4_ry4", 4, 4, 4, false, false},       // 3
    {"v4_by4_ry4_pf_nt", 4, 4, 4, true, true},   // 4
    {"v4_by4_ry2_nt", 4, 2, 4, false, true},     // 5
    {"v8_by4_ry2_nt", 4, 2, 8, false, true},     // 6
    {"v4_by2_ry4_nt", 2, 4, 4, false, true},     // 7
    {"v4_by8_ry2_nt", 8, 2, 4, false, true},     // 8
    {"v4_by4_ry8_nt", 4, 8, 4, false, true},     // 9
    {"v8_by2_ry2_nt", 2, 2, 8, false, true},     // 10
    {"v2_by4_ry8_nt", 4, 8, 2, false, true},     // 11
    {"v4_bz2_by8_ry4_nt", 8, 4, 4, false, true}, // 12 (1024-thread blocks)
    {"v4_bz2_by4_ry4_nt", 4, 4, 4, false, true}, // 13
    {"v4_bz2_by2_ry8_nt", 2, 8, 4, false, true}, // 14
    {"v2_bz2_by4_ry8_nt", 4, 8, 2, false, true}, // 15
    {"v4_bz2_by8_ry2_nt", 8, 2, 4, false, true}, // 16
    {"v2_bz4_by4_ry4_nt", 4, 4, 2, false, true}, // 17
    {"s_by4_ry1", 4, 1, 1, false, false},        // 18 (low-VGPR: thin send planes)
    {"v2_by4_ry1_nt", 4, 1, 2, false, true},     // 19 (low-VGPR vector)
    {"v4_by4_ry2", 4, 2, 4, false, false},       // 20
    // 21-25: inner box through the restrict-argument kernel of fused_kernels.hip
    // with the tiling of variant 0/2/9/11/14 (other boxes: that variant here).
    {"hx_v4_by4_ry4_nt", 4, 4, 4, false, true},     // 21
    {"hx_v2_by4_ry4_pf_nt", 4, 4, 2, true, true},   // 22
    {"hx_v4_by4_ry8_nt", 4, 8, 4, false, true},     // 23
    {"hx_v2_by4_ry8_nt", 4, 8, 2, false, true},     // 24
    {"hx_v4_bz2_by2_ry8_nt", 2, 8, 4, false, true}, // 25
    // 26-31: tilings only in the restrict form (fallback for other boxes: the
    // nearest stencil_kernels.hip variant)
    {"hx_v2_by2_ry8_nt", 2, 8, 2, false, true},     // 26
    {"hx_v2_by4_ry6_nt", 4, 6, 2, false, true},     // 27
    {"hx_v2_by4_ry8_pf_nt", 4, 8, 2, true, true},   // 28
    {"hx_v2_by4_ry4_nt", 4, 4, 2, false, true},     // 29
    {"hx_v4_by4_ry2_nt", 4, 2, 4, false, true},     // 30
    {"hx_v2_by8_ry4_nt", 8, 4, 2, false, true},     // 31
    // 32-35: restrict form with non-temporal Cp loads (tilings of 11, 0, 9, 14)
    {"hx_v2_by4_ry8_nt_ntc", 4, 8, 2, false, true},     // 32
    {"hx_v4_by4_ry4_nt_ntc", 4, 4, 4, false, true},     // 33
    {"hx_v4_by4_ry8_nt_ntc", 4, 8, 4, false, true},     // 34
    {"hx_v4_bz2_by2_ry8_nt_ntc", 2, 8, 4, false, true}, // 35
    // 36-39: restrict form with lane-distributed z-segment edge loads (tilings of 11, 9, 26, 0)
    {"hx_v2_by4_ry8_nt_zl", 4, 8, 2, false, true},      // 36
    {"hx_v4_by4_ry8_nt_zl", 4, 8, 4, false, true},      // 37
    {"hx_v2_by2_ry8_nt_zl", 2, 8, 2, false, true},      // 38
    {"hx_v4_by4_ry4_nt_zl", 4, 4, 4, false, true},      // 39
    {"hx_v2_by4_ry8_nt_zl_occ1", 4, 8, 2, false, true}, // 40 (one workgroup per CU)
    {"hx_v2_by4_ry10_nt_zl_occ1", 4, 10, 2, false, true}, // 41
    {"hx_v2_by4_ry12_nt_zl_occ1", 4, 12, 2, false, true}, // 42
    // 43: full-row z tiles (BZ 4 x 64 lanes x VZ 2 = 512 points, profiles/r2_fullrow/)
    {"hx_v2_bz4_by2_ry8_nt", 2, 8, 2, false, true},     // 43
    // 44: tiling 0 at most 2 workgroups per CU (f32 1024^3: 2.5 % ahead of its
    // 3-per-CU form, profiles/r6_vsweep/)
    {"hx_v4_by4_ry4_nt_occ2", 4, 4, 4, false, true},    // 44
};
// Variants 21..31: restrict-form tiling id (fused_kernels.hip dispatch_plain)
// and the stencil_kernels.hip variant used for boxes other than the inner box.
constexpr int HX_TILING[] = {0, 2, 9, 11, 14, 100, 101, 102, 103, 104, 105, 110, 111, 112, 113, 120, 121, 122, 123, 124, 125, 126, 141, 150};
constexpr int HX_FALLBACK[] = {0, 2, 9, 11, 14, 11, 11, 11, 2, 5, 11, 11, 0, 9, 14, 11, 9, 11, 0, 11, 11, 11, 11, 0};
constexpr int NVARIANTS = sizeof(VARIANTS) / sizeof(VARIANTS[0]);

// Grid sizing policy: `g_rounds` full residency rounds (resident workgroups =
// occupancy x CUs); the x-march is chunked so every block gets equal work and
// no partial last round leaves CUs idle. g_rounds <= 0: fixed 4096-block target.
int g_rounds = 1;
int g_call_rounds = 0;  // per-launch override (set by launch_diffusion3d for one call)

int resident_blocks(const void* kernel, int block) {
  static std::vector<std::pair<const void*, int>> cache;
  for (const auto& c : cache)
    if (c.first == kernel) return c.second;
  int dev = 0, cus = 0, occ = 0;
  IGG_HIP_CHECK(hipGetDevice(&dev));
  IGG_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  IGG_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel, block, 0));
  const int r = std::max(1, occ) * std::max(1, cus);
  cache.emplace_back(kernel, r);
  return r;
}

// Build the box tables (<= MAX_BOXES per launch) for tile width W (z) and
// tile height TY (y); `aligned`: z tiles start at multiples of W.
template <typename F>
void for_each_table(const std::vector<Box>& boxes, int W, int TY, bool aligned, int64_t target_blocks,
                    F&& launch) {
  size_t pos = 0;
  while (pos < boxes.size()) {
    std::vector<Box> grp;
    while (pos < boxes.size() && static_cast<int>(grp.size()) < MAX_BOXES) {
      if (!boxes[pos].empty()) grp.push_back(boxes[pos]);
      ++pos;
    }
    if (grp.empty()) continue;
    BoxTable bt{};
    bt.n = 0;
    int64_t blocks = 0, len_sum = 0;
    auto zt0 = [&](const Box& bx) { return aligned ? (bx.lo[2] / W) * W : bx.lo[2]; };
    for (const Box& bx : grp) {
      const int64_t t = ((bx.hi[2] - zt0(bx) + W - 1) / W) * ((bx.hi[1] - bx.lo[1] + TY - 1) / TY);
      len_sum += t * (bx.hi[0] - bx.lo[0]);
    }
    // Planes per block so that sum(tiles * len0 / ch) ~= target_blocks.
    int64_t ch_all = std::max<int64_t>(1, (len_sum + target_blocks - 1) / target_blocks);
    for (const Box& bx : grp) {
      const int k = bt.n++;
      for (int d = 0; d < 3; ++d) { bt.lo[k][d] = bx.lo[d]; bt.hi[k][d] = bx.hi[d]; }
      const int64_t len0 = bx.hi[0] - bx.lo[0];
      bt.zt0[k] = zt0(bx);
      bt.ntz[k] = (bx.hi[2] - bt.zt0[k] + W - 1) / W;
      bt.nty[k] = (bx.hi[1] - bx.lo[1] + TY - 1) / TY;
      // Equal-size chunks along the march (no short remainder chunk). A thin
      // box (few tiles, e.g. a one-row slab) gets shorter marches so it still
      // spreads over >= ~256 workgroups instead of a few latency-bound ones.
      const int64_t tiles_k = bt.ntz[k] * bt.nty[k];
      const int64_t ch_box =
          std::min<int64_t>(ch_all, std::max<int64_t>(4, (len0 * tiles_k + 255) / 256));
      const int64_t nch = std::max<int64_t>(1, (len0 + ch_box - 1) / ch_box);
      const int64_t ch = (len0 + nch - 1) / nch;
      bt.ch[k] = ch;
      bt.start[k] = blocks;
      blocks += bt.ntz[k] * bt.nty[k] * ((len0 + ch - 1) / ch);
    }
    bt.start[bt.n] = blocks;
    if (blocks > 0x7fffffffLL) fail("diffusion3d: grid too large");
    launch(bt, static_cast<unsigned>(blocks));
  }
}

int64_t target_for(const void* kernel, int block) {
  const int rounds = g_call_rounds != 0 ? g_call_rounds : g_rounds;
  if (rounds <= 0) return 4096 * (rounds < 0 ? -rounds : 1);
  return static_cast<int64_t>(rounds) * resident_blocks(kernel, block);
}

template <typename T, int BY, int RY, bool XCD>
void launch_scalar(const KArgs<T>& ka, const std::vector<Box>& boxes, hipStream_t stream) {
  const void* kern = reinterpret_cast<const void*>(&diffusion3d_kernel<T, BY, RY, XCD>);
  for_each_table(boxes, 64, BY * RY, false, target_for(kern, 64 * BY), [&](const BoxTable& bt, unsigned blocks) {
    hipLaunchKernelGGL((diffusion3d_kernel<T, BY, RY, XCD>), dim3(blocks), dim3(64 * BY), 0, stream, ka, bt);
    IGG_HIP_CHECK(hipGetLastError());
  });
}

template <typename T, int BY, int RY, int VZ, bool PF, bool NT, int BZ, bool HZ>
void launch_vector_form(const KArgs<T>& ka, const std::vector<Box>& boxes, hipStream_t stream) {
  const void* kern = reinterpret_cast<const void*>(&diffusion3d_vkernel<T, BY, RY, VZ, PF, NT, BZ, HZ>);
  for_each_table(boxes, 64 * VZ * BZ, BY * RY, true, target_for(kern, 64 * BY * BZ), [&](const BoxTable& bt, unsigned blocks) {
    hipLaunchKernelGGL((diffusion3d_vkernel<T, BY, RY, VZ, PF, NT, BZ, HZ>), dim3(blocks), dim3(64 * BY * BZ), 0,
                       stream, ka, bt);
    IGG_HIP_CHECK(hipGetLastError());
  });
}

template <typename T, int BY, int RY, int VZ, bool PF, bool NT, int BZ = 1>
void launch_vector(const KArgs<T>& ka, const std::vector<Box>& boxes, hipStream_t stream) {
  if (ka.n2 % VZ != 0 || ka.n2 < 2 * VZ) {  // vector path needs aligned rows
    launch_scalar<T, 4, 8, true>(ka, boxes, stream);
    return;
  }
  if (ka.halo_z) {
    launch_vector_form<T, BY, RY, VZ, PF, NT, BZ, true>(ka, boxes, stream);
  } else {
    launch_vector_form<T, BY, RY, VZ, PF, NT, BZ, false>(ka, boxes, stream);
  }
}

template <typename T>
void dispatch(const KArgs<T>& ka, const std::vector<Box>& boxes, int v, hipStream_t s) {
  switch (v) {
    case 0: launch_vector<T, 4, 4, 4, false, true>(ka, boxes, s); break;
    case 1: launch_scalar<T, 4, 8, true>(ka, boxes, s); break;
    case 2: launch_vector<T, 4, 4, 2, true, true>(ka, boxes, s); break;
    case 5: launch_vector<T, 4, 2, 4, false, true>(ka, boxes, s); break;
    case 9: launch_vector<T, 4, 8, 4, false, true>(ka, boxes, s); break;
    case 11: launch_vector<T, 4, 8, 2, false, true>(ka, boxes, s); break;
    case 14: launch_vector<T, 2, 8, 4, false, true, 2>(ka, boxes, s); break;
    case 18: launch_scalar<T, 4, 1, true>(ka, boxes, s); break;
#ifdef IGG_PROBES
    case 3: launch_vector<T, 4, 4, 4, false, false>(ka, boxes, s); break;
    case 4: launch_vector<T, 4, 4, 4, true, true>(ka, boxes, s); break;
    case 6: launch_vector<T, 4, 2, 8, false, true>(ka, boxes, s); break;
    case 7: launch_vector<T, 2, 4, 4, false, true>(ka, boxes, s); break;
    case 8: launch_vector<T, 8, 2, 4, false, true>(ka, boxes, s); break;
    case 10: launch_vector<T, 2, 2, 8, false, true>(ka, boxes, s); break;
    case 12: launch_vector<T, 8, 4, 4, false, true, 2>(ka, boxes, s); break;
    case 13: launch_vector<T, 4, 4, 4, false, true, 2>(ka, boxes, s); break;
    case 15: launch_vector<T, 4, 8, 2, false, true, 2>(ka, boxes, s); break;
    case 16: launch_vector<T, 8, 2, 4, false, true, 2>(ka, boxes, s); break;
    case 17: launch_vector<T, 4, 4, 2, false, true, 4>(ka, boxes, s); break;
    case 19: launch_vector<T, 4, 1, 2, false, true>(ka, boxes, s); break;
    case 20: launch_vector<T, 4, 2, 4, false, false>(ka, boxes, s); break;
#endif
    default: fail("diffusion3d: kernel variant ", v, " is not compiled in this build",
                  " (measurement-only variants: build.py --probes)");
  }
}

template <typename T>
KArgs<T> make_args(const DiffusionArgs& a) {
  KArgs<T> k;
  k.t2 = reinterpret_cast<T*>(a.t2);
  k.t = reinterpret_cast<const T*>(a.t);
  k.cp = reinterpret_cast<const T*>(a.cp);
  k.n0 = a.n[0]; k.n1 = a.n[1]; k.n2 = a.n[2];
  k.rdx2 = static_cast<T>(a.rd2[0]);
  k.rdy2 = static_cast<T>(a.rd2[1]);
  k.rdz2 = static_cast<T>(a.rd2[2]);
  k.dtlam = static_cast<T>(a.dt_lam);
  k.halo_z = a.halo_z ? 1 : 0;
  return k;
}

}  // namespace

// Compiled variants of the default build: the autotune shortlist
// (ops/stencil.py SHORTLIST: the variants that won an A/B on some box in rounds
// 2-4), the plain tilings the fused/overlap paths and the restrict-form
// variants fall back to for other boxes (0, 5, 9, 11, 14), the scalar fallback
// (1) and the one-row slab kernel (18). The other tilings were measured in
// rounds 1-4 and never won; they are built only with `build.py --probes`
// (IGG_PROBES) for re-measurement.
bool stencil_variant_compiled(int v) {
#ifdef IGG_PROBES
  return v >= 0 && v < NVARIANTS;
#else
  switch (v) {
    case 0: case 1: case 2: case 5: case 9: case 11: case 14: case 18:
    case 21: case 24: case 26: case 40: case 43: case 44:
      return true;
    default:
      return false;
  }
#endif
}

int diffusion3d_num_variants() { return NVARIANTS; }
void diffusion3d_set_rounds(int rounds) { g_rounds = rounds; }
int diffusion3d_get_rounds() { return g_rounds; }
const char* diffusion3d_variant_name(int v) {
  return (v >= 0 && v < NVARIANTS) ? VARIANTS[v].name : "invalid";
}
int diffusion3d_variant_tile(int v) {
  if (v < 0 || v >= NVARIANTS) return 0;
  if (v >= 21) v = HX_FALLBACK[v - 21];
  const int bz = (v >= 12 && v <= 16) ? 2 : (v == 17 ? 4 : 1);
  return 64 * VARIANTS[v].vz * bz;
}

void launch_diffusion3d(const DiffusionArgs& a, const std::vector<Box>& boxes, int variant,
                        hipStream_t stream) {
  struct RoundsGuard {
    explicit RoundsGuard(int r) { g_call_rounds = r; }
    ~RoundsGuard() { g_call_rounds = 0; }
  } guard(a.rounds);
  if (a.n[0] < 3 || a.n[1] < 3 || a.n[2] < 3) fail("diffusion3d: every extent must be >= 3");
  if (!stencil_variant_compiled(variant))
    fail("diffusion3d: kernel variant ", variant, " is not compiled in this build (measurement-only variants: "
         "build.py --probes)");
  for (const Box& b : boxes)
    for (int d = 0; d < 3; ++d)
      if (!b.empty() && (b.lo[d] < 1 || b.hi[d] > a.n[d] - 1))
        fail("diffusion3d: box outside the inner region [1, n-1) along dim ", d);
  if (variant >= 21 && variant < NVARIANTS) {
    const int tiling = HX_TILING[variant - 21];
    const bool inner = boxes.size() == 1 && boxes[0].lo[0] == 1 && boxes[0].lo[1] == 1 && boxes[0].lo[2] == 1 &&
                       boxes[0].hi[0] == a.n[0] - 1 && boxes[0].hi[1] == a.n[1] - 1 && boxes[0].hi[2] == a.n[2] - 1;
    const int vz = VARIANTS[variant].vz;
    if (inner && a.n[2] % vz == 0 && a.n[2] >= 2 * vz) {
      launch_diffusion3d_inner_hx(a, tiling, stream);
      return;
    }
    variant = HX_FALLBACK[variant - 21];
  }
  if (a.elem_bytes == 8) dispatch<double>(make_args<double>(a), boxes, variant, stream);
  else if (a.elem_bytes == 4) dispatch<float>(make_args<float>(a), boxes, variant, stream);
  else fail("diffusion3d: only float32/float64 are supported");
}

}  // namespace igg
