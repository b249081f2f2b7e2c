// Fused 3-D heat-diffusion stencil for gfx950 (CDNA4).
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

#include "igg/stencil.hpp"

namespace igg {
namespace {

constexpr int MAX_BOXES = 8;

struct BoxTable {
  int64_t lo[MAX_BOXES][3];
  int64_t hi[MAX_BOXES][3];
  int64_t ntz[MAX_BOXES], nty[MAX_BOXES], ch[MAX_BOXES];
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
  const T two = T(2);
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
      const T c2 = two * tc[r];
      const T lap = (tp[r] - c2 + tm[r]) * a.rdx2 + (ynext - c2 + yprev) * a.rdy2 +
                    (zp[r] - c2 + zm[r]) * a.rdz2;
      const T out = tc[r] + a.dtlam / cp[r] * lap;
      if (valid[r]) a.t2[off + row[r]] = out;
    }
#pragma unroll
    for (int r = 0; r < RY; ++r) {
      tm[r] = tc[r];
      tc[r] = tp[r];
    }
  }
}

struct Variant {
  const char* name;
  int by, ry;
  bool xcd;
};

// Keep in sync with dispatch() below.
constexpr Variant VARIANTS[] = {
    {"by4_ry4_xcd", 4, 4, true},  {"by4_ry2_xcd", 4, 2, true}, {"by2_ry8_xcd", 2, 8, true},
    {"by8_ry2_xcd", 8, 2, true},  {"by4_ry8_xcd", 4, 8, true}, {"by4_ry4_noxcd", 4, 4, false},
    {"by1_ry16_xcd", 1, 16, true},
};
constexpr int NVARIANTS = sizeof(VARIANTS) / sizeof(VARIANTS[0]);

template <typename T, int BY, int RY, bool XCD>
void launch_one(const KArgs<T>& ka, const std::vector<Box>& boxes, hipStream_t stream) {
  constexpr int TY = BY * RY;
  const int64_t target_blocks = 4096;
  size_t pos = 0;
  while (pos < boxes.size()) {
    BoxTable bt{};
    int64_t blocks = 0;
    bt.n = 0;
    // first pass: tile counts (for the chunk heuristic we need the total tiles)
    std::vector<Box> grp;
    while (pos < boxes.size() && static_cast<int>(grp.size()) < MAX_BOXES) {
      if (!boxes[pos].empty()) grp.push_back(boxes[pos]);
      ++pos;
    }
    if (grp.empty()) continue;
    int64_t tiles = 0;
    for (const Box& bx : grp)
      tiles += ((bx.hi[2] - bx.lo[2] + 63) / 64) * ((bx.hi[1] - bx.lo[1] + TY - 1) / TY);
    const int64_t chunks_wanted = std::max<int64_t>(1, (target_blocks + tiles - 1) / tiles);
    for (const Box& bx : grp) {
      const int k = bt.n++;
      for (int d = 0; d < 3; ++d) { bt.lo[k][d] = bx.lo[d]; bt.hi[k][d] = bx.hi[d]; }
      const int64_t len0 = bx.hi[0] - bx.lo[0];
      bt.ntz[k] = (bx.hi[2] - bx.lo[2] + 63) / 64;
      bt.nty[k] = (bx.hi[1] - bx.lo[1] + TY - 1) / TY;
      // March length: long enough to amortise the 2-plane prologue, short
      // enough to give ~target_blocks workgroups (>> 256 CUs).
      int64_t ch = (len0 + chunks_wanted - 1) / chunks_wanted;
      ch = std::max<int64_t>(ch, std::min<int64_t>(len0, 32));
      bt.ch[k] = ch;
      bt.start[k] = blocks;
      blocks += bt.ntz[k] * bt.nty[k] * ((len0 + ch - 1) / ch);
    }
    bt.start[bt.n] = blocks;
    if (blocks > 0x7fffffffLL) fail("diffusion3d: grid too large");
    hipLaunchKernelGGL((diffusion3d_kernel<T, BY, RY, XCD>), dim3(static_cast<unsigned>(blocks)),
                       dim3(64 * BY), 0, stream, ka, bt);
    IGG_HIP_CHECK(hipGetLastError());
  }
}

template <typename T>
void dispatch(const KArgs<T>& ka, const std::vector<Box>& boxes, int v, hipStream_t s) {
  switch (v) {
    case 0: launch_one<T, 4, 4, true>(ka, boxes, s); break;
    case 1: launch_one<T, 4, 2, true>(ka, boxes, s); break;
    case 2: launch_one<T, 2, 8, true>(ka, boxes, s); break;
    case 3: launch_one<T, 8, 2, true>(ka, boxes, s); break;
    case 4: launch_one<T, 4, 8, true>(ka, boxes, s); break;
    case 5: launch_one<T, 4, 4, false>(ka, boxes, s); break;
    case 6: launch_one<T, 1, 16, true>(ka, boxes, s); break;
    default: fail("diffusion3d: invalid kernel variant ", v);
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
  return k;
}

}  // namespace

int diffusion3d_num_variants() { return NVARIANTS; }
const char* diffusion3d_variant_name(int v) {
  return (v >= 0 && v < NVARIANTS) ? VARIANTS[v].name : "invalid";
}

void launch_diffusion3d(const DiffusionArgs& a, const std::vector<Box>& boxes, int variant,
                        hipStream_t stream) {
  if (a.n[0] < 3 || a.n[1] < 3 || a.n[2] < 3) fail("diffusion3d: every extent must be >= 3");
  for (const Box& b : boxes)
    for (int d = 0; d < 3; ++d)
      if (!b.empty() && (b.lo[d] < 1 || b.hi[d] > a.n[d] - 1))
        fail("diffusion3d: box outside the inner region [1, n-1) along dim ", d);
  if (a.elem_bytes == 8) dispatch<double>(make_args<double>(a), boxes, variant, stream);
  else if (a.elem_bytes == 4) dispatch<float>(make_args<float>(a), boxes, variant, stream);
  else fail("diffusion3d: only float32/float64 are supported");
}

}  // namespace igg
