// Host (CPU) diffusion step and the boundary/interior box decomposition.
// Same update as examples/diffusion3D_multicpu_novis.jl:42-46 (qx/qy/qz, dTedt,
// T interior), evaluated in one pass without the flux temporaries.
#include <algorithm>

#include "igg/copy.hpp"
#include "igg/stencil.hpp"

namespace igg {

namespace {
template <typename T>
void host_box(const DiffusionArgs& a, const Box& b) {
  T* t2 = reinterpret_cast<T*>(a.t2);
  const T* t = reinterpret_cast<const T*>(a.t);
  const T* cp = reinterpret_cast<const T*>(a.cp);
  const int64_t s1 = a.n[2], s0 = a.n[1] * a.n[2];
  const T rdx2 = static_cast<T>(a.rd2[0]), rdy2 = static_cast<T>(a.rd2[1]),
          rdz2 = static_cast<T>(a.rd2[2]), dtlam = static_cast<T>(a.dt_lam);
  host_parallel_for(b.hi[0] - b.lo[0], 1, [&](int64_t i0, int64_t i1) {
    for (int64_t x = b.lo[0] + i0; x < b.lo[0] + i1; ++x)
      for (int64_t y = b.lo[1]; y < b.hi[1]; ++y) {
        const int64_t r = x * s0 + y * s1;
        for (int64_t z = b.lo[2]; z < b.hi[2]; ++z) {
          const int64_t i = r + z;
          const T c2 = T(2) * t[i];
          const T lap = (t[i + s0] - c2 + t[i - s0]) * rdx2 + (t[i + s1] - c2 + t[i - s1]) * rdy2 +
                        (t[i + 1] - c2 + t[i - 1]) * rdz2;
          t2[i] = t[i] + dtlam / cp[i] * lap;
        }
      }
  });
}
}  // namespace

void host_diffusion3d(const DiffusionArgs& a, const std::vector<Box>& boxes) {
  for (const Box& b : boxes) {
    if (b.empty()) continue;
    for (int d = 0; d < 3; ++d)
      if (b.lo[d] < 1 || b.hi[d] > a.n[d] - 1)
        fail("diffusion3d: box outside the inner region [1, n-1) along dim ", d);
    if (a.elem_bytes == 8) host_box<double>(a, b);
    else if (a.elem_bytes == 4) host_box<float>(a, b);
    else fail("diffusion3d: only float32/float64 are supported");
  }
}

void split_boundary(const int64_t n[3], const bool active[3][2], const int64_t w[3],
                    std::vector<Box>& slabs, Box& interior) {
  // Inner region [1, n-1); the interior shrinks by w[d] at every active side
  // (a side with a neighbour); slabs are the (disjoint) difference, peeled
  // dim 0 first.
  Box cur{{1, 1, 1}, {n[0] - 1, n[1] - 1, n[2] - 1}};
  slabs.clear();
  for (int d = 0; d < 3; ++d) {
    const int64_t len = cur.hi[d] - cur.lo[d];
    const int64_t wd = std::max<int64_t>(1, std::min<int64_t>(w[d], len / 2));
    if (active[d][0]) {
      Box lo = cur;
      lo.hi[d] = cur.lo[d] + wd;
      if (!lo.empty()) slabs.push_back(lo);
      cur.lo[d] = lo.hi[d];
    }
    if (active[d][1]) {
      Box hi = cur;
      hi.lo[d] = std::max(cur.hi[d] - wd, cur.lo[d]);
      if (!hi.empty()) slabs.push_back(hi);
      cur.hi[d] = hi.lo[d];
    }
  }
  interior = cur;
}

}  // namespace igg
