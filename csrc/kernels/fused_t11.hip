// Fused halo-exchange diffusion kernels, tiling 11 (v2_by4_ry8) forms: fused variants 11, 40 (lane-distributed z-segment edges, one WG per CU) 41 (+ z edge through LDS) and 42 (+ edge-lane z exchange).
// One translation unit per tiling family (igg/fused_impl.hpp) so they compile in parallel.
#include "igg/fused_impl.hpp"

namespace igg {
namespace {

template <typename T>
bool dispatch_t11(const DiffusionArgs& d, const HaloIOArgs& io, int v, int mode, hipStream_t s) {
  switch (v) {
#ifdef IGG_PROBES  // measured, not adopted
    case 11: launch_mode<T, 4, 8, 2, false, 1>(d, io, mode, s); break;
#endif
    case 40: launch_mode<T, 4, 8, 2, false, 1, 512 | 1024>(d, io, mode, s); break;
#ifdef IGG_PROBES  // measured, not adopted
    case 41: launch_mode<T, 4, 8, 2, false, 1, 512 | 1024 | 4096>(d, io, mode, s); break;
#endif
    case 42: launch_mode<T, 4, 8, 2, false, 1, 512 | 1024 | 8192>(d, io, mode, s); break;  // 40 + edge-lane z
    default: return false;
  }
  return true;
}

}  // namespace

bool fused_launch_t11(const DiffusionArgs& d, const HaloIOArgs& io, int v, int mode, hipStream_t s) {
  if (d.elem_bytes == 8) return dispatch_t11<double>(d, io, v, mode, s);
  if (d.elem_bytes == 4) return dispatch_t11<float>(d, io, v, mode, s);
  fail("diffusion3d: only float32/float64 are supported");
  return false;
}

}  // namespace igg
