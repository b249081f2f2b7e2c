// Fused halo-exchange diffusion kernels, tiling 0 (v4_by4_ry4) forms: fused variants 0 and 50 (one workgroup per CU).
// One translation unit per tiling family (igg/fused_impl.hpp) so they compile in parallel.
#include "igg/fused_impl.hpp"

namespace igg {
namespace {

template <typename T>
bool dispatch_t0(const DiffusionArgs& d, const HaloIOArgs& io, int v, int mode, hipStream_t s) {
  switch (v) {
    case 0: launch_mode<T, 4, 4, 4, false, 1>(d, io, mode, s); break;
    case 50: launch_mode<T, 4, 4, 4, false, 1, 1024>(d, io, mode, s); break;  // tiling 0, one WG per CU
#ifdef IGG_PROBES  // measured, not adopted
    case 45: launch_mode<T, 4, 4, 4, false, 1, 8192>(d, io, mode, s); break;  // tiling 0 + edge-lane z
#endif
    default: return false;
  }
  return true;
}

}  // namespace

bool fused_launch_t0(const DiffusionArgs& d, const HaloIOArgs& io, int v, int mode, hipStream_t s) {
  if (d.elem_bytes == 8) return dispatch_t0<double>(d, io, v, mode, s);
  if (d.elem_bytes == 4) return dispatch_t0<float>(d, io, v, mode, s);
  fail("diffusion3d: only float32/float64 are supported");
  return false;
}

}  // namespace igg
