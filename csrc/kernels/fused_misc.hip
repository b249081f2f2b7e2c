// Fused halo-exchange diffusion kernels, fused variants 2 (v2_by4_ry4 prefetch), 9 (v4_by4_ry8), 14 (v4_bz2_by2_ry8), 44 (14 + edge-lane z).
// One translation unit per tiling family (igg/fused_impl.hpp) so they compile in parallel.
#include "igg/fused_impl.hpp"

namespace igg {
namespace {

template <typename T>
bool dispatch_misc(const DiffusionArgs& d, const HaloIOArgs& io, int v, int mode, hipStream_t s) {
  switch (v) {
#ifdef IGG_PROBES  // measured, not adopted
    case 2: launch_mode<T, 4, 4, 2, true, 1>(d, io, mode, s); break;
#endif
    case 9: launch_mode<T, 4, 8, 4, false, 1, ZSIDES>(d, io, mode, s); break;  // + side-only z forms
    case 14: launch_mode<T, 2, 8, 4, false, 2>(d, io, mode, s); break;
    // + edge-lane z exchange (FEAT 8192: no per-row v_readlane, which the
    // one-wave-per-SIMD f32 form of tiling 14 cannot hide: profiles/r2_f32_fused/)
    case 44: launch_mode<T, 2, 8, 4, false, 2, 8192>(d, io, mode, s); break;
    default: return false;
  }
  return true;
}

}  // namespace

bool fused_launch_misc(const DiffusionArgs& d, const HaloIOArgs& io, int v, int mode, hipStream_t s) {
  if (d.elem_bytes == 8) return dispatch_misc<double>(d, io, v, mode, s);
  if (d.elem_bytes == 4) return dispatch_misc<float>(d, io, v, mode, s);
  fail("diffusion3d: only float32/float64 are supported");
  return false;
}

}  // namespace igg
