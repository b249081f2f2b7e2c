#pragma once
// Fused halo-exchange kernel families (tiling x exchange forms) for the
// fused_t*_<dt>.hip translation units: each unit explicitly instantiates ONE
// family for ONE element type, so the build compiles them in parallel.
// Variants: bench.py FUSED_* and ops/stencil.py FUSED_VARIANTS; the forms that
// lost their A/Bs are compiled only with IGG_PROBES (build.py --probes).
#include "igg/fused_impl.hpp"

namespace igg {

// tiling 0 (v4_by4_ry4): fused variants 0 and 50 (one workgroup per CU)
template <typename T>
bool fused_family_t0(const DiffusionArgs& d, const HaloIOArgs& io, int v, int mode, hipStream_t s) {
  switch (v) {
    case 0: launch_mode<T, 4, 4, 4, false, 1>(d, io, mode, s); break;
    case 50: launch_mode<T, 4, 4, 4, false, 1, 1024>(d, io, mode, s); break;
#ifdef IGG_PROBES  // measured, not adopted
    case 45: launch_mode<T, 4, 4, 4, false, 1, 8192>(d, io, mode, s); break;  // tiling 0 + edge-lane z
#endif
    default: return false;
  }
  return true;
}

// tiling 11 (v2_by4_ry8): 40 (lane-distributed z-segment edges, one WG per
// CU) and 42 (40 + edge-lane z exchange)
template <typename T>
bool fused_family_t11(const DiffusionArgs& d, const HaloIOArgs& io, int v, int mode, hipStream_t s) {
  switch (v) {
#ifdef IGG_PROBES  // measured, not adopted
    case 11: launch_mode<T, 4, 8, 2, false, 1>(d, io, mode, s); break;
    case 41: launch_mode<T, 4, 8, 2, false, 1, 512 | 1024 | 4096>(d, io, mode, s); break;
#endif
    case 40: launch_mode<T, 4, 8, 2, false, 1, 512 | 1024>(d, io, mode, s); break;
    case 42: launch_mode<T, 4, 8, 2, false, 1, 512 | 1024 | 8192>(d, io, mode, s); break;
    default: return false;
  }
  return true;
}

// tiling 9 (v4_by4_ry8) with the side-only z forms (ZSIDES: the 2x2x2
// corner's best tiling, profiles/r4_shapes/ pass 4)
// 48: tiling 9 with the DPP z-edge lane moves (ZDPP, round 6)
template <typename T>
bool fused_family_t9(const DiffusionArgs& d, const HaloIOArgs& io, int v, int mode, hipStream_t s) {
  switch (v) {
    case 9: launch_mode<T, 4, 8, 4, false, 1, ZSIDES>(d, io, mode, s); break;
    case 48: launch_mode<T, 4, 8, 4, false, 1, ZSIDES | ZDPP>(d, io, mode, s); break;
    default: return false;
  }
  return true;
}

// tiling 14 (v4_bz2_by2_ry8): 14 and 44 (+ edge-lane z exchange, FEAT 8192:
// no per-row v_readlane, which the one-wave-per-SIMD f32 form cannot hide,
// profiles/r2_f32_fused/)
template <typename T>
bool fused_family_t14(const DiffusionArgs& d, const HaloIOArgs& io, int v, int mode, hipStream_t s) {
  switch (v) {
#ifdef IGG_PROBES  // measured, not adopted
    case 2: launch_mode<T, 4, 4, 2, true, 1>(d, io, mode, s); break;
#endif
    case 14: launch_mode<T, 2, 8, 4, false, 2>(d, io, mode, s); break;
    case 44: launch_mode<T, 2, 8, 4, false, 2, 8192>(d, io, mode, s); break;
    default: return false;
  }
  return true;
}

}  // namespace igg
