#pragma once
// Device arithmetic shared by every stencil form (plain vector/scalar kernels,
// the restrict-form and fused sweeps). The build turns floating-point
// contraction off (build.py): an FMA happens only where it is spelled out
// here, so all forms round identically whatever the compiler's scheduling -
// the bitwise interchangeability the bench checks and tests rely on.
#include <hip/hip_runtime.h>

namespace igg {

__device__ __forceinline__ double fmad(double a, double b, double c) { return __builtin_fma(a, b, c); }
__device__ __forceinline__ float fmad(float a, float b, float c) { return __builtin_fmaf(a, b, c); }

}  // namespace igg

namespace igg {

// One point of the explicit diffusion update (reference:
// examples/diffusion3D_multigpu_CuArrays_novis.jl:42-46, fused):
//   T2 = T + dt*lam/Cp * ((xp - 2c + xm)/dx^2 + (yp - 2c + ym)/dy^2 + (zp - 2c + zm)/dz^2)
// as 6 FMAs, 3 adds, 1 mul and the division, in this order in every kernel
// form (no other contraction happens: build.py -ffp-contract=off).
template <typename T>
__device__ __forceinline__ T diffusion_point(T c, T xm, T xp, T ym, T yp, T zm, T zp, T cp, T rdx2, T rdy2,
                                             T rdz2, T dtlam) {
  const T m2 = T(-2);
  const T dx = fmad(m2, c, xp) + xm;
  const T dy = fmad(m2, c, yp) + ym;
  const T dz = fmad(m2, c, zp) + zm;
  const T lap = fmad(dz, rdz2, fmad(dy, rdy2, dx * rdx2));
  return fmad(dtlam / cp, lap, c);
}

}  // namespace igg
