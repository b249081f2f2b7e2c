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
