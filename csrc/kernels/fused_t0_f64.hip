// Fused halo-exchange diffusion kernels, tiling 0: fused variants 0, 50 (double).
// One (family, element type) per translation unit: igg/fused_families.hpp.
#include "igg/fused_families.hpp"

namespace igg {
template bool fused_family_t0<double>(const DiffusionArgs&, const HaloIOArgs&, int, int, hipStream_t);
}  // namespace igg
