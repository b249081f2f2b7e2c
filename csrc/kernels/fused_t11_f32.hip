// Fused halo-exchange diffusion kernels, tiling 11: fused variants 40, 42 (float).
// One (family, element type) per translation unit: igg/fused_families.hpp.
#include "igg/fused_families.hpp"

namespace igg {
template bool fused_family_t11<float>(const DiffusionArgs&, const HaloIOArgs&, int, int, hipStream_t);
}  // namespace igg
