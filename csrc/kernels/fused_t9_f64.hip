// Fused halo-exchange diffusion kernels, tiling 9 with side-only z forms: fused variant 9 (double).
// One (family, element type) per translation unit: igg/fused_families.hpp.
#include "igg/fused_families.hpp"

namespace igg {
template bool fused_family_t9<double>(const DiffusionArgs&, const HaloIOArgs&, int, int, hipStream_t);
}  // namespace igg
