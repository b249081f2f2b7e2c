// Fused halo-exchange diffusion kernel for gfx950 (see igg/fused.hpp): the
// restrict-argument plain sweeps (stencil variants 21+) and the entry points.
// The kernel templates live in igg/fused_impl.hpp; the fused instantiations in
// fused_t{0,11,9,14}_{f64,f32}.hip (one tiling family and type each).
#include "igg/fused_impl.hpp"

namespace igg {

int64_t* g_hx_stamps = nullptr;
int g_hx_force_sel = -1;

namespace {

// The sweep without any exchange feature (FEAT=0): the plain inner-box
// update through this kernel's restrict-argument form, measured 13-26 us
// faster than diffusion3d_vkernel with the same tiling (profiles/r1_fused/
// feature_bisect_v11.log); bitwise identical arithmetic.
template <typename T>
void dispatch_plain(const DiffusionArgs& d, int v, hipStream_t s) {
  const HaloIOArgs none{};
  switch (v) {  // tilings of the shortlisted restrict-form variants 21/24/26/40/43/44
    // each tiling in the partial-line and the whole-line (HZ, halo_z) z-edge
    // store form: the autotune times both (models/diffusion3d.py)
#define IGG_PLAIN_HX(BY, RY, VZ, BZ, F)                                         \
  (d.halo_z ? launch_hx<T, BY, RY, VZ, false, BZ, false, (F) | HZ>(d, none, s) \
            : launch_hx<T, BY, RY, VZ, false, BZ, false, (F)>(d, none, s))
    case 0: IGG_PLAIN_HX(4, 4, 4, 1, 0); break;
    case 11: IGG_PLAIN_HX(4, 8, 2, 1, 0); break;
    case 100: IGG_PLAIN_HX(2, 8, 2, 1, 0); break;
    case 124: IGG_PLAIN_HX(4, 8, 2, 1, 512 | 1024); break;
    case 141: IGG_PLAIN_HX(2, 8, 2, 4, 0); break;
    case 150: IGG_PLAIN_HX(4, 4, 4, 1, OCC2); break;
#ifdef IGG_PROBES
    // restrict forms of tilings 9 and 14 (variants 23, 25): no A/B win in rounds 2-4
    case 9: IGG_PLAIN_HX(4, 8, 4, 1, 0); break;
    case 14: IGG_PLAIN_HX(2, 8, 4, 2, 0); break;
#endif
#undef IGG_PLAIN_HX
#ifdef IGG_PROBES
    // measured and not adopted (rounds 1-2): other tilings, non-temporal Cp,
    // lane-distributed z edges of other tilings, full-row z tiles, and the
    // timing probes whose results are wrong on purpose
    case 2: launch_hx<T, 4, 4, 2, true, 1, false, 0>(d, none, s); break;
    case 101: launch_hx<T, 4, 6, 2, false, 1, false, 0>(d, none, s); break;
    case 102: launch_hx<T, 4, 8, 2, true, 1, false, 0>(d, none, s); break;
    case 103: launch_hx<T, 4, 4, 2, false, 1, false, 0>(d, none, s); break;
    case 104: launch_hx<T, 4, 2, 4, false, 1, false, 0>(d, none, s); break;
    case 105: launch_hx<T, 8, 4, 2, false, 1, false, 0>(d, none, s); break;
    case 110: launch_hx<T, 4, 8, 2, false, 1, false, 256>(d, none, s); break;
    case 111: launch_hx<T, 4, 4, 4, false, 1, false, 256>(d, none, s); break;
    case 112: launch_hx<T, 4, 8, 4, false, 1, false, 256>(d, none, s); break;
    case 113: launch_hx<T, 2, 8, 4, false, 2, false, 256>(d, none, s); break;
    case 120: launch_hx<T, 4, 8, 2, false, 1, false, 512>(d, none, s); break;
    case 121: launch_hx<T, 4, 8, 4, false, 1, false, 512>(d, none, s); break;
    case 122: launch_hx<T, 2, 8, 2, false, 1, false, 512>(d, none, s); break;
    case 123: launch_hx<T, 4, 4, 4, false, 1, false, 512>(d, none, s); break;
    case 125: launch_hx<T, 4, 10, 2, false, 1, false, 512 | 1024>(d, none, s); break;
    case 126: launch_hx<T, 4, 12, 2, false, 1, false, 512 | 1024>(d, none, s); break;
    case 130: launch_hx<T, 4, 8, 2, false, 1, false, 512 | 1024 | 16384>(d, none, s); break;
    case 131: launch_hx<T, 4, 8, 2, false, 1, false, 512 | 1024 | 32768>(d, none, s); break;
    case 132: launch_hx<T, 4, 8, 2, false, 1, false, 512 | 1024 | 16384 | 32768>(d, none, s); break;
    case 140: launch_hx<T, 4, 8, 2, false, 4, false, 0>(d, none, s); break;
    case 142: launch_hx<T, 4, 4, 2, false, 4, false, 0>(d, none, s); break;
    case 143: launch_hx<T, 4, 4, 4, false, 2, false, 0>(d, none, s); break;
    case 144: launch_hx<T, 4, 8, 4, false, 2, false, 0>(d, none, s); break;
    case 145: launch_hx<T, 2, 8, 2, false, 4, false, 512>(d, none, s); break;
    case 200: launch_hx<T, 4, 4, 4, false, 1, false, 65536>(d, none, s); break;
    case 211: launch_hx<T, 4, 8, 2, false, 1, false, 65536>(d, none, s); break;
    case 300: launch_hx<T, 2, 8, 2, false, 1, false, 65536>(d, none, s); break;
    case 324: launch_hx<T, 4, 8, 2, false, 1, false, 512 | 1024 | 65536>(d, none, s); break;
    case 411: launch_hx<T, 4, 8, 2, false, 1, false, 131072>(d, none, s); break;
    case 611: launch_hx<T, 4, 8, 2, false, 1, false, 131072 | 65536>(d, none, s); break;
#endif
    default: fail("diffusion3d (restrict form): tiling ", v, " not instantiated");
  }
}

}  // namespace

void launch_diffusion3d_inner_hx(const DiffusionArgs& a, int tiling, hipStream_t stream) {
  if (a.n[0] < 3 || a.n[1] < 3 || a.n[2] < 3) fail("diffusion3d: every extent must be >= 3");
  if (a.elem_bytes == 8) dispatch_plain<double>(a, tiling, stream);
  else if (a.elem_bytes == 4) dispatch_plain<float>(a, tiling, stream);
  else fail("diffusion3d: only float32/float64 are supported");
}

void fused_debug(int64_t* stamps, int force_sel) {
  g_hx_stamps = stamps;
  g_hx_force_sel = force_sel;
}

bool diffusion3d_fused_variant_ok(int v) {
  // the fused A/B's tilings (bench.py FUSED_*); 2, 11, 41, 45 only with --probes
#ifdef IGG_PROBES
  if (v == 2 || v == 11 || v == 41 || v == 45) return true;
#endif
  return v == 0 || v == 9 || v == 14 || v == 40 || v == 42 || v == 44 || v == 48 || v == 50;
}

void launch_diffusion3d_fused(const DiffusionArgs& a, const HaloIOArgs& io, int variant, int mode,
                              hipStream_t stream) {
  if (a.n[0] < 3 || a.n[1] < 3 || a.n[2] < 3) fail("diffusion3d: every extent must be >= 3");
  if (mode < 0 || mode > 63 || (mode & 16))
    fail("diffusion3d (fused halo): send mode must be 0..63 without bit 16 (step sync: FusedHalo)");
  if (a.elem_bytes != 8 && a.elem_bytes != 4) fail("diffusion3d: only float32/float64 are supported");
  const bool ok = a.elem_bytes == 8 ? (fused_family_t0<double>(a, io, variant, mode, stream) ||
                                       fused_family_t11<double>(a, io, variant, mode, stream) ||
                                       fused_family_t9<double>(a, io, variant, mode, stream) ||
                                       fused_family_t14<double>(a, io, variant, mode, stream))
                                    : (fused_family_t0<float>(a, io, variant, mode, stream) ||
                                       fused_family_t11<float>(a, io, variant, mode, stream) ||
                                       fused_family_t9<float>(a, io, variant, mode, stream) ||
                                       fused_family_t14<float>(a, io, variant, mode, stream));
  if (!ok) fail("diffusion3d (fused halo): variant ", variant, " has no fused instantiation");
}

}  // namespace igg
