// Fused stencil kernels of the benchmark applications.
//
// 3-D heat diffusion (examples/diffusion3D_multigpu_CuArrays_novis.jl:42-46):
// the reference runs 5 broadcast kernels per step through 4 temporaries
// (qx, qy, qz, dTedt). Fused here into one pass:
//   T2 = T + dt*lam/Cp * (d2T/dx2 + d2T/dy2 + d2T/dz2)       (interior points)
// with ping-pong T/T2 and no temporaries, so the compulsory traffic is exactly
// A_eff = 3 arrays (read T, read Cp, write T2). The update region is a list of
// boxes so the same kernel computes boundary slabs (on the high-priority halo
// stream, ahead of the exchange) and the interior (on the compute stream).
#pragma once

#include <cstdint>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "igg/common.hpp"
#include "igg/put.hpp"

namespace igg {

struct Box {
  int64_t lo[3], hi[3];  // half-open index ranges along dims 0,1,2
  bool empty() const { return lo[0] >= hi[0] || lo[1] >= hi[1] || lo[2] >= hi[2]; }
};

struct DiffusionArgs {
  uintptr_t t2, t, cp;      // C-contiguous (n0,n1,n2) arrays, dim 2 fastest
  int64_t n[3];
  double rd2[3];            // 1/dx_d^2
  double dt_lam;            // dt*lam
  int elem_bytes;           // 8 (f64) or 4 (f32)
  int rounds = 0;           // grid sizing for this launch: 0 = global default,
                            // k > 0 = k residency rounds, k < 0 = |k|*4096 blocks
  // Z-edge stores of the inner box: false = only [1, n-1) is written (the
  // z-edge lanes store 1 or 3 elements, i.e. part of a cache line); true = those
  // lanes store their whole vector, writing t's value into t2's halo element
  // (z = 0 / n2-1) - a full-line store. Only where that is a no-op or is
  // overwritten later: t2's z halo equals t's (fixed boundaries, T2 = T.clone())
  // or the halo update that follows the stencil rewrites it, and nothing writes
  // t2's z halo concurrently. 1024^3 f32: -5.5..-6.8 % per step, 512^3 f64:
  // up to -2.9 % (profiles/r4_halo_z/).
  bool halo_z = false;
};

// Number of tuned kernel variants (see stencil_kernels.hip); variant 0 = default.
int diffusion3d_num_variants();
// Whether variant v is compiled in this build (measurement-only forms need build.py --probes).
bool stencil_variant_compiled(int v);
const char* diffusion3d_variant_name(int v);
// Width (points along dim 2) of one workgroup tile of variant v.
int diffusion3d_variant_tile(int v);
// Grid sizing: number of full residency rounds per launch (<= 0: fixed 4096-block target).
void diffusion3d_set_rounds(int rounds);
int diffusion3d_get_rounds();

void launch_diffusion3d(const DiffusionArgs& a, const std::vector<Box>& boxes, int variant,
                        hipStream_t stream);

// Fused halo exchange (see fused.hpp): the inner-box update additionally
// stores its send planes into the receivers' arena regions (`out`, 0 = no
// receiver at that side) and takes its face halos from its own arena regions
// (`in`, 0 = read the field's halo planes). Region layouts (elements):
//   dim 0 faces [n1][n2], dim 1 faces [n0][n2], dim 2 faces [n0][zpitch]
//   (index x*zpitch + (y-1)*zrow, zrow 0 meaning 1). Needs a vector variant
//   (fused_variant_ok) and n2 % vz == 0. Direct z (mode bit 4): the z sends
//   go straight into the halo elements of the receiver's next field
//   (zpitch = n1*n2, zrow = n2, `out` offset to the halo column), and no
//   z receive code is compiled (`in[2]` must be 0).
struct HaloIOArgs {
  uintptr_t in[3][2];
  uintptr_t out[3][2];
  int64_t zpitch;
  int64_t zrow;
  // Whole-line z-edge stores (DiffusionArgs::halo_z) per z side: 1 allowed
  // (no other writer of t2's halo column at that side during the kernel: no
  // neighbour, the arena z exchange, or the z-unpack form whose unpack kernel
  // rewrites the column after the step), 0 forbidden (direct z: the
  // neighbour stores into exactly that element while this kernel runs), -1
  // derived from in/out (no neighbour or an arena z input: allowed). FusedHalo
  // sets them explicitly; launch_mode rejects an allowed side that receives
  // direct-z stores (z_out_arena false).
  int zh[2] = {-1, -1};
  // The z sends (out[2]) go into arena regions, not into a neighbour's field.
  bool z_out_arena = true;
  // In-kernel step synchronisation (put.hpp StepSync; FusedHalo): the launch
  // takes it when it can count its exchanging waves and then sets *sync_used
  // (otherwise the caller follows the kernel with the sync kernel).
  StepSync sync;
  bool* sync_used = nullptr;
};
bool diffusion3d_fused_variant_ok(int v);
// Diagnostics of the fused kernel: per-wave {feature class, start, end, hw id}
// stamps (4 x int64 per wave, wall_clock64 ticks) into device memory `stamps`
// (nullptr: off), and force_sel >= 0 runs every wave with that feature class
// (-1: per-wave choice). Applies to subsequent fused launches.
void fused_debug(int64_t* stamps, int force_sel);
// Inner-box update through the fused kernel without exchange features
// (tiling = a fused-capable variant index); used by the "hx" variants.
void launch_diffusion3d_inner_hx(const DiffusionArgs& a, int tiling, hipStream_t stream);
// mode 0: sends stored as computed; 1: deferred one x step; + 2: z-edge exchange
// compiled out when there is no z neighbour; + 4: no z receive code (direct z,
// or FusedHalo's z-unpack form; see HaloIOArgs and fused_impl.hpp launch_mode).
void launch_diffusion3d_fused(const DiffusionArgs& a, const HaloIOArgs& io, int variant, int mode,
                              hipStream_t stream);
void host_diffusion3d(const DiffusionArgs& a, const std::vector<Box>& boxes);

// Boundary-slab / interior decomposition of the inner box [1,n-1)^3.
// At every side with `active[d][side]`, a slab of width w[d] is split off (it
// holds the plane that update_halo sends to that side). Returns {slabs, interior}.
void split_boundary(const int64_t n[3], const bool active[3][2], const int64_t w[3],
                    std::vector<Box>& slabs, Box& interior);

}  // namespace igg
