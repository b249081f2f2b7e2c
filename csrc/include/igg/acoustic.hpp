// 2-D acoustic wave propagation on a staggered grid — the staggered-field
// application of the framework (BASELINE config "2-D staggered-grid solver
// 8192^2/GPU Float32, 2x2"): pressure P at cell centres (nx, ny), velocities
// Vx on x-faces (nx+1, ny) and Vy on y-faces (nx, ny+1), C order (y fastest).
//
// One fused update per time step (ping-pong buffers):
//   P2 = P - dt*K * (dVx/dx + dVy/dy)                    all cells
//   Vx2 = Vx - dt/rho * dP2/dx   inner x-faces (1..nx-1), boundary faces copied
//   Vy2 = Vy - dt/rho * dP2/dy   inner y-faces (1..ny-1), boundary faces copied
// then update_halo!(Vx2, Vy2): the velocities have ol = overlap + 1 along
// their staggered dimension ("mixed overlaps"), and P needs no halo because it
// is recomputed from halo-consistent velocities on every rank.
// The kernel recomputes P2 of the left/lower neighbour cell in registers
// instead of a second pass: one read of P, Vx, Vy and one write of P2, Vx2,
// Vy2 per step (6 array passes instead of the 9 of two separate kernels).
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>

namespace igg {

struct AcousticArgs {
  uintptr_t p2, vx2, vy2;    // outputs
  uintptr_t p, vx, vy;       // inputs
  int64_t nx, ny;            // cell counts (P extents)
  double dtk, dt_rho;        // dt*K, dt/rho
  double rdx, rdy;           // 1/dx, 1/dy
  int elem_bytes;            // 4 or 8
};

void launch_acoustic2d(const AcousticArgs& a, hipStream_t stream);
// 0: one thread per cell with neighbour recomputation, 1 (default): marching.
void acoustic2d_set_variant(int v);
void acoustic2d_set_chunk(int64_t rows);  // rows of i per wave of the marching kernel
void host_acoustic2d(const AcousticArgs& a);

}  // namespace igg
