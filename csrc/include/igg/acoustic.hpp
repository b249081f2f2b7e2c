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

#include <array>
#include <cstdint>
#include <memory>
#include <vector>

#include "igg/put.hpp"

namespace igg {

class PeerMesh;

struct AcousticArgs {
  uintptr_t p2, vx2, vy2;    // outputs
  uintptr_t p, vx, vy;       // inputs
  int64_t nx, ny;            // cell counts (P extents)
  double dtk, dt_rho;        // dt*K, dt/rho
  double rdx, rdy;           // 1/dx, 1/dy
  int elem_bytes;            // 4 or 8
};

// Fused halo exchange of the acoustic step (FusedAcoustic below): where the
// step's output faces travel. x: Vx2 faces 0 / nx (ol = 3), y: Vy2 faces
// 0 / ny. For each side s with a neighbour, `send_*[s]` points at the
// neighbour's element that receives my face (x: its row nx for s = 0, row 0
// for s = 1; y: its element (0, ny) for s = 0, (0, 0) for s = 1) and my own
// face on that side is left to the neighbour (not written here).
struct AcousticHalo {
  uintptr_t send_x[2] = {0, 0};  // Vx2 rows (contiguous, pitch ny)
  uintptr_t send_y[2] = {0, 0};  // Vy2 columns (one element per row, pitch ny+1)
  bool nb_x[2] = {false, false}, nb_y[2] = {false, false};
  int plain_stores = 0;  // debug (IGG_FUSED_PLAIN_STORES=1): plain instead of system-scope remote stores
  StepSync sync;  // in-kernel step synchronisation (put.hpp); set by FusedAcoustic
};

void launch_acoustic2d(const AcousticArgs& a, hipStream_t stream);
// The vector-march step with the exchange fused in (system-scope stores into
// the neighbours' fields, docs/COHERENCE.md). Needs ny % VJ == 0, nx, ny >= 5.
void launch_acoustic2d_fused(const AcousticArgs& a, const AcousticHalo& h, hipStream_t stream);
// 0: one thread per cell with neighbour recomputation, 1 (default): marching.
void acoustic2d_set_variant(int v);
void acoustic2d_set_chunk(int64_t rows);  // rows of i per wave of the marching kernel
void host_acoustic2d(const AcousticArgs& a);

// Fused halo exchange of Acoustic2D, the counterpart of FusedHalo (fused.hpp)
// for the 2-D staggered step. update_halo!(Vx2, Vy2) (reference semantics,
// src/update_halo.jl:32-78) would overwrite Vx2's x-halo faces and y-halo
// columns and Vy2's y-halo faces and x-halo rows. With overlap 2, every one of
// those values except the staggered boundary faces (Vx2 faces 0 / nx, Vy2
// faces 0 / ny) is recomputed by this rank with the same arithmetic from
// halo-consistent inputs, so only those four faces need to travel: the kernel
// stores them straight into the neighbours' next Vx2 / Vy2 (rows of 4*ny B,
// columns of one element per row) while it sweeps, then one 1-wave sync kernel
// publishes "arrived" and waits for the neighbours' (bounded spins). Results
// are bitwise equal to the kernel + update_halo_(Vx2, Vy2) path
// (tests/test_acoustic.py). Ordering as for direct z (fused.hpp): a
// neighbour writes my buffer k during the step in which I write buffer k and
// read buffer 1-k; the per-step barrier bounds the skew to one step. The
// fields must be fine-grained (Acoustic2D allocates them so).
class FusedAcoustic {
 public:
  // nb[d][s]: neighbour rank at side s of dim d (d = 0 x, 1 y) in the mesh's
  // numbering, PROC_NULL if none. Collective over the mesh.
  FusedAcoustic(std::shared_ptr<PeerMesh> mesh, int64_t nx, int64_t ny, int elem_bytes,
                const std::array<std::array<int, 2>, 2>& nb);
  // Collective: the ping-pong buffers of Vx and Vy (same order on every rank).
  void set_fields(uintptr_t vx_a, uintptr_t vx_b, uintptr_t vy_a, uintptr_t vy_b);
  // `entry`: a sync kernel first (a neighbour's remote stores must not
  // overtake this rank's own earlier writes to the fields: FusedHalo::step).
  void step(const AcousticArgs& a, hipStream_t stream, bool entry = false);
  // Exit barrier after in-kernel synchronised steps (FusedHalo::drain):
  // collective, a sync kernel only if the last step left remote stores open.
  void drain(hipStream_t stream);
  void check_error() const;
  void clear_error();
  uint64_t flag(int index) const;  // own flag word (PutFlags), host read
  // Step synchronisation form (FusedHalo::set_step_sync).
  void set_step_sync(int mode) { sync_mode_ = mode; }
  bool in_kernel_sync() const;
  void close();

 private:
  std::shared_ptr<PeerMesh> mesh_;
  int64_t nx_, ny_;
  int elem_;
  std::array<std::array<int, 2>, 2> nb_;
  PutSync sync_{};
  int sync_mode_ = -1;
  bool open_ = false;  // the last step synchronised inside the kernel (drain() pending)
  std::vector<std::vector<char*>> fields_;  // [rank][vx_a, vx_b, vy_a, vy_b]
};

}  // namespace igg
