// Fused halo exchange of the 3-D diffusion model: the stencil kernel is the
// pack kernel and the transport.
//
// The reference exchanges halos after the compute (update_halo!, pack ->
// Isend/Irecv -> unpack per dimension, src/update_halo.jl:32-78); on one node
// of MI355X every GPU can store straight into a neighbour's HBM over xGMI. So
// a fused step is ONE launch on the caller's stream: the stencil
// (launch_diffusion3d_fused) stores, while sweeping the interior, the planes
// each neighbour needs (x=1/n0-2, y=1/n1-2, z=1/n2-2) into that neighbour's
// IPC-mapped, fine-grained arena with system-scope stores (st_sys), and reads
// its own face halos from its arena instead of from the field. A 1-wave sync
// kernel after the stencil synchronises the step with the neighbours (publish
// "arrived", wait for theirs; bounded spins, error flag on timeout). With send
// mode bit 16 the exchanging waves do that inside the stencil instead
// (put.hpp StepSync: wait for the neighbours' previous step, the last one
// publishes this step) - not where another rank shares the GPU (waiting waves
// could hold the compute units the other rank needs).
// The arena has two halves: step i writes half i&1 and reads half (i-1)&1, so
// a neighbour may run one step ahead without overwriting data still in use;
// the per-step neighbour synchronisation bounds the skew to one.
// The fields' own halo planes are not touched; sync_halo (update_halo_ of T)
// materialises them when a caller needs them (gather, output, mode switch).
// Direct z (mode bit 4, set_fields): the z faces skip the arena and land in
// the halo column of the neighbour's next field, which the neighbour's next
// step reads like any other element. Ordering: a neighbour writes my buffer k
// (halo elements only) during the step in which my stencil writes buffer k's
// interior and reads buffer 1-k; my previous step (which read buffer k)
// finished before that neighbour's step synchronisation let it start this step.
// Coherence: the halo element shares a cache line with interior elements my
// own kernel is writing at the same time, from another device. HIP defines
// that for fine-grained memory only, so across devices the fields must be
// fine-grained (Diffusion3D's default field_memory="fine"). docs/COHERENCE.md
// has the whole argument.
// Z unpack (mode bit 64): z sends into the arena as in the default form, but
// the z halo is read from the field by the next sweep, written there by a copy
// kernel after the step's synchronisation (unpack_z) - see Z_UNPACK below.
// Results are bitwise identical to stencil + update_halo_ (tests/test_fused.py).
#pragma once

#include <array>
#include <cstdint>
#include <memory>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "igg/peer.hpp"
#include "igg/put.hpp"
#include "igg/stencil.hpp"

namespace igg {

class FusedHalo {
 public:
  // nb[d][s]: rank of the neighbour at side s (0 = low, 1 = high) of dim d in
  // the mesh's numbering, PROC_NULL if none. Collective over the mesh (sizes
  // the arena; every rank has the same local shape).
  FusedHalo(std::shared_ptr<PeerMesh> mesh, const std::array<int64_t, 3>& n, int elem_bytes,
            const std::array<std::array<int, 2>, 3>& nb);

  // Arena regions of the step with counter `step` (writes half step&1; reads
  // half (step-1)&1 if `primed`, else the field's own halo planes). With
  // `direct_z`, the z sends target the halo column of the neighbour's buffer
  // that corresponds to `t2` (set_fields) and nothing is read from the arena
  // along z.
  // With `z_unpack` (send mode bit Z_UNPACK), the z sends go into the
  // neighbours' arenas (whole-line coalesced stores) and nothing is read from
  // the arena along z in the kernel: unpack_z() writes the received z faces
  // into t2's halo column after the step synchronisation.
  HaloIOArgs io(int64_t step, bool primed, uintptr_t t2 = 0, bool direct_z = false, bool z_unpack = false) const;
  // Collective: the two ping-pong field buffers of this rank (same order on
  // every rank, registered at the same step); needed by direct z (mode bit 4).
  // Every rank swaps them in lockstep, so "my t2 is buffer k" means "each
  // neighbour's t2 is its buffer k".
  void set_fields(uintptr_t a, uintptr_t b);
  bool has_fields() const { return !fields_.empty(); }
  // Stencil with fused send/receive and step synchronisation, on `stream`.
  // `entry`: a sync kernel first - the neighbours' remote stores of this step must not
  // overtake this rank's own earlier writes to the fields or the arena (a
  // restore, a switch into fused mode); every rank passes the same flag.
  void step(const DiffusionArgs& a, int variant, int mode, int64_t step, bool primed, hipStream_t stream,
            bool entry = false);
  // Fill the shape/dtype of `a` from this halo's local grid.
  void step_shape(DiffusionArgs& a) const {
    for (int d = 0; d < 3; ++d) a.n[d] = n_[d];
    a.elem_bytes = elem_;
  }
  // Only the sync kernel (e.g. to rehearse the barrier cost).
  void sync(hipStream_t stream) const;
  // Exit barrier: after steps synchronised inside the kernel, the last step's
  // remote stores into THIS rank's arena and fields are complete only once
  // every neighbour has finished that step - nothing on this rank waits for
  // that until the neighbours' next step. drain() launches the sync kernel if
  // the last step() left such stores open (none after a sync-kernel step), so
  // work queued behind it (a restore, a comparison, gather, another exchange)
  // sees the fields final. Collective: every rank drains at the same step.
  void drain(hipStream_t stream);
  // Step synchronisation inside the fused kernel (put.hpp StepSync) or by the
  // sync kernel after it: -1 the default (step_sync_in_kernel), 0 in the
  // kernel, 1 sync kernel. Every rank must use the same form.
  void set_step_sync(int mode) { sync_mode_ = mode; }
  // Send mode bit selecting the in-kernel step synchronisation (step()).
  static constexpr int IN_KERNEL_SYNC = 16;
  // Send mode bit of the z-unpack form (a 2x2x2 corner rank's z exchange out
  // of the sweep's receive path): the z-edge waves keep only their coalesced
  // arena send (one whole-line store per x step; no per-row patch of a
  // received halo, no scattered 8-B remote stores as with direct z), and after
  // the sync kernel a copy kernel writes the received z faces (my arena, this
  // step's half) into t2's z halo column, which the next sweep reads like any
  // other element. Excludes direct z (bit 4). With the in-kernel step sync
  // (bit 16) the unpack kernel waits for the z senders' ARRIVED flags itself
  // (no sync kernel runs between the stencil and the unpack).
  static constexpr int Z_UNPACK = 64;
  // The unpack of the z-unpack form (after the step synchronisation of `step`;
  // `wait`: the in-kernel form, the unpack first waits for the z senders).
  void unpack_z(int64_t step, uintptr_t t2, hipStream_t stream, bool wait = false) const;
  // Whether a step with send mode `mode` synchronises inside the kernel.
  bool in_kernel_sync(int mode = 0) const;

  int64_t region_offset(int d, int s) const { return off_[d][s]; }  // elements within a half
  int64_t half_elems() const { return half_; }
  int64_t zpitch() const { return zp_; }
  int n_peers() const { return sync_.n_out; }
  PeerMesh& mesh() { return *mesh_; }
  void close() {
    fields_.clear();
    mesh_->close();
  }

 private:
  std::shared_ptr<PeerMesh> mesh_;
  std::array<int64_t, 3> n_;
  int elem_;
  std::array<std::array<int, 2>, 3> nb_;
  int64_t off_[3][2];
  int64_t half_ = 0, zp_ = 0;
  PutSync sync_{};
  int sync_mode_ = -1;
  bool open_ = false;  // the last step synchronised inside the kernel (drain() pending)
  std::vector<std::vector<char*>> fields_;  // [rank][k]: ping-pong buffer k (set_fields)
};

}  // namespace igg
