// FusedAcoustic: the 2-D staggered step with its halo exchange folded into the
// sweep (see include/igg/acoustic.hpp). Produces what update_halo!(Vx2, Vy2)
// (src/update_halo.jl:32-78) would, with one sync kernel instead of
// pack / send / unpack per dimension.
#include <algorithm>
#include <cstdlib>

#include "igg/acoustic.hpp"
#include "igg/common.hpp"
#include "igg/peer.hpp"

namespace igg {

FusedAcoustic::FusedAcoustic(std::shared_ptr<PeerMesh> mesh, int64_t nx, int64_t ny, int elem_bytes,
                             const std::array<std::array<int, 2>, 2>& nb)
    : mesh_(std::move(mesh)), nx_(nx), ny_(ny), elem_(elem_bytes), nb_(nb) {
  if (!mesh_) fail("FusedAcoustic: no peer mesh");
  if (elem_bytes != 4 && elem_bytes != 8) fail("FusedAcoustic: only float32/float64 fields");
  if (nx < 5 || ny < 5) fail("FusedAcoustic: the local grid must be at least 5x5");
  std::vector<int> peers;
  for (int d = 0; d < 2; ++d)
    for (int s = 0; s < 2; ++s) {
      const int r = nb[d][s];
      if (r == PROC_NULL) continue;
      if (r < 0 || r >= mesh_->nranks()) fail("FusedAcoustic: neighbour rank ", r, " outside the mesh");
      if (std::find(peers.begin(), peers.end(), r) == peers.end()) peers.push_back(r);
    }
  // Face neighbourhoods are symmetric: every neighbour is a sender and a receiver.
  sync_.my_flags = mesh_->flags(mesh_->rank());
  for (size_t i = 0; i < peers.size(); ++i) {
    sync_.out_flags[i] = mesh_->flags(peers[i]);
    sync_.nb_flags[i] = mesh_->flags(peers[i]);
    sync_.out_rank[i] = peers[i];
    sync_.in_rank[i] = peers[i];
  }
  sync_.n_out = sync_.n_in = sync_.n_nb = static_cast<int>(peers.size());
  sync_.my_rank = mesh_->rank();
  sync_.nranks = mesh_->nranks();
  sync_.timeout_ticks = mesh_->timeout_ticks();
}

void FusedAcoustic::set_fields(uintptr_t vx_a, uintptr_t vx_b, uintptr_t vy_a, uintptr_t vy_b) {
  if (!vx_a || !vx_b || !vy_a || !vy_b || vx_a == vx_b || vy_a == vy_b)
    fail("FusedAcoustic.set_fields: two distinct buffers of Vx and of Vy expected");
  fields_ = mesh_->map_buffers({vx_a, vx_b, vy_a, vy_b});  // collective
}

void FusedAcoustic::step(const AcousticArgs& a, hipStream_t stream, bool entry) {
  if (fields_.empty()) fail("FusedAcoustic.step: set_fields first");
  if (a.nx != nx_ || a.ny != ny_ || a.elem_bytes != elem_)
    fail("FusedAcoustic.step: fields do not match the fused exchange's local grid");
  const auto& mine = fields_[mesh_->rank()];
  int k = -1;
  for (int i = 0; i < 2; ++i)
    if (reinterpret_cast<uintptr_t>(mine[i]) == a.vx2 && reinterpret_cast<uintptr_t>(mine[2 + i]) == a.vy2) k = i;
  if (k < 0) fail("FusedAcoustic.step: the output fields are not a registered buffer pair");
  // Every rank swaps its buffers in lockstep: my output buffer k is each
  // neighbour's output buffer k.
  const int64_t eb = elem_;
  AcousticHalo h;
  static const int plain = [] {
    const char* e = std::getenv("IGG_FUSED_PLAIN_STORES");
    return (e && e[0] == '1') ? 1 : 0;
  }();
  h.plain_stores = plain;
  for (int s = 0; s < 2; ++s) {
    if (const int r = nb_[0][s]; r != PROC_NULL) {
      h.nb_x[s] = true;
      // my row 2 -> x-low neighbour's row nx; my row nx-2 -> x-high neighbour's row 0
      h.send_x[s] = reinterpret_cast<uintptr_t>(fields_.at(r)[k] + (s == 0 ? nx_ * ny_ : 0) * eb);
    }
    if (const int r = nb_[1][s]; r != PROC_NULL) {
      h.nb_y[s] = true;
      // my column 2 -> y-low neighbour's column ny; my column ny-2 -> y-high's column 0
      h.send_y[s] = reinterpret_cast<uintptr_t>(fields_.at(r)[2 + k] + (s == 0 ? ny_ : 0) * eb);
    }
  }
  // Step synchronisation inside the kernel (put.hpp StepSync: no sync kernel
  // on the stream), or the 1-wave sync kernel after it (IGG_FUSED_SYNC_KERNEL=1).
  const bool sync_kernel = !in_kernel_sync();
  if (!sync_kernel) h.sync = step_sync_from(sync_);
  if (entry) launch_put_sync(sync_, stream);  // entry barrier
  launch_acoustic2d_fused(a, h, stream);
  if (sync_kernel) launch_put_sync(sync_, stream);
  open_ = !sync_kernel;
}

void FusedAcoustic::drain(hipStream_t stream) {
  if (open_) launch_put_sync(sync_, stream);
  open_ = false;
}

void FusedAcoustic::check_error() const { mesh_->check_error(); }

void FusedAcoustic::clear_error() { mesh_->clear_error(); }

uint64_t FusedAcoustic::flag(int index) const { return mesh_->read_flag(index); }

bool FusedAcoustic::in_kernel_sync() const {
  return sync_mode_ < 0 ? step_sync_in_kernel(mesh_->shares_device(), false) : sync_mode_ == 0;
}

void FusedAcoustic::close() {
  fields_.clear();
  mesh_->close();
}

}  // namespace igg
