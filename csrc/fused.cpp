// FusedHalo: arena regions and neighbour sync for the stencil kernel that stores its
// send planes straight into the neighbours' arenas. Produces the halos that
// update_halo!(T) (examples/diffusion3D_multigpu_CuArrays_novis.jl:47, update_halo.jl:32-78)
// would, without a separate pack/send/unpack pass.
#include "igg/fused.hpp"

#include <algorithm>
#include <vector>

#include "igg/copy.hpp"

namespace igg {

FusedHalo::FusedHalo(std::shared_ptr<PeerMesh> mesh, const std::array<int64_t, 3>& n, int elem_bytes,
                     const std::array<std::array<int, 2>, 3>& nb)
    : mesh_(std::move(mesh)), n_(n), elem_(elem_bytes), nb_(nb) {
  if (!mesh_) fail("FusedHalo: no peer mesh");
  if (elem_bytes != 4 && elem_bytes != 8) fail("FusedHalo: only float32/float64 fields");
  for (int d = 0; d < 3; ++d)
    if (n[d] < 3) fail("FusedHalo: every local extent must be >= 3");
  // Region sizes (elements): dim-0 faces [n1][n2], dim-1 [n0][n2], dim-2
  // [n0][zp] with zp >= n1-2 rounded to 16 (vector stores of up to 16 rows).
  // The x/y send planes are stored through buffer descriptors with 32-bit
  // byte offsets (st_sys_at, sysstore.hpp).
  if (std::max(n[1] * n[2], n[0] * n[2]) * elem_bytes >= (int64_t{1} << 31))
    fail("FusedHalo: a face of the local grid exceeds 2 GiB");
  zp_ = round_up(n[1] - 2, 16);
  const int64_t sz[3] = {n[1] * n[2], n[0] * n[2], n[0] * zp_};
  const int64_t g = static_cast<int64_t>(DEVICE_ALIGN) / elem_bytes;
  int64_t pos = 0;
  for (int d = 0; d < 3; ++d)
    for (int s = 0; s < 2; ++s) {
      off_[d][s] = pos;
      pos += round_up(sz[d], g);
    }
  half_ = pos;
  mesh_->ensure_arena(static_cast<size_t>(2 * half_ * elem_bytes));  // collective

  // Sync kernel: every distinct neighbour is both a receiver and a sender
  // (face neighbourhoods are symmetric, periodic or not).
  std::vector<int> peers;
  for (int d = 0; d < 3; ++d)
    for (int s = 0; s < 2; ++s) {
      const int r = nb[d][s];
      if (r == PROC_NULL) continue;
      if (r < 0 || r >= mesh_->nranks()) fail("FusedHalo: neighbour rank ", r, " outside the mesh");
      if (std::find(peers.begin(), peers.end(), r) == peers.end()) peers.push_back(r);
    }
  if (static_cast<int>(peers.size()) > PUT_MAX_PEERS) fail("FusedHalo: too many peers");
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

void FusedHalo::set_fields(uintptr_t a, uintptr_t b) {
  if (!a || !b || a == b) fail("FusedHalo.set_fields: two distinct field buffers expected");
  fields_ = mesh_->map_buffers({a, b});  // collective
}

HaloIOArgs FusedHalo::io(int64_t step, bool primed, uintptr_t t2, bool direct_z, bool z_unpack) const {
  HaloIOArgs io{};
  const int64_t eb = elem_;
  const int64_t wh = (step & 1) * half_, rh = ((step + 1) & 1) * half_;
  char* mine = mesh_->arena(mesh_->rank());
  for (int d = 0; d < 3; ++d)
    for (int s = 0; s < 2; ++s) {
      const int r = nb_[d][s];
      if (r == PROC_NULL) continue;
      // My plane next to side s is the halo at side 1-s of that neighbour.
      io.out[d][s] = reinterpret_cast<uintptr_t>(mesh_->arena(r) + (wh + off_[d][1 - s]) * eb);
      if (primed) io.in[d][s] = reinterpret_cast<uintptr_t>(mine + (rh + off_[d][s]) * eb);
    }
  io.zpitch = zp_;
  // Whole-line z-edge stores (HaloIOArgs::zh), explicit per side: allowed
  // where nobody else writes t2's z halo column during the kernel.
  for (int s = 0; s < 2; ++s) io.zh[s] = 1;
  io.z_out_arena = true;
  if (direct_z && z_unpack) fail("FusedHalo: direct z and z unpack are exclusive send modes");
  if (z_unpack)
    for (int s = 0; s < 2; ++s) io.in[2][s] = 0;  // the z halo comes from the field (unpack_z of the last step)
  if (direct_z && (nb_[2][0] != PROC_NULL || nb_[2][1] != PROC_NULL)) {
    if (fields_.empty()) fail("FusedHalo: direct z needs the field buffers (set_fields)");
    const char* mine_t2 = reinterpret_cast<const char*>(t2);
    int k = -1;
    for (int i = 0; i < 2; ++i)
      if (fields_[mesh_->rank()][i] == mine_t2) k = i;
    if (k < 0) fail("FusedHalo: direct z: the output field is not one of the registered buffers");
    const int64_t n1 = n_[1], n2 = n_[2];
    for (int s = 0; s < 2; ++s) {
      const int r = nb_[2][s];
      io.in[2][s] = 0;
      if (r == PROC_NULL) continue;
      // My z=1 (side 0) is the neighbour's z=n2-1 halo, my z=n2-2 its z=0;
      // + n2 absorbs the kernel's (y-1) row index.
      const int64_t col = (s == 0 ? n2 - 1 : 0) + n2;
      io.out[2][s] = reinterpret_cast<uintptr_t>(fields_.at(r).at(k) + col * eb);
      io.zh[s] = 0;  // this side's halo column receives the neighbour's direct-z stores during the kernel
    }
    io.zpitch = n1 * n2;
    io.zrow = n2;
    io.z_out_arena = false;
  }
  return io;
}

void FusedHalo::unpack_z(int64_t step, uintptr_t t2, hipStream_t stream, bool wait) const {
  // My arena half (step & 1) holds, at region off_[2][s], the z plane the
  // neighbour at side s computed in its step `step` (layout x*zp + (y-1),
  // x in [1, n0-2], y in [1, n1-2]): my z halo at side s (z = 0 / n2-1) of
  // t2 for those rows - the only rows of the halo column a sweep reads.
  const int64_t n0 = n_[0], n1 = n_[1], n2 = n_[2], eb = elem_;
  const char* mine = mesh_->arena(mesh_->rank()) + (step & 1) * half_ * eb;
  std::vector<Copy2D> cs;
  for (int s = 0; s < 2; ++s) {
    if (nb_[2][s] == PROC_NULL) continue;
    const int64_t col = s == 0 ? 0 : n2 - 1;
    Copy2D c;
    c.src = mine + (off_[2][s] + 1 * zp_) * eb;
    c.dst = reinterpret_cast<char*>(t2) + ((1 * n1 + 1) * n2 + col) * eb;
    c.n_outer = n0 - 2;
    c.n_inner = n1 - 2;
    c.src_so = zp_;
    c.src_si = 1;
    c.dst_so = n1 * n2;
    c.dst_si = n2;
    cs.push_back(c);
  }
  CopyWait w;
  if (wait) {
    // in-kernel step sync: no sync kernel ran since the stencil, whose last
    // exchanging wave advanced EPOCH; the z senders' ARRIVED for that step
    // orders this unpack after their sends (docs/COHERENCE.md, z unpack)
    w.flags = sync_.my_flags;
    w.timeout_ticks = sync_.timeout_ticks;
    for (int s = 0; s < 2; ++s) {
      const int r = nb_[2][s];
      if (r == PROC_NULL) continue;
      if (w.n == 1 && w.rank[0] == r) continue;  // both z sides one peer (dims 2, periodic)
      w.rank[w.n++] = r;
    }
  }
  launch_copy2d(cs, static_cast<int>(eb), stream, false, ParityShift{}, w);
}

void FusedHalo::step(const DiffusionArgs& a, int variant, int mode, int64_t step, bool primed,
                     hipStream_t stream, bool entry) {
  for (int d = 0; d < 3; ++d)
    if (a.n[d] != n_[d]) fail("FusedHalo.step: field shape does not match the fused halo's local grid");
  if (a.elem_bytes != elem_) fail("FusedHalo.step: field dtype does not match the fused halo");
  if (entry) sync(stream);  // entry barrier (fused.hpp)
  const bool zu = (mode & Z_UNPACK) != 0 && (nb_[2][0] != PROC_NULL || nb_[2][1] != PROC_NULL);
  if (zu && (mode & 4)) fail("FusedHalo.step: send mode bits 4 (direct z) and 64 (z unpack) are exclusive");
  HaloIOArgs x = io(step, primed, a.t2, (mode & 4) != 0, zu);
  // Step synchronisation: the 1-wave sync kernel after the stencil (default:
  // rehearsed with 8 ranks, and as fast as the in-kernel form,
  // profiles/r3_boxes/), or inside the kernel (put.hpp StepSync) with send
  // mode bit 16 - a separately validated candidate of the bench's A/B, never
  // where ranks share a GPU (its waiting waves can hold the CUs a co-resident
  // rank's kernel needs: the forced 8-rank shared-GPU rehearsal timed out).
  // IGG_FUSED_SYNC_KERNEL / set_step_sync override both.
  bool used = false;
  // (z unpack with the in-kernel form: the unpack kernel itself waits for the
  // z senders' ARRIVED of this step before it reads the arena)
  if (in_kernel_sync(mode) && sync_.n_out > 0) {  // no neighbour: nothing to synchronise in the kernel
    x.sync = step_sync_from(sync_);
    x.sync_used = &used;
  }
  // the kernel form: z unpack = the no-z-receive form (bit 4's kernel) with
  // the z sends into the arena (x.out[2], zrow 1)
  const int kmode = (mode & ~(IN_KERNEL_SYNC | Z_UNPACK)) | (zu ? 4 : 0);
  launch_diffusion3d_fused(a, x, variant, kmode, stream);
  if (!used) sync(stream);
  if (zu) unpack_z(step, a.t2, stream, used);
  open_ = used;
}

void FusedHalo::sync(hipStream_t stream) const { launch_put_sync(sync_, stream); }

void FusedHalo::drain(hipStream_t stream) {
  if (open_) sync(stream);
  open_ = false;
}

bool FusedHalo::in_kernel_sync(int mode) const {
  if (sync_mode_ >= 0) return sync_mode_ == 0;
  return step_sync_in_kernel(mesh_->shares_device(), (mode & IN_KERNEL_SYNC) != 0);
}

}  // namespace igg
