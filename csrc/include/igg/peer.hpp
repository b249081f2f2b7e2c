// Put transport: one-sided halo exchange between the GPUs of a node through
// IPC-mapped receive arenas, with command-processor flag signalling.
//
// Per exchange (epoch k, arena half p = k & 1), for every message S -> R with
// receiver-side direction key u (dir_key order, halo.hpp; S = R + u):
//   S: wait  S.freed[26-u] >= k-2   (R finished unpacking exchange k-2, the
//                                     last one that used half p of its arena)
//   S: put kernel: S's send region -> R.arena[p][slot(u, field)] (xGMI stores)
//   S: write R.arrived[u] = k
//   R: wait  R.arrived[u] >= k ; unpack kernel from R.arena[p]
//   R: write N.freed[26-u'] = k for EVERY neighbour N = R + u' (also those
//      that sent nothing this time: the next call may use another layout)
// Slots depend only on field shapes, so sender and receiver agree without
// negotiation; the two halves let exchange k+1's puts land while exchange k is
// still being unpacked. Waits/writes are
// hipStreamWaitValue64/WriteValue64 on the caller's stream; nothing blocks the
// host and no workgroup spins on a flag while the stencil owns the CUs.
//
// Arenas and flags are uncached device memory (coherent across devices: remote
// stores and CP writes land in HBM, local reads bypass L2), exported once with
// hipIpcGetMemHandle and re-exported (collectively) only when an arena grows.
#pragma once

#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "igg/comm.hpp"

namespace igg {

class PeerMesh {
 public:
  // allgather(bytes) -> bytes of every rank (rank order); collective over the mesh.
  using AllGather = std::function<std::vector<std::string>(const std::string&)>;
  static constexpr int NFLAGS = 64;  // [0,27): arrived[u], [32,59): freed[u]
  static constexpr int ARRIVED = 0, FREED = 32;

  PeerMesh(int rank, int nranks, AllGather allgather);
  ~PeerMesh();
  PeerMesh(const PeerMesh&) = delete;
  PeerMesh& operator=(const PeerMesh&) = delete;

  int rank() const { return rank_; }
  int nranks() const { return nranks_; }
  // Collective: every rank must call with the same `bytes` at the same point.
  void ensure_arena(size_t bytes);
  size_t arena_bytes() const { return arena_bytes_; }
  char* arena(int r) const { return r == rank_ ? arena_ : peer_arena_.at(r); }
  uint64_t* flags(int r) const { return r == rank_ ? flags_ : peer_flags_.at(r); }
  uint64_t next_epoch() { return ++epoch_; }
  uint64_t epoch() const { return epoch_; }
  // Collective teardown (also run by the destructor without the collectives).
  void close();

 private:
  void exchange_handles(bool flags_too);
  int rank_, nranks_;
  AllGather allgather_;
  uint64_t* flags_ = nullptr;
  char* arena_ = nullptr;
  size_t arena_bytes_ = 0;
  std::vector<uint64_t*> peer_flags_;
  std::vector<char*> peer_arena_;
  uint64_t epoch_ = 0;
  bool closed_ = false;
};

class PutTransport : public Transport {
 public:
  explicit PutTransport(std::shared_ptr<PeerMesh> mesh) : mesh_(std::move(mesh)) {}
  bool device_capable() const override { return true; }
  bool host_capable() const override { return false; }
  std::string name() const override { return "put"; }
  // Two-sided P2P is not expressible one-sided without the peer's addresses:
  // the halo engine drives PutTransport through its own one-phase put path.
  void exchange(const std::vector<P2POp>&, const std::vector<P2POp>&, bool, hipStream_t) override {
    fail("the 'put' transport only supports full halo updates (update_halo!), not raw P2P ops.");
  }
  PeerMesh& mesh() { return *mesh_; }
  std::shared_ptr<PeerMesh> mesh_ptr() const { return mesh_; }

 private:
  std::shared_ptr<PeerMesh> mesh_;
};

}  // namespace igg
