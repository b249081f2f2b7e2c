// Put transport: one-sided halo exchange between the GPUs of a node through
// IPC-mapped receive arenas, with command-processor flag signalling.
//
// Protocol (device-driven, no host in the loop; kernels in put.hpp): per
// exchange e every rank bumps its device epoch, signals "consumed e-1" to all
// neighbours, waits until its receivers consumed e-2 (the last exchange that
// used arena half e&1), packs straight into the receivers' arenas (stores over
// xGMI), publishes arrived[me] = e at each receiver, waits for arrived[s] >= e
// of each sender and unpacks from its own arena. Arena slots depend only on
// field shapes, so sender and receiver agree without negotiation; the two
// halves let exchange e+1's puts land while e is still being unpacked.
//
// Memory kinds (the full ordering / coherence argument: docs/COHERENCE.md):
// flag words are uncached (hipDeviceMallocUncached: every access goes to
// memory, polls see a peer's store without any cache maintenance); arenas are
// fine-grained (hipDeviceMallocFinegrained: HIP defines concurrent access by
// other devices while a kernel runs). A writer's stores into a peer arena may
// sit dirty in the writer's XCD L2 (the peer mapping is MTYPE NC there), so
// every storing wave ends with a system-scope release (buffer_wbl2 sc0 sc1)
// before the sync kernel publishes its flag. Both are exported once with
// hipIpcGetMemHandle and re-exported (collectively) only when an arena grows.
#pragma once

#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "igg/comm.hpp"
#include "igg/ipc.hpp"
#include "igg/put.hpp"

namespace igg {

class PeerMesh {
 public:
  // allgather(bytes) -> bytes of every rank (rank order); collective over the mesh.
  using AllGather = std::function<std::vector<std::string>(const std::string&)>;

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
  int flag_words() const { return PutFlags::words(nranks_); }
  // Host read of one of my flag words (side stream; never blocks on halo work).
  uint64_t read_flag(int idx) const;
  // Raises igg::Error if a put-transport kernel timed out waiting for a peer.
  void check_error() const;
  void clear_error();
  int64_t timeout_ticks() const { return timeout_ticks_; }
  // Collective: maps device buffers of every rank (each rank passes its own
  // pointers, the same count everywhere; pointers may lie inside larger
  // allocations, e.g. torch's). Returns out[r][i] = rank r's buffer i in this
  // process (this rank's own pointers as given). The mappings live until
  // close(); mapping again replaces them.
  std::vector<std::vector<char*>> map_buffers(const std::vector<uintptr_t>& mine);
  // Collective teardown (also run by the destructor without the collectives).
  void close();
  // Some other rank of the mesh runs on this rank's GPU (same host and PCI
  // bus id; determined collectively at construction). In-kernel waits for a
  // neighbour are then unsafe: the waiting kernel can hold the compute units
  // the neighbour's kernel needs (put.hpp StepSync).
  bool shares_device() const { return shares_device_; }

 private:
  void exchange_handles(bool flags_too);
  int rank_, nranks_;
  bool shares_device_ = false;
  AllGather allgather_;
  uint64_t* flags_ = nullptr;
  char* arena_ = nullptr;
  size_t arena_bytes_ = 0;
  std::vector<char*> retired_;  // grown-out arenas, freed at close() (never re-exported addresses)
  std::vector<uint64_t*> peer_flags_;
  std::vector<char*> peer_arena_;
  std::vector<void*> mapped_;  // map_buffers() mappings (one per distinct peer allocation)
  void unmap_buffers();
  int64_t timeout_ticks_ = 0;
  // Fine-grained: the fused stencil's halo reads from the arena cost 6 us/step
  // instead of 12 with the uncached kind, whose reads bypass the L2
  // (profiles/r2_arena/; IGG_PUT_ARENA_KIND=3 restores uncached).
  MemKind arena_kind_ = MemKind::FineGrained;
  hipStream_t side_ = nullptr;
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
