// PeerMesh: IPC-mapped peer arenas and epoch flags of the one-sided "put" transport.
// MI355X-specific replacement of the reference's MPI point-to-point layer
// (update_halo.jl:713-753); no counterpart exists in the reference.
#include "igg/peer.hpp"
#include "igg/fault.hpp"

#include "igg/ipc.hpp"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <ios>
#include <map>

#include <unistd.h>

namespace igg {

PeerMesh::PeerMesh(int rank, int nranks, AllGather allgather)
    : rank_(rank), nranks_(nranks), allgather_(std::move(allgather)) {
  if (nranks < 1 || rank < 0 || rank >= nranks) fail("PeerMesh: invalid rank ", rank, " of ", nranks);
  peer_flags_.assign(nranks, nullptr);
  peer_arena_.assign(nranks, nullptr);
  flags_ = static_cast<uint64_t*>(ipc_malloc(PutFlags::words(nranks) * sizeof(uint64_t), MemKind::Uncached));
  IGG_HIP_CHECK(hipStreamCreateWithFlags(&side_, hipStreamNonBlocking));
  double seconds = 120.0;
  if (const char* t = std::getenv("IGG_PUT_TIMEOUT")) seconds = std::atof(t);
  timeout_ticks_ = put_timeout_ticks(seconds);
  if (const char* k = std::getenv("IGG_PUT_ARENA_KIND")) arena_kind_ = static_cast<MemKind>(std::atoi(k));
  exchange_handles(true);
  {
    // Device identity: host name + PCI bus id of the current device.
    int dev = 0;
    char bus[64] = {0}, host[256] = {0};
    IGG_HIP_CHECK(hipGetDevice(&dev));
    IGG_HIP_CHECK(hipDeviceGetPCIBusId(bus, sizeof(bus) - 1, dev));
    (void)gethostname(host, sizeof(host) - 1);
    const std::string id = std::string(host) + "/" + bus;
    const std::vector<std::string> ids = allgather_(id);
    // Collective by construction: every rank sees the same id list, so if ANY
    // two ranks share a device, every rank treats the mesh as shared (the
    // step-sync form must be the same on all ranks, igg/fused.hpp; a rank-local
    // answer split the bench's in-kernel-sync A/B gate when ranks shared GPUs
    // unevenly, e.g. 3 ranks on 2 GPUs).
    for (int r = 0; r < static_cast<int>(ids.size()) && !shares_device_; ++r)
      for (int q = r + 1; q < static_cast<int>(ids.size()); ++q)
        if (ids[r] == ids[q]) {
          shares_device_ = true;
          break;
        }
  }
  if (const char* m = std::getenv("IGG_PUT_ARENA_MIN")) {
    const long long mb = std::atoll(m);
    if (mb > 0) ensure_arena(static_cast<size_t>(mb) << 20);  // collective
  }
}

uint64_t PeerMesh::read_flag(int idx) const {
  if (idx < 0 || idx >= flag_words() || !flags_) fail("PeerMesh.read_flag: index ", idx, " out of range");
  uint64_t v = 0;
  IGG_HIP_CHECK(hipMemcpyAsync(&v, flags_ + idx, 8, hipMemcpyDeviceToHost, side_));
  IGG_HIP_CHECK(hipStreamSynchronize(side_));
  return v;
}

void PeerMesh::check_error() const {
  if (!flags_) return;
  const uint64_t e = read_flag(PutFlags::ERROR);
  if (e != 0)
    fail("put transport: a synchronisation kernel timed out waiting for a peer (code 0x", std::hex, e,
         std::dec, "); the halo data of that exchange is invalid. Raise IGG_PUT_TIMEOUT if peers are "
         "legitimately slow.");
}

void PeerMesh::clear_error() {
  if (!flags_) return;
  IGG_HIP_CHECK(hipMemsetAsync(flags_ + PutFlags::ERROR, 0, 8, side_));
  IGG_HIP_CHECK(hipStreamSynchronize(side_));
}

PeerMesh::~PeerMesh() {
  // Non-collective fallback: unmap peers, free own memory (the collective
  // close() should have run first; by then these are no-ops).
  for (int r = 0; r < nranks_; ++r) {
    if (r == rank_) continue;
    if (peer_arena_[r]) (void)hipIpcCloseMemHandle(peer_arena_[r]);
    if (peer_flags_[r]) (void)hipIpcCloseMemHandle(peer_flags_[r]);
    peer_arena_[r] = nullptr;
    peer_flags_[r] = nullptr;
  }
  for (void* p : mapped_) (void)hipIpcCloseMemHandle(p);
  mapped_.clear();
  if (arena_) (void)hipFree(arena_);
  for (char* a : retired_) (void)hipFree(a);
  if (flags_) (void)hipFree(flags_);
  if (side_) (void)hipStreamDestroy(side_);
  arena_ = nullptr;
  flags_ = nullptr;
  side_ = nullptr;
}

void PeerMesh::exchange_handles(bool flags_too) {
  std::string mine;
  if (flags_too) mine += ipc_get_handle(flags_);
  if (arena_) mine += ipc_get_handle(arena_);
  const std::vector<std::string> all = allgather_(mine);
  if (static_cast<int>(all.size()) != nranks_) fail("PeerMesh: allgather returned ", all.size(), " entries");
  const size_t hb = sizeof(hipIpcMemHandle_t);
  std::string error;
  try {
    inject_fail("peer_map");  // tests: a rank that cannot map its peers (IGG_INJECT_FAIL)
    for (int r = 0; r < nranks_; ++r) {
      if (r == rank_) continue;
      const std::string& h = all[r];
      size_t pos = 0;
      if (flags_too) {
        peer_flags_[r] = static_cast<uint64_t*>(ipc_open(h.substr(pos, hb)));
        pos += hb;
      }
      if (arena_) peer_arena_[r] = static_cast<char*>(ipc_open(h.substr(pos, hb)));
    }
  } catch (const Error& e) {
    error = e.what();
  }
  // Agree on the outcome: a rank that cannot map its peers must not leave the
  // others waiting in the next collective, so every rank raises together.
  const std::vector<std::string> status = allgather_(error.empty() ? std::string("1") : std::string("0"));
  for (int r = 0; r < static_cast<int>(status.size()); ++r)
    if (status[r] != "1")
      fail("PeerMesh: rank ", r, " could not map the peer memory of the mesh",
           error.empty() ? std::string() : std::string(" (here: ") + error + ")");
}

void PeerMesh::ensure_arena(size_t bytes) {
  if (closed_) fail("PeerMesh: used after close()");
  if (bytes <= arena_bytes_) return;
  // Geometric growth with a floor: a regrowth is a collective re-export, so
  // make it rare (one field of 1024^3 f32 needs 2 x 24 MiB).
  static const size_t floor_bytes = [] {
    const char* f = std::getenv("IGG_PUT_ARENA_FLOOR_MB");  // tests lower it to exercise regrowth
    const long long mb = f ? std::atoll(f) : 64;
    return static_cast<size_t>(mb > 0 ? mb : 1) << 20;
  }();
  if (bytes >= IPC_MAX_BYTES)  // every rank computes the same size: all fail together
    fail("PeerMesh: a receive arena of ", bytes >> 20, " MiB exceeds the 2 GiB IPC limit (ipc.hpp IPC_MAX_BYTES)");
  bytes = static_cast<size_t>(round_up(static_cast<int64_t>(std::max({bytes, 2 * arena_bytes_, floor_bytes})), 1 << 20));
  bytes = std::min(bytes, IPC_MAX_BYTES - (size_t{1} << 20));  // geometric growth stays exportable
  // Every rank drains its own puts/unpacks into the old arenas, then agrees
  // (allgather = barrier) before anyone unmaps them.
  IGG_HIP_CHECK(hipDeviceSynchronize());
  (void)allgather_(std::string());
  for (int r = 0; r < nranks_; ++r)
    if (r != rank_ && peer_arena_[r]) {
      ipc_close(peer_arena_[r]);
      peer_arena_[r] = nullptr;
    }
  (void)allgather_(std::string());
  // The old arena is retired, not freed, until close(): a freed allocation's
  // address can come back for the new one, and an IPC export of an allocation
  // at a reused address was observed to map the OLD memory in the peers
  // (every message of that sender lost, deterministically for the rest of the
  // run; also hipIpcGetMemHandle 'invalid argument') on MI355X / ROCm 7.2
  // (profiles/r3_put_arena/). Keeping it alive makes every export address new.
  if (arena_) retired_.push_back(arena_);
  arena_ = static_cast<char*>(ipc_malloc(bytes, arena_kind_));
  arena_bytes_ = bytes;
  exchange_handles(false);
}

void PeerMesh::unmap_buffers() {
  for (void* p : mapped_) ipc_close(p);
  mapped_.clear();
}

std::vector<std::vector<char*>> PeerMesh::map_buffers(const std::vector<uintptr_t>& mine) {
  if (closed_) fail("PeerMesh: used after close()");
  // Old mappings go first: every rank drains its work into them, then agrees.
  if (!mapped_.empty()) {
    IGG_HIP_CHECK(hipDeviceSynchronize());
    (void)allgather_(std::string());
    unmap_buffers();
  }
  // Record per buffer: handle of its allocation + offset inside it, behind a
  // one-byte status. A rank that cannot export its buffers still joins the
  // allgather (status 0) so every rank fails together instead of the others
  // blocking in the collective.
  const size_t hb = sizeof(hipIpcMemHandle_t);
  std::string rec(1, '1'), error;
  try {
    if (nranks_ > 1)
      for (uintptr_t p : mine) {
        void* base = nullptr;
        size_t size = 0;
        IGG_HIP_CHECK(hipMemGetAddressRange(&base, &size, reinterpret_cast<void*>(p)));
        const uint64_t off = p - reinterpret_cast<uintptr_t>(base);
        rec += ipc_get_handle(base);
        rec.append(reinterpret_cast<const char*>(&off), 8);
      }
  } catch (const Error& e) {
    error = e.what();
    rec.assign(1, '0');
  }
  std::vector<std::string> all = allgather_(rec);
  if (static_cast<int>(all.size()) != nranks_) fail("PeerMesh: allgather returned ", all.size(), " entries");
  for (int r = 0; r < nranks_; ++r)
    if (all[r].empty() || all[r][0] != '1')
      fail("PeerMesh: rank ", r, " could not export its buffers",
           error.empty() ? std::string() : std::string(" (here: ") + error + ")");
  for (auto& a : all) a.erase(0, 1);
  std::vector<std::vector<char*>> out(nranks_);
  try {
    for (int r = 0; r < nranks_; ++r) {
      if (r == rank_) {
        for (uintptr_t p : mine) out[r].push_back(reinterpret_cast<char*>(p));
        continue;
      }
      const std::string& h = all[r];
      if (h.size() != mine.size() * (hb + 8)) fail("PeerMesh.map_buffers: rank ", r, " passed a different count");
      // One mapping per distinct allocation (two buffers of one allocation
      // share a handle; opening a handle twice in a process is not allowed).
      std::map<std::string, char*> opened;
      for (size_t i = 0; i < mine.size(); ++i) {
        const std::string key = h.substr(i * (hb + 8), hb);
        uint64_t off = 0;
        std::memcpy(&off, h.data() + i * (hb + 8) + hb, 8);
        auto it = opened.find(key);
        if (it == opened.end()) {
          char* base = static_cast<char*>(ipc_open(key));
          mapped_.push_back(base);
          it = opened.emplace(key, base).first;
        }
        out[r].push_back(it->second + off);
      }
    }
  } catch (const Error& e) {
    error = e.what();
  }
  const std::vector<std::string> status = allgather_(error.empty() ? std::string("1") : std::string("0"));
  for (int r = 0; r < static_cast<int>(status.size()); ++r)
    if (status[r] != "1")
      fail("PeerMesh: rank ", r, " could not map the peers' buffers",
           error.empty() ? std::string() : std::string(" (here: ") + error + ")");
  return out;
}

void PeerMesh::close() {
  if (closed_) return;
  IGG_HIP_CHECK(hipDeviceSynchronize());
  (void)allgather_(std::string());
  unmap_buffers();
  for (int r = 0; r < nranks_; ++r) {
    if (r == rank_) continue;
    if (peer_arena_[r]) ipc_close(peer_arena_[r]);
    if (peer_flags_[r]) ipc_close(peer_flags_[r]);
    peer_arena_[r] = nullptr;
    peer_flags_[r] = nullptr;
  }
  (void)allgather_(std::string());
  if (arena_) ipc_free(arena_);
  for (char* a : retired_) ipc_free(a);
  retired_.clear();
  if (flags_) ipc_free(flags_);
  arena_ = nullptr;
  flags_ = nullptr;
  arena_bytes_ = 0;
  closed_ = true;
}

}  // namespace igg
