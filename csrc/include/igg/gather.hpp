// Device-resident gather-to-root (gather!, src/gather.jl:25-65).
//
// Reference: non-root ranks Isend their whole local array; root Irecv's each
// block into a cached grow-only flat buffer, copies its own block, Waitall's,
// then scatters the blocks into the global layout with a host triple loop
// (gather.jl:60-63). Here: one RCCL group receives all blocks straight into a
// grow-only device buffer and a HIP reorder kernel writes the global layout
// (block from coords (c0,c1,c2) -> A_global[c0*s0:(c0+1)*s0, ...]).
#pragma once

#include <cstdint>
#include <functional>
#include <string>
#include <utility>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "igg/comm.hpp"
#include "igg/halo.hpp"

namespace igg {

// Reorder `nprocs` contiguous blocks of extent `s` (rank order = row-major
// Cartesian coords over `dims`) from `src` into the C-contiguous global array
// `dst` of extent dims*s.
void launch_gather_reorder(const void* src, void* dst, const Int3& s, const Int3& dims,
                           int elem_bytes, hipStream_t stream);

class Gatherer {
 public:
  ~Gatherer() { free(); }
  // `a` must be a C-contiguous device field; `dst` (device, C-contiguous
  // dims*size) is only used on `root`.
  void gather(const Field& a, void* dst, int root, const Int3& dims, RcclComm& comm,
              hipStream_t stream);
  size_t capacity() const { return bytes_; }
  void free();

 private:
  char* buf_ = nullptr;
  size_t bytes_ = 0;
};

// Non-blocking gather by root pull (MI355X copy engines), stream-ordered.
// start(): every rank records an interprocess event on its own stream where
// `a` is final (no host-side drain of the GPU) and publishes that event's IPC
// handle plus the IPC handle + offset of the allocation holding `a` (the root
// publishes the handles of its per-copy-stream "done" events instead); the
// root makes every copy stream it uses wait on its own event first (earlier
// work of its stream on `dst`, e.g. a zero fill, stays ahead of every copy),
// then on the event of the rank whose block it pulls, and enqueues ONE 3-D copy
// per block from the (peer-mapped) block straight into its place in `dst`
// (hipMemcpy3DAsync: rows of s2 elements at the global pitch; a P2P copy over
// xGMI for peer blocks), then records its done events. No staging buffer and
// no reorder pass: the global array is written once. Blocks are spread over up
// to 8 copy streams so the transfers from different peers (different xGMI
// links) run concurrently. start() returns immediately: the application keeps
// computing while the data moves.
// wait(): nothing blocks on the GPU. The root orders its stream after its done
// events; a host rendezvous (the done events of this gather are recorded before
// it) lets every other rank order ITS stream after the root's done events
// (opened once through IPC), so its later work on `a` (MPI_Igather semantics:
// `a` is read-only until then) queues behind the pulls on the device.
// Peer mappings are cached per rank and closed when that rank's allocation
// changes (after the copy streams drained) or at free().
// Large blocks: an IPC handle of an allocation of 2 GiB or more cannot be
// opened on this runtime (ipc.hpp IPC_MAX_BYTES). A rank whose allocation
// holding `a` is that large (or, for tests, larger than IGG_GATHER_CHUNK_BYTES)
// first copies `a` on its stream into grow-only staging chunks of whole
// x-planes, each its own exportable allocation (< 1 GiB by default), and
// publishes the chunks' handles; the root pulls each chunk as a 3-D sub-block.
// The staging copy precedes the ready event, and the next gather's copy
// follows wait()'s ordering behind the root's pulls, like `a` itself.
class PullGatherer {
 public:
  using AllGather = std::function<std::vector<std::string>(const std::string&)>;
  PullGatherer(int rank, int nranks, AllGather allgather);
  ~PullGatherer();
  PullGatherer(const PullGatherer&) = delete;
  PullGatherer& operator=(const PullGatherer&) = delete;
  // `dst` (root only): C-contiguous device array of extent dims*size; `stream`:
  // the stream on which `a` is produced (and, on the root, dst is consumed).
  // `snapshot`: every rank copies `a` now, on `stream` (non-root ranks into
  // their exportable staging chunks, the root straight into its place in
  // dst), so `a` may be modified as soon as start() returns - the copy is the
  // only serial part of the gather; the pulls of the chunks overlap whatever
  // the ranks do next.
  void start(const Field& a, void* dst, int root, const Int3& dims, hipStream_t stream, bool snapshot = false);
  void wait(hipStream_t stream);
  bool pending() const { return pending_; }
  // "root", "ipc", "chunks", "vmm", "dmabuf" or "vmm-staging": how start() published this rank's block
  const char* last_kind() const { return last_kind_; }
  void free();

 private:
  void ensure_streams();
  int rank_, nranks_;
  AllGather allgather_;
  std::vector<hipStream_t> side_;  // copy streams (root)
  std::vector<hipEvent_t> done_;   // one per copy stream (interprocess)
  hipEvent_t ready_ = nullptr;     // interprocess: `a` final on the caller's stream
  std::vector<std::string> peer_key_;  // IPC event handle bytes per rank (cache key)
  std::vector<hipEvent_t> peer_ev_;    // opened peer events (root)
  std::vector<std::string> root_key_;  // non-root: the root's done-event handles (cache keys)
  std::vector<hipEvent_t> root_done_;  // non-root: the root's done events, opened
  // root: per rank, per published buffer (one: `a`'s allocation; or its
  // staging chunks) the (handle, mapped base)
  std::vector<std::vector<std::pair<std::string, void*>>> mapped_;
  std::vector<char*> stage_;  // own staging chunks (a large `a`), grow-only
  size_t stage_bytes_ = 0;    // bytes of each staging chunk
  std::vector<char*> retired_;  // grown-out staging chunks, freed at free() (never re-exported addresses)
  // HIP VMM exports (vmm.hpp; round 6): an `a` living in a MemKind::Vmm
  // allocation is published as-is at ANY size ('V' record: a socket name the
  // root fetches the allocation's file descriptor from, once, plus size and
  // offset), and a large snapshot is staged into ONE grow-only VMM buffer
  // instead of IPC chunks. The root maps each once (cached by socket name)
  // and pulls it as one block.
  // Also published this way: an `a` in an ordinary hipMalloc allocation of
  // 2 GiB or more (above the IPC limit), as a dma-buf of the whole allocation
  // (range_export_fd; IGG_GATHER_DMABUF=0: the VMM staging copy instead). A
  // freed-and-reallocated range at the same address is told apart by its
  // runtime buffer id: a new id makes a new export (new name: the root maps
  // again). The descriptor is closed once served (it holds a reference to the
  // allocation) and exported again if the root asks again.
  struct VmmExport {
    void* base = nullptr;
    int listener = -1, fd = -1;
    std::string name;
    bool dmabuf = false;
    uint64_t buffer_id = 0;
  };
  std::vector<VmmExport> vexp_;
  int cur_vexp_ = -1;           // the export published by the pending gather (non-root)
  void* vstage_ = nullptr;      // VMM staging buffer (large snapshots)
  size_t vstage_bytes_ = 0;
  std::vector<void*> vretired_;
  std::vector<char> mapped_vmm_;  // root: mapped_[p] holds VMM imports (vmm_free) rather than IPC maps
  std::string vmm_record(void* base, size_t size, uint64_t off, bool dmabuf = false);
  void close_mapped(int p);
  void free_vmm();
  const char* last_kind_ = "";  // how this rank published its block in the last start() (last_kind())
  bool pending_ = false;
  int root_ = 0;
  int used_ = 0;  // copy streams used by the pending gather
};

}  // namespace igg
