// Halo exchange engine.
//
// Reference behaviour reproduced (ImplicitGlobalGrid.jl):
//   * ol(dim,A) = overlaps[dim] + size(A,dim) - nxyz[dim]; a field has a halo in
//     `dim` iff ol >= 2 (src/shared.jl:94, src/update_halo.jl:370,429,809).
//   * The halo is one plane per side whatever the overlap; send planes are
//     ol-1 (left) and size-ol (right), receive planes 0 and size-1, 0-based
//     (sendranges/recvranges, src/update_halo.jl:544-563).
//   * Dimensions are processed strictly x -> y -> z; each face spans the full
//     extent of the other dimensions so edges/corners come out right without
//     diagonal messages (src/update_halo.jl:40).
//   * Missing neighbours (PROC_NULL) are skipped; a dimension whose two
//     neighbours are this rank is exchanged locally (src/update_halo.jl:57-63);
//     one-sided self neighbours are an error (:64-65).
//   * Buffers: one send + one recv buffer per field position and side, sized by
//     the largest face (product of all but the smallest extent), rounded up to
//     32 elements, grow-only, reused across dimensions and element types
//     (src/update_halo.jl:150-210).
// MI355X-first differences: all faces of a dimension are packed by ONE kernel
// launch, moved by ONE RCCL group, unpacked by ONE launch; contiguous faces are
// sent/received in place (zero-copy, no pack/unpack); the self-periodic case is
// ONE in-place plane-copy launch with no buffers; everything is stream-ordered
// (no host synchronisation), so an exchange can be captured in a hipGraph.
#pragma once

#include <array>
#include <cstdint>
#include <memory>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "igg/comm.hpp"
#include "igg/peer.hpp"
#include "igg/copy.hpp"
#include "igg/topology.hpp"

namespace igg {

struct Field {
  uintptr_t ptr = 0;
  int ndims = 0;
  Int3 size{1, 1, 1};
  Int3 stride{1, 1, 1};  // in elements
  int elem_bytes = 0;
  bool device = false;
};

// Index of direction v in {-1,0,1}^3 (13 = centre).
inline int dir_key(int vx, int vy, int vz) { return (vx + 1) * 9 + (vy + 1) * 3 + (vz + 1); }

struct GridInfo {
  int64_t me = 0, nprocs = 1;
  Int3 nxyz{1, 1, 1};
  Int3 overlaps{2, 2, 2};
  std::array<Int3, NNEIGHBORS> neighbors{{{PROC_NULL, PROC_NULL, PROC_NULL},
                                          {PROC_NULL, PROC_NULL, PROC_NULL}}};
  // Rank at coords + disp*v for every direction v (dir_key order), PROC_NULL
  // where it leaves a non-periodic grid. Needed by the one-phase exchange.
  std::array<int64_t, 27> peers{};
  bool has_peers = false;
};

// Halo update schedule.
//   Sequential: x -> y -> z, faces only (the reference's algorithm).
//   OnePhase:   all faces, edges and corners as independent messages in ONE
//               pack launch / ONE communication group / ONE unpack launch;
//               bitwise the same result (see halo.cpp). On a fully connected
//               xGMI node every peer is one hop, so the 3 sequential latency
//               phases collapse into 1 and messages to distinct peers use
//               distinct links concurrently.
//   Auto:       OnePhase when a remote peer exists, else Sequential.
enum class HaloMode : int { Sequential = 0, OnePhase = 1, Auto = 2 };

// How the sequential schedule moves the strided faces of one dimension on the
// GPU (the reference packs with write_d2x!/read_x2d! kernels and, for dims
// 2/3 without GPU-aware MPI, with strided 3-D memcpys: src/update_halo.jl:
// 432-465, 628-649).
//   Kernel:   one batched copy2d launch for every face of every field.
//   Memcpy2D: hipMemcpy2DAsync (SDMA/blit) per face whose rows are
//             contiguous on both sides; other faces still use the kernel.
enum class PackMode : int { Kernel = 0, Memcpy2D = 1 };

// A face (one plane of a field orthogonal to `dim`) as a strided 2-D region.
struct Face {
  char* base;
  int64_t n_outer, n_inner, s_outer, s_inner;
  bool contiguous;
  size_t bytes;
};

// Half-open index box of a field.
struct Region {
  int64_t lo[3], hi[3];
  int64_t count() const { return (hi[0] - lo[0]) * (hi[1] - lo[1]) * (hi[2] - lo[2]); }
};

// A box with at most two non-singleton extents as a strided 2-D region.
Face region_face(const Field& f, const Region& r);

int64_t ol(const GridInfo& g, int dim, const Field& f);
int64_t max_halo_elems(const Field& f);
int64_t send_index(const GridInfo& g, int side, int dim, const Field& f);
int64_t recv_index(const GridInfo& g, int side, int dim, const Field& f);
Face face(const Field& f, int dim, int64_t index);

// Grow-only per (field slot, side) send/recv byte buffers; separate host and
// device pools (test hooks: capacities are observable).
class BufferPool {
 public:
  ~BufferPool();
  void ensure(const std::vector<Field>& fields, bool device);
  char* send(size_t slot, int side, bool device) const;
  char* recv(size_t slot, int side, bool device) const;
  size_t nslots(bool device) const { return (device ? dev_ : host_).size(); }
  size_t capacity(size_t slot, bool device) const;
  bool allocated(bool device) const { return device ? dev_alloc_ : host_alloc_; }
  // Grow-only send/recv arenas of the one-phase exchange.
  char* arena(int which, size_t bytes, bool device);
  void free_all();
  // While frozen (during a hipGraph capture) any growth is an error.
  void set_frozen(bool f) { frozen_ = f; }

 private:
  bool frozen_ = false;
  struct Buf { char* p = nullptr; size_t bytes = 0; };
  struct Slot { Buf send[NNEIGHBORS], recv[NNEIGHBORS]; };
  void grow(Buf& b, size_t bytes, bool device);
  void release(Buf& b, bool device);
  std::vector<Slot> host_, dev_;
  Buf arena_[2][2];  // [device][send/recv]
  bool host_alloc_ = false, dev_alloc_ = false;
};

class HaloEngine {
 public:
  explicit HaloEngine(const GridInfo& g);
  ~HaloEngine();
  // Transports for host (CPU) and device (GPU) fields respectively.
  void set_transport(std::shared_ptr<Transport> t, bool device) {
    (device ? dev_transport_ : host_transport_) = std::move(t);
  }
  std::shared_ptr<Transport> transport(bool device) const {
    return device ? dev_transport_ : host_transport_;
  }
  GridInfo& grid() { return grid_; }
  BufferPool& pool() { return pool_; }

  // Full update_halo! of `fields` (validated by the caller), stream-ordered.
  // `mode_override` >= 0 forces a schedule for this call (a measured per-field-
  // set choice of parallel/halo.py); -1 uses set_mode / Auto.
  void exchange(const std::vector<Field>& fields, hipStream_t stream, int mode_override = -1);
  // Only the dimension `dim` (0-based); used by tests and pipelined apps.
  void exchange_dim(const std::vector<Field>& fields, int dim, hipStream_t stream);
  void set_mode(HaloMode m) { mode_ = m; }
  HaloMode mode() const { return mode_; }
  void set_pack_mode(int dim, PackMode m) { pack_mode_.at(static_cast<size_t>(dim)) = m; }
  PackMode pack_mode(int dim) const { return pack_mode_.at(static_cast<size_t>(dim)); }
  // Mode the next exchange of `fields` would use (Auto resolved: Sequential,
  // the schedule measured faster by default; halo.py measures per field set).
  HaloMode resolved_mode(const std::vector<Field>& fields) const;
  int last_message_count() const { return last_msgs_; }

 private:
  void exchange_dim_impl(const std::vector<Field>& fields, int dim, bool device,
                         hipStream_t stream);
  void exchange_onephase(const std::vector<Field>& fields, bool device, hipStream_t stream);
  void exchange_put(const std::vector<Field>& fields, hipStream_t stream, PeerMesh& mesh);
  // Receive / send regions of the one-phase message with receiver-side
  // direction `key`; false if the field has no such message.
  bool dir_regions(const Field& f, int key, Region& rr, Region& sr) const;
  bool active(const Field& f, int d) const;
  GridInfo grid_;
  HaloMode mode_ = HaloMode::Auto;
  std::array<PackMode, NDIMS> pack_mode_{PackMode::Kernel, PackMode::Kernel, PackMode::Kernel};
  int last_msgs_ = 0;
  BufferPool pool_;
  std::shared_ptr<Transport> host_transport_, dev_transport_;
  hipEvent_t done_ = nullptr;
  hipStream_t last_stream_ = nullptr;
  bool have_event_ = false;
  // IGG_DEBUG_SYNC: drain and check the stream after every phase, naming it.
  void debug_phase(hipStream_t stream, bool device, const char* phase) const;
  bool debug_sync_ = false;
  // Put transport bookkeeping: exchanges issued, senders of the previous one.
  uint64_t put_count_ = 0;
  std::vector<int> prev_in_;
};

}  // namespace igg
