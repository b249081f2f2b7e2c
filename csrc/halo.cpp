// Halo exchange engine (see include/igg/halo.hpp for the behavioural contract).
#include "igg/halo.hpp"
#include "igg/ipc.hpp"
#include "igg/trace.hpp"

#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <limits>

#include <hip/hip_runtime_api.h>

namespace igg {

int64_t ol(const GridInfo& g, int dim, const Field& f) {
  return g.overlaps[dim] + (f.size[dim] - g.nxyz[dim]);
}

int64_t max_halo_elems(const Field& f) {
  if (f.ndims <= 1) return 1;
  std::vector<int64_t> s(f.size.begin(), f.size.begin() + f.ndims);
  std::sort(s.begin(), s.end());
  int64_t p = 1;
  for (size_t k = 1; k < s.size(); ++k) p *= s[k];
  return p;
}

static void require_halo(const GridInfo& g, int dim, const Field& f) {
  if (ol(g, dim, f) < 2) fail("Incoherent arguments: ol(A,dim)<2.");
}

int64_t send_index(const GridInfo& g, int side, int dim, const Field& f) {
  require_halo(g, dim, f);
  const int64_t o = ol(g, dim, f);
  return side == 0 ? o - 1 : f.size[dim] - o;
}

int64_t recv_index(const GridInfo& g, int side, int dim, const Field& f) {
  require_halo(g, dim, f);
  return side == 0 ? 0 : f.size[dim] - 1;
}

Face face(const Field& f, int dim, int64_t index) {
  int other[2], k = 0;
  for (int d = 0; d < NDIMS; ++d)
    if (d != dim) other[k++] = d;
  auto key = [&](int d) {
    return f.size[d] > 1 ? f.stride[d] : std::numeric_limits<int64_t>::max();
  };
  // Buffer order = memory order of the plane: the smaller-stride dim is inner
  // (ties -> higher index), so packs read/write coalesced for any dense layout.
  const int inner = key(other[0]) < key(other[1]) ? other[0] : other[1];
  const int outer = inner == other[0] ? other[1] : other[0];
  Face fc{};
  fc.base = reinterpret_cast<char*>(f.ptr) + index * f.stride[dim] * f.elem_bytes;
  fc.n_inner = f.size[inner];
  fc.n_outer = f.size[outer];
  fc.s_inner = fc.n_inner > 1 ? f.stride[inner] : 1;
  fc.s_outer = fc.n_outer > 1 ? f.stride[outer] : fc.n_inner * fc.s_inner;
  fc.contiguous = fc.s_inner == 1 && fc.s_outer == fc.n_inner;
  fc.bytes = static_cast<size_t>(fc.n_outer * fc.n_inner * f.elem_bytes);
  return fc;
}

Face region_face(const Field& f, const Region& r) {
  int ext[2] = {-1, -1}, k = 0;
  for (int d = 0; d < NDIMS; ++d)
    if (r.hi[d] - r.lo[d] > 1) {
      if (k == 2) fail("region_face: region has three non-singleton extents");
      ext[k++] = d;
    }
  Face fc{};
  int64_t off = 0;
  for (int d = 0; d < NDIMS; ++d) off += r.lo[d] * f.stride[d];
  fc.base = reinterpret_cast<char*>(f.ptr) + off * f.elem_bytes;
  int inner = -1, outer = -1;
  if (k == 2) {
    inner = f.stride[ext[0]] < f.stride[ext[1]] ? ext[0] : ext[1];
    outer = inner == ext[0] ? ext[1] : ext[0];
  } else if (k == 1) {
    inner = ext[0];
  }
  fc.n_inner = inner >= 0 ? r.hi[inner] - r.lo[inner] : 1;
  fc.s_inner = inner >= 0 ? f.stride[inner] : 1;
  fc.n_outer = outer >= 0 ? r.hi[outer] - r.lo[outer] : 1;
  fc.s_outer = outer >= 0 ? f.stride[outer] : fc.n_inner * fc.s_inner;
  if (fc.n_inner == 1) fc.s_inner = 1;
  if (fc.n_outer == 1) fc.s_outer = fc.n_inner * fc.s_inner;
  fc.contiguous = fc.s_inner == 1 && fc.s_outer == fc.n_inner;
  fc.bytes = static_cast<size_t>(fc.n_outer * fc.n_inner * f.elem_bytes);
  return fc;
}

// ---------------------------------------------------------------- BufferPool

BufferPool::~BufferPool() { free_all(); }

char* BufferPool::arena(int which, size_t bytes, bool device) {
  Buf& b = arena_[device ? 1 : 0][which];
  if (b.bytes < bytes) grow(b, round_up(static_cast<int64_t>(bytes), 1 << 16), device);
  return b.p;
}

void BufferPool::grow(Buf& b, size_t bytes, bool device) {
  if (b.bytes >= bytes) return;
  if (frozen_)
    fail("update_halo: halo buffers must grow during a hipGraph capture; run one eager "
         "update_halo with the same fields before capturing.");
  release(b, device);
  if (device) {
    IGG_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&b.p), bytes));
    IGG_HIP_CHECK(hipMemset(b.p, 0, bytes));
    // hipMemset runs on the null stream, which does not order against the
    // non-blocking streams torch hands us: finish it before any pack kernel on
    // the caller's stream can write the buffer (growth is rare).
    IGG_HIP_CHECK(hipDeviceSynchronize());
  } else {
    b.p = static_cast<char*>(std::aligned_alloc(64, round_up(bytes, 64)));
    if (!b.p) fail("BufferPool: host allocation of ", bytes, " bytes failed");
    std::fill(b.p, b.p + bytes, 0);
  }
  b.bytes = bytes;
}

void BufferPool::release(Buf& b, bool device) {
  if (!b.p) return;
  if (device) {
    // A buffer may still be referenced by enqueued work: drain first (growth is
    // rare — buffers are grow-only — so this never happens in steady state).
    (void)hipDeviceSynchronize();
    (void)hipFree(b.p);
  } else {
    std::free(b.p);
  }
  b.p = nullptr;
  b.bytes = 0;
}

void BufferPool::ensure(const std::vector<Field>& fields, bool device) {
  auto& slots = device ? dev_ : host_;
  (device ? dev_alloc_ : host_alloc_) = true;
  if (slots.size() < fields.size()) slots.resize(fields.size());
  for (size_t i = 0; i < fields.size(); ++i) {
    const Field& f = fields[i];
    const size_t need = static_cast<size_t>(round_up(max_halo_elems(f), ALLOC_GRANULARITY) *
                                            f.elem_bytes);
    for (int n = 0; n < NNEIGHBORS; ++n) {
      grow(slots[i].send[n], need, device);
      grow(slots[i].recv[n], need, device);
    }
  }
}

char* BufferPool::send(size_t slot, int side, bool device) const {
  return (device ? dev_ : host_).at(slot).send[side].p;
}
char* BufferPool::recv(size_t slot, int side, bool device) const {
  return (device ? dev_ : host_).at(slot).recv[side].p;
}
size_t BufferPool::capacity(size_t slot, bool device) const {
  return (device ? dev_ : host_).at(slot).send[0].bytes;
}

void BufferPool::free_all() {
  for (auto& s : host_)
    for (int n = 0; n < NNEIGHBORS; ++n) { release(s.send[n], false); release(s.recv[n], false); }
  for (auto& s : dev_)
    for (int n = 0; n < NNEIGHBORS; ++n) { release(s.send[n], true); release(s.recv[n], true); }
  for (int dv = 0; dv < 2; ++dv)
    for (int w = 0; w < 2; ++w) release(arena_[dv][w], dv == 1);
  host_.clear();
  dev_.clear();
  host_alloc_ = dev_alloc_ = false;
}

// ---------------------------------------------------------------- HaloEngine

HaloEngine::HaloEngine(const GridInfo& g) : grid_(g) {
  const char* e = std::getenv("IGG_DEBUG_SYNC");
  debug_sync_ = e && *e && *e != '0';
}

void HaloEngine::debug_phase(hipStream_t stream, bool device, const char* phase) const {
  if (!debug_sync_ || !device) return;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  IGG_HIP_CHECK(hipStreamIsCapturing(stream, &cs));
  if (cs != hipStreamCaptureStatusNone) return;
  const hipError_t e = hipStreamSynchronize(stream);
  const hipError_t l = hipGetLastError();
  if (e != hipSuccess || l != hipSuccess)
    fail("IGG_DEBUG_SYNC: update_halo phase '", phase, "' failed: ",
         hipGetErrorString(e != hipSuccess ? e : l));
}

HaloEngine::~HaloEngine() {
  if (done_) (void)hipEventDestroy(done_);
}

void HaloEngine::exchange(const std::vector<Field>& fields, hipStream_t stream, int mode_override) {
  if (fields.empty()) return;
  TraceRange tr("igg.update_halo");
  const bool device = fields[0].device;
  bool capturing = false;
  if (device) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    IGG_HIP_CHECK(hipStreamIsCapturing(stream, &cs));
    capturing = cs != hipStreamCaptureStatusNone;
  }
  // No allocation (hipMalloc / device-wide sync) may happen inside a capture.
  struct Freeze {
    BufferPool& p;
    Freeze(BufferPool& q, bool on) : p(q) { p.set_frozen(on); }
    ~Freeze() { p.set_frozen(false); }
  } freeze(pool_, capturing);
  pool_.ensure(fields, device);
  if (device) {
    if (!done_) IGG_HIP_CHECK(hipEventCreateWithFlags(&done_, hipEventDisableTiming));
    // Buffers are shared across calls: order against the previous exchange if it
    // ran on another stream. Inside a graph capture the graph's own edges order
    // the work (an event recorded outside the capture cannot be waited on), and
    // replays are stream-ordered with eager exchanges by the caller.
    if (!capturing && have_event_ && last_stream_ != stream)
      IGG_HIP_CHECK(hipStreamWaitEvent(stream, done_, 0));
  }
  auto* put = device ? dynamic_cast<PutTransport*>(dev_transport_.get()) : nullptr;
  if (put) {
    // Kernel arguments are epoch-independent (the epoch lives on the device),
    // so a captured exchange replays correctly.
    exchange_put(fields, stream, put->mesh());
  } else if ((mode_override >= 0 ? static_cast<HaloMode>(mode_override) : resolved_mode(fields)) ==
             HaloMode::OnePhase) {
    exchange_onephase(fields, device, stream);
  } else {
    last_msgs_ = 0;
    for (int dim = 0; dim < NDIMS; ++dim) exchange_dim_impl(fields, dim, device, stream);
  }
  if (device && !capturing) {
    IGG_HIP_CHECK(hipEventRecord(done_, stream));
    have_event_ = true;
    last_stream_ = stream;
  }
}

void HaloEngine::exchange_dim(const std::vector<Field>& fields, int dim, hipStream_t stream) {
  if (fields.empty()) return;
  if (dim < 0 || dim >= NDIMS) fail("exchange_dim: invalid dim ", dim);
  const bool device = fields[0].device;
  pool_.ensure(fields, device);
  exchange_dim_impl(fields, dim, device, stream);
}

void HaloEngine::exchange_dim_impl(const std::vector<Field>& fields, int dim, bool device,
                                   hipStream_t stream) {
  const GridInfo& g = grid_;
  const int64_t left = g.neighbors[0][dim], right = g.neighbors[1][dim];
  const bool has[2] = {left != PROC_NULL, right != PROC_NULL};
  if (!has[0] && !has[1]) return;
  const int eb = fields[0].elem_bytes;
  const bool blit = device && pack_mode_[dim] == PackMode::Memcpy2D;
  auto do_copies = [&](const std::vector<Copy2D>& cps) {
    if (cps.empty()) return;
    if (!device) return host_copy2d(cps, eb);
    if (!blit) return launch_copy2d(cps, eb, stream);
    std::vector<Copy2D> rest;
    for (const Copy2D& c : cps) {
      if (c.src_si != 1 || c.dst_si != 1) {
        rest.push_back(c);
        continue;
      }
      const size_t w = static_cast<size_t>(c.n_inner) * eb;
      const size_t sp = c.n_outer > 1 ? static_cast<size_t>(c.src_so) * eb : w;
      const size_t dp = c.n_outer > 1 ? static_cast<size_t>(c.dst_so) * eb : w;
      IGG_HIP_CHECK(hipMemcpy2DAsync(c.dst, dp, c.src, sp, w, static_cast<size_t>(c.n_outer),
                                     hipMemcpyDeviceToDevice, stream));
    }
    if (!rest.empty()) launch_copy2d(rest, eb, stream);
  };

  if (left == g.me && right == g.me) {
    // Periodic with a single process along `dim`: in-place plane copies. The
    // planes read (ol-1, size-ol) and written (0, size-1) are disjoint for every
    // admissible overlap (periodic requires n >= 2*ol-1), so one launch suffices.
    std::vector<Copy2D> cps;
    for (const Field& f : fields) {
      if (ol(g, dim, f) < 2) continue;
      for (int s = 0; s < NNEIGHBORS; ++s) {
        const Face src = face(f, dim, send_index(g, s, dim, f));
        const Face dst = face(f, dim, recv_index(g, 1 - s, dim, f));
        cps.push_back({src.base, dst.base, src.n_outer, src.n_inner, src.s_outer, src.s_inner,
                       dst.s_outer, dst.s_inner});
      }
    }
    do_copies(cps);
    return;
  }
  if (left == g.me || right == g.me)
    fail("Incoherent neighbors in dimension ", dim + 1, ": either all neighbors must equal to me, or none.");
  const std::shared_ptr<Transport>& transport_ = device ? dev_transport_ : host_transport_;
  if (!transport_)
    fail("update_halo: no transport available to reach neighbours in dimension ", dim + 1,
         " (multi-process exchange needs an initialised communicator).");
  if (device && !transport_->device_capable())
    fail("update_halo: transport '", transport_->name(), "' cannot move GPU memory.");
  if (!device && !transport_->host_capable())
    fail("update_halo: transport '", transport_->name(), "' cannot move host memory.");

  std::vector<Copy2D> pack, unpack;
  std::vector<P2POp> recvs, sends;
  // Receives: right side first, then left (update_halo.jl:47-49); sends: left
  // then right (:50-55). RCCL matches same-peer messages in issue order.
  for (int s = NNEIGHBORS - 1; s >= 0; --s) {
    if (!has[s]) continue;
    for (size_t i = 0; i < fields.size(); ++i) {
      const Field& f = fields[i];
      if (ol(g, dim, f) < 2) continue;
      const Face rf = face(f, dim, recv_index(g, s, dim, f));
      char* ptr = rf.contiguous ? rf.base : pool_.recv(i, s, device);
      recvs.push_back({ptr, rf.bytes, static_cast<int>(g.neighbors[s][dim]),
                       static_cast<int>(i * 2 + s)});
      if (!rf.contiguous)
        unpack.push_back({ptr, rf.base, rf.n_outer, rf.n_inner, rf.n_inner, 1, rf.s_outer,
                          rf.s_inner});
    }
  }
  for (int s = 0; s < NNEIGHBORS; ++s) {
    if (!has[s]) continue;
    for (size_t i = 0; i < fields.size(); ++i) {
      const Field& f = fields[i];
      if (ol(g, dim, f) < 2) continue;
      const Face sf = face(f, dim, send_index(g, s, dim, f));
      char* ptr = sf.contiguous ? sf.base : pool_.send(i, s, device);
      if (!sf.contiguous)
        pack.push_back({sf.base, ptr, sf.n_outer, sf.n_inner, sf.s_outer, sf.s_inner, sf.n_inner,
                        1});
      // The receiver files this message under its opposite side.
      sends.push_back({ptr, sf.bytes, static_cast<int>(g.neighbors[s][dim]),
                       static_cast<int>(i * 2 + (1 - s))});
    }
  }
  static const char* const kPack[3] = {"igg.seq.pack.x", "igg.seq.pack.y", "igg.seq.pack.z"};
  static const char* const kComm[3] = {"igg.seq.transport.x", "igg.seq.transport.y", "igg.seq.transport.z"};
  static const char* const kUnpack[3] = {"igg.seq.unpack.x", "igg.seq.unpack.y", "igg.seq.unpack.z"};
  {
    TraceRange r(kPack[dim]);
    do_copies(pack);
    debug_phase(stream, device, kPack[dim]);
  }
  {
    TraceRange r(kComm[dim]);
    transport_->exchange(recvs, sends, device, stream);
    debug_phase(stream, device, kComm[dim]);
  }
  TraceRange r(kUnpack[dim]);
  do_copies(unpack);
  debug_phase(stream, device, kUnpack[dim]);
}

}  // namespace igg

// ------------------------------------------------------- one-phase exchange
//
// Equivalence with the sequential x -> y -> z schedule (reference
// update_halo.jl:40): with sequential faces spanning the full extent of the
// other dims, the value finally landing at a halo position p comes from the
// rank at coords + v, where v_d = -1/+1 for every dim d in which p lies on the
// left/right halo plane (with a neighbour there), read at that rank's send
// plane in those dims and at p in the others. The one-phase schedule sends
// exactly these values directly: one message per direction v (faces |v|=1,
// edges |v|=2, corners |v|=3). In a dim d with v_d = 0 a message covers
// [lo_d, hi_d) where the halo planes are excluded iff a neighbour exists on that
// side (those positions belong to the message of a longer direction), so all
// receive regions are disjoint and unpacking needs no ordering. Sender and
// receiver agree on the extents because they share the coordinate in every dim
// with v_d = 0, hence the same neighbour existence there.

namespace igg {

bool HaloEngine::active(const Field& f, int d) const {
  return ol(grid_, d, f) >= 2 &&
         (grid_.neighbors[0][d] != PROC_NULL || grid_.neighbors[1][d] != PROC_NULL);
}

HaloMode HaloEngine::resolved_mode(const std::vector<Field>& fields) const {
  // Auto without a measurement: the sequential x -> y -> z schedule (3 RCCL
  // groups of <= 2 peers). One-phase (one group, up to 26 peers incl. edges and
  // corners) measured 2x slower on the 1-GPU loopback of a 512^3 field
  // (profiles/r1_graph/lb_one.log vs lb_seq.log); parallel/halo.py times both
  // per field set on first use and passes the winner as mode_override.
  (void)fields;
  return mode_ == HaloMode::Auto ? HaloMode::Sequential : mode_;
}

namespace {
struct Msg {
  size_t field;
  int key;  // direction as seen by the receiver
  int64_t peer;
  Face face;
  size_t off;
  bool zero_copy;
};
constexpr size_t MSG_ALIGN = 256;
}  // namespace

bool HaloEngine::dir_regions(const Field& f, int key, Region& rr, Region& sr) const {
  const GridInfo& g = grid_;
  const int u[3] = {key / 9 - 1, (key / 3) % 3 - 1, key % 3 - 1};  // receiver-side direction
  for (int d = 0; d < NDIMS; ++d) {
    const int64_t n = f.size[d];
    if (u[d] != 0) {
      if (!active(f, d)) return false;
      const int64_t o = ol(g, d, f);
      // receive into my halo plane on side u_d; the matching send (direction
      // -u) reads my send plane on side -u_d.
      rr.lo[d] = u[d] < 0 ? 0 : n - 1;
      sr.lo[d] = u[d] < 0 ? n - o : o - 1;
      rr.hi[d] = rr.lo[d] + 1;
      sr.hi[d] = sr.lo[d] + 1;
    } else {
      // Exclude the halo planes that another message fills (neighbour exists).
      const bool act = active(f, d);
      rr.lo[d] = sr.lo[d] = (act && g.neighbors[0][d] != PROC_NULL) ? 1 : 0;
      rr.hi[d] = sr.hi[d] = (act && g.neighbors[1][d] != PROC_NULL) ? n - 1 : n;
    }
  }
  return rr.count() > 0;
}

void HaloEngine::exchange_put(const std::vector<Field>& fields, hipStream_t stream, PeerMesh& mesh) {
  const GridInfo& g = grid_;
  if (!g.has_peers) fail("the put transport needs the peer table (GridInfo.peers)");
  const size_t nf = fields.size();
  const int eb = fields[0].elem_bytes;
  // Arena slot of (key, field): a function of the field shapes and of the
  // dimensions in which the grid has neighbours at all, so every rank computes
  // the same layout for the same call. (A dimension has neighbours on every
  // rank or on none: periodic, or split over >= 2 ranks, gives each rank at
  // least one.) Directions along a dimension without neighbours get no slot:
  // for a 2-D field (nz = 1) a "z face" would be the whole field, and 2 x 26
  // such slots made the acoustic model's arena exceed the IPC size limit.
  bool dim_has_nb[NDIMS];
  for (int d = 0; d < NDIMS; ++d) dim_has_nb[d] = g.neighbors[0][d] != PROC_NULL || g.neighbors[1][d] != PROC_NULL;
  std::vector<size_t> slot(27 * nf, 0);
  bool has_slot[27] = {};
  size_t per = 0;
  for (int key = 0; key < 27; ++key) {
    if (key == 13) continue;
    const int u[3] = {key / 9 - 1, (key / 3) % 3 - 1, key % 3 - 1};
    if ((u[0] != 0 && !dim_has_nb[0]) || (u[1] != 0 && !dim_has_nb[1]) || (u[2] != 0 && !dim_has_nb[2])) continue;
    has_slot[key] = true;
    for (size_t i = 0; i < nf; ++i) {
      int64_t elems = 1;
      for (int d = 0; d < NDIMS; ++d) elems *= u[d] != 0 ? 1 : fields[i].size[d];
      slot[key * nf + i] = per;
      per += static_cast<size_t>(round_up(elems * eb, static_cast<int64_t>(MSG_ALIGN)));
    }
  }
  mesh.ensure_arena(2 * per);  // collective, grow-only
  // Fixed halves per epoch parity (independent of this call's layout); the
  // kernels pick the half from the device-resident epoch.
  const int64_t half = static_cast<int64_t>(mesh.arena_bytes() / 2);
  const int me = mesh.rank();
  std::vector<Copy2D> put, unpack;
  std::vector<int> out_ranks, in_ranks, nb_ranks;
  auto add = [](std::vector<int>& v, int r) {
    if (std::find(v.begin(), v.end(), r) == v.end()) v.push_back(r);
  };
  for (int key = 0; key < 27; ++key) {
    if (key == 13) continue;
    const int64_t from = g.peers[key], to = g.peers[26 - key];
    if (!has_slot[key]) {
      if (from != PROC_NULL || to != PROC_NULL) fail("put transport: a peer along a dimension without neighbours");
      continue;
    }
    if (from != PROC_NULL) add(nb_ranks, static_cast<int>(from));
    for (size_t i = 0; i < nf; ++i) {
      const Field& f = fields[i];
      Region rr{}, sr{};
      if (!dir_regions(f, key, rr, sr)) continue;
      const size_t off = slot[key * nf + i];
      if (to != PROC_NULL) {
        const Face sf = region_face(f, sr);
        put.push_back({sf.base, mesh.arena(static_cast<int>(to)) + off, sf.n_outer, sf.n_inner, sf.s_outer,
                       sf.s_inner, sf.n_inner, 1});
        add(out_ranks, static_cast<int>(to));
      }
      if (from != PROC_NULL) {
        const Face rf = region_face(f, rr);
        unpack.push_back({mesh.arena(me) + off, rf.base, rf.n_outer, rf.n_inner, rf.n_inner, 1, rf.s_outer,
                          rf.s_inner});
        add(in_ranks, static_cast<int>(from));
      }
    }
  }
  last_msgs_ = static_cast<int>(put.size());
  if (out_ranks.size() > PUT_MAX_PEERS || in_ranks.size() > PUT_MAX_PEERS || nb_ranks.size() > PUT_MAX_PEERS)
    fail("put transport: too many distinct peers");
  PutSync ps{};
  ps.my_flags = mesh.flags(me);
  ps.my_rank = me;
  ps.nranks = mesh.nranks();
  ps.timeout_ticks = mesh.timeout_ticks();
  ps.n_out = static_cast<int>(out_ranks.size());
  ps.n_in = static_cast<int>(in_ranks.size());
  ps.n_nb = static_cast<int>(nb_ranks.size());
  for (int j = 0; j < ps.n_out; ++j) {
    ps.out_rank[j] = out_ranks[j];
    ps.out_flags[j] = mesh.flags(out_ranks[j]);
  }
  for (int j = 0; j < ps.n_in; ++j) ps.in_rank[j] = in_ranks[j];
  for (int j = 0; j < ps.n_nb; ++j) ps.nb_flags[j] = mesh.flags(nb_ranks[j]);
  const uint64_t* epoch = mesh.flags(me) + PutFlags::EPOCH;
  // [begin] -> put (stores into the receivers' arenas) -> sync -> unpack
  bool implied = put_count_ >= 2;  // exchanges 1 and 2 use fresh halves
  for (int r : out_ranks)
    if (std::find(prev_in_.begin(), prev_in_.end(), r) == prev_in_.end()) implied = false;
  if (!implied && put_count_ >= 2) {
    TraceRange r("igg.put.begin");
    launch_put_begin(ps, stream);
  }
  ++put_count_;
  prev_in_ = in_ranks;
  {
    TraceRange r("igg.put.pack");
    launch_copy2d(put, eb, stream, /*system_fence=*/true, ParityShift{epoch, half, 1, 1});
    debug_phase(stream, true, "igg.put.pack");
  }
  {
    TraceRange r("igg.put.sync");
    launch_put_sync(ps, stream);
    debug_phase(stream, true, "igg.put.sync");
  }
  {
    TraceRange r("igg.put.unpack");
    launch_copy2d(unpack, eb, stream, false, ParityShift{epoch, half, 2, 0});
    debug_phase(stream, true, "igg.put.unpack");
  }
  if (debug_sync_) mesh.check_error();  // a bounded wait of this exchange timed out
}

void HaloEngine::exchange_onephase(const std::vector<Field>& fields, bool device,
                                   hipStream_t stream) {
  const GridInfo& g = grid_;
  if (!g.has_peers) fail("one-phase halo exchange needs the peer table (GridInfo.peers)");
  std::vector<Msg> sends, recvs;
  size_t send_bytes = 0, recv_bytes = 0;
  bool any_remote = false;
  for (int key = 0; key < 27; ++key) {
    if (key == 13) continue;
    const int u[3] = {key / 9 - 1, (key / 3) % 3 - 1, key % 3 - 1};  // receiver-side direction
    const int64_t from = g.peers[key];                 // I receive from coords + u
    const int64_t to = g.peers[26 - key];              // I send in direction -u
    for (size_t i = 0; i < fields.size(); ++i) {
      const Field& f = fields[i];
      Region rr{}, sr{};
      if (!dir_regions(f, key, rr, sr)) continue;
      // A face (one non-zero component) whose FULL plane is contiguous (the
      // outermost dim of a C-order field) travels as that whole plane, zero-copy
      // on both sides. The rows it carries beyond the region (halo rows of the
      // other dims) are stale, but exactly those rows arrive as edge/corner
      // messages, which always go through the receive arena and are unpacked
      // after the RCCL group has completed — so they overwrite the stale rows
      // deterministically. Edge/corner receives are therefore never zero-copy.
      const int nnz = (u[0] != 0) + (u[1] != 0) + (u[2] != 0);
      Region rfull = rr, sfull = sr;
      for (int d = 0; d < NDIMS; ++d)
        if (u[d] == 0) { rfull.lo[d] = sfull.lo[d] = 0; rfull.hi[d] = sfull.hi[d] = f.size[d]; }
      if (from != PROC_NULL) {
        Msg m{i, key, from, region_face(f, rr), 0, false};
        if (from != g.me && nnz == 1) {
          const Face full = region_face(f, rfull);
          if (full.contiguous) { m.face = full; m.zero_copy = true; }
        }
        if (!m.zero_copy) { m.off = recv_bytes; recv_bytes += round_up(m.face.bytes, MSG_ALIGN); }
        any_remote |= from != g.me;
        recvs.push_back(m);
      }
      if (to != PROC_NULL) {
        Msg m{i, key, to, region_face(f, sr), 0, false};
        if (to != g.me) {
          if (nnz == 1) {
            const Face full = region_face(f, sfull);
            if (full.contiguous) { m.face = full; m.zero_copy = true; }
          } else {
            m.zero_copy = m.face.contiguous;  // sends only read: safe
          }
        }
        if (!m.zero_copy) { m.off = send_bytes; send_bytes += round_up(m.face.bytes, MSG_ALIGN); }
        sends.push_back(m);
      }
    }
  }
  last_msgs_ = static_cast<int>(sends.size());
  if (sends.empty() && recvs.empty()) return;
  const std::shared_ptr<Transport>& tr = device ? dev_transport_ : host_transport_;
  if (any_remote) {
    if (!tr) fail("update_halo: no transport available to reach remote neighbours.");
    if (device ? !tr->device_capable() : !tr->host_capable())
      fail("update_halo: transport '", tr->name(), "' cannot move ", device ? "GPU" : "host", " memory.");
  }
  char* sbuf = send_bytes ? pool_.arena(0, send_bytes, device) : nullptr;
  char* rbuf = recv_bytes ? pool_.arena(1, recv_bytes, device) : nullptr;
  const int eb = fields[0].elem_bytes;
  auto do_copies = [&](const std::vector<Copy2D>& cps) {
    if (cps.empty()) return;
    if (device) launch_copy2d(cps, eb, stream); else host_copy2d(cps, eb);
  };
  // 1. pack every non-zero-copy send region (one launch for all fields/directions)
  std::vector<Copy2D> pack;
  std::vector<P2POp> tsend, trecv;
  std::vector<const char*> self_src(27 * fields.size(), nullptr);
  for (const Msg& m : sends) {
    const Face& fc = m.face;
    char* dst = m.zero_copy ? fc.base : sbuf + m.off;
    if (!m.zero_copy)
      pack.push_back({fc.base, dst, fc.n_outer, fc.n_inner, fc.s_outer, fc.s_inner, fc.n_inner, 1});
    if (m.peer == g.me) self_src[m.field * 27 + m.key] = dst;
    else tsend.push_back({dst, fc.bytes, static_cast<int>(m.peer), static_cast<int>(m.field * 27 + m.key)});
  }
  {
    TraceRange r("igg.onephase.pack");
    do_copies(pack);
    debug_phase(stream, device, "igg.onephase.pack");
  }
  // 2. one communication phase for all remote messages
  std::vector<Copy2D> unpack;
  for (const Msg& m : recvs) {
    const Face& fc = m.face;
    const char* src;
    if (m.peer == g.me) {
      src = self_src[m.field * 27 + m.key];
      if (!src) fail("one-phase exchange: missing self message (inconsistent peer table)");
    } else {
      char* dst = m.zero_copy ? fc.base : rbuf + m.off;
      trecv.push_back({dst, fc.bytes, static_cast<int>(m.peer), static_cast<int>(m.field * 27 + m.key)});
      src = dst;
      if (m.zero_copy) continue;
    }
    unpack.push_back({src, fc.base, fc.n_outer, fc.n_inner, fc.n_inner, 1, fc.s_outer, fc.s_inner});
  }
  if (!tsend.empty() || !trecv.empty()) {
    TraceRange r("igg.onephase.transport");
    tr->exchange(trecv, tsend, device, stream);
    debug_phase(stream, device, "igg.onephase.transport");
  }
  // 3. unpack every receive region (disjoint: one launch)
  TraceRange r3("igg.onephase.unpack");
  do_copies(unpack);
  debug_phase(stream, device, "igg.onephase.unpack");
}

}  // namespace igg
