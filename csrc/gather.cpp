// Device gather-to-root (see include/igg/gather.hpp).
#include "igg/gather.hpp"
#include "igg/fault.hpp"
#include "igg/trace.hpp"
#include "igg/ipc.hpp"
#include "igg/vmm.hpp"

#include <unistd.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include <hip/hip_runtime_api.h>

namespace igg {

void Gatherer::free() {
  if (buf_) {
    (void)hipDeviceSynchronize();
    (void)hipFree(buf_);
  }
  buf_ = nullptr;
  bytes_ = 0;
}

void Gatherer::gather(const Field& a, void* dst, int root, const Int3& dims, RcclComm& comm,
                      hipStream_t stream) {
  TraceRange tr("igg.gather");
  if (!a.device) fail("Gatherer: the local array must be a GPU array.");
  const int64_t len = a.size[0] * a.size[1] * a.size[2];
  const size_t blk = static_cast<size_t>(len) * a.elem_bytes;
  const int nprocs = comm.nranks();
  if (dims[0] * dims[1] * dims[2] != nprocs) fail("Gatherer: dims do not match the communicator size.");
  void* src = reinterpret_cast<void*>(a.ptr);
  if (comm.rank() != root) {
    comm.exchange({}, {{src, blk, root, 0}}, true, stream);
    return;
  }
  if (!dst) fail("The input argument A_global can't be `nothing` on the root");
  // Grow-only cache, GG_ALLOC_GRANULARITY elements granular (gather.jl:40-46).
  const size_t need =
      static_cast<size_t>(round_up(nprocs * len, ALLOC_GRANULARITY)) * a.elem_bytes;
  if (bytes_ < need) {
    free();
    IGG_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&buf_), need));
    bytes_ = need;
  }
  std::vector<P2POp> recvs;
  for (int p = 0; p < nprocs; ++p)
    if (p != root) recvs.push_back({buf_ + static_cast<size_t>(p) * blk, blk, p, 0});
  comm.exchange(recvs, {}, true, stream);
  IGG_HIP_CHECK(hipMemcpyAsync(buf_ + static_cast<size_t>(root) * blk, src, blk,
                               hipMemcpyDeviceToDevice, stream));
  launch_gather_reorder(buf_, dst, a.size, dims, a.elem_bytes, stream);
}

// ------------------------------------------------------------ PullGatherer

namespace {

constexpr int MAX_COPY_STREAMS = 8;

// One 3-D copy of planes [x0, x0 + nx) of a C-contiguous block of extent s
// (elements; `src` points at plane x0) into their place (block coords c) in the
// C-contiguous global array of extent dims*s.
void copy_block(const void* src, void* dst, const Int3& s, const Int3& dims, const Int3& c, int64_t x0, int64_t nx,
                int eb, hipStream_t stream) {
  const size_t row = static_cast<size_t>(s[2]) * eb;
  hipMemcpy3DParms p{};
  p.srcPtr = make_hipPitchedPtr(const_cast<void*>(src), row, row, static_cast<size_t>(s[1]));
  p.dstPtr = make_hipPitchedPtr(dst, static_cast<size_t>(dims[2] * s[2]) * eb, static_cast<size_t>(dims[2] * s[2]) * eb,
                                static_cast<size_t>(dims[1] * s[1]));
  p.srcPos = make_hipPos(0, 0, 0);
  p.dstPos = make_hipPos(static_cast<size_t>(c[2] * s[2]) * eb, static_cast<size_t>(c[1] * s[1]),
                         static_cast<size_t>(c[0] * s[0] + x0));
  p.extent = make_hipExtent(row, static_cast<size_t>(s[1]), static_cast<size_t>(nx));
  p.kind = hipMemcpyDeviceToDevice;
  IGG_HIP_CHECK(hipMemcpy3DAsync(&p, stream));
}

// Staging chunk size for blocks that cannot be exported whole:
// IGG_GATHER_CHUNK_BYTES (tests: blocks larger than this are staged too),
// else half the IPC limit.
size_t chunk_cap(bool* forced) {
  static const long long b = [] {
    const char* e = std::getenv("IGG_GATHER_CHUNK_BYTES");
    return e ? std::atoll(e) : 0LL;
  }();
  *forced = b > 0;
  return b > 0 ? static_cast<size_t>(b) : IPC_MAX_BYTES / 2;
}

void put_u32(std::string& r, uint32_t v) { r.append(reinterpret_cast<const char*>(&v), 4); }
uint32_t get_u32(const std::string& r, size_t at) {
  uint32_t v = 0;
  std::memcpy(&v, r.data() + at, 4);
  return v;
}

}  // namespace

// IGG_GATHER_VMM=1: large snapshots go through ONE VMM staging buffer
// instead of IPC staging chunks (rounds 3-5). Off by default: allocated on the
// first gather of a running job (hipMemCreate + map while this process's
// kernels run), it ended in an illegal-address error in an 8-rank 1024^3 f32
// run on one GPU (profiles/r6_vmm/NOTES.md), and it was no faster than the
// chunks (4.10 vs 3.83 ms).
bool vmm_staging() {
  static const bool on = [] {
    const char* e = std::getenv("IGG_GATHER_VMM");
    return e && e[0] == '1';
  }();
  return on;
}

PullGatherer::PullGatherer(int rank, int nranks, AllGather allgather)
    : rank_(rank), nranks_(nranks), allgather_(std::move(allgather)) {
  peer_key_.assign(nranks, std::string());
  peer_ev_.assign(nranks, nullptr);
  mapped_.assign(nranks, {});
  mapped_vmm_.assign(nranks, 0);
}

namespace {
uint64_t buffer_id(void* p) {
  unsigned long long id = 0;
  IGG_HIP_CHECK(hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, reinterpret_cast<hipDeviceptr_t>(p)));
  return id;
}

int export_fd(void* base, bool dmabuf) {
  return dmabuf ? range_export_fd(base, nullptr, nullptr) : vmm_export_fd(base);
}
}  // namespace

// IGG_GATHER_DMABUF=0: an ordinary allocation of 2 GiB or more is staged into
// the VMM buffer (one copy) instead of being exported as a dma-buf.
bool dmabuf_gather() {
  static const bool on = [] {
    const char* e = std::getenv("IGG_GATHER_DMABUF");
    return !(e && e[0] == '0');
  }();
  return on;
}

std::string PullGatherer::vmm_record(void* base, size_t size, uint64_t off, bool dmabuf) {
  const uint64_t id = dmabuf ? buffer_id(base) : 0;
  int k = 0;
  while (k < static_cast<int>(vexp_.size()) && vexp_[k].base != base) ++k;
  if (k < static_cast<int>(vexp_.size()) && (vexp_[k].dmabuf != dmabuf || vexp_[k].buffer_id != id)) {
    // another allocation at this address now: retire the old export
    fd_close(vexp_[k].listener);
    fd_close(vexp_[k].fd);
    vexp_.erase(vexp_.begin() + k);
    k = static_cast<int>(vexp_.size());
  }
  if (k == static_cast<int>(vexp_.size())) {
    VmmExport e;
    e.base = base;
    e.dmabuf = dmabuf;
    e.buffer_id = id;
    e.fd = export_fd(base, dmabuf);
    static int serial = 0;
    e.name = "igg-gather-" + std::to_string(::getpid()) + "-" + std::to_string(rank_) + "-" + std::to_string(serial++);
    e.listener = fd_listen(e.name);
    vexp_.push_back(e);
  }
  cur_vexp_ = k;
  std::string rec(1, 'V');
  put_u32(rec, static_cast<uint32_t>(vexp_[k].name.size()));
  rec += vexp_[k].name;
  const uint64_t sz = size;
  rec.append(reinterpret_cast<const char*>(&sz), 8);
  rec.append(reinterpret_cast<const char*>(&off), 8);
  return rec;
}

void PullGatherer::close_mapped(int p) {
  auto& per = mapped_[p];
  if (!per.empty()) {
    for (hipStream_t q : side_) IGG_HIP_CHECK(hipStreamSynchronize(q));  // rare: old copies drained
    for (auto& m : per) {
      if (mapped_vmm_[p]) vmm_free(m.second);
      else ipc_close(m.second);
    }
  }
  per.clear();
  mapped_vmm_[p] = 0;
}

void PullGatherer::free_vmm() {
  for (auto& e : vexp_) {
    fd_close(e.listener);
    fd_close(e.fd);
  }
  vexp_.clear();
  cur_vexp_ = -1;
  if (vstage_) vmm_free(vstage_);
  for (void* v : vretired_) vmm_free(v);
  vstage_ = nullptr;
  vstage_bytes_ = 0;
  vretired_.clear();
}

PullGatherer::~PullGatherer() {
  for (hipStream_t s : side_) (void)hipStreamSynchronize(s);
  for (int p = 0; p < static_cast<int>(mapped_.size()); ++p)
    for (auto& m : mapped_[p])
      if (m.second) {
        if (mapped_vmm_[p]) vmm_free(m.second);
        else (void)hipIpcCloseMemHandle(m.second);
      }
  free_vmm();
  if (!stage_.empty() || !retired_.empty()) (void)hipDeviceSynchronize();
  for (char* c : stage_) (void)hipFree(c);
  for (char* c : retired_) (void)hipFree(c);
  for (hipEvent_t& e : peer_ev_)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t& e : root_done_)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : done_) (void)hipEventDestroy(e);
  if (ready_) (void)hipEventDestroy(ready_);
  for (hipStream_t s : side_) (void)hipStreamDestroy(s);
}

void PullGatherer::ensure_streams() {
  if (!ready_)
    IGG_HIP_CHECK(hipEventCreateWithFlags(&ready_, hipEventInterprocess | hipEventDisableTiming));
  while (static_cast<int>(side_.size()) < std::min(nranks_, MAX_COPY_STREAMS)) {
    hipStream_t s;
    hipEvent_t e;
    IGG_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    IGG_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventInterprocess | hipEventDisableTiming));
    side_.push_back(s);
    done_.push_back(e);
  }
}

void PullGatherer::free() {
  if (pending_) fail("gather_async: free while a gather is pending (call wait() first)");
  for (hipStream_t s : side_) IGG_HIP_CHECK(hipStreamSynchronize(s));
  for (int p = 0; p < static_cast<int>(mapped_.size()); ++p) {
    for (auto& m : mapped_[p])
      if (m.second) {
        if (mapped_vmm_[p]) vmm_free(m.second);
        else (void)hipIpcCloseMemHandle(m.second);
      }
    mapped_[p].clear();
    mapped_vmm_[p] = 0;
  }
  free_vmm();
  if (!stage_.empty() || !retired_.empty()) IGG_HIP_CHECK(hipDeviceSynchronize());
  for (char* c : stage_) IGG_HIP_CHECK(hipFree(c));
  for (char* c : retired_) IGG_HIP_CHECK(hipFree(c));
  stage_.clear();
  retired_.clear();
  stage_bytes_ = 0;
}

void PullGatherer::start(const Field& a, void* dst, int root, const Int3& dims, hipStream_t stream,
                         bool snapshot) {
  TraceRange tr("igg.gather_async.start");
  if (pending_) fail("gather_async: a gather is already pending (call wait() first)");
  if (!a.device) fail("gather_async: the local array must be a GPU array.");
  if (dims[0] * dims[1] * dims[2] != nranks_) fail("gather_async: dims do not match the number of processes.");
  if (root < 0 || root >= nranks_) fail("gather_async: root ", root, " out of range");
  if (rank_ == root && !dst) fail("The input argument A_global can't be `nothing` on the root");
  ensure_streams();
  const size_t EH = sizeof(hipIpcEventHandle_t), MH = sizeof(hipIpcMemHandle_t);
  const size_t plane = static_cast<size_t>(a.size[1] * a.size[2]) * a.elem_bytes;
  // Every rank prepares its record (export handles, staged chunks) and joins
  // the allgather whatever happens: a rank that failed sends status '0' and
  // its error, so every rank raises together instead of the others blocking
  // in a collective (as PeerMesh::map_buffers does).
  std::string mine(1, '1'), error;
  try {
    inject_fail("gather_export");
    std::string rec;  // after the event handle: 'D' handle offset | 'C' nchunks planes/chunk handles...
    cur_vexp_ = -1;
    last_kind_ = "root";
    if (rank_ != root) {
      void* base = nullptr;
      size_t size = 0;
      bool vown = false;
      const bool a_vmm = vmm_find(reinterpret_cast<const void*>(a.ptr), &base, &size, &vown) && vown;
      if (!a_vmm) IGG_HIP_CHECK(hipMemGetAddressRange(&base, &size, reinterpret_cast<void*>(a.ptr)));
      bool forced = false;
      const size_t cap = chunk_cap(&forced);
      const size_t abytes = plane * static_cast<size_t>(a.size[0]);
      // snapshot: `a` may change as soon as start() returns, so it is copied
      // into the staging chunks in any case (the chunks are the snapshot).
      int dev = 0;
      IGG_HIP_CHECK(hipGetDevice(&dev));
      if (a_vmm && !snapshot) {
        // a VMM allocation: exportable at any size, pulled in place
        rec = vmm_record(base, size, a.ptr - reinterpret_cast<uintptr_t>(base));
        last_kind_ = "vmm";
      } else if (!a_vmm && !snapshot && size >= IPC_MAX_BYTES && !forced && dmabuf_gather() &&
                 size % vmm_granularity(dev) == 0) {
        // an ordinary allocation above the IPC limit: its dma-buf, pulled in place
        rec = vmm_record(base, size, a.ptr - reinterpret_cast<uintptr_t>(base), true);
        last_kind_ = "dmabuf";
      } else if ((snapshot || size >= IPC_MAX_BYTES) && !forced && vmm_staging() && abytes >= IPC_MAX_BYTES / 2) {
        // a large snapshot / an unexportable allocation: ONE VMM staging
        // buffer (grow-only; a grown-out one is retired, its export name dies
        // with it, so the root re-imports)
        if (vstage_bytes_ < abytes) {
          if (vstage_) vretired_.push_back(vstage_);
          vstage_ = vmm_alloc(abytes, &vstage_bytes_);
        }
        IGG_HIP_CHECK(hipMemcpyAsync(vstage_, reinterpret_cast<const void*>(a.ptr), abytes, hipMemcpyDeviceToDevice,
                                     stream));
        rec = vmm_record(vstage_, vstage_bytes_, 0);
        last_kind_ = "vmm-staging";
      } else if (snapshot || size >= IPC_MAX_BYTES || (forced && plane * a.size[0] > cap)) {
        // Stage into exportable chunks of whole planes (class comment).
        const int64_t ppc = std::max<int64_t>(1, static_cast<int64_t>(cap / std::max<size_t>(plane, 1)));
        const size_t cb = static_cast<size_t>(ppc) * plane;
        if (cb >= IPC_MAX_BYTES) fail("gather_async: one x-plane of the local array exceeds the IPC limit");
        const int64_t nch = (a.size[0] + ppc - 1) / ppc;
        if (stage_bytes_ < cb || static_cast<int64_t>(stage_.size()) < nch) {
          // Rare (grow-only). The grown-out chunks are RETIRED, not freed,
          // until free(): an IPC export of a new allocation at a freed one's
          // address was seen to map the OLD memory in the peer
          // (profiles/r3_put_arena/), so every export address stays new and
          // the root, seeing new handles, re-maps.
          for (char* c : stage_) retired_.push_back(c);
          stage_.clear();
          for (int64_t k = 0; k < nch; ++k) {
            char* c = nullptr;
            IGG_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&c), cb));
            stage_.push_back(c);
          }
          stage_bytes_ = cb;
        }
        rec.push_back('C');
        last_kind_ = "chunks";
        put_u32(rec, static_cast<uint32_t>(nch));
        put_u32(rec, static_cast<uint32_t>(ppc));
        for (int64_t k = 0; k < nch; ++k) {
          const int64_t nx = std::min<int64_t>(ppc, a.size[0] - k * ppc);
          IGG_HIP_CHECK(hipMemcpyAsync(stage_[k], reinterpret_cast<const char*>(a.ptr) + k * ppc * plane,
                                       static_cast<size_t>(nx) * plane, hipMemcpyDeviceToDevice, stream));
          rec += ipc_get_handle(stage_[k]);
        }
      } else {
        const uint64_t off = a.ptr - reinterpret_cast<uintptr_t>(base);
        rec.push_back('D');
        last_kind_ = "ipc";
        rec += ipc_get_handle(base);
        rec.append(reinterpret_cast<const char*>(&off), sizeof(off));
      }
    }
    // `a` (or its staged copy; on the root also dst) is final where the
    // caller's stream has got to now: an interprocess event marks that point
    // (no host drain).
    IGG_HIP_CHECK(hipEventRecord(ready_, stream));
    hipIpcEventHandle_t eh;
    IGG_HIP_CHECK(hipIpcGetEventHandle(&eh, ready_));
    mine.append(reinterpret_cast<const char*>(&eh), EH);
    mine += rec;
    if (rank_ == root) {
      for (hipEvent_t e : done_) {  // the peers order their streams after these in wait()
        IGG_HIP_CHECK(hipIpcGetEventHandle(&eh, e));
        mine.append(reinterpret_cast<const char*>(&eh), EH);
      }
    }
  } catch (const Error& e) {
    error = e.what();
    mine.assign("0");
    mine += error;
  }
  // Host rendezvous only (every rank has recorded its event before the root
  // waits on it), not a GPU drain.
  std::vector<std::string> all = allgather_(mine);
  if (static_cast<int>(all.size()) != nranks_) fail("gather_async: allgather returned ", all.size(), " entries");
  for (int r = 0; r < nranks_; ++r)
    if (all[r].empty() || all[r][0] != '1')
      fail("gather_async: rank ", r, " could not export its block",
           all[r].size() > 1 ? std::string(" (") + all[r].substr(1, 300) + ")" : std::string());
  for (auto& x : all) x.erase(0, 1);
  const int nside = static_cast<int>(side_.size());
  used_ = std::min(nranks_, nside);
  // VMM records: the root asks every rank whose export it has not mapped yet
  // for the file descriptor (one more host rendezvous, only when some rank
  // published a 'V' record - every rank sees every record, so all agree).
  auto vname = [&](const std::string& rec) {
    const uint32_t n = rec.size() >= EH + 5 ? get_u32(rec, EH + 1) : 0;
    return rec.size() >= EH + 5 + n + 16 ? rec.substr(EH + 5, n) : std::string();
  };
  bool any_v = false;
  for (int p = 0; p < nranks_; ++p) any_v = any_v || (p != root && all[p].size() > EH && all[p][EH] == 'V');
  std::string need;
  if (any_v) {
    std::string mine_need;
    if (rank_ == root) {
      mine_need.assign(nranks_, '0');
      for (int p = 0; p < nranks_; ++p)
        if (p != root && all[p].size() > EH && all[p][EH] == 'V' &&
            !(mapped_vmm_[p] && mapped_[p].size() == 1 && mapped_[p][0].first == vname(all[p])))
          mine_need[p] = '1';
    }
    const std::vector<std::string> needs = allgather_(mine_need);
    need = needs[root];
  }
  // The root maps the blocks and enqueues the pulls; a second status round
  // tells the peers whether that worked (they would otherwise wait for a
  // gather that never comes in wait()'s rendezvous).
  std::string status("1");
  try {
    if (rank_ == root) {
      // Every copy stream starts behind the root's own stream: its earlier work
      // on dst (a fill, a previous consumer of a reused allocation) comes first.
      for (int k = 0; k < used_; ++k) IGG_HIP_CHECK(hipStreamWaitEvent(side_[k], ready_, 0));
      for (int p = 0; p < nranks_; ++p) {
        const Int3 c{p / (dims[1] * dims[2]), (p / dims[2]) % dims[1], p % dims[2]};
        hipStream_t s = side_[p % nside];
        const void* src = nullptr;
        if (p == root) {
          src = reinterpret_cast<const void*>(a.ptr);
        } else {
          const std::string& rec = all[p];
          if (rec.size() < EH + 1) fail("gather_async: malformed handles from rank ", p);
          const std::string ekey = rec.substr(0, EH);
          if (peer_key_[p] != ekey) {  // opened once per peer event
            if (peer_ev_[p]) IGG_HIP_CHECK(hipEventDestroy(peer_ev_[p]));
            hipIpcEventHandle_t peh;
            std::memcpy(&peh, ekey.data(), EH);
            IGG_HIP_CHECK(hipIpcOpenEventHandle(&peer_ev_[p], peh));
            peer_key_[p] = ekey;
          }
          IGG_HIP_CHECK(hipStreamWaitEvent(s, peer_ev_[p], 0));
          const char mode = rec[EH];
          if (mode == 'V') {
            const std::string name = vname(rec);
            if (name.empty()) fail("gather_async: malformed VMM record from rank ", p);
            const size_t n = name.size();
            uint64_t vsz = 0, off = 0;
            std::memcpy(&vsz, rec.data() + EH + 5 + n, 8);
            std::memcpy(&off, rec.data() + EH + 13 + n, 8);
            if (need.size() == static_cast<size_t>(nranks_) && need[p] == '1') {
              close_mapped(p);
              inject_fail("gather_open");
              const int fd = fd_fetch(name, first_contact_timeout());
              void* q = nullptr;
              try {
                q = vmm_import_fd(fd, vsz, first_contact_timeout());
              } catch (...) {
                fd_close(fd);
                throw;
              }
              fd_close(fd);
              mapped_[p].emplace_back(name, q);
              mapped_vmm_[p] = 1;
            }
            copy_block(static_cast<const char*>(mapped_[p][0].second) + off, dst, a.size, dims, c, 0, a.size[0],
                       a.elem_bytes, s);
            continue;
          }
          const size_t nbuf = mode == 'C' && rec.size() >= EH + 9 ? get_u32(rec, EH + 1) : 1;
          const size_t hdr = mode == 'C' ? EH + 9 : EH + 1;
          if ((mode != 'C' && mode != 'D') || (mode == 'D' && rec.size() != hdr + MH + 8) ||
              (mode == 'C' && rec.size() != hdr + nbuf * MH))
            fail("gather_async: malformed handles from rank ", p);
          auto& per = mapped_[p];
          bool changed = per.size() != nbuf;
          for (size_t k = 0; k < nbuf && !changed; ++k) changed = per[k].first != rec.substr(hdr + k * MH, MH);
          if (changed || mapped_vmm_[p]) {  // this rank's array (or staging) lives in other allocations now
            close_mapped(p);
            inject_fail("gather_open");
            for (size_t k = 0; k < nbuf; ++k) {
              const std::string key = rec.substr(hdr + k * MH, MH);
              per.emplace_back(key, ipc_open(key));
            }
          }
          if (mode == 'C') {
            const int64_t ppc = get_u32(rec, EH + 5);
            for (size_t k = 0; k < nbuf; ++k) {
              const int64_t x0 = static_cast<int64_t>(k) * ppc;
              copy_block(per[k].second, dst, a.size, dims, c, x0, std::min<int64_t>(ppc, a.size[0] - x0),
                         a.elem_bytes, s);
            }
            continue;
          }
          uint64_t off = 0;
          std::memcpy(&off, rec.data() + hdr + MH, 8);
          src = static_cast<const char*>(per[0].second) + off;
        }
        // the root's own block under snapshot: copied on the caller's stream
        // now, so `a` may change right after start() like on the other ranks
        copy_block(src, dst, a.size, dims, c, 0, a.size[0], a.elem_bytes, (snapshot && p == root) ? stream : s);
      }
      for (int k = 0; k < used_; ++k) IGG_HIP_CHECK(hipEventRecord(done_[k], side_[k]));
    } else {
      // the root asked for this rank's VMM descriptor: hand it over (bounded)
      if (need.size() == static_cast<size_t>(nranks_) && need[rank_] == '1') {
        if (cur_vexp_ < 0) fail("gather_async: the root asked for a VMM export this rank did not publish");
        VmmExport& e = vexp_[cur_vexp_];
        if (e.fd < 0) e.fd = export_fd(e.base, e.dmabuf);  // served and closed before: export again
        fd_serve(e.listener, e.fd, 1, first_contact_timeout());
        if (e.dmabuf) {  // the root holds its own reference now; ours would keep a freed array alive
          fd_close(e.fd);
          e.fd = -1;
        }
      }
      const std::string& rec = all[root];
      if (rec.size() != EH * (1 + used_)) fail("gather_async: malformed handles from the root");
      if (static_cast<int>(root_done_.size()) < used_) {
        root_done_.resize(used_, nullptr);
        root_key_.resize(used_);
      }
      for (int k = 0; k < used_; ++k) {
        const std::string key = rec.substr(EH * (1 + k), EH);
        if (root_key_[k] != key) {
          if (root_done_[k]) IGG_HIP_CHECK(hipEventDestroy(root_done_[k]));
          hipIpcEventHandle_t h;
          std::memcpy(&h, key.data(), EH);
          IGG_HIP_CHECK(hipIpcOpenEventHandle(&root_done_[k], h));
          root_key_[k] = key;
        }
      }
    }
  } catch (const Error& e) {
    status = std::string("0") + e.what();
  }
  const std::vector<std::string> st = allgather_(status);
  for (int r = 0; r < static_cast<int>(st.size()); ++r)
    if (st[r].empty() || st[r][0] != '1')
      fail("gather_async: rank ", r, " could not map or pull the blocks",
           st[r].size() > 1 ? std::string(" (") + st[r].substr(1, 300) + ")" : std::string());
  root_ = root;
  pending_ = true;
}

void PullGatherer::wait(hipStream_t stream) {
  TraceRange tr("igg.gather_async.wait");
  if (!pending_) fail("gather_async: no pending gather");
  if (rank_ == root_)
    for (int k = 0; k < used_; ++k) IGG_HIP_CHECK(hipStreamWaitEvent(stream, done_[k], 0));  // later work on dst
  // The root recorded its done events in start(), before this rendezvous: from
  // here on every rank's waits refer to this gather's records.
  (void)allgather_(std::string());
  if (rank_ != root_)
    for (int k = 0; k < used_; ++k) IGG_HIP_CHECK(hipStreamWaitEvent(stream, root_done_[k], 0));  // later writes to `a`
  pending_ = false;
}

}  // namespace igg
