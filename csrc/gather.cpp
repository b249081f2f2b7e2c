// Device gather-to-root (see include/igg/gather.hpp).
#include "igg/gather.hpp"
#include "igg/trace.hpp"
#include "igg/ipc.hpp"

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

PullGatherer::PullGatherer(int rank, int nranks, AllGather allgather)
    : rank_(rank), nranks_(nranks), allgather_(std::move(allgather)) {}

PullGatherer::~PullGatherer() {
  if (side_) (void)hipStreamSynchronize(side_);
  for (auto& o : opened_) (void)hipIpcCloseMemHandle(o.second);
  opened_.clear();
  if (buf_) (void)hipFree(buf_);
  if (done_) (void)hipEventDestroy(done_);
  if (side_) (void)hipStreamDestroy(side_);
}

void PullGatherer::free() {
  if (pending_) fail("gather_async: free while a gather is pending (call wait() first)");
  if (side_) IGG_HIP_CHECK(hipStreamSynchronize(side_));
  for (auto& o : opened_) (void)hipIpcCloseMemHandle(o.second);
  opened_.clear();
  if (buf_) {
    IGG_HIP_CHECK(hipDeviceSynchronize());
    IGG_HIP_CHECK(hipFree(buf_));
  }
  buf_ = nullptr;
  bytes_ = 0;
}

void PullGatherer::start(const Field& a, int root, const Int3& dims) {
  TraceRange tr("igg.gather_async.start");
  if (pending_) fail("gather_async: a gather is already pending (call wait() first)");
  if (!a.device) fail("gather_async: the local array must be a GPU array.");
  if (dims[0] * dims[1] * dims[2] != nranks_) fail("gather_async: dims do not match the number of processes.");
  const size_t blk = static_cast<size_t>(a.size[0] * a.size[1] * a.size[2]) * a.elem_bytes;
  if (!side_) {
    IGG_HIP_CHECK(hipStreamCreateWithFlags(&side_, hipStreamNonBlocking));
    IGG_HIP_CHECK(hipEventCreateWithFlags(&done_, hipEventDisableTiming));
  }
  // `a` must be final before the root's copy engines read it.
  IGG_HIP_CHECK(hipDeviceSynchronize());
  std::string mine;
  if (rank_ != root) {
    void* base = nullptr;
    size_t size = 0;
    IGG_HIP_CHECK(hipMemGetAddressRange(&base, &size, reinterpret_cast<void*>(a.ptr)));
    hipIpcMemHandle_t h;
    IGG_HIP_CHECK(hipIpcGetMemHandle(&h, base));
    const uint64_t off = a.ptr - reinterpret_cast<uintptr_t>(base);
    mine.assign(reinterpret_cast<const char*>(&h), sizeof(h));
    mine.append(reinterpret_cast<const char*>(&off), sizeof(off));
  }
  const std::vector<std::string> all = allgather_(mine);
  if (rank_ == root) {
    const size_t need = blk * static_cast<size_t>(nranks_);
    if (bytes_ < need) {
      if (buf_) {
        IGG_HIP_CHECK(hipDeviceSynchronize());
        IGG_HIP_CHECK(hipFree(buf_));
      }
      IGG_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&buf_), need));
      bytes_ = need;
    }
    for (int p = 0; p < nranks_; ++p) {
      char* dst = buf_ + static_cast<size_t>(p) * blk;
      if (p == root) {
        IGG_HIP_CHECK(hipMemcpyAsync(dst, reinterpret_cast<const void*>(a.ptr), blk, hipMemcpyDeviceToDevice, side_));
        continue;
      }
      const std::string& rec = all[p];
      if (rec.size() != sizeof(hipIpcMemHandle_t) + 8) fail("gather_async: malformed handle from rank ", p);
      const std::string hkey = rec.substr(0, sizeof(hipIpcMemHandle_t));
      uint64_t off = 0;
      std::memcpy(&off, rec.data() + sizeof(hipIpcMemHandle_t), 8);
      // Mapped for this gather only: the peer may free its array after wait().
      void* base = ipc_open(hkey);
      opened_.emplace_back(hkey, base);
      IGG_HIP_CHECK(hipMemcpyAsync(dst, static_cast<const char*>(base) + off, blk, hipMemcpyDeviceToDevice, side_));
    }
    IGG_HIP_CHECK(hipEventRecord(done_, side_));
  }
  field_ = a;
  root_ = root;
  dims_ = dims;
  pending_ = true;
}

void PullGatherer::wait(void* dst, hipStream_t stream) {
  TraceRange tr("igg.gather_async.wait");
  if (!pending_) fail("gather_async: no pending gather");
  if (rank_ == root_) {
    if (!dst) fail("The input argument A_global can't be `nothing` on the root");
    IGG_HIP_CHECK(hipStreamWaitEvent(stream, done_, 0));
    launch_gather_reorder(buf_, dst, field_.size, dims_, field_.elem_bytes, stream);
    IGG_HIP_CHECK(hipEventSynchronize(done_));  // pulls done: peers may reuse their arrays
    for (auto& o : opened_) ipc_close(o.second);
    opened_.clear();
  }
  (void)allgather_(std::string());
  pending_ = false;
}

}  // namespace igg
