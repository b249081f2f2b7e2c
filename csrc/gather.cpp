// Device gather-to-root (see include/igg/gather.hpp).
#include "igg/gather.hpp"
#include "igg/trace.hpp"

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

}  // namespace igg
