// RCCL transport (see include/igg/comm.hpp).
// Replaces the reference's per-(side, field) MPI.Irecv!/Isend with tag 0
// (update_halo.jl:713-735) by one ncclGroupStart/End of raw-byte ncclSend/ncclRecv
// per exchange phase on the halo stream.
#include <cstdlib>
#include <cstring>

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include "igg/comm.hpp"

#define IGG_NCCL_CHECK(expr)                                                        \
  do {                                                                              \
    ncclResult_t _r = (expr);                                                       \
    if (_r != ncclSuccess)                                                          \
      ::igg::fail("RCCL error '", ncclGetErrorString(_r), "' at ", __FILE__, ":",   \
                  __LINE__, " in ", #expr);                                         \
  } while (0)

namespace igg {

static_assert(sizeof(ncclUniqueId) == RcclComm::UID_BYTES, "unexpected ncclUniqueId size");

std::vector<uint8_t> RcclComm::unique_id() {
  ncclUniqueId id;
  IGG_NCCL_CHECK(ncclGetUniqueId(&id));
  std::vector<uint8_t> out(sizeof(id));
  std::memcpy(out.data(), &id, sizeof(id));
  return out;
}

RcclComm::RcclComm(const std::vector<uint8_t>& uid, int nranks, int rank)
    : rank_(rank), nranks_(nranks) {
  if (uid.size() != sizeof(ncclUniqueId)) fail("RcclComm: bad unique id size ", uid.size());
  ncclUniqueId id;
  std::memcpy(&id, uid.data(), sizeof(id));
  // IGG_RCCL_MAX_CTAS caps the workgroups (channels) of RCCL's kernels, which
  // otherwise take CUs from a concurrently running interior stencil in the
  // overlapped step (RCCL interplay). Unset = RCCL's default.
  const char* env = std::getenv("IGG_RCCL_MAX_CTAS");
  const int max_ctas = env ? std::atoi(env) : 0;
  if (max_ctas > 0) {
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.minCTAs = 1;
    cfg.maxCTAs = max_ctas;
    IGG_NCCL_CHECK(ncclCommInitRankConfig(&comm_, nranks, id, rank, &cfg));
  } else {
    IGG_NCCL_CHECK(ncclCommInitRank(&comm_, nranks, id, rank));
  }
  IGG_HIP_CHECK(hipMalloc(&scratch_, 256));
  IGG_HIP_CHECK(hipMemset(scratch_, 0, 256));
  IGG_HIP_CHECK(hipDeviceSynchronize());
}

RcclComm::~RcclComm() {
  if (scratch_) (void)hipFree(scratch_);
  if (comm_ && !aborted_) (void)ncclCommDestroy(comm_);
}

void RcclComm::exchange(const std::vector<P2POp>& recvs, const std::vector<P2POp>& sends,
                        bool device, hipStream_t stream) {
  if (!device) fail("RCCL transport can only move device (GPU) memory.");
  if (aborted_) fail("RCCL communicator was aborted after a communication failure (IGG_COMM_TIMEOUT); "
                     "re-initialise the grid.");
  if (recvs.empty() && sends.empty()) return;
  IGG_NCCL_CHECK(ncclGroupStart());
  try {
    for (const P2POp& r : recvs)
      IGG_NCCL_CHECK(ncclRecv(r.ptr, r.bytes, ncclUint8, r.peer, comm_, stream));
    for (const P2POp& s : sends)
      IGG_NCCL_CHECK(ncclSend(s.ptr, s.bytes, ncclUint8, s.peer, comm_, stream));
  } catch (...) {
    // Never leave the thread's RCCL group open: a later group would nest into
    // it and hang. The group's own error (if any) is secondary to the first.
    (void)ncclGroupEnd();
    throw;
  }
  IGG_NCCL_CHECK(ncclGroupEnd());
}

void RcclComm::barrier(hipStream_t stream) {
  if (aborted_) fail("RCCL communicator was aborted");
  IGG_NCCL_CHECK(ncclAllReduce(scratch_, scratch_, 1, ncclInt32, ncclSum, comm_, stream));
}

namespace {

ncclDataType_t nccl_type(int d) {
  switch (d) {
    case RcclComm::I8: return ncclInt8;
    case RcclComm::U8: return ncclUint8;
    case RcclComm::I32: return ncclInt32;
    case RcclComm::U32: return ncclUint32;
    case RcclComm::I64: return ncclInt64;
    case RcclComm::U64: return ncclUint64;
    case RcclComm::F16: return ncclFloat16;
    case RcclComm::F32: return ncclFloat32;
    case RcclComm::F64: return ncclFloat64;
    case RcclComm::BF16: return ncclBfloat16;
    default: fail("RcclComm: unsupported dtype code ", d);
  }
  return ncclUint8;
}

ncclRedOp_t nccl_op(int op) {
  switch (op) {
    case 0: return ncclSum;
    case 1: return ncclProd;
    case 2: return ncclMax;
    case 3: return ncclMin;
    default: fail("RcclComm: unsupported reduction op ", op);
  }
  return ncclSum;
}

}  // namespace

void RcclComm::allreduce(const void* send, void* recv, size_t count, int dtype, int op, hipStream_t stream) {
  if (aborted_) fail("RCCL communicator was aborted");
  if (count == 0) return;
  IGG_NCCL_CHECK(ncclAllReduce(send, recv, count, nccl_type(dtype), nccl_op(op), comm_, stream));
}

void RcclComm::broadcast(const void* send, void* recv, size_t count, int dtype, int root, hipStream_t stream) {
  if (aborted_) fail("RCCL communicator was aborted");
  if (root < 0 || root >= nranks_) fail("RcclComm.broadcast: root ", root, " out of range");
  if (count == 0) return;
  IGG_NCCL_CHECK(ncclBroadcast(send, recv, count, nccl_type(dtype), root, comm_, stream));
}

void RcclComm::check_async_error() {
  if (aborted_) fail("RCCL communicator was aborted after a communication failure");
  ncclResult_t st = ncclSuccess;
  IGG_NCCL_CHECK(ncclCommGetAsyncError(comm_, &st));
  if (st != ncclSuccess && st != ncclInProgress)
    fail("RCCL asynchronous error: ", ncclGetErrorString(st));
}

void RcclComm::abort() {
  if (comm_ && !aborted_) {
    (void)ncclCommAbort(comm_);
    aborted_ = true;
  }
}

std::string rccl_version() {
  int v = 0;
  if (ncclGetVersion(&v) != ncclSuccess) return "unknown";
  return std::to_string(v / 10000) + "." + std::to_string((v / 100) % 100) + "." +
         std::to_string(v % 100);
}

}  // namespace igg
