// RCCL transport (see include/igg/comm.hpp).
// Replaces the reference's per-(side, field) MPI.Irecv!/Isend with tag 0
// (update_halo.jl:713-735) by one ncclGroupStart/End of raw-byte ncclSend/ncclRecv
// per exchange phase on the halo stream.
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include "igg/comm.hpp"
#include "igg/fault.hpp"

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

RcclComm::RcclComm(const std::vector<uint8_t>& uid, int nranks, int rank, double timeout_s)
    : rank_(rank), nranks_(nranks), timeout_s_(timeout_s > 0 ? timeout_s : first_contact_timeout()) {
  if (uid.size() != sizeof(ncclUniqueId)) fail("RcclComm: bad unique id size ", uid.size());
  ncclUniqueId id;
  std::memcpy(&id, uid.data(), sizeof(id));
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  // Non-blocking communicator: the bootstrap (a TCP rendezvous of all ranks,
  // then the topology exchange) runs in RCCL's background and this thread
  // polls it with a deadline, so a rank that never arrives fails the
  // initialisation instead of blocking it forever; ncclCommAbort then
  // releases the half-built communicator. IGG_RCCL_BLOCKING=1 restores the
  // blocking form.
  const char* blk = std::getenv("IGG_RCCL_BLOCKING");
  cfg.blocking = (blk && blk[0] == '1') ? 1 : 0;
  // IGG_RCCL_MAX_CTAS caps the workgroups (channels) of RCCL's kernels, which
  // otherwise take CUs from a concurrently running interior stencil in the
  // overlapped step (RCCL interplay). Unset = RCCL's default.
  const char* env = std::getenv("IGG_RCCL_MAX_CTAS");
  const int max_ctas = env ? std::atoi(env) : 0;
  if (max_ctas > 0) {
    cfg.minCTAs = 1;
    cfg.maxCTAs = max_ctas;
  }
  inject_delay("rccl_init");
  const ncclResult_t r = ncclCommInitRankConfig(&comm_, nranks, id, rank, &cfg);
  if (r != ncclSuccess && r != ncclInProgress) {
    if (comm_) (void)ncclCommAbort(comm_);
    comm_ = nullptr;
    fail("RCCL error '", ncclGetErrorString(r), "' in ncclCommInitRankConfig (rank ", rank, " of ", nranks, ")");
  }
  try {
    wait_ready("ncclCommInitRankConfig (communicator bootstrap)");
  } catch (...) {
    comm_ = nullptr;  // aborted by wait_ready
    throw;
  }
  IGG_HIP_CHECK(hipMalloc(&scratch_, 256));
  IGG_HIP_CHECK(hipMemset(scratch_, 0, 256));
  IGG_HIP_CHECK(hipDeviceSynchronize());
}

RcclComm::~RcclComm() {
  if (scratch_) (void)hipFree(scratch_);
  if (!comm_ || aborted_) return;
  // Finalize (flushes outstanding work; non-blocking: polled with a bound),
  // then destroy; a communicator that cannot finalize is aborted instead.
  ncclResult_t st = ncclCommFinalize(comm_);
  const auto t0 = std::chrono::steady_clock::now();
  while (st == ncclInProgress || st == ncclSuccess) {
    if (ncclCommGetAsyncError(comm_, &st) != ncclSuccess) break;
    if (st != ncclInProgress) break;
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > 10.0) break;
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
  if (st == ncclSuccess) (void)ncclCommDestroy(comm_);
  else (void)ncclCommAbort(comm_);
  comm_ = nullptr;
}

void RcclComm::wait_ready(const char* what) {
  // Poll the communicator's state until the last call completed (ncclSuccess),
  // failed, or the deadline passed (then abort: RCCL work waiting on a peer
  // exits, and every later call raises).
  const auto t0 = std::chrono::steady_clock::now();
  for (int spins = 0;; ++spins) {
    ncclResult_t st = ncclSuccess;
    const ncclResult_t q = ncclCommGetAsyncError(comm_, &st);
    if (q != ncclSuccess) st = q;
    if (st == ncclSuccess) return;
    if (st != ncclInProgress) {
      (void)ncclCommAbort(comm_);
      aborted_ = true;
      fail("RCCL error '", ncclGetErrorString(st), "' in ", what, " (rank ", rank_, " of ", nranks_, ")");
    }
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s_) {
      (void)ncclCommAbort(comm_);
      aborted_ = true;
      fail(what, " did not complete within ", timeout_s_, " s on rank ", rank_, " of ", nranks_,
           " (a peer rank never arrived?); the RCCL communicator was aborted");
    }
    if (spins < 1000) std::this_thread::yield();
    else std::this_thread::sleep_for(std::chrono::microseconds(500));
  }
}

void RcclComm::settle(int result, const char* what) {
  const ncclResult_t r = static_cast<ncclResult_t>(result);
  if (r == ncclSuccess) return;
  if (r == ncclInProgress) {  // non-blocking: a first contact (p2p connection setup) runs in the background
    wait_ready(what);
    return;
  }
  fail("RCCL error '", ncclGetErrorString(r), "' in ", what);
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
  settle(ncclGroupEnd(), "ncclGroupEnd (halo send/recv group)");
}

void RcclComm::barrier(hipStream_t stream) {
  if (aborted_) fail("RCCL communicator was aborted");
  settle(ncclAllReduce(scratch_, scratch_, 1, ncclInt32, ncclSum, comm_, stream), "ncclAllReduce (barrier)");
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
  settle(ncclAllReduce(send, recv, count, nccl_type(dtype), nccl_op(op), comm_, stream), "ncclAllReduce");
}

void RcclComm::broadcast(const void* send, void* recv, size_t count, int dtype, int root, hipStream_t stream) {
  if (aborted_) fail("RCCL communicator was aborted");
  if (root < 0 || root >= nranks_) fail("RcclComm.broadcast: root ", root, " out of range");
  if (count == 0) return;
  settle(ncclBroadcast(send, recv, count, nccl_type(dtype), root, comm_, stream), "ncclBroadcast");
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
