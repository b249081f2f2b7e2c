// Point-to-point transports for halo and gather traffic.
//
// Reference: every byte moves through MPI.Isend/Irecv with tag 0
// (src/update_halo.jl:713-735, src/gather.jl:33-59); GPU buffers are only used
// when IGG_ROCMAWARE_MPI is set, otherwise data is staged through host memory.
// Here the device path is always device-resident: RCCL ncclSend/ncclRecv of raw
// bytes (ncclUint8, so any element type incl. complex/half works) grouped in one
// ncclGroupStart/End per exchange phase, enqueued on a HIP stream — no host
// synchronisation. Ops are issued in the order given; for a peer that is both
// left and right neighbour (dims==2, periodic) the engine orders receives
// right-then-left and sends left-then-right, which RCCL matches in order
// (SURVEY.md §2.4 invariant 4).
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "igg/common.hpp"

typedef struct ncclComm* ncclComm_t;

namespace igg {

struct P2POp {
  void* ptr;
  size_t bytes;
  int peer;
  int tag;  // used by tag-matching transports (gloo); RCCL matches by order
};

class Transport {
 public:
  virtual ~Transport() = default;
  virtual bool device_capable() const = 0;
  virtual bool host_capable() const = 0;
  virtual std::string name() const = 0;
  // Post all receives then all sends as one phase; complete (or stream-order)
  // them before returning.
  virtual void exchange(const std::vector<P2POp>& recvs, const std::vector<P2POp>& sends,
                        bool device, hipStream_t stream) = 0;
};

// Native RCCL communicator over the node's xGMI links.
class RcclComm : public Transport {
 public:
  static constexpr size_t UID_BYTES = 128;
  static std::vector<uint8_t> unique_id();
  // Bounded bootstrap: a non-blocking communicator polled for at most
  // `timeout_s` seconds (<= 0: first_contact_timeout(), IGG_FIRST_CONTACT_TIMEOUT);
  // on expiry it is aborted and igg::Error raised. Callers make the outcome
  // collective (parallel/comm.py ensure_rccl: every rank raises together).
  RcclComm(const std::vector<uint8_t>& uid, int nranks, int rank, double timeout_s = 0);
  ~RcclComm() override;
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  bool device_capable() const override { return true; }
  bool host_capable() const override { return false; }
  std::string name() const override { return "rccl"; }
  void exchange(const std::vector<P2POp>& recvs, const std::vector<P2POp>& sends, bool device,
                hipStream_t stream) override;

  // Device-side barrier: 1-element all-reduce on `stream` (caller syncs).
  void barrier(hipStream_t stream);
  // Collectives on raw device buffers, enqueued on `stream` (comm_cart interop:
  // the applications' MPI.Allreduce!/MPI.Bcast! on the grid communicator,
  // README.md:166-178 of the reference). dtype: DType codes below; op:
  // 0 sum, 1 prod, 2 max, 3 min. In place when send == recv.
  enum DType : int { I8 = 0, U8 = 1, I32 = 2, U32 = 3, I64 = 4, U64 = 5, F16 = 6, F32 = 7, F64 = 8, BF16 = 9 };
  void allreduce(const void* send, void* recv, size_t count, int dtype, int op, hipStream_t stream);
  void broadcast(const void* send, void* recv, size_t count, int dtype, int root, hipStream_t stream);
  // Raises igg::Error if the communicator reported an asynchronous failure.
  void check_async_error();
  void abort();
  int rank() const { return rank_; }
  int nranks() const { return nranks_; }
  ncclComm_t handle() const { return comm_; }

 private:
  ncclComm_t comm_ = nullptr;
  int rank_ = 0, nranks_ = 1;
  void* scratch_ = nullptr;  // device int for the barrier
  bool aborted_ = false;
  double timeout_s_ = 120.0;
  // Non-blocking communicator: a call that returned ncclInProgress (the
  // bootstrap, a first p2p contact's connection setup) is polled until it
  // completes, fails, or timeout_s_ passes (then the communicator is aborted).
  void wait_ready(const char* what);
  void settle(int result, const char* what);
};

std::string rccl_version();

}  // namespace igg
