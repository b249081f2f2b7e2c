// Put-transport synchronisation kernels (one workgroup of one wave each).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "igg/common.hpp"
#include "igg/devsync.hpp"
#include "igg/put.hpp"

namespace igg {
namespace {

// Spin until *p >= v (devsync.hpp), then one system acquire that orders the
// caller's later reads.
__device__ bool wait_geq(const uint64_t* p, uint64_t v, const PutSync& s, uint64_t code) {
  if (!spin_geq(p, v, s.my_flags, s.timeout_ticks, code)) return false;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  return true;
}

// The EPOCH word counts completed exchanges (c); exchange e = c + 1.
__global__ void __launch_bounds__(64) put_begin_kernel(const PutSync s) {
  const int lane = threadIdx.x;
  // own EPOCH word: written by this GPU's previous sync kernel (kernel order)
  const uint64_t e = load_sys_relaxed(s.my_flags + PutFlags::EPOCH) + 1;
  const int freed = PutFlags::freed(s.nranks);
  // Each receiver must have finished unpacking exchange e-2 (the last one
  // that used arena half e&1) before my put kernel writes into it.
  if (lane < s.n_out && e > 2) wait_geq(s.my_flags + freed + s.out_rank[lane], e - 2, s, 0x100 + lane);
}

__global__ void __launch_bounds__(64) put_sync_kernel(const PutSync s) {
  __shared__ int ok;
  const int lane = threadIdx.x;
  const uint64_t e = load_sys_relaxed(s.my_flags + PutFlags::EPOCH) + 1;
  const int freed = PutFlags::freed(s.nranks);
  if (lane == 0) ok = 1;
  __syncthreads();
  // My unpack of e-1 completed before this kernel (stream order): release my
  // arena half to every neighbour. The put kernel(s) of e finished with their
  // stores acknowledged; ONE system-scope release fence orders both before the
  // flags, which are then relaxed system-scope stores (round 1 had a full
  // __threadfence_system() plus a release per flag store: four L2 write-backs
  // per exchange, ~5 us of the sync kernel).
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  if (lane < s.n_nb && e > 1) store_sys_relaxed(s.nb_flags[lane] + freed + s.my_rank, e - 1);
  if (lane < s.n_out) store_sys_relaxed(s.out_flags[lane] + PutFlags::ARRIVED + s.my_rank, e);
  if (lane < s.n_in && !wait_geq(s.my_flags + PutFlags::ARRIVED + s.in_rank[lane], e, s, 0x200 + lane)) ok = 0;
  __syncthreads();
  // A timed-out wait (ok == 0) already left its code in the sticky ERROR word
  // (wait_geq); the epoch still advances so the stream drains instead of
  // hanging the GPU. The host reports it at the next check_transport() /
  // update_halo_ poll (IGG_POLL_EVERY) / finalize, never silently.
  (void)ok;
  // exchange e complete (unpack reads parity e): read by this GPU's next
  // kernels on the same stream, ordered by the kernel boundary
  if (lane == 0) store_sys_relaxed(s.my_flags + PutFlags::EPOCH, e);
}

// Failure-path test aid: one wave that spins for `ticks` wall-clock ticks (a
// bounded stand-in for a kernel blocked on a peer that never answers).
__global__ void __launch_bounds__(64) spin_kernel(int64_t ticks) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(10);
}

}  // namespace

void launch_spin(double seconds, hipStream_t stream) {
  if (seconds < 0 || seconds > 60) fail("launch_spin: 0..60 s");
  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, stream, put_timeout_ticks(seconds));
  IGG_HIP_CHECK(hipGetLastError());
}

void launch_put_begin(const PutSync& s, hipStream_t stream) {
  if (s.n_out > 64 || s.n_nb > 64) fail("launch_put_begin: too many peers");
  hipLaunchKernelGGL(put_begin_kernel, dim3(1), dim3(64), 0, stream, s);
  IGG_HIP_CHECK(hipGetLastError());
}

void launch_put_sync(const PutSync& s, hipStream_t stream) {
  if (s.n_out > 64 || s.n_in > 64) fail("launch_put_sync: too many peers");
  hipLaunchKernelGGL(put_sync_kernel, dim3(1), dim3(64), 0, stream, s);
  IGG_HIP_CHECK(hipGetLastError());
}

StepSync step_sync_from(const PutSync& p) {
  if (p.n_in != p.n_out) fail("step_sync_from: asymmetric neighbourhood (", p.n_in, " senders, ", p.n_out, " receivers)");
  if (p.n_in < 1 || p.n_in > STEP_SYNC_MAX_PEERS) fail("step_sync_from: 1..", STEP_SYNC_MAX_PEERS, " peers expected, got ", p.n_in);
  StepSync s;
  s.my_flags = p.my_flags;
  s.n_peers = p.n_in;
  for (int i = 0; i < p.n_in; ++i) {
    if (p.in_rank[i] != p.out_rank[i]) fail("step_sync_from: sender and receiver lists differ");
    s.peer_flags[i] = p.out_flags[i];
    s.peer_rank[i] = p.in_rank[i];
  }
  s.my_rank = p.my_rank;
  s.timeout_ticks = p.timeout_ticks;
  static const int acq = [] {
    const char* e = std::getenv("IGG_STEP_SYNC_ACQUIRE");
    return e && (e[0] == '0' || e[0] == '1') ? e[0] - '0' : 2;
  }();
  s.acquire = acq;
  return s;
}

bool step_sync_in_kernel(bool shares_device, bool by_default) {
  static const int mode = [] {  // -1 auto, 0 in the kernel, 1 sync kernel
    const char* e = std::getenv("IGG_FUSED_SYNC_KERNEL");
    return (e && e[0] == '1') ? 1 : ((e && e[0] == '0') ? 0 : -1);
  }();
  return mode == 0 || (mode < 0 && by_default && !shares_device);
}

int64_t put_timeout_ticks(double seconds) {
  int dev = 0, khz = 0;
  IGG_HIP_CHECK(hipGetDevice(&dev));
  IGG_HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
  if (khz <= 0) khz = 100000;
  return static_cast<int64_t>(seconds * khz * 1000.0);
}

}  // namespace igg
