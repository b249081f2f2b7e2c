#pragma once
// Device-side flag primitives of the one-sided exchanges (device code): the
// flag words live in uncached memory (PutFlags, put.hpp), so relaxed
// system-scope accesses reach memory on every poll. Shared by the put sync
// kernels (put_kernels.hip) and the in-kernel step synchronisation of the
// fused acoustic exchange (acoustic_kernels.hip).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "igg/put.hpp"

namespace igg {

// Relaxed system-scope store: flag stores follow one explicit system-scope
// release fence where one is needed (a release store per flag would emit its
// own L2 write-back, ~1.7 us each on gfx950).
__device__ __forceinline__ void store_sys_relaxed(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ uint64_t load_sys_relaxed(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Spin until *p >= v; false (and `code` recorded in the sticky ERROR word of
// `my_flags`) on timeout. The poll is relaxed (system scope: it bypasses the
// caches and sees the peer's store); the caller issues the acquire fence it
// needs after the spin (an acquire load per poll would invalidate the caches
// on every iteration). Once an exchange has timed out (ERROR set), later waits
// give up at once: a dead or diverged peer costs ONE timeout, not one per step
// (the host reports the error at its next check and the data is invalid
// anyway).
__device__ inline bool spin_geq(const uint64_t* p, uint64_t v, uint64_t* my_flags, int64_t timeout_ticks,
                                uint64_t code) {
  const long long t0 = wall_clock64();
  while (load_sys_relaxed(p) < v) {
    __builtin_amdgcn_s_sleep(2);
    if (load_sys_relaxed(my_flags + PutFlags::ERROR) != 0) return false;
    if (wall_clock64() - t0 > timeout_ticks) {
      uint64_t expected = 0;
      __hip_atomic_compare_exchange_strong(my_flags + PutFlags::ERROR, &expected, code, __ATOMIC_RELAXED,
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return false;
    }
  }
  return true;
}

// StepSync (put.hpp), at the start of an exchanging wave: returns c, the
// number of completed steps (this is step c + 1), after every neighbour has
// completed step c. EPOCH is advanced only by the last exchanging wave of this
// kernel, after every exchanging wave read it. The system acquire drops any
// stale copy of a received halo from this CU's L1 before the sweep loads it
// (the L2 copies were invalidated by the writers' coherent stores).
__device__ inline uint64_t step_sync_enter(const StepSync& s, int lane) {
  const uint64_t c = load_sys_relaxed(s.my_flags + PutFlags::EPOCH);
  if (lane < s.n_peers)
    spin_geq(s.my_flags + PutFlags::ARRIVED + s.peer_rank[lane], c, s.my_flags, s.timeout_ticks, 0x300 + lane);
  if (s.acquire >= 2) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  else if (s.acquire == 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  else __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  return c;
}

// At the end of an exchanging wave: its system-scope sends acknowledged and
// every load returned (s_waitcnt 0), it counts itself; the last one publishes
// step c + 1 (ARRIVED at every neighbour, then own EPOCH).
__device__ inline void step_sync_exit(const StepSync& s, int lane, uint64_t c) {
  __builtin_amdgcn_s_waitcnt(0);
  uint64_t old = 0;
  if (lane == 0)
    old = __hip_atomic_fetch_add(s.my_flags + PutFlags::COUNT, uint64_t{1}, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  old = __shfl(old, 0);
  if (old + 1 == static_cast<uint64_t>(s.feat_waves)) {
    if (lane == 0) __hip_atomic_store(s.my_flags + PutFlags::COUNT, uint64_t{0}, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (lane < s.n_peers) store_sys_relaxed(s.peer_flags[lane] + PutFlags::ARRIVED + s.my_rank, c + 1);
    if (lane == 0) store_sys_relaxed(s.my_flags + PutFlags::EPOCH, c + 1);
  }
}

// Per-workgroup forms for kernels whose workgroups hold several exchanging
// waves (diffusion3d_hx_kernel). `wsync` is the workgroup's LDS block
// {entered, go, c, retired}, zeroed behind a barrier before any wave uses it.
// Enter: the workgroup's first exchanging wave runs step_sync_enter (the
// flag polls and the system acquire, which also drops stale lines from the
// CU's L1 that every wave of the workgroup shares) and publishes c in LDS;
// the others wait for it there. The poller is a wave of the same (resident)
// workgroup and sets `go` even after a timed-out wait, so the waiters always
// finish.
__device__ inline uint64_t step_sync_enter_wg(const StepSync& s, int lane, uint64_t* wsync) {
  uint64_t first = 0;
  if (lane == 0)
    first = __hip_atomic_fetch_add(wsync + 0, uint64_t{1}, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  first = __shfl(first, 0);
  if (first == 0) {
    const uint64_t c = step_sync_enter(s, lane);
    if (lane == 0) {
      wsync[2] = c;
      __hip_atomic_store(wsync + 1, uint64_t{1}, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    return c;
  }
  while (__hip_atomic_load(wsync + 1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) __builtin_amdgcn_s_sleep(1);
  return wsync[2];
}

// Exit: every exchanging wave waits for its own stores (s_waitcnt 0) and
// counts itself in LDS; the workgroup's last one counts the workgroup in
// COUNT (step_sync_exit; StepSync::feat_waves = exchanging workgroups), and
// the launch's last workgroup publishes step c + 1.
__device__ inline void step_sync_exit_wg(const StepSync& s, int lane, uint64_t c, uint64_t* wsync, int n_ex) {
  __builtin_amdgcn_s_waitcnt(0);
  uint64_t old = 0;
  if (lane == 0) old = __hip_atomic_fetch_add(wsync + 3, uint64_t{1}, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
  old = __shfl(old, 0);
  if (old + 1 == static_cast<uint64_t>(n_ex)) step_sync_exit(s, lane, c);
}

}  // namespace igg
