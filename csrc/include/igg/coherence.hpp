// Coherence probe (tests/test_coherence.py; docs/COHERENCE.md fact 4).
//
// Checks the reader side of the one-sided exchanges with the reader's caches
// deliberately WARM: rank 0 (reader R) first reads its receive arena from two
// workgroups on every CU, so every XCD's L2 holds every line of it (the
// arena is small: nothing streams it out afterwards, unlike the 3 GiB a
// 512^3 step streams between two uses of an arena half); rank 1 (writer W)
// then stores a new value into R's arena through its IPC mapping with the
// production system-scope store (st_sys, sysstore.hpp) and publishes it with
// the production synchronisation; R synchronises the same way and reads
// every word again from every XCD. A stale L2 (or L1) line shows up as a
// mismatch. Two synchronisation forms, as in the fused exchange:
//   * SyncKernel: W's put_sync_kernel publishes ARRIVED (system release +
//     relaxed flag store); R's put_sync_kernel waits for it and acquires
//     (one wave, one XCD); the check kernel follows on R's stream.
//   * InKernel: no sync kernels. W's write kernel ends with
//     step_sync_exit_wg (every wave's st_sys stores acknowledged, the last
//     workgroup publishes ARRIVED, no release fence); R's check kernel starts
//     every workgroup with step_sync_enter_wg (the first wave polls, acquires
//     at system scope, releases the others through LDS) - devsync.hpp.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <memory>

#include "igg/peer.hpp"

namespace igg {

class CoherenceProbe {
 public:
  // Collective over the 2-rank mesh: every rank's arena holds `bytes`.
  CoherenceProbe(std::shared_ptr<PeerMesh> mesh, size_t bytes);
  ~CoherenceProbe();
  // R: every workgroup (2 per CU) reads the whole arena (warms every XCD's L2).
  void warm(hipStream_t s);
  // W: stores `value` into every word of R's arena (st_sys), then publishes:
  // in_kernel false -> put_sync_kernel, true -> step_sync_exit_wg in the kernel.
  // plain: write-back stores instead (positive control of the test's sensitivity).
  void write(uint64_t value, bool in_kernel, hipStream_t s, bool plain = false);
  // R: synchronises with W (put_sync_kernel, or step_sync_enter_wg in every
  // workgroup of the check kernel), then every workgroup compares every word
  // with `value`; returns the number of mismatching reads (stream-synchronous).
  // In-kernel form: R's step c+1 consumes W's step c, so R's first check
  // (value 0, the zero-filled arena) precedes W's first write.
  int64_t check(uint64_t value, bool in_kernel, hipStream_t s);
  // R, negative control: launches (asynchronously) a kernel that warms the
  // caches, waits for ARRIVED[W] >= target with relaxed polls and NO acquire,
  // then re-reads (l2: skipping the L1); mismatches() returns its count.
  void control(uint64_t value, uint64_t target, bool l2, hipStream_t s);
  int64_t mismatches(hipStream_t s);
  int workgroups() const { return wgs_; }
  size_t words() const { return words_; }

 private:
  std::shared_ptr<PeerMesh> mesh_;
  size_t words_ = 0;
  int wgs_ = 0;
  unsigned long long* bad_ = nullptr;  // device counter
  uint64_t* sink_ = nullptr;           // warm kernel output (keeps its loads)
};

}  // namespace igg
