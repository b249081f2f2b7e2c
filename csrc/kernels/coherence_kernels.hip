// Coherence probe kernels (igg/coherence.hpp; tests/test_coherence.py).
#include <hip/hip_runtime.h>

#include <utility>

#include "igg/coherence.hpp"
#include "igg/common.hpp"
#include "igg/devsync.hpp"
#include "igg/sysstore.hpp"

namespace igg {
namespace {

constexpr int BLOCK = 256;  // 4 waves
constexpr int WAVES = BLOCK / 64;

// Every workgroup reads EVERY word of the arena (lanes stride by the block),
// so each XCD - workgroups are dealt round-robin to the XCDs - loads every
// line into its L2 and each CU into its L1. mode 0: warm (XOR into sink);
// mode 1: compare with `expect`; mode 2: step_sync_enter_wg first, compare,
// then step_sync_exit_wg (the in-kernel form of the fused exchange).
__global__ void __launch_bounds__(BLOCK) coh_read_kernel(const uint64_t* __restrict__ a, int64_t n, uint64_t expect,
                                                        unsigned long long* bad, uint64_t* sink, StepSync s,
                                                        int mode) {
  __shared__ uint64_t wsync[4];
  const int lane = threadIdx.x & 63;
  uint64_t c = 0;
  if (mode == 2) {
    if (threadIdx.x < 4) wsync[threadIdx.x] = 0;
    __syncthreads();
    c = step_sync_enter_wg(s, lane, wsync);
  }
  uint64_t acc = 0;
  unsigned long long nbad = 0;
  for (int64_t i = threadIdx.x; i < n; i += BLOCK) {
    const uint64_t v = a[i];
    acc ^= v;
    nbad += v != expect;
  }
  if (mode == 0) {
    sink[static_cast<int64_t>(blockIdx.x) * BLOCK + threadIdx.x] = acc;
  } else if (nbad) {
    atomicAdd(bad, nbad);
  }
  if (mode == 2) step_sync_exit_wg(s, lane, c, wsync, WAVES);
}

// W: the production system-scope store of every word (write-through, its
// acknowledgement means the bytes left for R's memory), then either nothing
// (a put_sync_kernel publishes next on the stream) or the in-kernel exit.
__global__ void __launch_bounds__(BLOCK) coh_write_kernel(uint64_t* a, int64_t n, uint64_t value, StepSync s,
                                                         int in_kernel, int plain) {
  __shared__ uint64_t wsync[4];
  const int lane = threadIdx.x & 63;
  uint64_t c = 0;
  if (in_kernel) {
    if (threadIdx.x < 4) wsync[threadIdx.x] = 0;
    __syncthreads();
    c = step_sync_enter_wg(s, lane, wsync);
  }
  const int64_t stride = static_cast<int64_t>(gridDim.x) * BLOCK;
  // plain (positive control only): write-back stores, which may stay dirty in
  // this XCD's L2 - the writer-side hazard the production st_sys avoids
  if (plain) {
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * BLOCK + threadIdx.x; i < n; i += stride) a[i] = value;
  } else {
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * BLOCK + threadIdx.x; i < n; i += stride) st_sys(a + i, value);
  }
  __builtin_amdgcn_s_waitcnt(0);
  if (in_kernel) step_sync_exit_wg(s, lane, c, wsync, WAVES);
}

// Negative control (no acquire): every workgroup reads the arena (warm),
// waits until W's ARRIVED reaches `target` with relaxed polls only (no fence,
// no kernel boundary), then reads every word again - plain loads (which may
// hit this CU's L1 and the XCD's L2) or, `l2`, loads that skip the L1 (sc0),
// which can hit only the L2 - and counts the words still != value. A nonzero
// count shows that the caches DO hold stale lines, i.e. that the production
// forms' zero comes from their synchronisation, not from an uncached arena.
__global__ void __launch_bounds__(BLOCK) coh_control_kernel(const uint64_t* __restrict__ a, int64_t n, uint64_t value,
                                                           unsigned long long* bad, uint64_t* sink,
                                                           const uint64_t* arrived, uint64_t target,
                                                           uint64_t* my_flags, int64_t timeout, int l2) {
  uint64_t acc = 0;
  for (int64_t i = threadIdx.x; i < n; i += BLOCK) acc ^= a[i];
  sink[static_cast<int64_t>(blockIdx.x) * BLOCK + threadIdx.x] = acc;
  if (threadIdx.x == 0) spin_geq(arrived, target, my_flags, timeout, 0x500);
  __syncthreads();
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint64_t*>(a), static_cast<short>(0), 0x7fffffff, 0x00020000);
  unsigned long long nbad = 0;
  for (int64_t i = threadIdx.x; i < n; i += BLOCK) {
    uint64_t v;
    if (l2) {
      v = __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(rs, static_cast<int>(i * 8), 0, 1));
    } else {
      v = a[i];
    }
    nbad += v != value;
  }
  if (nbad) atomicAdd(bad, nbad);
}

StepSync probe_sync(const PeerMesh& m, int64_t units) {
  StepSync s;
  const int peer = 1 - m.rank();
  s.my_flags = m.flags(m.rank());
  s.peer_flags[0] = m.flags(peer);
  s.peer_rank[0] = peer;
  s.n_peers = 1;
  s.my_rank = m.rank();
  s.timeout_ticks = m.timeout_ticks();
  s.feat_waves = units;
  s.acquire = 2;
  return s;
}

PutSync probe_put_sync(const PeerMesh& m) {
  PutSync p{};
  p.my_flags = m.flags(m.rank());
  p.my_rank = m.rank();
  p.nranks = m.nranks();
  p.timeout_ticks = m.timeout_ticks();
  if (m.rank() == 1) {  // W publishes to R
    p.n_out = 1;
    p.out_flags[0] = m.flags(0);
    p.out_rank[0] = 0;
  } else {  // R waits for W
    p.n_in = 1;
    p.in_rank[0] = 1;
  }
  return p;
}

}  // namespace

CoherenceProbe::CoherenceProbe(std::shared_ptr<PeerMesh> mesh, size_t bytes) : mesh_(std::move(mesh)) {
  if (mesh_->nranks() != 2) fail("CoherenceProbe: a 2-rank mesh (reader 0, writer 1) expected");
  if (bytes < 4096 || bytes > (size_t{64} << 20) || bytes % 8) fail("CoherenceProbe: 4 KiB .. 64 MiB of words");
  mesh_->ensure_arena(bytes);  // collective; zero-filled fine-grained memory (the production arena)
  words_ = bytes / 8;
  int dev = 0, cus = 0;
  IGG_HIP_CHECK(hipGetDevice(&dev));
  IGG_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  wgs_ = 2 * cus;
  IGG_HIP_CHECK(hipMalloc(&bad_, sizeof(unsigned long long)));
  IGG_HIP_CHECK(hipMalloc(&sink_, sizeof(uint64_t) * BLOCK * wgs_));
}

CoherenceProbe::~CoherenceProbe() {
  (void)hipDeviceSynchronize();
  if (bad_) (void)hipFree(bad_);
  if (sink_) (void)hipFree(sink_);
}

void CoherenceProbe::warm(hipStream_t s) {
  if (mesh_->rank() != 0) fail("CoherenceProbe.warm: the reader is rank 0");
  hipLaunchKernelGGL(coh_read_kernel, dim3(wgs_), dim3(BLOCK), 0, s,
                     reinterpret_cast<const uint64_t*>(mesh_->arena(0)), static_cast<int64_t>(words_), uint64_t{0},
                     bad_, sink_, StepSync{}, 0);
  IGG_HIP_CHECK(hipGetLastError());
}

void CoherenceProbe::write(uint64_t value, bool in_kernel, hipStream_t s, bool plain) {
  if (mesh_->rank() != 1) fail("CoherenceProbe.write: the writer is rank 1");
  const int wg = wgs_ / 2;  // every workgroup resident (the exit counts them all)
  hipLaunchKernelGGL(coh_write_kernel, dim3(wg), dim3(BLOCK), 0, s, reinterpret_cast<uint64_t*>(mesh_->arena(0)),
                     static_cast<int64_t>(words_), value, in_kernel ? probe_sync(*mesh_, wg) : StepSync{},
                     in_kernel ? 1 : 0, plain ? 1 : 0);
  IGG_HIP_CHECK(hipGetLastError());
  if (!in_kernel) launch_put_sync(probe_put_sync(*mesh_), s);
}

void CoherenceProbe::control(uint64_t value, uint64_t target, bool l2, hipStream_t s) {
  if (mesh_->rank() != 0) fail("CoherenceProbe.control: the reader is rank 0");
  IGG_HIP_CHECK(hipMemsetAsync(bad_, 0, sizeof(unsigned long long), s));
  uint64_t* f = mesh_->flags(0);
  hipLaunchKernelGGL(coh_control_kernel, dim3(wgs_), dim3(BLOCK), 0, s,
                     reinterpret_cast<const uint64_t*>(mesh_->arena(0)), static_cast<int64_t>(words_), value, bad_,
                     sink_, f + PutFlags::ARRIVED + 1, target, f, mesh_->timeout_ticks(), l2 ? 1 : 0);
  IGG_HIP_CHECK(hipGetLastError());
}

int64_t CoherenceProbe::mismatches(hipStream_t s) {
  unsigned long long h = 0;
  IGG_HIP_CHECK(hipMemcpyAsync(&h, bad_, sizeof(h), hipMemcpyDeviceToHost, s));
  IGG_HIP_CHECK(hipStreamSynchronize(s));
  return static_cast<int64_t>(h);
}

int64_t CoherenceProbe::check(uint64_t value, bool in_kernel, hipStream_t s) {
  if (mesh_->rank() != 0) fail("CoherenceProbe.check: the reader is rank 0");
  IGG_HIP_CHECK(hipMemsetAsync(bad_, 0, sizeof(unsigned long long), s));
  if (!in_kernel) launch_put_sync(probe_put_sync(*mesh_), s);
  hipLaunchKernelGGL(coh_read_kernel, dim3(wgs_), dim3(BLOCK), 0, s,
                     reinterpret_cast<const uint64_t*>(mesh_->arena(0)), static_cast<int64_t>(words_), value, bad_,
                     sink_, in_kernel ? probe_sync(*mesh_, wgs_) : StepSync{}, in_kernel ? 2 : 1);
  IGG_HIP_CHECK(hipGetLastError());
  unsigned long long h = 0;
  IGG_HIP_CHECK(hipMemcpyAsync(&h, bad_, sizeof(h), hipMemcpyDeviceToHost, s));
  IGG_HIP_CHECK(hipStreamSynchronize(s));
  return static_cast<int64_t>(h);
}

}  // namespace igg
