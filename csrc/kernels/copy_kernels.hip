// Batched strided 2-D copy kernel for gfx950 (pack / unpack / self-periodic /
// one-phase messages). One launch covers every face (and edge/corner message)
// of every field: the reference launches one (1,32,1)/(32,1,1)-thread kernel per
// field and side (src/update_halo.jl:497-501), i.e. 32-lane groups that waste
// half of every 64-lane CDNA wavefront. Here: 256-thread workgroups (4 full
// waves); a workgroup copies one CHUNK of one row (the inner, fastest-varying
// extent of the region), so the per-element index math is a single multiply-add
// and the block->(copy, row, chunk) decode is scalar (once per workgroup).
// Rows with unit stride on both sides move 4 elements per lane in flight.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "igg/copy.hpp"
#include "igg/devsync.hpp"
#include "igg/sysstore.hpp"

namespace igg {

extern bool g_copy_gather;

namespace {

constexpr int BLOCK = 256;
constexpr int EPT = 4;                         // elements per thread per chunk
constexpr int64_t CHUNK = BLOCK * EPT;         // elements of a row per workgroup
// Strided rows (gather path): a wave covers 64 consecutive inner elements of
// GROWS outer rows, so each lane keeps GROWS independent line loads in flight;
// a workgroup is 4 such waves (4 * GROWS outer rows).
constexpr int GROWS = 8;

// 16-B elements (complex128): a vector type, which stays in VGPRs; a struct
// element of the GROWS-deep load array was kept in scratch (144 B per lane,
// tools/kernel_resources.py).
typedef uint64_t B16 __attribute__((ext_vector_type(2)));

// Byte shift of the arena half selected by the device-resident epoch (odd ->
// second half). The epoch lives in the uncached flag words, written by the
// put transport's sync kernel earlier on the same stream.
__device__ __forceinline__ int64_t parity_shift(const CopyBatch& b) {
  if (b.parity_side == 0) return 0;
  const uint64_t e = __hip_atomic_load(b.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return ((e + b.parity_add) & 1) ? b.parity_bytes : 0;
}

// Element store: plain, or (SYS, put transport) a system-scope store
// (st_sys, igg/sysstore.hpp).
template <typename T, bool SYS>
__device__ __forceinline__ void store(T* p, const T& v) {
  if constexpr (SYS) st_sys(p, v);
  else *p = v;
}

template <typename T, bool FENCE>
__global__ void __launch_bounds__(BLOCK) copy2d_batch_kernel(const CopyBatch batch) {
  const int64_t b = blockIdx.x;
  if (batch.wait.n > 0) {
    // (CopyWait) the senders' data of the step this GPU has just completed
    // (EPOCH) must have arrived: their ARRIVED flags publish it
    if (threadIdx.x == 0) {
      const uint64_t e = load_sys_relaxed(batch.wait.flags + PutFlags::EPOCH);
      for (int k = 0; k < batch.wait.n; ++k)
        spin_geq(batch.wait.flags + PutFlags::ARRIVED + batch.wait.rank[k], e, batch.wait.flags,
                 batch.wait.timeout_ticks, 0x400 + k);
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  int c = 0;
  // Wave-uniform scan over <= MAX_BATCH prefix sums (scalar loads from kernarg).
  while (c + 1 < batch.n && b >= batch.block_start[c + 1]) ++c;
  const Copy2D& cp = batch.c[c];
  const int64_t local = b - batch.block_start[c];
  const int64_t shift = parity_shift(batch);
  const char* sbase = cp.src + (batch.parity_side == 2 ? shift : 0);
  char* dbase = cp.dst + (batch.parity_side == 1 ? shift : 0);
  if ((batch.flat_mask >> c) & 1u) {
    // Short rows (n_inner < 64: narrow faces, edges, corners): one element per
    // lane over the flattened region.
    const int64_t e = local * BLOCK + threadIdx.x;
    if (e < cp.n_outer * cp.n_inner) {
      const int64_t o = e / cp.n_inner, i = e - o * cp.n_inner;
      store<T, FENCE>(reinterpret_cast<T*>(dbase) + o * cp.dst_so + i * cp.dst_si,
                      reinterpret_cast<const T*>(sbase)[o * cp.src_so + i * cp.src_si]);
    }
  } else if ((batch.gather_mask >> c) & 1u) {
    // A face of a C-ordered field across its fastest dim (z): every element
    // of the row sits in its own cache line on the strided side, so the copy
    // is bound by how many line requests are in flight, not by bytes. The
    // row-chunk path put one 512-element row in a 1024-element workgroup
    // (half the lanes idle, 2 loads per lane, one workgroup per row: 2 x 514
    // workgroups for a 512^3 z face pair - 19.7 us, profiles/r4_trace/); here
    // the block decode is scalar and every lane issues GROWS loads before its
    // first store.
    const int64_t nic = (cp.n_inner + 63) / 64;
    const int64_t og = local / nic, ic = local - og * nic;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t i = ic * 64 + lane;
    const int64_t o0 = (og * 4 + w) * GROWS;
    if (i < cp.n_inner && o0 < cp.n_outer) {
      const T* __restrict__ src = reinterpret_cast<const T*>(sbase) + i * cp.src_si;
      T* __restrict__ dst = reinterpret_cast<T*>(dbase) + i * cp.dst_si;
      const int nr = static_cast<int>(min<int64_t>(GROWS, cp.n_outer - o0));
      T v[GROWS];
#pragma unroll
      for (int k = 0; k < GROWS; ++k)
        if (k < nr) v[k] = src[(o0 + k) * cp.src_so];
#pragma unroll
      for (int k = 0; k < GROWS; ++k)
        if (k < nr) store<T, FENCE>(dst + (o0 + k) * cp.dst_so, v[k]);
    }
  } else {
    const int64_t nchunks = (cp.n_inner + CHUNK - 1) / CHUNK;
    const int64_t o = local / nchunks;              // row (outer index)
    const int64_t i0 = (local - o * nchunks) * CHUNK;
    const T* __restrict__ src = reinterpret_cast<const T*>(sbase) + o * cp.src_so;
    T* __restrict__ dst = reinterpret_cast<T*>(dbase) + o * cp.dst_so;
    const int64_t n = cp.n_inner;
    T v[EPT];
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      const int64_t i = i0 + k * BLOCK + threadIdx.x;
      if (i < n) v[k] = src[i * cp.src_si];
    }
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      const int64_t i = i0 + k * BLOCK + threadIdx.x;
      if (i < n) store<T, FENCE>(dst + i * cp.dst_si, v[k]);
    }
  }
  // Put transport (FENCE): every store above was a system-scope store into a
  // peer's fine-grained arena (written through this XCD's L2, where the peer
  // mapping could keep a plain store dirty); the wave waits for their
  // acknowledgements before it retires, then the sync kernel that runs next
  // on this stream publishes the ARRIVED flag and the receiver reads the
  // arena only after observing it (docs/COHERENCE.md).
  if (FENCE) __builtin_amdgcn_s_waitcnt(0);
}

template <typename T, bool FENCE>
void launch_typed(const std::vector<Copy2D>& copies, hipStream_t stream, const ParityShift& par,
                  const CopyWait& wait) {
  size_t pos = 0;
  while (pos < copies.size()) {
    CopyBatch batch{};
    batch.n = 0;
    batch.epoch = par.epoch;
    batch.parity_bytes = par.bytes;
    batch.parity_side = par.side;
    batch.parity_add = par.add;
    batch.wait = wait;
    int64_t blocks = 0;
    while (pos < copies.size() && batch.n < MAX_BATCH) {
      const Copy2D& c = copies[pos++];
      const int64_t total = c.n_outer * c.n_inner;
      if (total <= 0) continue;
      const bool is_flat = c.n_inner < 64;
      const bool is_gather = !is_flat && (c.src_si != 1 || c.dst_si != 1) && g_copy_gather;
      batch.c[batch.n] = c;
      batch.block_start[batch.n] = blocks;
      if (is_flat) batch.flat_mask |= 1u << batch.n;
      if (is_gather) batch.gather_mask |= 1u << batch.n;
      blocks += is_flat     ? (total + BLOCK - 1) / BLOCK
                : is_gather ? ((c.n_inner + 63) / 64) * ((c.n_outer + 4 * GROWS - 1) / (4 * GROWS))
                            : c.n_outer * ((c.n_inner + CHUNK - 1) / CHUNK);
      ++batch.n;
    }
    if (batch.n == 0) continue;
    batch.block_start[batch.n] = blocks;
    if (blocks > 0x7fffffffLL) fail("launch_copy2d: too many blocks (", blocks, ")");
    hipLaunchKernelGGL((copy2d_batch_kernel<T, FENCE>), dim3(static_cast<unsigned>(blocks)), dim3(BLOCK), 0,
                       stream, batch);
    IGG_HIP_CHECK(hipGetLastError());
  }
}

}  // namespace

// Gather path for strided long rows (IGG_COPY_GATHER=0: the row-chunk path,
// for A/B measurements: benchmarks/pack_faces.py).
bool g_copy_gather = [] {
  const char* e = std::getenv("IGG_COPY_GATHER");
  return !(e && e[0] == '0');
}();

template <bool FENCE>
void launch_sized(const std::vector<Copy2D>& copies, int elem_bytes, hipStream_t stream,
                  const ParityShift& par, const CopyWait& wait) {
  switch (elem_bytes) {
    case 1: launch_typed<uint8_t, FENCE>(copies, stream, par, wait); break;
    case 2: launch_typed<uint16_t, FENCE>(copies, stream, par, wait); break;
    case 4: launch_typed<uint32_t, FENCE>(copies, stream, par, wait); break;
    case 8: launch_typed<uint64_t, FENCE>(copies, stream, par, wait); break;
    case 16: launch_typed<B16, FENCE>(copies, stream, par, wait); break;
    default: fail("launch_copy2d: unsupported element size ", elem_bytes, " bytes");
  }
}

void launch_copy2d(const std::vector<Copy2D>& copies, int elem_bytes, hipStream_t stream,
                   bool system_fence, const ParityShift& parity, const CopyWait& wait) {
  if (copies.empty()) return;
  if (wait.n < 0 || wait.n > 2 || (wait.n > 0 && !wait.flags)) fail("launch_copy2d: invalid CopyWait");
  if (system_fence) launch_sized<true>(copies, elem_bytes, stream, parity, wait);
  else launch_sized<false>(copies, elem_bytes, stream, parity, wait);
}

}  // namespace igg
