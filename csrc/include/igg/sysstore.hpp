#pragma once
// System-scope stores for data that another GPU reads (device code; the
// writer side of docs/COHERENCE.md).
//
// `sc0 sc1` on a store is the gfx942/gfx950 encoding of a relaxed
// system-scope atomic store: it writes through this XCD's L2 (where a peer
// mapping, MTYPE NC, could keep a plain store dirty) and its vmcnt
// acknowledgement means the bytes reached the owner's memory. The caller ends
// every storing wave with s_waitcnt vmcnt(0) before the flag that publishes
// the data is set (next kernel on the stream).
//
// INVARIANT for the in-kernel step synchronisation (send mode bit 16,
// devsync.hpp step_sync_exit): the last exchanging wave publishes ARRIVED
// with relaxed system-scope stores and NO release fence. That is correct only
// because EVERY store a fused kernel makes into a peer's memory goes through
// st_sys / st_sys_at (write-through, acknowledged before the wave counts
// itself). A plain store into peer memory anywhere in a fused kernel would
// break that form (docs/COHERENCE.md, "No release fence in K4").
//
// The stores are relaxed system-scope atomic stores of 1, 2, 4 or 8 bytes (a
// wider value is split), which the compiler emits as `global_store_{byte,
// short,dword,dwordx2} ... sc0 sc1` and schedules like any other memory instruction. (Rounds 2-3 used
// inline-asm `global_store_dwordx4 ... sc0 sc1` for 16-B vectors: the
// compiler's hazard recognizer does not see inside inline asm, and with the
// fused kernels at the 256-VGPR limit (spilling to AGPRs) a wrong interior
// value appeared in one fused form after an unrelated code change,
// deterministic per binary; profiles/r3_sysstore/.)
#include <hip/hip_runtime.h>

#include <cstdint>

namespace igg {

template <typename V>
__device__ __forceinline__ void st_sys(V* p, const V& v) {
  static_assert(sizeof(V) == 1 || sizeof(V) == 2 || (sizeof(V) % 4 == 0 && sizeof(V) <= 32),
                "st_sys: 1, 2 or 4..32 bytes (a multiple of 4)");
  if constexpr (sizeof(V) == 1) {
    __hip_atomic_store(reinterpret_cast<uint8_t*>(p), __builtin_bit_cast(uint8_t, v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  } else if constexpr (sizeof(V) == 2) {
    __hip_atomic_store(reinterpret_cast<uint16_t*>(p), __builtin_bit_cast(uint16_t, v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  } else if constexpr (sizeof(V) % 8 == 0) {
    struct W { uint64_t w[sizeof(V) / 8]; };
    const W x = __builtin_bit_cast(W, v);
    uint64_t* q = reinterpret_cast<uint64_t*>(p);
#pragma unroll
    for (int i = 0; i < static_cast<int>(sizeof(V) / 8); ++i)
      __hip_atomic_store(q + i, x.w[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  } else {
    struct W { uint32_t w[sizeof(V) / 4]; };
    const W x = __builtin_bit_cast(W, v);
    uint32_t* q = reinterpret_cast<uint32_t*>(p);
#pragma unroll
    for (int i = 0; i < static_cast<int>(sizeof(V) / 4); ++i)
      __hip_atomic_store(q + i, x.w[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// A 16- or 32-B vector at `base` + `off` bytes as `buffer_store_dwordx4 ...
// sc0 sc1` (one or two): the same write-through system-scope store as st_sys,
// without splitting the vector into 8-B atomic stores (a `sc0 sc1` store is
// one fabric write each: dwordx2 costs 2.7x a dwordx4 per byte,
// MI355X_MICROARCH.md). A compiler builtin, so its hazards are tracked like
// any other store (unlike rounds 2-3's inline asm). `base` must be
// wave-uniform (it becomes the buffer descriptor in SGPRs) and `off` < 2 GiB.
template <typename V>
__device__ __forceinline__ void st_sys_at(const void* base, uint32_t off, const V& v) {
  if constexpr (sizeof(V) == 16 || sizeof(V) == 32) {
    typedef unsigned int U4 __attribute__((ext_vector_type(4)));
    struct W { U4 q[sizeof(V) / 16]; };
    const W x = __builtin_bit_cast(W, v);
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), static_cast<short>(0), 0x7fffffff, 0x00020000);
    constexpr int SC0_SC1 = 1 | 16;  // cache policy bits of the gfx94x/gfx950 encoding
#pragma unroll
    for (int i = 0; i < static_cast<int>(sizeof(V) / 16); ++i)
      __builtin_amdgcn_raw_buffer_store_b128(x.q[i], r, static_cast<int>(off) + 16 * i, 0, SC0_SC1);
  } else {
    st_sys(reinterpret_cast<V*>(static_cast<char*>(const_cast<void*>(base)) + off), v);
  }
}

}  // namespace igg
