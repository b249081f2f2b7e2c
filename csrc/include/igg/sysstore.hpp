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

}  // namespace igg
