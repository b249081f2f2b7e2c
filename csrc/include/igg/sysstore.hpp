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
// HIP has no builtin for these cache-policy bits on a flat/global store, so
// the stores are inline asm, which the compiler's hazard recognizer does not
// see: a store of more than 64 bits reads its data VGPRs after issue, and a
// VALU write to those VGPRs right behind it (the "VMEM store data" hazard)
// would change the bytes in flight - observed on MI355X as the fourth dword of
// dwordx4 stores carrying the NEXT value (tools/acoustic_fused_debug.py,
// profiles/r3_acoustic/). The s_nop after every dwordx4 store covers the
// required wait states. No memory clobber: the destinations never alias
// anything the kernel reads (restrict arguments), so the compiler may keep
// scheduling loads across them; as untracked vector-memory operations they
// only make its vmcnt waits more conservative (in-order vmcnt on gfx9).
#include <hip/hip_runtime.h>

namespace igg {

template <typename V>
__device__ __forceinline__ void st_sys(V* p, const V& v) {
  static_assert(sizeof(V) == 1 || sizeof(V) == 2 || sizeof(V) == 4 || sizeof(V) == 8 || sizeof(V) == 16 ||
                    sizeof(V) == 32,
                "st_sys: 1, 2, 4, 8, 16 or 32 bytes");
  using U4 = unsigned __attribute__((ext_vector_type(4)));
  if constexpr (sizeof(V) == 32) {
    struct P2 { U4 lo, hi; };
    const P2 h = __builtin_bit_cast(P2, v);
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 4" ::"v"(p), "v"(h.lo));
    asm volatile("global_store_dwordx4 %0, %1, off offset:16 sc0 sc1\n\ts_nop 4" ::"v"(p), "v"(h.hi));
  } else if constexpr (sizeof(V) == 16) {
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 4" ::"v"(p), "v"(__builtin_bit_cast(U4, v)));
  } else if constexpr (sizeof(V) == 8) {
    asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1" ::"v"(p), "v"(__builtin_bit_cast(unsigned long long, v)));
  } else if constexpr (sizeof(V) == 4) {
    asm volatile("global_store_dword %0, %1, off sc0 sc1" ::"v"(p), "v"(__builtin_bit_cast(unsigned, v)));
  } else if constexpr (sizeof(V) == 2) {
    asm volatile("global_store_short %0, %1, off sc0 sc1" ::"v"(p),
                 "v"(static_cast<unsigned>(__builtin_bit_cast(unsigned short, v))));
  } else {
    asm volatile("global_store_byte %0, %1, off sc0 sc1" ::"v"(p),
                 "v"(static_cast<unsigned>(__builtin_bit_cast(unsigned char, v))));
  }
}

}  // namespace igg
