// Intra-node peer memory for the put transport: IPC export/import of device
// allocations and command-processor (CP) flag operations on HIP streams.
//
// A put transport moves halo data with ordinary stores from a pack kernel into
// a peer GPU's receive arena mapped into this process (xGMI), and signals with
// hipStreamWriteValue64 / hipStreamWaitValue64 packets that the CP executes —
// no compute unit spins on a flag, so the exchange can run next to a stencil
// kernel that occupies every CU (RCCL's p2p kernels cannot: they stall until
// the co-running kernel drains, see profiles/overlap/).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "igg/common.hpp"

namespace igg {

enum class MemKind : int {
  Default = 0,     // hipMalloc (coarse-grained)
  FineGrained = 1, // hipDeviceMallocFinegrained
  Signal = 2,      // hipMallocSignalMemory
  Uncached = 3,    // hipDeviceMallocUncached (coherent across devices, bypasses L2)
  Vmm = 4,         // hipMemCreate + map (vmm.hpp): exportable at any size (a file descriptor)
  Contiguous = 5,  // hipDeviceMallocContiguous (physically contiguous, coarse-grained; the runtime
                   // refuses it combined with fine-grained: 'invalid argument')
};

// Largest allocation this framework exports through IPC. On this image
// (ROCm 7.x, dmabuf IPC: HSA_ENABLE_IPC_MODE_LEGACY=0) hipIpcOpenMemHandle of
// an allocation above 2 GiB never returns (2047 MiB opens in 0.4 ms, 2049 MiB
// hangs: profiles/r3_ipc/ipc_open_probe.py, profiles/r3_ipc/). ipc_get_handle
// refuses larger allocations with an error instead, so a collective caller
// fails on every rank (or falls back) rather than hanging in the open.
constexpr size_t IPC_MAX_BYTES = size_t{1} << 31;
size_t alloc_bytes(const void* p);             // size of the allocation holding p (hipMemGetAddressRange)

void* ipc_malloc(size_t bytes, MemKind kind);  // zero-filled, device-synchronised
void ipc_free(void* p);
std::string ipc_get_handle(void* p);           // opaque hipIpcMemHandle_t bytes
void* ipc_open(const std::string& handle);     // map a peer's allocation
void ipc_close(void* p);

void stream_write_u64(hipStream_t s, void* p, uint64_t v);
void stream_wait_u64_geq(hipStream_t s, void* p, uint64_t v);
bool can_stream_wait_value();

}  // namespace igg
