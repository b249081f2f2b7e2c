#include "igg/ipc.hpp"

#include <cstring>

#include "igg/fault.hpp"
#include "igg/vmm.hpp"

namespace igg {

void* ipc_malloc(size_t bytes, MemKind kind) {
  void* p = nullptr;
  switch (kind) {
    case MemKind::Default: IGG_HIP_CHECK(hipMalloc(&p, bytes)); break;
    case MemKind::FineGrained: IGG_HIP_CHECK(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocFinegrained)); break;
    case MemKind::Signal: IGG_HIP_CHECK(hipExtMallocWithFlags(&p, bytes, hipMallocSignalMemory)); break;
    case MemKind::Uncached: IGG_HIP_CHECK(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached)); break;
    case MemKind::Vmm: return vmm_alloc(bytes, nullptr);  // zero-filled, synchronised
    case MemKind::Contiguous: IGG_HIP_CHECK(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocContiguous)); break;
    default: fail("ipc_malloc: unknown memory kind ", static_cast<int>(kind));
  }
  IGG_HIP_CHECK(hipMemset(p, 0, bytes));
  IGG_HIP_CHECK(hipDeviceSynchronize());
  return p;
}

void ipc_free(void* p) {
  if (!p) return;
  if (vmm_find(p, nullptr, nullptr)) {
    vmm_free(p);
    return;
  }
  (void)hipDeviceSynchronize();
  IGG_HIP_CHECK(hipFree(p));
}

size_t alloc_bytes(const void* p) {
  void* base = nullptr;
  size_t size = 0;
  IGG_HIP_CHECK(hipMemGetAddressRange(&base, &size, const_cast<void*>(p)));
  return size;
}

std::string ipc_get_handle(void* p) {
  if (const size_t n = alloc_bytes(p); n >= IPC_MAX_BYTES)
    fail("IPC export of a ", n >> 20, " MiB allocation refused: opening IPC handles of allocations of 2 GiB or "
         "more hangs on this ROCm runtime (profiles/r3_ipc/)");
  hipIpcMemHandle_t h;
  IGG_HIP_CHECK(hipIpcGetMemHandle(&h, p));
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

void* ipc_open(const std::string& handle) {
  if (handle.size() != sizeof(hipIpcMemHandle_t))
    fail("ipc_open: handle has ", handle.size(), " bytes, expected ", sizeof(hipIpcMemHandle_t));
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle.data(), sizeof(h));
  // First contact with a peer's memory: bounded (fault.hpp). This runtime has
  // been seen to never return from an open (allocations of 2 GiB or more,
  // profiles/r3_ipc/); a stuck open must fail the mesh on every rank, not hang
  // the job.
  auto p = std::make_shared<void*>(nullptr);
  run_bounded(
      [p, h]() {
        inject_delay("ipc_open");
        void* q = nullptr;
        IGG_HIP_CHECK(hipIpcOpenMemHandle(&q, h, hipIpcMemLazyEnablePeerAccess));
        *p = q;
      },
      first_contact_timeout(), "hipIpcOpenMemHandle (mapping a peer's memory)");
  return *p;
}

void ipc_close(void* p) {
  if (p) IGG_HIP_CHECK(hipIpcCloseMemHandle(p));
}

void stream_write_u64(hipStream_t s, void* p, uint64_t v) {
  IGG_HIP_CHECK(hipStreamWriteValue64(s, p, v, 0));
}

void stream_wait_u64_geq(hipStream_t s, void* p, uint64_t v) {
  IGG_HIP_CHECK(hipStreamWaitValue64(s, p, v, hipStreamWaitValueGte, ~uint64_t(0)));
}

bool can_stream_wait_value() {
  int dev = 0, v = 0;
  IGG_HIP_CHECK(hipGetDevice(&dev));
  IGG_HIP_CHECK(hipDeviceGetAttribute(&v, hipDeviceAttributeCanUseStreamWaitValue, dev));
  return v != 0;
}

}  // namespace igg
