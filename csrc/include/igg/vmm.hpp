// HIP virtual memory management export/import of large allocations (csrc/vmm.cpp).
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <string>

namespace igg {

// Allocation granularity of hipMemCreate on `device`.
size_t vmm_granularity(int device);
// Physical memory of >= `bytes` on the current device, mapped read/write at a
// reserved VA range (zero-filled); *mapped = the rounded size.
void* vmm_alloc(size_t bytes, size_t* mapped);
// A POSIX file descriptor of a vmm_alloc allocation (the caller closes it).
int vmm_export_fd(void* ptr);
// Map a peer's exported allocation (`size` = its mapped size) into this
// process for the current device; bounded by `seconds` (run_bounded).
void* vmm_import_fd(int fd, size_t size, double seconds);
// Unmap / release (owner or importer).
void vmm_free(void* ptr);
// A dma-buf file descriptor of the whole ordinary (hipMalloc) allocation that
// holds `ptr`, its base and size: importable with vmm_import_fd like a VMM
// export (round 6 probe: tests/test_vmm.py).
int range_export_fd(void* ptr, void** base, size_t* size);
// Whether `p` lies in a mapping made by vmm_alloc (owner) / vmm_import_fd; its
// base and mapped size.
bool vmm_find(const void* p, void** base, size_t* size, bool* owner = nullptr);
// File descriptor passing over an abstract-namespace Unix socket (SCM_RIGHTS).
int fd_listen(const std::string& name);
void fd_serve(int listener, int fd, int clients, double seconds);
int fd_fetch(const std::string& name, double seconds);
void fd_close(int fd);

}  // namespace igg
