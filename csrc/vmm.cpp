// HIP virtual-memory-management export of large allocations.
//
// hipIpcGetMemHandle / hipIpcOpenMemHandle of an allocation of 2 GiB or more
// never returns on this runtime (ipc.hpp IPC_MAX_BYTES, profiles/r3_ipc/), so
// 4 GiB fields (1024^3 f32) cannot be mapped by a peer that way. The VMM route:
// the owner creates physical memory with hipMemCreate (requesting a POSIX file
// descriptor handle type), maps it into a reserved VA range of its own,
// exports the allocation as a file descriptor, and hands the descriptor to the
// importing process over a Unix-domain socket (SCM_RIGHTS: a file descriptor
// is a per-process object, the number alone means nothing elsewhere). The
// importer turns it back into an allocation handle, maps it into its own
// reserved VA range and grants its device read/write access.
//
// Every blocking step is bounded: socket waits poll with a timeout, and the
// runtime's import/map runs under run_bounded (fault.hpp) so a runtime call that
// never returns fails the caller instead of hanging it.
#include "igg/vmm.hpp"

#include <poll.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>

#include "igg/fault.hpp"

namespace igg {

namespace {

struct Mapping {
  size_t size = 0;
  hipMemGenericAllocationHandle_t handle{};
  bool owner = false;
};
std::mutex g_mu;
std::map<void*, Mapping> g_maps;

hipMemAllocationProp prop_for(int device) {
  hipMemAllocationProp p{};
  p.type = hipMemAllocationTypePinned;
  p.requestedHandleTypes = hipMemHandleTypePosixFileDescriptor;
  p.location.type = hipMemLocationTypeDevice;
  p.location.id = device;
  return p;
}

size_t round_up(size_t n, size_t g) { return (n + g - 1) / g * g; }

// Placement knobs, read per allocation (benchmarks/memkind_ab.py A/Bs them in
// one process): IGG_VMM_GRAN = "min" | "rec" (allocation granularity the size
// is rounded to), IGG_VMM_ALIGN_MIB = alignment of the reserved VA range
// (0 = the runtime's choice).
bool recommended_gran() {
  const char* e = std::getenv("IGG_VMM_GRAN");
  return !(e && std::strcmp(e, "min") == 0);
}

size_t va_alignment(size_t gran) {
  const char* e = std::getenv("IGG_VMM_ALIGN_MIB");
  const size_t mib = e ? std::strtoull(e, nullptr, 10) : 2;
  const size_t a = mib << 20;
  return a > gran ? a : (mib ? gran : 0);
}

void* map_handle(hipMemGenericAllocationHandle_t h, size_t size, int device, size_t align) {
  void* va = nullptr;
  IGG_HIP_CHECK(hipMemAddressReserve(&va, size, align, nullptr, 0));
  IGG_HIP_CHECK(hipMemMap(va, size, 0, h, 0));
  hipMemAccessDesc acc{};
  acc.location.type = hipMemLocationTypeDevice;
  acc.location.id = device;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  IGG_HIP_CHECK(hipMemSetAccess(va, size, &acc, 1));
  return va;
}

// Abstract-namespace socket address (no file system entry, gone with the process).
sockaddr_un abstract_addr(const std::string& name, socklen_t* len) {
  if (name.size() + 2 > sizeof(sockaddr_un::sun_path)) fail("vmm: socket name too long");
  sockaddr_un a{};
  a.sun_family = AF_UNIX;
  a.sun_path[0] = '\0';
  std::memcpy(a.sun_path + 1, name.data(), name.size());
  *len = static_cast<socklen_t>(offsetof(sockaddr_un, sun_path) + 1 + name.size());
  return a;
}

bool wait_fd(int fd, short events, double seconds) {
  pollfd p{fd, events, 0};
  const int ms = static_cast<int>(seconds * 1000.0);
  for (;;) {
    const int r = ::poll(&p, 1, ms);
    if (r > 0) return true;
    if (r == 0) return false;
    if (errno != EINTR) return false;
  }
}

}  // namespace

size_t vmm_granularity(int device) {
  hipMemAllocationProp p = prop_for(device);
  size_t g = 0;
  IGG_HIP_CHECK(hipMemGetAllocationGranularity(
      &g, &p, recommended_gran() ? hipMemAllocationGranularityRecommended : hipMemAllocationGranularityMinimum));
  return g ? g : (size_t{2} << 20);
}

void* vmm_alloc(size_t bytes, size_t* mapped) {
  int dev = 0;
  IGG_HIP_CHECK(hipGetDevice(&dev));
  const size_t gran = vmm_granularity(dev);
  const size_t size = round_up(bytes, gran);
  hipMemAllocationProp p = prop_for(dev);
  hipMemGenericAllocationHandle_t h{};
  IGG_HIP_CHECK(hipMemCreate(&h, size, &p, 0));
  void* va = map_handle(h, size, dev, va_alignment(gran));
  IGG_HIP_CHECK(hipMemset(va, 0, size));
  IGG_HIP_CHECK(hipDeviceSynchronize());
  {
    std::lock_guard<std::mutex> lk(g_mu);
    g_maps[va] = Mapping{size, h, true};
  }
  if (mapped) *mapped = size;
  return va;
}

int vmm_export_fd(void* ptr) {
  Mapping m;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_maps.find(ptr);
    if (it == g_maps.end() || !it->second.owner) fail("vmm_export_fd: not a vmm_alloc pointer");
    m = it->second;
  }
  int fd = -1;
  IGG_HIP_CHECK(hipMemExportToShareableHandle(&fd, m.handle, hipMemHandleTypePosixFileDescriptor, 0));
  if (fd < 0) fail("vmm_export_fd: the runtime returned no file descriptor");
  return fd;
}

void* vmm_import_fd(int fd, size_t size, double seconds) {
  int dev = 0;
  IGG_HIP_CHECK(hipGetDevice(&dev));
  auto out = std::make_shared<std::pair<void*, hipMemGenericAllocationHandle_t>>(nullptr, hipMemGenericAllocationHandle_t{});
  run_bounded(
      [out, fd, size, dev]() {
        inject_delay("vmm_import");
        hipMemGenericAllocationHandle_t h{};
        // osHandle: the ADDRESS of the descriptor, as for the export. (Passed
        // as the descriptor's value cast to a pointer, as CUDA takes it, the
        // runtime dereferenced it: SIGSEGV, round-6 GPU run r6h.)
        int fdv = fd;
        IGG_HIP_CHECK(hipMemImportFromShareableHandle(&h, &fdv, hipMemHandleTypePosixFileDescriptor));
        out->first = map_handle(h, size, dev, va_alignment(vmm_granularity(dev)));
        out->second = h;
      },
      seconds, "vmm_import_fd (hipMemImportFromShareableHandle + map)");
  {
    std::lock_guard<std::mutex> lk(g_mu);
    g_maps[out->first] = Mapping{size, out->second, false};
  }
  return out->first;
}

void vmm_free(void* ptr) {
  Mapping m;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_maps.find(ptr);
    if (it == g_maps.end()) return;
    m = it->second;
    g_maps.erase(it);
  }
  (void)hipDeviceSynchronize();
  (void)hipMemUnmap(ptr, m.size);
  (void)hipMemRelease(m.handle);
  // The VA range stays reserved (never hipMemAddressFree): a new allocation
  // mapped at a just-freed range read the OLD pages through the copy engine
  // (a gather right after re-allocating an array of the same size got the
  // previous array's values, GPU run r6j). Reserved-but-unmapped VA costs no
  // memory; the process's VA space is 47+ bits.
}

int range_export_fd(void* ptr, void** base, size_t* size) {
  hipDeviceptr_t b = nullptr;
  size_t n = 0;
  IGG_HIP_CHECK(hipMemGetAddressRange(&b, &n, ptr));
  int fd = -1;
  IGG_HIP_CHECK(hipMemGetHandleForAddressRange(&fd, b, n, hipMemRangeHandleTypeDmaBufFd, 0));
  if (fd < 0) fail("range_export_fd: the runtime returned no file descriptor");
  if (base) *base = b;
  if (size) *size = n;
  return fd;
}

bool vmm_find(const void* p, void** base, size_t* size, bool* owner) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_maps.upper_bound(const_cast<void*>(p));
  if (it == g_maps.begin()) return false;
  --it;
  const char* b = static_cast<const char*>(it->first);
  if (static_cast<const char*>(p) >= b + it->second.size) return false;
  if (base) *base = it->first;
  if (size) *size = it->second.size;
  if (owner) *owner = it->second.owner;
  return true;
}

int fd_listen(const std::string& name) {
  const int s = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (s < 0) fail("fd_listen: socket: ", std::strerror(errno));
  socklen_t len = 0;
  sockaddr_un a = abstract_addr(name, &len);
  if (::bind(s, reinterpret_cast<sockaddr*>(&a), len) != 0 || ::listen(s, 64) != 0) {
    const int e = errno;
    ::close(s);
    fail("fd_listen: bind/listen '", name, "': ", std::strerror(e));
  }
  return s;
}

void fd_serve(int listener, int fd, int clients, double seconds) {
  for (int c = 0; c < clients; ++c) {
    if (!wait_fd(listener, POLLIN, seconds)) fail("fd_serve: no importer connected within ", seconds, " s");
    const int conn = ::accept4(listener, nullptr, nullptr, SOCK_CLOEXEC);
    if (conn < 0) fail("fd_serve: accept: ", std::strerror(errno));
    char byte = 'F';
    iovec io{&byte, 1};
    alignas(cmsghdr) char ctl[CMSG_SPACE(sizeof(int))] = {};
    msghdr msg{};
    msg.msg_iov = &io;
    msg.msg_iovlen = 1;
    msg.msg_control = ctl;
    msg.msg_controllen = sizeof(ctl);
    cmsghdr* cm = CMSG_FIRSTHDR(&msg);
    cm->cmsg_level = SOL_SOCKET;
    cm->cmsg_type = SCM_RIGHTS;
    cm->cmsg_len = CMSG_LEN(sizeof(int));
    std::memcpy(CMSG_DATA(cm), &fd, sizeof(int));
    const ssize_t r = ::sendmsg(conn, &msg, MSG_NOSIGNAL);
    const int e = errno;
    ::close(conn);
    if (r != 1) fail("fd_serve: sendmsg: ", std::strerror(e));
  }
}

int fd_fetch(const std::string& name, double seconds) {
  const auto t0 = std::chrono::steady_clock::now();
  socklen_t len = 0;
  sockaddr_un a = abstract_addr(name, &len);
  int s = -1;
  for (;;) {  // the owner may not be listening yet: retry until the deadline
    s = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
    if (s < 0) fail("fd_fetch: socket: ", std::strerror(errno));
    if (::connect(s, reinterpret_cast<sockaddr*>(&a), len) == 0) break;
    ::close(s);
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > seconds)
      fail("fd_fetch: could not connect to '", name, "' within ", seconds, " s");
    ::usleep(2000);
  }
  if (!wait_fd(s, POLLIN, seconds)) {
    ::close(s);
    fail("fd_fetch: no descriptor from '", name, "' within ", seconds, " s");
  }
  char byte = 0;
  iovec io{&byte, 1};
  alignas(cmsghdr) char ctl[CMSG_SPACE(sizeof(int))] = {};
  msghdr msg{};
  msg.msg_iov = &io;
  msg.msg_iovlen = 1;
  msg.msg_control = ctl;
  msg.msg_controllen = sizeof(ctl);
  const ssize_t r = ::recvmsg(s, &msg, MSG_CMSG_CLOEXEC);
  const int e = errno;
  ::close(s);
  if (r != 1) fail("fd_fetch: recvmsg: ", r < 0 ? std::strerror(e) : "connection closed");
  cmsghdr* cm = CMSG_FIRSTHDR(&msg);
  if (!cm || cm->cmsg_type != SCM_RIGHTS) fail("fd_fetch: no descriptor in the message");
  int fd = -1;
  std::memcpy(&fd, CMSG_DATA(cm), sizeof(int));
  return fd;
}

void fd_close(int fd) {
  if (fd >= 0) ::close(fd);
}

}  // namespace igg
