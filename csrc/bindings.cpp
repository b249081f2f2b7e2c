// pybind11 bindings of the native IGG runtime (_igg_native).
//
// The Python layer passes raw pointers, extents and strides of torch tensors
// (CPU or HIP) plus the current HIP stream handle; nothing here links libtorch,
// so the runtime is a self-contained C++/HIP library with a thin binding.
#include <pybind11/functional.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <chrono>
#include <mutex>
#include <thread>
#include <utility>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "igg/acoustic.hpp"
#include "igg/coherence.hpp"
#include "igg/comm.hpp"
#include "igg/copy.hpp"
#include "igg/fault.hpp"
#include "igg/fused.hpp"
#include "igg/gather.hpp"
#include "igg/halo.hpp"
#include "igg/ipc.hpp"
#include "igg/stencil.hpp"
#include "igg/topology.hpp"
#include "igg/trace.hpp"
#include "igg/vmm.hpp"

namespace igg {
void launch_zcol_probe(int dir, const void* src, void* dst, int64_t rows, int64_t pitch, int aux,
                       hipStream_t stream);
void launch_stream_probe(int kind, double* out, const double* a, const double* b, int64_t n, int blocks,
                         hipStream_t stream);
}

namespace py = pybind11;
using namespace igg;

namespace {

// DLPack (v0.8 ABI, the layout torch.utils.dlpack consumes): a native device
// allocation of a given memory kind handed to torch as a 1-D uint8 tensor
// whose deleter frees it. Lets a model keep its fields in fine-grained memory
// (docs/COHERENCE.md) without linking libtorch.
struct DLDevice { int32_t device_type; int32_t device_id; };
struct DLDataType { uint8_t code; uint8_t bits; uint16_t lanes; };
struct DLTensor {
  void* data;
  DLDevice device;
  int32_t ndim;
  DLDataType dtype;
  int64_t* shape;
  int64_t* strides;
  uint64_t byte_offset;
};
struct DLManagedTensor {
  DLTensor dl_tensor;
  void* manager_ctx;
  void (*deleter)(DLManagedTensor*);
};
constexpr int32_t kDLROCM = 10;

struct DlpackAlloc {
  int64_t shape[1];
  int device;
};

// Freeing a field whose tensor was garbage-collected: kernels queued on any
// stream may still use it, and a device synchronisation right here would
// invalidate a hipGraph capture in progress on this thread. So the
// release is DEFERRED: the buffer joins a list that is drained (one device
// synchronisation, then hipFree) at the next native allocation, at
// finalize_global_grid / model close, or at exit - never inside a capture.
std::mutex g_deferred_mu;
std::vector<std::pair<void*, int>> g_deferred;  // (pointer, device)

void flush_deferred_frees() {
  std::vector<std::pair<void*, int>> v;
  {
    std::lock_guard<std::mutex> lk(g_deferred_mu);
    v.swap(g_deferred);
  }
  if (v.empty()) return;
  int cur = 0;
  (void)hipGetDevice(&cur);
  int synced = -1;
  for (const auto& [p, dev] : v) {
    if (dev != synced) {
      (void)hipSetDevice(dev);
      (void)hipDeviceSynchronize();  // no kernel may still use the buffers
      synced = dev;
    }
    if (vmm_find(p, nullptr, nullptr)) vmm_free(p);  // a MemKind::Vmm field
    else (void)hipFree(p);
  }
  (void)hipSetDevice(cur);
}

void dlpack_free(DLManagedTensor* t) {
  if (!t) return;
  auto* ctx = static_cast<DlpackAlloc*>(t->manager_ctx);
  {
    std::lock_guard<std::mutex> lk(g_deferred_mu);
    g_deferred.emplace_back(t->dl_tensor.data, ctx->device);
  }
  delete ctx;
  delete t;
}

py::capsule alloc_dlpack(size_t bytes, int kind) {
  if (bytes == 0) fail("alloc_dlpack: zero bytes");
  flush_deferred_frees();  // allocation time is a safe point (no capture in progress)
  int dev = 0;
  IGG_HIP_CHECK(hipGetDevice(&dev));
  void* p = ipc_malloc(bytes, static_cast<MemKind>(kind));
  auto* ctx = new DlpackAlloc{{static_cast<int64_t>(bytes)}, dev};
  auto* t = new DLManagedTensor{};
  t->dl_tensor.data = p;
  t->dl_tensor.device = {kDLROCM, dev};
  t->dl_tensor.ndim = 1;
  t->dl_tensor.dtype = {1 /* kDLUInt */, 8, 1};
  t->dl_tensor.shape = ctx->shape;
  t->dl_tensor.strides = nullptr;
  t->dl_tensor.byte_offset = 0;
  t->manager_ctx = ctx;
  t->deleter = dlpack_free;
  // Unconsumed capsules free their tensor; torch renames a consumed one to
  // "used_dltensor" and owns the deleter from then on.
  return py::capsule(t, "dltensor", [](PyObject* cap) {
    if (PyCapsule_IsValid(cap, "dltensor")) dlpack_free(static_cast<DLManagedTensor*>(PyCapsule_GetPointer(cap, "dltensor")));
  });
}

hipStream_t as_stream(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

using FieldTuple = std::tuple<uintptr_t, int, std::array<int64_t, 3>, std::array<int64_t, 3>, int, bool>;

Field to_field(const FieldTuple& t) {
  Field f;
  f.ptr = std::get<0>(t);
  f.ndims = std::get<1>(t);
  f.size = std::get<2>(t);
  f.stride = std::get<3>(t);
  f.elem_bytes = std::get<4>(t);
  f.device = std::get<5>(t);
  return f;
}

std::vector<Field> to_fields(const std::vector<FieldTuple>& ts) {
  std::vector<Field> fs;
  fs.reserve(ts.size());
  for (const auto& t : ts) fs.push_back(to_field(t));
  return fs;
}

GridInfo make_grid(int64_t me, int64_t nprocs, const Int3& nxyz, const Int3& overlaps,
                   const std::array<Int3, 2>& neighbors, const std::vector<int64_t>& peers) {
  GridInfo g;
  g.me = me;
  g.nprocs = nprocs;
  g.nxyz = nxyz;
  g.overlaps = overlaps;
  g.neighbors = neighbors;
  if (!peers.empty()) {
    if (peers.size() != 27) fail("GridInfo: peers must have 27 entries (dir_key order)");
    for (int k = 0; k < 27; ++k) g.peers[k] = peers[k];
    g.has_peers = true;
  }
  return g;
}

// Transport implemented in Python (torch.distributed gloo/nccl point-to-point).
class PyTransport : public Transport {
 public:
  PyTransport(py::function fn, bool host, bool dev, std::string name)
      : fn_(std::move(fn)), host_(host), dev_(dev), name_(std::move(name)) {}
  bool device_capable() const override { return dev_; }
  bool host_capable() const override { return host_; }
  std::string name() const override { return name_; }
  void exchange(const std::vector<P2POp>& recvs, const std::vector<P2POp>& sends, bool device,
                hipStream_t stream) override {
    auto conv = [](const std::vector<P2POp>& ops) {
      py::list l;
      for (const auto& o : ops)
        l.append(py::make_tuple(reinterpret_cast<uintptr_t>(o.ptr), o.bytes, o.peer, o.tag));
      return l;
    };
    fn_(conv(recvs), conv(sends), device, reinterpret_cast<uintptr_t>(stream));
  }

 private:
  py::function fn_;
  bool host_, dev_;
  std::string name_;
};

// Pre-converted field list: the update_halo hot path converts tuples once per
// plan, not per call.
struct FieldSet {
  std::vector<Field> f;
};

std::vector<Box> to_boxes(const std::vector<std::pair<Int3, Int3>>& bs) {
  std::vector<Box> out;
  for (const auto& b : bs) {
    Box x;
    for (int d = 0; d < 3; ++d) { x.lo[d] = b.first[d]; x.hi[d] = b.second[d]; }
    out.push_back(x);
  }
  return out;
}

std::pair<Int3, Int3> from_box(const Box& b) {
  return {{b.lo[0], b.lo[1], b.lo[2]}, {b.hi[0], b.hi[1], b.hi[2]}};
}

}  // namespace

PYBIND11_MODULE(_igg_native, m) {
  m.doc() = "Native MI355X runtime of the implicit global grid (HIP kernels + RCCL).";
  py::register_exception<Error>(m, "IGGError", PyExc_RuntimeError);

  m.attr("PROC_NULL") = PROC_NULL;
  m.attr("NDIMS") = NDIMS;
  m.attr("NNEIGHBORS") = NNEIGHBORS;
  m.attr("ALLOC_GRANULARITY") = ALLOC_GRANULARITY;
  m.attr("THREADCOPY_THRESHOLD") = THREADCOPY_THRESHOLD;

  // --- topology
  m.def("dims_create", &dims_create, py::arg("nprocs"), py::arg("dims"));
  m.def("cart_coords", &cart_coords, py::arg("rank"), py::arg("dims"));
  m.def("cart_rank", &cart_rank, py::arg("coords"), py::arg("dims"));
  m.def("cart_shift", &cart_shift, py::arg("rank"), py::arg("dim"), py::arg("disp"),
        py::arg("dims"), py::arg("periods"));
  m.def("global_size", &global_size);
  m.def("coord_g", &coord_g);

  // --- device
  m.def("device_count", []() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
  });
  m.def("set_device", [](int d) { IGG_HIP_CHECK(hipSetDevice(d)); });
  m.def("get_device", []() {
    int d = 0;
    IGG_HIP_CHECK(hipGetDevice(&d));
    return d;
  });
  m.def("device_synchronize", []() {
    py::gil_scoped_release nogil;
    IGG_HIP_CHECK(hipDeviceSynchronize());
  });
  // Bounded, low-latency wait for everything enqueued on stream `s` so far:
  // an event recorded there is polled (GIL released) until it completes or
  // `timeout` seconds pass (returns false; the caller aborts communicators).
  // Unlike a helper thread around hipDeviceSynchronize it returns within
  // microseconds of completion, so a timed region pays no wake-up latency.
  m.def("stream_wait_bounded", [](uintptr_t s, double timeout) {
    thread_local hipEvent_t ev = nullptr;
    if (!ev) IGG_HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    IGG_HIP_CHECK(hipEventRecord(ev, as_stream(s)));
    py::gil_scoped_release nogil;
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      const hipError_t e = hipEventQuery(ev);
      if (e == hipSuccess) return true;
      if (e != hipErrorNotReady) IGG_HIP_CHECK(e);
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout) return false;
      std::this_thread::yield();
    }
  }, py::arg("stream"), py::arg("timeout"));
  m.def("stream_synchronize", [](uintptr_t s) {
    py::gil_scoped_release nogil;
    IGG_HIP_CHECK(hipStreamSynchronize(as_stream(s)));
  });
  m.def("memcpy_d2h", [](uintptr_t src, size_t n) {
    std::string out(n, '\0');
    IGG_HIP_CHECK(hipMemcpy(out.data(), reinterpret_cast<void*>(src), n, hipMemcpyDeviceToHost));
    return py::bytes(out);
  });
  m.def("clear_last_error", []() {
    const hipError_t e = hipGetLastError();  // reads and resets the thread's sticky error
    return e == hipSuccess ? std::string() : std::string(hipGetErrorString(e));
  }, "Reset the HIP runtime's last-error state (after a failed capture); returns the error it held.");
  m.def("rccl_version", &rccl_version);
  m.def("abandoned_waits", &abandoned_waits,
        "Bounded first-contact calls this process gave up on (their helper threads are still stuck in the "
        "runtime): a process with any should be replaced, not reused (fault.hpp).");
  m.def("first_contact_timeout", &first_contact_timeout);
  m.def("install_crash_handler", &install_crash_handler,
        "Print a native backtrace on SIGSEGV/SIGBUS/SIGABRT, then chain to the previous handler "
        "(faulthandler's Python stack).");
  m.def("trace_enabled", &trace_enabled);
  m.def("trace_push", [](const std::string& n) { trace_push(n.c_str()); });
  m.def("trace_pop", &trace_pop);
  m.def("trace_mark", [](const std::string& n) { trace_mark(n.c_str()); });

  // --- intra-node peer memory (put transport primitives)
  m.def("ipc_malloc", [](size_t bytes, int kind) {
    return reinterpret_cast<uintptr_t>(ipc_malloc(bytes, static_cast<MemKind>(kind)));
  });
  m.def("ipc_free", [](uintptr_t p) { ipc_free(reinterpret_cast<void*>(p)); });
  m.def("flush_deferred_frees", &flush_deferred_frees,
        "Free the native field buffers whose tensors were released (one device synchronisation); "
        "called at finalize / model close. Never call it inside a hipGraph capture.");
  m.def("deferred_frees", []() {
    std::lock_guard<std::mutex> lk(g_deferred_mu);
    return g_deferred.size();
  });
  m.def("alloc_dlpack", &alloc_dlpack, py::arg("bytes"), py::arg("kind"),
        "Zeroed device allocation of a MemKind as a DLPack capsule (1-D uint8; torch.utils.dlpack.from_dlpack).");
  m.def("ipc_get_handle", [](uintptr_t p) { return py::bytes(ipc_get_handle(reinterpret_cast<void*>(p))); });
  m.def("alloc_bytes", [](uintptr_t p) { return alloc_bytes(reinterpret_cast<const void*>(p)); }, py::arg("ptr"),
        "Size of the device allocation holding `ptr` (hipMemGetAddressRange).");
  m.attr("IPC_MAX_BYTES") = py::int_(IPC_MAX_BYTES);
  m.def("ipc_open", [](const std::string& h) { return reinterpret_cast<uintptr_t>(ipc_open(h)); });
  m.def("ipc_close", [](uintptr_t p) { ipc_close(reinterpret_cast<void*>(p)); });
  m.def("stream_write_u64", [](uintptr_t s, uintptr_t p, uint64_t v) {
    stream_write_u64(as_stream(s), reinterpret_cast<void*>(p), v);
  });
  m.def("stream_wait_u64_geq", [](uintptr_t s, uintptr_t p, uint64_t v) {
    stream_wait_u64_geq(as_stream(s), reinterpret_cast<void*>(p), v);
  });
  m.def("can_stream_wait_value", &can_stream_wait_value);
  m.def("gpu_spin", [](double seconds, uintptr_t s) { launch_spin(seconds, as_stream(s)); },
        py::arg("seconds"), py::arg("stream"));
  m.def("read_u64", [](uintptr_t p) {
    uint64_t v = 0;
    IGG_HIP_CHECK(hipMemcpy(&v, reinterpret_cast<void*>(p), 8, hipMemcpyDeviceToHost));
    return v;
  });
  // Streams restricted to a subset of CUs (MI355X CU masking): the halo stream
  // can own a few CUs so communication kernels (RCCL's spin on each other and
  // need all their workgroups resident) never wait behind a compute kernel
  // that fills every CU. Returns the hipStream_t as an integer.
  m.def("stream_create_cu_mask", [](const std::vector<uint32_t>& mask, int priority) {
    hipStream_t s = nullptr;
    if (mask.empty()) {
      IGG_HIP_CHECK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority));
    } else {
      IGG_HIP_CHECK(hipExtStreamCreateWithCUMask(&s, static_cast<uint32_t>(mask.size()), mask.data()));
    }
    return reinterpret_cast<uintptr_t>(s);
  }, py::arg("mask"), py::arg("priority") = 0);
  m.def("stream_destroy", [](uintptr_t s) { IGG_HIP_CHECK(hipStreamDestroy(as_stream(s))); });
  m.def("stream_get_cu_mask", [](uintptr_t s, int words) {
    std::vector<uint32_t> m(static_cast<size_t>(words), 0u);
    IGG_HIP_CHECK(hipExtStreamGetCUMask(as_stream(s), static_cast<uint32_t>(words), m.data()));
    return m;
  });
  m.def("cu_count", []() {
    int dev = 0, cus = 0;
    IGG_HIP_CHECK(hipGetDevice(&dev));
    IGG_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    return cus;
  });
  // Stream-ordered blocking copies for the host-staged transport: wait for all
  // prior work on `stream`, copy, wait again.
  m.def("memcpy_d2h_stream", [](uintptr_t dst, uintptr_t src, size_t n, uintptr_t s) {
    py::gil_scoped_release nogil;
    IGG_HIP_CHECK(hipStreamSynchronize(as_stream(s)));
    IGG_HIP_CHECK(hipMemcpyAsync(reinterpret_cast<void*>(dst), reinterpret_cast<const void*>(src), n,
                                 hipMemcpyDeviceToHost, as_stream(s)));
    IGG_HIP_CHECK(hipStreamSynchronize(as_stream(s)));
  });
  m.def("memcpy_h2d_stream", [](uintptr_t dst, uintptr_t src, size_t n, uintptr_t s) {
    py::gil_scoped_release nogil;
    IGG_HIP_CHECK(hipStreamSynchronize(as_stream(s)));
    IGG_HIP_CHECK(hipMemcpyAsync(reinterpret_cast<void*>(dst), reinterpret_cast<const void*>(src), n,
                                 hipMemcpyHostToDevice, as_stream(s)));
    IGG_HIP_CHECK(hipStreamSynchronize(as_stream(s)));
  });

  // --- field geometry helpers (test hooks)
  m.def("ol", [](const GridInfo& g, int dim, const FieldTuple& f) { return ol(g, dim, to_field(f)); });
  m.def("max_halo_elems", [](const FieldTuple& f) { return max_halo_elems(to_field(f)); });
  m.def("send_index", [](const GridInfo& g, int side, int dim, const FieldTuple& f) {
    return send_index(g, side, dim, to_field(f));
  });
  m.def("recv_index", [](const GridInfo& g, int side, int dim, const FieldTuple& f) {
    return recv_index(g, side, dim, to_field(f));
  });
  m.def("face_info", [](const FieldTuple& f, int dim, int64_t index) {
    const Face fc = face(to_field(f), dim, index);
    return py::make_tuple(reinterpret_cast<uintptr_t>(fc.base), fc.n_outer, fc.n_inner, fc.s_outer,
                          fc.s_inner, fc.contiguous, fc.bytes);
  });

  py::class_<GridInfo>(m, "GridInfo")
      .def(py::init(&make_grid), py::arg("me"), py::arg("nprocs"), py::arg("nxyz"),
           py::arg("overlaps"), py::arg("neighbors"), py::arg("peers") = std::vector<int64_t>{})
      .def_readonly("peers", &GridInfo::peers)
      .def_readonly("has_peers", &GridInfo::has_peers)
      .def_readwrite("me", &GridInfo::me)
      .def_readwrite("nprocs", &GridInfo::nprocs)
      .def_readwrite("nxyz", &GridInfo::nxyz)
      .def_readwrite("overlaps", &GridInfo::overlaps)
      .def_readwrite("neighbors", &GridInfo::neighbors);

  // --- copies
  m.def("copy2d",
        [](const std::vector<std::tuple<uintptr_t, uintptr_t, int64_t, int64_t, int64_t, int64_t,
                                        int64_t, int64_t>>& cs,
           int elem_bytes, bool device, uintptr_t stream, bool system) {
          std::vector<Copy2D> v;
          for (const auto& c : cs)
            v.push_back({reinterpret_cast<const char*>(std::get<0>(c)),
                         reinterpret_cast<char*>(std::get<1>(c)), std::get<2>(c), std::get<3>(c),
                         std::get<4>(c), std::get<5>(c), std::get<6>(c), std::get<7>(c)});
          if (device) launch_copy2d(v, elem_bytes, as_stream(stream), system);
          else host_copy2d(v, elem_bytes);
        },
        py::arg("copies"), py::arg("elem_bytes"), py::arg("device"), py::arg("stream") = 0,
        py::arg("system") = false,
        "Batched strided 2-D copies; system: the put transport's system-scope (sc0 sc1) stores.");

  // --- transports
  py::class_<Transport, std::shared_ptr<Transport>>(m, "Transport")
      .def_property_readonly("name", &Transport::name)
      .def_property_readonly("device_capable", &Transport::device_capable)
      .def_property_readonly("host_capable", &Transport::host_capable);
  py::class_<PyTransport, Transport, std::shared_ptr<PyTransport>>(m, "PyTransport")
      .def(py::init<py::function, bool, bool, std::string>(), py::arg("fn"), py::arg("host"),
           py::arg("device"), py::arg("name"));
  py::class_<PeerMesh, std::shared_ptr<PeerMesh>>(m, "PeerMesh")
      .def(py::init([](int rank, int nranks, py::function allgather) {
             // Called from C++ (GIL held: exchanges run with the GIL).
             PeerMesh::AllGather ag = [allgather](const std::string& mine) {
               py::gil_scoped_acquire gil;
               py::list out = allgather(py::bytes(mine));
               std::vector<std::string> v;
               for (auto h : out) v.push_back(h.cast<std::string>());
               return v;
             };
             return std::make_shared<PeerMesh>(rank, nranks, ag);
           }),
           py::arg("rank"), py::arg("nranks"), py::arg("allgather"))
      .def_property_readonly("rank", &PeerMesh::rank)
      .def_property_readonly("nranks", &PeerMesh::nranks)
      .def_property_readonly("arena_bytes", &PeerMesh::arena_bytes)
      .def_property_readonly("epoch", [](const PeerMesh& m) { return m.read_flag(PutFlags::EPOCH); })
      .def_property_readonly("flag_words", &PeerMesh::flag_words)
      .def("flag", &PeerMesh::read_flag)
      .def("check_error", &PeerMesh::check_error)
      .def("clear_error", &PeerMesh::clear_error)
      .def("close", &PeerMesh::close);
  // --- HIP virtual memory management (allocations >= 2 GiB across processes)
  m.def("vmm_granularity", &vmm_granularity, py::arg("device"));
  m.def("vmm_alloc",
        [](size_t bytes) {
          size_t mapped = 0;
          void* p = vmm_alloc(bytes, &mapped);
          return py::make_tuple(reinterpret_cast<uintptr_t>(p), mapped);
        },
        py::arg("bytes"), "(pointer, mapped bytes) of new hipMemCreate memory on the current device");
  m.def("vmm_export_fd", [](uintptr_t p) { return vmm_export_fd(reinterpret_cast<void*>(p)); }, py::arg("ptr"));
  m.def("vmm_import_fd",
        [](int fd, size_t size, double seconds) {
          py::gil_scoped_release nogil;
          return reinterpret_cast<uintptr_t>(vmm_import_fd(fd, size, seconds));
        },
        py::arg("fd"), py::arg("size"), py::arg("seconds"));
  m.def("vmm_free", [](uintptr_t p) { vmm_free(reinterpret_cast<void*>(p)); }, py::arg("ptr"));
  m.def(
      "range_export_fd",
      [](uintptr_t p) {
        void* base = nullptr;
        size_t size = 0;
        const int fd = range_export_fd(reinterpret_cast<void*>(p), &base, &size);
        return py::make_tuple(fd, reinterpret_cast<uintptr_t>(base), size);
      },
      py::arg("ptr"), "(fd, base, size): dma-buf descriptor of the hipMalloc allocation holding ptr");
  m.def("fd_listen", &fd_listen, py::arg("name"));
  m.def("fd_serve",
        [](int listener, int fd, int clients, double seconds) {
          py::gil_scoped_release nogil;
          fd_serve(listener, fd, clients, seconds);
        },
        py::arg("listener"), py::arg("fd"), py::arg("clients"), py::arg("seconds"));
  m.def("fd_fetch",
        [](const std::string& name, double seconds) {
          py::gil_scoped_release nogil;
          return fd_fetch(name, seconds);
        },
        py::arg("name"), py::arg("seconds"));
  m.def("fd_close", &fd_close, py::arg("fd"));
  py::class_<CoherenceProbe, std::shared_ptr<CoherenceProbe>>(m, "CoherenceProbe")
      .def(py::init<std::shared_ptr<PeerMesh>, size_t>(), py::arg("mesh"), py::arg("bytes"),
           "Collective over a 2-rank mesh (reader 0, writer 1): arenas of `bytes` (igg/coherence.hpp).")
      .def("warm", [](CoherenceProbe& p, uintptr_t s) { p.warm(as_stream(s)); }, py::arg("stream"))
      .def("write",
           [](CoherenceProbe& p, uint64_t v, bool in_kernel, uintptr_t s, bool plain) {
             p.write(v, in_kernel, as_stream(s), plain);
           },
           py::arg("value"), py::arg("in_kernel"), py::arg("stream"), py::arg("plain") = false)
      .def("check",
           [](CoherenceProbe& p, uint64_t v, bool in_kernel, uintptr_t s) {
             py::gil_scoped_release nogil;
             return p.check(v, in_kernel, as_stream(s));
           },
           py::arg("value"), py::arg("in_kernel"), py::arg("stream"))
      .def("control",
           [](CoherenceProbe& p, uint64_t v, uint64_t target, bool l2, uintptr_t s) {
             p.control(v, target, l2, as_stream(s));
           },
           py::arg("value"), py::arg("target"), py::arg("l2"), py::arg("stream"))
      .def("mismatches",
           [](CoherenceProbe& p, uintptr_t s) {
             py::gil_scoped_release nogil;
             return p.mismatches(as_stream(s));
           },
           py::arg("stream"))
      .def_property_readonly("workgroups", &CoherenceProbe::workgroups)
      .def_property_readonly("words", &CoherenceProbe::words);
  py::class_<PutTransport, Transport, std::shared_ptr<PutTransport>>(m, "PutTransport")
      .def(py::init<std::shared_ptr<PeerMesh>>(), py::arg("mesh"))
      .def_property_readonly("mesh", &PutTransport::mesh_ptr);
  py::class_<RcclComm, Transport, std::shared_ptr<RcclComm>>(m, "RcclComm")
      .def_static("unique_id", []() {
        auto v = RcclComm::unique_id();
        return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
      })
      .def(py::init([](py::bytes uid, int nranks, int rank, double timeout) {
             std::string s = uid;
             std::vector<uint8_t> v(s.begin(), s.end());
             py::gil_scoped_release nogil;  // bounded rendezvous (polled)
             return std::make_shared<RcclComm>(v, nranks, rank, timeout);
           }),
           py::arg("uid"), py::arg("nranks"), py::arg("rank"), py::arg("timeout") = 0.0,
           "Bounded RCCL bootstrap (non-blocking communicator polled for `timeout` s; <= 0: "
           "IGG_FIRST_CONTACT_TIMEOUT, default 120); aborts and raises on expiry.")
      .def("barrier", [](RcclComm& c, uintptr_t s) { c.barrier(as_stream(s)); })
      .def("allreduce",
           [](RcclComm& c, uintptr_t send, uintptr_t recv, size_t count, int dtype, int op, uintptr_t s) {
             c.allreduce(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), count, dtype, op,
                         as_stream(s));
           },
           py::arg("send"), py::arg("recv"), py::arg("count"), py::arg("dtype"), py::arg("op"), py::arg("stream"))
      .def("broadcast",
           [](RcclComm& c, uintptr_t send, uintptr_t recv, size_t count, int dtype, int root, uintptr_t s) {
             c.broadcast(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), count, dtype, root,
                         as_stream(s));
           },
           py::arg("send"), py::arg("recv"), py::arg("count"), py::arg("dtype"), py::arg("root"), py::arg("stream"))
      .def("check_async_error", &RcclComm::check_async_error)
      .def("abort", &RcclComm::abort)
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("nranks", &RcclComm::nranks)
      .def("p2p",
           [](RcclComm& c, const std::vector<std::tuple<uintptr_t, size_t, int>>& recvs,
              const std::vector<std::tuple<uintptr_t, size_t, int>>& sends, uintptr_t s) {
             std::vector<P2POp> r, sd;
             for (const auto& x : recvs)
               r.push_back({reinterpret_cast<void*>(std::get<0>(x)), std::get<1>(x), std::get<2>(x), 0});
             for (const auto& x : sends)
               sd.push_back({reinterpret_cast<void*>(std::get<0>(x)), std::get<1>(x), std::get<2>(x), 0});
             c.exchange(r, sd, true, as_stream(s));
           });

  // --- halo engine
  py::class_<FieldSet>(m, "FieldSet")
      .def(py::init([](const std::vector<FieldTuple>& ts) { return FieldSet{to_fields(ts)}; }))
      .def("__len__", [](const FieldSet& s) { return s.f.size(); });
  py::class_<HaloEngine>(m, "HaloEngine")
      .def(py::init<const GridInfo&>())
      .def_property_readonly("grid", [](HaloEngine& e) { return e.grid(); })
      .def("set_grid", [](HaloEngine& e, const GridInfo& g) { e.grid() = g; })
      .def("set_transport", &HaloEngine::set_transport, py::arg("transport"), py::arg("device"))
      .def("clear_transport", [](HaloEngine& e, bool device) { e.set_transport(nullptr, device); })
      .def("transport_name", [](HaloEngine& e, bool device) {
        auto t = e.transport(device);
        return t ? t->name() : std::string("none");
      })
      .def("exchange",
           [](HaloEngine& e, const std::vector<FieldTuple>& fs, uintptr_t s) {
             e.exchange(to_fields(fs), as_stream(s));
           })
      .def("set_mode", [](HaloEngine& e, int m) { e.set_mode(static_cast<HaloMode>(m)); })
      .def_property_readonly("mode", [](HaloEngine& e) { return static_cast<int>(e.mode()); })
      .def("set_pack_mode",
           [](HaloEngine& e, int dim, int m) {
             if (dim < 0 || dim >= NDIMS || m < 0 || m > 1) throw std::invalid_argument("set_pack_mode: bad dim/mode");
             e.set_pack_mode(dim, static_cast<PackMode>(m));
           })
      .def("pack_mode", [](HaloEngine& e, int dim) { return static_cast<int>(e.pack_mode(dim)); })
      .def("resolved_mode", [](HaloEngine& e, const FieldSet& fs) {
        return static_cast<int>(e.resolved_mode(fs.f));
      })
      .def_property_readonly("last_message_count", &HaloEngine::last_message_count)
      .def("exchange_set",
           [](HaloEngine& e, const FieldSet& fs, uintptr_t s, int mode) { e.exchange(fs.f, as_stream(s), mode); },
           py::arg("fields"), py::arg("stream"), py::arg("mode") = -1)
      .def("exchange_dim",
           [](HaloEngine& e, const std::vector<FieldTuple>& fs, int dim, uintptr_t s) {
             e.exchange_dim(to_fields(fs), dim, as_stream(s));
           })
      .def("pool_ensure",
           [](HaloEngine& e, const std::vector<FieldTuple>& fs, bool device) {
             e.pool().ensure(to_fields(fs), device);
           })
      .def("pool_free", [](HaloEngine& e) { e.pool().free_all(); })
      .def("pool_allocated", [](HaloEngine& e, bool device) { return e.pool().allocated(device); })
      .def("pool_nslots", [](HaloEngine& e, bool device) { return e.pool().nslots(device); })
      .def("pool_capacity",
           [](HaloEngine& e, size_t slot, bool device) { return e.pool().capacity(slot, device); })
      .def("pool_ptrs", [](HaloEngine& e, size_t slot, bool device) {
        auto& p = e.pool();
        return py::make_tuple(reinterpret_cast<uintptr_t>(p.send(slot, 0, device)),
                              reinterpret_cast<uintptr_t>(p.send(slot, 1, device)),
                              reinterpret_cast<uintptr_t>(p.recv(slot, 0, device)),
                              reinterpret_cast<uintptr_t>(p.recv(slot, 1, device)));
      });

  // --- gather
  py::class_<Gatherer>(m, "Gatherer")
      .def(py::init<>())
      .def("gather",
           [](Gatherer& g, const FieldTuple& a, uintptr_t dst, int root, const Int3& dims,
              RcclComm& comm, uintptr_t s) {
             g.gather(to_field(a), reinterpret_cast<void*>(dst), root, dims, comm, as_stream(s));
           })
      .def("free", &Gatherer::free)
      .def_property_readonly("capacity", &Gatherer::capacity);
  py::class_<PullGatherer>(m, "PullGatherer")
      .def(py::init([](int rank, int nranks, py::function allgather) {
             PullGatherer::AllGather ag = [allgather](const std::string& mine) {
               py::gil_scoped_acquire gil;
               py::list out = allgather(py::bytes(mine));
               std::vector<std::string> v;
               for (auto h : out) v.push_back(h.cast<std::string>());
               return v;
             };
             return std::make_unique<PullGatherer>(rank, nranks, ag);
           }),
           py::arg("rank"), py::arg("nranks"), py::arg("allgather"))
      .def("start", [](PullGatherer& g, const FieldTuple& a, uintptr_t dst, int root, const Int3& dims,
                       uintptr_t s, bool snapshot) {
             g.start(to_field(a), reinterpret_cast<void*>(dst), root, dims, as_stream(s), snapshot);
           },
           py::arg("a"), py::arg("dst"), py::arg("root"), py::arg("dims"), py::arg("stream"),
           py::arg("snapshot") = false)
      .def("wait", [](PullGatherer& g, uintptr_t s) { g.wait(as_stream(s)); }, py::arg("stream"))
      .def_property_readonly("pending", &PullGatherer::pending)
      .def_property_readonly("last_kind", [](const PullGatherer& g) { return std::string(g.last_kind()); })
      .def("free", &PullGatherer::free);
  m.def("gather_reorder", [](uintptr_t src, uintptr_t dst, const Int3& s, const Int3& dims,
                             int eb, uintptr_t stream) {
    launch_gather_reorder(reinterpret_cast<const void*>(src), reinterpret_cast<void*>(dst), s, dims,
                          eb, as_stream(stream));
  });

  // --- stencils
  m.def("diffusion3d_variants", []() {
    std::vector<std::string> v;
    for (int i = 0; i < diffusion3d_num_variants(); ++i) v.push_back(diffusion3d_variant_name(i));
    return v;
  });
  m.def("diffusion3d_variant_tile", &diffusion3d_variant_tile);
  m.def("zcol_probe",
        [](int dir, uintptr_t src, uintptr_t dst, int64_t rows, int64_t pitch, int aux, uintptr_t stream) {
          launch_zcol_probe(dir, reinterpret_cast<const void*>(src), reinterpret_cast<void*>(dst), rows, pitch, aux,
                            as_stream(stream));
        },
        py::arg("dir"), py::arg("src"), py::arg("dst"), py::arg("rows"), py::arg("pitch"), py::arg("aux"),
        py::arg("stream") = 0,
        "z-face column probe: dir 0 pack (strided reads), 1 unpack (strided writes), 8-B elements; aux = cache "
        "policy bits of the strided access (1 sc0, 2 nt, 16 sc1).");
  m.def("stream_probe", [](int kind, uintptr_t out, uintptr_t a, uintptr_t b, int64_t n, int blocks,
                           uintptr_t stream) {
    launch_stream_probe(kind, reinterpret_cast<double*>(out), reinterpret_cast<const double*>(a),
                        reinterpret_cast<const double*>(b), n, blocks, as_stream(stream));
  });
  m.def("acoustic2d",
        [](uintptr_t p2, uintptr_t vx2, uintptr_t vy2, uintptr_t p, uintptr_t vx, uintptr_t vy, int64_t nx,
           int64_t ny, double dtk, double dt_rho, double rdx, double rdy, int elem_bytes, bool device,
           uintptr_t stream) {
          TraceRange tr("igg.acoustic2d");
          AcousticArgs a{p2, vx2, vy2, p, vx, vy, nx, ny, dtk, dt_rho, rdx, rdy, elem_bytes};
          if (device) {
            launch_acoustic2d(a, as_stream(stream));
          } else {
            py::gil_scoped_release nogil;
            host_acoustic2d(a);
          }
        },
        py::arg("p2"), py::arg("vx2"), py::arg("vy2"), py::arg("p"), py::arg("vx"), py::arg("vy"), py::arg("nx"),
        py::arg("ny"), py::arg("dtk"), py::arg("dt_rho"), py::arg("rdx"), py::arg("rdy"), py::arg("elem_bytes"),
        py::arg("device"), py::arg("stream") = 0);
  py::class_<FusedAcoustic, std::shared_ptr<FusedAcoustic>>(m, "FusedAcoustic")
      .def(py::init([](std::shared_ptr<PeerMesh> mesh, int64_t nx, int64_t ny, int elem_bytes,
                       const std::array<std::array<int, 2>, 2>& nb) {
             return std::make_shared<FusedAcoustic>(mesh, nx, ny, elem_bytes, nb);
           }),
           py::arg("mesh"), py::arg("nx"), py::arg("ny"), py::arg("elem_bytes"), py::arg("neighbors"))
      .def("set_fields", &FusedAcoustic::set_fields, py::arg("vx_a"), py::arg("vx_b"), py::arg("vy_a"),
           py::arg("vy_b"))
      .def("step",
           [](FusedAcoustic& f, uintptr_t p2, uintptr_t vx2, uintptr_t vy2, uintptr_t p, uintptr_t vx, uintptr_t vy,
              int64_t nx, int64_t ny, double dtk, double dt_rho, double rdx, double rdy, int elem_bytes,
              uintptr_t stream, bool entry) {
             TraceRange tr("igg.acoustic2d_fused");
             AcousticArgs a{p2, vx2, vy2, p, vx, vy, nx, ny, dtk, dt_rho, rdx, rdy, elem_bytes};
             f.step(a, as_stream(stream), entry);
           },
           py::arg("p2"), py::arg("vx2"), py::arg("vy2"), py::arg("p"), py::arg("vx"), py::arg("vy"), py::arg("nx"),
           py::arg("ny"), py::arg("dtk"), py::arg("dt_rho"), py::arg("rdx"), py::arg("rdy"), py::arg("elem_bytes"),
           py::arg("stream"), py::arg("entry") = false)
      .def("drain", [](FusedAcoustic& f, uintptr_t s) { f.drain(as_stream(s)); }, py::arg("stream"),
           "Exit barrier after in-kernel synchronised steps (collective; no-op after a sync-kernel step).")
      .def("check_error", &FusedAcoustic::check_error)
      .def("clear_error", &FusedAcoustic::clear_error,
           "Reset this rank's sticky timeout word (after a failed exchange was handled).")
      .def("set_step_sync", &FusedAcoustic::set_step_sync, py::arg("mode"),
           "Step synchronisation: -1 default, 0 inside the fused kernel, 1 sync kernel (same on every rank).")
      .def_property_readonly("in_kernel_sync", &FusedAcoustic::in_kernel_sync)
      .def("flag", [](FusedAcoustic& f, int i) { return f.flag(i); }, py::arg("index"),
           "Word `index` of this rank's flag block (PutFlags: 0 EPOCH = completed steps, 2 COUNT).")
      .def("close", &FusedAcoustic::close);
  m.def("acoustic2d_set_variant", &acoustic2d_set_variant);
  m.def("acoustic2d_set_chunk", &acoustic2d_set_chunk);
  m.def("diffusion3d_set_rounds", &diffusion3d_set_rounds);
  m.def("diffusion3d_get_rounds", &diffusion3d_get_rounds);
  m.def("diffusion3d",
        [](uintptr_t t2, uintptr_t t, uintptr_t cp, const Int3& n, const std::array<double, 3>& rd2,
           double dtlam, int elem_bytes, const std::vector<std::pair<Int3, Int3>>& boxes,
           bool device, int variant, uintptr_t stream, int rounds, bool halo_z) {
          TraceRange tr("igg.diffusion3d");
          DiffusionArgs a{t2, t, cp, {n[0], n[1], n[2]}, {rd2[0], rd2[1], rd2[2]}, dtlam, elem_bytes, rounds, halo_z};
          const auto bx = to_boxes(boxes);
          if (device) {
            launch_diffusion3d(a, bx, variant, as_stream(stream));
          } else {
            py::gil_scoped_release nogil;
            host_diffusion3d(a, bx);
          }
        },
        py::arg("t2"), py::arg("t"), py::arg("cp"), py::arg("n"), py::arg("rd2"), py::arg("dtlam"),
        py::arg("elem_bytes"), py::arg("boxes"), py::arg("device"), py::arg("variant") = 0,
        py::arg("stream") = 0, py::arg("rounds") = 0, py::arg("halo_z") = false);
  // Inner-box sweep through one restrict-form tiling id (fused_kernels.hip
  // dispatch_plain); the measurement-only tilings (incl. the timing probes
  // 130-132 of profiles/r2_refetch/refetch_probe.py) exist only in a --probes build.
  m.def("diffusion3d_hx_tiling",
        [](uintptr_t t2, uintptr_t t, uintptr_t cp, const Int3& n, const std::array<double, 3>& rd2,
           double dtlam, int elem_bytes, int tiling, uintptr_t stream, int rounds, bool halo_z) {
          DiffusionArgs a{t2, t, cp, {n[0], n[1], n[2]}, {rd2[0], rd2[1], rd2[2]}, dtlam, elem_bytes, rounds, halo_z};
          launch_diffusion3d_inner_hx(a, tiling, as_stream(stream));
        },
        py::arg("t2"), py::arg("t"), py::arg("cp"), py::arg("n"), py::arg("rd2"), py::arg("dtlam"),
        py::arg("elem_bytes"), py::arg("tiling"), py::arg("stream") = 0, py::arg("rounds") = 0,
        py::arg("halo_z") = false);
  m.def("diffusion3d_fused_variant_ok", &diffusion3d_fused_variant_ok);
  m.def("diffusion3d_variant_compiled", &stencil_variant_compiled,
        "Whether stencil variant v is compiled in this build (measurement-only ones: build.py --probes).");
  m.def("probes_build", []() {
#ifdef IGG_PROBES
    return true;
#else
    return false;
#endif
  });
  m.def("fused_debug", [](uintptr_t stamps, int force_sel) {
    fused_debug(reinterpret_cast<int64_t*>(stamps), force_sel);
  }, py::arg("stamps"), py::arg("force_sel") = -1);
  py::class_<FusedHalo, std::shared_ptr<FusedHalo>>(m, "FusedHalo")
      .def(py::init([](std::shared_ptr<PeerMesh> mesh, const Int3& n, int elem_bytes,
                       const std::array<std::array<int, 2>, 3>& nb) {
             return std::make_shared<FusedHalo>(mesh, std::array<int64_t, 3>{n[0], n[1], n[2]}, elem_bytes, nb);
           }),
           py::arg("mesh"), py::arg("n"), py::arg("elem_bytes"), py::arg("neighbors"))
      .def("step",
           [](FusedHalo& f, uintptr_t t2, uintptr_t t, uintptr_t cp, const std::array<double, 3>& rd2,
              double dtlam, int variant, int64_t step, bool primed, uintptr_t stream, int rounds, int mode,
              bool entry, bool halo_z) {
             TraceRange tr("igg.diffusion3d_fused");
             DiffusionArgs a{t2, t, cp, {0, 0, 0}, {rd2[0], rd2[1], rd2[2]}, dtlam, 0, rounds, halo_z};
             f.step_shape(a);
             f.step(a, variant, mode, step, primed, as_stream(stream), entry);
           },
           py::arg("t2"), py::arg("t"), py::arg("cp"), py::arg("rd2"), py::arg("dtlam"), py::arg("variant"),
           py::arg("step"), py::arg("primed"), py::arg("stream"), py::arg("rounds") = 0, py::arg("mode") = 0,
           py::arg("entry") = false, py::arg("halo_z") = false)
      .def("sync", [](FusedHalo& f, uintptr_t s) { f.sync(as_stream(s)); })
      .def("drain", [](FusedHalo& f, uintptr_t s) { f.drain(as_stream(s)); }, py::arg("stream"),
           "Exit barrier after in-kernel synchronised steps (collective; no-op after a sync-kernel step).")
      .def("set_fields", &FusedHalo::set_fields, py::arg("a"), py::arg("b"))
      .def_property_readonly("has_fields", &FusedHalo::has_fields)
      .def("io", [](FusedHalo& f, int64_t step, bool primed, uintptr_t t2, bool direct_z) {
        const HaloIOArgs io = f.io(step, primed, t2, direct_z);
        py::list in, out;
        for (int d = 0; d < 3; ++d) {
          in.append(py::make_tuple(io.in[d][0], io.in[d][1]));
          out.append(py::make_tuple(io.out[d][0], io.out[d][1]));
        }
        return py::make_tuple(in, out, io.zpitch, io.zrow);
      }, py::arg("step"), py::arg("primed"), py::arg("t2") = 0, py::arg("direct_z") = false)
      .def("region_offset", &FusedHalo::region_offset)
      .def_property_readonly("half_elems", &FusedHalo::half_elems)
      .def_property_readonly("zpitch", &FusedHalo::zpitch)
      .def_property_readonly("n_peers", &FusedHalo::n_peers)
      .def("check_error", [](FusedHalo& f) { f.mesh().check_error(); })
      .def("clear_error", [](FusedHalo& f) { f.mesh().clear_error(); },
           "Reset this rank's sticky timeout word (after a failed exchange was handled).")
      .def("set_step_sync", &FusedHalo::set_step_sync, py::arg("mode"),
           "Step synchronisation: -1 default, 0 inside the fused kernel, 1 sync kernel (same on every rank).")
      .def_property_readonly("in_kernel_sync", [](const FusedHalo& f) { return f.in_kernel_sync(0); },
                             "Whether a step with the default send mode synchronises inside the kernel.")
      .def("in_kernel_sync_for", &FusedHalo::in_kernel_sync, py::arg("mode"),
           "Whether a step with send mode `mode` synchronises inside the kernel (bit 16 asks for it).")
      .def("flag", [](FusedHalo& f, int i) { return f.mesh().read_flag(i); }, py::arg("index"),
           "Word `index` of this rank's flag block (PutFlags: 0 EPOCH = completed steps, 2 COUNT).")
      .def("close", [](FusedHalo& f) { f.close(); });
  m.def("split_boundary", [](const Int3& n, const std::array<std::array<bool, 2>, 3>& active,
                             const Int3& w) {
    std::vector<Box> slabs;
    Box interior;
    int64_t nn[3] = {n[0], n[1], n[2]}, ww[3] = {w[0], w[1], w[2]};
    bool aa[3][2];
    for (int d = 0; d < 3; ++d) { aa[d][0] = active[d][0]; aa[d][1] = active[d][1]; }
    split_boundary(nn, aa, ww, slabs, interior);
    std::vector<std::pair<Int3, Int3>> out;
    for (const Box& b : slabs) out.push_back(from_box(b));
    return py::make_tuple(out, from_box(interior));
  });
}
