// Optional roctx instrumentation (rocprofv3 --marker-trace shows the ranges).
//
// Enabled with IGG_TRACE=1: librocprofiler-sdk-roctx is dlopen'ed on first use,
// so the runtime has no link dependency on it and tracing costs one branch
// when off. Ranges mark the host-side enqueue of each phase (pack, transport,
// unpack, stencil); GPU execution of the kernels comes from --kernel-trace.
#pragma once

namespace igg {

bool trace_enabled();
void trace_push(const char* name);
void trace_pop();
void trace_mark(const char* name);

struct TraceRange {
  explicit TraceRange(const char* name) : on_(trace_enabled()) {
    if (on_) trace_push(name);
  }
  ~TraceRange() {
    if (on_) trace_pop();
  }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;

 private:
  bool on_;
};

}  // namespace igg
