// roctx ranges (loaded with dlopen, no link-time dependency). The reference has no
// tracing beyond tic/toc (tools.jl:205-236); see SURVEY.md §5.1.
#include "igg/trace.hpp"

#include <dlfcn.h>

#include <cstdlib>
#include <mutex>

namespace igg {
namespace {

struct Roctx {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
  void (*mark)(const char*) = nullptr;
  bool on = false;
};

Roctx& roctx() {
  static Roctx r;
  static std::once_flag once;
  std::call_once(once, [] {
    const char* e = std::getenv("IGG_TRACE");
    if (!e || !*e || *e == '0') return;
    const char* libs[] = {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4",
                          "libroctx64.so"};
    for (const char* name : libs) {
      void* h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
      if (!h) continue;
      r.push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
      r.pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
      r.mark = reinterpret_cast<void (*)(const char*)>(dlsym(h, "roctxMarkA"));
      if (r.push && r.pop) {
        r.on = true;
        return;
      }
    }
  });
  return r;
}

}  // namespace

bool trace_enabled() { return roctx().on; }
void trace_push(const char* name) {
  if (roctx().on) roctx().push(name);
}
void trace_pop() {
  if (roctx().on) roctx().pop();
}
void trace_mark(const char* name) {
  if (roctx().on && roctx().mark) roctx().mark(name);
}

}  // namespace igg
