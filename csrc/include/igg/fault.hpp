// Failure detection helpers of the native runtime.
//
// The reference has none: MPI aborts the job when a rank fails
// (src/init_global_grid.jl:80-92 initialises MPI; every later error is an
// MPI abort). Here every first-contact call of the multi-GPU path (RCCL
// bootstrap, IPC mapping of a peer's memory) is bounded:
//
//   * run_bounded(f, seconds, what) runs `f` on a helper thread bound to the
//     caller's HIP device and gives up after `seconds`: the helper is
//     abandoned (it may hold runtime locks forever), the process is marked
//     with abandoned_waits() > 0, and igg::Error is raised. Callers turn that
//     into a collective outcome (every rank raises together); a process with
//     an abandoned wait must not be trusted with more GPU work - the bench's
//     supervisor replaces it with a fresh process (utils/supervise.py).
//   * inject_delay(point) sleeps when IGG_INJECT_HANG names `point` for this
//     rank ("point@rank:seconds[,...]"; RANK from the launcher environment):
//     the fault-injection knob of the hang tests (rccl_init, ipc_open).
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <exception>
#include <memory>
#include <mutex>
#include <thread>

#include <hip/hip_runtime_api.h>

#include "igg/common.hpp"

namespace igg {

// Sleep if IGG_INJECT_HANG asks for a delay at `point` on this rank.
void inject_delay(const char* point);
// Raise igg::Error if IGG_INJECT_FAIL ("point@rank[,...]") names `point` for
// this rank (collective-failure tests).
void inject_fail(const char* point);
// Number of bounded waits this process abandoned (helper threads still stuck).
int abandoned_waits();
void note_abandoned_wait();
// SIGSEGV/SIGBUS/SIGABRT handler printing a native backtrace to stderr, then
// chaining to the previous handler (install after faulthandler.enable(): the
// C frames come first, then Python's stack). IGG_CRASH_BACKTRACE=1 installs it
// at import (parallel/grid.py).
void install_crash_handler();
// Seconds allowed for a first-contact call (IGG_FIRST_CONTACT_TIMEOUT, default 120).
double first_contact_timeout();

template <typename F>
void run_bounded(F&& f, double seconds, const char* what) {
  struct State {
    std::mutex m;
    std::condition_variable cv;
    bool done = false;
    std::exception_ptr err;
  };
  auto st = std::make_shared<State>();
  int dev = 0;
  IGG_HIP_CHECK(hipGetDevice(&dev));
  std::thread th([st, dev, fn = std::forward<F>(f)]() mutable {
    try {
      IGG_HIP_CHECK(hipSetDevice(dev));  // the HIP device is per thread
      fn();
    } catch (...) {
      st->err = std::current_exception();
    }
    std::lock_guard<std::mutex> lk(st->m);
    st->done = true;
    st->cv.notify_all();
  });
  std::unique_lock<std::mutex> lk(st->m);
  const bool ok = st->cv.wait_for(lk, std::chrono::duration<double>(seconds), [&] { return st->done; });
  lk.unlock();
  if (!ok) {
    th.detach();  // stuck inside the runtime: abandon it (st stays alive with it)
    note_abandoned_wait();
    fail(what, " did not complete within ", seconds, " s (IGG_FIRST_CONTACT_TIMEOUT); the call was abandoned "
         "and this process should be replaced");
  }
  th.join();
  if (st->err) std::rethrow_exception(st->err);
}

}  // namespace igg
