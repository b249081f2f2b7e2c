// Failure detection helpers (include/igg/fault.hpp).
#include "igg/fault.hpp"

#include <csignal>
#include <cstdlib>
#include <cstring>
#include <string>

#include <execinfo.h>
#include <unistd.h>

namespace igg {

namespace {
std::atomic<int> g_abandoned{0};
}

int abandoned_waits() { return g_abandoned.load(); }
void note_abandoned_wait() { g_abandoned.fetch_add(1); }

double first_contact_timeout() {
  const char* e = std::getenv("IGG_FIRST_CONTACT_TIMEOUT");
  const double t = e ? std::atof(e) : 0.0;
  return t > 0 ? t : 120.0;
}

namespace {
// The entry of `spec` ("point@rank[:value],...") naming `point` for this rank
// (RANK from the launcher), or nullptr-equivalent false.
bool match_point(const char* env, const char* point, double* value) {
  const char* spec = std::getenv(env);
  if (!spec || !*spec) return false;
  const char* r = std::getenv("RANK");
  const std::string me = r ? r : "0";
  std::string s(spec);
  size_t pos = 0;
  while (pos <= s.size()) {
    const size_t end = std::min(s.find(',', pos), s.size());
    const std::string item = s.substr(pos, end - pos);
    pos = end + 1;
    const size_t at = item.find('@'), colon = item.find(':');
    if (at == std::string::npos || item.substr(0, at) != point) continue;
    const std::string rank = item.substr(at + 1, (colon == std::string::npos ? item.size() : colon) - at - 1);
    if (rank != me && rank != "*") continue;
    if (value) *value = colon == std::string::npos ? -1.0 : std::atof(item.c_str() + colon + 1);
    return true;
  }
  return false;
}
}  // namespace

void inject_delay(const char* point) {
  double secs = -1.0;
  if (!match_point("IGG_INJECT_HANG", point, &secs)) return;
  std::this_thread::sleep_for(std::chrono::duration<double>(secs < 0 ? 3600.0 : secs));
}

void inject_fail(const char* point) {
  if (match_point("IGG_INJECT_FAIL", point, nullptr)) fail("injected failure at '", point, "' (IGG_INJECT_FAIL)");
}

namespace {
struct sigaction g_prev_segv, g_prev_bus, g_prev_abrt;

void crash_handler(int sig, siginfo_t* info, void* ctx) {
  // Async-signal-safe enough for a crash report: write + backtrace_symbols_fd.
  static const char head[] = "\n[igg] fatal signal in native code; C backtrace:\n";
  (void)!write(2, head, sizeof(head) - 1);
  void* frames[64];
  const int n = backtrace(frames, 64);
  backtrace_symbols_fd(frames, n, 2);
  // Chain to the previous handler (Python's faulthandler: the Python stack),
  // which re-raises with the default action.
  const struct sigaction* prev = sig == SIGSEGV ? &g_prev_segv : (sig == SIGBUS ? &g_prev_bus : &g_prev_abrt);
  if (prev->sa_flags & SA_SIGINFO) {
    if (prev->sa_sigaction) prev->sa_sigaction(sig, info, ctx);
  } else if (prev->sa_handler != SIG_DFL && prev->sa_handler != SIG_IGN && prev->sa_handler) {
    prev->sa_handler(sig);
  }
  signal(sig, SIG_DFL);
  raise(sig);
}
}  // namespace

void install_crash_handler() {
  void* warm[1];
  (void)backtrace(warm, 1);  // load libgcc's unwinder now, not inside the handler
  struct sigaction sa {};
  sa.sa_sigaction = crash_handler;
  sa.sa_flags = SA_SIGINFO | SA_RESETHAND;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGSEGV, &sa, &g_prev_segv);
  sigaction(SIGBUS, &sa, &g_prev_bus);
  sigaction(SIGABRT, &sa, &g_prev_abrt);
}

}  // namespace igg
