// Shared constants, error type and small helpers of the native IGG runtime.
//
// Behavioural parity notes (reference = ImplicitGlobalGrid.jl v0.13):
//   * NDIMS / NNEIGHBORS / ALLOC_GRANULARITY mirror src/shared.jl:29-32.
//   * PROC_NULL marks a missing neighbour (non-periodic edge), like MPI.PROC_NULL
//     as used by Cart_shift in src/init_global_grid.jl:89-92.
#pragma once

#include <cstdint>
#include <cstddef>
#include <stdexcept>
#include <string>
#include <sstream>

namespace igg {

constexpr int NDIMS = 3;                 // shared.jl:29 (NDIMS_MPI)
constexpr int NNEIGHBORS = 2;            // shared.jl:30 (left = 0, right = 1)
constexpr int64_t ALLOC_GRANULARITY = 32;  // shared.jl:31, in elements
constexpr int64_t THREADCOPY_THRESHOLD = 32768;  // shared.jl:32, bytes
constexpr int PROC_NULL = -1;
constexpr size_t DEVICE_ALIGN = 256;     // device buffer alignment in bytes

// Error type for every user-visible failure; surfaced to Python as igg.IGGError.
class Error : public std::runtime_error {
 public:
  explicit Error(const std::string& msg) : std::runtime_error(msg) {}
};

template <typename... Args>
[[noreturn]] inline void fail(Args&&... args) {
  std::ostringstream os;
  (os << ... << args);
  throw Error(os.str());
}

inline int64_t round_up(int64_t v, int64_t g) { return ((v + g - 1) / g) * g; }

}  // namespace igg

// HIP error check used by every runtime call of the native library.
#define IGG_HIP_CHECK(expr)                                                    \
  do {                                                                         \
    hipError_t _e = (expr);                                                    \
    if (_e != hipSuccess) {                                                    \
      (void)hipGetLastError(); /* clear the sticky copy of this error */       \
      ::igg::fail("HIP error '", hipGetErrorString(_e), "' at ", __FILE__, ":", \
                  __LINE__, " in ", #expr);                                    \
    }                                                                          \
  } while (0)
