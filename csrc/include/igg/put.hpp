// Device-side synchronisation of the put transport (see peer.hpp).
//
// Every exchange is four launches on the caller's stream, with no host
// involvement and no per-exchange kernel arguments (so it can live in a
// hipGraph): the exchange epoch is a counter in device memory.
//   begin  (1 workgroup): e = ++epoch; tell every neighbour "consumed e-1"
//          (my unpack of e-1 ran before me on this stream); wait until each
//          receiver of mine has consumed e-2 (the last use of arena half e&1).
//   put    (pack kernel, dst = peer arenas shifted by half (e&1)); every thread
//          ends with a system-scope release fence.
//   sync   (1 workgroup): publish arrived[me] = e at every receiver; wait until
//          arrived[sender] >= e for every sender.
//   unpack (copy kernel, src = own arena shifted by half (e&1)).
// Spins poll uncached flags with system-scope atomics and s_sleep, bounded by a
// wall-clock timeout: on expiry the kernel records an error code and exits, so
// a missing peer can never leave a wave running forever.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>

namespace igg {

constexpr int PUT_MAX_PEERS = 27;

// Flag block layout (uint64 words, uncached device memory, IPC-exported).
struct PutFlags {
  static constexpr int EPOCH = 0;     // local exchange counter
  static constexpr int ERROR = 1;     // 0 ok, else 1 + code of the first timeout
  static constexpr int ARRIVED = 8;   // [ARRIVED + r]: last epoch rank r's data arrived
  __host__ __device__ static inline int freed(int nranks) { return ARRIVED + nranks; }  // [freed + r]
  __host__ __device__ static inline int words(int nranks) { return ARRIVED + 2 * nranks; }
};

struct PutSync {
  uint64_t* my_flags;                     // own flag block
  uint64_t* out_flags[PUT_MAX_PEERS];     // flag blocks of my receivers
  uint64_t* nb_flags[PUT_MAX_PEERS];      // flag blocks of all my neighbours
  int out_rank[PUT_MAX_PEERS];            // ranks of my receivers
  int in_rank[PUT_MAX_PEERS];             // ranks of my senders
  int n_out, n_in, n_nb;
  int my_rank, nranks;
  int64_t timeout_ticks;                  // wall_clock64 ticks
};

void launch_put_begin(const PutSync& s, hipStream_t stream);
void launch_put_sync(const PutSync& s, hipStream_t stream);
int64_t put_timeout_ticks(double seconds);

}  // namespace igg
