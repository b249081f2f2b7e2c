// Device-side synchronisation of the put transport (see peer.hpp).
//
// Every exchange is three (sometimes four) launches on the caller's stream,
// with no host involvement and no per-exchange kernel arguments (so it can
// live in a hipGraph): the device word EPOCH counts completed exchanges c, and
// the running exchange is e = c + 1.
//   [begin (1 wave): wait until each receiver has consumed e-2, the last use of
//          arena half e&1. Launched only when the host cannot prove it: halo
//          neighbourhoods are symmetric, so if every receiver of e also sent to
//          me in e-1, my sync of e-1 already waited for its arrival, which it
//          published only after unpacking e-2.]
//   put    (pack kernel, dst = peer arenas shifted by half (c+1)&1); every
//          thread waits for its stores to be acknowledged.
//   sync   (1 wave): release "consumed e-1" to every neighbour (my unpack of
//          e-1 ran before), publish arrived[me] = e at every receiver, wait for
//          arrived[sender] >= e of every sender, then EPOCH = e.
//   unpack (copy kernel, src = own arena shifted by half c&1 = e&1).
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
  static constexpr int EPOCH = 0;     // completed exchanges (the running one is EPOCH + 1)
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
// One wave spinning `seconds` of wall-clock time on `stream` (failure-path tests).
void launch_spin(double seconds, hipStream_t stream);

}  // namespace igg
