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
  static constexpr int COUNT = 2;     // exchanging waves retired in the running step (in-kernel step sync)
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

// In-kernel step synchronisation of the fused exchanges (FusedHalo,
// FusedAcoustic), replacing the sync kernel after every step: only the
// exchanging waves of the step kernel take part (those whose tile reads a
// received halo or stores a sent one; every other wave touches no memory a
// neighbour reads or writes). Each of them first waits until every neighbour
// has completed the previous step (ARRIVED[nb] >= own EPOCH: its sends of the
// halos the wave reads have arrived, and its reads of the memory the wave
// overwrites in it are done), and the last one of them to retire (the COUNT
// word reaches `feat_waves`) publishes ARRIVED = EPOCH + 1 at the neighbours
// and advances EPOCH. docs/COHERENCE.md has the ordering argument.
// my_flags == nullptr: not used (a sync kernel follows the step kernel).
constexpr int STEP_SYNC_MAX_PEERS = 6;  // face neighbours of a 3-D rank
struct StepSync {
  uint64_t* my_flags = nullptr;
  uint64_t* peer_flags[STEP_SYNC_MAX_PEERS] = {};
  int peer_rank[STEP_SYNC_MAX_PEERS] = {};
  int n_peers = 0, my_rank = 0;
  int64_t timeout_ticks = 0;
  // counting units of the launch (set by the launcher): exchanging waves
  // (acoustic kernel), or workgroups holding one (diffusion: step_sync_exit_wg)
  int64_t feat_waves = 0;
  // Acquire after the wait (measurement knob IGG_STEP_SYNC_ACQUIRE): 2 system
  // (buffer_inv sc0 sc1, the default), 1 agent (buffer_inv sc1), 0 workgroup
  // (compiler ordering only; the kernel start invalidated the L1).
  int acquire = 2;
};
// The StepSync of a face-neighbour PutSync (every peer both sends and receives).
StepSync step_sync_from(const PutSync& s);
// Whether a fused exchange synchronises its steps inside the step kernel.
// IGG_FUSED_SYNC_KERNEL unset: `by_default` unless another rank of the mesh
// shares this rank's GPU (its waiting waves could starve that rank's kernel);
// "1": never (the sync kernel after every step); "0": always (tests whose
// kernels cannot fill the GPU). FusedHalo passes by_default = send mode bit 16
// (an A/B candidate of its own; the sync kernel is the default); the
// acoustic step false: its ~8,300 exchanging waves per 8192^2 step each count
// themselves with one atomic on the same uncached word, and those serialise
// (0.70-0.75 vs 0.306 ms/step with the sync kernel, profiles/r3_stepsync/).
bool step_sync_in_kernel(bool shares_device, bool by_default);

void launch_put_begin(const PutSync& s, hipStream_t stream);
void launch_put_sync(const PutSync& s, hipStream_t stream);
int64_t put_timeout_ticks(double seconds);
// One wave spinning `seconds` of wall-clock time on `stream` (failure-path tests).
void launch_spin(double seconds, hipStream_t stream);

}  // namespace igg
