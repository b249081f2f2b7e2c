#!/usr/bin/env python3
"""Headline benchmark: 3-D heat diffusion, 512^3 Float64 per GPU, weak scaling.

Metric (BASELINE.json): effective memory throughput T_eff = A_eff / t_it with
A_eff = 3 * n_local * sizeof(T) (T read, Cp read, T2 written) per GPU, and the
weak-scaling efficiency E(N) = t_it(1)/t_it(N). The driver computes E(N) from its
own per-N runs; this script also measures it inside one job (``config.efficiency``:
the 1-GPU run's local problem timed on the same ranks, interleaved with the real
step in alternating order, so no box-to-box spread enters).

``value`` is the WHOLE-JOB aggregate T_eff (sum of the per-GPU T_eff over the
N GPUs), as the bench contract prescribes; at N=1 it equals the per-GPU number.
The per-GPU T_eff is ``config.t_eff_per_gpu_GBs`` (``value / n_gpus``), the
per-step time ``ms_per_step`` (= ``config.t_it_ms``). ``vs_baseline`` compares
the per-GPU T_eff with the reference's derived 23 GB/s per GPU (BASELINE.md:
8x P100, 256^3/GPU diffusion example), like for like.

Launch: one process per GPU. Under torchrun (``WORLD_SIZE`` set) every rank
runs this file. ``python bench.py --gpus N`` WITHOUT a launcher starts the N
ranks itself (``self_launch``: a parent that never touches the GPU spawns N
single-GPU children with the torch.distributed environment, prints rank 0's
JSON line, and fails if any rank fails or ``n_gpus != N``); a ``--gpus`` that
contradicts ``WORLD_SIZE`` is an error, never a silent 1-GPU number.
(Reference: nprocs comes from the communicator, src/init_global_grid.jl:84-93.)

Multi-GPU: before anything is timed, every device transport / schedule
(RCCL sequential, RCCL one-phase, one-sided put) is checked BITWISE against the
host-staged gloo exchange (the reference's non-GPU-aware MPI path) on a
rank-distinct payload with poisoned halo planes; failures are recorded in
``config.validation`` and excluded. The survivors are A/B-timed on the model
(hipGraph-replayed steps, MAX over ranks) and the fastest is kept; then the
fused exchange (the stencil kernel stores its send planes into the
neighbours' IPC-mapped arenas over xGMI; igg/fused.hpp) is checked bitwise
against the chosen update_halo_ schedule over 24 steps and A/B-timed too.
Every host wait on the GPU is bounded (IGG_COMM_TIMEOUT): a rank whose peer
died aborts RCCL and fails instead of hanging.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--n 512]
                       [--dtype float64] [--overlap] [--variant V|auto]
                       [--transport auto|rccl|put] [--no-graph] [--device gpu|cpu]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

# Fused-halo kernel candidates of the A/B: (tiling variant, send mode, grid
# residency rounds) - the front of benchmarks/fused_sweep.py --grid on MI355X.
# Modes 2/3 = 0/1 with the z-edge exchange compiled out when there is no z
# neighbour (2x1x1, 2x2x1): that form of tiling 11 (the fastest plain tiling,
# which pays for the z exchange at its register cliff) is tried as well
# (profiles/r1_noz/: loopback 2x2x1 rank 0.632 vs 0.651 ms/step).
# (Fused variant 40 - tiling 11 with lane-distributed z-segment edge loads at
# one workgroup per CU, no register spill - measured 0.65-0.75 ms in every
# loopback topology, slower than these: profiles/r1_zl/.)
# Round 2: the fused kernel runs each wave with only the exchange features its
# tile touches (profiles/r2_fused_spec/), so variant 40 (the fastest plain
# tiling) is exchange-free away from the exchanged faces and joins the A/B;
# tiling 11's z-compiled-out modes (superseded by that) left it. Variant 42 is
# 40 with the edge-lane z exchange (no per-row cross-lane ops): same as 40
# without z neighbours, z-edge waves 6-10 % faster than 40's with them. Its
# deferred-send mode is kept in the A/B for real xGMI links, where a remote
# store's acknowledgement is slower than in the loopback measurements.
FUSED_CANDIDATES = ((0, 0, 3), (0, 1, 3), (0, 0, 1), (0, 1, 1), (9, 0, 2), (9, 0, 3), (14, 0, 3),
                    (40, 0, 2), (42, 0, 2), (42, 1, 2), (50, 0, 2), (50, 1, 2), (50, 1, 3),
                    # round 6: tiling 9 with DPP z-edge lane moves (ties v9 at a loopback corner,
                    # profiles/r6_corner/NOTES.md; a real node's A/B decides)
                    (48, 0, 3), (48, 8, 2))
# Direct z (send mode bit 4: the z faces go straight into the neighbours' next
# T, no z receive code in the z-edge waves; igg/fused.hpp). Only with a z
# neighbour (without one these equal their mode & 3 forms).
FUSED_DIRECT = ((40, 4, 2), (42, 4, 2), (42, 5, 2), (50, 4, 2), (0, 4, 3))
# f32 (1024^3 config): tiling 14 with the edge-lane z exchange (fused variant
# 44) is the fastest fused form there (profiles/r2_f32_fused/).
FUSED_DIRECT_F32 = ((44, 4, 3), (44, 4, 4), (14, 4, 4), (44, 36, 4))
# z unpack (send mode bit 64, FusedHalo::Z_UNPACK): the z sends go into the
# neighbours' arenas as coalesced whole-line stores, the sweep has no z receive
# code, and a copy kernel writes the received z faces into the next T's halo
# column after the step synchronisation - the z exchange out of the sweep's
# receive path without direct z's scattered 8-B remote stores. With a z
# neighbour only (without one these equal their mode & ~64 forms).
FUSED_ZUNPACK = ((9, 64, 3), (42, 64, 2), (40, 64, 2), (0, 64, 3))
FUSED_ZUNPACK_F32 = ((44, 64, 4), (14, 64, 3))
# (send mode bit 32 = z-edge tiles dispatched first: the f32 2x2x2 corner's best
# form at 4 grid rounds; slower for f64 at every round count, profiles/r4_shapes/)
# Win record of the fused forms (rounds 2-4: the bench's A/Bs on every box and
# rehearsal, profiles/r4_shapes/ per rank shape; the in-kernel-sync forms, bit
# 16, are derived from the front later): tried first, so a spent A/B budget
# (IGG_BENCH_AB_BUDGET) drops forms that never won anywhere.
#   (9, 8, 2) / (9, 0, 2): the 2x2x2 corner's best forms on every round-5 box
#   (0.2-1.1 % ahead of their 3-round forms: profiles/r5_unpack/, r5_shapes/)
#   (9, 8, 3)  8-rank 2x2x2 rehearsal winner (r4), (9, 0, 3) 2x2x2 corner (r4 pass 4)
#   (42, 12, 2) interior + corner f64 (m28 = 12|16), (42, 9, 2) x+/xy+ (m25 = 9|16)
#   (14, 8, 3) f32 x/xy (m24 = 8|16), (44, 44, 4) / (44, 12, 4) f32 corner
#   (9, 72, 3) / (42, 72, 2): the round-5 z-unpack corner forms (no record yet;
#   right behind the record's front so a spent budget still times them)
#   (40, 8, 2) / (40, 0, 2): x+ / xy+ f64 since round 6 (plain waves on the
#   vector march, igg/vsweep.hpp: 1.012-1.017x, profiles/r6_vsweep/)
FUSED_WIN_ORDER = ((9, 8, 2), (9, 0, 2), (40, 8, 2), (40, 0, 2), (9, 8, 3), (42, 12, 2), (42, 9, 2), (9, 0, 3),
                   (9, 72, 3), (42, 72, 2),
                   (42, 8, 2), (14, 8, 3), (44, 44, 4), (44, 12, 4), (44, 72, 4), (42, 4, 2), (0, 12, 3), (42, 0, 2),
                   (40, 12, 2))


def _win_order(cands: list) -> list:
    """``cands`` with the forms of FUSED_WIN_ORDER first (in that order, if
    present), then the rest in their listed order."""
    first = [c for c in FUSED_WIN_ORDER if c in cands]
    return first + [c for c in cands if c not in first]


BASELINE_PER_GPU_GBS = 23.0  # BASELINE.md, derived T_eff per P100 GPU
METRIC = ("effective GB/s per GPU + weak-scaling parallel efficiency, "
          "3-D diffusion 512^3/GPU at 1/2/4/8 MI355X")
# What "value" is, appended to every metric label (BASELINE.json names the
# metric per GPU; the bench contract asks for the whole-job aggregate).
VALUE_LABEL = (" [value: whole-job aggregate GB/s = sum of the per-GPU T_eff over n_gpus GPUs; "
               "per GPU: config.t_eff_per_gpu_GBs]")
# Bitwise checks of the fused exchange against the update_halo_ path: a quick
# filter before the A/B, a long one for the candidate that is kept, and one
# after the timed region (from the state the timed steps left).
FUSED_CHECK_STEPS = 24
FUSED_KEEP_CHECK_STEPS = 200
# BASELINE.json configs. The driver runs the default (the headline metric).
CONFIGS = {
    "diffusion3d": dict(model="diffusion3d", n=512, dtype="float64", gather_every=0, metric=METRIC),
    "diffusion3d_f32_gather": dict(
        model="diffusion3d", n=1024, dtype="float32", gather_every=100,
        metric="effective GB/s per GPU, 3-D diffusion 1024^3/GPU Float32 with gather_ every 100 steps"),
    "acoustic2d": dict(
        model="acoustic2d", n=8192, dtype="float32", gather_every=0,
        metric="effective GB/s per GPU, 2-D staggered acoustic solver 8192^2/GPU Float32"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="diffusion3d", choices=sorted(CONFIGS))
    ap.add_argument("--n", "--local-n", dest="n", type=int, default=None,
                    help="local grid points per dimension (default: per config)")
    ap.add_argument("--dtype", default=None, choices=["float64", "float32"])
    ap.add_argument("--gather-every", type=int, default=None, help="gather_ the field to rank 0 every K steps")
    ap.add_argument("--gather-mode", default="async", choices=["async", "sync"],
                    help="async: gather_async_(snapshot=True): one copy per rank, then the root pulls with its "
                         "copy engines while stepping continues")
    ap.add_argument("--overlap", action="store_true",
                    help="force the boundary/interior split with the halo on a second stream (default: A/B decides)")
    ap.add_argument("--variant", default=None, help="stencil kernel variant (int) or 'auto'")
    ap.add_argument("--periodic", action="store_true", help="periodic boundaries in every dim")
    ap.add_argument("--periodic-dims", default=None,
                    help="periodic boundaries in a subset of 'xyz' only (with --loopback, 'xy' emulates "
                         "an interior rank of a 2x2x1 topology: no z exchange)")
    ap.add_argument("--loopback", action="store_true",
                    help="1 GPU: route all 6 faces through the RCCL remote path to itself (interior-rank emulation)")
    ap.add_argument("--graph", dest="graph", action="store_true", default=True,
                    help="replay the steps from a hipGraph (GRAPH_STEPS captured steps per replay; default)")
    ap.add_argument("--no-graph", dest="graph", action="store_false")
    ap.add_argument("--transport", default="auto", choices=["auto", "rccl", "put"],
                    help="device transport of the halo exchange (multi-GPU / loopback)")
    ap.add_argument("--fused", default="auto", choices=["auto", "on", "off"],
                    help="fused halo exchange inside the stencil kernel (diffusion3d; auto: bitwise check + A/B)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal only: every rank on device 0, 'staged' instead of RCCL as the A/B reference")
    ap.add_argument("--device", default="gpu", choices=["gpu", "cpu"],
                    help="cpu: host fields and the gloo exchange (launch/plumbing check, no GPU needed)")
    ap.add_argument("--launch-timeout", type=float, default=1800.0,
                    help="self-launch: seconds before the ranks are stopped and the run fails")
    return ap.parse_args()


def _supervise():
    """utils/supervise.py, loaded by path: a supervisor never imports the
    package (nor touches the GPU)."""
    import importlib.util as ilu

    mod = sys.modules.get("igg_supervise")
    if mod is None:
        p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "implicitglobalgrid.jl_amd", "utils",
                         "supervise.py")
        spec = ilu.spec_from_file_location("igg_supervise", p)
        mod = ilu.module_from_spec(spec)
        sys.modules["igg_supervise"] = mod
        spec.loader.exec_module(mod)
    return mod


def _share_gpu_env(args, env: dict) -> None:
    if args.share_gpu and args.gpus > 2:
        # Rehearsal with every rank on one GPU: N processes x 4 hardware
        # queues oversubscribe the device's queue slots and the command
        # processor time-slices them (8 ranks: 7.9 ms/step vs 0.25 with one
        # queue per process, profiles/r2_reh8/). One rank per GPU never does.
        # Overrides the environment's value (the GPU boxes export 4).
        env["GPU_MAX_HW_QUEUES"] = "1"


def self_launch(args) -> int:
    """``--gpus N`` without a launcher: start N ranks of this script (one per
    GPU, LOCAL_RANK = GPU index) from this parent, which never touches the GPU
    (it does not even import torch), and supervise them
    (igg/utils/supervise.py): a rank that dies or stalls past its phase
    deadline stops the attempt, and fresh ranks are started without the path
    that phase exercised (``config.excluded`` lists it). Prints rank 0's JSON
    line; non-zero exit if no attempt succeeded, the run timed out, or the
    line's n_gpus differs from N."""
    sup = _supervise()
    argv = [sys.executable, os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ, IGG_BENCH_SELF_LAUNCHED="1")
    rc, rec, excl = sup.run_local(argv, args.gpus, env, timeout=args.launch_timeout,
                                  env_for_rank=lambda r, e: _share_gpu_env(args, e))
    if rc != 0:
        print("bench self-launch: no attempt produced a result", file=sys.stderr)
        return rc
    if rec is None:
        print("bench self-launch: rank 0 printed no result line", file=sys.stderr)
        return 1
    got = json.loads(rec).get("n_gpus")
    if got != args.gpus:
        print(f"bench self-launch: result reports n_gpus={got}, expected {args.gpus}", file=sys.stderr)
        return 1
    print(rec, flush=True)
    return 0


def launcher_supervise(args) -> int:
    """Under a launcher (torchrun: WORLD_SIZE set, N > 1) this process becomes
    the supervisor of its rank: it starts the real worker (same rank / world,
    a per-attempt rendezvous port) and agrees with the other ranks'
    supervisors over the launcher's TCP store on done / relaunch without a
    path / fail (igg/utils/supervise.py). It never touches the GPU."""
    sup = _supervise()
    argv = [sys.executable, os.path.abspath(__file__), *sys.argv[1:]]
    return sup.run_torchrun(argv, timeout=args.launch_timeout, env_adjust=lambda e: _share_gpu_env(args, e))


def _first_contact() -> float:
    return float(os.environ.get("IGG_FIRST_CONTACT_TIMEOUT", "120"))


def _max_over_ranks(comm, v: float) -> float:
    import torch
    import torch.distributed as dist

    t = torch.tensor([v], dtype=torch.float64)
    if comm.size > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=comm.gloo)
    return float(t.item())


def _sync(comm=None) -> None:
    """Drain the GPU, bounded by IGG_COMM_TIMEOUT (aborts RCCL and raises
    instead of hanging on a dead peer)."""
    from igg.parallel.comm import bounded_device_sync

    bounded_device_sync(what="bench", comm=comm)


# Barrier flavour of the timed regions (set in main once RCCL is validated).
_BRACKET = {"dev": False, "gpu": True}


def _bracket(comm) -> None:
    """One side of a timed region: a barrier of all ranks + synchronize.
    GPU, several ranks with a validated RCCL communicator: a one-element RCCL
    all-reduce on the stream (it completes on a rank only once every rank has
    reached it: tens of us over xGMI), a bounded event poll of the stream
    (microseconds after completion; aborts RCCL on a dead peer) and
    torch.cuda.synchronize(). Otherwise drain, then the host barrier (gloo:
    0.2-0.7 ms, i.e. 2-5 % of a 20-step region: profiles/r2_bracket/)."""
    import torch

    if not _BRACKET["gpu"]:
        comm.barrier()
        return
    from igg.parallel.comm import bounded_stream_sync

    if _BRACKET["dev"] and comm.size > 1:
        comm.device_barrier()
        bounded_stream_sync(what="bench", comm=comm)
    else:
        bounded_stream_sync(what="bench", comm=comm)
        comm.barrier()
    torch.cuda.synchronize()


def _timed(model, comm, k: int) -> float:
    return _timed_fn(model.run, comm, k)[0]


def _timed_fn(run, comm, k: int) -> tuple[float, float]:
    """Seconds per step of ``run(k)`` between two barrier+synchronize
    brackets: (MAX over ranks, this rank's own)."""
    if _BRACKET["gpu"]:
        _sync(comm)
    _bracket(comm)
    t0 = time.perf_counter()
    run(k)
    _bracket(comm)
    own = time.perf_counter() - t0
    return _max_over_ranks(comm, own) / k, own / k


def _all_ranks(comm, v: float) -> list:
    """``v`` of every rank, in rank order (gloo all-gather)."""
    import torch
    import torch.distributed as dist

    t = torch.tensor([v], dtype=torch.float64)
    if comm.size == 1:
        return [float(v)]
    out = [torch.zeros(1, dtype=torch.float64) for _ in range(comm.size)]
    dist.all_gather(out, t, group=comm.gloo)
    return [float(x.item()) for x in out]


# Same-process weak-scaling efficiency (config.efficiency): interleaved pairs
# of [the local problem, the multi-rank step] in alternating order (even pairs
# local first, odd pairs step first: a fixed order biased round 5's N=1 value
# to 1.005 with a cold first local sample), after one untimed run of each form;
# medians.
EFF_PAIRS = 7
# steps per efficiency sample: at least this many (a 20-step sample of a
# 0.6 ms step is 12 ms, and its +-0.3 % run-to-run noise moved the N=1 value
# by 0.0045 on a round-6 box)
EFF_MIN_STEPS = 100
LOCAL_GRAPH_STEPS = 10


def _median(xs):
    s = sorted(xs)
    return s[len(s) // 2] if len(s) % 2 else 0.5 * (s[len(s) // 2 - 1] + s[len(s) // 2])


def _begin_local_steps(model) -> dict | None:
    """State kept across the efficiency phase's local steps, for models whose
    halo exchange cannot repair what local steps leave (no ``exchange_halos``:
    the acoustic model's staggered fields have planes computed on both ranks
    that drift apart, models/acoustic2d.py local_step; a fused post-check
    after this phase failed without the restore, profiles/r5_checks/c15)."""
    if hasattr(model, "exchange_halos"):
        return None
    return {n: getattr(model, n).clone() for n in _state(model)}


def _end_local_steps(model, saved: dict | None) -> None:
    """After the local steps: restore the kept state by content (buffer roles
    may have swapped) or re-exchange the halos; then the next fused step
    starts with its entry barrier (mark_modified)."""
    if saved is None:
        model.exchange_halos()  # also marks the fields modified
        return
    for n, t in saved.items():
        getattr(model, n).copy_(t)
    if hasattr(model, "mark_modified"):
        model.mark_modified()


def measure_efficiency(model, comm, log, graph: bool, k: int, pairs: int = EFF_PAIRS) -> dict | None:
    """Weak-scaling efficiency measured in THIS job: E = t_it(local) / t_it(step).

    ``t_it(step)``: the model's step as the timed region runs it (exchange
    included: update_halo_ or the fused exchange; hipGraph replays).
    ``t_it(local)``: the identical local problem as the 1-GPU run times it -
    the same plain stencil (variant, grid rounds, z-edge form) on the same
    arrays, no exchange (update_halo_ with PROC_NULL neighbours is a no-op,
    src/update_halo.jl:40-42), replayed from its own hipGraph - on every rank
    at once, so both numbers come from the same GPUs, processes, clocks and
    brackets (MAX over ranks each). ``pairs`` interleaved [local, step] pairs
    of ``k`` steps, medians. This removes the box-to-box spread (+-2-3 %)
    that a ratio of two different jobs' numbers carries (E(N) =
    t_it(1) / t_it(N)). Collective. The local steps leave the halo planes
    unexchanged; ``_end_local_steps`` repairs the state at the end. The
    caller takes any starting-state snapshot afterwards."""
    if not hasattr(model, "local_step"):
        return None
    saved = _begin_local_steps(model)
    k = max(EFF_MIN_STEPS, k)
    k = max(2, k + (k % 2))  # even: the ping-pong buffers keep their roles
    on_gpu = getattr(model, "device", None) is not None and model.device.type == "cuda"
    gl = None
    if on_gpu and graph:
        from igg.parallel.halo import capture_graph

        def rec():
            for _ in range(LOCAL_GRAPH_STEPS):
                model.local_step()

        model.local_step()
        model.local_step()
        try:
            gl = capture_graph(rec, "bench.local_problem", uses_halo=False)
        except Exception as e:
            log(f"efficiency: local-problem capture failed, eager ({type(e).__name__}: {e})"[:200])
            gl = None
        # every rank replays or none (the timings must be of the same form)
        if _max_over_ranks(comm, 0.0 if gl is not None else 1.0) > 0:
            gl = None

    def run_local(n):
        if gl is not None:
            for _ in range(n // LOCAL_GRAPH_STEPS):
                gl.replay()
            n %= LOCAL_GRAPH_STEPS
        for _ in range(n):
            model.local_step()

    # one untimed run of each form first (graph upload, clocks, caches), so
    # neither side's first sample is cold
    run_local(k)
    model.run(k)
    tl, tm, own_l, own_m, order = [], [], [], [], []
    for i in range(pairs):
        first_local = i % 2 == 0
        order.append("local,step" if first_local else "step,local")
        for is_local in ((True, False) if first_local else (False, True)):
            a, b = _timed_fn(run_local if is_local else model.run, comm, k)
            (tl if is_local else tm).append(a)
            (own_l if is_local else own_m).append(b)
    used_graph, gl = gl is not None, None
    _end_local_steps(model, saved)
    t_loc, t_step = _median(tl), _median(tm)
    per_rank_loc = _all_ranks(comm, _median(own_l))
    per_rank_step = _all_ranks(comm, _median(own_m))
    eff = t_loc / t_step if t_step > 0 else None
    log(f"efficiency (same process, {pairs} pairs in alternating order x {k} steps, medians): local "
        f"{t_loc * 1e3:.4f} ms [{min(tl) * 1e3:.4f}-{max(tl) * 1e3:.4f}], step {t_step * 1e3:.4f} ms "
        f"[{min(tm) * 1e3:.4f}-{max(tm) * 1e3:.4f}] -> E = {eff:.4f}")

    def _ms(xs):
        return {"min": round(min(xs) * 1e3, 5), "median": round(_median(xs) * 1e3, 5),
                "max": round(max(xs) * 1e3, 5)}

    return {
        "value": round(eff, 5) if eff is not None else None,
        "definition": "t_it(local problem) / t_it(step), same job: every rank times the identical local "
                      "problem of the 1-GPU run (plain stencil, no exchange) interleaved with the real step "
                      "(pair order alternates, one untimed run of each first); medians of the MAX over ranks",
        "t_local_ms": round(t_loc * 1e3, 5),
        "t_step_ms": round(t_step * 1e3, 5),
        "local_ms": _ms(tl),
        "step_ms": _ms(tm),
        "pairs": pairs,
        "pair_order": order,
        "steps": k,
        "local_ms_samples": [round(x * 1e3, 5) for x in tl],
        "step_ms_samples": [round(x * 1e3, 5) for x in tm],
        "per_rank_local_ms": [round(x * 1e3, 5) for x in per_rank_loc],
        "per_rank_step_ms": [round(x * 1e3, 5) for x in per_rank_step],
        # each rank's own local time over its own step time (both medians)
        "per_rank_efficiency": [round(a / s, 5) if s > 0 else None for a, s in zip(per_rank_loc, per_rank_step)],
        "local_graph": used_graph,
    }


class _ABBudget:
    """Total wall budget of the A/B stages (IGG_BENCH_AB_BUDGET seconds,
    default 150): candidates are tried in the order of their win record and
    the rest is skipped once the budget is spent. ``left()`` is collective
    (every rank takes the same decision: the MAX of the ranks' elapsed time)."""

    def __init__(self, comm, seconds: float | None = None):
        self.comm = comm
        self.seconds = float(os.environ.get("IGG_BENCH_AB_BUDGET", "150")) if seconds is None else seconds
        self.t0 = time.monotonic()
        self.skipped: list = []

    def elapsed(self) -> float:
        return time.monotonic() - self.t0

    def left(self) -> bool:
        return _max_over_ranks(self.comm, self.elapsed()) <= self.seconds


AB_BUDGET = None  # _ABBudget of the run (set in main)
# Host-side record of the stages around the timed region, in execution order
# (config.stage_order; tests/test_bench.py checks that nothing - no snapshot
# allocation or copy, no check - runs between the warm load and the bracket).
ORDER: list = []


def _timed_candidate(model, comm, k: int, graph: bool) -> float:
    """ms/step of the model's current schedule as the timed loop runs it:
    hipGraph replays of captured steps (eager if capture is unsupported)."""
    model.graph = None
    model.step()
    if graph:
        try:
            model.capture()
        except Exception:
            model.graph = None
    return _timed(model, comm, k)


def _step_estimate_ms(model, comm) -> tuple[float, int]:
    """(ms per step of the current schedule, steps run): one untimed replay
    (or step), MAX over ranks so every rank runs the same number of warm-up
    steps."""
    k = model.graph_steps if getattr(model, "graph", None) is not None else 1
    _sync(comm)
    t0 = time.perf_counter()
    model.run(k)
    _sync(comm)
    return max(0.05, _max_over_ranks(comm, (time.perf_counter() - t0) * 1e3 / k)), k


class _NoPhases:
    supervised = False

    def enter(self, *a, **k):
        pass

    def printed(self):
        pass

    def relaunch(self, keys, code=3):
        raise SystemExit(f"bench: relaunch without {sorted(keys)} requested outside a supervisor")


# Phase announcements to the supervisor and the paths excluded by it (set in
# main; igg/utils/supervise.py). Exclusion keys: rccl, put, fused,
# fused-inkernel, graph, host-ordered, host-tagged.
PH = _NoPhases()
EXCL: dict = {}


def _transport_key(t: str) -> str | None:
    return {"rccl": "rccl", "put": "put", "torch": "rccl"}.get(t)


def _path_key(model) -> str | None:
    """Exclusion key of what a time step of the model currently exercises."""
    from igg.parallel import halo as H

    if getattr(model, "fused", False):
        return "fused-inkernel" if getattr(model, "fused_mode", 0) & 16 else "fused"
    if getattr(model, "overlap", False):
        return "overlap"
    return _transport_key(H.transport_name())


def _check_abandoned(comm, key: str, what: str, log) -> None:
    """A bounded first-contact call (RCCL bootstrap, IPC open) that had to be
    abandoned leaves a thread stuck in the HIP runtime: such a process is not
    trusted with more GPU work. If it happened on any rank, every rank asks
    the supervisor for fresh processes without ``key`` (collective)."""
    from igg import native

    n = native.abandoned_waits() + (1 if _inject(f"abandon-{key}") else 0)  # test hook
    if _max_over_ranks(comm, float(n)) > 0:
        log(f"bench: {what}: a bounded first-contact call was abandoned; relaunching without {key!r}")
        PH.relaunch({key: f"{what}: a first-contact call (RCCL bootstrap / IPC open) was abandoned"})


def _probe_field(field):
    """Rank-distinct payload (exact in fp64) with every boundary plane poisoned,
    so a missing, misplaced or wrong-rank receive cannot go unnoticed."""
    import torch

    from igg.parallel.grid import global_grid

    me = int(global_grid().me)
    # built a slab of the outermost dim at a time (no field-size float64
    # temporary: 8 ranks x 1024^3 sharing one GPU ran out of memory here)
    X = torch.empty_like(field)
    n0 = field.shape[0]
    per = max(1, field.numel() // max(1, n0))
    slab = max(1, (1 << 24) // per)
    for a in range(0, n0, slab):
        b = min(n0, a + slab)
        v = torch.arange(a * per, b * per, dtype=torch.float64, device=field.device) + float(me + 1) * 2.0 ** 30
        X[a:b] = v.view((b - a,) + tuple(field.shape[1:]))
    for d in range(field.dim()):
        X.select(d, 0).fill_(-7.0)
        X.select(d, field.shape[d] - 1).fill_(-7.0)
    return X


# (name, transport, halo schedule) checked and A/B-timed at N > 1
TRANSPORT_CANDIDATES = (("rccl-sequential", "rccl", "sequential"),
                        ("rccl-onephase", "rccl", "onephase"),
                        ("put", "put", "auto"))


def validate_transports(field, comm, log, ref: str = "staged", names=None) -> dict:
    """Bitwise check of every device transport / schedule against the
    host-staged gloo exchange. Returns {name: "ok" | reason}; collective, and
    every rank agrees (a failure on any rank fails the candidate)."""
    import torch

    from igg.parallel import halo as H

    # the reference's boundary planes only (the only entries an exchange
    # writes), and one field-size probe at a time
    H.set_transport(ref)
    H.set_halo_mode("sequential")
    R = _probe_field(field)
    H.update_halo_(R)
    _sync(comm)
    Rb = _boundary(R)
    del R
    out = {}
    for name, t, mode in TRANSPORT_CANDIDATES:
        if names is not None and name not in names:
            continue
        key = _transport_key(t)
        if key in EXCL:
            out[name] = f"excluded: {EXCL[key]}"
            log(f"validation {name}: {out[name]}")
            continue
        # deadline: a bounded first contact (IGG_FIRST_CONTACT_TIMEOUT) + the exchange
        PH.enter(f"validate:{name}", key, deadline=2 * _first_contact() + 120)
        why, X = "", None
        try:
            H.set_transport(t)  # collective (outcome agreed): creates the RCCL communicator / put mesh
            H.set_halo_mode(mode)
            X = _probe_field(field)
        except Exception as e:  # e.g. no IPC mapping between these GPUs
            why = f"{type(e).__name__}: {e}"[:300]
        if _all_ok(comm, why):  # every rank has its probe: the exchange can start
            try:
                H.update_halo_(X)
                _sync(comm)
                H.check_transport()
                for k, (a, b) in enumerate(zip(_boundary(X), Rb)):
                    if not torch.equal(a, b):
                        bad = (a != b).nonzero()
                        why = f"mismatch in boundary plane {k} at {bad.shape[0]} entries, first {bad[0].tolist()}"
                        break
            except Exception as e:  # a bounded spin timed out, a transport error
                why = f"{type(e).__name__}: {e}"[:300]
                if getattr(comm, "mesh", None) is not None:
                    comm.mesh.clear_error()
        X = None
        fails = _max_over_ranks(comm, 1.0 if why else 0.0)
        out[name] = "ok" if fails == 0.0 else (why or "failed on another rank")
        log(f"validation {name} vs {ref}: {out[name]}")
        _check_abandoned(comm, key, f"validation of {name}", log)
    H.set_transport("rccl" if out.get("rccl-sequential") == "ok" else ref)
    H.set_halo_mode("auto")
    return out


def _boundary(X) -> list:
    """Copies of the boundary planes of ``X`` (index 0 and n-1 of every dim):
    the only entries a halo update writes (the halo is one plane wide whatever
    the overlap, SURVEY invariant 2) - compared instead of whole probe copies."""
    out = []
    for d in range(X.dim()):
        out.append(X.select(d, 0).clone())
        if X.shape[d] > 1:
            out.append(X.select(d, X.shape[d] - 1).clone())
    return out


def _all_ok(comm, why: str) -> bool:
    """Collective: True iff no rank reported a failure. Called between the
    collective stages of a check, so one rank's local failure (an allocation,
    a transport error before its messages were posted) never leaves the others
    waiting inside the next exchange."""
    return _max_over_ranks(comm, 1.0 if why else 0.0) == 0.0


def post_validate(field, comm, log, on_gpu: bool) -> dict:
    """After the timed region: one update_halo_ of the probe payload through
    the transport and schedule the timed steps used, compared bitwise with the
    host-staged gloo exchange (the reference's non-GPU-aware path). Collective;
    every rank agrees, stage by stage. The transport / schedule settings are
    restored. At most one field-size probe exists at a time (8 ranks of
    1024^3 f32 sharing one GPU ran out of memory with three).
    (CPU plumbing runs: the timed host matching form against the other one,
    order-only vs tagged, unless that one is excluded.)"""
    import torch

    from igg.parallel import halo as H

    if on_gpu:
        t, gmode = H.transport_name(), H.halo_mode()
        sched = "put" if t == "put" else H.plan_mode(field)
    else:
        m = os.environ.get("IGG_HOST_MATCHING", "ordered")
        t, gmode, sched = f"host-{m}", None, "sequential"
        other = "tagged" if m == "ordered" else "ordered"
    why, Xb = "", None

    def err(e) -> str:
        if getattr(comm, "mesh", None) is not None:
            try:
                comm.mesh.clear_error()
            except Exception:
                pass
        return f"{type(e).__name__}: {e}"[:300]

    try:
        X = None
        try:
            if on_gpu and t != "put":
                H.set_halo_mode(sched)
            X = _probe_field(field)
        except Exception as e:
            why = err(e)
        if _all_ok(comm, why):
            try:  # the timed path
                H.update_halo_(X)
                if on_gpu:
                    _sync(comm)
                H.check_transport()
                Xb = _boundary(X)
            except Exception as e:  # a bounded wait expired, a transport error
                why = err(e)
            X = None
        R = None
        if _all_ok(comm, why):
            try:  # the reference path
                if on_gpu:
                    H.set_transport("staged")
                    H.set_halo_mode("sequential")
                elif f"host-{other}" not in EXCL:
                    os.environ["IGG_HOST_MATCHING"] = other
                R = _probe_field(field)
            except Exception as e:
                why = err(e)
        if _all_ok(comm, why):
            try:
                H.update_halo_(R)
                if on_gpu:
                    _sync(comm)
                Rb = _boundary(R)
                R = None
                if _inject("post_validation"):
                    Xb[0].view(-1)[Xb[0].numel() // 2] += 1
                for k, (a, b) in enumerate(zip(Xb, Rb)):
                    if not torch.equal(a, b):
                        bad = (a != b).nonzero()
                        why = (f"mismatch in boundary plane {k} (dim {k // 2}) at {bad.shape[0]} entries, "
                               f"first {bad[0].tolist()}")
                        break
            except Exception as e:
                why = err(e)
    finally:
        if on_gpu:
            H.set_transport(t)
            H.set_halo_mode(gmode)
        else:
            os.environ["IGG_HOST_MATCHING"] = m
    fails = _max_over_ranks(comm, 1.0 if why else 0.0)
    res = "ok" if fails == 0.0 else (why or "failed on another rank")
    log(f"post-timing validation {t}/{sched} vs {'staged' if on_gpu else 'host-' + other}: {res}")
    return {"transport": t, "schedule": sched, "result": res}


def select_transport(model, comm, log, valid: dict, graph: bool) -> tuple[str, dict]:
    """A/B timing of the validated transports / schedules on the model's step
    (graph replays, MAX over ranks); keeps the fastest."""
    from igg.parallel import halo as H

    cands = [(name, t, mode, False) for name, t, mode in TRANSPORT_CANDIDATES if valid.get(name) == "ok"]
    # Overlap (boundary planes first, exchange on a second stream next to the
    # interior) only pays without z-neighbours: x/y boundary planes are cheap
    # rows, z-planes of a C-ordered field are maximally strided. (RCCL's p2p
    # kernels next to a full-GPU stencil measured slower than serial in
    # loopback, profiles/r1_ctas/; over real xGMI the A/B decides.)
    # Round 3 took them out of the default A/B after a SIGSEGV in the replay of
    # the captured overlapped put step (4 ranks sharing a GPU, 2x2x1,
    # profiles/r3_overlap_crash/); round 4 traced it to processes with ONE
    # hardware queue (GPU_MAX_HW_QUEUES=1, which the shared-GPU rehearsal
    # sets), where the model now runs the three parts in stream order
    # (profiles/r4_overlap_crash/). A crash of a candidate is a supervisor
    # relaunch without 'overlap'. IGG_BENCH_OVERLAP=0 leaves them out.
    if (os.environ.get("IGG_BENCH_OVERLAP", "1") != "0" and "overlap" not in EXCL
            and getattr(model, "can_overlap", False) and not any(model.sides[2])):
        if valid.get("put") == "ok":
            cands.append(("put+overlap", "put", "auto", True))
        if valid.get("rccl-sequential") == "ok":
            cands.append(("rccl+overlap", "rccl", "sequential", True))
    only = os.environ.get("IGG_BENCH_SCHEDULES")  # diagnosis: "put,put+overlap,..." limits the A/B
    if only:
        cands = [c for c in cands if c[0] in only.split(",")]
    if not cands:
        raise RuntimeError("no device transport passed the bitwise validation against the host-staged path")
    times = {}
    for i, (name, t, mode, ov) in enumerate(cands):
        if i > 0 and AB_BUDGET is not None and not AB_BUDGET.left():
            AB_BUDGET.skipped.append(name)
            continue
        PH.enter(f"ab:{name}", "overlap" if ov else _transport_key(t), deadline=300)
        H.set_transport(t)
        H.set_halo_mode(mode)
        if hasattr(model, "set_overlap"):
            model.set_overlap(ov)
        times[name] = (_timed_candidate(model, comm, 20, graph), t, mode, ov)
    best = min(times, key=lambda k: times[k][0])
    _, t, mode, ov = times[best]
    H.set_transport(t)
    H.set_halo_mode(mode)
    if hasattr(model, "set_overlap"):
        model.set_overlap(ov)
    model.graph = None
    log(f"schedule A/B (ms/step): {', '.join(f'{k}={v[0] * 1e3:.4f}' for k, v in times.items())} -> {best}")
    return best, {k: round(v[0] * 1e3, 5) for k, v in times.items()}


def _inject(what: str) -> bool:
    """Test hook (IGG_BENCH_INJECT=what[,what]): corrupt one element on rank 0
    of the named check's result, to prove the check fails closed."""
    from igg.parallel.grid import global_grid

    return what in os.environ.get("IGG_BENCH_INJECT", "").split(",") and int(global_grid().me) == 0


def _state(model) -> list[str]:
    """Names of the model fields a time step evolves (saved and restored)."""
    return ["P", "Vx", "Vy", "P2", "Vx2", "Vy2"] if hasattr(model, "Vx") else ["T", "T2"]


def _compared(model) -> list[str]:
    """The fields the fused check compares bitwise: every acoustic field (its
    fused step leaves every halo as update_halo_ would); the diffusion model's
    T only (after sync_halo; T2, the previous step's buffer, keeps stale halo
    planes in fused mode by design and is rewritten by the next step)."""
    return _state(model) if hasattr(model, "Vx") else ["T"]


def _fused_name(model) -> str:
    if hasattr(model, "fused_variant"):
        return f"v{model.fused_variant}/m{model.fused_mode}/r{model.fused_rounds}"
    return "fused"


def _fused_check(model, comm, log, nchk: int = FUSED_CHECK_STEPS, inject: str = "") -> bool:
    """Bitwise check of the model's CURRENT fused exchange (diffusion: variant /
    send mode / grid rounds; acoustic: the fused staggered step) against the
    update_halo_ path: ``nchk`` steps from the same state on every rank, in the
    timed run's execution shape (hipGraph replays of captured fused steps plus
    eager steps for the parity). Collective; every rank agrees. The model's
    state is restored (by content)."""
    import torch

    names = _state(model)
    model.set_fused(False)
    # The reference is the serial update_halo_ step: an overlapped schedule
    # (boundary slabs by another kernel variant) is not bitwise comparable
    # with the fused kernel in every dtype (f32 contraction differs).
    ov = bool(getattr(model, "overlap", False))
    if ov:
        model.set_overlap(False)
    # The state to restore: on the host when ranks share one GPU (8 ranks of
    # 1024^3 f32 ran out of the shared device memory with it on the device:
    # 8 x 8 GiB, profiles/r6_checks/rehearsals/).
    host = bool(_BRACKET.get("shared"))
    saved = {n: (getattr(model, n).to("cpu") if host else getattr(model, n).clone()) for n in names}

    def restore():
        for n in names:
            getattr(model, n).copy_(saved[n])

    model.run(nchk)
    ref = {n: getattr(model, n).clone() for n in names}
    restore()
    ok, exc = False, ""
    try:
        model.set_fused(True)
        model.step()
        model.capture(steps=4)
        model.run(nchk - 1)
        model.graph = None
        if hasattr(model, "sync_halo"):
            model.sync_halo()
        _sync(comm)
        model.check()
        if inject and _inject(inject):
            t = getattr(model, _compared(model)[0])
            t.view(-1)[t.numel() // 2] += 1
        cmp = _compared(model)
        ok = all(bool(torch.equal(ref[n], getattr(model, n))) for n in cmp)
        if not ok:
            n = next(n for n in cmp if not torch.equal(ref[n], getattr(model, n)))
            d = (ref[n] != getattr(model, n)).nonzero()
            from igg.parallel.grid import global_grid

            print(f"rank {int(global_grid().me)}: fused check {_fused_name(model)}: {n} differs in "
                  f"{d.shape[0]} entries, first {d[:4].tolist()}", file=sys.stderr, flush=True)
    except Exception as e:  # e.g. a sync kernel timed out: this fused kernel does not work here
        exc = f"{type(e).__name__}: {e}"[:300]
        from igg.parallel.grid import global_grid

        print(f"rank {int(global_grid().me)}: fused check {_fused_name(model)} failed: {exc}", file=sys.stderr,
              flush=True)
        if getattr(comm, "mesh", None) is not None:
            comm.mesh.clear_error()
    if _max_over_ranks(comm, 1.0 if exc else 0.0) and PH.supervised:
        # An exception in the middle of collective steps (a timeout, out of
        # memory) can leave the ranks' exchange counters out of step: not a
        # state to continue from. Fresh processes without this form instead.
        key = "fused-inkernel" if getattr(model, "fused_mode", 0) & 16 else "fused"
        PH.relaunch({key: f"fused check {_fused_name(model)} raised on some rank ({exc or 'another rank'})"})
    bad = _max_over_ranks(comm, 0.0 if ok else 1.0)
    if bad:
        # A timed-out fused step leaves the fused mesh's sticky error word set
        # on some ranks: drain, then reset it, so the update_halo_ path the
        # bench falls back to does not report the dropped form's error.
        try:
            _sync(comm)
        except Exception as e:
            log(f"fused check: drain after the failure: {type(e).__name__}: {e}"[:200])
        if hasattr(model, "clear_error"):
            model.clear_error()
    restore()
    model.fused, model.graph = False, None
    if hasattr(model, "_fprimed"):
        model._fprimed = False  # T was restored: halos valid
    if ov:
        model.set_overlap(True)
    del ref, saved
    return bad == 0.0


def select_fused(model, comm, log, mode: str, graph: bool = True) -> dict | None:
    """Fused halo exchange (the kernel stores its send planes / faces into the
    neighbours' memory; igg/fused.hpp, igg/acoustic.hpp) vs the schedule chosen
    so far: bitwise check of 24 steps from the same state on every rank, A/B
    timing of the candidates (MAX over ranks), then a 200-step bitwise check
    of the candidate that is kept (falling back to the next fastest that
    passes). ``mode``: auto (keep the faster), on (force when it checks out), off."""
    if mode == "off" or not getattr(model, "can_fuse", False):
        return None
    if "fused" in EXCL:
        log(f"fused halo exchange: excluded ({EXCL['fused']})")
        return {"fused_ok": False, "excluded": EXCL["fused"]}
    # the first switch-on maps the neighbours' arenas and fields (IPC, bounded)
    PH.enter("fused:check", "fused", deadline=2 * _first_contact() + 300)
    ok = _fused_check(model, comm, log)
    _check_abandoned(comm, "fused", "fused exchange setup", log)
    if not ok:
        log("fused halo exchange mismatched the update_halo_ path on some rank: excluded")
        return {"fused_ok": False}
    diffusion = hasattr(model, "fused_variant")
    if diffusion:
        # Fused kernel candidates: tiling variant x send mode (0 = stores as
        # computed, 1 = deferred one x step: robust to slow remote
        # acknowledgements). Two interleaved passes of 20 steps, best of the
        # two per candidate: the candidates differ by a few us/step, about the
        # size of one pass's noise.
        cands = list(FUSED_CANDIDATES)
        if any(model.sides[2]) and model._fh is not None and model._fh.has_fields:
            cands += FUSED_DIRECT
            if model.T.dtype.itemsize == 4:
                cands += FUSED_DIRECT_F32
        if any(model.sides[2]):
            cands += FUSED_ZUNPACK
            if model.T.dtype.itemsize == 4:
                cands += FUSED_ZUNPACK_F32
        # every form also with its exchanged x planes peeled off the chunk sweep
        # (send mode bit 8: profiles/r2_peel/, -1.8 % f64 / -2.8 % f32 interior rank)
        cands += [(v, fm | 8, gr) for v, fm, gr in cands]
        cands = _win_order(cands)
        if os.environ.get("IGG_FUSED_CANDIDATES"):  # "v/mode/rounds,..." (measurements)
            cands = [tuple(int(x) for x in c.split("/")) for c in os.environ["IGG_FUSED_CANDIDATES"].split(",")]
    else:
        cands = [None]  # the acoustic step has one fused form

    def use(c):
        if c is not None:
            model.fused_variant, model.fused_mode, model.fused_rounds = c

    name = (lambda k: f"v{k[0]}/m{k[1]}/r{k[2]}") if diffusion else (lambda k: "fused")  # noqa: E731
    ckey = (lambda k: "fused-inkernel" if k is not None and k[1] & 16 else "fused")  # noqa: E731
    unf_key = _path_key(model)
    t_unf, times = float("inf"), {}

    def timing_passes(cs):
        nonlocal t_unf
        for p in range(2):
            if p > 0 and AB_BUDGET is not None and not AB_BUDGET.left():
                break  # the first pass's numbers stand
            PH.enter("fused:ab:update_halo", unf_key, deadline=300)
            model.set_fused(False)
            t_unf = min(t_unf, _timed_candidate(model, comm, 20, graph))
            model.set_fused(True)
            for i, c in enumerate(cs):
                if times.get(c) == float("inf"):
                    continue  # failed in the first pass
                if p > 0 and c not in times:
                    continue  # skipped for the budget in the first pass
                # the first candidate of the first pass always runs (the
                # record's best form); later ones while the budget lasts
                if (p > 0 or i > 0) and AB_BUDGET is not None and not AB_BUDGET.left():
                    if p == 0:
                        AB_BUDGET.skipped.extend(name(x) for x in cs[i:])
                    break
                use(c)
                PH.enter(f"fused:ab:{name(c)}", ckey(c), deadline=300)
                err = ""
                try:
                    t = _timed_candidate(model, comm, 20, graph)
                except Exception as e:  # this form cannot run here (e.g. a bounded wait expired)
                    t, err = float("inf"), f"{type(e).__name__}: {e}"[:200]
                if _max_over_ranks(comm, 1.0 if err else 0.0):
                    if PH.supervised:  # fresh processes without this class of forms (see _fused_check)
                        PH.relaunch({ckey(c): f"fused candidate {name(c)} raised on some rank ({err or 'another'})"})
                    # every rank drops the form together; a neighbour's timed-out
                    # waits left the sticky error word set: drain and reset it
                    log(f"fused candidate {name(c)} failed: {err or 'on another rank'}")
                    try:
                        _sync(comm)
                    except Exception:
                        pass
                    if hasattr(model, "clear_error"):
                        model.clear_error()
                    model.graph = None
                    t = float("inf")
                times[c] = min(times.get(c, float("inf")), t)

    timing_passes(cands)
    # The step synchronisation inside the fused kernel (send mode bit 16, put.hpp
    # StepSync) is a candidate of its own: the two fastest sync-kernel forms are
    # re-timed with it, where it is allowed (not where ranks share a GPU, not
    # excluded by the supervisor after a failure). Its kept check below is the
    # same 200-step bitwise check; if it fails, the next fastest form - a
    # sync-kernel one - is kept.
    # The gate depends on per-rank facts (a rank shares its GPU, the
    # IGG_FUSED_SYNC_KERNEL of its environment): every rank takes it only if
    # every rank can (timing_passes is collective; a split decision would leave
    # some ranks waiting in its collectives until the phase deadline).
    inkernel_ok = (diffusion and "fused-inkernel" not in EXCL and model._fh is not None
                   and model._fh.in_kernel_sync_for(16) and not model._fh.in_kernel_sync_for(0)
                   and os.environ.get("IGG_FUSED_INKERNEL", "1") != "0")
    if diffusion and _max_over_ranks(comm, 0.0 if inkernel_ok else 1.0) == 0.0:
        front = [c for c, _t in sorted(times.items(), key=lambda kv: kv[1]) if not c[1] & 16][:2]
        timing_passes([(v, fm | 16, gr) for v, fm, gr in front])
    model.set_fused(False)
    model.graph = None
    keep, best, rejected = False, None, []
    for cand, t_fus in sorted(times.items(), key=lambda kv: kv[1]):
        if t_fus == float("inf") or not (mode == "on" or t_fus < t_unf):
            break
        use(cand)
        # the kept candidate: a long check whatever the quick one said
        PH.enter(f"fused:keep:{name(cand)}", ckey(cand), deadline=600)
        if _fused_check(model, comm, log, nchk=FUSED_KEEP_CHECK_STEPS):
            keep, best = True, cand
            break
        rejected.append(name(cand))
    if keep:
        use(best)
    model.set_fused(keep)
    model.graph = None
    log(f"fused A/B (ms/step): update_halo={t_unf * 1e3:.4f}, "
        + ", ".join(f"fused {name(k)}={t * 1e3:.4f}" for k, t in times.items())
        + f" -> {'fused ' + name(best) if keep else 'update_halo'}"
        + (f" (failed their bitwise check: {', '.join(rejected)})" if rejected else ""))
    out = {"fused_ok": True, "update_halo": round(t_unf * 1e3, 5),
           "kept_check_steps": FUSED_KEEP_CHECK_STEPS if keep else None}
    out.update({f"fused_{name(k)}": (round(t * 1e3, 5) if t != float("inf") else None) for k, t in times.items()})
    if rejected:
        out["fused_rejected"] = rejected
    return out


def _second_variant(model):
    """A compiled stencil variant other than the timed one (every rank picks
    the same: the autotune's ranking is summed over ranks), or None on CPU."""
    if getattr(model, "variant", None) is None:
        return None
    from igg.ops import stencil

    ranked = []
    for k, t in sorted((model.variant_times or {}).items(), key=lambda kv: kv[1]):
        v = int(k.split("@")[0])
        if v not in ranked:
            ranked.append(v)
    compiled = set(stencil.compiled_variants())
    for v in ranked + list(stencil.SHORTLIST):
        if v != model.variant and v in compiled:
            return v
    return None


def _save_start(model, pre: dict) -> None:
    """Save the state a timed region starts from into ``pre`` (reused buffers):
    the compared fields whole; any other state field (the diffusion model's T2)
    only by its boundary planes - its interior is rewritten by the first step
    and its halo planes by that step's exchange, so the planes at physical
    boundaries (never written) are all of it that the re-run depends on. Keeps
    the check to one extra field copy per compared field (1024^3 f32 x 8 ranks
    on one GPU did not fit two)."""
    import torch

    ORDER.append("snapshot")
    cmp = _compared(model)
    for nm in _state(model):
        src = getattr(model, nm)
        if nm in cmp:
            if nm not in pre:
                pre[nm] = torch.empty_like(src)
            pre[nm].copy_(src)
        else:
            pre[nm] = _boundary(src)


def _restore_start(model, pre: dict) -> None:
    for nm in _state(model):
        dst, src = getattr(model, nm), pre[nm]
        if isinstance(src, list):
            i = 0
            for d in range(dst.dim()):
                dst.select(d, 0).copy_(src[i])
                i += 1
                if dst.shape[d] > 1:
                    dst.select(d, dst.shape[d] - 1).copy_(src[i])
                    i += 1
        else:
            dst.copy_(src)
    if hasattr(model, "mark_modified"):
        model.mark_modified()


def stencil_post_check(model, comm, log, pre: dict, k: int, on_gpu: bool, timed_steps: int | None = None) -> dict:
    """After the timed region (update_halo_ path, any N): restore the state
    of the snapshot taken before the warm load, run the same ``k`` steps
    (warm load + timed steps: ``timed_steps`` of them timed) eagerly with a
    SECOND compiled stencil variant (bitwise interchangeable by construction,
    tests/test_gpu_stencil.py) and compare the result bitwise with the field
    the timed steps produced. A mismatch means the timed run computed a wrong
    field: the caller prints no number. Collective (every rank agrees).
    Only the compared fields of the timed end state are kept: when the check
    passes the re-run has reproduced that state (deterministic steps), when
    it fails those fields are put back and no number is printed. (CPU
    plumbing: the host kernel again, i.e. a determinism check.)"""
    import torch

    names = _compared(model)
    v_timed, graph = getattr(model, "variant", None), model.graph
    v2 = _second_variant(model) if on_gpu else None
    why, done = "", None
    try:
        done = {n: getattr(model, n).clone() for n in names}
    except Exception as e:  # e.g. out of memory: every rank skips the re-run together
        why = f"{type(e).__name__}: {e}"[:300]
    if not _all_ok(comm, why):
        res = why or "failed on another rank"
        log(f"post-timing stencil check: could not start ({res})")
        return {"steps": k, "timed_steps": timed_steps, "variant": v_timed, "check_variant": v2, "result": res}
    try:
        _restore_start(model, pre)
        model.graph = None
        if v2 is not None:
            model.variant = v2
        model.run(k)
        if on_gpu:
            _sync(comm)
        if _inject("stencil_post"):
            t = getattr(model, names[0])
            t.view(-1)[t.numel() // 2] += 1
        cmp = _compared(model)
        bad = [n for n in cmp if not torch.equal(getattr(model, n), done[n])]
        if bad:
            d = (getattr(model, bad[0]) != done[bad[0]]).nonzero()
            why = f"{bad[0]} differs in {d.shape[0]} entries, first {d[0].tolist()}"
    except Exception as e:
        why = f"{type(e).__name__}: {e}"[:300]
    finally:
        model.variant = v_timed
        if why:
            for n in names:
                getattr(model, n).copy_(done[n])
            if hasattr(model, "mark_modified"):
                model.mark_modified()
        done = None
        model.graph = graph
    fails = _max_over_ranks(comm, 1.0 if why else 0.0)
    res = "ok" if fails == 0.0 else (why or "failed on another rank")
    log(f"post-timing stencil check ({k} steps from the pre-warm-load snapshot, variant {v_timed} vs "
        f"{v2 if v2 is not None else 'same'}): {res}")
    return {"steps": k, "timed_steps": timed_steps, "variant": v_timed, "check_variant": v2, "result": res}


def validate_host_matching(field, comm, log) -> dict:
    """CPU plumbing runs with several ranks: the probe payload through the
    order-only host matching (one tag-0 message per peer and phase, paired by
    issue order - RCCL's rule) and through the tagged one; both must agree
    bitwise. Excluded forms are skipped; the first that passes is used."""
    import torch

    from igg.parallel import halo as H

    X0 = _probe_field(field)
    outs, res = {}, {}
    for name in ("host-ordered", "host-tagged"):
        if name in EXCL:
            res[name] = f"excluded: {EXCL[name]}"
            continue
        PH.enter(f"validate:{name}", name, deadline=300)
        os.environ["IGG_HOST_MATCHING"] = name.split("-")[1]
        X = X0.clone()
        try:
            H.update_halo_(X)
            outs[name] = X
        except Exception as e:
            res[name] = f"{type(e).__name__}: {e}"[:300]
        _check_abandoned(comm, name, f"validation of {name}", log)
    if len(outs) == 2:
        same = torch.equal(outs["host-ordered"], outs["host-tagged"])
        if _inject("host_matching") or not same:
            res["host-ordered"] = res["host-tagged"] = "the two matching forms disagree"
    for name in outs:
        res.setdefault(name, "ok")
    for name in ("host-ordered", "host-tagged"):
        if name in res and name not in EXCL:
            fails = _max_over_ranks(comm, 0.0 if res[name] == "ok" else 1.0)
            if fails and res[name] == "ok":
                res[name] = "failed on another rank"
    ok = [n for n in ("host-ordered", "host-tagged") if res.get(n) == "ok"]
    if not ok:
        raise RuntimeError(f"no host matching form passed the probe exchange: {res}")
    os.environ["IGG_HOST_MATCHING"] = ok[0].split("-")[1]
    log(f"host matching validation: {res} -> {ok[0]}")
    return res


T_START = time.monotonic()


def main():
    global AB_BUDGET
    args = parse()
    import faulthandler

    faulthandler.enable()  # a fatal signal (segfault, abort) prints the rank's Python stack
    if os.environ.get("IGG_BENCH_STACKS"):  # diagnosis of a hang: every rank's Python stack every N s
        faulthandler.dump_traceback_later(float(os.environ["IGG_BENCH_STACKS"]), repeat=True)
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(self_launch(args))
    world = int(world_env or "1")
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report an "
                         f"{world}-process number as an {args.gpus}-GPU one")
    if (world > 1 and os.environ.get("IGG_SUP_CHILD") != "1"
            and os.environ.get("IGG_BENCH_SUPERVISE", "1") != "0"):
        sys.exit(launcher_supervise(args))
    global PH, EXCL
    sup = _supervise()
    PH, EXCL = sup.Phases(), sup.excluded()
    PH.enter("init", None, deadline=600)
    import torch

    import igg
    from igg.models.acoustic2d import Acoustic2D
    from igg.models.diffusion3d import Diffusion3D

    if args.variant is not None:
        os.environ["IGG_STENCIL_VARIANT"] = str(args.variant)
    from igg.parallel import halo as H

    cfg = CONFIGS[args.config]
    dtype = getattr(torch, args.dtype or cfg["dtype"])
    n = args.n or cfg["n"]
    gather_every = cfg["gather_every"] if args.gather_every is None else args.gather_every
    is2d = cfg["model"] == "acoustic2d"
    on_gpu = args.device == "gpu"
    pdims = "xyz" if args.periodic else (args.periodic_dims or "")
    if set(pdims) - set("xyz"):
        raise SystemExit(f"--periodic-dims: expected a subset of 'xyz', got {pdims!r}")
    perx, pery, perz = (int(c in pdims) for c in "xyz")
    if args.transport != "auto":
        os.environ["IGG_TRANSPORT"] = args.transport
    # A put exchange that cannot complete must not stall the run for long.
    os.environ.setdefault("IGG_PUT_TIMEOUT", "20")
    if args.share_gpu:
        os.environ.setdefault("IGG_TRANSPORT", "staged")
        _BRACKET["shared"] = True  # the ranks' device memory is one pool (_fused_check keeps its copy on the host)
    # The bench validates and A/B-times the transports itself (validate_transports,
    # select_transport below): the library's own first-exchange choice
    # (IGG_TRANSPORT=auto) stays out of the model setup before them.
    os.environ.setdefault("IGG_TRANSPORT", "rccl")
    if "gather-pull" in EXCL:
        os.environ["IGG_GATHER_PULL"] = "0"
    me, dims, nprocs, coords, comm = igg.init_global_grid(
        n, n, 1 if is2d else n, periodx=perx, periody=pery, periodz=0 if is2d else perz, quiet=True,
        select_device=on_gpu and not args.share_gpu, device_type="auto" if on_gpu else "none")
    if nprocs != args.gpus:
        raise SystemExit(f"bench: the grid has {nprocs} ranks, --gpus is {args.gpus}")
    log = (lambda m: print(m, file=sys.stderr, flush=True)) if me == 0 else (lambda m: None)
    if on_gpu and not torch.cuda.is_available():
        raise SystemExit("bench: no GPU visible (use --device cpu for a plumbing run)")
    if args.loopback:
        lb = (bool(perx), bool(pery), bool(perz)) if pdims else (True, True, True)
        H.enable_loopback((lb[0], lb[1], lb[2] and not is2d))
    dev = None if on_gpu else "cpu"
    PH.enter("model", None, deadline=900)  # allocation + stencil autotune
    model = Acoustic2D(dtype=dtype) if is2d else Diffusion3D(dtype=dtype, overlap=args.overlap, device=dev)
    if me == 0 and getattr(model, "placement", None):
        pl = model.placement
        print(f"field placement: {pl['candidates']} candidate allocations, ms/step {pl['ms']} -> #{pl['chosen']}",
              file=sys.stderr, flush=True)
    field = (lambda: model.P) if is2d else (lambda: model.T)
    sync = (lambda: _sync(comm)) if on_gpu else (lambda: None)
    A_global = None
    if gather_every > 0 and me == 0:
        # gather_ concatenates the local blocks (halos included) in Cartesian order
        A_global = torch.empty([int(d) * int(s) for d, s in zip(dims, field().shape)],
                               dtype=dtype, device=field().device)
    graph_ok = args.graph and on_gpu and "graph" not in EXCL
    _BRACKET["gpu"], _BRACKET["dev"] = on_gpu, False
    valid, ab = None, None
    AB_BUDGET = _ABBudget(comm)  # the transport + fused A/B stages share one wall budget
    AB_BUDGET.elapsed_at_end = 0.0
    if on_gpu and nprocs > 1:
        ref = "staged"
        names = None if args.transport == "auto" else [c[0] for c in TRANSPORT_CANDIDATES if c[1] == args.transport]
        if args.share_gpu:  # ranks share one device: RCCL refuses duplicate GPUs
            names = ["put"]
        valid = validate_transports(field(), comm, log, ref=ref, names=names)
        AB_BUDGET.t0 = time.monotonic()  # the budget covers the A/B timing, not the correctness checks
        _BRACKET["dev"] = bool(comm.rccl is not None and valid.get("rccl-sequential") == "ok")
        if args.share_gpu and valid.get("put") != "ok":
            H.set_transport("staged")
        elif not args.overlap:
            _, ab = select_transport(model, comm, log, valid, graph_ok)
        elif any(v == "ok" for v in valid.values()):
            first = next(c for c in TRANSPORT_CANDIDATES if valid.get(c[0]) == "ok")
            H.set_transport(first[1])
            H.set_halo_mode(first[2])
        else:
            raise RuntimeError("no device transport passed the bitwise validation")
    host_valid = None
    if not on_gpu and nprocs > 1:
        host_valid = validate_host_matching(field(), comm, log)
    fused_ab = None
    if on_gpu and not args.overlap and (nprocs > 1 or args.loopback or pdims):
        fused_ab = select_fused(model, comm, log, args.fused, graph_ok)
    AB_BUDGET.elapsed_at_end = AB_BUDGET.elapsed() if (valid is not None or fused_ab is not None) else 0.0
    if AB_BUDGET.skipped:
        log(f"A/B budget ({AB_BUDGET.seconds:.0f} s) spent: skipped {', '.join(AB_BUDGET.skipped)}")
    PH.enter("warmup", _path_key(model), deadline=300)
    for _ in range(args.warmup):
        model.step()
    graph_error = None
    if graph_ok:
        PH.enter("capture", "graph", deadline=300)
        try:
            model.capture()
        except Exception as e:  # capture unsupported here: time eager steps
            graph_error = f"{type(e).__name__}: {e}"[:200]
            model.graph = None
            log(f"hipGraph capture failed, running eager: {graph_error}")
    # Same-process weak-scaling efficiency (config.efficiency): interleaved
    # pairs of the 1-GPU run's local problem and the real step, on these GPUs
    # and processes. Before the snapshot and the warm load below (it ends with
    # one halo exchange: the local steps leave the halos unexchanged).
    eff = None
    if os.environ.get("IGG_BENCH_EFFICIENCY", "1") != "0":
        PH.enter("efficiency", _path_key(model), deadline=300)
        eff = measure_efficiency(model, comm, log, graph_ok, args.steps)
        ORDER.append("efficiency")
    pre = {}  # the state a non-fused timed region starts from (stencil_post_check)
    warm = {"extra": None, "since_snapshot": 0}

    def warm_load():
        """Snapshot, then the untimed warm load, then NOTHING but the timed
        region's bracket. The post-timing stencil check replays every step
        from the snapshot (warm load + timed steps), so its buffers are
        allocated and copied here, before the warm load, never between the
        warm load and the bracket (round 4 lost 2.9 % of the driver's
        20-step number to a 1 GiB snapshot taken right before the bracket).
        Steady-state warm-up through the timed path: MI355X needs ~10-20 ms
        of continuous load after a lighter phase (autotune launches with host
        syncs, capture, this snapshot) before its clocks settle; the first
        two 10-step replays after capture measured 5-7 % slower
        (profiles/r2_gap/NOTES.md). So the W requested warm-up steps are
        followed by enough untimed replays to keep the GPU busy for
        IGG_BENCH_WARM_MS (default 40 ms) right before the timed region,
        which is unchanged: exactly K full steps."""
        PH.enter("warmup", _path_key(model), deadline=300)
        if not getattr(model, "fused", False):
            _save_start(model, pre)
        else:
            pre.clear()
        since = 0
        warm_ms = float(os.environ.get("IGG_BENCH_WARM_MS", "40"))
        if on_gpu and warm_ms > 0:
            if warm["extra"] is None:
                est, k_est = _step_estimate_ms(model, comm)
                since += k_est
                k = max(1, getattr(model, "graph_steps", 1) if getattr(model, "graph", None) is not None else 1)
                warm["extra"] = int(-(-warm_ms // (est * k))) * k
            model.run(warm["extra"])
            since += warm["extra"]
        warm["since_snapshot"] = since
        ORDER.append("warm_load")

    timed_graph = [False]  # whether the last timed region replayed a hipGraph

    def timed_region() -> float:
        """The timed region: exactly ``args.steps`` full steps (plus the
        configured gathers) between two barrier+synchronize brackets; MAX over
        ranks of the wall time. Preceded directly by ``warm_load``."""
        PH.enter("timed", _path_key(model), deadline=600)
        timed_graph[0] = getattr(model, "graph", None) is not None
        ORDER.append("timed")
        sync()
        _bracket(comm)
        t0 = time.perf_counter()
        if gather_every > 0:
            done, pending = 0, None
            async_gather = args.gather_mode == "async" and on_gpu
            while done < args.steps:
                k = min(gather_every, args.steps - done)
                model.run(k)
                done += k
                if done % gather_every == 0:
                    if getattr(model, "fused", False):
                        model.sync_halo()  # fused steps leave the halo planes stale
                    if not async_gather:
                        igg.gather_(field(), A_global)
                    else:
                        if pending is not None:
                            pending.wait()
                        # snapshot: every rank copies T now (its staging chunks /
                        # the root's block of A_global), the only serial part; the
                        # root pulls the chunks while the next steps run
                        pending = igg.gather_async_(field(), A_global, snapshot=True)
            if pending is not None:
                pending.wait()
        else:
            model.run(args.steps)
        _bracket(comm)
        t1 = time.perf_counter()
        return _max_over_ranks(comm, t1 - t0)

    warm_load()
    elapsed = timed_region()
    H.check_transport()
    if hasattr(model, "check"):
        model.check()
    # After the timed region: prove the steps that were timed computed the
    # right field, and fail closed if not (a wrong field never yields a number).
    #  1. fused exchange: K fused vs K update_halo_ steps from the state the
    #     timed steps left, bitwise; on a mismatch the fused exchange is
    #     dropped and the region re-timed on the update_halo_ path;
    #  2. every multi-rank run: the probe payload through the transport and
    #     schedule the timed steps used, bitwise vs the host-staged reference;
    #     on a mismatch the run is re-timed on the next validated schedule, and
    #     fails (no JSON line) when none is left.
    fused_post = None
    if getattr(model, "fused", False):
        PH.enter("post:fused", _path_key(model), deadline=600)
        n_post = max(args.steps, FUSED_KEEP_CHECK_STEPS)
        ok = _fused_check(model, comm, log, nchk=n_post, inject="fused_post")
        fused_post = {"steps": n_post, "result": "ok" if ok else "mismatch"}
        if ok:
            model.set_fused(True)
        else:
            log("fused halo exchange: post-timing check FAILED; re-timing on the update_halo_ path")
            fused_post["fallback"] = "update_halo_ (re-timed)"
            model.graph = None
            if graph_ok:
                model.capture()
            warm_load()  # snapshot + the same untimed warm load as before the first region
            elapsed = timed_region()
            H.check_transport()
    post_valid = None
    if nprocs > 1:
        PH.enter("post:transport", _path_key(model), deadline=300)
        post_valid = post_validate(field(), comm, log, on_gpu)
        tried = [(post_valid["transport"], post_valid["schedule"])]
        while post_valid["result"] != "ok":
            nxt = next(((t, m) for name, t, m in TRANSPORT_CANDIDATES
                        if (valid or {}).get(name) == "ok" and (t, m) not in tried), None)
            if nxt is None:
                log(f"bench: post-timing validation failed ({post_valid['result']}) and no validated schedule "
                    f"is left: no result")
                raise SystemExit(1)
            log(f"bench: post-timing validation of {tried[-1]} failed: re-timing with {nxt}")
            tried.append(nxt)
            if getattr(model, "fused", False):
                model.set_fused(False)
            H.set_transport(nxt[0])
            H.set_halo_mode(nxt[1])
            model.graph = None
            if graph_ok:
                model.capture()
            warm_load()
            elapsed = timed_region()
            H.check_transport()
            failed = post_valid
            post_valid = post_validate(field(), comm, log, on_gpu)
            post_valid["replaced"] = failed
    # 3. every non-fused run (N = 1 included): the same K steps from the saved
    #    starting state through a second compiled stencil variant, bitwise;
    #    a mismatch fails closed (no JSON line).
    stencil_post = None
    if pre and not getattr(model, "fused", False):
        PH.enter("post:stencil", _path_key(model), deadline=300)
        ORDER.append("stencil_post_check")
        stencil_post = stencil_post_check(model, comm, log, pre, warm["since_snapshot"] + args.steps, on_gpu,
                                          timed_steps=args.steps)
        if stencil_post["result"] != "ok":
            log(f"bench: post-timing stencil check failed ({stencil_post['result']}): no result")
            raise SystemExit(1)
    pre.clear()
    PH.enter("report", None, deadline=300)
    t_it = elapsed / args.steps
    per_gpu = model.a_eff_bytes / t_it / 1e9
    total = per_gpu * nprocs
    if getattr(model, "fused", False):
        model.sync_halo()
    finite = bool(torch.isfinite(field()).all().item())
    phase_ms = None
    if on_gpu and (not is2d and nprocs > 1 or args.loopback):
        # stencil vs halo split of a few eager steps (events on the stream)
        from igg.utils.trace import PhaseTimer

        model.timer = PhaseTimer()
        for _ in range(10):
            model.step()
        phase_ms = {k: v["mean_ms"] for k, v in model.timer.summary().items()}
        model.timer = None
    gather_ms = None
    if gather_every > 0:
        # two blocking gathers, both reported: the first after the timed
        # region may still pay one-time costs (staging chunks of the blocking
        # form, peer mappings), the second is the steady-state cost
        gather_ms = []
        for _ in range(2):
            sync()
            comm.barrier()
            tg = time.perf_counter()
            if getattr(model, "fused", False):
                model.sync_halo()
            igg.gather_(field(), A_global)
            sync()
            gather_ms.append(round(_max_over_ranks(comm, time.perf_counter() - tg) * 1e3, 3))
    if me == 0:
        out = {
            "metric": cfg["metric"] + VALUE_LABEL,
            "value": round(total, 3),
            "unit": "GB/s (aggregate over n_gpus)",
            "n_gpus": nprocs,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_it * 1e3, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(per_gpu / BASELINE_PER_GPU_GBS, 3) if args.config == "diffusion3d" else None,
            "dtype": "fp64" if dtype == torch.float64 else "fp32",
            "data": "synthetic (Gaussian-anomaly initial conditions, reference example physics)",
            "config": {
                "model": cfg["model"],
                "bench_config": args.config,
                "global_batch": nprocs,
                "seq_len": n,
                "parallelism": f"spatial {dims[0]}x{dims[1]}x{dims[2]}",
                "value_semantics": "whole-job aggregate T_eff = sum over the n_gpus GPUs (bench contract); "
                                   "per-GPU T_eff in t_eff_per_gpu_GBs",
                "device": args.device,
                "local_grid": [n, n] if is2d else [n, n, n],
                "global_grid": [int(v) for v in igg.get_global_grid().nxyz_g],
                "overlap_comm": bool(getattr(model, "overlap", False)),
                "gather_every": gather_every,
                "gather_ms": gather_ms,
                "gather_mode": args.gather_mode if gather_every > 0 else None,
                "phase_ms": phase_ms,
                "t_it_ms": round(t_it * 1e3, 5),
                "t_eff_per_gpu_GBs": round(per_gpu, 3),
                "t_eff_aggregate_GBs": round(total, 3),
                "a_eff_bytes_per_gpu": model.a_eff_bytes,
                "transport": H.transport_name(),
                "halo_schedule": (H.plan_mode(field()) if H.transport_name() != "put" else "put")
                if nprocs > 1 or args.loopback else None,
                "halo_mode_measured": H.tuned_modes() or None,
                "validation": valid if on_gpu else host_valid,
                "post_validation": post_valid,
                "stencil_post_check": stencil_post,
                "excluded": EXCL or None,
                "supervisor_attempt": (int(os.environ["IGG_SUP_ATTEMPT"]) if "IGG_SUP_ATTEMPT" in os.environ
                                       else None),
                "fused_post_check": fused_post,
                "transport_ab_ms": ab,
                "fused_halo": bool(getattr(model, "fused", False)),
                "fused_kernel": (({"variant": model.fused_variant, "mode": model.fused_mode,
                                   "grid_rounds": model.fused_rounds} if hasattr(model, "fused_variant")
                                  else {"acoustic": "fused staggered faces"})
                                 if getattr(model, "fused", False) else None),
                "stencil_grid_rounds": getattr(model, "rounds", None),
                "stencil_halo_z": getattr(model, "halo_z", None),
                "fused_ab_ms": fused_ab,
                "field_placement": getattr(model, "placement", None),
                "stencil_variant": getattr(model, "variant", None),
                "stencil_variant_ms": getattr(model, "variant_times", None),
                "finite": finite,
                "warmup_steps_run": args.warmup + (warm["extra"] or 0),
                "efficiency": eff,
                "stage_order": list(ORDER),
                "ab_wall_s": round(AB_BUDGET.elapsed_at_end, 2) if AB_BUDGET is not None else None,
                "ab_budget_s": AB_BUDGET.seconds if AB_BUDGET is not None else None,
                "ab_skipped_for_budget": (AB_BUDGET.skipped or None) if AB_BUDGET is not None else None,
                "wall_s": round(time.monotonic() - T_START, 2),
                "loopback_emulation": bool(args.loopback),
                "self_launched": os.environ.get("IGG_BENCH_SELF_LAUNCHED") == "1",
                "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                "hip_graph": timed_graph[0],
                "hip_graph_error": graph_error,
                "timing_bracket": ("rccl all-reduce + stream event + synchronize" if _BRACKET["dev"] and nprocs > 1
                                   else ("host barrier + stream event + synchronize" if on_gpu else "host barrier")),
            },
        }
        print(json.dumps(out), flush=True)
    PH.printed()
    PH.enter("finalize", None, deadline=120)
    if hasattr(model, "close"):
        model.close()  # collective: unmap the fused exchange's peer arenas
    igg.finalize_global_grid()


if __name__ == "__main__":
    main()
