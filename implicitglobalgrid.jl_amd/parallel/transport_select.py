"""Pick the device transport of ``update_halo_`` on the actual GPUs: every
candidate is checked bitwise against the host-staged exchange with a probe
payload, and the fastest checked one is kept.

The reference decides per dimension whether its MPI is GPU-aware from
environment flags (`IGG_ROCMAWARE_MPI_DIMX`..., src/init_global_grid.jl:51-68)
and trusts the answer. Here the device transports differ in speed by node
rank shape (RCCL p2p groups vs the IPC put transport: 1.098 vs 1.046 x the
plain step at a 2x2x2 corner rank, profiles/r5_update_halo/) and the put
transport's correctness rests on cross-device coherence of the node it runs
on. So ``select_transport`` measures both on the node: the same probe check
``bench.py`` runs before and after its timed region, as a library call.
"""
from __future__ import annotations

import socket
import time

import torch

from .._native import IGGError
from . import grid as _grid
from . import halo as _halo

DEFAULT_CANDIDATES = ("put", "rccl")


def _probe(A: torch.Tensor, rank: int) -> torch.Tensor:
    """Rank-distinct payload of A's shape and dtype, exact in every dtype the
    halo engine moves (integer-valued and small), boundary planes poisoned:
    a missing, misplaced or wrong-rank receive changes the result."""
    n = A.numel()
    span = max(2, min(n, 1 << 11))
    v = (torch.arange(n, device=A.device, dtype=torch.int64) % span) + (rank + 1) * span
    X = v.to(A.dtype).view(A.shape).clone()
    for d in range(A.dim()):
        if A.shape[d] > 1:
            X.select(d, 0).fill_(-7)
            X.select(d, A.shape[d] - 1).fill_(-7)
    return X


def _agree_max(comm, v: float) -> float:
    return float(comm.allreduce(float(v), op="max")) if comm.size > 1 else float(v)


def select_transport(A: torch.Tensor, candidates=DEFAULT_CANDIDATES, steps: int = 10,
                     keep_fastest: bool = True) -> dict:
    """Check each device transport in ``candidates`` ('put', 'rccl', 'torch')
    with ``update_halo_`` of a probe shaped like ``A`` against the host-staged
    exchange, bitwise; time ``steps`` exchanges of each checked one (the MAX
    over ranks); switch ``update_halo_`` to the fastest (``keep_fastest``).

    Collective: every rank calls it at the same point, with the same
    ``candidates``, and every decision is agreed over ranks (a candidate that
    fails on one rank - no IPC mapping, an RCCL bootstrap error, a mismatch -
    fails on all). ``A`` itself is not modified; two probes of its size are
    allocated while this runs. Returns ``{"checked": {name: "ok" | reason},
    "ms": {name: ms per exchange}, "chosen": name}``; on a single-process or
    CPU grid nothing is switched and ``chosen`` is the current transport.
    Raises IGGError if no candidate passes (the previous transport is then
    restored where it still works)."""
    gg = _grid.global_grid()
    _grid.check_initialized()
    out = {"checked": {}, "ms": {}, "chosen": _halo.transport_name()}
    if gg.nprocs == 1 or not gg.amdgpu_enabled or A.device.type != "cuda":
        out["reason"] = "single process or CPU field: update_halo_ has no device transport to choose"
        return out
    comm = gg.comm
    before = _halo.transport_name()
    # RCCL (and torch's NCCL group) refuse ranks that share a device
    me_dev = (socket.gethostname(), int(torch.cuda.current_device()))
    devs = comm.all_gather_object(me_dev)
    shared = len(set(devs)) < len(devs)
    # reference: the host-staged exchange (the reference's non-GPU-aware path)
    _halo.set_transport("staged")
    R = _probe(A, int(gg.me))
    _halo.update_halo_(R)
    torch.cuda.synchronize()
    for name in candidates:
        why = ""
        X = None
        if shared and name in ("rccl", "torch"):
            out["checked"][name] = "skipped: ranks share a GPU (RCCL refuses duplicate devices)"
            continue
        try:
            _halo.set_transport(name)  # collective; creates the communicator / peer mesh
            X = _probe(A, int(gg.me))
        except Exception as e:  # e.g. RCCL refuses ranks that share a GPU
            why = f"{type(e).__name__}: {e}"[:300]
        if _agree_max(comm, 1.0 if why else 0.0) == 0:  # every rank has its probe: exchange
            try:
                _halo.update_halo_(X)
                torch.cuda.synchronize()
                _halo.check_transport()
                if not torch.equal(X, R):
                    bad = (X != R).nonzero()
                    why = f"mismatch in {bad.shape[0]} elements, first {bad[:4].tolist()}"
            except Exception as e:
                why = f"{type(e).__name__}: {e}"[:300]
            if _agree_max(comm, 1.0 if why else 0.0) > 0 and not why:
                why = "failed on another rank"
            if why and getattr(comm, "mesh", None) is not None:
                comm.mesh.clear_error()  # a timed-out put sync leaves a sticky error word
        elif not why:
            why = "failed on another rank"
        out["checked"][name] = why or "ok"
        if why:
            continue
        # timing: the probe again (A stays untouched), MAX over ranks
        _halo.update_halo_(X)
        torch.cuda.synchronize()
        comm.barrier()
        t0 = time.perf_counter()
        for _ in range(max(1, int(steps))):
            _halo.update_halo_(X)
        torch.cuda.synchronize()
        dt = _agree_max(comm, time.perf_counter() - t0)
        out["ms"][name] = round(dt / max(1, int(steps)) * 1e3, 5)
        del X
    del R
    ok = [n for n in candidates if out["checked"].get(n) == "ok"]
    if not ok:
        try:
            _halo.set_transport(before)
        except Exception:
            pass
        raise IGGError(f"select_transport: no candidate passed the probe exchange: {out['checked']}")
    best = min(ok, key=lambda n: out["ms"][n]) if keep_fastest else ok[0]
    _halo.set_transport(best)
    out["chosen"] = _halo.transport_name()
    return out
