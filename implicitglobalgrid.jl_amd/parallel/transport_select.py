"""Pick the device transport of ``update_halo_`` on the actual GPUs: every
candidate is checked bitwise against the host-staged exchange with a probe
payload, and the fastest checked one is kept.

The reference decides per dimension whether its MPI is GPU-aware from
environment flags (`IGG_ROCMAWARE_MPI_DIMX`..., src/init_global_grid.jl:51-68)
and trusts the answer. Here the device transports differ in speed by node
rank shape (RCCL p2p groups vs the IPC put transport: 1.098 vs 1.046 x the
plain step at a 2x2x2 corner rank, profiles/r5_update_halo/) and the put
transport's correctness rests on cross-device coherence of the node it runs
on. So the choice is measured on the node:

* ``select_transport(A)``: explicit library call (the same probe check
  ``bench.py`` runs before and after its timed region);
* ``auto_select(fields)``: what ``update_halo_`` runs by itself on the first
  eager device exchange of a field-set signature when ``IGG_TRANSPORT=auto``
  (the default): same check, probe shaped like the call's fields, winner cached
  per signature (parallel/halo.py).
"""
from __future__ import annotations

import math
import socket
import time
import warnings

import torch

from .._native import IGGError
from . import grid as _grid
from . import halo as _halo

DEFAULT_CANDIDATES = ("put", "rccl")


def _exact_limit(dtype: torch.dtype) -> int:
    """Integers 0..limit-1 are exact (and distinct) in ``dtype``."""
    if dtype.is_complex:
        dtype = {torch.complex32: torch.float16, torch.complex64: torch.float32}.get(dtype, torch.float64)
    if dtype == torch.bool:
        return 2
    if dtype.is_floating_point:  # 2 ** (mantissa bits + 1): eps = 2 ** -mantissa bits
        return 1 << (round(-math.log2(torch.finfo(dtype).eps)) + 1)
    return int(torch.iinfo(dtype).max) + 1


def _probe(A: torch.Tensor, rank: int, nranks: int = 1) -> torch.Tensor:
    """Rank-distinct payload of A's shape and dtype, boundary planes poisoned
    with 0: a missing, misplaced or wrong-rank receive changes the result.
    Rank r's values lie in [(r+1)*span, (r+2)*span), all exact and distinct in
    the dtype (float16: 2048 integers, bfloat16: 256, uint8: 256), so 0 is in
    no rank's range and neighbouring positions never round together."""
    n = A.numel()
    limit = min(_exact_limit(A.dtype), 1 << 53)
    span = max(1, min(n, 1 << 11, limit // (max(1, nranks) + 1)))
    v = (torch.arange(n, device=A.device, dtype=torch.int64) % span) + (rank + 1) * span
    X = v.to(A.dtype).view(A.shape).clone()
    for d in range(A.dim()):
        if A.shape[d] > 1:
            X.select(d, 0).fill_(0)
            X.select(d, A.shape[d] - 1).fill_(0)
    return X


def _agree_max(comm, v: float) -> float:
    return float(comm.allreduce(float(v), op="max")) if comm is not None and comm.size > 1 else float(v)


def _check_and_time(fields, names, switch, comm, rank: int, nranks: int, ref, steps: int,
                    skip: dict | None = None, compare: bool = True, rounds: int = 3,
                    reswitch=None) -> tuple[dict, dict]:
    """For each transport name: ``switch(name)`` (collective), one
    ``update_halo_`` of probes shaped like ``fields``, compared with ``ref``
    (the probes after the reference exchange; None: every candidate must equal
    the first one that passed; ``compare`` False: no comparison, the exchange
    must only complete). Then the ones that passed are timed in ``rounds``
    interleaved rounds of ``steps`` exchanges each (the MAX over ranks per
    round, the best round kept), so no candidate is favoured by running first
    or last. ``reswitch`` (default ``switch``) moves between the checked
    transports in those rounds (select_transport: without ending the
    schedule caches each time). Every outcome is agreed over ranks. Returns
    (checked, ms)."""
    checked, ms = {}, {}
    first_ok = None
    probes = {}
    for name in names:
        if skip and name in skip:
            checked[name] = skip[name]
            continue
        why = ""
        X = None
        try:
            switch(name)  # collective; creates the communicator / peer mesh
            X = [_probe(A, rank, nranks) for A in fields]
        except Exception as e:  # e.g. RCCL refuses ranks that share a GPU
            why = f"{type(e).__name__}: {e}"[:300]
        if _agree_max(comm, 1.0 if why else 0.0) == 0:  # every rank has its probes: exchange
            try:
                _halo.update_halo_(*X)
                torch.cuda.synchronize()
                _halo.check_transport()
                want = ref if ref is not None else first_ok
                if want is not None and compare:
                    for x, r in zip(X, want):
                        if not torch.equal(x, r):
                            bad = (x != r).nonzero()
                            why = f"mismatch in {bad.shape[0]} elements, first {bad[:4].tolist()}"
                            break
            except Exception as e:
                why = f"{type(e).__name__}: {e}"[:300]
            if _agree_max(comm, 1.0 if why else 0.0) > 0 and not why:
                why = "failed on another rank"
            if why:
                for m in _halo.meshes():
                    m.clear_error()  # a timed-out put sync leaves a sticky error word
        elif not why:
            why = "failed on another rank"
        checked[name] = why or "ok"
        if why:
            continue
        if ref is None and first_ok is None:
            first_ok = [x.clone() for x in X]
        # timed below on ONE probe set shared by the candidates (the caller's
        # fields stay untouched; probes per candidate would hold that many
        # field-sized copies, which ranks sharing a GPU ran out of memory on)
        if not probes:
            Xt = X
        probes[name] = True
        del X
    del first_ok
    n = max(1, int(steps))
    for _ in range(max(1, int(rounds))):
        for name in probes:
            X = Xt
            (reswitch or switch)(name)
            _halo.update_halo_(*X)  # warm: the switch may have left another transport's state behind
            torch.cuda.synchronize()
            if comm is not None:
                comm.barrier()
            t0 = time.perf_counter()
            for _ in range(n):
                _halo.update_halo_(*X)
            torch.cuda.synchronize()
            dt = _agree_max(comm, time.perf_counter() - t0)
            ms[name] = min(ms.get(name, float("inf")), round(dt / n * 1e3, 5))
    if probes:
        del X, Xt
    # the probes' memory back to the device (other processes may share it)
    torch.cuda.empty_cache()
    return checked, ms


def _shared_device(comm) -> bool:
    """Some ranks share a GPU (RCCL and torch's NCCL group refuse that). Collective."""
    me_dev = (socket.gethostname(), int(torch.cuda.current_device()))
    devs = comm.all_gather_object(me_dev)
    return len(set(devs)) < len(devs)


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
    An explicit choice: ``update_halo_`` no longer selects by itself
    (IGG_TRANSPORT=auto) afterwards. Raises IGGError if no candidate passes
    (the previous transport is then restored where it still works)."""
    gg = _grid.global_grid()
    _grid.check_initialized()
    out = {"checked": {}, "ms": {}, "chosen": _halo.transport_name()}
    if gg.nprocs == 1 or not gg.amdgpu_enabled or A.device.type != "cuda":
        out["reason"] = "single process or CPU field: update_halo_ has no device transport to choose"
        return out
    comm = gg.comm
    before = _halo.transport_name()
    shared = _shared_device(comm)
    with _halo.selecting():
        # reference: the host-staged exchange (the reference's non-GPU-aware path)
        _halo.set_transport("staged")
        R = _probe(A, int(gg.me), int(gg.nprocs))
        _halo.update_halo_(R)
        torch.cuda.synchronize()
        skip = {n: "skipped: ranks share a GPU (RCCL refuses duplicate devices)"
                for n in candidates if shared and n in ("rccl", "torch")}
        out["checked"], out["ms"] = _check_and_time([A], list(candidates), _halo.set_transport, comm, int(gg.me),
                                                    int(gg.nprocs), [R], steps, skip, reswitch=_halo.use_transport)
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


# auto_select: timed exchanges per candidate and round (3 interleaved rounds,
# each after one untimed warm-up exchange; the best round counts)
AUTO_STEPS = 5


def auto_select(fields) -> tuple[str, dict]:
    """IGG_TRANSPORT=auto: the device transport for this field set, chosen on
    the first eager device exchange of its signature (collective: every rank
    makes the same update_halo_ calls on the same local shapes).

    * ranks on several nodes: 'rccl' (IPC peer mappings need one node);
    * one node: 'put' and 'rccl' (not where ranks share a GPU: RCCL refuses
      duplicate devices) are each checked bitwise against the host-staged
      exchange of probes shaped like ``fields`` and timed; the fastest that
      passed wins. None passed: 'staged' (always correct, slow), with a warning;
    * loopback emulation (one process, every neighbour itself): 'put' and
      'rccl' loopback transports, checked against each other (there is no
      second rank for a host-staged reference; a one-sided emulated shape
      only times them, its halos being undefined) and timed; a disagreement
      keeps 'rccl', the loopback's former default.

    The caller's fields are not modified. Returns (name, record)."""
    gg = _grid.global_grid()
    rec = {"shapes": [tuple(A.shape) for A in fields], "dtype": str(fields[0].dtype), "checked": {}, "ms": {}}
    with _halo.selecting():
        if _halo.loopback_active():
            # a one-sided emulated shape (a node's edge / corner rank) reads
            # halos nobody wrote: its values are undefined by construction, so
            # the two loopback transports are only timed there
            one_sided = _halo.loopback_one_sided()
            rec["checked"], rec["ms"] = _check_and_time(fields, ["rccl", "put"], _halo.use_transport, None, 0, 1,
                                                        None, AUTO_STEPS, compare=not one_sided)
            if one_sided:
                rec["reason"] = "one-sided loopback emulation: timed only (its halos are undefined)"
            ok = [n for n in ("rccl", "put") if rec["checked"].get(n) == "ok"]
            if rec["checked"].get("put", "").startswith("mismatch"):
                warnings.warn(f"update_halo_ (IGG_TRANSPORT=auto, loopback): put and rccl disagree; keeping rccl "
                              f"({rec['checked']['put']})")
                ok = ["rccl"]
            name = min(ok, key=lambda n: rec["ms"][n]) if ok else "rccl"
        else:
            comm = gg.comm
            if not comm.one_node:
                rec["reason"] = "ranks on several nodes: IPC peer mappings need one node"
                name = "rccl"
            else:
                shared = _shared_device(comm)
                _halo.use_transport("staged")
                R = [_probe(A, int(gg.me), int(gg.nprocs)) for A in fields]
                _halo.update_halo_(*R)
                torch.cuda.synchronize()
                skip = {"rccl": "skipped: ranks share a GPU (RCCL refuses duplicate devices)"} if shared else None
                rec["checked"], rec["ms"] = _check_and_time(fields, list(DEFAULT_CANDIDATES), _halo.use_transport,
                                                            comm, int(gg.me), int(gg.nprocs), R, AUTO_STEPS, skip)
                del R
                ok = [n for n in DEFAULT_CANDIDATES if rec["checked"].get(n) == "ok"]
                if ok:
                    name = min(ok, key=lambda n: rec["ms"][n])
                else:
                    warnings.warn(f"update_halo_ (IGG_TRANSPORT=auto): no device transport passed the probe "
                                  f"exchange ({rec['checked']}); using the host-staged transport")
                    name = "staged"
        _halo.use_transport(name)
    rec["chosen"] = name
    return name, rec
