"""Configuration from environment variables.

Reference flags (src/init_global_grid.jl:51-68, module docs
src/ImplicitGlobalGrid.jl:26-33) are parsed with the reference's precedence
rules and stored on the grid:

* ``IGG_ROCMAWARE_MPI`` / ``IGG_CUDAAWARE_MPI`` set all three dims; the per-dim
  ``*_DIMX/_DIMY/_DIMZ`` variants are only honoured if the global variable left
  every dim false.
* ``IGG_LOOPVECTORIZATION`` sets all dims; per-dim variants are only honoured if
  the global variable set every dim true (they can only *disable* dims).

On MI355X device data always moves device-resident (RCCL), so the "aware" flags
are informational; ``loopvectorization[d]`` selects the threaded host copy for
CPU fields in dim ``d`` (default: on).

Framework knobs (new): ``IGG_TRANSPORT`` (``auto`` | ``put`` | ``rccl`` |
``torch`` | ``staged``) for GPU point-to-point: ``auto`` (default) checks
``put`` and ``rccl`` bitwise against the host-staged exchange on the first
eager device exchange of each field set and keeps the faster (``rccl`` across
nodes; parallel/transport_select.py); ``put`` = one-sided IPC stores over xGMI
(one node); ``rccl`` = grouped ncclSend/ncclRecv; ``staged`` = host-staged
gloo, the reference's non-GPU-aware path. Also ``IGG_STENCIL_VARIANT`` (int or
``auto``), ``IGG_DEBUG_SYNC`` (synchronise after every halo update), ``IGG_QUIET``.
"""
from __future__ import annotations

import os
from typing import Mapping


def _flag(env: Mapping[str, str], key: str) -> bool:
    return int(env[key]) > 0


def parse_aware_flags(prefix: str, env: Mapping[str, str] | None = None) -> list[bool]:
    """``IGG_<prefix>`` then per-dim overrides if the global left all dims false."""
    env = os.environ if env is None else env
    flags = [False, False, False]
    if f"IGG_{prefix}" in env:
        flags = [_flag(env, f"IGG_{prefix}")] * 3
    if not any(flags):
        for d, ax in enumerate("XYZ"):
            k = f"IGG_{prefix}_DIM{ax}"
            if k in env:
                flags[d] = _flag(env, k)
    return list(flags)


def parse_loopvectorization(env: Mapping[str, str] | None = None) -> list[bool]:
    """``IGG_LOOPVECTORIZATION``; per-dim variables only honoured if all dims true."""
    env = os.environ if env is None else env
    flags = [False, False, False]
    if "IGG_LOOPVECTORIZATION" in env:
        flags = [_flag(env, "IGG_LOOPVECTORIZATION")] * 3
    if all(flags):
        for d, ax in enumerate("XYZ"):
            k = f"IGG_LOOPVECTORIZATION_DIM{ax}"
            if k in env:
                flags[d] = _flag(env, k)
    return list(flags)


def transport_choice(env: Mapping[str, str] | None = None) -> str:
    env = os.environ if env is None else env
    t = env.get("IGG_TRANSPORT", "auto").strip().lower()
    if t not in ("auto", "rccl", "torch", "staged", "put"):
        raise ValueError(f"IGG_TRANSPORT must be 'auto', 'put', 'rccl', 'torch' or 'staged' (got {t!r})")
    return t


def halo_mode(env: Mapping[str, str] | None = None) -> str:
    """``IGG_HALO_MODE``: ``auto`` (default) | ``sequential`` | ``onephase``."""
    env = os.environ if env is None else env
    m = env.get("IGG_HALO_MODE", "auto").strip().lower()
    if m not in ("auto", "sequential", "onephase"):
        raise ValueError(f"IGG_HALO_MODE must be auto, sequential or onephase (got {m!r})")
    return m


PACK_MODES = ("kernel", "memcpy2d")


def pack_modes(env: Mapping[str, str] | None = None) -> list[str]:
    """``IGG_PACK`` sets all dims, ``IGG_PACK_DIMX/Y/Z`` override one dim:
    ``kernel`` (default, batched copy kernel) | ``memcpy2d`` (hipMemcpy2DAsync
    for faces with contiguous rows)."""
    env = os.environ if env is None else env
    modes = [env.get("IGG_PACK", "kernel").strip().lower()] * 3
    for d, ax in enumerate("XYZ"):
        k = f"IGG_PACK_DIM{ax}"
        if k in env:
            modes[d] = env[k].strip().lower()
    for m in modes:
        if m not in PACK_MODES:
            raise ValueError(f"IGG_PACK / IGG_PACK_DIM*: expected kernel or memcpy2d (got {m!r})")
    return modes


def debug_sync(env: Mapping[str, str] | None = None) -> bool:
    env = os.environ if env is None else env
    return env.get("IGG_DEBUG_SYNC", "0") not in ("", "0")


def poll_every(env: Mapping[str, str] | None = None) -> int:
    """``IGG_POLL_EVERY``: check the transports' asynchronous error state every
    N update_halo_ calls (default 1000, 0 = only at check_transport/finalize)."""
    env = os.environ if env is None else env
    return int(env.get("IGG_POLL_EVERY", "1000"))


def comm_timeout(env: Mapping[str, str] | None = None) -> float:
    """``IGG_COMM_TIMEOUT``: seconds a host-side wait (barrier, tic/toc, eager
    RCCL exchange) may block before the communicators are aborted and every
    rank raises (default 300)."""
    env = os.environ if env is None else env
    return float(env.get("IGG_COMM_TIMEOUT", "300"))


def gather_pull(env: Mapping[str, str] | None = None) -> bool:
    """IGG_GATHER_PULL (default 1): GPU ``gather_`` on a single node pulls every
    block with the root's copy engines straight into ``A_global`` (no staging
    buffer of nprocs*|A|, no reorder pass); 0 = RCCL receives + reorder kernel."""
    env = os.environ if env is None else env
    return env.get("IGG_GATHER_PULL", "1").strip() not in ("0", "false", "no")


def first_contact_timeout(env: Mapping[str, str] | None = None) -> float:
    """``IGG_FIRST_CONTACT_TIMEOUT``: seconds a first-contact call of the
    multi-GPU path may take - the RCCL bootstrap, mapping a peer's memory over
    IPC (default 120). On expiry the call is abandoned and every rank raises
    together (csrc/include/igg/fault.hpp)."""
    env = os.environ if env is None else env
    return float(env.get("IGG_FIRST_CONTACT_TIMEOUT", "120"))


def host_matching(env: Mapping[str, str] | None = None) -> str:
    """``IGG_HOST_MATCHING``: how the host (gloo) paths pair messages.
    ``ordered`` (default): order-only, like RCCL and the reference's tag-0 MPI
    messages - one message per peer and phase, paired by issue position;
    ``tagged``: one message per halo face, paired by a per-face tag."""
    env = os.environ if env is None else env
    m = env.get("IGG_HOST_MATCHING", "ordered").strip().lower()
    if m not in ("ordered", "tagged"):
        raise ValueError(f"IGG_HOST_MATCHING must be 'ordered' or 'tagged' (got {m!r})")
    return m
