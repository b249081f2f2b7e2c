"""Observability: roctx ranges and per-phase GPU timers.

* ``trace_range(name)`` — a roctx range (visible with ``rocprofv3
  --marker-trace``) when ``IGG_TRACE=1``; the native runtime also marks its own
  phases (``igg.update_halo``, ``igg.put.*``, ``igg.seq.*``, ``igg.onephase.*``,
  ``igg.diffusion3d``, ``igg.acoustic2d``, ``igg.gather``).
* ``PhaseTimer`` — hipEvent pairs around named phases of a time step on the
  current stream; ``summary()`` gives the mean GPU time per phase. Models
  accept one (``model.timer = PhaseTimer()``) to split stencil from halo time.
"""
from __future__ import annotations

import contextlib
from collections import defaultdict

import torch

from .._native import native


def tracing() -> bool:
    """Whether roctx ranges are emitted (IGG_TRACE / rocprofv3 marker tracing)."""
    return bool(native.trace_enabled())


@contextlib.contextmanager
def trace_range(name: str):
    """Context manager: a named roctx range around a block (no-op when tracing is off)."""
    on = native.trace_enabled()
    if on:
        native.trace_push(name)
    try:
        yield
    finally:
        if on:
            native.trace_pop()


class PhaseTimer:
    """Accumulates GPU time per phase; events are resolved lazily in summary()."""

    def __init__(self):
        self._pending = defaultdict(list)

    @contextlib.contextmanager
    def phase(self, name: str):
        if not torch.cuda.is_available():
            yield
            return
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        with trace_range(name):
            yield
        e1.record(s)
        self._pending[name].append((e0, e1))

    def summary(self) -> dict:
        """{phase: {"calls": k, "mean_ms": t}} (synchronises on the last events)."""
        out = {}
        for name, evs in self._pending.items():
            if not evs:
                continue
            evs[-1][1].synchronize()
            ts = [a.elapsed_time(b) for a, b in evs]
            out[name] = {"calls": len(ts), "mean_ms": round(sum(ts) / len(ts), 5)}
        return out

    def reset(self) -> None:
        self._pending.clear()
