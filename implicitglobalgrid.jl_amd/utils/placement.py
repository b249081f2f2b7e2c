"""Field placement probe (round 6, profiles/r6_placement/NOTES.md).

An HBM-bound sweep over the same carve of fields runs at one of two speeds,
depending on which physical pages the allocator gave it:

* 512^3 f64 diffusion: 0.578 vs 0.603 ms/step;
* 1024^3 f32 diffusion: 2.42 vs 2.54 ms;
* 8192^2 f32 acoustic: 0.282 vs 0.300 ms.

This holds for torch, fine-grained and VMM memory alike. An allocation keeps
its speed for its lifetime, and its virtual address does not predict the
speed. Slow allocations come in runs by allocation order: the first 4-7 of a
fresh process's carves were slow on some boxes, 0-2 on others.

So a model allocates ``CANDIDATES`` carves side by side, times a short
ping-pong sweep of its own kernel on each, keeps the fastest and frees the
rest. If all of them are alike (within ``SPREAD``) it cannot tell a box of
only slow pages from one of only fast pages, so it allocates more, another
batch at a time, up to ``MAX_CANDIDATES`` or ``MEMORY_SHARE`` of the free device
memory, and
stops as soon as a batch shows two speeds. ``IGG_FIELD_PLACEMENT=<k>`` probes
exactly k candidates; ``1`` turns the probe off. The probe is also off in
three cases:

* fields under ``MIN_FIELD_BYTES``;
* ranks that share a GPU: their probes would time each other;
* candidates that would not fit in ``MEMORY_SHARE`` of the free device memory.

The reference has no counterpart: Julia arrays are allocated once by the
application (examples/diffusion3D_multigpu_CuArrays_novis.jl:24-31).
"""
from __future__ import annotations

import os

import torch

CANDIDATES = 16
MAX_CANDIDATES = 64
SPREAD = 1.025  # fast and slow carves differ by 4.5-6 %; the noise of one probe is < 0.5 %
MIN_FIELD_BYTES = 256 << 20
# Share of the free device memory the candidates may hold while they are
# timed (all but the chosen one are freed before the model allocates anything
# else): 1024^3 f32 carves are 12 GiB, so on a 288 GB GPU this allows 16.
MEMORY_SHARE = 0.75


def candidate_count(gg, field_bytes: int, carve_bytes: int, device):
    """``(batch, limit)``: candidate carves per probe batch and in total
    (``(1, 1)`` = no probe). Collective on a multi-rank grid: every rank must
    call it at the same point with the same environment."""
    env = os.environ.get("IGG_FIELD_PLACEMENT")
    k = int(env) if env is not None else CANDIDATES
    if k <= 1 or torch.device(device).type != "cuda" or field_bytes < MIN_FIELD_BYTES:
        return 1, 1
    if int(gg.nprocs) > 1:
        from ..parallel.transport_select import _shared_device

        if _shared_device(gg.comm):
            return 1, 1
    free, _ = torch.cuda.mem_get_info(device)
    fit = max(1, int(free * MEMORY_SHARE) // max(1, carve_bytes))
    limit = min(fit, k if env is not None else MAX_CANDIDATES)
    return min(k, limit), limit


def time_candidates(cands, launch, steps: int = 6, rounds: int = 3, warm: int = 2) -> list:
    """Median ms per step of each candidate. ``launch(cand, j)`` enqueues
    ping-pong step ``j`` on the current stream. Rounds are interleaved over
    the candidates, so a drifting clock affects all of them alike."""
    s = torch.cuda.current_stream()
    for c in cands:
        for j in range(warm):
            launch(c, j)
    times = [[] for _ in cands]
    for _ in range(rounds):
        for i, c in enumerate(cands):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for j in range(steps):
                launch(c, j)
            e1.record(s)
            e1.synchronize()
            times[i].append(e0.elapsed_time(e1) / steps)
    return [sorted(t)[len(t) // 2] for t in times]


def placed(carve, count, timer):
    """``(fields, record)``: the fastest of the carves from ``carve()`` by
    ``timer(cands) -> [ms]``. ``count`` is ``(batch, limit)`` from
    ``candidate_count`` (or an int: one batch). Later batches are timed
    together with the best so far, so every decision compares times from one
    run. The other carves are released when this returns. ``record`` is
    ``{"candidates", "batches", "ms", "chosen"}``, or None without a probe."""
    batch, limit = (count, count) if isinstance(count, int) else count
    if batch <= 1:
        return carve(), None
    cands, ms, batches = [], [], 0
    while True:
        new = [carve() for _ in range(min(batch, limit - len(cands)))]
        if cands:
            best = min(range(len(ms)), key=lambda i: ms[i])
            t = timer([cands[best]] + new)
            ms[best] = t[0]
            ms += t[1:]
        else:
            ms = list(timer(new))
        cands += new
        batches += 1
        if max(ms) >= SPREAD * min(ms) or len(cands) >= limit:
            break
    best = min(range(len(ms)), key=lambda i: ms[i])
    return cands[best], {"candidates": len(cands), "batches": batches, "ms": [round(t, 5) for t in ms],
                         "chosen": best}
