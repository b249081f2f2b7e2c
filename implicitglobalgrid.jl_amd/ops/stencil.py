"""Stencil operators backed by the native kernels (csrc/kernels/stencil_kernels.hip).

``diffusion3d_`` computes one explicit heat-diffusion update of the interior
(or of a list of boxes inside it) in a single fused pass:

    T2 = T + dt*lam/Cp * (d2T/dx2 + d2T/dy2 + d2T/dz2)

which is the five broadcast kernels of the reference example
(examples/diffusion3D_multigpu_CuArrays_novis.jl:42-46) fused, with no
temporaries. GPU tensors run the hand-written HIP kernel on the current stream;
CPU tensors run the threaded C++ host kernel.
"""
from __future__ import annotations

import os

import torch

from .._native import IGGError, native

_autotune_cache: dict = {}


def variants() -> list[str]:
    """Names of every variant index (measurement-only ones included)."""
    return list(native.diffusion3d_variants())


def compiled_variants() -> list[int]:
    """Variant indices compiled in this build (``build.py --probes`` adds the
    measurement-only tilings of rounds 1-2)."""
    return [v for v in range(len(variants())) if native.diffusion3d_variant_compiled(v)]


FUSED_VARIANTS = (0, 2, 9, 11, 14, 40, 41, 42, 44, 45, 48, 50)


def compiled_fused_variants() -> list[int]:
    """Fused-exchange variants compiled in this build."""
    return [v for v in FUSED_VARIANTS if native.diffusion3d_fused_variant_ok(v)]


def _check(T2, T, Cp):
    for name, A in (("T2", T2), ("T", T), ("Cp", Cp)):
        if A.dim() != 3:
            raise IGGError(f"diffusion3d: {name} must be 3-D")
        if not A.is_contiguous():
            raise IGGError(f"diffusion3d: {name} must be C-contiguous")
        if A.shape != T.shape or A.dtype != T.dtype or A.device != T.device:
            raise IGGError("diffusion3d: T2, T and Cp must have identical shape, dtype and device")
    if T.dtype not in (torch.float32, torch.float64):
        raise IGGError("diffusion3d: only float32 and float64 are supported")
    if T2.data_ptr() == T.data_ptr():
        raise IGGError("diffusion3d: T2 must not alias T (use ping-pong buffers)")


def inner_box(shape) -> tuple:
    return ((1, 1, 1), tuple(int(s) - 1 for s in shape))


def _variant_for(T, boxes, rd2, dtlam, T2, Cp, stream) -> int:
    env = os.environ.get("IGG_STENCIL_VARIANT", "0").strip().lower()
    if env != "auto":
        return int(env)
    key = (tuple(T.shape), T.dtype, tuple(map(tuple, (b[0] for b in boxes))), tuple(map(tuple, (b[1] for b in boxes))))
    v = _autotune_cache.get(key)
    if v is None:
        v = autotune(T2, T, Cp, rd2, dtlam, boxes)
        _autotune_cache[key] = v
    return v


# The variants that won the autotune on some box in rounds 2-4 (the bench's
# 512^3 f64 / 1024^3 f32 configs, profiles/ and BENCH_r0*.json): 40, 24, 43,
# 11, 2 (f64), 14, 21, 26 (f32 and both). 21+: restrict-argument (fused-kernel)
# form; 40: lane-distributed z-segment edge loads at one workgroup per CU
# (profiles/r1_zl/); 43: full-row z tiles (profiles/r2_fullrow/). 0, 9, 23 and
# 25 never won a real config in rounds 2-4 (23/25 are --probes builds now).
# 44 (round 6): tiling 0 at 2 workgroups per CU (f32, profiles/r6_vsweep/).
SHORTLIST = (2, 11, 14, 21, 24, 26, 40, 43, 44)
# Grid residency rounds tried per variant by the model autotune: 1-4 measured
# best depending on the box and variant (profiles/r1_fused/grid.log,
# variant_sweep.log, r1_zl/: 1-2.5 %).
GRID_ROUNDS = (1, 2, 3, 4)


def _cand(c, halo_z: bool):
    """(variant, grid rounds, halo_z) of a candidate: a variant index, a
    (variant, rounds) pair or a (variant, rounds, halo_z) triple."""
    if isinstance(c, int):
        return c, 0, halo_z
    return (int(c[0]), int(c[1]), bool(c[2]) if len(c) > 2 else halo_z)


def time_variants(T2, T, Cp, rd2, dtlam, boxes, candidates=None, reps: int = 5, rounds: int = 3,
                  halo_z: bool = False) -> dict:
    """Median-of-rounds time (ms) of each candidate on these arrays, interleaved
    (the update is pure: T2 = f(T, Cp), so T2 can be scribbled). A candidate is
    a variant index, a (variant, grid_rounds) pair (grid residency rounds of
    the launch, see diffusion3d_) or a (variant, grid_rounds, halo_z) triple
    (``halo_z`` applies to the others)."""
    n = list(T.shape)
    cands = compiled_variants() if candidates is None else list(candidates)
    s = torch.cuda.current_stream()
    times = {c: [] for c in cands}

    def launch(c):
        v, gr, hz = _cand(c, halo_z)
        native.diffusion3d(T2.data_ptr(), T.data_ptr(), Cp.data_ptr(), n, rd2, dtlam, T.element_size(), boxes, True,
                           v, s.cuda_stream, gr, hz)

    for v in cands:  # warm every code object once
        launch(v)
    for _ in range(rounds):
        for v in cands:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(reps):
                launch(v)
            e1.record(s)
            e1.synchronize()
            times[v].append(e0.elapsed_time(e1) / reps)
    return {v: sorted(t)[len(t) // 2] for v, t in times.items()}


def time_variants_pingpong(T2, T, Cp, rd2, dtlam, boxes, candidates, steps: int = 10, rounds: int = 3,
                           halo_z: bool = False) -> dict:
    """Like ``time_variants`` but in the time loop's shape: ``steps`` (even)
    launches alternating T2 = f(T) and T = f(T2) on the model's own two
    buffers (their HBM placement alternates exactly as in the run). T is saved
    and restored around the measurement; T2's interior is scribbled (it is
    overwritten by the next step anyway)."""
    n = list(T.shape)
    s = torch.cuda.current_stream()
    times = {c: [] for c in candidates}
    backup = T.clone()

    def launch(c, dst, src):
        v, gr, hz = _cand(c, halo_z)
        native.diffusion3d(dst.data_ptr(), src.data_ptr(), Cp.data_ptr(), n, rd2, dtlam, T.element_size(), boxes,
                           True, v, s.cuda_stream, gr, hz)

    try:
        for c in candidates:
            launch(c, T2, T)
            launch(c, T, T2)
        for _ in range(rounds):
            for c in candidates:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for k in range(steps):
                    if k % 2 == 0:
                        launch(c, T2, T)
                    else:
                        launch(c, T, T2)
                e1.record(s)
                e1.synchronize()
                times[c].append(e0.elapsed_time(e1) / steps)
    finally:
        T.copy_(backup)
        torch.cuda.synchronize()
        del backup
    return {c: sorted(t)[len(t) // 2] for c, t in times.items()}


def autotune(T2, T, Cp, rd2, dtlam, boxes, reps: int = 5, candidates=None) -> int:
    """Fastest variant on these arrays (this process only)."""
    t = time_variants(T2, T, Cp, rd2, dtlam, boxes, candidates, reps)
    return min(t, key=t.get)


def diffusion3d_(T2, T, Cp, *, lam: float, dt: float, dx: float, dy: float, dz: float,
                 boxes=None, variant: int | None = None, stream: int | None = None, rounds: int = 0,
                 halo_z: bool = False) -> None:
    """One fused diffusion update of ``T2`` from ``T`` on ``boxes`` (default: whole interior).

    ``rounds`` sizes the grid of this launch: 0 = library default, k > 0 = k
    residency rounds (k x resident workgroups), k < 0 = |k| x 4096 workgroups.
    ``halo_z``: a box spanning the whole inner z range also writes ``T``'s values
    into ``T2``'s z halo elements (z = 0 and nz-1), so the z-edge stores are
    whole cache lines (5-7 % faster for 1024^3 f32, profiles/r4_halo_z/). Only
    where that is harmless: ``T2``'s z halo equals ``T``'s (fixed boundaries) or
    a halo update after the stencil rewrites it, and nothing writes ``T2``'s z
    halo concurrently. GPU only (the host kernel ignores it).
    """
    _check(T2, T, Cp)
    rd2 = [1.0 / (dx * dx), 1.0 / (dy * dy), 1.0 / (dz * dz)]
    dtlam = dt * lam
    if boxes is None:
        boxes = [inner_box(T.shape)]
    boxes = [(list(b[0]), list(b[1])) for b in boxes]
    dev = T.is_cuda
    if dev:
        s = torch.cuda.current_stream().cuda_stream if stream is None else stream
        v = _variant_for(T, boxes, rd2, dtlam, T2, Cp, s) if variant is None else variant
    else:
        s, v = 0, 0
    native.diffusion3d(T2.data_ptr(), T.data_ptr(), Cp.data_ptr(), list(T.shape), rd2, dtlam,
                       T.element_size(), boxes, dev, v, s, rounds, bool(halo_z) and dev)


def diffusion3d_reference(T, Cp, *, lam, dt, dx, dy, dz) -> torch.Tensor:
    """Plain-PyTorch (fp64) reference of the reference example's 5 broadcasts."""
    T = T.double()
    Cp = Cp.double()
    qx = -lam * (T[1:, 1:-1, 1:-1] - T[:-1, 1:-1, 1:-1]) / dx
    qy = -lam * (T[1:-1, 1:, 1:-1] - T[1:-1, :-1, 1:-1]) / dy
    qz = -lam * (T[1:-1, 1:-1, 1:] - T[1:-1, 1:-1, :-1]) / dz
    dTedt = 1.0 / Cp[1:-1, 1:-1, 1:-1] * (
        -(qx[1:] - qx[:-1]) / dx - (qy[:, 1:] - qy[:, :-1]) / dy - (qz[:, :, 1:] - qz[:, :, :-1]) / dz)
    out = T.clone()
    out[1:-1, 1:-1, 1:-1] = T[1:-1, 1:-1, 1:-1] + dt * dTedt
    return out


def split_boundary(shape, active, widths):
    """Boundary slabs + interior box of the inner region (see csrc/stencil_host.cpp).

    ``active[d]`` is a bool (both sides) or a (left, right) pair of bools.
    """
    act = [[bool(a), bool(a)] if isinstance(a, (bool, int)) else [bool(a[0]), bool(a[1])] for a in active]
    slabs, interior = native.split_boundary(list(shape), act, list(widths))
    return slabs, interior
