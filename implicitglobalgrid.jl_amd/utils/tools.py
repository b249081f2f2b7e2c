"""Global sizes, global coordinates and timing (reference: src/tools.jl).

``x_g(ix, dx, A)`` keeps the reference's 1-based ``ix`` (so the reference
doctests and test vectors carry over verbatim); ``coords_g`` returns all
coordinates of an axis as a tensor (vectorised, same fp64 operation order as
``x_g`` so both agree bitwise; used to build initial conditions on the device).
"""
from __future__ import annotations

import time

import torch

from ..parallel import comm as _comm
from ..parallel import grid as _grid


def _size(A, dim0: int) -> int:
    return int(A.shape[dim0]) if A.dim() > dim0 else 1


def nx_g(A=None) -> int:
    """Global grid size in x; with ``A``, the global size of array ``A``."""
    gg = _grid.global_grid()
    return int(gg.nxyz_g[0]) if A is None else int(gg.nxyz_g[0] + (_size(A, 0) - gg.nxyz[0]))


def ny_g(A=None) -> int:
    """Global grid size in y; with ``A``, the global size of array ``A`` (tools.jl:3-59)."""
    gg = _grid.global_grid()
    return int(gg.nxyz_g[1]) if A is None else int(gg.nxyz_g[1] + (_size(A, 1) - gg.nxyz[1]))


def nz_g(A=None) -> int:
    """Global grid size in z; with ``A``, the global size of array ``A`` (tools.jl:3-59)."""
    gg = _grid.global_grid()
    return int(gg.nxyz_g[2]) if A is None else int(gg.nxyz_g[2] + (_size(A, 2) - gg.nxyz[2]))


def _coord(i: int, d: float, A, dim0: int) -> float:
    gg = _grid.global_grid()
    n = int(gg.nxyz[dim0])
    x0 = 0.5 * (n - _size(A, dim0)) * d
    x = (int(gg.coords[dim0]) * (n - int(gg.overlaps[dim0])) + i - 1) * d + x0
    if bool(gg.periods[dim0]):
        ng = int(gg.nxyz_g[dim0])
        x = x - d
        if x > (ng - 1) * d:
            x = x - ng * d
        if x < 0:
            x = x + ng * d
    return x


def x_g(ix: int, dx: float, A) -> float:
    """Global x-coordinate of element ``ix`` (1-based) of the local array ``A``."""
    return _coord(ix, dx, A, 0)


def y_g(iy: int, dy: float, A) -> float:
    """Global y-coordinate of element ``iy`` (1-based) of the local array ``A`` (tools.jl:146-155)."""
    return _coord(iy, dy, A, 1)


def z_g(iz: int, dz: float, A) -> float:
    """Global z-coordinate of element ``iz`` (1-based) of the local array ``A`` (tools.jl:194-203)."""
    return _coord(iz, dz, A, 2)


def coords_g(dim0: int, d: float, A, *, dtype=torch.float64, device=None) -> torch.Tensor:
    """All global coordinates of axis ``dim0`` (0-based) of ``A`` as a 1-D tensor."""
    gg = _grid.global_grid()
    m = _size(A, dim0)
    n = int(gg.nxyz[dim0])
    x0 = 0.5 * (n - m) * d
    base = int(gg.coords[dim0]) * (n - int(gg.overlaps[dim0]))
    x = (torch.arange(m, dtype=torch.float64) + float(base)) * d + x0  # (base + i - 1) * d + x0, i 1-based
    if bool(gg.periods[dim0]):
        ng = int(gg.nxyz_g[dim0])
        x = x - d
        x = torch.where(x > (ng - 1) * d, x - ng * d, x)
        x = torch.where(x < 0, x + ng * d, x)
    return x.to(dtype=dtype, device=device if device is not None else A.device)


# --- timing (tools.jl:205-236) -------------------------------------------------
_t0 = None


def _sync_all() -> None:
    gg = _grid.global_grid()
    if gg.amdgpu_enabled and torch.cuda.is_available():
        # bounded (IGG_COMM_TIMEOUT): aborts RCCL and raises instead of hanging
        _comm.bounded_device_sync(what="tic/toc", comm=gg.comm)
    gg.comm.barrier()


def tic() -> float:
    """Start the chronometer once all processes reached this point (GPU drained)."""
    global _t0
    _sync_all()
    _t0 = time.perf_counter()
    return _t0


def toc() -> float:
    """Seconds since ``tic()`` once all processes reached this point (GPU drained)."""
    _sync_all()
    return time.perf_counter() - _t0


def init_timing_functions() -> None:
    tic()
    toc()
