"""Global grid state, ``init_global_grid`` and ``finalize_global_grid``.

Reference: src/shared.jl:46-111 (GlobalGrid struct, singleton, accessors),
src/init_global_grid.jl:40-105 and src/finalize_global_grid.jl:15-27.

The grid is a module-level singleton. Its array fields are mutable numpy
arrays, so — exactly as in the reference tests (test/test_tools.jl:116-166) — a
test may overwrite ``global_grid().dims`` / ``.coords`` / ``.nxyz_g`` in place
to simulate another topology in one process.
"""
from __future__ import annotations

import copy
from dataclasses import dataclass, field

import numpy as np

from .._native import NDIMS, NNEIGHBORS, PROC_NULL, IGGError, native
from ..utils import config
from . import comm as _comm

DEVICE_TYPE_AUTO = "auto"
DEVICE_TYPE_CUDA = "CUDA"
DEVICE_TYPE_AMDGPU = "AMDGPU"
DEVICE_TYPE_NONE = "none"  # extension: host (CPU) fields only, even on a GPU node
_DEVICE_TYPES = (DEVICE_TYPE_AUTO, DEVICE_TYPE_CUDA, DEVICE_TYPE_AMDGPU, DEVICE_TYPE_NONE)


def _i3(v=-1):
    return np.full(3, v, dtype=np.int64)


@dataclass
class GlobalGrid:
    """Mirror of the reference ``GlobalGrid`` (src/shared.jl:46-65)."""

    nxyz_g: np.ndarray = field(default_factory=_i3)
    nxyz: np.ndarray = field(default_factory=_i3)
    dims: np.ndarray = field(default_factory=_i3)
    overlaps: np.ndarray = field(default_factory=_i3)
    nprocs: int = -1
    me: int = -1
    coords: np.ndarray = field(default_factory=_i3)
    neighbors: np.ndarray = field(default_factory=lambda: np.full((NNEIGHBORS, NDIMS), -1, dtype=np.int64))
    periods: np.ndarray = field(default_factory=_i3)
    disp: int = -1
    reorder: int = -1
    comm: object = None
    cuda_enabled: bool = False
    amdgpu_enabled: bool = False
    cudaaware_MPI: list = field(default_factory=lambda: [False] * 3)
    amdgpuaware_MPI: list = field(default_factory=lambda: [False] * 3)
    loopvectorization: list = field(default_factory=lambda: [False] * 3)
    quiet: bool = False
    # MI355X runtime objects (not part of the reference struct)
    engine: object = field(default=None, repr=False)
    owns_runtime: bool = field(default=False, repr=False)

    def __deepcopy__(self, memo):
        # get_global_grid() returns a deep copy of the data; runtime handles
        # (communicator, engine) are shared, not copied.
        out = copy.copy(self)
        for k in ("nxyz_g", "nxyz", "dims", "overlaps", "coords", "neighbors", "periods"):
            setattr(out, k, getattr(self, k).copy())
        for k in ("cudaaware_MPI", "amdgpuaware_MPI", "loopvectorization"):
            setattr(out, k, list(getattr(self, k)))
        return out


GLOBAL_GRID_NULL = GlobalGrid()
_global_grid = GLOBAL_GRID_NULL


def grid_is_initialized() -> bool:
    return _global_grid.nprocs > 0


def check_initialized() -> None:
    if not grid_is_initialized():
        raise IGGError(
            "No function of the module can be called before init_global_grid() or after finalize_global_grid()."
        )


def global_grid() -> GlobalGrid:
    check_initialized()
    return _global_grid


def set_global_grid(gg: GlobalGrid) -> None:
    global _global_grid
    _global_grid = gg


def get_global_grid() -> GlobalGrid:
    """Return a deep copy of the global grid (shared.jl:79-80)."""
    return copy.deepcopy(_global_grid)


# --- accessors (shared.jl:87-111) -----------------------------------------
def me() -> int:
    return global_grid().me


def comm():
    return global_grid().comm


def ol(dim: int, A=None) -> int:
    """Overlap in ``dim`` (1-based); for an array, the effective overlap
    ``overlaps[dim] + size(A,dim) - nxyz[dim]`` (shared.jl:93-94)."""
    gg = global_grid()
    o = int(gg.overlaps[dim - 1])
    if A is None:
        return o
    return o + (_size(A, dim) - int(gg.nxyz[dim - 1]))


def _size(A, dim: int) -> int:
    return int(A.shape[dim - 1]) if A.dim() >= dim else 1


def neighbors(dim: int) -> np.ndarray:
    return global_grid().neighbors[:, dim - 1]


def neighbor(n: int, dim: int) -> int:
    return int(global_grid().neighbors[n - 1, dim - 1])


def has_neighbor(n: int, dim: int) -> bool:
    return neighbor(n, dim) != PROC_NULL


def amdgpu_enabled() -> bool:
    return global_grid().amdgpu_enabled


def cuda_enabled() -> bool:
    return global_grid().cuda_enabled


def amdgpu_functional() -> bool:
    """HIP device probe (reference: AMDGPU.functional(), shared.jl:10-23)."""
    return native.device_count() > 0


def cuda_functional() -> bool:
    return False  # no CUDA path on this framework


# --- lifecycle ----------------------------------------------------------------
def init_global_grid(
    nx: int,
    ny: int,
    nz: int,
    *,
    dimx: int = 0,
    dimy: int = 0,
    dimz: int = 0,
    periodx: int = 0,
    periody: int = 0,
    periodz: int = 0,
    overlapx: int = 2,
    overlapy: int = 2,
    overlapz: int = 2,
    disp: int = 1,
    reorder: int = 1,
    comm=None,
    init_MPI: bool = True,
    device_type: str = DEVICE_TYPE_AUTO,
    select_device: bool = True,
    quiet: bool = False,
):
    """Initialise the Cartesian process grid that implicitly defines the global grid.

    Returns ``(me, dims, nprocs, coords, comm_cart)`` like the reference
    (src/init_global_grid.jl:40-99). ``init_MPI`` controls the distributed
    runtime (torch.distributed + RCCL) instead of MPI; ``comm`` may be a
    ``torch.distributed`` process group. ``reorder`` is accepted and ignored
    (ranks map row-major onto Cartesian coordinates).
    """
    if grid_is_initialized():
        raise IGGError("The global grid has already been initialized.")
    nxyz = np.array([nx, ny, nz], dtype=np.int64)
    dims = np.array([dimx, dimy, dimz], dtype=np.int64)
    periods = np.array([periodx, periody, periodz], dtype=np.int64)
    overlaps = np.array([overlapx, overlapy, overlapz], dtype=np.int64)
    cudaaware = config.parse_aware_flags("CUDAAWARE_MPI")
    amdgpuaware = config.parse_aware_flags("ROCMAWARE_MPI")
    loopvect = config.parse_loopvectorization()
    if device_type == "HIP":
        device_type = DEVICE_TYPE_AMDGPU
    if device_type not in _DEVICE_TYPES:
        raise IGGError(
            f"Argument `device_type`: invalid value obtained ({device_type}). Valid values are: "
            f"{DEVICE_TYPE_CUDA}, {DEVICE_TYPE_AMDGPU}, {DEVICE_TYPE_AUTO}"
        )
    if device_type == DEVICE_TYPE_AUTO and cuda_functional() and amdgpu_functional():
        raise IGGError(
            "Automatic detection of the device type to be used not possible: both CUDA and AMDGPU are functional. "
            f"Set keyword argument `device_type` to {DEVICE_TYPE_CUDA} or {DEVICE_TYPE_AMDGPU}."
        )
    cuda_en = device_type in (DEVICE_TYPE_CUDA, DEVICE_TYPE_AUTO) and cuda_functional()
    amdgpu_en = device_type in (DEVICE_TYPE_AMDGPU, DEVICE_TYPE_AUTO) and amdgpu_functional()
    if nx == 1:
        raise IGGError("Invalid arguments: nx can never be 1.")
    if ny == 1 and nz > 1:
        raise IGGError("Invalid arguments: ny cannot be 1 if nz is greater than 1.")
    if np.any((nxyz == 1) & (dims > 1)):
        raise IGGError(
            "Incoherent arguments: if nx, ny, or nz is 1, then the corresponding dimx, dimy or dimz must not be set (or set 0 or 1)."
        )
    if np.any((nxyz < 2 * overlaps - 1) & (periods > 0)):
        raise IGGError(
            "Incoherent arguments: if nx, ny, or nz is smaller than 2*overlapx-1, 2*overlapy-1 or 2*overlapz-1, "
            "respectively, then the corresponding periodx, periody or periodz must not be set (or set 0)."
        )
    dims[(nxyz == 1) & (dims == 0)] = 1
    owns = False
    if init_MPI:
        if _comm.runtime_initialized():
            raise IGGError("MPI is already initialized. Set the argument 'init_MPI=false'.")
        _comm.init_runtime()
        owns = True
    elif not _comm.runtime_initialized():
        raise IGGError("MPI has not been initialized beforehand. Remove the argument 'init_MPI=false'.")
    cm = _comm.make_communicator(comm)
    nprocs = cm.size
    dims = np.array(native.dims_create(nprocs, dims.tolist()), dtype=np.int64)
    me_ = cm.rank
    coords = np.array(native.cart_coords(me_, dims.tolist()), dtype=np.int64)
    nbrs = np.full((NNEIGHBORS, NDIMS), PROC_NULL, dtype=np.int64)
    for d in range(NDIMS):
        nbrs[:, d] = native.cart_shift(me_, d, disp, dims.tolist(), periods.tolist())
    nxyz_g = dims * (nxyz - overlaps) + overlaps * (periods == 0)
    gg = GlobalGrid(
        nxyz_g=nxyz_g, nxyz=nxyz, dims=dims, overlaps=overlaps, nprocs=nprocs, me=me_, coords=coords,
        neighbors=nbrs, periods=periods, disp=disp, reorder=reorder, comm=cm, cuda_enabled=cuda_en,
        amdgpu_enabled=amdgpu_en, cudaaware_MPI=cudaaware, amdgpuaware_MPI=amdgpuaware,
        loopvectorization=loopvect, quiet=quiet, owns_runtime=owns,
    )
    set_global_grid(gg)
    if not quiet and me_ == 0:
        print(f"Global grid: {nxyz_g[0]}x{nxyz_g[1]}x{nxyz_g[2]} (nprocs: {nprocs}, dims: {dims[0]}x{dims[1]}x{dims[2]})")
    if (cuda_en or amdgpu_en) and select_device:
        from .device import select_device as _sel

        _sel()
    from . import halo as _halo

    _halo._init_engine(gg)
    from ..utils.tools import init_timing_functions

    init_timing_functions()
    return me_, dims, nprocs, coords, cm


def finalize_global_grid(*, finalize_MPI: bool = True) -> None:
    """Free buffers, release the communicators, optionally finalize the runtime
    (src/finalize_global_grid.jl:15-27)."""
    check_initialized()
    from . import gather as _gather
    from . import halo as _halo

    if finalize_MPI and not _comm.runtime_initialized():
        raise IGGError("MPI cannot be finalized as it has not been initialized. ")
    # A transport error (a put sync kernel that timed out, an asynchronous RCCL
    # failure) is reported AFTER everything is released: finalize must always
    # leave the grid reset, or neither a re-init nor a second finalize could
    # succeed and buffers / communicators would leak.
    transport_error = None
    try:
        _halo.check_transport()
    except IGGError as e:
        transport_error = e
    gg = _global_grid
    try:
        _gather.free_gather_buffer()
        _halo.free_update_halo_buffers()
        _halo._drop_engine()
        if gg.comm is not None:
            gg.comm.destroy()
        if finalize_MPI:
            _comm.finalize_runtime()
    finally:
        set_global_grid(GLOBAL_GRID_NULL)
        import gc

        gc.collect()  # the reference runs GC.gc() here (finalize_global_grid.jl:26)
        from .._native import native

        native.flush_deferred_frees()  # native field buffers released by the collection
    if transport_error is not None:
        raise transport_error
