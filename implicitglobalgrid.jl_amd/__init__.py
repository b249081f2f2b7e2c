"""MI355X-native implicit global grid (capabilities of ImplicitGlobalGrid.jl).

Distributed stencil computing on regular, optionally staggered 1-D/2-D/3-D
grids: write a single-device solver on a *local* grid; ``init_global_grid``
builds a Cartesian process topology (one process per MI355X) and the *global*
grid follows implicitly; ``update_halo_`` exchanges one-plane halos (RCCL over
xGMI, HIP pack/unpack kernels); ``gather_`` assembles the global array on a
root rank.

Public API (reference names in parentheses, src/ImplicitGlobalGrid.jl:9-23):
``init_global_grid``, ``finalize_global_grid``, ``update_halo_``
(``update_halo!``), ``gather_`` (``gather!``), ``select_device``, ``nx_g``,
``ny_g``, ``nz_g``, ``x_g``, ``y_g``, ``z_g``, ``tic``, ``toc`` and
``get_global_grid``.
"""
from ._native import IGGError, PROC_NULL, native, native_path  # noqa: F401
from .parallel.grid import (  # noqa: F401
    GlobalGrid,
    finalize_global_grid,
    get_global_grid,
    global_grid,
    grid_is_initialized,
    init_global_grid,
)
from .parallel.device import select_device  # noqa: F401
from .parallel.halo import update_halo, update_halo_  # noqa: F401
from .parallel.transport_select import select_transport  # noqa: F401
from .parallel.gather import gather, gather_, gather_async_  # noqa: F401
from .utils.tools import coords_g, nx_g, ny_g, nz_g, tic, toc, x_g, y_g, z_g  # noqa: F401
from .utils.checkpoint import load_checkpoint, save_checkpoint  # noqa: F401

__version__ = "0.1.0"

__all__ = [
    "init_global_grid", "finalize_global_grid", "update_halo_", "update_halo", "gather_", "gather",
    "select_device", "nx_g", "ny_g", "nz_g", "x_g", "y_g", "z_g", "tic", "toc", "get_global_grid",
    "IGGError", "coords_g", "gather_async_", "save_checkpoint", "load_checkpoint", "select_transport",
]
