"""Device selection (reference: src/select_device.jl:15-38).

The node-local rank (``LOCAL_RANK`` from the launcher, or hostname grouping
over the gloo group — the ``MPI.Comm_split_type(COMM_TYPE_SHARED)``
equivalent) selects the MI355X of this process. Device ids are 0-based (HIP).
"""
from __future__ import annotations

import torch

from .._native import IGGError, native
from . import grid as _grid


def select_device() -> int:
    """Select the GPU of the node-local rank and return its (0-based) id."""
    if _grid.cuda_enabled() or _grid.amdgpu_enabled():
        _grid.check_initialized()
        if _grid.cuda_enabled():
            raise IGGError("CUDA devices are not supported by this framework (MI355X/HIP only).")
        nb_devices = native.device_count()
        c = _grid.comm()
        if c.local_size > nb_devices:
            raise IGGError("More processes have been launched per node than there are GPUs available.")
        device_id = c.local_rank
        torch.cuda.set_device(device_id)
        native.set_device(device_id)
        return device_id
    raise IGGError(
        "Cannot select a device because neither CUDA nor AMDGPU is enabled (possibly detected non functional "
        "when the ImplicitGlobalGrid module was loaded)."
    )


_select_device = select_device
