"""Per-rank checkpoint / restart of distributed fields.

The reference has no checkpointing: ``gather!`` is its only way to collect the
global state and applications save the gathered array themselves
(src/gather.jl:25-65). Gathering 8 x 4 GiB to one rank for a
restart file is the wrong shape on an MI355X node, so here every rank writes
its own local block (halos included) next to a small JSON manifest that
records the implicit global grid it belongs to. A restart validates the
topology (dims, local sizes, overlaps, periodicity, this rank's coordinates)
before loading, so a checkpoint cannot silently be applied to a different
decomposition. Files are ``safetensors`` (no pickle: nothing in a checkpoint
executes on load).

    save_checkpoint("run/ckpt", step=it, T=T, Cp=Cp)      # collective
    meta, fields = load_checkpoint("run/ckpt")             # collective
"""
from __future__ import annotations

import json
import os

import torch

from .._native import IGGError
from ..parallel import grid as _grid

_FORMAT = 1


def _grid_meta() -> dict:
    gg = _grid.global_grid()
    return {
        "format": _FORMAT,
        "nprocs": int(gg.nprocs),
        "dims": [int(v) for v in gg.dims],
        "nxyz": [int(v) for v in gg.nxyz],
        "nxyz_g": [int(v) for v in gg.nxyz_g],
        "overlaps": [int(v) for v in gg.overlaps],
        "periods": [int(v) for v in gg.periods],
    }


def _rank_file(prefix: str, me: int) -> str:
    return f"{prefix}.rank{me:05d}.safetensors"


def save_checkpoint(prefix: str, step: int = 0, **fields: torch.Tensor) -> str:
    """Write this rank's ``fields`` (local blocks, any device) to
    ``<prefix>.rankNNNNN.safetensors``; rank 0 writes ``<prefix>.json``.
    Collective: every rank calls it with the same field names; returns the
    rank's file name once all ranks have written theirs."""
    from safetensors.torch import save_file

    _grid.check_initialized()
    gg = _grid.global_grid()
    me = int(gg.me)
    if not fields:
        raise IGGError("save_checkpoint: no fields given")
    d = os.path.dirname(os.path.abspath(prefix))
    os.makedirs(d, exist_ok=True)
    meta = _grid_meta()
    meta["step"] = int(step)
    meta["fields"] = {k: {"shape": list(v.shape), "dtype": str(v.dtype).replace("torch.", "")}
                      for k, v in sorted(fields.items())}
    tensors = {k: v.detach().contiguous().cpu() for k, v in fields.items()}
    local = {"coords": json.dumps([int(c) for c in gg.coords]), "step": str(int(step))}
    path = _rank_file(prefix, me)
    tmp = path + ".tmp"
    err = ""
    try:
        save_file(tensors, tmp, metadata=local)
        os.replace(tmp, path)  # a crash mid-write never leaves a truncated checkpoint under the final name
    except Exception as e:  # reported collectively below, so no rank waits forever
        err = f"{type(e).__name__}: {e}"
    # The manifest names the step only once EVERY rank has its block on disk:
    # a crash before this point leaves the previous manifest (and a step check
    # in load_checkpoint catches a block that was not rewritten).
    errs = gg.comm.all_gather_object(err) if gg.comm is not None else [err]
    bad = [(r, e) for r, e in enumerate(errs) if e]
    if bad:
        raise IGGError(f"save_checkpoint: rank {bad[0][0]} failed to write its block: {bad[0][1]}")
    if me == 0:
        with open(prefix + ".json.tmp", "w") as f:
            json.dump(meta, f, indent=1, sort_keys=True)
        os.replace(prefix + ".json.tmp", prefix + ".json")
    if gg.comm is not None:
        gg.comm.barrier()
    return path


def load_checkpoint(prefix: str, device=None) -> tuple[dict, dict]:
    """Read this rank's block of a checkpoint written by ``save_checkpoint``
    on the same decomposition. Returns ``(meta, {name: tensor})`` with tensors
    on ``device`` (default: the grid's GPU if it was initialised for GPUs,
    else CPU). Raises IGGError on any topology or field mismatch."""
    from safetensors import safe_open

    _grid.check_initialized()
    gg = _grid.global_grid()
    me = int(gg.me)
    try:
        with open(prefix + ".json") as f:
            meta = json.load(f)
    except FileNotFoundError:
        raise IGGError(f"load_checkpoint: no manifest {prefix}.json") from None
    if meta.get("format") != _FORMAT:
        raise IGGError(f"load_checkpoint: unsupported checkpoint format {meta.get('format')!r}")
    cur = _grid_meta()
    for k in ("nprocs", "dims", "nxyz", "overlaps", "periods"):
        if meta[k] != cur[k]:
            raise IGGError(f"load_checkpoint: checkpoint {k}={meta[k]} does not match the current grid ({cur[k]})")
    path = _rank_file(prefix, me)
    if not os.path.exists(path):
        raise IGGError(f"load_checkpoint: missing block file {path}")
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if gg.amdgpu_enabled else torch.device("cpu")
    out = {}
    with safe_open(path, framework="pt") as f:
        local = f.metadata() or {}
        if json.loads(local.get("coords", "null")) != [int(c) for c in gg.coords]:
            raise IGGError(f"load_checkpoint: {path} was written by the rank at coords {local.get('coords')}, "
                           f"this rank is at {[int(c) for c in gg.coords]}")
        if str(local.get("step")) != str(meta["step"]):
            raise IGGError(f"load_checkpoint: {path} holds step {local.get('step')}, the manifest names "
                           f"step {meta['step']} (blocks from different saves)")
        names = set(f.keys())
        if names != set(meta["fields"]):
            raise IGGError(f"load_checkpoint: {path} holds fields {sorted(names)}, manifest {sorted(meta['fields'])}")
        for k in sorted(names):
            out[k] = f.get_tensor(k).to(device)
    return meta, out
