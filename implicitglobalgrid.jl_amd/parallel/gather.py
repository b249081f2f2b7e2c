"""``gather_`` — assemble the global array on a root rank.

Reference: ``gather!(A, A_global; root=0)`` (src/gather.jl:25-65). The block of
the process with Cartesian coords (cx,cy,cz) lands at
``A_global[cx*nx:(cx+1)*nx, cy*ny:..., cz*nz:...]``; only
``A_global.numel() == nprocs*A.numel()`` is required (a 1-D ``A`` may be
gathered into a 3-D ``A_global``); ``A_global`` may be ``None`` off-root; the
root keeps a grow-only internal buffer until ``finalize_global_grid``.

MI355X paths (csrc/gather.cpp):
* GPU ``A``, all ranks on one node (the default; IGG_GATHER_PULL=0 disables;
  a block in an allocation too large to export is staged in chunks first):
  the root's copy engines pull every block over xGMI straight into its place
  in ``A_global`` (one 3-D peer copy per block, up to 8 concurrent copy
  streams, ordered by interprocess events): no staging buffer of
  nprocs*|A| on the root and no reorder pass. Stream-ordered, no host drain.
* GPU ``A`` otherwise: one RCCL group of receives on the root into a grow-only
  device buffer + a HIP reorder kernel.
* CPU ``A``: gloo point-to-point into a grow-only host buffer + one strided
  reorder copy.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .._native import ALLOC_GRANULARITY, IGGError, native
from ..utils import config
from . import grid as _grid
from .halo import field_tuple

_host_buf = None  # grow-only flat uint8 host buffer
_gatherer = None  # native device gatherer (grow-only device buffer)
_puller = None  # native PullGatherer (gather_async_)
_sync_puller = None  # native PullGatherer of the synchronous gather_ (pull path)


def free_gather_buffer() -> None:
    global _host_buf, _gatherer, _puller, _sync_puller
    _host_buf = None
    if _gatherer is not None:
        _gatherer.free()
    _gatherer = None
    if _puller is not None:
        if _puller.pending:
            raise IGGError("free_gather_buffer: a gather_async_ is still pending (call wait() first).")
        _puller.free()
    _puller = None
    if _sync_puller is not None:
        _sync_puller.free()
    _sync_puller = None


def _pull_ok(gg, A: torch.Tensor) -> bool:
    """Pull path for GPU fields: every rank on this node (IPC-mappable peers).
    The same answer on every rank (the choice is collective). A rank whose
    allocation holding ``A`` is too large to export (``native.IPC_MAX_BYTES``:
    opening a larger handle hangs on this ROCm runtime) stages ``A`` into
    exportable chunks itself (csrc/include/igg/gather.hpp PullGatherer)."""
    c = gg.comm
    return int(gg.nprocs) > 1 and c is not None and c.one_node and config.gather_pull()


def _padded_shape(A: torch.Tensor) -> list[int]:
    return list(A.shape) + [1] * (3 - A.dim())


def _global_view(A_global: torch.Tensor, s, dims) -> torch.Tensor:
    shape = [int(dims[d]) * s[d] for d in range(3)]
    if not A_global.is_contiguous():
        raise IGGError("The input argument A_global must be a contiguous array.")
    return A_global.view(shape)


def gather_(A: torch.Tensor, A_global: torch.Tensor | None, *, root: int = 0) -> None:
    """Gather ``A`` from every process into ``A_global`` on ``root``."""
    gg = _grid.global_grid()
    c = gg.comm
    nprocs = int(gg.nprocs)
    dims = [int(d) for d in gg.dims]
    me = int(gg.me)
    if me == root:
        if A_global is None:
            raise IGGError("The input argument A_global can't be `nothing` on the root")
        if A_global.numel() != nprocs * A.numel():
            raise IGGError("The input argument A_global must be of length nprocs*length(A)")
        if A_global.dtype != A.dtype:
            raise IGGError("The input arguments A and A_global must have the same element type.")
    s = _padded_shape(A)
    if A.is_cuda and gg.amdgpu_enabled:
        A = A.contiguous()
        if _pull_ok(gg, A):
            _gather_pull(A, A_global, root, s, dims, me, nprocs, c)
            return
    if A.is_cuda and nprocs > 1 and c.rccl is None and gg.amdgpu_enabled and config.transport_choice() in ("rccl", "auto"):
        c.ensure_rccl()
    if A.is_cuda and (nprocs == 1 or c.rccl is not None):
        _gather_device(A, A_global, root, s, dims, me, nprocs, c)
    else:
        _gather_host(A.cpu() if A.is_cuda else A, A_global, root, s, dims, me, nprocs, c)


def _gather_device(A, A_global, root, s, dims, me, nprocs, c) -> None:
    global _gatherer
    A = A.contiguous()
    stream = torch.cuda.current_stream().cuda_stream
    dst = None
    if me == root:
        dst = A_global if (A_global.is_cuda and A_global.is_contiguous()) else torch.empty(
            A_global.shape, dtype=A.dtype, device=A.device)
        _global_view(dst, s, dims)  # validates the shape
    if nprocs == 1:
        _global_view(dst, s, dims).copy_(A.view(s))
    else:
        if _gatherer is None:
            _gatherer = native.Gatherer()
        _gatherer.gather(field_tuple(A), dst.data_ptr() if dst is not None else 0, root, dims, c.rccl, stream)
    if me == root and dst is not A_global:
        A_global.copy_(dst)


def _gather_pull(A, A_global, root, s, dims, me, nprocs, c) -> None:
    """Synchronous gather_ through the pull path: start + wait of a native
    PullGatherer (stream-ordered on the current stream of every rank)."""
    global _sync_puller
    A = A.contiguous()
    dst = None
    if me == root:
        dst = A_global if (A_global.is_cuda and A_global.is_contiguous()) else torch.empty(
            A_global.shape, dtype=A.dtype, device=A.device)
        _global_view(dst, s, dims)  # validates the shape
    if _sync_puller is None:
        _sync_puller = native.PullGatherer(me, nprocs, lambda b: c.all_gather_object(bytes(b)))
    stream = torch.cuda.current_stream().cuda_stream
    _sync_puller.start(field_tuple(A), dst.data_ptr() if dst is not None else 0, root, dims, stream)
    _sync_puller.wait(stream)
    if me == root and dst is not A_global:
        A_global.copy_(dst)


def _gather_host(A, A_global, root, s, dims, me, nprocs, c) -> None:
    global _host_buf
    A = A.contiguous()
    nbytes = A.numel() * A.element_size()
    if me != root:
        dist.send(A.view(-1).view(torch.uint8), dst=c.global_rank(root), group=c.gloo)
        return
    need = -(-nprocs * A.numel() // ALLOC_GRANULARITY) * ALLOC_GRANULARITY * A.element_size()
    if _host_buf is None or _host_buf.numel() < need:
        _host_buf = None
        _host_buf = torch.empty(need, dtype=torch.uint8)
    flat = _host_buf[: nprocs * nbytes]
    reqs = []
    for p in range(nprocs):
        if p != root:
            reqs.append(dist.irecv(flat[p * nbytes:(p + 1) * nbytes], src=c.global_rank(p), group=c.gloo))
    flat[root * nbytes:(root + 1) * nbytes].copy_(A.view(-1).view(torch.uint8))
    for r in reqs:
        r.wait()
    blocks = flat.view(A.dtype).view(dims[0], dims[1], dims[2], s[0], s[1], s[2])
    glob = blocks.permute(0, 3, 1, 4, 2, 5).reshape(dims[0] * s[0], dims[1] * s[1], dims[2] * s[2])
    if A_global.is_contiguous() and A_global.device.type == "cpu":
        _global_view(A_global, s, dims).copy_(glob)
    else:
        A_global.copy_(glob.reshape(A_global.shape).to(A_global.device))


class GatherHandle:
    """Result of ``gather_async_``; ``wait()`` completes the gather (collective)."""

    def __init__(self, A_global, done: bool):
        self._A_global = A_global
        self._done = done

    def wait(self) -> None:
        if self._done:
            return
        _puller.wait(torch.cuda.current_stream().cuda_stream)
        self._done = True

    @property
    def done(self) -> bool:
        return self._done


def gather_async_(A: torch.Tensor, A_global: torch.Tensor | None, *, root: int = 0,
                  snapshot: bool = False) -> GatherHandle:
    """Non-blocking ``gather_``: returns a handle whose ``wait()`` (collective)
    completes it. GPU fields on several ranks: the root pulls every block with
    the copy engines straight into its place in ``A_global`` (one 3-D
    peer-to-peer copy per block over xGMI, ordered after the point of every
    rank's current stream where ``A`` is final by interprocess events: no GPU
    drain at the call, no compute units, no staging buffer) while the
    application continues; ``A`` must not be modified before ``wait()``
    (MPI_Igather semantics) and ``A_global`` (root) must be a C-contiguous GPU
    tensor. Other cases complete synchronously.

    ``snapshot=True``: every rank copies ``A`` at the call, stream-ordered
    (into its exportable staging chunks; the root straight into its block of
    ``A_global``), and ``A`` may be modified right away: the copy is the only
    serial part; the root's pulls of the chunks overlap the ranks' next steps
    (in-situ visualisation every K steps, BASELINE config 5)."""
    global _puller
    gg = _grid.global_grid()
    nprocs, me = int(gg.nprocs), int(gg.me)
    if not (A.is_cuda and nprocs > 1) or not _pull_ok(gg, A):
        # one process, or not IPC-mappable (another node): the synchronous
        # gather_ (RCCL / host)
        gather_(A, A_global, root=root)
        return GatherHandle(A_global, True)
    if me == root:
        if A_global is None:
            raise IGGError("The input argument A_global can't be `nothing` on the root")
        if A_global.numel() != nprocs * A.numel():
            raise IGGError("The input argument A_global must be of length nprocs*length(A)")
        if A_global.dtype != A.dtype:
            raise IGGError("The input arguments A and A_global must have the same element type.")
        if not (A_global.is_cuda and A_global.is_contiguous()):
            raise IGGError("gather_async_: A_global must be a C-contiguous GPU tensor on the root.")
        _global_view(A_global, _padded_shape(A), [int(d) for d in gg.dims])
    if not A.is_contiguous():
        raise IGGError("gather_async_: A must be contiguous (it is read in place by the root, or snapshot).")
    if _puller is None:
        c = gg.comm
        _puller = native.PullGatherer(me, nprocs, lambda b: c.all_gather_object(bytes(b)))
    dims = [int(d) for d in gg.dims]
    _puller.start(field_tuple(A), A_global.data_ptr() if me == root else 0, root, dims,
                  torch.cuda.current_stream().cuda_stream, bool(snapshot))
    return GatherHandle(A_global if me == root else None, False)


gather = gather_
