"""``update_halo_`` — halo update of one or more fields (CPU or GPU tensors).

Reference: ``update_halo!`` (src/update_halo.jl:25-78) with its argument checks
(:804-834), ranges (:544-563) and buffer pool (:92-339). The data path is the
native C++ ``HaloEngine`` (csrc/halo.cpp): per dimension x -> y -> z, ONE fused
pack launch for every face of every field, ONE RCCL group (device) or gloo
phase (host), ONE fused unpack launch; contiguous faces go zero-copy; the
periodic single-process case is one in-place copy launch. All GPU work is
enqueued on the caller's current HIP stream with no host synchronisation.

Layout: a field's logical axes (0, 1, 2) are the grid's (x, y, z); any dense
memory layout works (the engine reads strides). PyTorch's default C order makes
z contiguous, so the x-face is the zero-copy one and the z-face the strided one.
"""
from __future__ import annotations

import numpy as np
import torch

from .._native import NDIMS, NNEIGHBORS, PROC_NULL, IGGError, native
from ..utils import config
from . import grid as _grid

_engine = None
_plans: dict = {}
_MAX_PLANS = 512
# 'auto' schedule winners by a rank-invariant field-set signature (shapes,
# strides, dtypes, device kind): every rank makes the same update_halo_ calls
# on the same local shapes, so whether a call runs the (collective) tuning
# never depends on per-rank allocator state such as data pointers or plan-cache
# evictions (a rank that tuned alone would pair its extra exchanges with the
# other ranks' normal ones).
_sig_modes: dict = {}
# IGG_TRANSPORT=auto (the default; off after an explicit set_transport): the
# device transport by the same field-set signature, chosen on the signature's
# first eager device exchange (transport_select.auto_select: bitwise against
# the host-staged exchange, timed, collective) and switched to per call.
_auto = False
_selecting = False  # inside a selection: its own probe exchanges use the transport as set
_sig_transport: dict = {}
_transport_log: list = []
_cur_transport = None  # name of the device transport the engine holds (None: pending / none)
_buf_dtype = {False: None, True: None}
_debug_sync = False
_graphs: list = []  # weakrefs to hipGraphs that captured update_halo_


def register_graph(g) -> None:
    """Record a captured ``torch.cuda.CUDAGraph`` whose nodes use the halo
    buffers / RCCL communicator, so freeing those resets the graph first (a
    replay then fails loudly instead of touching freed memory, and RCCL's
    communicator is never destroyed under a live graph, which hangs)."""
    import weakref

    _graphs[:] = [r for r in _graphs if r() is not None]
    _graphs.append(weakref.ref(g))


def _release_graphs() -> None:
    live = [r() for r in _graphs]
    _graphs.clear()
    if any(g is not None for g in live):
        torch.cuda.synchronize()
    for g in live:
        if g is not None:
            g.reset()


def _join(items) -> str:
    """Julia's ``join(v, ", ", " and ")``."""
    s = [str(x) for x in items]
    if len(s) <= 1:
        return "".join(s)
    return ", ".join(s[:-1]) + " and " + s[-1]


def _jl_vec(v) -> str:
    return "[" + ", ".join(str(x) for x in v) + "]"


def _is_dense(t: torch.Tensor) -> bool:
    if t.numel() <= 1:
        return True
    dims = sorted((st, sz) for st, sz in zip(t.stride(), t.shape) if sz > 1)
    expect = 1
    for st, sz in dims:
        if st != expect:
            return False
        expect *= sz
    return True


def field_tuple(t: torch.Tensor):
    """(ptr, ndims, size3, stride3, elem_bytes, device) for the native engine."""
    nd = t.dim()
    if nd < 1 or nd > NDIMS:
        raise IGGError(f"Fields must have 1 to {NDIMS} dimensions (got {nd}).")
    size = list(t.shape) + [1] * (NDIMS - nd)
    stride = list(t.stride()) + [t.numel()] * (NDIMS - nd)
    return (t.data_ptr(), nd, size, stride, t.element_size(), bool(t.is_cuda))


def peer_table(gg) -> list[int]:
    """Rank at coords + disp*v for all 27 directions v (dir_key order: v in
    {-1,0,1}^3, last component fastest), PROC_NULL off a non-periodic grid."""
    dims = [int(d) for d in gg.dims]
    out = []
    for vx in (-1, 0, 1):
        for vy in (-1, 0, 1):
            for vz in (-1, 0, 1):
                c, ok = [], True
                for d, v in enumerate((vx, vy, vz)):
                    x = int(gg.coords[d]) + int(gg.disp) * v
                    if x < 0 or x >= dims[d]:
                        if not gg.periods[d]:
                            ok = False
                            break
                        x %= dims[d]
                    c.append(x)
                out.append(native.cart_rank(c, dims) if ok else PROC_NULL)
    return out


def _grid_info(gg) -> "native.GridInfo":
    return native.GridInfo(int(gg.me), int(gg.nprocs), gg.nxyz.tolist(), gg.overlaps.tolist(),
                           gg.neighbors.tolist(), peer_table(gg))


HALO_MODES = {"sequential": 0, "onephase": 1, "auto": 2}


def set_halo_mode(mode: str) -> None:
    """Select the exchange schedule: 'sequential' (x->y->z faces, the reference
    algorithm), 'onephase' (faces+edges+corners in one phase) or 'auto'."""
    _grid.check_initialized()
    if mode == "onephase" and _loopback_one_sided and "rccl" in _loopback_comms:
        raise IGGError(_ONE_SIDED_ONEPHASE)
    _engine.set_mode(HALO_MODES[mode])
    _sig_modes.clear()
    for p in _plans.values():
        p[3] = None  # an explicit mode wins; 'auto' measures again


def halo_mode() -> str:
    """The exchange schedule set by ``set_halo_mode`` / ``IGG_HALO_MODE``."""
    _grid.check_initialized()
    return {v: k for k, v in HALO_MODES.items()}[_engine.mode]


def set_pack_mode(mode: str, dims=(True, True, True)) -> None:
    """GPU face copies of the sequential schedule in the selected dims:
    'kernel' (one batched copy launch per dim) or 'memcpy2d'
    (hipMemcpy2DAsync per face with contiguous rows, the reference's strided
    memcpy alternative; other faces keep the kernel). Also IGG_PACK[_DIMX/Y/Z]."""
    _grid.check_initialized()
    m = config.PACK_MODES.index(mode)
    for d in range(NDIMS):
        if dims[d]:
            _engine.set_pack_mode(d, m)


def pack_mode(dim: int) -> str:
    """Pack mode of dimension ``dim`` (1-based, like the reference's dims)."""
    _grid.check_initialized()
    return config.PACK_MODES[_engine.pack_mode(dim - 1)]


def _init_engine(gg) -> None:
    global _engine, _debug_sync
    _plans.clear()
    _sig_modes.clear()
    _engine = native.HaloEngine(_grid_info(gg))
    _engine.set_mode(HALO_MODES[config.halo_mode()])
    for d, m in enumerate(config.pack_modes()):
        _engine.set_pack_mode(d, config.PACK_MODES.index(m))
    _debug_sync = config.debug_sync()
    _set_poll_every(config.poll_every())
    global _auto, _cur_transport
    _auto = gg.nprocs > 1 and bool(gg.amdgpu_enabled) and config.transport_choice() == "auto"
    _sig_transport.clear()
    _transport_log.clear()
    _cur_transport = None
    if gg.nprocs > 1:
        _engine.set_transport(gg.comm.host_transport(), False)
        # The device transport (RCCL communicator, put mesh) is created by the
        # first device exchange, not here: init_global_grid must not depend on
        # a first contact with the other GPUs (a bootstrap that fails or hangs
        # fails that exchange - or the transport validation that selects
        # another transport - not the grid itself).
        _set_dev_pending(bool(gg.amdgpu_enabled))


_dev_pending = False
_PENDING_NAMES = {"rccl": "rccl", "put": "put", "staged": "gloo-staged", "torch": "torch-nccl", "auto": "auto"}


def _set_dev_pending(flag: bool) -> None:
    global _dev_pending
    _dev_pending = flag


def _ensure_device_transport() -> None:
    """Create the configured device transport on first use (collective: every
    rank's first device exchange happens at the same point). With
    IGG_TRANSPORT=auto this is the transport of exchanges that are not
    selected (a field set first seen inside a hipGraph capture): RCCL, or the
    host-staged transport where ranks share a GPU (RCCL refuses that); the
    selection of the first eager exchange replaces it."""
    global _dev_pending
    if _dev_pending:
        _dev_pending = False
        choice = config.transport_choice()
        if choice == "auto":
            from .transport_select import _shared_device

            choice = "staged" if _shared_device(_grid.global_grid().comm) else "rccl"
        use_transport(choice)


def use_transport(name: str) -> None:
    """Point the engine at device transport ``name`` without ending the
    automatic choice (internal: IGG_TRANSPORT=auto selection and per-signature
    switches; the schedule caches stay, they are per signature too).
    Collective on first use of a transport (creates it)."""
    global _cur_transport
    name = {v: k for k, v in _PENDING_NAMES.items()}.get(name, name)
    if _loopback_comm is not None:
        _use_loopback(name)
    else:
        _engine.set_transport(_grid.global_grid().comm.device_transport(name), True)
    _set_dev_pending(False)
    _cur_transport = name


class selecting:
    """Context of a transport selection: the probe exchanges inside use the
    transport as set (no nested automatic selection)."""

    def __enter__(self):
        global _selecting
        self._prev, _selecting = _selecting, True
        return self

    def __exit__(self, *exc):
        global _selecting
        _selecting = self._prev
        return False


def tuned_transports() -> list:
    """IGG_TRANSPORT=auto selections so far: one record per field-set
    signature (shapes, dtype, per-candidate check outcome and ms per exchange,
    the chosen transport)."""
    return list(_transport_log)


def auto_transport() -> bool:
    """Whether update_halo_ chooses the device transport itself (IGG_TRANSPORT=auto)."""
    return _auto


def meshes() -> list:
    """The put transport's peer meshes of this grid (multi-rank and loopback)."""
    out = []
    gg = _grid.global_grid()
    if gg.comm is not None and getattr(gg.comm, "mesh", None) is not None:
        out.append(gg.comm.mesh)
    for c in _loopback_comms.values():
        if hasattr(c, "mesh"):
            out.append(c.mesh)
    return out


_poll_every = 1000


def _set_poll_every(n: int) -> None:
    global _poll_every, _poll_count
    _poll_every, _poll_count = int(n), 0


def _drop_engine() -> None:
    global _engine, _loopback_comm, _loopback_one_sided, _auto, _cur_transport
    _release_graphs()
    _plans.clear()
    _sig_modes.clear()
    _sig_transport.clear()
    _loopback_comms.clear()
    _auto, _cur_transport = False, None
    if _engine is not None:
        _engine.pool_free()
    _engine = None
    _loopback_comm = None
    _loopback_one_sided = False
    _set_dev_pending(False)


def set_transport(name: str) -> None:
    """Switch the device transport of ``update_halo_`` ('rccl', 'put', 'torch'
    or 'staged'). Collective: every rank must switch at the same point (the
    first use of a transport creates its communicator / peer mesh). An
    explicit choice: update_halo_ stops choosing by itself (IGG_TRANSPORT=auto)."""
    global _auto, _cur_transport
    name = {v: k for k, v in _PENDING_NAMES.items()}.get(name, name)  # transport_name() spellings too
    gg = _grid.global_grid()
    if gg.nprocs == 1:
        raise IGGError("set_transport: a single-process grid has no device transport")
    if not gg.amdgpu_enabled:
        raise IGGError("set_transport: the grid was not initialised for GPU fields")
    if name == "auto":
        raise IGGError("set_transport: 'auto' is the IGG_TRANSPORT default, not a transport")
    _engine.set_transport(gg.comm.device_transport(name), True)
    _set_dev_pending(False)
    _auto, _cur_transport = False, name
    _sig_transport.clear()
    _sig_modes.clear()
    for p in _plans.values():
        p[3] = None  # schedule costs differ per transport: 'auto' measures again


def transport_name() -> str:
    """Name of the device transport update_halo_ currently uses ('none' if single-process)."""
    _grid.check_initialized()
    if _dev_pending:  # not created yet: the configured choice
        return _PENDING_NAMES[config.transport_choice()]
    return _engine.transport_name(True)


def check_transport() -> None:
    """Raise if a put-transport synchronisation kernel timed out (its spin
    waits are bounded; a timeout means some exchange's halo is invalid) or an
    RCCL communicator reported an asynchronous error."""
    for m in meshes():
        m.check_error()
    gg = _grid.global_grid()
    rcc = [getattr(gg.comm, "rccl", None) if gg.comm is not None else None]
    rcc += [c for c in _loopback_comms.values() if isinstance(c, native.RcclComm)]
    for c in rcc:
        if c is not None:
            c.check_async_error()  # ncclCommGetAsyncError: raises on an asynchronous RCCL failure


def abort_loopback() -> None:
    """Abort the single-GPU loopback RCCL communicator (bounded-wait expiry)."""
    for c in _loopback_comms.values():
        if isinstance(c, native.RcclComm):
            try:
                c.abort()
            except Exception:
                pass


# Device transports whose exchanges can be recorded in a hipGraph: RCCL
# (grouped ncclSend/ncclRecv on the stream) and put (kernels + device-side
# flags). 'gloo-staged' and 'torch-nccl' synchronise with the host inside an
# exchange.
CAPTURABLE = ("rccl", "put", "none")


def capturable() -> bool:
    """Whether ``update_halo_`` of device fields can be captured in a hipGraph
    with the current transport (single-process grids: always)."""
    if _loopback_comm is not None:
        return _engine.transport_name(True) in CAPTURABLE
    if _grid.global_grid().nprocs == 1:
        return True
    # pending auto: the first exchange creates RCCL (or staged where ranks share a GPU)
    return transport_name() in CAPTURABLE + ("auto",)


def capture_graph(record, what: str, uses_halo: bool = True):
    """A hipGraph of ``record()`` (which enqueues work on the current stream).
    Raises IGGError before beginning if the halo transport cannot be captured.
    If the capture fails, the runtime's sticky error from the failed capture is
    reset, so the next kernel launch does not report it (round 4: a rehearsal
    with the host-staged transport died at the first eager step after a failed
    capture)."""
    if uses_halo and not capturable():
        raise IGGError(f"{what}: the '{transport_name()}' transport synchronises with the host inside an exchange "
                       "and cannot be captured in a hipGraph; run eager steps")
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            record()
    except Exception:
        try:
            torch.cuda.synchronize()
        except Exception:
            pass
        native.clear_last_error()
        raise
    torch.cuda.synchronize()
    register_graph(g)
    return g


def engine():
    _grid.check_initialized()
    return _engine


def sync_grid() -> None:
    """Push the (possibly test-mutated) grid topology into the native engine."""
    _plans.clear()
    _sig_modes.clear()
    _engine.set_grid(_grid_info(_grid.global_grid()))


_loopback_comm = None
# Loopback transports by kind ('rccl', 'put'): one with IGG_TRANSPORT=rccl|put,
# both with auto (kept alive side by side: replacing one destroyed it
# mid-process, round 5); _loopback_comm is the one the engine holds.
_loopback_comms: dict = {}
# Loopback emulation of a shape with one side in some dim (a node's edge or
# corner rank): one process plays every neighbour through ONE self-peer, so
# RCCL pairs messages by issue order alone. The sequential schedule issues one
# receive and one send of equal size per emulated side; the one-phase
# schedule's receive order (by receiver-side direction) differs from its send
# order there, pairing messages of different sizes - a p2p receive larger than
# its matched send reads past the send buffer (round 5: GPU memory fault in
# benchmarks/rank_shapes.py, found on the CPU with a host loopback transport).
_loopback_one_sided = False
_ONE_SIDED_ONEPHASE = ("loopback emulation of a one-sided shape: the one-phase schedule cannot pair its messages "
                       "through one self-peer over RCCL; use the sequential schedule (or the put transport)")


def enable_loopback(dims=(True, True, True)) -> None:
    """Single-GPU emulation of a rank surrounded by neighbours (perf analysis).

    ``dims[d]``: True (both sides), False (none) or a (low, high) pair of
    bools - one side only emulates a node's edge/corner ranks (a 2x2x2 corner
    rank has one neighbour per dim: ``((False, True),) * 3`` for coords 0).
    Every selected side gets the neighbour rank 0 while the engine
    believes it is rank 1, so each face takes the full remote path — pack ->
    grouped ncclSend/ncclRecv over a 1-rank RCCL communicator (to itself) ->
    unpack (or, with IGG_TRANSPORT=put, put kernel -> own arena -> flags ->
    unpack) — with real communication kernels competing for CUs, like an
    interior rank of a multi-GPU run. The grid's neighbour table is updated
    too, so apps enable their boundary/interior overlap. Results equal a
    periodic exchange.
    """
    global _loopback_comm, _loopback_one_sided
    gg = _grid.global_grid()
    if gg.nprocs != 1 or not gg.amdgpu_enabled:
        raise IGGError("loopback mode needs a single-process grid with a GPU")
    sides = [(bool(x[0]), bool(x[1])) if isinstance(x, (tuple, list)) else (bool(x), bool(x)) for x in dims]
    nb = gg.neighbors.tolist()  # the grid's table changes only once every check passed
    for d in range(NDIMS):
        for s in range(2):
            if sides[d][s]:
                nb[s][d] = 0
    one_sided = any(sd[0] != sd[1] for sd in sides)
    global _auto
    choice = config.transport_choice()
    kinds = ("rccl", "put") if choice == "auto" else (("put",) if choice == "put" else ("rccl",))
    if one_sided and _engine.mode == HALO_MODES["onephase"]:
        if choice == "auto":
            kinds = ("put",)  # the only loopback transport that pairs one-sided one-phase messages
        elif "rccl" in kinds:
            raise IGGError(_ONE_SIDED_ONEPHASE)  # before the grid or the engine changes
    want = kinds[0]
    # A later call (another emulated shape) reuses the loopback transports
    # instead of replacing them: a replaced RCCL communicator or put mesh is
    # destroyed mid-process, and a put -> RCCL switch that way was followed
    # by a GPU memory fault (round 5, benchmarks/rank_shapes.py).
    for k in kinds:
        if k not in _loopback_comms and _loopback_comms and choice != "auto":
            raise IGGError(f"loopback mode: the '{next(iter(_loopback_comms))}' loopback transport exists; one "
                           f"transport kind per process (IGG_TRANSPORT={k} requested)")
        if k not in _loopback_comms:
            _loopback_comms[k] = (native.PutTransport(native.PeerMesh(0, 1, lambda b: [bytes(b)])) if k == "put"
                                  else native.RcclComm(native.RcclComm.unique_id(), 1, 0))
    _loopback_comm = _loopback_comms[want]
    _auto = choice == "auto"
    _sig_transport.clear()
    # one-phase directions (k = 9*cx + 3*cy + cz, c = 0 low / 1 none / 2 high):
    # a peer where every non-zero component points at an emulated side
    peers = [0 if all(c == 1 or sides[d][c // 2] for d, c in enumerate((k // 9, (k // 3) % 3, k % 3)))
             else PROC_NULL for k in range(27)]
    peers[13] = 1
    _loopback_one_sided = one_sided
    for s_ in range(2):
        for d in range(NDIMS):
            gg.neighbors[s_, d] = nb[s_][d]
    _engine.set_grid(native.GridInfo(1, 2, gg.nxyz.tolist(), gg.overlaps.tolist(), nb, peers))
    _engine.set_transport(_loopback_comm, True)
    global _cur_transport
    _cur_transport = want
    _plans.clear()
    _sig_modes.clear()


def loopback_active() -> bool:
    """The single-GPU loopback emulation is on (enable_loopback)."""
    return _loopback_comm is not None


def loopback_one_sided() -> bool:
    """The loopback emulation covers a one-sided shape (a node's edge or corner rank)."""
    return _loopback_comm is not None and _loopback_one_sided


def _use_loopback(name: str) -> None:
    global _loopback_comm
    if name not in _loopback_comms:
        raise IGGError(f"loopback mode: no '{name}' loopback transport in this process")
    if name == "rccl" and _loopback_one_sided and _engine.mode == HALO_MODES["onephase"]:
        raise IGGError(_ONE_SIDED_ONEPHASE)
    _loopback_comm = _loopback_comms[name]
    _engine.set_transport(_loopback_comm, True)


# --- argument checks (update_halo.jl:804-834) ---------------------------------
def _ol(gg, dim0: int, t: torch.Tensor) -> int:
    s = int(t.shape[dim0]) if t.dim() > dim0 else 1
    return int(gg.overlaps[dim0]) + s - int(gg.nxyz[dim0])


def check_fields(*fields) -> None:
    gg = _grid.global_grid()
    for i, A in enumerate(fields):
        if not isinstance(A, torch.Tensor):
            raise IGGError(f"The field at position {i + 1} is not a torch.Tensor.")
    no_halo = [i + 1 for i, A in enumerate(fields) if all(_ol(gg, d, A) < 2 for d in range(A.dim()))]
    if len(no_halo) > 1:
        raise IGGError(f"The fields at positions {_join(no_halo)} have no halo; remove them from the call.")
    if len(no_halo) > 0:
        raise IGGError(f"The field at position {no_halo[0]} has no halo; remove it from the call.")
    dups = [
        [i + 1, j + 1]
        for i in range(len(fields))
        for j in range(i + 1, len(fields))
        if fields[i].device == fields[j].device and fields[i].data_ptr() == fields[j].data_ptr()
    ]
    if len(dups) > 2:
        raise IGGError(
            f"The pairs of fields with the positions {_join(_jl_vec(d) for d in dups)} are the same; "
            "remove any duplicates from the call."
        )
    if len(dups) > 0:
        raise IGGError(
            f"The field at position {dups[0][1]} is a duplicate of the one at the position {dups[0][0]}; "
            "remove the duplicate from the call."
        )

    def typ(A):
        return (A.dtype, A.dim(), A.device.type)

    diff = [i + 1 for i in range(1, len(fields)) if typ(fields[i]) != typ(fields[0])]
    if len(diff) > 1:
        raise IGGError(
            f"The fields at positions {_join(diff)} are of different type than the first field; "
            "make sure that in a same call all fields are of the same type."
        )
    if len(diff) == 1:
        raise IGGError(
            f"The field at position {diff[0]} is of different type than the first field; "
            "make sure that in a same call all fields are of the same type."
        )
    for i, A in enumerate(fields):
        if not _is_dense(A):
            raise IGGError(
                f"The field at position {i + 1} is not a dense array (a strided view); pass the full array."
            )


def _plan(fields):
    key = tuple((A.data_ptr(), A.shape, A.stride(), A.dtype, A.device) for A in fields)
    p = _plans.get(key)
    if p is None:
        check_fields(*fields)
        gg = _grid.global_grid()
        device = fields[0].is_cuda
        if device and not gg.amdgpu_enabled:
            raise IGGError(
                "AMDGPU is not enabled (possibly detected non functional when the ImplicitGlobalGrid module was loaded)."
            )
        if len(_plans) >= _MAX_PLANS:
            _plans.clear()
        p = [native.FieldSet([field_tuple(A) for A in fields]), device, fields[0].dtype, None]
        _plans[key] = p
    return p


# --- measured schedule choice ('auto' mode) -----------------------------------
# Timed exchanges per schedule (after one untimed warm-up exchange each, which
# also opens RCCL's lazily connected peer channels).
_TUNE_REPS = 5
_tuned_log: list = []  # (field shapes, {mode: ms}, winner) of every measurement


def _remote_peers() -> bool:
    """A device exchange of this grid reaches another rank (or the loopback
    emulation): only then do the schedules differ in cost."""
    gg = _grid.global_grid()
    if _loopback_comm is not None:
        return True
    nb = gg.neighbors
    return bool(((nb != PROC_NULL) & (nb != gg.me)).any())


def _tune_mode(fs, stream: int) -> int:
    if _loopback_one_sided and _loopback_comm is not None and _loopback_comm.name == "rccl":
        return HALO_MODES["sequential"]  # the only schedule a one-sided RCCL loopback can pair
    return _tune_mode_timed(fs, stream)


def _tune_mode_timed(fs, stream: int) -> int:
    """Time the sequential and one-phase schedules on this field set (MAX over
    ranks, so every rank picks the same winner) and return the faster mode.
    Collective like update_halo_ itself. Safe to run on live data: a halo
    exchange is idempotent (send planes are interior, receive planes halo)."""
    import time

    gg = _grid.global_grid()
    times = {}
    for name in ("sequential", "onephase"):
        m = HALO_MODES[name]
        _engine.exchange_set(fs, stream, m)
        native.stream_synchronize(stream)
        if gg.comm is not None:
            gg.comm.barrier()
        t0 = time.perf_counter()
        for _ in range(_TUNE_REPS):
            _engine.exchange_set(fs, stream, m)
        native.stream_synchronize(stream)
        dt = (time.perf_counter() - t0) / _TUNE_REPS
        if gg.comm is not None and gg.comm.size > 1:
            import torch.distributed as dist

            t = torch.tensor([dt], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=gg.comm.gloo)
            dt = float(t.item())
        times[name] = dt
    win = min(times, key=times.get)
    _tuned_log.append(({k: round(v * 1e3, 4) for k, v in times.items()}, win))
    return HALO_MODES[win]


def tuned_modes() -> list:
    """Measurements of the 'auto' schedule choice so far: ``[({mode: ms}, winner), ...]``."""
    return list(_tuned_log)


def plan_mode(*fields) -> str:
    """Schedule the next ``update_halo_(*fields)`` uses: the measured winner for
    this field set if 'auto' measured one, else the engine's mode (auto
    without a measurement resolves to sequential)."""
    p = _plan(fields)
    if p[3] is not None:
        return {v: k for k, v in HALO_MODES.items()}[p[3]]
    return {v: k for k, v in HALO_MODES.items()}[_engine.resolved_mode(p[0])]


def update_halo_(*fields) -> None:
    """Update the halo of the given field(s) (``update_halo!``).

    Group fields in one call for better performance: every dimension then needs
    one pack launch, one communication phase and one unpack launch for all of
    them. GPU work is stream-ordered on ``torch.cuda.current_stream()``.

    Schedule ('auto', the default): the first eager exchange of a GPU field set
    that reaches other ranks times the sequential and the one-phase schedule
    (collectively; a few extra exchanges) and keeps the faster for that field
    set; later calls and hipGraph captures reuse the choice.
    """
    _grid.check_initialized()
    if not fields:
        return
    p = _plan(fields)
    fs, device, dtype, mode = p
    if device and _dev_pending:
        _ensure_device_transport()
    stream = torch.cuda.current_stream().cuda_stream if device else 0
    sig = None
    if device and _auto and not _selecting:
        # IGG_TRANSPORT=auto: this signature's transport (chosen on its first
        # eager exchange that reaches another rank; collective)
        sig = tuple((tuple(A.shape), tuple(A.stride()), A.dtype) for A in fields)
        name = _sig_transport.get(sig)
        if name is None and _remote_peers() and not torch.cuda.is_current_stream_capturing():
            from .transport_select import auto_select

            name, rec = auto_select(fields)
            _sig_transport[sig] = name
            _transport_log.append(rec)
        if name is not None and name != _cur_transport:
            use_transport(name)
    if mode is None and device and _engine.mode == HALO_MODES["auto"]:
        sig = sig or tuple((tuple(A.shape), tuple(A.stride()), A.dtype) for A in fields)
        mode = p[3] = _sig_modes.get(sig)
        if mode is None and _remote_peers() and _engine.transport_name(True) != "put" \
                and not torch.cuda.is_current_stream_capturing():
            mode = p[3] = _sig_modes[sig] = _tune_mode(fs, stream)
    _engine.exchange_set(fs, stream, -1 if mode is None or _engine.mode != HALO_MODES["auto"] else mode)
    _buf_dtype[device] = dtype
    if _debug_sync and device and not torch.cuda.is_current_stream_capturing():
        native.stream_synchronize(stream)
    _poll_transport()


_poll_count = 0


def _poll_transport() -> None:
    """Every IGG_POLL_EVERY exchanges (default 1000; 0 = never) read the put
    transport's sticky error word on a side stream (no sync of the caller's
    stream), so a timed-out synchronisation surfaces within a bounded number
    of steps instead of only at check_transport()/finalize."""
    global _poll_count
    if _poll_every <= 0:
        return
    _poll_count += 1
    if _poll_count % _poll_every == 0 and not torch.cuda.is_current_stream_capturing():
        check_transport()


update_halo = update_halo_


# --- ranges (update_halo.jl:544-563), 1-based like the reference --------------
def sendranges(n: int, dim: int, A: torch.Tensor) -> list[range]:
    """1-based index ranges of the plane of ``A`` sent to side ``n`` (1 left, 2 right) in ``dim``
    (update_halo.jl:544-552)."""
    gg = _grid.global_grid()
    o = _ol(gg, dim - 1, A)
    if o < 2:
        raise IGGError("Incoherent arguments: ol(A,dim)<2.")
    size = [int(A.shape[d]) if A.dim() > d else 1 for d in range(NDIMS)]
    i = size[dim - 1] - (o - 1) if n == 2 else 1 + (o - 1)
    r = [range(1, s + 1) for s in size]
    r[dim - 1] = range(i, i + 1)
    return r


def recvranges(n: int, dim: int, A: torch.Tensor) -> list[range]:
    """1-based index ranges of the halo plane of ``A`` received from side ``n`` in ``dim``
    (update_halo.jl:555-563)."""
    gg = _grid.global_grid()
    if _ol(gg, dim - 1, A) < 2:
        raise IGGError("Incoherent arguments: ol(A,dim)<2.")
    size = [int(A.shape[d]) if A.dim() > d else 1 for d in range(NDIMS)]
    i = size[dim - 1] if n == 2 else 1
    r = [range(1, s + 1) for s in size]
    r[dim - 1] = range(i, i + 1)
    return r


def halosize(dim: int, A: torch.Tensor) -> tuple:
    """Shape of the halo of ``A`` in ``dim`` (update_halo.jl:84)."""
    if A.dim() > 1:
        return tuple(int(s) for d, s in enumerate(A.shape) if d != dim - 1)
    return (1,)


# --- buffer pool hooks (update_halo.jl:104-187, 332-338) ------------------------
def allocate_bufs(*fields) -> None:
    _grid.check_initialized()
    device = fields[0].is_cuda
    _engine.pool_ensure([field_tuple(A) for A in fields], device)
    _buf_dtype[device] = fields[0].dtype


def free_update_halo_buffers() -> None:
    """Free the halo send/recv buffers (update_halo.jl:104-122); they are re-allocated on demand."""
    _release_graphs()
    if _engine is not None:
        native.device_synchronize() if _engine.pool_allocated(True) else None
        _engine.pool_free()
    _buf_dtype[False] = _buf_dtype[True] = None


def _bufs(which: int, device: bool):
    if _engine is None or not _engine.pool_allocated(device):
        return None
    dtype = _buf_dtype[device] or torch.float64
    esize = torch.empty(0, dtype=dtype).element_size()
    out = []
    from .comm import _device_view, _host_view

    for slot in range(_engine.pool_nslots(device)):
        ptrs = _engine.pool_ptrs(slot, device)
        cap = _engine.pool_capacity(slot, device)
        pair = []
        for n in range(NNEIGHBORS):
            ptr = ptrs[which * 2 + n]
            raw = _device_view(ptr, cap) if device else _host_view(ptr, cap)
            pair.append(raw[: (cap // esize) * esize].view(dtype))
        out.append(pair)
    return out


def get_sendbufs_raw(device: bool = False):
    """Views of the send buffers (list per field slot of [left, right]); None if freed."""
    return _bufs(0, device)


def get_recvbufs_raw(device: bool = False):
    return _bufs(1, device)


def halo_plan_summary(*fields) -> list[dict]:
    """Describe what an exchange of ``fields`` does per dim (debug/profiling aid)."""
    gg = _grid.global_grid()
    out = []
    for d in range(NDIMS):
        nb = gg.neighbors[:, d]
        entry = {"dim": d + 1, "neighbors": nb.tolist(), "faces": []}
        for i, A in enumerate(fields):
            if _ol(gg, d, A) < 2:
                continue
            ft = field_tuple(A)
            for s in range(NNEIGHBORS):
                if nb[s] == PROC_NULL:
                    continue
                idx = native.send_index(_engine.grid, s, d, ft)
                info = native.face_info(ft, d, idx)
                entry["faces"].append({"field": i + 1, "side": s + 1, "bytes": info[6], "zero_copy": bool(info[5])})
        out.append(entry)
    return out


def _buf_view(which: int, n: int, dim: int, i: int, A: torch.Tensor, flat: bool):
    bufs = _bufs(which, A.is_cuda)
    if bufs is None:
        raise IGGError("The halo buffers are not allocated.")
    shape = halosize(dim, A)
    numel = int(np.prod(shape))
    b = bufs[i - 1][n - 1]
    v = b.view(torch.uint8)[: b.numel() * b.element_size()].view(A.dtype)[:numel]
    return v if flat else v.view(shape)


def sendbuf_flat(n: int, dim: int, i: int, A: torch.Tensor):
    """Flat send buffer of field slot ``i`` (1-based), side ``n``, typed as ``A``."""
    return _buf_view(0, n, dim, i, A, True)


def recvbuf_flat(n: int, dim: int, i: int, A: torch.Tensor):
    return _buf_view(1, n, dim, i, A, True)


def sendbuf(n: int, dim: int, i: int, A: torch.Tensor):
    """Send buffer shaped like the halo of ``A`` in ``dim`` (update_halo.jl:288-290)."""
    return _buf_view(0, n, dim, i, A, False)


def recvbuf(n: int, dim: int, i: int, A: torch.Tensor):
    return _buf_view(1, n, dim, i, A, False)


def _face_copy(buf: torch.Tensor, A: torch.Tensor, ranges, dim: int, pack: bool) -> None:
    if buf.dtype != A.dtype or buf.device != A.device:
        raise IGGError("buffer and array must have the same element type and device")
    idx = ranges[dim - 1].start - 1
    ft = field_tuple(A)
    base, n_outer, n_inner, s_outer, s_inner, _contig, nbytes = native.face_info(ft, dim - 1, idx)
    if buf.numel() * buf.element_size() < nbytes or not buf.is_contiguous():
        raise IGGError("buffer too small or not contiguous")
    if pack:
        c = (base, buf.data_ptr(), n_outer, n_inner, s_outer, s_inner, n_inner, 1)
    else:
        c = (buf.data_ptr(), base, n_outer, n_inner, n_inner, 1, s_outer, s_inner)
    stream = torch.cuda.current_stream().cuda_stream if A.is_cuda else 0
    native.copy2d([c], A.element_size(), A.is_cuda, stream)


def write_face(buf: torch.Tensor, A: torch.Tensor, ranges, dim: int) -> None:
    """Pack the plane ``ranges`` (1-based, single index in ``dim``) of ``A`` into
    ``buf`` (reference write_h2h!/write_d2x!, update_halo.jl:569-612)."""
    _face_copy(buf, A, ranges, dim, True)


def read_face(buf: torch.Tensor, A: torch.Tensor, ranges, dim: int) -> None:
    """Unpack ``buf`` into the plane ``ranges`` of ``A`` (read_h2h!/read_x2d!)."""
    _face_copy(buf, A, ranges, dim, False)
