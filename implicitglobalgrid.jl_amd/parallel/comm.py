"""Distributed runtime: process group, RCCL communicator and transports.

Reference: MPI.jl drives all communication (src/shared.jl:1; MPI.Init in
src/init_global_grid.jl:78-83, Finalize in src/finalize_global_grid.jl:19-23).
MPI is not part of the MI355X stack; the replacement is

* one process per GPU, started by ``torchrun`` (or any launcher exporting
  ``RANK``/``WORLD_SIZE``/``MASTER_ADDR``/``MASTER_PORT``), bootstrapped through
  ``torch.distributed`` (TCP store at 127.0.0.1 on one node);
* a ``gloo`` group for host-side control traffic (barriers, the RCCL unique-id
  broadcast, CPU-tensor halos and gathers);
* a native RCCL communicator (``_igg_native.RcclComm``) for device-resident
  point-to-point traffic over xGMI — grouped ncclSend/ncclRecv enqueued on HIP
  streams by the C++ halo engine, no Python on the data path.

``IGG_TRANSPORT=torch`` swaps the native RCCL transport for torch.distributed's
``nccl`` (= RCCL) ``batch_isend_irecv`` (debug/A-B only); ``staged`` stages
device halos through host memory over gloo (the reference's non-GPU-aware MPI
path); ``put`` is the one-sided intra-node transport of csrc/peer.cpp (pack
kernels store straight into IPC-mapped peer arenas, CP flag signalling) that
lets the halo exchange run next to a stencil occupying the GPU.
"""
from __future__ import annotations

import ctypes
import datetime
import os
import socket
from dataclasses import dataclass, field

import torch
import torch.distributed as dist

from .._native import IGGError, native
from ..utils import config


def _host_view(ptr: int, nbytes: int) -> torch.Tensor:
    """uint8 CPU tensor aliasing native host memory (no copy)."""
    if nbytes == 0:
        return torch.empty(0, dtype=torch.uint8)
    buf = (ctypes.c_uint8 * nbytes).from_address(ptr)
    return torch.frombuffer(buf, dtype=torch.uint8)


class _DeviceBuf:
    """__cuda_array_interface__ wrapper to alias a raw HIP pointer as a tensor."""

    def __init__(self, ptr: int, nbytes: int):
        self.__cuda_array_interface__ = {
            "shape": (nbytes,),
            "typestr": "|u1",
            "data": (ptr, False),
            "version": 3,
        }


def _device_view(ptr: int, nbytes: int) -> torch.Tensor:
    return torch.as_tensor(_DeviceBuf(ptr, nbytes), device="cuda")


def runtime_initialized() -> bool:
    return dist.is_available() and dist.is_initialized()


def init_runtime(timeout_s: float | None = None) -> None:
    """Initialise torch.distributed (the MPI.Init equivalent).

    With launcher environment variables (``WORLD_SIZE`` etc.) this joins the
    job over ``env://``; otherwise a single-process group is created on an
    in-memory store.
    """
    if runtime_initialized():
        raise IGGError("The distributed runtime is already initialized.")
    # Every host collective is bounded (IGG_COMM_TIMEOUT, with a floor so a
    # long first-use autotune on one rank never trips it).
    timeout_s = max(60.0, config.comm_timeout()) if timeout_s is None else timeout_s
    timeout = datetime.timedelta(seconds=timeout_s)
    if "WORLD_SIZE" in os.environ and "RANK" in os.environ:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", init_method="env://", timeout=timeout)
    else:
        dist.init_process_group("gloo", store=dist.HashStore(), rank=0, world_size=1, timeout=timeout)


def finalize_runtime() -> None:
    if not runtime_initialized():
        raise IGGError("The distributed runtime cannot be finalized as it has not been initialized.")
    dist.destroy_process_group()


@dataclass
class Communicator:
    """The Cartesian communicator returned by ``init_global_grid`` (comm_cart).

    ``rank``/``size`` are ranks of ``group`` (row-major Cartesian order, no
    reordering). ``gloo`` carries host traffic; ``rccl`` device traffic.
    """

    group: object = None
    gloo: object = None
    rank: int = 0
    size: int = 1
    rccl: object = None
    torch_nccl: object = None
    mesh: object = None  # native.PeerMesh of the 'put' transport
    _stage: dict = field(default_factory=dict)  # pinned host staging buffers
    local_rank: int = 0
    local_size: int = 1
    _transports: dict = field(default_factory=dict)
    aborted: str = ""
    rccl_error: str = ""  # a failed RCCL bootstrap (every rank agrees): not retried

    def __eq__(self, other):  # identity semantics like MPI.Comm handles
        return self is other

    __hash__ = object.__hash__

    def global_rank(self, r: int) -> int:
        if self.gloo is None or self.gloo == dist.GroupMember.WORLD:
            return r
        return dist.get_global_rank(self.gloo, r)

    # -- collectives -------------------------------------------------------
    def barrier(self, timeout: float | None = None) -> None:
        """Host barrier of all ranks, bounded by ``timeout`` seconds (default
        IGG_COMM_TIMEOUT). On expiry the device communicators are aborted (a
        peer blocked in an RCCL kernel is released) and IGGError is raised,
        naming the ranks that did not arrive."""
        if self.size <= 1:
            return
        t = config.comm_timeout() if timeout is None else float(timeout)
        try:
            dist.monitored_barrier(group=self.gloo, timeout=datetime.timedelta(seconds=t), wait_all_ranks=True)
        except RuntimeError as e:
            self.abort(f"barrier timed out after {t:.0f} s")
            raise IGGError(f"barrier: not every rank arrived within {t:.0f} s (IGG_COMM_TIMEOUT); "
                           f"device communicators aborted: {str(e).splitlines()[0][:300]}") from None

    def device_barrier(self, stream: int | None = None) -> None:
        """Barrier of all ranks ordered on ``stream`` (default: current): a
        one-element RCCL all-reduce when the grid's RCCL communicator exists
        (tens of microseconds over xGMI), else the host barrier (gloo: hundreds
        of microseconds). Completes on a rank's stream only once every rank
        has enqueued it; a following stream sync makes it a host barrier."""
        if self.size <= 1:
            return
        if self.rccl is not None and not self.aborted:
            self.rccl.barrier(torch.cuda.current_stream().cuda_stream if stream is None else int(stream))
        else:
            self.barrier()

    def abort(self, reason: str = "") -> None:
        """Abort the device communicators (ncclCommAbort: RCCL kernels waiting
        on a peer exit) after an unrecoverable communication failure; later
        device exchanges raise instead of hanging."""
        self.aborted = reason or "aborted"
        if self.rccl is not None:
            try:
                self.rccl.abort()
            except Exception:
                pass

    # -- tensor collectives (comm_cart interop) --------------------------------
    # The reference hands applications its MPI Cartesian communicator for their
    # own collectives (README.md:166-178: e.g. a global residual). Here: CPU
    # tensors over gloo, GPU tensors over the grid's own native RCCL
    # communicator (the one that carries the halo traffic: one RCCL
    # communicator per rank), ordered on the caller's current stream.
    _OPS = {"sum": "SUM", "max": "MAX", "min": "MIN", "prod": "PRODUCT"}
    _RCCL_OPS = {"sum": 0, "prod": 1, "max": 2, "min": 3}
    _RCCL_TYPES = {torch.int8: 0, torch.uint8: 1, torch.int32: 2, torch.int64: 4, torch.float16: 6,
                   torch.float32: 7, torch.float64: 8, torch.bfloat16: 9}

    def _rccl_tensor(self, t: torch.Tensor):
        """(rccl communicator, dtype code, count) for a GPU tensor; complex
        tensors travel as their real pairs."""
        if not t.is_contiguous():
            raise IGGError("comm collectives on GPU tensors need a contiguous tensor")
        v = torch.view_as_real(t) if t.is_complex() else t
        if v.dtype not in self._RCCL_TYPES:
            raise IGGError(f"comm collectives: unsupported GPU dtype {t.dtype}")
        return self.ensure_rccl(), self._RCCL_TYPES[v.dtype], v.numel()

    def allreduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        """In-place all-reduce of ``t`` over the grid's ranks (``op``: sum,
        max, min, prod); returns ``t``. MPI.Allreduce! on comm_cart."""
        if op not in self._OPS:
            raise IGGError(f"allreduce_: op must be one of {sorted(self._OPS)} (got {op!r})")
        if self.size > 1:
            if t.is_cuda:
                if t.is_complex() and op != "sum":
                    raise IGGError(f"allreduce_: op {op!r} is not defined for complex tensors")
                rc, dt, n = self._rccl_tensor(t)
                rc.allreduce(t.data_ptr(), t.data_ptr(), n, dt, self._RCCL_OPS[op],
                             torch.cuda.current_stream().cuda_stream)
            else:
                dist.all_reduce(t, op=getattr(dist.ReduceOp, self._OPS[op]), group=self.gloo)
        return t

    def bcast_(self, t: torch.Tensor, root: int = 0) -> torch.Tensor:
        """In-place broadcast of ``t`` from grid rank ``root``; returns ``t``
        (MPI.Bcast! on comm_cart)."""
        if not 0 <= root < self.size:
            raise IGGError(f"bcast_: root {root} out of range 0..{self.size - 1}")
        if self.size > 1:
            if t.is_cuda:
                rc, dt, n = self._rccl_tensor(t)
                rc.broadcast(t.data_ptr(), t.data_ptr(), n, dt, root, torch.cuda.current_stream().cuda_stream)
            else:
                dist.broadcast(t, src=self.global_rank(root), group=self.gloo)
        return t

    def allreduce(self, value: float, op: str = "sum") -> float:
        """All-reduce of a Python scalar (host), e.g. a global residual norm."""
        t = torch.tensor([float(value)], dtype=torch.float64)
        return float(self.allreduce_(t, op).item())

    def broadcast_object(self, obj, root: int = 0):
        if self.size == 1:
            return obj
        lst = [obj]
        dist.broadcast_object_list(lst, src=self.global_rank(root), group=self.gloo)
        return lst[0]

    def all_gather_object(self, obj) -> list:
        if self.size == 1:
            return [obj]
        out = [None] * self.size
        dist.all_gather_object(out, obj, group=self.gloo)
        return out

    # -- transports ----------------------------------------------------------
    def host_transport(self):
        t = self._transports.get("gloo")
        if t is None:
            t = native.PyTransport(self._gloo_p2p, True, False, "gloo")
            self._transports["gloo"] = t
        return t

    def device_transport(self, choice: str | None = None):
        """Device transport ``choice`` (default: ``IGG_TRANSPORT``), created once
        and cached; creating the RCCL communicator or the put mesh is collective."""
        if self.size == 1:
            return None
        choice = config.transport_choice() if choice is None else choice
        if choice == "auto":  # no selection here (parallel/halo.py chooses per field set): RCCL
            choice = "rccl"
        if choice not in ("rccl", "torch", "staged", "put"):
            raise IGGError(f"unknown device transport {choice!r}")
        if choice == "staged":
            t = self._transports.get("staged")
            if t is None:
                t = native.PyTransport(self._staged_p2p, False, True, "gloo-staged")
                self._transports["staged"] = t
            return t
        if choice == "put":
            t = self._transports.get("put")
            if t is None:
                self.require_one_node("the 'put' transport")
                self.mesh = native.PeerMesh(self.rank, self.size, self._allgather_bytes)
                t = native.PutTransport(self.mesh)
                self._transports["put"] = t
            return t
        if choice == "torch":
            t = self._transports.get("torch")
            if t is None:
                self._ensure_torch_nccl()
                t = native.PyTransport(self._torch_p2p, False, True, "torch-nccl")
                self._transports["torch"] = t
            return t
        self.ensure_rccl()
        return self.rccl

    @property
    def one_node(self) -> bool:
        """Every rank of the communicator runs on this node (IPC peer mappings,
        the put transport, the fused exchanges and the gather pull need it)."""
        return self.local_size == self.size

    def require_one_node(self, what: str) -> None:
        """Raise on every rank (no collective is entered) when the ranks span
        several nodes: IPC handles cannot be opened on another node. RCCL and
        the staged transport work across nodes."""
        if not self.one_node:
            raise IGGError(f"{what} maps peer memory over IPC and needs every rank on one node "
                           f"({self.local_size} of {self.size} ranks are on this one); use IGG_TRANSPORT=rccl")

    def _allgather_bytes(self, b: bytes) -> list:
        return self.all_gather_object(bytes(b))

    def ensure_rccl(self):
        """The grid's native RCCL communicator, created on first use
        (collective). The bootstrap is bounded (a non-blocking communicator
        polled for IGG_FIRST_CONTACT_TIMEOUT seconds, then aborted) and its
        outcome is agreed over gloo: if any rank failed, every rank raises the
        same IGGError, and later calls raise it again at once instead of
        re-running a bootstrap that already failed (reference: a failing rank
        aborts the MPI job, src/init_global_grid.jl:80-92)."""
        if self.rccl is None and self.size > 1:
            if self.rccl_error:
                raise IGGError(self.rccl_error)
            uid = native.RcclComm.unique_id() if self.rank == 0 else None
            uid = self.broadcast_object(uid, root=0)
            rc, err = None, ""
            try:
                rc = native.RcclComm(uid, self.size, self.rank, config.first_contact_timeout())
            except Exception as e:  # bounded bootstrap expired, or RCCL refused (e.g. ranks sharing a GPU)
                err = f"{type(e).__name__}: {e}"
            errs = self.all_gather_object(err)
            bad = [r for r, e in enumerate(errs) if e]
            if bad:
                if rc is not None:
                    rc.abort()
                self.rccl_error = (f"RCCL communicator could not be created (failed on rank(s) {bad}; "
                                   f"rank {bad[0]}: {errs[bad[0]][:300]})")
                raise IGGError(self.rccl_error)
            self.rccl = rc
        return self.rccl

    def _ensure_torch_nccl(self):
        if self.torch_nccl is None:
            ranks = [self.global_rank(r) for r in range(self.size)]
            self.torch_nccl = dist.new_group(ranks=ranks, backend="nccl")

    def _gloo_p2p(self, recvs, sends, device, stream):
        if device:
            raise IGGError("gloo transport cannot move GPU memory.")
        if config.host_matching() == "ordered":
            self._ordered_exchange([(_host_view(p, n), peer) for p, n, peer, _t in recvs],
                                   [(_host_view(p, n), peer) for p, n, peer, _t in sends])
            return
        reqs = []
        for ptr, nbytes, peer, tag in recvs:
            reqs.append(dist.irecv(_host_view(ptr, nbytes), src=self.global_rank(peer), group=self.gloo, tag=tag))
        for ptr, nbytes, peer, tag in sends:
            reqs.append(dist.isend(_host_view(ptr, nbytes), dst=self.global_rank(peer), group=self.gloo, tag=tag))
        for r in reqs:
            r.wait()

    def _ordered_exchange(self, recvs, sends) -> None:
        """Order-only point-to-point phase over gloo: the messages of a phase
        to one peer travel as ONE tag-0 message, concatenated in issue order,
        and the receiver splits its single message from that peer over its
        receives in ITS issue order. Nothing but the position pairs the k-th
        send to a peer with the peer's k-th receive from this rank - exactly
        RCCL's matching of grouped ncclSend/ncclRecv, and MPI's with every tag
        0 as in the reference (update_halo.jl:713-735; SURVEY invariant 4:
        with dims=2 periodic both sides' messages go to ONE peer, and only the
        right-then-left receive / left-then-right send order makes them land
        in the right halo). ``recvs``/``sends``: [(uint8 CPU tensor, peer)].
        IGG_DEBUG_SWAP_SENDS=1 reverses each peer's send order (a test hook:
        the halo tests must then fail)."""
        by_s, by_r = {}, {}
        for t, p in sends:
            by_s.setdefault(p, []).append(t)
        for t, p in recvs:
            by_r.setdefault(p, []).append(t)
        if os.environ.get("IGG_DEBUG_SWAP_SENDS") == "1":
            for ts in by_s.values():
                ts.reverse()
        reqs, rbuf = [], {}
        for p, ts in by_r.items():
            n = sum(t.numel() for t in ts)
            if n == 0:
                continue
            b = ts[0] if len(ts) == 1 else torch.empty(n, dtype=torch.uint8)
            rbuf[p] = b
            reqs.append(dist.irecv(b, src=self.global_rank(p), group=self.gloo, tag=0))
        for p, ts in by_s.items():
            n = sum(t.numel() for t in ts)
            if n == 0:
                continue
            b = ts[0] if len(ts) == 1 else torch.cat(ts)
            reqs.append(dist.isend(b, dst=self.global_rank(p), group=self.gloo, tag=0))
        for r in reqs:
            r.wait()
        for p, ts in by_r.items():
            if len(ts) > 1 and p in rbuf:
                o = 0
                for t in ts:
                    t.copy_(rbuf[p][o:o + t.numel()])
                    o += t.numel()

    def _pinned(self, role: str, k: int, n: int) -> torch.Tensor:
        """Grow-only page-locked host staging buffer (reference: registered host
        buffers, src/shared.jl:117-129): DMA engines copy it without bouncing."""
        key = (role, k)
        b = self._stage.get(key)
        if b is None or b.numel() < n:
            b = torch.empty(max(n, 1 << 16), dtype=torch.uint8, pin_memory=True)
            self._stage[key] = b
        return b[:n]

    def _staged_p2p(self, recvs, sends, device, stream):
        """Host-staged device exchange (the reference's non-GPU-aware MPI path,
        update_halo.jl:437,465): D2H of the send buffers, gloo, H2D."""
        hs = []
        for k, (p, n, peer, tag) in enumerate(sends):
            h = self._pinned("s", k, n)
            native.memcpy_d2h_stream(h.data_ptr(), p, n, stream)
            hs.append((h, peer, tag))
        hr = [(self._pinned("r", k, n), p, peer, tag) for k, (p, n, peer, tag) in enumerate(recvs)]
        if config.host_matching() == "ordered":
            self._ordered_exchange([(h, peer) for h, _p, peer, _t in hr], [(h, peer) for h, peer, _t in hs])
        else:
            reqs = [dist.irecv(h, src=self.global_rank(peer), group=self.gloo, tag=tag) for h, _p, peer, tag in hr]
            reqs += [dist.isend(h, dst=self.global_rank(peer), group=self.gloo, tag=tag) for h, peer, tag in hs]
            for r in reqs:
                r.wait()
        for h, p, _peer, _tag in hr:
            native.memcpy_h2d_stream(p, h.data_ptr(), h.numel(), stream)

    def _torch_p2p(self, recvs, sends, device, stream):
        ops = []
        for ptr, nbytes, peer, _tag in recvs:
            ops.append(dist.P2POp(dist.irecv, _device_view(ptr, nbytes), self.global_rank(peer), self.torch_nccl))
        for ptr, nbytes, peer, _tag in sends:
            ops.append(dist.P2POp(dist.isend, _device_view(ptr, nbytes), self.global_rank(peer), self.torch_nccl))
        if not ops:
            return
        with torch.cuda.stream(torch.cuda.ExternalStream(stream)):
            for r in dist.batch_isend_irecv(ops):
                r.wait()

    def destroy(self) -> None:
        if self.mesh is not None:
            try:
                self.mesh.close()  # collective: unmap peers, free arenas/flags
            except Exception:
                pass
            self.mesh = None
        if self.rccl is not None:
            try:
                native.device_synchronize()
            except Exception:
                pass
            self.rccl = None
        self._transports.clear()
        if self.torch_nccl is not None:
            try:
                dist.destroy_process_group(self.torch_nccl)
            except Exception:
                pass
            self.torch_nccl = None
        if self.gloo is not None and self.gloo is not self.group and runtime_initialized():
            try:
                dist.destroy_process_group(self.gloo)
            except Exception:
                pass
        self.gloo = None


def bounded_device_sync(timeout: float | None = None, what: str = "device synchronize", comm=None) -> None:
    """``hipDeviceSynchronize`` that gives up after ``timeout`` seconds
    (default IGG_COMM_TIMEOUT): the wait runs in a helper thread; on expiry the
    grid's device communicators are aborted (so RCCL kernels blocked on a
    dead or diverged peer exit) and IGGError is raised. SURVEY §5.3: a rank
    must never hang silently on a peer that will not answer."""
    import threading

    t = config.comm_timeout() if timeout is None else float(timeout)
    done = threading.Event()
    err: list = []

    def run():
        try:
            native.device_synchronize()
        except Exception as e:  # surfaced on the caller's thread
            err.append(e)
        finally:
            done.set()

    th = threading.Thread(target=run, name="igg-bounded-sync", daemon=True)
    th.start()
    if not done.wait(t):
        if comm is not None:
            comm.abort(f"{what} timed out after {t:.0f} s")
        from . import halo as _halo

        _halo.abort_loopback()
        raise IGGError(f"{what}: the GPU did not drain within {t:.0f} s (IGG_COMM_TIMEOUT): a peer rank "
                       "is probably dead or skipped a collective exchange; device communicators aborted.")
    if err:
        raise err[0]


def bounded_stream_sync(stream: int | None = None, timeout: float | None = None, what: str = "stream synchronize",
                        comm=None) -> None:
    """Wait for everything enqueued on ``stream`` (default: the current
    stream) with a bound of ``timeout`` seconds (default IGG_COMM_TIMEOUT), by
    polling an event natively: no helper thread, microseconds of latency after
    completion (timed regions), same failure path as ``bounded_device_sync``."""
    t = config.comm_timeout() if timeout is None else float(timeout)
    s = torch.cuda.current_stream().cuda_stream if stream is None else int(stream)
    if not native.stream_wait_bounded(s, t):
        if comm is not None:
            comm.abort(f"{what} timed out after {t:.0f} s")
        from . import halo as _halo

        _halo.abort_loopback()
        raise IGGError(f"{what}: the GPU did not drain within {t:.0f} s (IGG_COMM_TIMEOUT): a peer rank "
                       "is probably dead or skipped a collective exchange; device communicators aborted.")


def make_communicator(group=None) -> Communicator:
    """Build the Communicator over ``group`` (default: WORLD)."""
    if not runtime_initialized():
        raise IGGError("The distributed runtime has not been initialized.")
    group = dist.GroupMember.WORLD if group is None else group
    size = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if dist.get_backend(group) == "gloo":
        gloo = group
    else:
        ranks = dist.get_process_group_ranks(group)
        gloo = dist.new_group(ranks=ranks, backend="gloo")
    c = Communicator(group=group, gloo=gloo, rank=rank, size=size)
    c.local_rank, c.local_size = _local_rank(c)
    return c


def _local_rank(c: Communicator) -> tuple[int, int]:
    """Node-local rank/size (MPI.Comm_split_type(COMM_TYPE_SHARED) equivalent)."""
    lr, ls = os.environ.get("LOCAL_RANK"), os.environ.get("LOCAL_WORLD_SIZE")
    if lr is not None and ls is not None and c.gloo == dist.GroupMember.WORLD:
        return int(lr), int(ls)
    host = socket.gethostname()
    hosts = c.all_gather_object(host)
    same = [r for r, h in enumerate(hosts) if h == host]
    return same.index(c.rank), len(same)
