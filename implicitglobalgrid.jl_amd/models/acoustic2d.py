"""2-D acoustic waves on a staggered grid: the staggered-field application.

BASELINE.json config "2-D staggered-grid solver 8192^2/GPU Float32 on 4
MI355X, 2x2 topology (staggered halo widths + mixed overlaps)". The reference
library has no such example; it is the canonical use of its staggered-array
support (fields one cell larger than the grid, ``ol(dim, A) = overlap +
size(A, dim) - n``: src/shared.jl:94, tools ``nx_g(A)``/``x_g(ix, dx, A)``:
src/tools.jl:3-107), as in ParallelStencil's acoustic examples.

Fields: P (nx, ny) at cell centres, Vx (nx+1, ny) on x-faces, Vy (nx, ny+1) on
y-faces. One time step = ONE fused HIP kernel (csrc/kernels/acoustic_kernels.hip:
P2 everywhere, then Vx2/Vy2 on inner faces from P2 recomputed in registers)
followed by ``update_halo_(Vx2, Vy2)`` (ol = 3 along the staggered dimension,
2 along the other: mixed overlaps in one call) and a buffer swap.

``set_fused(True)`` (GPU, a neighbour, overlap 2): the exchange moves into the
sweep (csrc/include/igg/acoustic.hpp FusedAcoustic): the kernel stores the
staggered boundary faces straight into the neighbours' next Vx2/Vy2 over xGMI
and one 1-wave sync kernel completes the step; every other halo value is
recomputed locally with the same arithmetic, so the fields are bitwise equal to
the update_halo_ path (tests/test_acoustic.py) - the communication is hidden
inside the HBM-bound sweep instead of following it.
"""
from __future__ import annotations

import math

import torch

from .. import parallel  # noqa: F401
from .._native import native
from ..parallel import grid as _grid
from ..parallel.halo import capture_graph, update_halo_
from ..utils import placement as _placement
from .diffusion3d import GRAPH_STEPS
from ..utils.tools import coords_g, nx_g, ny_g


class Acoustic2D:
    """2-D staggered acoustic wave propagation (pressure P at cell centres,
    velocities Vx/Vy on staggered faces: nx+1 / ny+1) with one fused HIP kernel
    per step and one ``update_halo_(Vx2, Vy2)`` (mixed overlaps); the 2-D
    staggered config of BASELINE.json."""

    def __init__(self, *, dtype=torch.float32, device=None, K: float = 1.0, rho: float = 1.0,
                 lx: float = 10.0, ly: float = 10.0):
        gg = _grid.global_grid()
        nx, ny = int(gg.nxyz[0]), int(gg.nxyz[1])
        if int(gg.nxyz[2]) != 1:
            raise ValueError("Acoustic2D needs a 2-D grid (init_global_grid(nx, ny, 1))")
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if gg.amdgpu_enabled else torch.device("cpu")
        self.device = torch.device(device)
        self.dtype = dtype
        self.nx, self.ny = nx, ny
        self.K, self.rho = K, rho
        self.dx = lx / (nx_g() - 1)
        self.dy = ly / (ny_g() - 1)
        self.dt = min(self.dx, self.dy) / math.sqrt(K / rho) / 4.1
        probe = torch.empty((nx, ny), device="meta")
        kw = dict(dtype=torch.float64, device=self.device)
        x = coords_g(0, self.dx, probe, **kw).view(-1, 1)
        y = coords_g(1, self.dy, probe, **kw).view(1, -1)
        P = torch.exp(-((x - lx / 2) ** 2) - (y - ly / 2) ** 2).to(dtype).contiguous()
        Vx = torch.zeros((nx + 1, ny), dtype=dtype, device=self.device)
        Vy = torch.zeros((nx, ny + 1), dtype=dtype, device=self.device)
        fields = [P, Vx, Vy, P.clone(), Vx.clone(), Vy.clone()]
        import os as _os

        self.placement = None
        if self.device.type == "cuda" and _os.environ.get("IGG_FIELD_MEMORY", "fine") != "torch":
            # One fine-grained allocation (the fused exchange stores into the
            # neighbours' Vx2/Vy2 while their kernels run: docs/COHERENCE.md),
            # the fastest of several candidates (utils/placement.py: 0.282 vs
            # 0.300 ms/step at 8192^2 between fast and slow carves).
            init = fields
            nbytes = P.numel() * P.element_size()
            k = _placement.candidate_count(gg, nbytes, sum(t.numel() * t.element_size() for t in init), self.device)
            fields, self.placement = _placement.placed(lambda: _carve_fine(init, split=int(gg.nprocs) > 1), k,
                                                       self._time_placements)
            if self.placement is not None:  # the probe stepped the chosen carve: back to the initial state
                for dst, src in zip(fields, init):
                    dst.copy_(src)
        self.P, self.Vx, self.Vy, self.P2, self.Vx2, self.Vy2 = fields
        # P's halo cells, evaluated from the global coordinates above, equal
        # the neighbours' cells only up to rounding (periodic wrap of x_g);
        # one exchange makes them bitwise consistent, so every halo value the
        # step recomputes locally equals what update_halo_ would deliver (the
        # fused exchange relies on it: set_fused). P itself is never exchanged
        # again: P2 is recomputed everywhere from halo-consistent inputs.
        update_halo_(self.P)
        self.graph = None
        self.graph_steps = 2
        self._graph_P = 0  # P's buffer when the graph was captured
        self._warm = False
        self.fused = False
        self._fa = None  # native FusedAcoustic (set_fused)
        # The next fused step starts with an entry barrier: the neighbours'
        # remote stores must not overtake this rank's own writes to the fields
        # (switch into fused mode, restore, external edits: mark_modified).
        self._entry = True

    def _time_placements(self, cands) -> list:
        """ms per step of this model's kernel on each candidate carve
        (P, Vx, Vy, P2, Vx2, Vy2), ping-pong (utils/placement.py)."""

        def launch(c, j):
            a, b = (c[3:], c[:3]) if j % 2 == 0 else (c[:3], c[3:])
            self._update(*a, *b)

        return _placement.time_candidates(cands, launch)

    def _update(self, P2, Vx2, Vy2, P, Vx, Vy) -> None:
        dev = self.device.type == "cuda"
        s = torch.cuda.current_stream().cuda_stream if dev else 0
        native.acoustic2d(P2.data_ptr(), Vx2.data_ptr(), Vy2.data_ptr(), P.data_ptr(), Vx.data_ptr(), Vy.data_ptr(),
                          self.nx, self.ny, self.dt * self.K, self.dt / self.rho, 1.0 / self.dx, 1.0 / self.dy,
                          P.element_size(), dev, s)

    @property
    def can_fuse(self) -> bool:
        """Fused exchange possible: GPU, a neighbour in x or y, overlap 2 in
        both, the vector kernel's shape (ny % 16 B-vector width, >= 5x5)."""
        gg = _grid.global_grid()
        if self.device.type != "cuda":
            return False
        if not any(int(gg.neighbors[s, d]) != -1 for s in range(2) for d in range(2)):
            return False
        if int(gg.overlaps[0]) != 2 or int(gg.overlaps[1]) != 2:
            return False
        if gg.nprocs > 1 and not gg.comm.one_node:  # IPC peer mappings: one node only
            return False
        vj = 4 if self.P.element_size() == 4 else 2
        return self.ny % vj == 0 and self.nx >= 5 and self.ny >= 5

    def set_fused(self, flag: bool) -> bool:
        """Switch the fused halo exchange on/off (collective: every rank at the
        same point; the first switch-on maps the neighbours' fields)."""
        flag = bool(flag) and self.can_fuse
        if flag == self.fused:
            return flag
        if flag and self._fa is None:
            gg = _grid.global_grid()
            nb = [[int(gg.neighbors[s, d]) for s in range(2)] for d in range(2)]
            if gg.nprocs > 1:
                mesh = native.PeerMesh(gg.comm.rank, gg.comm.size, gg.comm._allgather_bytes)
            else:  # periodic / loopback single process: every neighbour is this rank
                nb = [[0 if v >= 0 else -1 for v in row] for row in nb]
                mesh = native.PeerMesh(0, 1, lambda b: [bytes(b)])
            self._fa = native.FusedAcoustic(mesh, self.nx, self.ny, self.P.element_size(), nb)
            self._fa.set_fields(self.Vx.data_ptr(), self.Vx2.data_ptr(), self.Vy.data_ptr(), self.Vy2.data_ptr())
        self.fused = flag
        self._entry = True
        self.graph = None
        return flag

    def mark_modified(self) -> None:
        """Declare that the fields were written outside the time loop (e.g. a
        copy into P/Vx/Vy): the next fused step first synchronises with the
        neighbours, which store into this rank's fields (collective: every rank
        calls it at the same point)."""
        self._entry = True

    def sync_halo(self) -> None:
        """No-op: the fused step leaves every halo value as update_halo_ would
        (the API matches Diffusion3D's, whose fused step defers halo planes)."""

    def clear_error(self) -> None:
        """Reset the fused exchange's sticky timeout word on this rank (after
        a failed fused step was handled, e.g. the fused exchange was dropped)."""
        if self._fa is not None:
            self._fa.clear_error()

    def check(self) -> None:
        """Raise if a fused-exchange sync kernel timed out waiting for a neighbour."""
        if self._fa is not None:
            self._fa.check_error()

    def close(self) -> None:
        """Release the fused exchange's peer mappings (collective: every rank)."""
        if self._fa is not None:
            torch.cuda.synchronize()
            self._fa.close()
            self._fa = None
            self.fused = False
            self.graph = None

    def step(self) -> None:
        """Advance one time step. In fused mode the fields are final when the
        call returns (as far as stream order goes): the neighbours' stores of
        this step into them precede later work on the stream (``_drain``)."""
        self._step()
        self._drain()

    def _drain(self) -> None:
        """Exit barrier of in-kernel synchronised fused steps (collective): the
        last step's neighbour stores into this rank's fields are complete before
        anything queued after it (a restore, a comparison, gather_, a mode
        switch) touches the fields. No-op after a sync-kernel step."""
        if self.fused:
            self._fa.drain(torch.cuda.current_stream().cuda_stream)

    def _step(self) -> None:
        if self.fused:
            s = torch.cuda.current_stream().cuda_stream
            self._fa.step(self.P2.data_ptr(), self.Vx2.data_ptr(), self.Vy2.data_ptr(), self.P.data_ptr(),
                          self.Vx.data_ptr(), self.Vy.data_ptr(), self.nx, self.ny, self.dt * self.K,
                          self.dt / self.rho, 1.0 / self.dx, 1.0 / self.dy, self.P.element_size(), s,
                          self._entry)
            self._entry = False
        else:
            self._update(self.P2, self.Vx2, self.Vy2, self.P, self.Vx, self.Vy)
            update_halo_(self.Vx2, self.Vy2)
        self.P, self.P2 = self.P2, self.P
        self.Vx, self.Vx2 = self.Vx2, self.Vx
        self.Vy, self.Vy2 = self.Vy2, self.Vy
        self._warm = True

    def local_step(self) -> None:
        """One step of the LOCAL problem (what a rank without neighbours runs:
        the staggered update, no exchange - update_halo_ with PROC_NULL
        neighbours is a no-op, reference src/update_halo.jl:40-42). Timing
        only (the bench's same-process efficiency, which restores the state
        afterwards). No halo exchange repairs the state it leaves: the
        staggered fields' overlap is 3 along their staggered dim, so one plane
        next to each halo is computed on both ranks (never exchanged) and
        drifts apart under local steps, and the fused step is bitwise equal to
        the update_halo_ path only from states where those copies agree."""
        self._update(self.P2, self.Vx2, self.Vy2, self.P, self.Vx, self.Vy)
        self.P, self.P2 = self.P2, self.P
        self.Vx, self.Vx2 = self.Vx2, self.Vx
        self.Vy, self.Vy2 = self.Vy2, self.Vy

    def capture(self, steps: int = GRAPH_STEPS) -> None:
        """hipGraph of ``steps`` (even) time steps: buffers are back in their
        roles after a replay; replay launch overhead (~9 us on MI355X) is paid
        once per ``steps``."""
        if self.device.type != "cuda":
            raise RuntimeError("Acoustic2D.capture: hipGraphs need a GPU model")
        if steps < 2 or steps % 2:
            raise ValueError("Acoustic2D.capture: steps must be even and >= 2")
        if not self._warm or (self.fused and self._entry):
            self.step()  # the graph holds steady-state steps only (no entry barrier)
        def record():
            for _ in range(steps):
                self._step()  # no exit barrier inside the graph: run() drains once

        self.graph = None
        # fused steps exchange through their own peer mesh, not update_halo_
        g = capture_graph(record, f"{type(self).__name__}.capture", uses_halo=not self.fused)
        self.graph = g
        self.graph_steps = steps
        self._graph_P = self.P.data_ptr()

    def run(self, nt: int) -> None:
        """Advance ``nt`` steps (graph replays where captured); one exit barrier
        at the end in fused mode (``_drain``), none between the steps."""
        ran = nt > 0
        if self.graph is not None:
            # The captured steps read the capture's P/Vx/Vy first and hold no
            # entry barrier: one eager step realigns an odd step count or
            # performs a pending barrier (mark_modified, restore).
            while nt > 0 and not self._graph_ready():
                self._step()
                nt -= 1
            for _ in range(nt // self.graph_steps):
                self.graph.replay()
            nt %= self.graph_steps
        for _ in range(nt):
            self._step()
        if ran:
            self._drain()

    def _graph_ready(self) -> bool:
        return self.P.data_ptr() == self._graph_P and not (self.fused and self._entry)

    def save(self, prefix: str, step: int = 0) -> str:
        """Per-rank checkpoint of the model state (collective; utils.checkpoint)."""
        from ..utils.checkpoint import save_checkpoint

        return save_checkpoint(prefix, step=step, P=self.P, Vx=self.Vx, Vy=self.Vy, P2=self.P2, Vx2=self.Vx2,
                               Vy2=self.Vy2)

    def restore(self, prefix: str) -> int:
        """Load a checkpoint written by ``save`` on the same decomposition (in
        place); returns the saved step."""
        from ..utils.checkpoint import load_checkpoint

        meta, f = load_checkpoint(prefix, device=self.device)
        for name in ("P", "Vx", "Vy", "P2", "Vx2", "Vy2"):
            dst = getattr(self, name)
            if f[name].shape != dst.shape or f[name].dtype != dst.dtype:
                raise ValueError(f"Acoustic2D.restore: {name} is {tuple(f[name].shape)}/{f[name].dtype}, "
                                 f"the model has {tuple(dst.shape)}/{dst.dtype}")
            dst.copy_(f[name])
        self._entry = True
        return int(meta["step"])

    @property
    def a_eff_bytes(self) -> int:
        """Each of P, Vx, Vy read once and written once per step."""
        return 2 * (self.P.numel() + self.Vx.numel() + self.Vy.numel()) * self.P.element_size()


def _carve_fine(tensors, split: bool = False):
    """Copies of ``tensors`` carved from one native fine-grained allocation
    (256 B-aligned slices). ``split``: if that allocation would reach the IPC
    size limit (the neighbours map the velocity buffers), one allocation per
    tensor instead."""
    from .diffusion3d import _ipc_limit, native_buffer

    sizes = [t.numel() * t.element_size() for t in tensors]
    offs, pos = [], 0
    for n in sizes:
        offs.append(pos)
        pos += -(-n // 256) * 256
    if split and pos >= _ipc_limit() and len(tensors) > 1:
        return [_carve_fine([t])[0] for t in tensors]
    buf = native_buffer(pos, 1, tensors[0].device)
    out = []
    for t, o, n in zip(tensors, offs, sizes):
        v = buf[o:o + n].view(t.dtype).view(t.shape)
        v.copy_(t)
        out.append(v)
    return out


def acoustic2d_reference(P, Vx, Vy, *, dt, K, rho, dx, dy):
    """Plain-PyTorch fp64 reference of one fused step (same update order)."""
    P, Vx, Vy = P.double(), Vx.double(), Vy.double()
    P2 = P - dt * K * ((Vx[1:, :] - Vx[:-1, :]) / dx + (Vy[:, 1:] - Vy[:, :-1]) / dy)
    Vx2, Vy2 = Vx.clone(), Vy.clone()
    Vx2[1:-1, :] = Vx[1:-1, :] - dt / rho * (P2[1:, :] - P2[:-1, :]) / dx
    Vy2[:, 1:-1] = Vy[:, 1:-1] - dt / rho * (P2[:, 1:] - P2[:, :-1]) / dy
    return P2, Vx2, Vy2
