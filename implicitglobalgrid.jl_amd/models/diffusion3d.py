"""3-D heat diffusion with Gaussian-anomaly initial conditions (the benchmark).

Reference application: examples/diffusion3D_multigpu_CuArrays_novis.jl (and its
CPU twin diffusion3D_multicpu_novis.jl): lam=1, cp_min=1, l=10 per axis, two
Gaussian anomalies in Cp and two in T built from x_g/y_g/z_g,
dt = min(dx^2,dy^2,dz^2)*cp_min/lam/8.1, per step: stencil update of the
interior then ``update_halo!(T)``.

MI355X design of a time step (``overlap=True`` and at least one neighbour):

  halo stream (high priority): boundary slabs of T2 (the planes update_halo
      sends) -> update_halo_(T2)  [pack -> RCCL -> unpack, x->y->z]
  compute stream:              interior of T2 (everything else)
  join, swap T <-> T2.
  (With the RCCL transport the exchange stays on the issuing stream and the
  interior goes to the forked one: RCCL captured on a forked stream crashes
  hipGraph capture, benchmarks/rccl_capture_repro.py.)

Both read T only; they write disjoint parts of T2, so the exchange hides behind
the interior update. Without neighbours (1 GPU, non-periodic) the step is one
fused kernel and update_halo_ is a no-op, as in the reference.

``fused=True`` (GPU, at least one neighbour; csrc/include/igg/fused.hpp): the
stencil kernel itself stores the send planes into the neighbours' IPC-mapped
arenas over xGMI while it sweeps, and reads its face halos from its own arena;
a 1-wave sync kernel is the whole exchange. The fields' halo planes are then
stale until ``sync_halo()`` (update_halo_ of T), which ``run``/``capture``
callers invoke before reading halos (gather, output). Interior values are
bitwise identical to the update_halo_ path.
"""
from __future__ import annotations

import os
import warnings

import torch

from .. import parallel  # noqa: F401
from ..ops import stencil
from ..parallel import grid as _grid
from ..parallel.halo import capture_graph, update_halo_
from ..utils import placement as _placement
from ..utils.tools import coords_g, nx_g, ny_g, nz_g


# Time steps per captured hipGraph (even): one replay launch (~9 us) per
# GRAPH_STEPS steps instead of per 2 (profiles/r1_fused/graph_gaps.txt).
GRAPH_STEPS = 10
# Candidates re-timed by the autotune's ping-pong stage (_choose_variant).
PINGPONG_FRONT = 4
# Whole-line z-edge stores of the full-box steps (ops.stencil.diffusion3d_
# halo_z; the fused step on its z sides without a neighbour): T2's z halo gets
# T's values, which is a no-op at fixed boundaries (T2 = T.clone() at init,
# neither is ever changed there) and is rewritten by the exchange elsewhere.
# 1024^3 f32 -5.5..-6.8 %, 512^3 f64 up to -2.9 % per variant
# (profiles/r4_halo_z/). IGG_HALO_Z=0 restores partial-line edge stores.
HALO_Z = os.environ.get("IGG_HALO_Z", "1").strip() != "0"


def _rccl_transport() -> bool:
    from ..parallel import halo as H

    return H.transport_name() == "rccl"


class Diffusion3D:
    """3-D heat diffusion with variable heat capacity on the local grid of the
    implicit global grid (examples/diffusion3D_multigpu_CuArrays_novis.jl):
    ``T2 = T + dt*lam/Cp * laplace(T)`` by one fused HIP kernel, then
    ``update_halo_(T2)`` (or the fused exchange, ``set_fused``), ping-pong T/T2.
    ``step``/``run`` advance, ``capture`` records hipGraphs, ``save``/``restore``
    checkpoint."""

    def __init__(self, *, dtype=torch.float64, device=None, lam: float = 1.0, cp_min: float = 1.0,
                 lx: float = 10.0, ly: float = 10.0, lz: float = 10.0, overlap: bool = False,
                 slab_width=None, variant=None, halo_variant=None, interior_rounds: int = 0,
                 halo_rounds: int = 0, reserve_cus: int = 0, field_memory: str = None):
        gg = _grid.global_grid()
        nx, ny, nz = (int(v) for v in gg.nxyz)
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if gg.amdgpu_enabled else torch.device("cpu")
        self.device = torch.device(device)
        self.dtype = dtype
        self.lam, self.cp_min = lam, cp_min
        self.dx = lx / (nx_g() - 1)
        self.dy = ly / (ny_g() - 1)
        self.dz = lz / (nz_g() - 1)
        self.dt = min(self.dx ** 2, self.dy ** 2, self.dz ** 2) * cp_min / lam / 8.1
        self.variant = variant
        self.rounds = 0  # grid residency rounds of the full-interior launch (0: library default)
        self.halo_z = HALO_Z  # whole-line z-edge stores of the full-interior launch (autotuned per variant)
        self.variant_times = None  # per-variant ms when autotuned (see _choose_variant)
        self.timer = None  # optional utils.trace.PhaseTimer (eager steps only)
        # Overlap tuning knobs: kernel variant / grid rounds of the boundary
        # slabs and grid rounds of the interior launch (see ops.stencil).
        self.halo_variant = halo_variant
        self.interior_rounds = interior_rounds
        self.halo_rounds = halo_rounds
        self.interior_first = False
        self.graph = None
        self.graph_steps = 2
        self._warm = False
        shape = (nx, ny, nz)
        probe = torch.empty(shape, device="meta")  # sizes only, for coords_g
        kw = dict(dtype=torch.float64, device=self.device)
        x = coords_g(0, self.dx, probe, **kw).view(-1, 1, 1)
        y = coords_g(1, self.dy, probe, **kw).view(1, -1, 1)
        z = coords_g(2, self.dz, probe, **kw).view(1, 1, -1)
        # field_memory (IGG_FIELD_MEMORY): "fine" (default: one native
        # fine-grained allocation) or "torch" (coarse-grained, torch's caching
        # allocator). The direct-z fused exchange stores into the neighbours'
        # T/T2 while their kernels run, which HIP defines for fine-grained
        # memory only (docs/COHERENCE.md); the plain sweep runs as fast on it
        # (profiles/r3_coherence/: 0.6222 vs 0.6263 ms/step).
        # One allocation with gaps between the three arrays: measured 1-3 %
        # faster than back-to-back 2 MiB-aligned tensors on MI355X
        # (profiles/r2_offsets/stencil_offsets.py: HBM channel placement). The
        # fields are allocated first and the initial conditions written into
        # them (no full-size temporary copies).
        import os as _os

        self.field_memory = (field_memory or _os.environ.get("IGG_FIELD_MEMORY", "fine")).strip().lower()
        if self.field_memory not in ("torch", "fine", "vmm"):
            raise ValueError(f"Diffusion3D: field_memory must be 'torch', 'fine' or 'vmm', got {self.field_memory!r}")
        if self.device.type == "cuda":
            # With neighbours in other processes T/T2 may be IPC-mapped (direct
            # z, gather_ pull): no allocation may reach the IPC size limit, so
            # a carve that would is split into one allocation per array. An
            # array that alone reaches it (1024^3 f32: 4 GiB) can never be IPC
            # mapped; with "fine" it then lives in HIP VMM memory (MemKind 4,
            # csrc/vmm.cpp), which gather_ maps through a file descriptor at
            # any size instead of staging it in chunks (round 6).
            kinds = {"torch": None, "fine": 1, "vmm": 4}
            spec = [torch.empty(shape, dtype=dtype, device="meta")] * 3
            multi = int(gg.nprocs) > 1
            big = multi and spec[0].numel() * spec[0].element_size() >= _ipc_limit()

            def carve():
                return _carve(spec, gap=266240, kind=kinds[self.field_memory],
                              split_at=_ipc_limit() if multi else None, device=self.device,
                              split_kind=4 if (big and self.field_memory == "fine") else None)

            (self.T, self.Cp, self.T2), self.placement = _placed_fields(carve, gg, spec[0], self.device)
            self._ipc_fields = self.field_memory == "fine" and not big  # direct z can map T/T2
        else:
            self.T, self.Cp, self.T2 = (torch.empty(shape, dtype=dtype) for _ in range(3))
            self.placement = None
        # Gaussian anomalies, evaluated in float64 a slab of x planes at a time
        # into the target dtype: the float64 temporaries of the whole field
        # (several x 8 bytes per point) would otherwise be the memory peak of a
        # 1024^3 rank - 8 ranks sharing one GPU ran out of memory here - while
        # every value is the same elementwise expression as before.
        slab = max(1, (1 << 24) // max(1, ny * nz))
        for x0 in range(0, nx, slab):
            xs = x[x0:x0 + slab]
            self.Cp[x0:x0 + slab] = (cp_min + 5 * torch.exp(-(xs - lx / 1.5) ** 2 - (y - ly / 2) ** 2 - (z - lz / 1.5) ** 2)
                                     + 5 * torch.exp(-(xs - lx / 3.0) ** 2 - (y - ly / 2) ** 2 - (z - lz / 1.5) ** 2))
            self.T[x0:x0 + slab] = (100 * torch.exp(-((xs - lx / 2) / 2) ** 2 - ((y - ly / 2) / 2) ** 2
                                                    - ((z - lz / 3.0) / 2) ** 2)
                                    + 50 * torch.exp(-((xs - lx / 2) / 2) ** 2 - ((y - ly / 2) / 2) ** 2
                                                     - ((z - lz / 1.5) / 2) ** 2))
        self.T2.copy_(self.T)
        sides = [[bool(gg.neighbors[0, d] != -1), bool(gg.neighbors[1, d] != -1)] for d in range(3)]
        self.sides = sides
        self.can_overlap = self.device.type == "cuda" and any(any(sd) for sd in sides)
        self.inner = [stencil.inner_box(shape)]
        z_split = any(sides[2])
        if overlap and self.can_overlap and z_split and self.variant is None:
            self.variant = 11  # 128-point tiles: z-slabs stay one full tile wide
        if self.variant is None and self.device.type == "cuda":
            self.variant = _choose_variant(self)
        if slab_width is None:
            # A slab at every side with a neighbour, just wide enough to hold
            # the plane update_halo sends there (index ol-1 / n-ol) along dims
            # 0/1; along the contiguous dim 2 (where a thin slab would waste
            # whole cache lines per row) it is exactly one kernel tile wide, so
            # both the slab launch and the interior launch run full tiles.
            o = [int(v) for v in gg.overlaps]
            tile = max(1, int(stencil.native.diffusion3d_variant_tile(self.variant or 0)))
            slab_width = (max(1, o[0] - 1), max(1, o[1] - 1), max(o[2] - 1, tile - 1))
        self.slabs, self.interior = stencil.split_boundary(shape, sides, slab_width)
        if self.halo_variant is None and not z_split:
            self.halo_variant = 18  # x/y boundary planes: the one-row scalar kernel is fastest
        self.compute_stream = None
        self.halo_stream = None
        self._reserve_cus = reserve_cus
        self.overlap = False
        if overlap:
            self.set_overlap(True)
        # Fused halo exchange (set_fused): native FusedHalo, step counter (arena
        # half parity), whether the arena holds the halos of the current T.
        self.fused = False
        # Fused kernel: variant (tiling; one with a fused instantiation) and
        # send mode (0 stores as computed, 1 deferred one x step; +2 compiles the
        # z-edge exchange out when there is no z neighbour; +4 direct z: the z
        # faces go straight into the neighbours' next T, no z receive code; +8
        # peel: x-chunk waves sweep only x = 1 / n0-2 with the x exchange,
        # profiles/r2_peel/).
        self.fused_variant = 0
        self.fused_mode = 8
        self.fused_rounds = 3  # grid residency rounds (profiles/r1_fused/grid.log)
        self._fh = None
        self._fstep = 0
        self._fprimed = False
        # Entry barrier before the next fused step (neighbours store into this
        # rank's arena and, with direct z, its fields: their stores must not
        # overtake this rank's own earlier writes - a switch into fused mode, a
        # restore, external edits: mark_modified).
        self._fentry = True
        # Receive form of the last fused step (send-mode bits 4 / 64 / 16): where
        # the primed halos live (arena, T's z halo column) and how the step
        # synchronises. A step in another form re-primes first (_align_form).
        self._fform = None
        self._graph_fused = None  # fused mode / step parity the graph was captured with
        self._graph_parity = 0
        self._graph_cfg = None  # fused (variant, mode, rounds) of the capture
        self._graph_T = 0  # T's buffer when the graph was captured

    @property
    def can_fuse(self) -> bool:
        """Fused halo exchange possible: GPU, a neighbour, overlap 2 where split,
        n2 a multiple of 4 (vector kernels)."""
        gg = _grid.global_grid()
        if self.device.type != "cuda" or not any(any(sd) for sd in self.sides):
            return False
        if any(any(self.sides[d]) and int(gg.overlaps[d]) != 2 for d in range(3)):
            return False
        if gg.nprocs > 1 and not gg.comm.one_node:  # IPC peer mappings: one node only
            return False
        return int(self.T.shape[2]) % 4 == 0 and int(self.T.shape[2]) >= 8

    def set_fused(self, flag: bool) -> bool:
        """Switch the fused halo exchange on/off (collective: every rank at the
        same point; the first switch-on creates the peer mesh). Switching off
        materialises the halos first. Returns the mode."""
        flag = bool(flag) and self.can_fuse
        if flag == self.fused:
            return flag
        if flag:
            if self._fh is None:
                self._fh = _make_fused_halo(self)
                # Direct z sends (fused_mode bit 4) write into the neighbours'
                # T/T2 while their kernels run: defined for fine-grained fields
                # (docs/COHERENCE.md); torch-allocated fields only on one GPU.
                if getattr(self, "_ipc_fields", False) or _grid.global_grid().nprocs == 1:
                    try:
                        self._fh.set_fields(self.T.data_ptr(), self.T2.data_ptr())
                    except Exception as e:  # collective outcome: every rank gets here together
                        warnings.warn(f"Diffusion3D: direct z sends unavailable ({e})")
            if self.fused_mode & 4 and not self._fh.has_fields:
                self.fused_mode &= ~4
            if not stencil.native.diffusion3d_fused_variant_ok(int(self.fused_variant)):
                self.fused_variant = 0
            self.set_overlap(False)
            self._fprimed = False  # the field's halo planes are valid right now
            self._fentry = True
        else:
            self.sync_halo()
        self.fused = flag
        self.graph = None
        return flag

    def sync_halo(self) -> None:
        """Materialise the halo planes of T (fused mode leaves them stale):
        one update_halo_(T). Later fused steps read halos from T again."""
        if self.fused and self._fprimed:
            update_halo_(self.T)
            self._fprimed = False

    def mark_modified(self) -> None:
        """Declare that T/T2 were written outside the time loop: the next fused
        step first synchronises with the neighbours (collective) and reads its
        halos from T."""
        self._fprimed = False
        self._fentry = True

    def exchange_halos(self) -> None:
        """Make T's halo planes equal the neighbours' (update_halo_(T);
        collective) and mark the fields modified: after ``local_step`` calls
        the state is again one the time loop could have produced."""
        update_halo_(self.T)
        self.mark_modified()

    def close(self) -> None:
        """Release the fused exchange's peer mesh (collective: every rank)."""
        if self._fh is not None:
            if self.fused:
                self.sync_halo()
                self.fused = False
            torch.cuda.synchronize()
            self._fh.close()
            self._fh = None
            self.graph = None

    def save(self, prefix: str, step: int = 0) -> str:
        """Per-rank checkpoint of the model state (collective; utils.checkpoint).
        Materialises fused-mode halos first, so the files hold consistent fields."""
        from ..utils.checkpoint import save_checkpoint

        self.sync_halo()
        return save_checkpoint(prefix, step=step, T=self.T, T2=self.T2, Cp=self.Cp)

    def restore(self, prefix: str) -> int:
        """Load a checkpoint written by ``save`` on the same decomposition into
        the model's buffers (in place: captured graphs stay valid); returns the
        saved step."""
        from ..utils.checkpoint import load_checkpoint

        meta, f = load_checkpoint(prefix, device=self.device)
        for name in ("T", "T2", "Cp"):
            dst = getattr(self, name)
            if f[name].shape != dst.shape or f[name].dtype != dst.dtype:
                raise ValueError(f"Diffusion3D.restore: {name} is {tuple(f[name].shape)}/{f[name].dtype}, "
                                 f"the model has {tuple(dst.shape)}/{dst.dtype}")
            dst.copy_(f[name])
        self._fprimed = False  # the fused arena does not hold these halos; T's own halo planes do
        self._fentry = True
        return int(meta["step"])

    def clear_error(self) -> None:
        """Reset the fused exchange's sticky timeout word on this rank (after
        a failed fused step was handled, e.g. the fused exchange was dropped)."""
        if self._fh is not None:
            self._fh.clear_error()

    def check(self) -> None:
        """Raise if a fused-exchange sync kernel timed out waiting for a neighbour."""
        if self._fh is not None:
            self._fh.check_error()

    def set_overlap(self, flag: bool) -> bool:
        """Switch between the serial step and the boundary/interior overlapped
        step (needs a GPU model with at least one neighbour); returns the mode."""
        flag = bool(flag) and self.can_overlap
        if flag and self.halo_stream is None:
            if self._reserve_cus > 0:
                from ..utils.streams import cu_partition

                self.compute_stream, self.halo_stream = cu_partition(self._reserve_cus)
            else:
                _least, greatest = torch.cuda.Stream.priority_range()
                self.halo_stream = torch.cuda.Stream(device=self.device, priority=greatest)
        if flag != self.overlap:
            self.graph = None  # a captured schedule no longer matches
        self.overlap = flag
        return flag

    def _overlap_streams(self) -> int:
        """Concurrent streams of the overlapped step: the issuing stream and
        the forked halo stream, plus the CU-masked compute stream of
        ``reserve_cus`` on the put path (RCCL path: one side stream)."""
        if _rccl_transport():
            return 2
        return 3 if self.compute_stream is not None else 2

    def _kw(self, variant=None, rounds=None):
        return dict(lam=self.lam, dt=self.dt, dx=self.dx, dy=self.dy, dz=self.dz,
                    variant=self.variant if variant is None else variant,
                    rounds=self.rounds if rounds is None else rounds)

    def step(self) -> None:
        """Advance one time step (T <- T2 after the update and halo exchange).
        In fused mode the neighbours' stores of this step into this rank's
        arena and fields precede later work on the stream (``_drain``)."""
        self._step()
        self._drain()

    def _drain(self) -> None:
        """Exit barrier of in-kernel synchronised fused steps (collective): the
        last step's neighbour stores (arena, direct-z halo column) are complete
        before anything queued after it touches them (sync_halo, a restore, a
        comparison, gather_). No-op after a sync-kernel step."""
        if self.fused:
            self._fh.drain(torch.cuda.current_stream().cuda_stream)

    def _fused_step_mode(self) -> int:
        # direct z (bit 4) needs the registered field buffers; where they
        # could not be mapped (fields above the IPC limit) the same form runs
        # with the arena z exchange
        return self.fused_mode if self._fh.has_fields else self.fused_mode & ~4

    def _align_form(self) -> None:
        """Before a fused step: if the send mode's receive form changed since
        the last primed step, re-prime. A primed step reads its halos where the
        previous form's senders put them: the arena (arena z), T's z halo
        column (direct z, bit 4; z unpack, bit 64, written by the previous
        step's unpack copy) - a step of another form would read halos nobody
        wrote (switching 8 -> 72 read a stale z column). So the
        halos are materialised (update_halo_(T), collective: mode switches are
        collective) and the next step reads them from T behind an entry
        barrier (bit 16 changes how the neighbours' arrivals are counted)."""
        form = self._fused_step_mode() & (4 | 16 | 64)
        if self._fprimed and self._fform is not None and form != self._fform:
            self.sync_halo()
            self._fentry = True
        self._fform = form

    def _step(self) -> None:
        T, T2, Cp = self.T, self.T2, self.Cp
        if self.fused:
            rd2 = [1.0 / self.dx ** 2, 1.0 / self.dy ** 2, 1.0 / self.dz ** 2]
            s = torch.cuda.current_stream().cuda_stream
            self._align_form()  # (sync_halo leaves the buffer roles in place)
            mode = self._fused_step_mode()
            if self.timer is not None:
                with self.timer.phase("stencil+exchange"):
                    self._fh.step(T2.data_ptr(), T.data_ptr(), Cp.data_ptr(), rd2, self.dt * self.lam,
                                  self.fused_variant, self._fstep, self._fprimed, s, self.fused_rounds,
                                  mode, self._fentry, HALO_Z)
            else:
                self._fh.step(T2.data_ptr(), T.data_ptr(), Cp.data_ptr(), rd2, self.dt * self.lam,
                              self.fused_variant, self._fstep, self._fprimed, s, self.fused_rounds,
                              mode, self._fentry, HALO_Z)
            self._fentry = False
            self._fstep += 1
            self._fprimed = True
        elif self.overlap and _serial_overlap(self._overlap_streams()):
            # Fewer hardware queues per process than concurrent streams in the
            # overlapped step (GPU_MAX_HW_QUEUES=1, e.g. many ranks sharing a
            # GPU): the streams cannot all run concurrently, and a hipGraph
            # captured with the forked exchange crashed in replay with one
            # queue (profiles/r4_overlap_crash/). Same three parts in stream
            # order - identical results (disjoint writes), nothing lost.
            stencil.diffusion3d_(T2, T, Cp, boxes=self.slabs, **self._kw(self.halo_variant, self.halo_rounds))
            update_halo_(T2)
            stencil.diffusion3d_(T2, T, Cp, boxes=[self.interior], **self._kw(None, self.interior_rounds))
        elif self.overlap:
            # 1. boundary slabs on the compute stream (full bandwidth, nothing
            #    else running), 2. the halo exchange of T2 on the high-priority
            #    stream after an event, 3. the interior concurrently on the
            #    compute stream; slabs/interior/halo planes are disjoint.
            main = torch.cuda.current_stream()
            hs = self.halo_stream
            cs = self.compute_stream or main
            stencil.diffusion3d_(T2, T, Cp, boxes=self.slabs, **self._kw(self.halo_variant, self.halo_rounds))
            if _rccl_transport():
                # RCCL's p2p group must run on the stream the step was issued
                # on: captured on a stream forked from the capture origin it
                # crashes hipGraph capture (RCCL 2.26, SIGSEGV at the end of
                # the capture); on the origin, with the interior on a forked
                # stream running concurrently, it captures and replays
                # (benchmarks/rccl_capture_repro.py, profiles/r2_rccl_capture/).
                # So the roles swap: interior on the side stream, exchange here.
                side = cs if cs is not main else hs
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    stencil.diffusion3d_(T2, T, Cp, boxes=[self.interior], **self._kw(None, self.interior_rounds))
                update_halo_(T2)
                main.wait_stream(side)
            else:
                hs.wait_stream(main)
                if cs is not main:
                    cs.wait_stream(main)
                with torch.cuda.stream(hs):
                    update_halo_(T2)
                with torch.cuda.stream(cs):
                    stencil.diffusion3d_(T2, T, Cp, boxes=[self.interior], **self._kw(None, self.interior_rounds))
                main.wait_stream(hs)
                if cs is not main:
                    main.wait_stream(cs)
        elif self.timer is not None:
            with self.timer.phase("stencil"):
                stencil.diffusion3d_(T2, T, Cp, boxes=self.inner, halo_z=self.halo_z, **self._kw())
            with self.timer.phase("update_halo"):
                update_halo_(T2)
        else:
            # halo_z: T2's z halo gets T's values (whole-line z-edge stores):
            # at a physical boundary both hold the same fixed values, and
            # update_halo_(T2) right after rewrites every exchanged one
            stencil.diffusion3d_(T2, T, Cp, boxes=self.inner, halo_z=self.halo_z, **self._kw())
            update_halo_(T2)
        self.T, self.T2 = T2, T
        self._warm = True

    def local_step(self) -> None:
        """One step of the LOCAL problem: what a rank without neighbours runs
        (the N = 1 run of the weak-scaling curve): the plain stencil with this
        model's variant, grid rounds and z-edge store form on the whole
        interior; update_halo_ with PROC_NULL neighbours is a no-op
        (reference: src/update_halo.jl:40-42, no neighbour -> nothing sent).
        Used by the bench's same-process efficiency E = t(local) / t(step).
        Leaves the halo planes unexchanged: timing only (callers that go on
        with real steps call ``exchange_halos`` afterwards)."""
        T, T2 = self.T, self.T2
        stencil.diffusion3d_(T2, T, self.Cp, boxes=self.inner, halo_z=self.halo_z, **self._kw())
        self.T, self.T2 = T2, T

    def capture(self, steps: int = None) -> None:
        """Record ``steps`` (even, default GRAPH_STEPS) time steps in a hipGraph for ``run``.

        A step is a chain of launches (stencil, pack, RCCL group, unpack per
        dimension; or fused stencil + sync) whose gaps are host launch latency;
        replaying a graph removes that latency, and a graph replay costs ~9 us
        to launch on MI355X (profiles/r1_fused/), so several steps are captured
        per graph. An even count puts the ping-pong buffers back in their roles
        after every replay. Needs one eager step first (halo buffers, plan
        cache and kernel variant are set up outside the capture); ``capture``
        performs that step itself if none ran yet (and one fused step if the
        fused arena does not hold T's halos).
        """
        steps = GRAPH_STEPS if steps is None else int(steps)
        if steps < 2 or steps % 2:
            raise ValueError("Diffusion3D.capture: steps must be even and >= 2")
        if self.device.type != "cuda":
            raise RuntimeError("Diffusion3D.capture: hipGraphs need a GPU model")
        if not self._warm:
            self.step()
        if self.fused:
            self._align_form()  # no re-priming inside the capture
        if self.fused and not self._fprimed:
            self.step()  # captured fused steps read the arena: it must hold T's halos
        def record():
            for _ in range(steps):
                self._step()  # no exit barrier inside the graph: run() drains once

        self.graph = None
        # fused steps exchange through their own peer mesh, not update_halo_
        g = capture_graph(record, f"{type(self).__name__}.capture", uses_halo=not self.fused)
        self.graph = g
        self.graph_steps = steps
        self._graph_fused = self.fused
        self._graph_cfg = self._fused_cfg()
        self._graph_parity = self._fstep % 2
        self._graph_T = self.T.data_ptr()

    def run(self, nt: int) -> None:
        """Advance ``nt`` steps (by graph replays of ``graph_steps`` steps if
        captured); in fused mode one exit barrier at the end (``_drain``)."""
        ran = nt > 0
        if self.graph is not None and self._graph_fused == self.fused and self._graph_cfg == self._fused_cfg():
            # The captured steps have their buffer roles baked in (T of the
            # capture is read first) and, fused, their arena halves too: they
            # assume a primed arena, no pending entry barrier and the
            # step-counter parity of the capture. Eager steps realign (at most
            # two; a mode switch between captures can make the two parities
            # disagree for good: then the rest runs eagerly).
            for _ in range(2):
                if nt == 0 or self._graph_ready():
                    break
                self._step()
                nt -= 1
            if self._graph_ready():
                k = self.graph_steps
                for _ in range(nt // k):
                    self.graph.replay()
                if self.fused:
                    self._fstep += k * (nt // k)
                nt %= k
        for _ in range(nt):
            self._step()
        if ran:
            self._drain()

    def _fused_cfg(self):
        """The fused kernel form a captured graph bakes in (a graph of another
        form is not replayed: the steps run eagerly until the next capture)."""
        return (self.fused_variant, self.fused_mode, self.fused_rounds) if self.fused else None

    def _graph_ready(self) -> bool:
        if self.T.data_ptr() != self._graph_T:
            return False
        if self.fused:
            return self._fstep % 2 == self._graph_parity and self._fprimed and not self._fentry
        return True

    @property
    def a_eff_bytes(self) -> int:
        """A_eff = (2*D_u + D_k) * n_local * sizeof(T) with D_u = D_k = 1."""
        return 3 * self.T.numel() * self.T.element_size()


def _hw_queues() -> int | None:
    """Hardware queues per process of the HIP runtime (GPU_MAX_HW_QUEUES,
    parsed as an integer: ' 01' is 1); None = the runtime's default (4)."""
    v = os.environ.get("GPU_MAX_HW_QUEUES", "").strip()
    try:
        return int(v) if v else None
    except ValueError:
        return None


def _serial_overlap(streams: int) -> bool:
    """Run the overlapped step's parts in stream order when the process has
    fewer hardware queues than the step has concurrent streams: they could
    not run concurrently anyway, and a captured fork in a one-queue process
    crashed the runtime's graph replay (profiles/r4_overlap_crash/: 2 side
    streams at GPU_MAX_HW_QUEUES=1; the full cell table is in its NOTES)."""
    q = _hw_queues()
    return q is not None and q < streams


def _make_fused_halo(m: "Diffusion3D"):
    """Native FusedHalo over a dedicated peer mesh (collective over the grid)."""
    from .._native import native

    gg = _grid.global_grid()
    nb = [[int(gg.neighbors[s, d]) for s in range(2)] for d in range(3)]
    if gg.nprocs > 1:
        mesh = native.PeerMesh(gg.comm.rank, gg.comm.size, gg.comm._allgather_bytes)
    else:  # periodic / loopback single process: every neighbour is this rank
        nb = [[0 if v >= 0 else -1 for v in row] for row in nb]
        mesh = native.PeerMesh(0, 1, lambda b: [bytes(b)])
    return native.FusedHalo(mesh, list(m.T.shape), m.T.element_size(), nb)


def _ipc_limit() -> int:
    """Allocation size from which IPC export is refused (csrc/include/igg/ipc.hpp)."""
    from .._native import native

    return int(native.IPC_MAX_BYTES)


def _carve(tensors, gap: int, kind=None, split_at=None, device=None, split_kind=None):
    """Copies of equally sized tensors placed in one buffer ``gap`` bytes apart.
    ``kind``: None = torch's caching allocator, else a native MemKind (1 =
    fine-grained, 4 = HIP VMM) allocated by the runtime and handed over through
    DLPack. ``split_at``: if the one buffer would reach this many bytes, one
    allocation per tensor instead (the IPC size limit), of MemKind
    ``split_kind`` if given. Meta tensors give shape and dtype only:
    uninitialised views on ``device``."""
    nbytes = tensors[0].numel() * tensors[0].element_size()
    stride = nbytes + gap
    device = tensors[0].device if device is None else device
    if split_at is not None and stride * len(tensors) >= split_at and len(tensors) > 1:
        k = kind if split_kind is None else split_kind
        return [_carve([t], 0, k, device=device)[0] for t in tensors]
    if kind is None:
        buf = torch.empty(stride * len(tensors), dtype=torch.uint8, device=device)
    else:
        buf = native_buffer(stride * len(tensors), kind, device)
    out = []
    for k, t in enumerate(tensors):
        v = buf[k * stride:k * stride + nbytes].view(t.dtype).view(t.shape)
        if t.device.type != "meta":
            v.copy_(t)
        out.append(v)
    return out


def _placed_fields(carve, gg, meta: torch.Tensor, device):
    """(T, Cp, T2) from ``carve()``, the fastest of several candidate carves
    (utils/placement.py), and the probe's record (None without a probe)."""
    nbytes = meta.numel() * meta.element_size()
    k = _placement.candidate_count(gg, nbytes, 3 * nbytes, device)
    return _placement.placed(carve, k, lambda cands: _time_placements(cands, meta.dtype))


def _time_placements(cands, dtype, v=None, rounds: int = 3, halo_z: bool = False, steps: int = 6) -> list:
    """Median ms per ping-pong step of each (T, Cp, T2) candidate with a fixed
    plain variant (43 f64 / 14 f32 without whole-line z stores: separates fast
    from slow carves by 4.5-5 %, benchmarks/placement_probe.py). Values: T = 0,
    Cp = 1 (the model writes its initial conditions afterwards)."""
    if v is None:
        v = 43 if dtype == torch.float64 else 14
    if not stencil.native.diffusion3d_variant_compiled(v):
        v = stencil.compiled_variants()[0]
    for T, Cp, T2 in cands:
        T.zero_()
        T2.zero_()
        Cp.fill_(1)
    shape = list(cands[0][0].shape)
    boxes = [(list(b[0]), list(b[1])) for b in [stencil.inner_box(shape)]]
    s = torch.cuda.current_stream()
    es = cands[0][0].element_size()

    def launch(c, j):
        T, Cp, T2 = c
        dst, src = (T2, T) if j % 2 == 0 else (T, T2)
        stencil.native.diffusion3d(dst.data_ptr(), src.data_ptr(), Cp.data_ptr(), shape, [1.0, 1.0, 1.0], 1e-3,
                                   es, boxes, True, v, s.cuda_stream, rounds, halo_z)

    return _placement.time_candidates(cands, launch, steps=steps)


def native_buffer(nbytes: int, kind: int, device) -> torch.Tensor:
    """1-D uint8 device tensor of ``nbytes`` in native memory of MemKind
    ``kind`` (csrc/include/igg/ipc.hpp), owned by torch (freed with it)."""
    from torch.utils import dlpack

    from .._native import native

    with torch.cuda.device(device):
        return dlpack.from_dlpack(native.alloc_dlpack(int(nbytes), int(kind)))


def _choose_variant(m: "Diffusion3D") -> int:
    """Kernel variant for this model: IGG_STENCIL_VARIANT if it is an integer,
    else the fastest of the shortlist timed on the model's own arrays, summed
    over all ranks so every rank runs the same kernel."""
    import os

    env = os.environ.get("IGG_STENCIL_VARIANT", "auto").strip().lower()
    if env != "auto":
        return int(env)
    rd2 = [1.0 / m.dx ** 2, 1.0 / m.dy ** 2, 1.0 / m.dz ** 2]
    boxes = [(list(b[0]), list(b[1])) for b in m.inner]
    gg = _grid.global_grid()

    def summed(t: dict):
        cands = sorted(t)
        tot = torch.tensor([t[c] for c in cands], dtype=torch.float64)
        if gg.nprocs > 1:
            import torch.distributed as dist

            dist.all_reduce(tot, group=gg.comm.gloo)
        return cands, tot

    # Stage 1: every (variant, rounds, z-edge store form) on fixed buffers
    # (T2 = f(T), cheap). The whole-line form (halo_z) wins for most tilings
    # and costs tiling 11 2.7 % (profiles/r4_halo_z/), so both are timed.
    forms = (True, False) if HALO_Z else (False,)
    t = stencil.time_variants(m.T2, m.T, m.Cp, rd2, m.dt * m.lam, boxes,
                              [(v, r, hz) for v in stencil.SHORTLIST for r in stencil.GRID_ROUNDS for hz in forms])
    cands, tot = summed(t)

    def key(v, r, hz):
        return f"{v}@r{r}" + ("/hz" if hz else "")

    m.variant_times = {key(*c): round(float(x) / max(1, int(gg.nprocs)), 5) for c, x in zip(cands, tot)}
    # Stage 2: the stage-1 front again, in the time loop's ping-pong shape and
    # with more launches: the minimum over ~44 noisy fixed-buffer timings is
    # biased low and the alternating buffers cost ~1 % (profiles/r2_gap/), so
    # the pick is made on what the run actually does.
    front = [cands[i] for i in torch.argsort(tot)[:PINGPONG_FRONT].tolist()]
    # 5 interleaved rounds of 20 steps, medians: the front differs by less
    # than the box noise of one sample (the round-4 picks varied run to run)
    t2 = stencil.time_variants_pingpong(m.T2, m.T, m.Cp, rd2, m.dt * m.lam, boxes, front, steps=20, rounds=5)
    cands2, tot2 = summed(t2)
    m.variant_times.update({key(*c) + "/pp": round(float(x) / max(1, int(gg.nprocs)), 5)
                            for c, x in zip(cands2, tot2)})
    v, r, hz = cands2[int(torch.argmin(tot2))]
    m.rounds = int(r)
    m.halo_z = bool(hz)
    return int(v)


def t_eff_gbs(model: Diffusion3D, t_it: float) -> float:
    return model.a_eff_bytes / t_it / 1e9


def run_diffusion3d(nx=128, ny=128, nz=128, nt=100, **kw):
    """Example driver mirroring diffusion3D_multicpu_novis.jl / _multigpu_ (novis)."""
    from ..parallel.grid import finalize_global_grid, init_global_grid
    from ..utils.tools import tic, toc

    init_global_grid(nx, ny, nz, quiet=kw.pop("quiet", False))
    m = Diffusion3D(**kw)
    tic()
    m.run(nt)
    t = toc()
    finalize_global_grid()
    return m, t
