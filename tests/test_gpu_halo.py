"""GPU halo updates (HIP pack/unpack/self-periodic kernels) against the oracle
of test/test_update_halo.jl:748-1053 — bitwise equality, no tolerance."""
import pytest
import torch

import igg
from tests.helpers import encode, zero_boundaries

pytestmark = pytest.mark.gpu

nx, ny, nz = 7, 5, 6


def _check(fields, refs, gpu):
    for A, R in zip(fields, refs):
        assert not torch.equal(A.cpu(), R)
    igg.update_halo_(*fields)
    torch.cuda.synchronize()
    for A, R in zip(fields, refs):
        assert torch.equal(A.cpu(), R)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32, torch.float16, torch.complex64, torch.complex128])
@pytest.mark.parametrize("shape_delta", [(0, 0, 0), (1, 0, 0), (0, 1, 0), (0, 0, 1), (2, -1, 1)])
def test_gpu_periodic_3d(gpu, dtype, shape_delta):
    igg.init_global_grid(nx, ny, nz, periodx=1, periody=1, periodz=1, quiet=True, init_MPI=False)
    shape = tuple(n + d for n, d in zip((nx, ny, nz), shape_delta))
    A = torch.zeros(shape, dtype=dtype)
    encode(A, complex_factor=(1 + 1j) if dtype.is_complex else None)
    R = A.clone()
    Ag = zero_boundaries(A.clone()).to(gpu)
    if shape_delta == (2, -1, 1):  # no halo in y: only the x/z boundaries are restored
        igg.update_halo_(Ag)
        torch.cuda.synchronize()
        assert torch.equal(Ag.cpu()[:, 1:-1, :], R[:, 1:-1, :])
        assert (Ag.cpu()[:, [0, -1], :] == 0).all()
    else:
        _check([Ag], [R], gpu)
    igg.finalize_global_grid(finalize_MPI=False)


def test_gpu_two_fields_and_overlap(gpu):
    igg.init_global_grid(nx, ny, nz, periodx=1, periody=1, periodz=1, overlapx=3, overlapz=3, quiet=True,
                         init_MPI=False)
    Vz = encode(torch.zeros(nx, ny, nz + 1, dtype=torch.float64))
    Vx = encode(torch.zeros(nx + 1, ny, nz, dtype=torch.float64))
    refs = [Vz.clone(), Vx.clone()]
    fs = [zero_boundaries(Vz.clone()).to(gpu), zero_boundaries(Vx.clone()).to(gpu)]
    _check(fs, refs, gpu)
    igg.finalize_global_grid(finalize_MPI=False)


def test_gpu_permuted_layout(gpu):
    """A field stored x-fastest (Julia/Fortran order) works via strides."""
    igg.init_global_grid(nx, ny, nz, periodx=1, periody=1, periodz=1, quiet=True, init_MPI=False)
    base = torch.zeros(nz, ny, nx, dtype=torch.float64)
    A = base.permute(2, 1, 0)  # logical (x,y,z), x contiguous
    encode(A)
    R = A.clone()
    Ag = zero_boundaries(A.clone().permute(2, 1, 0).contiguous().permute(2, 1, 0)).to(gpu)
    assert Ag.stride()[0] == 1
    igg.update_halo_(Ag)
    torch.cuda.synchronize()
    assert torch.equal(Ag.cpu(), R)
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.parametrize("ndim", [1, 2])
def test_gpu_periodic_1d_2d(gpu, ndim):
    if ndim == 1:
        igg.init_global_grid(nx, 1, 1, periodx=1, quiet=True, init_MPI=False)
        A = encode(torch.zeros(nx + 1, dtype=torch.float64))
    else:
        igg.init_global_grid(nx, ny, 1, periodx=1, periody=1, quiet=True, init_MPI=False)
        A = encode(torch.zeros(nx, ny + 1, dtype=torch.float64))
    R = A.clone()
    _check([zero_boundaries(A.clone()).to(gpu)], [R], gpu)
    igg.finalize_global_grid(finalize_MPI=False)


def test_gpu_large_faces(gpu):
    """Faces bigger than one copy block; exercises the batched copy kernel."""
    n = (130, 67, 257)
    igg.init_global_grid(*n, periodx=1, periody=1, periodz=1, quiet=True, init_MPI=False)
    A = encode(torch.zeros(n, dtype=torch.float64))
    R = A.clone()
    _check([zero_boundaries(A.clone()).to(gpu)], [R], gpu)
    igg.finalize_global_grid(finalize_MPI=False)


def test_gpu_diffusion_matches_reference(gpu):
    from igg.models.diffusion3d import Diffusion3D
    from igg.ops import stencil

    igg.init_global_grid(40, 33, 70, periodx=1, periodz=1, quiet=True, init_MPI=False)
    for dtype, tol in ((torch.float64, 1e-11), (torch.float32, 2e-3)):
        m = Diffusion3D(dtype=dtype)
        ref = m.T.cpu().double()
        for _ in range(3):
            ref = stencil.diffusion3d_reference(ref, m.Cp.cpu().double(), lam=m.lam, dt=m.dt, dx=m.dx, dy=m.dy, dz=m.dz)
            igg.update_halo_(ref)
            m.step()
        torch.cuda.synchronize()
        d = (m.T.cpu().double() - ref).abs()
        err = d.max().item()
        bad = (~(d < tol)).nonzero()
        assert err < tol, (dtype, err, f"variant {m.variant} rounds {m.rounds} overlap {m.overlap}",
                           f"{len(bad)} bad cells, first {bad[:6].tolist()}", m.variant_times)
    igg.finalize_global_grid(finalize_MPI=False)


def test_gpu_gather_single(gpu):
    igg.init_global_grid(nx, ny, nz, quiet=True, init_MPI=False)
    A = torch.arange(nx * ny * nz, dtype=torch.float64, device=gpu).view(nx, ny, nz)
    G = torch.zeros(nx, ny, nz, dtype=torch.float64, device=gpu)
    igg.gather_(A, G)
    torch.cuda.synchronize()
    assert torch.equal(A, G)
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.parametrize("s,dims,dtype", [
    ((3, 4, 5), (2, 3, 2), torch.float32),      # 20-byte rows: element path
    ((3, 4, 8), (2, 3, 2), torch.float32),      # 32-byte rows: 16-byte units
    ((5, 3, 7), (1, 2, 3), torch.float16),      # 2-byte elements, odd rows
    ((4, 6, 130), (2, 2, 2), torch.float64),    # rows longer than one wave pass
    ((2, 3, 300), (2, 1, 3), torch.complex128),  # 16-byte elements
    ((7, 1, 1), (3, 1, 1), torch.int16),        # 1-element rows
])
def test_gpu_gather_reorder_kernel(gpu, s, dims, dtype):
    """The root-side block reorder kernel (one wave per row) vs a torch permute."""
    from igg._native import native

    nb = dims[0] * dims[1] * dims[2]
    n = s[0] * s[1] * s[2]
    src = torch.arange(nb * n, dtype=torch.float64, device=gpu).to(dtype)
    dst = torch.full((nb * n,), -1, dtype=torch.float64, device=gpu).to(dtype)
    native.gather_reorder(src.data_ptr(), dst.data_ptr(), list(s), list(dims), src.element_size(),
                          torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ref = src.view(*dims, *s).permute(0, 3, 1, 4, 2, 5).reshape(-1)
    assert torch.equal(dst, ref)


def _native_fields(*ts):
    from igg.parallel.halo import field_tuple

    return [field_tuple(t) for t in ts]


def test_gpu_rccl_remote_path_via_self_peer(gpu):
    """Full remote exchange path on RCCL in one process: the engine believes it
    is rank 1 while both neighbours in every dim are rank 0, so every face goes
    pack -> grouped ncclSend/ncclRecv (peer 0 = this process) -> unpack, with
    left == right == same peer (the dims==2 periodic ordering case)."""
    from igg._native import native

    n = (9, 7, 8)
    igg.init_global_grid(*n, periodx=1, periody=1, periodz=1, quiet=True, init_MPI=False)
    A = encode(torch.zeros(n[0], n[1], n[2] + 1, dtype=torch.float64))
    B = encode(torch.zeros(n[0] + 1, n[1], n[2], dtype=torch.float64))
    refs = [A.clone(), B.clone()]
    Ag, Bg = zero_boundaries(A.clone()).to(gpu), zero_boundaries(B.clone()).to(gpu)
    gi = native.GridInfo(1, 2, list(n), [2, 2, 2], [[0, 0, 0], [0, 0, 0]])
    eng = native.HaloEngine(gi)
    comm = native.RcclComm(native.RcclComm.unique_id(), 1, 0)
    eng.set_transport(comm, True)
    eng.exchange(_native_fields(Ag, Bg), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    comm.check_async_error()
    assert torch.equal(Ag.cpu(), refs[0])
    assert torch.equal(Bg.cpu(), refs[1])
    del eng, comm
    igg.finalize_global_grid(finalize_MPI=False)


def test_gpu_rccl_p2p_and_barrier(gpu):
    from igg._native import native

    comm = native.RcclComm(native.RcclComm.unique_id(), 1, 0)
    src = torch.arange(1000, dtype=torch.float32, device=gpu)
    dst = torch.zeros_like(src)
    s = torch.cuda.current_stream().cuda_stream
    comm.p2p([(dst.data_ptr(), 4000, 0)], [(src.data_ptr(), 4000, 0)], s)
    comm.barrier(s)
    torch.cuda.synchronize()
    assert torch.equal(src, dst)
    assert native.rccl_version().count(".") == 2


@pytest.mark.parametrize("mode", ["sequential", "onephase"])
def test_gpu_loopback_both_schedules(gpu, mode):
    """Loopback: every face/edge/corner through the RCCL remote path; both
    schedules must reproduce the periodic oracle bitwise."""
    from igg.parallel import halo as H

    n = (10, 9, 12)
    igg.init_global_grid(*n, periodx=1, periody=1, periodz=1, quiet=True, init_MPI=False)
    H.enable_loopback()
    H.set_halo_mode(mode)
    A = encode(torch.zeros(n[0] + 1, n[1], n[2], dtype=torch.float64))
    B = encode(torch.zeros(n[0], n[1], n[2] + 1, dtype=torch.float64))
    refs = [A.clone(), B.clone()]
    Ag, Bg = zero_boundaries(A.clone()).to(gpu), zero_boundaries(B.clone()).to(gpu)
    igg.update_halo_(Ag, Bg)
    torch.cuda.synchronize()
    assert torch.equal(Ag.cpu(), refs[0]) and torch.equal(Bg.cpu(), refs[1])
    if mode == "onephase":
        assert H.engine().last_message_count == 52  # 26 directions x 2 fields
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.parametrize("mode", ["sequential", "onephase"])
def test_gpu_graph_replay_matches_eager(gpu, mode):
    """A hipGraph of two diffusion steps (stencil + pack + RCCL + unpack, loopback
    so every face takes the remote path) replays bitwise like eager steps."""
    from igg.models.diffusion3d import Diffusion3D
    from igg.parallel import halo as H

    n = (40, 36, 70)
    igg.init_global_grid(*n, periodx=1, periody=1, periodz=1, quiet=True, init_MPI=False)
    H.enable_loopback()
    H.set_halo_mode(mode)
    a = Diffusion3D(dtype=torch.float64)
    b = Diffusion3D(dtype=torch.float64)
    a.run(7)
    b.step()
    b.capture(steps=4)  # graph of four steps; b has done 1 eager step
    b.run(6)  # one replay + two eager steps
    torch.cuda.synchronize()
    assert b.graph is not None
    assert torch.equal(a.T, b.T)
    igg.finalize_global_grid(finalize_MPI=False)


def test_gpu_loopback_put_transport(gpu, monkeypatch):
    """Loopback through the put transport: every message is a put into the own
    IPC-exportable arena + device-side flag signalling; periodic oracle,
    bitwise, over several exchanges (both arena halves, epoch-2 reuse), eager,
    overlapped and replayed from a hipGraph."""
    from igg.models.diffusion3d import Diffusion3D
    from igg.parallel import halo as H

    monkeypatch.setenv("IGG_TRANSPORT", "put")
    n = (10, 9, 12)
    igg.init_global_grid(*n, periodx=1, periody=1, periodz=1, quiet=True, init_MPI=False)
    H.enable_loopback()
    for _ in range(3):
        A = encode(torch.zeros(n[0] + 1, n[1], n[2], dtype=torch.float64))
        B = encode(torch.zeros(n[0], n[1], n[2] + 1, dtype=torch.float64))
        refs = [A.clone(), B.clone()]
        Ag, Bg = zero_boundaries(A.clone()).to(gpu), zero_boundaries(B.clone()).to(gpu)
        igg.update_halo_(Ag, Bg)
        torch.cuda.synchronize()
        assert torch.equal(Ag.cpu(), refs[0]) and torch.equal(Bg.cpu(), refs[1])
    assert H.engine().last_message_count == 52
    # the model (eager, serial and overlapped) matches the RCCL-free periodic run
    m1 = Diffusion3D(dtype=torch.float64)
    m2 = Diffusion3D(dtype=torch.float64, overlap=True)
    m3 = Diffusion3D(dtype=torch.float64)
    m1.run(7)
    m2.run(7)
    m3.step()
    m3.capture(steps=2)  # epoch lives on the device: replays are valid exchanges
    m3.run(6)
    torch.cuda.synchronize()
    assert torch.equal(m1.T, m2.T)
    assert torch.equal(m1.T, m3.T)
    mesh = H._loopback_comm.mesh
    mesh.check_error()
    assert mesh.epoch >= 3 + 3 * 7
    igg.finalize_global_grid(finalize_MPI=False)


def test_gpu_loopback_auto_transport(gpu, monkeypatch):
    """IGG_TRANSPORT=auto in the loopback emulation: both loopback transports
    exist side by side; the first exchange of each field-set signature checks
    them against each other (periodic: the values are defined), times both and
    keeps the faster; later exchanges reuse it, bitwise on the periodic
    oracle. A one-sided emulated shape (a corner rank) only times them."""
    from igg.parallel import halo as H

    monkeypatch.setenv("IGG_TRANSPORT", "auto")
    n = (10, 9, 12)
    igg.init_global_grid(*n, periodx=1, periody=1, periodz=1, quiet=True, init_MPI=False)
    H.enable_loopback()
    assert H.auto_transport()
    for _ in range(3):
        A = encode(torch.zeros(n[0] + 1, n[1], n[2], dtype=torch.float64))
        B = encode(torch.zeros(n[0], n[1], n[2] + 1, dtype=torch.float64))
        refs = [A.clone(), B.clone()]
        Ag, Bg = zero_boundaries(A.clone()).to(gpu), zero_boundaries(B.clone()).to(gpu)
        igg.update_halo_(Ag, Bg)
        torch.cuda.synchronize()
        assert torch.equal(Ag.cpu(), refs[0]) and torch.equal(Bg.cpu(), refs[1])
    log = H.tuned_transports()
    assert len(log) == 1, log
    assert log[0]["checked"] == {"rccl": "ok", "put": "ok"}, log
    assert log[0]["chosen"] == min(log[0]["ms"], key=log[0]["ms"].get)
    assert H.transport_name() == log[0]["chosen"]
    H.check_transport()
    # a corner rank's shape: timed only
    H.set_halo_mode("sequential")
    igg.get_global_grid()  # (the grid's table is rewritten by enable_loopback)
    import igg.parallel.grid as G

    G.global_grid().neighbors[:, :] = -1
    H.enable_loopback(((False, True),) * 3)
    X = torch.rand(n, dtype=torch.float64, device=gpu)
    igg.update_halo_(X)
    torch.cuda.synchronize()
    rec = H.tuned_transports()[-1]
    assert "timed only" in rec.get("reason", ""), rec
    assert rec["chosen"] in ("rccl", "put")
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.parametrize("transport", ["rccl", "put"])
def test_gpu_debug_sync_phases(gpu, monkeypatch, transport):
    """IGG_DEBUG_SYNC=1 drains and checks the stream after every phase of
    every schedule; results stay bitwise."""
    from igg.parallel import halo as H

    monkeypatch.setenv("IGG_DEBUG_SYNC", "1")
    monkeypatch.setenv("IGG_TRANSPORT", transport)
    n = (9, 8, 10)
    igg.init_global_grid(*n, periodx=1, periody=1, periodz=1, quiet=True, init_MPI=False)
    H.enable_loopback()
    for mode in (["sequential", "onephase"] if transport == "rccl" else ["auto"]):
        H.set_halo_mode(mode)
        A = encode(torch.zeros(*n, dtype=torch.float32))
        ref = A.clone()
        Ag = zero_boundaries(A.clone()).to(gpu)
        igg.update_halo_(Ag)
        assert torch.equal(Ag.cpu(), ref)
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32, torch.complex128])
@pytest.mark.parametrize("loopback", [False, True])
def test_gpu_pack_memcpy2d(gpu, dtype, loopback):
    """IGG_PACK=memcpy2d (hipMemcpy2DAsync for faces with contiguous rows,
    the kernel for the others) gives the same halos as the copy kernel:
    self-periodic in-place path and the loopback pack -> transport -> unpack
    path, sequential schedule, staggered fields in one call."""
    from igg.parallel import halo as H

    igg.init_global_grid(nx, ny, nz, periodx=1, periody=1, periodz=1, quiet=True, init_MPI=False)
    if loopback:
        H.enable_loopback()
    H.set_halo_mode("sequential")
    H.set_pack_mode("memcpy2d")
    assert [H.pack_mode(d) for d in (1, 2, 3)] == ["memcpy2d"] * 3
    cf = (1 + 1j) if dtype.is_complex else None
    fs = [encode(torch.zeros(s, dtype=dtype), complex_factor=cf) for s in ((nx, ny, nz), (nx + 1, ny, nz),
                                                                           (nx, ny, nz + 1))]
    refs = [A.clone() for A in fs]
    _check([zero_boundaries(A.clone()).to(gpu) for A in fs], refs, gpu)
    H.set_pack_mode("kernel", dims=(False, True, False))
    assert [H.pack_mode(d) for d in (1, 2, 3)] == ["memcpy2d", "kernel", "memcpy2d"]
    _check([zero_boundaries(A.clone()).to(gpu) for A in fs], refs, gpu)
    igg.finalize_global_grid(finalize_MPI=False)


def test_gpu_pack_memcpy2d_in_graph(gpu):
    """memcpy2d face copies are captured as graph memcpy nodes and replay."""
    from igg.parallel import halo as H

    igg.init_global_grid(16, 12, 10, periodx=1, periody=1, periodz=1, quiet=True, init_MPI=False)
    H.set_pack_mode("memcpy2d")
    A = encode(torch.zeros(16, 12, 10, dtype=torch.float64))
    R = A.clone()
    X = zero_boundaries(A.clone()).to(gpu)
    igg.update_halo_(X)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        igg.update_halo_(X)
    torch.cuda.synchronize()
    H.register_graph(g)
    X.copy_(zero_boundaries(A.clone()).to(gpu))
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(X.cpu(), R)
    del g
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.parametrize("transport", ["rccl", "put"])
def test_gpu_overlap_capture(gpu, monkeypatch, transport):
    """Overlapped step (boundary slabs, exchange and interior on two streams)
    captured in a hipGraph replays bitwise like serial eager steps, with both
    transports. RCCL runs its group on the capture-origin stream and the
    interior on the forked stream (RCCL on a forked stream crashed the
    capture: benchmarks/rccl_capture_repro.py)."""
    from igg.models.diffusion3d import Diffusion3D
    from igg.parallel import halo as H

    monkeypatch.setenv("IGG_TRANSPORT", transport)
    igg.init_global_grid(24, 22, 40, periodx=1, periody=1, periodz=1, quiet=True, init_MPI=False)
    H.enable_loopback()
    assert H.transport_name() == transport
    a = Diffusion3D(dtype=torch.float64)
    b = Diffusion3D(dtype=torch.float64, overlap=True)
    assert b.overlap
    a.run(7)
    b.step()
    b.capture(steps=2)
    assert b.graph is not None
    b.run(6)
    torch.cuda.synchronize()
    assert torch.equal(a.T, b.T)
    igg.finalize_global_grid(finalize_MPI=False)


def test_gpu_auto_mode_picks_the_timed_winner(gpu):
    """'auto' times sequential vs one-phase on the first eager exchange of a
    field set that reaches other ranks (here: the RCCL loopback) and keeps the
    faster for that field set; results stay bitwise."""
    from igg.parallel import halo as H

    n = (40, 36, 32)
    igg.init_global_grid(*n, periodx=1, periody=1, periodz=1, quiet=True, init_MPI=False)
    H.enable_loopback()
    assert H.halo_mode() == "auto"
    before = len(H.tuned_modes())
    A = encode(torch.zeros(*n, dtype=torch.float64))
    ref = A.clone()
    Ag = zero_boundaries(A.clone()).to(gpu)
    igg.update_halo_(Ag)
    assert torch.equal(Ag.cpu(), ref)
    log = H.tuned_modes()
    assert len(log) == before + 1
    times, win = log[-1]
    assert set(times) == {"sequential", "onephase"}
    assert win == min(times, key=times.get)
    assert H.plan_mode(Ag) == win
    igg.update_halo_(Ag)  # cached: no second measurement
    assert len(H.tuned_modes()) == before + 1
    H.set_halo_mode("onephase")  # an explicit mode wins over the measurement
    assert H.plan_mode(Ag) == "onephase"
    igg.finalize_global_grid(finalize_MPI=False)


def test_gpu_bounded_sync_raises_instead_of_hanging(gpu):
    """A kernel that does not finish (stand-in: a 4 s spin, like an RCCL kernel
    waiting on a dead peer) makes the bounded device wait raise after its
    timeout instead of blocking; once the kernel ends the GPU drains normally."""
    import time

    from igg import native
    from igg.parallel.comm import bounded_device_sync

    s = torch.cuda.Stream()
    native.gpu_spin(4.0, s.cuda_stream)
    t0 = time.time()
    with pytest.raises(igg.IGGError, match="did not drain"):
        bounded_device_sync(timeout=1.0, what="test")
    assert 0.9 <= time.time() - t0 < 3.5
    bounded_device_sync(timeout=30.0, what="test")
    assert time.time() - t0 >= 3.5


def test_gpu_bounded_stream_sync(gpu):
    """The timed regions' stream wait (native event poll): raises after its
    bound while a kernel on that stream still runs, returns promptly once it
    is done, and costs little on an idle stream."""
    import time

    from igg import native
    from igg.parallel.comm import bounded_stream_sync

    s = torch.cuda.Stream()
    native.gpu_spin(2.0, s.cuda_stream)
    t0 = time.time()
    with pytest.raises(igg.IGGError, match="did not drain"):
        bounded_stream_sync(s.cuda_stream, timeout=0.5, what="test")
    assert 0.4 <= time.time() - t0 < 1.9
    bounded_stream_sync(s.cuda_stream, timeout=30.0, what="test")
    assert time.time() - t0 >= 1.9
    t1 = time.perf_counter()
    for _ in range(100):
        bounded_stream_sync(s.cuda_stream, timeout=5.0)
    assert (time.perf_counter() - t1) / 100 < 2e-3  # microseconds in practice, generous bound


def test_gpu_tensor_collectives_single_rank(gpu):
    igg.init_global_grid(6, 5, 4, quiet=True, init_MPI=False)
    comm = igg.get_global_grid().comm
    t = torch.arange(4, dtype=torch.float64, device=gpu)
    assert torch.equal(comm.allreduce_(t, "sum").cpu(), torch.arange(4, dtype=torch.float64))
    assert torch.equal(comm.bcast_(t, 0).cpu(), torch.arange(4, dtype=torch.float64))
    assert comm.allreduce(3.5, "max") == 3.5
    assert comm.torch_nccl is None  # no second (torch) RCCL communicator
    igg.finalize_global_grid(finalize_MPI=False)
