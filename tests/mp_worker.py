"""Per-rank test scenarios (launched by tests/_mp.py, one process per rank)."""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import igg  # noqa: E402
from tests.helpers import encode, expected_after_halo, has_halo, zero_boundaries  # noqa: E402

DTYPES = {"f64": torch.float64, "f32": torch.float32, "f16": torch.float16, "c128": torch.complex128, "i16": torch.int16}


def _device(kind):
    """cpu | gpu (every rank on device 0) | mgpu (one rank per device: LOCAL_RANK)."""
    if kind == "mgpu":
        r = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(r)
        return torch.device("cuda", r)
    if kind == "gpu":
        torch.cuda.set_device(0)
        return torch.device("cuda", 0)
    return torch.device("cpu")


def _plain(v: int) -> int:
    """Plain stencil variant for a fused-variant id (the fused ids reuse the
    plain index space; a fused-only or measurement-only id maps to 0)."""
    return v if igg.native.diffusion3d_variant_compiled(v) else 0


def scenario_halo(dev, nx, ny, nz, px, py, pz, dt, dimx=0, dimy=0, dimz=0):
    device = _device(dev)
    nx, ny, nz, px, py, pz = map(int, (nx, ny, nz, px, py, pz))
    dtype = DTYPES[dt]
    igg.init_global_grid(nx, ny, nz, periodx=px, periody=py, periodz=pz, dimx=int(dimx), dimy=int(dimy),
                         dimz=int(dimz), quiet=True, select_device=False,
                         device_type="none" if dev == "cpu" else "AMDGPU")
    gg = igg.get_global_grid()
    nd = 3 if nz > 1 else (2 if ny > 1 else 1)
    base = (nx, ny, nz)[:nd]
    deltas = [(0, 0, 0), (1, 0, 0), (0, 1, 0), (0, 0, 1), (-1, 2, 1), (2, -1, 1)]
    seen = set()
    for dl in deltas:
        shape = tuple(b + d for b, d in zip(base, dl[:nd]))
        if shape in seen or min(shape) < 1:
            continue
        seen.add(shape)
        A = torch.zeros(shape, dtype=dtype)
        if not any(has_halo(A, gg)[:nd]):
            continue
        encode(A, complex_factor=(1 + 1j) if dtype.is_complex else None)
        ref = expected_after_halo(A, has_halo(A, gg), gg.neighbors.tolist())
        X = zero_boundaries(A.clone()).to(device)
        igg.update_halo_(X)
        got = X.cpu()
        if not torch.equal(got, ref):
            bad = (got != ref).nonzero()[:5].tolist()
            raise AssertionError(f"rank {gg.me} shape {shape} dims {gg.dims.tolist()} mismatch at {bad}")
    # two fields in one call (staggered Vx, Vz) + three fields of different sizes
    if nd == 3:
        fs = [torch.zeros(nx + 1, ny, nz, dtype=dtype), torch.zeros(nx, ny, nz + 1, dtype=dtype),
              torch.zeros(nx, ny + 1, nz, dtype=dtype)]
        refs = []
        for F in fs:
            encode(F, complex_factor=(1 + 1j) if dtype.is_complex else None)
            refs.append(expected_after_halo(F, has_halo(F, gg), gg.neighbors.tolist()))
        Xs = [zero_boundaries(F.clone()).to(device) for F in fs]
        igg.update_halo_(*Xs)
        for X, R in zip(Xs, refs):
            assert torch.equal(X.cpu(), R), f"rank {gg.me}: multi-field mismatch"
    igg.finalize_global_grid()
    print(f"rank {gg.me} OK dims={gg.dims.tolist()}")


def scenario_gather(dev, dt):
    device = _device(dev)
    dtype = DTYPES[dt]
    nx, ny, nz = 4, 3, 2
    me, dims, nprocs, coords, comm = igg.init_global_grid(nx, ny, nz, quiet=True, select_device=False,
                                                          device_type="none" if dev == "cpu" else "AMDGPU")
    for root in sorted({0, nprocs - 1}):
        for shape in [(nx,), (nx, ny), (nx, ny, nz)]:
            A = torch.full(shape, float(me + 1), dtype=dtype).to(device)
            flat = torch.arange(A.numel(), dtype=torch.float64).view(shape).to(dtype).to(device)
            A = A * 100 + flat
            s = list(shape) + [1] * (3 - len(shape))
            G = torch.zeros(dims[0] * s[0], dims[1] * s[1], dims[2] * s[2], dtype=dtype).to(device) if me == root else None
            igg.gather_(A, G, root=root)
            if me == root:
                G = G.cpu()
                for p in range(nprocs):
                    c = igg.native.cart_coords(p, dims.tolist())
                    blk = G[c[0] * s[0]:(c[0] + 1) * s[0], c[1] * s[1]:(c[1] + 1) * s[1], c[2] * s[2]:(c[2] + 1) * s[2]]
                    exp = (torch.full(s, float(p + 1), dtype=torch.float64) * 100 +
                           torch.arange(blk.numel(), dtype=torch.float64).view(s)).to(dtype)
                    assert torch.equal(blk, exp), f"root {root}: block of rank {p} wrong"
        # 1-D A gathered into a 3-D A_global (only the length must match)
        A = torch.full((nx,), float(me), dtype=dtype).to(device)
        G = torch.zeros(nx * dims[0], dims[1], dims[2], dtype=dtype).to(device) if me == root else None
        igg.gather_(A, G, root=root)
    igg.finalize_global_grid()
    print(f"rank {me} gather OK")


def scenario_gather_vmm(big_mib):
    """gather_ of blocks in HIP VMM memory (MemKind 4, csrc/vmm.cpp): pulled in
    place through a file descriptor at any size ('V' records), a second array
    (a new allocation) re-imported; then gather_async_(snapshot=True) of a
    block of ``big_mib`` MiB, staged into ONE VMM buffer instead of IPC chunks.
    Every gathered block is checked."""
    from igg.models.diffusion3d import native_buffer

    device = _device("gpu")
    me, dims, nprocs, coords, comm = igg.init_global_grid(8, 8, 8, quiet=True, select_device=False,
                                                          device_type="AMDGPU")

    def block(shape, k, p):
        return torch.arange(math.prod(shape), dtype=torch.float32).view(shape) + 1e5 * (p + 1) + 1e6 * k

    def check(G, shape, k):
        Gc = G.cpu()
        for p in range(nprocs):
            c = igg.native.cart_coords(p, dims.tolist())
            blk = Gc[c[0] * shape[0]:(c[0] + 1) * shape[0], c[1] * shape[1]:(c[1] + 1) * shape[1],
                     c[2] * shape[2]:(c[2] + 1) * shape[2]]
            assert torch.equal(blk, block(shape, k, p)), f"gather {k} {shape}: block of rank {p} wrong"

    for k, shape in enumerate([(4, 256, 512), (4, 256, 512), (6, 128, 256)]):
        n = math.prod(shape) * 4
        A = native_buffer(n + 4096, 4, device)[4096:4096 + n].view(torch.float32).view(shape)  # offset inside
        A.copy_(block(shape, k, me))
        G = torch.zeros([int(dims[d]) * shape[d] for d in range(3)], dtype=torch.float32, device=device) \
            if me == 0 else None
        igg.gather_(A, G, root=0)
        if me == 0:
            check(G, shape, k)
        del A, G
    # a large snapshot: one VMM staging buffer (>= half the IPC limit), not chunks
    nx = max(1, (int(big_mib) << 20) // (512 * 512 * 4))
    shape = (nx, 512, 512)
    A = block(shape, 7, me).to(device)
    G = torch.zeros([int(dims[d]) * shape[d] for d in range(3)], dtype=torch.float32, device=device) \
        if me == 0 else None
    h = igg.gather_async_(A, G, root=0, snapshot=True)
    A.fill_(-1.0)  # the snapshot was taken: A may change at once
    h.wait()
    if me == 0:
        check(G, shape, 7)
    igg.finalize_global_grid()
    print(f"rank {me} gather vmm OK", flush=True)


def scenario_gather_dmabuf(big_mib):
    """gather_ of ordinary (torch / hipMalloc) blocks above the IPC limit:
    each rank's allocation is exported as a dma-buf and pulled in place
    (csrc/gather.cpp; IGG_GATHER_DMABUF=0: staged copies). Three
    gathers: a first one, the same array with new values (the root's mapping
    is reused), and a new array after the old one was freed back to the runtime
    (a new buffer id: a new export). Every block is checked; the times printed."""
    import time

    device = _device("gpu")
    me, dims, nprocs, coords, comm = igg.init_global_grid(8, 8, 8, quiet=True, select_device=False,
                                                          device_type="AMDGPU")
    nx = max(1, (int(big_mib) << 20) // (512 * 512 * 4))
    shape = (nx, 512, 512)

    def fill(A, k, p):
        A.copy_(torch.arange(A.numel(), dtype=torch.float32, device=device).view(A.shape) % 1000003
                + 1e7 * (p + 1) + 1e8 * k)

    G = torch.zeros([int(dims[d]) * shape[d] for d in range(3)], dtype=torch.float32, device=device) \
        if me == 0 else None
    A = torch.empty(shape, dtype=torch.float32, device=device)
    times = []
    for k in range(3):
        if k == 2:  # free the array back to the runtime and allocate a new one
            del A
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            A = torch.empty(shape, dtype=torch.float32, device=device)
        fill(A, k, me)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        igg.gather_(A, G, root=0)
        torch.cuda.synchronize()
        times.append((time.perf_counter() - t0) * 1e3)
        from igg.parallel import gather as _g

        kinds = comm.all_gather_object(_g._sync_puller.last_kind)
        want = ("dmabuf" if os.environ.get("IGG_GATHER_DMABUF", "1") != "0"
                else "vmm-staging" if os.environ.get("IGG_GATHER_VMM") == "1" else "chunks")
        assert kinds[1:] == [want] * (nprocs - 1), f"gather {k}: blocks published as {kinds}, expected {want}"
        if me == 0:
            for p in range(nprocs):
                c = igg.native.cart_coords(p, dims.tolist())
                blk = G[c[0] * shape[0]:(c[0] + 1) * shape[0], c[1] * shape[1]:(c[1] + 1) * shape[1],
                        c[2] * shape[2]:(c[2] + 1) * shape[2]]
                ref = torch.empty_like(blk)
                fill(ref, k, p)
                assert torch.equal(blk, ref), f"gather {k}: block of rank {p} wrong"
                del ref
    if me == 0:
        print(f"gather dmabuf {big_mib} MiB per rank ({kinds[1]}): ms {[round(t, 2) for t in times]}", flush=True)
    igg.finalize_global_grid()
    print(f"rank {me} gather dmabuf OK", flush=True)


def scenario_gather_regrow():
    """gather_ (IPC pull of staged chunks, IGG_GATHER_CHUNK_BYTES set by the
    test) of blocks whose chunks are MiB-sized dedicated allocations and grow
    between gathers: the grown-out chunks are retired, not freed, so no new
    export reuses an address the root still has mapped (ADVICE r3:
    gather.cpp:174); every gathered block is checked."""
    _device("gpu")
    me, dims, nprocs, coords, comm = igg.init_global_grid(8, 8, 8, quiet=True, select_device=False,
                                                          device_type="AMDGPU")
    for k, shape in enumerate([(8, 256, 256), (8, 512, 512), (8, 256, 256), (6, 768, 512)]):
        A = (torch.arange(math.prod(shape), dtype=torch.float64).view(shape) + 1e7 * (me + 1) + 1e9 * k).cuda()
        G = (torch.zeros(dims[0] * shape[0], dims[1] * shape[1], dims[2] * shape[2], dtype=torch.float64).cuda()
             if me == 0 else None)
        igg.gather_(A, G, root=0)
        if me == 0:
            Gc = G.cpu()
            for p in range(nprocs):
                c = igg.native.cart_coords(p, dims.tolist())
                blk = Gc[c[0] * shape[0]:(c[0] + 1) * shape[0], c[1] * shape[1]:(c[1] + 1) * shape[1],
                         c[2] * shape[2]:(c[2] + 1) * shape[2]]
                exp = torch.arange(math.prod(shape), dtype=torch.float64).view(shape) + 1e7 * (p + 1) + 1e9 * k
                assert torch.equal(blk, exp), f"gather {k} {shape}: block of rank {p} wrong"
        del A, G
    igg.finalize_global_grid()
    print(f"rank {me} gather regrow OK")


def scenario_gather_fail(expect):
    """IGG_INJECT_FAIL makes one rank's export (or the root's mapping) fail:
    every rank must raise, none may hang in the collective."""
    _device("gpu")
    me, dims, nprocs, coords, comm = igg.init_global_grid(6, 5, 4, quiet=True, select_device=False,
                                                          device_type="AMDGPU")
    A = torch.full((6, 5, 4), float(me), dtype=torch.float64, device="cuda")
    G = torch.zeros(dims[0] * 6, dims[1] * 5, dims[2] * 4, dtype=torch.float64, device="cuda") if me == 0 else None
    try:
        igg.gather_(A, G, root=0)
    except Exception as e:
        assert expect in str(e), f"rank {me}: unexpected error {e}"
        print(f"rank {me} raised as expected: {str(e)[:200]}")
    else:
        raise AssertionError(f"rank {me}: gather_ did not raise")
    os._exit(0)  # the failed gather's state is not torn down collectively


def scenario_rccl_init_bounded(max_seconds):
    """RCCL bootstrap bounded and collective: ranks sharing one GPU (RCCL
    refuses duplicate devices) and/or a rank that arrives late
    (IGG_INJECT_HANG=rccl_init@r:seconds) - every rank raises the same
    IGGError within the bound, none hangs; a second attempt raises at once."""
    import time as _time

    _device("gpu")
    me, dims, nprocs, coords, comm = igg.init_global_grid(6, 5, 4, quiet=True, select_device=False,
                                                          device_type="AMDGPU")
    t0 = _time.monotonic()
    try:
        comm.ensure_rccl()
    except igg.IGGError as e:
        dt = _time.monotonic() - t0
        assert "RCCL communicator could not be created" in str(e), str(e)
        assert dt < float(max_seconds), f"rank {me}: took {dt:.1f} s"
        print(f"rank {me}: raised after {dt:.1f} s: {str(e)[:240]}", flush=True)
    else:
        raise AssertionError(f"rank {me}: RCCL with ranks sharing a GPU did not fail")
    t1 = _time.monotonic()
    try:
        comm.ensure_rccl()
    except igg.IGGError:
        assert _time.monotonic() - t1 < 1.0, "a failed bootstrap was retried"
    else:
        raise AssertionError("second ensure_rccl did not raise")
    igg.finalize_global_grid()
    print(f"rank {me} rccl init bounded OK", flush=True)


def scenario_diffusion(dev, nx, ny, nz, steps, overlap):
    from igg.models.diffusion3d import Diffusion3D
    from igg.ops import stencil

    device = _device(dev)
    nx, ny, nz, steps = int(nx), int(ny), int(nz), int(steps)
    # IGG_TEST_DIMS="a,b,c" fixes the topology (e.g. 2,2,1: two split dims);
    # IGG_TEST_GRAPH=k captures k steps in a hipGraph and replays them
    dims_env = [int(v) for v in os.environ.get("IGG_TEST_DIMS", "0,0,0").split(",")]
    me, dims, nprocs, coords, comm = igg.init_global_grid(nx, ny, nz, dimx=dims_env[0], dimy=dims_env[1],
                                                          dimz=dims_env[2], quiet=True, select_device=False,
                                                          device_type="none" if dev == "cpu" else "AMDGPU")
    gg = igg.get_global_grid()
    v = os.environ.get("IGG_TEST_VARIANT")
    # IGG_TEST_RESERVE_CUS=k: the overlapped step's interior on a CU-masked
    # compute stream (two forked side streams per step: the graph-fork cell
    # that crashed the HIP runtime with one hardware queue)
    m = Diffusion3D(dtype=torch.float64, device=device, overlap=bool(int(overlap)),
                    variant=None if v is None else int(v),
                    reserve_cus=int(os.environ.get("IGG_TEST_RESERVE_CUS", "0")))
    if int(os.environ.get("IGG_TEST_RESERVE_CUS", "0")) and m.overlap:
        from igg.parallel import halo as _H

        assert m._overlap_streams() == (2 if _H.transport_name() == "rccl" else 3)
    g = int(os.environ.get("IGG_TEST_GRAPH", "0"))
    if g:
        assert m.overlap == bool(int(overlap))
        m.capture(steps=g)  # performs the eager first step itself (no step is run by the capture)
        m.run(steps - 1)  # graph replays (after at most two eager steps that realign the buffers)
        assert steps - 1 >= g + 2, "too few steps for a replay"
    else:
        m.run(steps)
    loc = m.T.cpu()
    # global reference: same physics on the implicit global grid, one array
    ng = [int(v) for v in gg.nxyz_g]
    lx = ly = lz = 10.0
    dx, dy, dz = lx / (ng[0] - 1), ly / (ng[1] - 1), lz / (ng[2] - 1)
    x = (torch.arange(ng[0], dtype=torch.float64) * dx).view(-1, 1, 1)
    y = (torch.arange(ng[1], dtype=torch.float64) * dy).view(1, -1, 1)
    z = (torch.arange(ng[2], dtype=torch.float64) * dz).view(1, 1, -1)
    Cp = 1 + 5 * torch.exp(-(x - lx / 1.5) ** 2 - (y - ly / 2) ** 2 - (z - lz / 1.5) ** 2) + \
        5 * torch.exp(-(x - lx / 3.0) ** 2 - (y - ly / 2) ** 2 - (z - lz / 1.5) ** 2)
    T = 100 * torch.exp(-((x - lx / 2) / 2) ** 2 - ((y - ly / 2) / 2) ** 2 - ((z - lz / 3.0) / 2) ** 2) + \
        50 * torch.exp(-((x - lx / 2) / 2) ** 2 - ((y - ly / 2) / 2) ** 2 - ((z - lz / 1.5) / 2) ** 2)
    for _ in range(steps):
        T = stencil.diffusion3d_reference(T, Cp, lam=m.lam, dt=m.dt, dx=m.dx, dy=m.dy, dz=m.dz)
    o = [int(coords[d]) * (int(gg.nxyz[d]) - int(gg.overlaps[d])) for d in range(3)]
    blk = T[o[0]:o[0] + nx, o[1]:o[1] + ny, o[2]:o[2] + nz]
    err = (loc - blk).abs().max().item()
    assert err < 1e-10, f"rank {me}: diffusion mismatch {err}"
    igg.finalize_global_grid()
    print(f"rank {me} diffusion OK err={err:.2e}")


def scenario_diffusion_fused(nx, ny, nz, steps, periodic, graph):
    """Fused halo exchange (stencil stores send planes into the neighbours'
    arenas) vs stencil + update_halo_: bitwise equal T on every rank."""
    from igg.models.diffusion3d import Diffusion3D

    device = _device(os.environ.get("IGG_TEST_DEV", "gpu"))
    nx, ny, nz, steps, per = int(nx), int(ny), int(nz), int(steps), int(periodic)
    me, dims, nprocs, coords, comm = igg.init_global_grid(nx, ny, nz, periodx=per, periody=per, periodz=per,
                                                          quiet=True, select_device=False)
    v = int(os.environ.get("IGG_TEST_VARIANT", "0"))
    a = Diffusion3D(dtype=torch.float64, device=device, variant=_plain(v))
    b = Diffusion3D(dtype=torch.float64, device=device, variant=_plain(v))
    b.fused_variant, b.fused_mode = v, int(os.environ.get("IGG_TEST_FUSED_MODE", "0"))
    b.fused_rounds = int(os.environ.get("IGG_TEST_FUSED_ROUNDS", str(b.fused_rounds)))
    want = b.fused_mode
    assert b.set_fused(True), "fused mode unavailable"
    assert b.fused_variant == v, f"fused variant {v} is not compiled in this build"
    assert b.fused_mode == want, f"send mode {want} unavailable (direct z needs the peers' field buffers)"
    a.run(steps)
    if int(graph):
        b.step()
        b.capture(steps=2)
        b.run(steps - 1)
    else:
        b.run(steps)
    b.sync_halo()
    torch.cuda.synchronize()
    b.check()
    if not torch.equal(a.T, b.T):
        bad = (a.T != b.T).nonzero()[:5].tolist()
        raise AssertionError(f"rank {me} dims {dims.tolist()}: fused differs at {bad}")
    # switching back to the update_halo_ path continues bitwise
    b.set_fused(False)
    a.run(3)
    b.run(3)
    torch.cuda.synchronize()
    assert torch.equal(a.T, b.T), f"rank {me}: mismatch after leaving fused mode"
    b.close()  # collective unmap of the peer arenas
    igg.finalize_global_grid()
    print(f"rank {me} fused OK")


def scenario_acoustic(dev, nx, ny, steps):
    """2-D staggered acoustic solver on a 2-D process grid vs the same physics
    on the implicit global grid in one array (bitwise on CPU)."""
    from igg.models.acoustic2d import Acoustic2D

    device = _device(dev)
    nx, ny, steps = int(nx), int(ny), int(steps)
    me, dims, nprocs, coords, comm = igg.init_global_grid(nx, ny, 1, quiet=True, select_device=False,
                                                          device_type="none" if dev == "cpu" else "AMDGPU")
    gg = igg.get_global_grid()
    m = Acoustic2D(dtype=torch.float64, device=device)
    m.run(steps)
    got = [t.cpu().double() for t in (m.P, m.Vx, m.Vy)]
    o = [int(coords[d]) * (int(gg.nxyz[d]) - int(gg.overlaps[d])) for d in range(2)]
    ng = [int(v) for v in gg.nxyz_g[:2]]
    from igg.models.acoustic2d import acoustic2d_reference

    lx = ly = 10.0
    dx, dy = lx / (ng[0] - 1), ly / (ng[1] - 1)
    x = (torch.arange(ng[0], dtype=torch.float64) * dx).view(-1, 1)
    y = (torch.arange(ng[1], dtype=torch.float64) * dy).view(1, -1)
    P = torch.exp(-((x - lx / 2) ** 2) - (y - ly / 2) ** 2)
    Vx = torch.zeros(ng[0] + 1, ng[1], dtype=torch.float64)
    Vy = torch.zeros(ng[0], ng[1] + 1, dtype=torch.float64)
    for _ in range(steps):
        P, Vx, Vy = acoustic2d_reference(P, Vx, Vy, dt=m.dt, K=m.K, rho=m.rho, dx=m.dx, dy=m.dy)
    for name, a, r in zip(("P", "Vx", "Vy"), got, (P, Vx, Vy)):
        blk = r[o[0]:o[0] + a.shape[0], o[1]:o[1] + a.shape[1]]
        err = (a - blk).abs().max().item()
        assert err < 1e-12, f"rank {me}: {name} mismatch {err}"
    igg.finalize_global_grid()
    print(f"rank {me} acoustic OK dims={dims.tolist()}")


def scenario_acoustic_fused(dev, nx, ny, steps, periodic):
    """Acoustic2D with the fused exchange vs the update_halo_ path, bitwise in
    every field on every rank (eager steps, then hipGraph replays)."""
    from igg.models.acoustic2d import Acoustic2D

    _device(dev)
    nx, ny, steps, per = int(nx), int(ny), int(steps), int(periodic)
    me, dims, nprocs, coords, comm = igg.init_global_grid(nx, ny, 1, periodx=per, periody=per, quiet=True,
                                                          select_device=False, device_type="AMDGPU")
    a, b = Acoustic2D(dtype=torch.float32), Acoustic2D(dtype=torch.float32)
    assert b.set_fused(True), "fused exchange unavailable"
    a.run(steps)
    b.run(steps)
    b.capture(steps=4)
    a.run(8)
    b.run(8)
    # state written outside the time loop (a restore): the next fused step
    # synchronises first, so no neighbour's store is overwritten by the copy
    names = ("P", "Vx", "Vy", "P2", "Vx2", "Vy2")
    saved = {n: getattr(a, n).clone() for n in names}
    a.run(5)
    b.run(5)
    for m in (a, b):
        for n in names:
            getattr(m, n).copy_(saved[n])
    b.mark_modified()
    a.run(12)
    b.run(12)
    torch.cuda.synchronize()
    b.check()
    for n in names:
        x, y = getattr(a, n), getattr(b, n)
        if not torch.equal(x, y):
            bad = (x != y).nonzero()[:5].tolist()
            raise AssertionError(f"rank {me} dims {dims.tolist()}: {n} differs at {bad}")
    b.close()
    igg.finalize_global_grid()
    print(f"rank {me} acoustic fused OK dims={dims.tolist()}")


def scenario_put_after_model(n, graph, steps):
    """Put transport: the acoustic model's (Vx2, Vy2) exchanges (eager, then
    hipGraph replays if ``graph``), then a single-field probe exchange, bitwise
    against the host-staged path on every rank (bench.py's post-timing
    validation in miniature); prints the put epoch of every rank."""
    from igg.models.acoustic2d import Acoustic2D
    from igg.parallel import halo as H

    _device("gpu")
    n, graph, steps = int(n), int(graph), int(steps)
    me, dims, nprocs, coords, comm = igg.init_global_grid(n, n, 1, quiet=True, select_device=False,
                                                          device_type="AMDGPU")
    gg = igg.get_global_grid()
    m = Acoustic2D(dtype=torch.float32)
    H.set_transport("put")
    m.run(3)
    if graph:
        m.capture(steps=4)
    m.run(steps)
    torch.cuda.synchronize()
    A = torch.zeros(n, n, dtype=torch.float32)
    encode(A)
    ref = expected_after_halo(A, has_halo(A, gg), gg.neighbors.tolist())
    X = zero_boundaries(A.clone()).cuda()
    igg.update_halo_(X)
    torch.cuda.synchronize()
    ep = comm.mesh.epoch
    got = X.cpu()
    bad = (got != ref).nonzero()
    print(f"rank {me} epoch {ep} mismatches {bad.shape[0]} first {bad[:6].tolist()}", flush=True)
    eps = comm.all_gather_object(int(ep))
    assert len(set(eps)) == 1, f"put epochs differ across ranks: {eps}"
    assert bad.shape[0] == 0, f"rank {me}: probe mismatch at {bad[:6].tolist()}"
    igg.finalize_global_grid()
    print(f"rank {me} put after model OK", flush=True)


def scenario_select_transport(dev):
    """select_transport: on GPU ranks sharing one device, 'put' passes the
    probe check against the host-staged exchange, RCCL is skipped (it refuses
    duplicate devices) and update_halo_ runs on 'put' afterwards, bitwise vs
    the expected halos; one rank per device (mgpu): both pass and the faster
    is kept; on a CPU grid nothing is switched."""
    device = _device(dev)
    n = 20
    me, dims, nprocs, coords, comm = igg.init_global_grid(n, n - 2, 12, quiet=True, select_device=False,
                                                          device_type="none" if dev == "cpu" else "AMDGPU")
    gg = igg.get_global_grid()
    A = torch.zeros(n, n - 2, 12, dtype=torch.float64)
    encode(A)
    ref = expected_after_halo(A, has_halo(A, gg), gg.neighbors.tolist())
    X = zero_boundaries(A.clone()).to(device)
    before = X.clone()
    res = igg.select_transport(X, steps=3)
    print(f"rank {me} select_transport {res}", flush=True)
    assert torch.equal(X, before), "select_transport modified its argument"
    if dev == "cpu":
        assert "reason" in res and not res["checked"]
    elif dev == "gpu":  # every rank on device 0
        assert res["checked"]["put"] == "ok", res
        assert res["checked"]["rccl"].startswith("skipped"), res
        assert res["chosen"] == "put" and res["ms"]["put"] > 0, res
    else:  # mgpu: one rank per device, both checked, the faster kept
        assert res["checked"] == {"put": "ok", "rccl": "ok"}, res
        assert res["chosen"] == min(res["ms"], key=res["ms"].get), res
    igg.update_halo_(X)
    got = X.cpu()
    bad = (got != ref).nonzero()
    assert bad.shape[0] == 0, f"rank {me}: halo mismatch after select_transport at {bad[:6].tolist()}"
    igg.finalize_global_grid()
    print(f"rank {me} select transport OK", flush=True)


def scenario_auto_transport(dev, expect):
    """IGG_TRANSPORT=auto (the default): the first eager device exchange of a
    field set checks put and rccl against the host-staged exchange and keeps
    the fastest that passed, per field-set signature. ``expect``: the
    transport it must choose ('put' on ranks sharing a GPU, where RCCL is
    skipped; 'staged' when put's peer mapping is injected to fail there;
    'fastest' with one rank per device). The caller's halo is exact either way."""
    from igg.parallel import halo as H

    device = _device(dev)
    n = 20
    me, dims, nprocs, coords, comm = igg.init_global_grid(n, n - 2, 12, quiet=True, select_device=False,
                                                          device_type="AMDGPU")
    gg = igg.get_global_grid()
    assert H.auto_transport() and H.transport_name() == "auto", H.transport_name()
    for dt in (torch.float64, torch.float32):
        A = torch.zeros(n, n - 2, 12, dtype=dt)
        encode(A)
        ref = expected_after_halo(A, has_halo(A, gg), gg.neighbors.tolist())
        X = zero_boundaries(A.clone()).to(device)
        igg.update_halo_(X)
        igg.update_halo_(X)  # the cached choice, no second selection
        bad = (X.cpu() != ref).nonzero()
        assert bad.shape[0] == 0, f"rank {me}: halo mismatch ({dt}) at {bad[:6].tolist()}"
    log = H.tuned_transports()
    print(f"rank {me} auto transport {log}", flush=True)
    assert len(log) == 2, log  # one selection per signature (two dtypes)
    for rec in log:
        if expect == "fastest":
            assert rec["checked"] == {"put": "ok", "rccl": "ok"}, rec
            assert rec["chosen"] == min(rec["ms"], key=rec["ms"].get), rec
        else:
            assert rec["chosen"] == expect, rec
            assert rec["checked"]["rccl"].startswith("skipped"), rec
            if expect == "staged":
                assert "could not map" in rec["checked"]["put"], rec
    assert H.transport_name() == {"staged": "gloo-staged"}.get(log[-1]["chosen"], log[-1]["chosen"])
    assert H.auto_transport()
    H.set_transport("staged")  # an explicit choice ends the automatic one
    assert not H.auto_transport()
    igg.finalize_global_grid()
    print(f"rank {me} auto transport OK", flush=True)


def scenario_coherence(dev, form, nbytes, rounds, plain_writer=0):
    """docs/COHERENCE.md fact 4 with WARM caches (igg/coherence.hpp): rank 0
    reads its receive arena from 2 workgroups per CU (every XCD's L2 holds
    every line), rank 1 stores a new value into it with the production
    system-scope stores and publishes it with the production synchronisation
    (``form``: 'kernel' = put_sync_kernel on both sides, 'inkernel' =
    step_sync_exit_wg / step_sync_enter_wg inside the kernels); rank 0 then
    reads every word from every XCD. Any stale line is a mismatch."""
    device = _device(dev)
    me, dims, nprocs, coords, comm = igg.init_global_grid(8, 8, 8, quiet=True, select_device=False,
                                                          device_type="AMDGPU")
    assert nprocs == 2
    gg = igg.get_global_grid()
    mesh = igg.native.PeerMesh(gg.comm.rank, gg.comm.size, gg.comm._allgather_bytes)
    probe = igg.native.CoherenceProbe(mesh, int(nbytes))
    ik = form == "inkernel"
    s = torch.cuda.current_stream(device).cuda_stream
    bad = []
    if me == 0 and ik:
        bad.append(probe.check(0, True, s))  # the reader's step 1 consumes the writer's step 0
    for e in range(1, int(rounds) + 1):
        if me == 0:
            probe.warm(s)  # every XCD's L2 now holds the arena's lines (value e - 1)
            torch.cuda.synchronize()
        comm.barrier()  # the writer starts only after the warm reads completed
        if me == 1:
            probe.write(e, ik, s, bool(int(plain_writer)))
        else:
            bad.append(probe.check(e, ik, s))
    torch.cuda.synchronize()
    comm.barrier()
    mesh.check_error()  # no synchronisation timed out
    if me == 0:
        print(f"rank 0 coherence {form}{' PLAIN-STORE WRITER' if int(plain_writer) else ''} "
              f"{int(nbytes) >> 10} KiB x {rounds} rounds ({probe.workgroups} workgroups per read): "
              f"stale reads {sum(bad)}, per round {bad[:8]}", flush=True)
        if not int(plain_writer):
            assert sum(bad) == 0, f"stale reads after the synchronisation: {bad}"
    del probe
    mesh.close()
    igg.finalize_global_grid()
    print(f"rank {me} coherence OK", flush=True)


def scenario_coherence_control(dev, nbytes, rounds, l2):
    """Negative control of scenario_coherence: the reader warms its caches
    and then re-reads the arena in the SAME kernel after seeing the writer's
    ARRIVED flag with relaxed polls only - no acquire, no kernel boundary
    (l2 = 1: the re-read skips the L1). Prints the stale-read count; a
    nonzero count shows that the warm caches do hold stale lines, so the
    production forms' zero (scenario_coherence) comes from their acquires."""
    import time

    device = _device(dev)
    me, dims, nprocs, coords, comm = igg.init_global_grid(8, 8, 8, quiet=True, select_device=False,
                                                          device_type="AMDGPU")
    gg = igg.get_global_grid()
    mesh = igg.native.PeerMesh(gg.comm.rank, gg.comm.size, gg.comm._allgather_bytes)
    probe = igg.native.CoherenceProbe(mesh, int(nbytes))
    s = torch.cuda.current_stream(device).cuda_stream
    bad = []
    for e in range(1, int(rounds) + 1):
        if me == 0:
            probe.control(e, e, bool(int(l2)), s)
            time.sleep(0.005)  # the kernel's warm read completes before the writer starts
        comm.barrier()
        if me == 1:
            probe.write(e, False, s)
            torch.cuda.synchronize()
        else:
            bad.append(probe.mismatches(s))
    torch.cuda.synchronize()
    comm.barrier()
    mesh.check_error()
    if me == 0:
        print(f"rank 0 coherence control ({'L1 bypass' if int(l2) else 'plain loads'}, no acquire) "
              f"{int(nbytes) >> 10} KiB x {rounds} rounds: stale reads {sum(bad)} of "
              f"{int(rounds) * probe.words * probe.workgroups}, per round {bad[:8]}", flush=True)
    del probe
    mesh.close()
    igg.finalize_global_grid()
    print(f"rank {me} coherence control done", flush=True)


def scenario_vmm_map(dev, nbytes, source="vmm"):
    """HIP VMM export of a large allocation (csrc/vmm.cpp): rank 1 creates
    ``nbytes`` with hipMemCreate, writes a pattern at four offsets (the last
    beyond 2 GiB), exports a POSIX fd and hands it over a Unix socket; rank 0
    imports and maps it (bounded), reads the four regions back and copies the
    whole allocation into its own memory (timed). hipIpcOpenMemHandle of
    such an allocation never returns on this runtime (ipc.hpp).
    ``source="malloc"``: the allocation is torch's (hipMalloc), exported as a
    dma-buf of its whole hipMalloc range (native.range_export_fd)."""
    import time
    import uuid

    from igg._native import native

    device = _device(dev)
    me, dims, nprocs, coords, comm = igg.init_global_grid(8, 8, 8, quiet=True, select_device=False,
                                                          device_type="AMDGPU")
    nbytes = int(nbytes)
    s = torch.cuda.current_stream(device).cuda_stream
    chunk = 1 << 20  # bytes per pattern region
    pat = [(torch.arange(chunk // 8, dtype=torch.int64, device=device) * 7 + k * 1000003) for k in range(4)]

    def regions(size):
        return [0, 1 << 30, (2 << 30) + (8 << 20), size - chunk]

    if me == 1:
        if source == "vmm":
            ptr, size = native.vmm_alloc(nbytes)
            fd, offset, msize = native.vmm_export_fd(ptr), 0, size
        else:
            buf = torch.zeros(nbytes, dtype=torch.uint8, device=device)
            ptr, size = buf.data_ptr(), nbytes
            fd, base, msize = native.range_export_fd(ptr)
            offset = ptr - base
            print(f"rank 1 hipMalloc range {msize >> 20} MiB, tensor at offset {offset}", flush=True)
        for k, off in enumerate(regions(size)):
            native.copy2d([(pat[k].data_ptr(), ptr + off, 1, chunk // 8, 0, 1, 0, 1)], 8, True, s)
        torch.cuda.synchronize()
        name = f"igg-vmm-{uuid.uuid4().hex}"
        lis = native.fd_listen(name)
        comm.all_gather_object((name, size, msize, offset))
        native.fd_serve(lis, fd, 1, 60.0)
        native.fd_close(lis)
        native.fd_close(fd)
        comm.barrier()  # the importer is done with the mapping
        if source == "vmm":
            native.vmm_free(ptr)
    else:
        name, size, msize, offset = comm.all_gather_object(None)[1]
        t0 = time.perf_counter()
        fd = native.fd_fetch(name, 60.0)
        base = native.vmm_import_fd(fd, msize, 60.0)
        ptr = base + offset
        t_map = time.perf_counter() - t0
        for k, off in enumerate(regions(size)):
            got = torch.empty_like(pat[k])
            native.copy2d([(ptr + off, got.data_ptr(), 1, chunk // 8, 0, 1, 0, 1)], 8, True, s)
            torch.cuda.synchronize()
            assert torch.equal(got, pat[k]), f"region {k} at byte {off}: mismatch"
        dst = torch.empty(size // 8, dtype=torch.int64, device=device)
        rows = size // (4 << 20)
        cp = [(ptr, dst.data_ptr(), rows, (4 << 20) // 8, (4 << 20) // 8, 1, (4 << 20) // 8, 1)]
        native.copy2d(cp, 8, True, s)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        native.copy2d(cp, 8, True, s)
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1)
        assert torch.equal(dst[: chunk // 8], pat[0])
        print(f"rank 0 vmm map of {size >> 20} MiB: fd + import + map {t_map * 1e3:.1f} ms, 4 regions ok, "
              f"full copy {ms:.3f} ms ({size / ms / 1e6:.0f} GB/s)", flush=True)
        del dst
        native.vmm_free(base)
        native.fd_close(fd)
        comm.barrier()
    igg.finalize_global_grid()
    print(f"rank {me} vmm map OK", flush=True)


def scenario_put_regrow():
    """Put transport with field sets that force the receive arenas to grow
    (a collective re-export of IPC memory) several times (growth floor
    lowered by IGG_PUT_ARENA_FLOOR_MB), each exchange checked against the
    halo oracle; then small field sets again (profiles/r3_put_arena/: an
    export at a reused address mapped stale memory in the peers)."""
    _device("gpu")
    n = 40
    me, dims, nprocs, coords, comm = igg.init_global_grid(n, n, n, periodx=1, periody=1, periodz=1, quiet=True,
                                                          select_device=False, device_type="AMDGPU")
    gg = igg.get_global_grid()
    from igg.parallel import halo as H

    H.set_transport("put")
    sizes = []
    for k in (1, 3, 8, 20, 1, 5, 40, 2):
        fs, refs = [], []
        for i in range(k):
            A = torch.zeros(n, n, n, dtype=torch.float64)
            encode(A)
            A += 1000 * i
            refs.append(expected_after_halo(A, has_halo(A, gg), gg.neighbors.tolist()))
            fs.append(zero_boundaries(A.clone()).cuda())
        igg.update_halo_(*fs)
        igg.update_halo_(*fs)  # both arena halves
        for i, (X, R) in enumerate(zip(fs, refs)):
            got = X.cpu()
            assert torch.equal(got, R), f"rank {me} k={k} field {i}: mismatch at {(got != R).nonzero()[:5].tolist()}"
        sizes.append(gg.comm.mesh.arena_bytes >> 10)
        print(f"rank {me} k={k} arena {sizes[-1]} KiB OK", flush=True)
    assert len(set(sizes)) >= 3, f"the arena did not regrow: {sizes}"
    igg.finalize_global_grid()
    print(f"rank {me} put regrow OK", flush=True)


def scenario_acoustic_fused_soak(nx, ny, steps, periodic, graph):
    """Long fused acoustic run vs the update_halo_ path (put transport), compared
    after every step (eager) or every 4 (graph replays): reports the first
    diverging step, field and position on this rank."""
    from igg.models.acoustic2d import Acoustic2D

    _device("gpu")
    nx, ny, steps, per, graph = int(nx), int(ny), int(steps), int(periodic), int(graph)
    me, dims, nprocs, coords, comm = igg.init_global_grid(nx, ny, 1, periodx=per, periody=per, quiet=True,
                                                          select_device=False, device_type="AMDGPU")
    from igg.parallel import halo as H

    H.set_transport("put")
    a, b = Acoustic2D(dtype=torch.float32), Acoustic2D(dtype=torch.float32)
    assert b.set_fused(True)
    if graph:
        a.capture(steps=4)
        b.capture(steps=4)
    k = 4 if graph else 1
    first = None
    for s in range(0, steps, k):
        a.run(k)
        b.run(k)
        torch.cuda.synchronize()
        if first is None:
            for n in ("P", "Vx", "Vy"):
                x, y = getattr(a, n), getattr(b, n)
                if not torch.equal(x, y):
                    first = (s + k, n, (x != y).nonzero()[:4].tolist(), int((x != y).sum()))
                    break
    b.check()
    print(f"rank {me} coords {coords.tolist()} first divergence: {first}", flush=True)
    flag = comm.all_gather_object(first is None)
    b.close()
    igg.finalize_global_grid()
    assert all(flag), f"rank {me}: diverged {first}"
    print(f"rank {me} acoustic fused soak OK", flush=True)


def scenario_acoustic_fused_skew(nx, ny, rounds, per_round, periodic):
    """Fused acoustic steps under random host skew (a rank enqueues late, so
    its neighbours' exchanging waves wait inside their kernels for its previous
    step), graph replays with odd and even counts, one restore-like write with
    mark_modified; bitwise vs the update_halo_ path at the end."""
    import random
    import time

    from igg.models.acoustic2d import Acoustic2D

    _device("gpu")
    nx, ny, rounds, per_round, per = int(nx), int(ny), int(rounds), int(per_round), int(periodic)
    me, dims, nprocs, coords, comm = igg.init_global_grid(nx, ny, 1, periodx=per, periody=per, quiet=True,
                                                          select_device=False, device_type="AMDGPU")
    a, b = Acoustic2D(dtype=torch.float32), Acoustic2D(dtype=torch.float32)
    assert b.set_fused(True)
    b.capture(steps=4)
    total = 1
    rng = random.Random(99 + me)
    for k in range(rounds):
        time.sleep(rng.random() * 0.02)
        n = per_round + (k % 3)
        b.run(n)
        total += n
        if k == rounds // 2:
            a.run(total)
            total = 0
            torch.cuda.synchronize()
            for name in ("P", "Vx", "Vy", "P2", "Vx2", "Vy2"):
                getattr(b, name).copy_(getattr(a, name))
            b.mark_modified()
    a.run(total)
    torch.cuda.synchronize()
    b.check()
    for name in ("P", "Vx", "Vy", "P2", "Vx2", "Vy2"):
        x, y = getattr(a, name), getattr(b, name)
        if not torch.equal(x, y):
            raise AssertionError(f"rank {me}: {name} differs at {(x != y).nonzero()[:5].tolist()}")
    b.close()
    igg.finalize_global_grid()
    print(f"rank {me} acoustic fused skew OK")


def scenario_gather_async():
    """gather_async_: root pulls every block (IPC + copy engine), the caller
    overlaps other work, wait() reorders; then A may change again."""
    _device(os.environ.get("IGG_TEST_DEV", "gpu"))
    me, dims, nprocs, coords, comm = igg.init_global_grid(6, 5, 4, quiet=True, select_device=False,
                                                          device_type="AMDGPU")
    s = (6, 5, 4)
    for root in sorted({0, nprocs - 1}):
        for dt in (torch.float64, torch.float32):
            final = (torch.full(s, float(me + 1), dtype=torch.float64) * 1000
                     + torch.arange(120, dtype=torch.float64).view(s)).to(dt).cuda()
            A = torch.zeros(s, dtype=dt, device="cuda")
            G = torch.empty(dims[0] * 6, dims[1] * 5, dims[2] * 4, dtype=dt, device="cuda") if me == root else None
            # No host sync anywhere below. A becomes final only behind a long
            # kernel on every rank's stream (the root's is longer), and the
            # root zero-fills G behind it: the root's pulls must be ordered
            # after its own stream's fill (every copy stream waits on the
            # root's event) and after each peer's point where A is final (the
            # peers' interprocess events); after wait() the peers overwrite A
            # at once, which must queue behind the root's pulls on the device.
            delay = torch.rand(1536, 1536, device="cuda", dtype=torch.float64)
            for _ in range(8 if me == root else 4):
                delay = delay @ delay * 1e-3
            A.copy_(final)
            if me == root:
                G.zero_()
            h = igg.gather_async_(A, G, root=root)
            busy = torch.rand(256, 256, device="cuda") @ torch.rand(256, 256, device="cuda")  # overlapped work
            h.wait()
            A.fill_(-1)  # allowed after wait(): device-ordered behind the root's pulls
            torch.cuda.synchronize()
            del busy, delay
            if me == root:
                Gc = G.cpu().double()
                for p in range(nprocs):
                    c = igg.native.cart_coords(p, dims.tolist())
                    blk = Gc[c[0] * 6:(c[0] + 1) * 6, c[1] * 5:(c[1] + 1) * 5, c[2] * 4:(c[2] + 1) * 4]
                    exp = (torch.full(s, float(p + 1), dtype=torch.float64) * 1000
                           + torch.arange(120, dtype=torch.float64).view(s)).to(dt).double()
                    assert torch.equal(blk, exp), f"root {root}: block of rank {p} wrong"
            # snapshot=True: A may change right after the call (the copy is
            # stream-ordered before the change), the gather still sees the
            # values of the call
            A.copy_(final)
            if me == root:
                G.zero_()
            h = igg.gather_async_(A, G, root=root, snapshot=True)
            A.fill_(-5)  # before wait(): allowed with snapshot
            delay = torch.rand(1024, 1024, device="cuda", dtype=torch.float64)
            delay = delay @ delay
            h.wait()
            torch.cuda.synchronize()
            del delay
            if me == root:
                Gc = G.cpu().double()
                for p in range(nprocs):
                    c = igg.native.cart_coords(p, dims.tolist())
                    blk = Gc[c[0] * 6:(c[0] + 1) * 6, c[1] * 5:(c[1] + 1) * 5, c[2] * 4:(c[2] + 1) * 4]
                    exp = (torch.full(s, float(p + 1), dtype=torch.float64) * 1000
                           + torch.arange(120, dtype=torch.float64).view(s)).to(dt).double()
                    assert torch.equal(blk, exp), f"snapshot, root {root}: block of rank {p} wrong"
    igg.finalize_global_grid()
    print(f"rank {me} gather_async OK")


def scenario_fused_soak(nx, ny, nz, rounds, per_round):
    """Fused exchange under load: ``rounds`` x ``per_round`` graph-replayed
    fused steps with random host-side delays between rounds (ranks drift
    apart; the device-side neighbour barrier must absorb it), odd step counts
    (eager steps re-align the captured parity) and a sync_halo every few
    rounds; compared bitwise with stencil + update_halo_ at the end."""
    import random
    import time

    from igg.models.diffusion3d import Diffusion3D

    device = _device(os.environ.get("IGG_TEST_DEV", "gpu"))
    nx, ny, nz, rounds, per_round = int(nx), int(ny), int(nz), int(rounds), int(per_round)
    me, dims, nprocs, coords, comm = igg.init_global_grid(nx, ny, nz, periodx=1, periody=1, periodz=1,
                                                          quiet=True, select_device=False)
    v = int(os.environ.get("IGG_TEST_VARIANT", "0"))
    a = Diffusion3D(dtype=torch.float64, device=device, variant=_plain(v))
    b = Diffusion3D(dtype=torch.float64, device=device, variant=_plain(v))
    b.fused_variant, b.fused_mode = v, int(os.environ.get("IGG_TEST_FUSED_MODE", "0"))
    assert b.set_fused(True)
    b.step()
    b.capture(steps=4)
    rng = random.Random(1234 + me)
    total = 1  # steps b has done
    for k in range(rounds):
        time.sleep(rng.random() * 0.02)  # host skew: this rank enqueues late
        n = per_round + (k % 3)  # odd and even counts
        b.run(n)
        total += n
        if k % 7 == 6:
            b.sync_halo()
    a.run(total)
    b.sync_halo()
    torch.cuda.synchronize()
    b.check()
    if not torch.equal(a.T, b.T):
        bad = (a.T != b.T).nonzero()[:5].tolist()
        raise AssertionError(f"rank {me}: fused soak differs after {total} steps at {bad}")
    b.close()
    igg.finalize_global_grid()
    print(f"rank {me} fused soak OK ({total} steps)")


def scenario_checkpoint(dev, model, tmpdir):
    """Run 6 steps, checkpoint, run 5 more; a fresh model restored from the
    checkpoint and run 5 steps must match bitwise (per rank)."""
    from igg.models.acoustic2d import Acoustic2D
    from igg.models.diffusion3d import Diffusion3D

    device = _device(dev)
    is2d = model == "acoustic"
    me, dims, nprocs, coords, comm = igg.init_global_grid(18, 16, 1 if is2d else 14, periodx=1, quiet=True,
                                                          select_device=False,
                                                          device_type="none" if dev == "cpu" else "AMDGPU")
    make = (lambda: Acoustic2D(dtype=torch.float64, device=device)) if is2d else \
        (lambda: Diffusion3D(dtype=torch.float64, device=device))
    a = make()
    a.run(6)
    prefix = os.path.join(tmpdir, "ckpt")
    a.save(prefix, step=6)
    a.run(5)
    b = make()
    assert b.restore(prefix) == 6
    b.run(5)
    names = ("P", "Vx", "Vy") if is2d else ("T",)
    for n in names:
        assert torch.equal(getattr(a, n), getattr(b, n)), f"rank {me}: {n} differs after restart"
    igg.finalize_global_grid()
    print(f"rank {me} checkpoint OK")


def scenario_put_timeout():
    """Rank 1 skips one update_halo_: rank 0's bounded waits expire (short
    IGG_PUT_TIMEOUT), its kernels exit, and check_transport reports it."""
    import time

    from igg.parallel import halo as H

    me, dims, nprocs, coords, comm = igg.init_global_grid(8, 6, 5, periodx=1, quiet=True, select_device=False,
                                                          device_type="AMDGPU")
    A = torch.zeros(8, 6, 5, dtype=torch.float64, device="cuda")
    igg.update_halo_(A)  # a healthy exchange first
    torch.cuda.synchronize()
    H.check_transport()
    comm.barrier()
    if me == 0:
        t0 = time.time()
        igg.update_halo_(A)
        torch.cuda.synchronize()  # returns once the spin times out (no hang)
        waited = time.time() - t0
        # after the first timeout the sticky error makes later waits give up
        # at once: five more exchanges cost far less than five timeouts (2 s each)
        t1 = time.time()
        for _ in range(5):
            igg.update_halo_(A)
        torch.cuda.synchronize()
        assert time.time() - t1 < 1.5, time.time() - t1
        try:
            H.check_transport()
            raise AssertionError("expected a put-transport timeout error")
        except igg.IGGError as e:
            assert "timed out" in str(e)
        assert waited >= 1.0, waited
    comm.barrier()
    if me == 0:
        # The sticky error is reported by finalize, but only after every
        # resource was released: the grid is reset and can be re-initialised.
        try:
            igg.finalize_global_grid()
            raise AssertionError("expected finalize to report the put-transport timeout")
        except igg.IGGError as e:
            assert "timed out" in str(e)
        assert not igg.grid_is_initialized()
    else:
        igg.finalize_global_grid()
    print(f"rank {me} put timeout OK")


def scenario_put_skew(steps):
    """Ranks reach the exchanges at very different times (random host sleeps):
    the device-side waits absorb the skew and every halo stays exact."""
    import random
    import time

    steps = int(steps)
    me, dims, nprocs, coords, comm = igg.init_global_grid(7, 5, 6, periodx=1, periody=1, periodz=1, quiet=True,
                                                          select_device=False, device_type="AMDGPU")
    gg = igg.get_global_grid()
    rng = random.Random(1234 + me)
    A = torch.zeros(7, 5, 6, dtype=torch.float64)
    encode(A)
    ref = expected_after_halo(A, has_halo(A, gg), gg.neighbors.tolist())
    X = zero_boundaries(A.clone()).to("cuda")
    for k in range(steps):
        time.sleep(rng.random() * 0.05)
        X = zero_boundaries(X.cpu()).to("cuda") if k % 3 == 0 else X
        igg.update_halo_(X)
    got = X.cpu()
    assert torch.equal(got, ref), f"rank {me}: halo mismatch after skewed exchanges"
    from igg.parallel import halo as H

    H.check_transport()
    igg.finalize_global_grid()
    print(f"rank {me} put skew OK")


def scenario_ring(dev):
    """Transport-level ring exchange (test_update_halo.jl:697-743 analogue)."""
    device = _device(dev)
    me, dims, nprocs, coords, comm = igg.init_global_grid(8, 4, 4, dimx=0, dimy=1, dimz=1, periodx=1, quiet=True,
                                                          select_device=False,
                                                          device_type="none" if dev == "cpu" else "AMDGPU")
    gg = igg.get_global_grid()
    left, right = int(gg.neighbors[0, 0]), int(gg.neighbors[1, 0])
    # side-distinct payloads: what goes left is me + 0.25, what goes right me + 0.5
    # (with 2 ranks left == right: only the issue order tells the two apart)
    send = torch.cat([torch.full((16,), me + 0.25, dtype=torch.float64),
                      torch.full((16,), me + 0.5, dtype=torch.float64)]).to(device)
    recv = torch.zeros(32, dtype=torch.float64, device=device)
    t = comm.host_transport() if dev == "cpu" else comm.device_transport()
    recvs = [(recv.data_ptr() + 128, 128, right, 1), (recv.data_ptr(), 128, left, 0)]
    sends = [(send.data_ptr(), 128, left, 1), (send.data_ptr() + 128, 128, right, 0)]
    fn = {"gloo": comm._gloo_p2p, "gloo-staged": comm._staged_p2p}.get(t.name)
    stream = torch.cuda.current_stream().cuda_stream if dev != "cpu" else 0
    if fn is not None:
        fn(recvs, sends, dev != "cpu", stream)
    elif t.name == "rccl":
        # grouped ncclRecv/ncclSend: same-peer messages (2 ranks: left == right)
        # match in issue order, like the reference's tagged MPI messages
        t.p2p([r[:3] for r in recvs], [x[:3] for x in sends], stream)
    else:
        raise SystemExit(f"ring: transport {t.name!r} has no point-to-point interface")
    if dev != "cpu":
        torch.cuda.synchronize()
    r = recv.cpu()
    assert (r[:16] == left + 0.5).all() and (r[16:] == right + 0.25).all(), f"rank {me}: ring wrong {r}"
    igg.finalize_global_grid()
    print(f"rank {me} ring OK")


def scenario_barrier_timeout():
    """Rank 1 never reaches the barrier: rank 0's bounded barrier
    (IGG_COMM_TIMEOUT) raises IGGError naming the failure instead of hanging."""
    import time

    me, dims, nprocs, coords, comm = igg.init_global_grid(6, 5, 4, quiet=True, device_type="none")
    comm.barrier()  # a healthy barrier first
    if me == 0:
        t0 = time.time()
        try:
            comm.barrier()
            raise AssertionError("expected a barrier timeout")
        except igg.IGGError as e:
            assert "IGG_COMM_TIMEOUT" in str(e), str(e)
        waited = time.time() - t0
        assert 1.5 <= waited < 30, waited
        assert comm.aborted
    else:
        time.sleep(float(os.environ["IGG_COMM_TIMEOUT"]) + 4)
    print(f"rank {me} barrier timeout OK", flush=True)
    os._exit(0)  # the process group is broken by design: skip finalize


def scenario_collectives(dev):
    """comm_cart interop: tensor all-reduce / broadcast and a scalar residual."""
    device = _device(dev)
    me, dims, nprocs, coords, comm = igg.init_global_grid(6, 5, 4, quiet=True, select_device=False,
                                                          device_type="AMDGPU" if dev != "cpu" else "none")
    n = nprocs
    for dtype in (torch.float64, torch.float32, torch.int32):
        t = torch.full((5,), me + 1, dtype=dtype, device=device)
        assert comm.allreduce_(t, "sum") is t
        assert (t.cpu() == n * (n + 1) // 2).all(), t
        for op, want in (("max", n), ("min", 1), ("prod", __import__("math").factorial(n))):
            t = torch.full((3,), me + 1, dtype=dtype, device=device)
            comm.allreduce_(t, op)
            assert (t.cpu() == want).all(), (op, t)
    for root in sorted({0, n - 1}):
        t = torch.arange(7, dtype=torch.float64, device=device) * (me + 1)
        comm.bcast_(t, root=root)
        assert torch.equal(t.cpu(), torch.arange(7, dtype=torch.float64) * (root + 1)), (root, t)
    if dev != "cpu":  # complex tensors reduce as real pairs
        t = torch.full((3,), complex(me + 1, -(me + 1)), dtype=torch.complex64, device=device)
        comm.allreduce_(t, "sum")
        assert (t.cpu() == complex(n * (n + 1) // 2, -(n * (n + 1) // 2))).all(), t
    r = comm.allreduce(float(me), "max")
    assert r == float(n - 1), r
    # one RCCL communicator per rank: GPU collectives ride the grid's native
    # communicator, no torch nccl process group is created next to it
    assert comm.torch_nccl is None
    try:
        comm.allreduce_(torch.zeros(1), "mean")
        raise AssertionError("expected IGGError for an unknown op")
    except igg.IGGError:
        pass
    if dev != "cpu":
        torch.cuda.synchronize()
    igg.finalize_global_grid()
    print(f"rank {me} collectives OK")



def scenario_suite(*items):
    """Several scenarios in ONE launch of the ranks (the multigpu tier's time
    budget: one process start, one torch import and one rendezvous per suite
    instead of per check). ``items``: "name:arg:arg|VAR=val;VAR=val" - the
    scenario's env vars are set for it only. The grid is re-initialised per
    item on the same process group (init_MPI / finalize_MPI false in between).
    Progress lines name every item, so a hang or failure is attributable."""
    import time

    import torch.distributed as dist

    orig_init, orig_fin = igg.init_global_grid, igg.finalize_global_grid

    def init(*a, **k):
        k.setdefault("init_MPI", not dist.is_initialized())
        return orig_init(*a, **k)

    def fin(*a, **k):
        k.setdefault("finalize_MPI", False)
        return orig_fin(*a, **k)

    igg.init_global_grid, igg.finalize_global_grid = init, fin
    me = int(os.environ.get("RANK", "0"))
    t_all = time.time()
    for item in items:
        spec, _, envs = item.partition("|")
        name, *args = spec.split(":")
        saved = {}
        for kv in filter(None, envs.split(";")):
            k, v = kv.split("=", 1)
            saved[k] = os.environ.get(k)
            os.environ[k] = v
        t0 = time.time()
        try:
            globals()[f"scenario_{name}"](*args)
        except BaseException as e:
            print(f"rank {me} suite item {item!r} FAILED: {type(e).__name__}: {e}", flush=True)
            raise
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        print(f"rank {me} suite item {item!r} OK in {time.time() - t0:.1f} s", flush=True)
    igg.init_global_grid, igg.finalize_global_grid = orig_init, orig_fin
    if dist.is_initialized():
        dist.destroy_process_group()
    print(f"rank {me} suite OK ({len(items)} items, {time.time() - t_all:.1f} s)", flush=True)


if __name__ == "__main__":
    name, *args = sys.argv[1:]
    globals()[f"scenario_{name}"](*args)
