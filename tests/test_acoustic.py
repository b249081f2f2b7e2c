"""2-D staggered acoustic solver (models/acoustic2d.py): the native fused step
(C++ host path here, HIP kernel in the gpu tests) against the plain-PyTorch
reference, and the multi-process run (2x2 ranks, staggered Vx/Vy halos with
mixed overlaps) against the same physics on the implicit global grid."""
import pytest
import torch

import igg
from igg._native import native
from igg.models.acoustic2d import Acoustic2D, acoustic2d_reference
from tests._mp import run_ranks


def _fields(nx, ny, dtype, device="cpu"):
    g = torch.Generator().manual_seed(3)
    P = torch.rand(nx, ny, generator=g, dtype=torch.float64)
    Vx = torch.rand(nx + 1, ny, generator=g, dtype=torch.float64)
    Vy = torch.rand(nx, ny + 1, generator=g, dtype=torch.float64)
    return [t.to(dtype).to(device) for t in (P, Vx, Vy)]


def _step(P, Vx, Vy, dev, **kw):
    P2, Vx2, Vy2 = torch.empty_like(P), torch.empty_like(Vx), torch.empty_like(Vy)
    s = torch.cuda.current_stream().cuda_stream if dev else 0
    native.acoustic2d(P2.data_ptr(), Vx2.data_ptr(), Vy2.data_ptr(), P.data_ptr(), Vx.data_ptr(), Vy.data_ptr(),
                      P.shape[0], P.shape[1], kw["dt"] * kw["K"], kw["dt"] / kw["rho"], 1 / kw["dx"], 1 / kw["dy"],
                      P.element_size(), dev, s)
    return P2, Vx2, Vy2


KW = dict(dt=0.01, K=1.3, rho=0.8, dx=0.1, dy=0.07)


@pytest.mark.parametrize("dtype,tol", [(torch.float64, 1e-13), (torch.float32, 2e-6)])
@pytest.mark.parametrize("shape", [(7, 5), (33, 70), (1, 4)])
def test_host_step_matches_reference(dtype, tol, shape):
    P, Vx, Vy = _fields(*shape, dtype)
    got = _step(P, Vx, Vy, False, **KW)
    ref = acoustic2d_reference(P, Vx, Vy, **KW)
    for g, r in zip(got, ref):
        assert (g.double() - r).abs().max().item() < tol


def test_model_single_process_cpu():
    igg.init_global_grid(20, 16, 1, quiet=True, init_MPI=False)
    m = Acoustic2D(dtype=torch.float64)
    P, Vx, Vy = m.P.clone(), m.Vx.clone(), m.Vy.clone()
    m.run(5)
    for _ in range(5):
        P, Vx, Vy = acoustic2d_reference(P, Vx, Vy, dt=m.dt, K=m.K, rho=m.rho, dx=m.dx, dy=m.dy)
    assert (m.P - P).abs().max().item() < 1e-12
    assert (m.Vx - Vx).abs().max().item() < 1e-12 and (m.Vy - Vy).abs().max().item() < 1e-12
    assert m.Vx.shape == (21, 16) and m.Vy.shape == (20, 17)
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.parametrize("nprocs", [2, 4])
def test_multirank_matches_global(nprocs):
    run_ranks(nprocs, "acoustic", "cpu", 12, 10, 6)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 1, 2])
@pytest.mark.parametrize("dtype,tol", [(torch.float64, 1e-13), (torch.float32, 2e-6)])
@pytest.mark.parametrize("shape", [(130, 257), (64, 63), (200, 64), (3, 2), (130, 256), (17, 1000), (5, 8)])
def test_gpu_step_matches_reference(gpu, variant, dtype, tol, shape):
    P, Vx, Vy = _fields(*shape, dtype, gpu)
    native.acoustic2d_set_variant(variant)
    try:
        got = _step(P, Vx, Vy, True, **KW)
        torch.cuda.synchronize()
    finally:
        native.acoustic2d_set_variant(2)
    ref = acoustic2d_reference(P.cpu(), Vx.cpu(), Vy.cpu(), **KW)
    for g, r in zip(got, ref):
        assert (g.cpu().double() - r).abs().max().item() < tol


@pytest.mark.gpu
def test_gpu_multirank_put_matches_global():
    run_ranks(4, "acoustic", "gpu", 40, 36, 8, env_extra={"IGG_TRANSPORT": "put"})


@pytest.mark.gpu
def test_gpu_model_graph_matches_eager(gpu):
    igg.init_global_grid(64, 48, 1, periodx=1, periody=1, quiet=True, init_MPI=False)
    a, b = Acoustic2D(dtype=torch.float32), Acoustic2D(dtype=torch.float32)
    a.run(9)
    b.step()
    b.capture(steps=4)
    b.run(8)
    torch.cuda.synchronize()
    assert torch.equal(a.P, b.P) and torch.equal(a.Vx, b.Vx)
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.gpu
@pytest.mark.parametrize("fused", [False, True])
def test_gpu_graph_after_odd_step_counts(gpu, fused):
    """run() after an odd number of steps (and after a restore-like write with
    mark_modified) realigns the buffer roles the graph was captured with."""
    igg.init_global_grid(64, 48, 1, periodx=1, periody=1, quiet=True, init_MPI=False)
    a, b = Acoustic2D(dtype=torch.float32), Acoustic2D(dtype=torch.float32)
    if fused:
        assert b.set_fused(True)
    b.capture(steps=4)
    a.run(1)  # capture ran one eager step
    for k in (5, 3, 8, 7):
        a.run(k)
        b.run(k)
    saved = {n: getattr(a, n).clone() for n in ("P", "Vx", "Vy", "P2", "Vx2", "Vy2")}
    for m in (a, b):
        for n, t in saved.items():
            getattr(m, n).copy_(t)
    b.mark_modified()
    a.run(9)
    b.run(9)
    torch.cuda.synchronize()
    b.check()
    assert _same(a, b)
    b.close()
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("shape", [(300, 1024), (64, 520), (9, 16)])
def test_gpu_vector_march_bitwise_equals_march(gpu, dtype, shape):
    """Variant 2 (16 B per lane) evaluates the same expressions as variant 1
    (up to the compiler's FMA contraction choices: a few ulp)."""
    P, Vx, Vy = _fields(*shape, dtype, gpu)
    out = []
    for v in (1, 2):
        native.acoustic2d_set_variant(v)
        try:
            out.append(_step(P, Vx, Vy, True, **KW))
            torch.cuda.synchronize()
        finally:
            native.acoustic2d_set_variant(2)
    eps = torch.finfo(dtype).eps
    for a, b in zip(*out):
        assert torch.allclose(a, b, rtol=8 * eps, atol=8 * eps)


def _fused_pair(shape, periods, dtype, loopback=False):
    from igg.parallel import halo as H

    igg.init_global_grid(shape[0], shape[1], 1, periodx=periods[0], periody=periods[1], quiet=True, init_MPI=False)
    if loopback:
        H.enable_loopback((bool(periods[0]), bool(periods[1]), False))
    a, b = Acoustic2D(dtype=dtype), Acoustic2D(dtype=dtype)
    assert b.set_fused(True)
    return a, b


def _same(a, b):
    bad = []
    for n in ("P", "Vx", "Vy", "P2", "Vx2", "Vy2"):
        x, y = getattr(a, n), getattr(b, n)
        if not torch.equal(x, y):
            d = (x != y).nonzero()
            bad.append(f"{n}: {d.shape[0]} entries, first {d[:4].tolist()}, max |diff| "
                       f"{(x.double() - y.double()).abs().max().item():.3e}")
    assert not bad, "; ".join(bad)
    return True


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("periods", [(1, 0), (0, 1), (1, 1)])
@pytest.mark.parametrize("shape", [(64, 48), (37, 520), (9, 16), (40, 496)])
def test_gpu_fused_matches_update_halo(gpu, dtype, periods, shape):
    """Fused exchange (the kernel stores the staggered boundary faces into the
    neighbours' next Vx2/Vy2; here the periodic neighbour is this rank) is
    bitwise equal to kernel + update_halo_(Vx2, Vy2) in every field."""
    a, b = _fused_pair(shape, periods, dtype)
    a.run(9)
    b.run(9)
    torch.cuda.synchronize()
    b.check()
    assert _same(a, b)
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.gpu
def test_gpu_fused_loopback_graph_and_switch(gpu):
    """Loopback grid (every face through the remote path), hipGraph replays,
    switching back to update_halo_ and on again."""
    a, b = _fused_pair((66, 64), (1, 1), torch.float32, loopback=True)
    a.run(3)
    b.run(3)
    b.capture(steps=4)
    a.run(12)
    b.run(12)
    torch.cuda.synchronize()
    b.check()
    assert _same(a, b)
    b.set_fused(False)
    a.run(3)
    b.run(3)
    assert b.set_fused(True)
    a.run(4)
    b.run(4)
    torch.cuda.synchronize()
    assert _same(a, b)
    b.close()
    igg.finalize_global_grid(finalize_MPI=False)


def _bench_module():
    import importlib.util as ilu
    import os

    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")
    spec = ilu.spec_from_file_location("bench_mod", path)
    b = ilu.module_from_spec(spec)
    spec.loader.exec_module(b)
    return b


@pytest.mark.gpu
@pytest.mark.parametrize("loopback", [False, True])
def test_gpu_fused_after_local_steps(gpu, loopback):
    """The bench's efficiency phase runs local steps (no exchange) on the
    model, then restores its state: the fused step is bitwise equal to the
    update_halo_ path afterwards (a halo exchange alone does not repair the
    staggered fields' doubly computed planes: the fused post-check failed
    after it, profiles/r5_checks/c16)."""
    bench = _bench_module()
    a, b = _fused_pair((66, 64), (1, 1), torch.float32, loopback=loopback)
    for m in (a, b):
        m.run(3)
    saved = bench._begin_local_steps(b)
    assert saved is not None
    for _ in range(5):
        b.local_step()
    bench._end_local_steps(b, saved)
    assert b._entry
    b.capture(steps=4)
    a.run(1)  # capture ran one eager step
    a.run(12)
    b.run(12)
    torch.cuda.synchronize()
    b.check()
    assert _same(a, b)
    b.close()
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.gpu
@pytest.mark.parametrize("nprocs,per,sync_kernel", [(2, 1, 0), (4, 0, 0), (4, 1, 0), (4, 1, 1)])
def test_gpu_fused_multirank(nprocs, per, sync_kernel):
    """Ranks sharing one GPU (put transport for the update_halo_ reference):
    fused == update_halo_ bitwise on every rank, incl. graph replays; step
    synchronisation inside the fused kernel (default) or by a sync kernel."""
    env = {"IGG_TRANSPORT": "put", "IGG_PUT_TIMEOUT": "20", "IGG_FUSED_SYNC_KERNEL": str(sync_kernel)}
    if nprocs > 2:
        env["GPU_MAX_HW_QUEUES"] = "1"
    run_ranks(nprocs, "acoustic_fused", "gpu", 40, 36, 12, per, env_extra=env, timeout=150)


@pytest.mark.gpu
@pytest.mark.parametrize("sync_kernel", [0, 1])
def test_gpu_fused_multirank_skew(sync_kernel):
    """4 ranks on one GPU, random host skew between graph-replayed fused steps:
    the step synchronisation absorbs the drift; bitwise vs update_halo_."""
    env = {"IGG_TRANSPORT": "put", "IGG_PUT_TIMEOUT": "20", "IGG_FUSED_SYNC_KERNEL": str(sync_kernel),
           "GPU_MAX_HW_QUEUES": "1"}
    run_ranks(4, "acoustic_fused_skew", 40, 36, 12, 9, 1, env_extra=env, timeout=150)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(64, 48), (37, 520), (40, 496), (9, 16)])
def test_gpu_in_kernel_step_sync_counts_every_step(gpu, shape):
    """EPOCH advances once per fused step and COUNT returns to 0 (the host's
    count of exchanging waves matches the kernel's)."""
    a, b = _fused_pair(shape, (1, 1), torch.float32)
    assert not b._fa.in_kernel_sync  # the acoustic default: the sync kernel (put.hpp)
    b._fa.set_step_sync(0)
    assert b._fa.in_kernel_sync
    e0 = b._fa.flag(0)
    b.run(5)
    torch.cuda.synchronize()
    # + the entry barrier and run()'s exit barrier (drain)
    assert b._fa.flag(0) == e0 + 7 and b._fa.flag(2) == 0
    a.run(5)
    torch.cuda.synchronize()
    assert _same(a, b)
    b.close()
    igg.finalize_global_grid(finalize_MPI=False)
