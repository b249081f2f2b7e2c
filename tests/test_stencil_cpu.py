"""Host (C++) diffusion kernel vs the plain-PyTorch fp64 reference of the
reference example's five broadcasts, boundary/interior box decomposition, and
the CPU config of BASELINE.json (32^3 Float64, world_size=1)."""
import pytest
import torch

import igg
from igg.ops import stencil


@pytest.mark.parametrize("dtype,tol", [(torch.float64, 1e-12), (torch.float32, 1e-4)])
def test_host_kernel_matches_reference(dtype, tol):
    g = torch.Generator().manual_seed(1)
    T = torch.rand(9, 11, 13, generator=g, dtype=torch.float64)
    Cp = 1 + torch.rand(9, 11, 13, generator=g, dtype=torch.float64)
    kw = dict(lam=1.3, dt=0.01, dx=0.5, dy=0.7, dz=0.9)
    ref = stencil.diffusion3d_reference(T, Cp, **kw)
    T2 = T.to(dtype).clone()
    stencil.diffusion3d_(T2, T.to(dtype), Cp.to(dtype), **kw)
    assert (T2.double() - ref).abs().max().item() < tol


def test_boxes_partition_the_inner_region():
    n = (20, 17, 40)
    for active in ([1, 1, 1], [1, 0, 0], [0, 0, 1], [0, 1, 1]):
        slabs, interior = stencil.split_boundary(n, active, (1, 2, 15))
        mask = torch.zeros(n, dtype=torch.int32)
        for lo, hi in slabs + [interior]:
            mask[lo[0]:hi[0], lo[1]:hi[1], lo[2]:hi[2]] += 1
        assert (mask[1:-1, 1:-1, 1:-1] == 1).all()
        assert mask.sum() == (n[0] - 2) * (n[1] - 2) * (n[2] - 2)
        # the send planes (index 1 and n-2) of active dims lie in slabs
        for d in range(3):
            if active[d]:
                for idx in (1, n[d] - 2):
                    for lo, hi in [interior]:
                        assert not (lo[d] <= idx < hi[d])


def test_sliced_update_equals_full_update():
    g = torch.Generator().manual_seed(2)
    n = (12, 10, 33)
    T = torch.rand(n, generator=g, dtype=torch.float64)
    Cp = 1 + torch.rand(n, generator=g, dtype=torch.float64)
    kw = dict(lam=1.0, dt=0.01, dx=0.3, dy=0.3, dz=0.3)
    full = T.clone()
    stencil.diffusion3d_(full, T, Cp, **kw)
    part = T.clone()
    slabs, interior = stencil.split_boundary(n, [1, 1, 1], (1, 1, 15))
    stencil.diffusion3d_(part, T, Cp, boxes=slabs, **kw)
    stencil.diffusion3d_(part, T, Cp, boxes=[interior], **kw)
    assert torch.equal(full, part)


def test_cpu_config_32cubed_periodic_runs():
    """BASELINE.json config 1: 3-D diffusion 32^3 Float64 on CPU, world_size=1."""
    from igg.models.diffusion3d import Diffusion3D

    igg.init_global_grid(32, 32, 32, periodx=1, periody=1, periodz=1, quiet=True, init_MPI=False)
    m = Diffusion3D(dtype=torch.float64, device="cpu")
    e0 = m.T.sum().item()
    ref = m.T.clone()
    for _ in range(5):
        ref = stencil.diffusion3d_reference(ref, m.Cp, lam=m.lam, dt=m.dt, dx=m.dx, dy=m.dy, dz=m.dz)
        igg.update_halo_(ref)
    m.run(5)
    assert torch.allclose(m.T, ref, rtol=0, atol=1e-12)
    assert abs(m.T.sum().item() - e0) / abs(e0) < 0.05
    igg.finalize_global_grid(finalize_MPI=False)


def test_invalid_arguments():
    T = torch.zeros(5, 5, 5)
    with pytest.raises(igg.IGGError):
        stencil.diffusion3d_(T, T, T, lam=1, dt=1, dx=1, dy=1, dz=1)  # aliasing
    with pytest.raises(igg.IGGError):
        stencil.diffusion3d_(torch.zeros(5, 5, 5, dtype=torch.int32), torch.zeros(5, 5, 5, dtype=torch.int32),
                             torch.zeros(5, 5, 5, dtype=torch.int32), lam=1, dt=1, dx=1, dy=1, dz=1)
    with pytest.raises(igg.IGGError):
        stencil.diffusion3d_(torch.zeros(5, 5, 5), torch.zeros(5, 5, 5), torch.zeros(5, 5, 5), lam=1, dt=1, dx=1,
                             dy=1, dz=1, boxes=[((0, 1, 1), (4, 4, 4))])


def test_overlap_serial_rule_parses_queue_counts(monkeypatch):
    """The overlapped step runs its parts in stream order when the process has
    fewer hardware queues than the step has concurrent streams; the queue
    count is parsed as an integer (' 01' is one queue)."""
    from igg.models import diffusion3d as D

    for v, streams, want in (("1", 2, True), (" 01", 2, True), ("2", 2, False), ("2", 3, True), ("4", 3, False),
                             ("", 3, False), ("junk", 3, False)):
        monkeypatch.setenv("GPU_MAX_HW_QUEUES", v)
        assert D._serial_overlap(streams) is want, (v, streams)
