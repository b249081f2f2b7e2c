"""Every HIP diffusion kernel variant on arbitrary sub-boxes (the boundary slabs
and interior boxes of the overlapped step) against the plain-PyTorch fp64
reference of the reference example's update (diffusion3D_multigpu_CuArrays_novis.jl).
Cells outside the boxes must stay untouched."""
import itertools

import pytest
import torch

import igg  # noqa: F401
from igg.ops import stencil

pytestmark = pytest.mark.gpu

KW = dict(lam=1.0, dt=0.01, dx=0.3, dy=0.25, dz=0.2)


def _fields(shape, dtype, gpu):
    g = torch.Generator().manual_seed(1)
    T = torch.rand(shape, generator=g, dtype=torch.float64)
    Cp = 1 + torch.rand(shape, generator=g, dtype=torch.float64)
    return T, Cp, T.to(dtype).to(gpu), Cp.to(dtype).to(gpu)


def _run_boxes(shape, boxes, variant, dtype, gpu):
    T, Cp, Tg, Cpg = _fields(shape, dtype, gpu)
    sentinel = -7.0
    T2g = torch.full(shape, sentinel, dtype=dtype, device=gpu)
    stencil.diffusion3d_(T2g, Tg, Cpg, boxes=boxes, variant=variant, **KW)
    if T2g.is_cuda:
        torch.cuda.synchronize()
    ref = stencil.diffusion3d_reference(Tg.double().cpu(), Cpg.double().cpu(), **KW)
    got = T2g.double().cpu()
    mask = torch.zeros(shape, dtype=torch.bool)
    for lo, hi in boxes:
        mask[lo[0]:hi[0], lo[1]:hi[1], lo[2]:hi[2]] = True
    tol = 1e-12 if dtype == torch.float64 else 1e-5
    assert (got[~mask] == sentinel).all(), "kernel wrote outside its boxes"
    err = (got[mask] - ref[mask]).abs().max().item() if mask.any() else 0.0
    return err, tol


@pytest.mark.parametrize("variant", stencil.compiled_variants())
def test_variant_full_inner_box(gpu, variant):
    for shape in [(24, 20, 18), (37, 33, 131), (9, 70, 5), (20, 22, 72)]:
        err, tol = _run_boxes(shape, [stencil.inner_box(shape)], variant, torch.float64, gpu)
        assert err < tol, (shape, err)


@pytest.mark.parametrize("variant", stencil.compiled_variants())
def test_variant_split_boxes(gpu, variant):
    """Slabs + interior of split_boundary for one-sided and two-sided neighbours."""
    shape = (24, 20, 18)
    for act, w in itertools.product([[(0, 1), (1, 0), (0, 1)], [(1, 1), (1, 1), (1, 1)], [(1, 0), (0, 0), (1, 1)]],
                                    [(1, 1, 1), (1, 1, 127), (2, 3, 63)]):
        slabs, interior = stencil.split_boundary(shape, act, w)
        for boxes in (slabs, [interior], list(slabs) + [interior]):
            boxes = [b for b in boxes if all(h > l for l, h in zip(b[0], b[1]))]
            if not boxes:
                continue
            err, tol = _run_boxes(shape, boxes, variant, torch.float64, gpu)
            assert err < tol, (act, w, boxes, err)


@pytest.mark.parametrize("variant", [0, 11, 21, 24])
def test_variant_float32(gpu, variant):
    shape = (40, 36, 70)
    err, tol = _run_boxes(shape, [stencil.inner_box(shape)], variant, torch.float32, gpu)
    assert err < tol


_HX_PAIRS = [(21, 0), (22, 2), (23, 9), (24, 11), (25, 14), (32, 11), (33, 0), (34, 9),
             (35, 14), (36, 11), (37, 9), (38, 26), (39, 0), (40, 11)]


@pytest.mark.parametrize("hx,tiling", [p for p in _HX_PAIRS if set(p) <= set(stencil.compiled_variants())])
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_restrict_form_bitwise_equals_vkernel(gpu, hx, tiling, dtype):
    """Variants 21-25 (inner box through fused_kernels.hip without exchange
    features) compute exactly what the stencil_kernels.hip variant with the
    same tiling computes; 32-39 (non-temporal Cp, lane-distributed z-segment
    edges) exactly what the plain restrict form computes."""
    shape = (26, 35, 136)
    _, _, Tg, Cpg = _fields(shape, dtype, gpu)
    a = torch.zeros_like(Tg)
    b = torch.zeros_like(Tg)
    stencil.diffusion3d_(a, Tg, Cpg, variant=tiling, **KW)
    stencil.diffusion3d_(b, Tg, Cpg, variant=hx, **KW)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


def _nan_padded(shape, dtype, gpu, src, pad=4096):
    """A view of ``src`` in the middle of a buffer filled with NaN: any read
    outside the array that leaks into a stored value shows up as NaN."""
    n = src.numel()
    buf = torch.full((n + 2 * pad,), float("nan"), dtype=dtype, device=gpu)
    v = buf[pad:pad + n].view(shape)
    v.copy_(src)
    return v


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_variants_ignore_memory_around_arrays(gpu, dtype):
    """Kernels never let a value from outside T / Cp (e.g. the gaps of the
    model's carved buffer) reach a stored cell, for every variant, grid-rounds
    setting and the boundary-slab / interior boxes of the overlapped step."""
    bad = []
    for shape in [(40, 33, 70), (37, 33, 131), (24, 20, 18), (9, 70, 5), (20, 22, 72)]:
        T, Cp, Tg, Cpg = _fields(shape, dtype, gpu)
        Tn, Cpn = _nan_padded(shape, dtype, gpu, Tg), _nan_padded(shape, dtype, gpu, Cpg)
        ref = stencil.diffusion3d_reference(Tg.double().cpu(), Cpg.double().cpu(), **KW)
        slabs, interior = stencil.split_boundary(shape, [(1, 1), (1, 1), (1, 1)], (1, 1, 1))
        box_sets = [[stencil.inner_box(shape)], [b for b in list(slabs) + [interior]
                                                 if all(h > l for l, h in zip(b[0], b[1]))]]
        for v in stencil.compiled_variants():
            for r in (0, 1, 2, 3):
                for boxes in box_sets:
                    T2 = _nan_padded(shape, dtype, gpu, Tg)
                    stencil.diffusion3d_(T2, Tn, Cpn, boxes=boxes, variant=v, rounds=r, **KW)
                    torch.cuda.synchronize()
                    got = T2.double().cpu()
                    tol = 1e-12 if dtype == torch.float64 else 1e-5
                    inner = (slice(1, -1),) * 3
                    err = (got[inner] - ref[inner]).abs().max().item()
                    if not err < tol:
                        bad.append((shape, v, r, len(boxes), err))
    assert not bad, bad[:10]


def test_autotune_pingpong_stage(gpu):
    """The model autotune's second stage re-times its front in the time loop's
    ping-pong shape on the model's own buffers and restores T afterwards: an
    autotuned model starts from the same state as one with a pinned variant."""
    from igg.models.diffusion3d import PINGPONG_FRONT, Diffusion3D

    igg.init_global_grid(40, 36, 72, quiet=True, init_MPI=False)
    try:
        m = Diffusion3D(dtype=torch.float64)
        ref = Diffusion3D(dtype=torch.float64, variant=0)
        pp = [k for k in m.variant_times if k.endswith("/pp")]
        assert len(pp) == PINGPONG_FRONT
        assert f"{m.variant}@r{m.rounds}/pp" in pp  # the pick comes from stage 2
        assert torch.equal(m.T, ref.T)
        m.run(4)
        ref.run(4)
        torch.cuda.synchronize()
        assert torch.equal(m.T, ref.T)  # variants are bitwise interchangeable
    finally:
        igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.parametrize("variant", stencil.compiled_variants())
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_halo_z_whole_line_edges(gpu, variant, dtype):
    """halo_z=True: the full inner box computes the same interior bitwise, and
    the only other cells written are T2's z halo elements (z = 0, nz-1) of the
    inner rows, which get T's values; a box that does not span the whole inner
    z range writes nothing outside itself."""
    for shape in [(24, 20, 72), (9, 70, 16), (20, 22, 132)]:
        T, Cp, Tg, Cpg = _fields(shape, dtype, gpu)
        a = torch.full(shape, -7.0, dtype=dtype, device=gpu)
        b = a.clone()
        stencil.diffusion3d_(a, Tg, Cpg, variant=variant, **KW)
        stencil.diffusion3d_(b, Tg, Cpg, variant=variant, halo_z=True, **KW)
        torch.cuda.synchronize()
        n0, n1, n2 = shape
        inner = (slice(1, n0 - 1), slice(1, n1 - 1))
        assert torch.equal(a[1:-1, 1:-1, 1:-1], b[1:-1, 1:-1, 1:-1]), shape
        want = a.clone()
        want[inner + (0,)] = Tg[inner + (0,)]
        want[inner + (n2 - 1,)] = Tg[inner + (n2 - 1,)]
        # vector kernels write whole edge vectors; the scalar fallbacks (and
        # shapes the vector path cannot take) leave the halo untouched
        same_as_plain = torch.equal(b, a)
        assert same_as_plain or torch.equal(b, want), (shape, variant)
        c = torch.full(shape, -7.0, dtype=dtype, device=gpu)
        box = [([1, 1, 2], [n0 - 1, n1 - 1, n2 - 1])]
        stencil.diffusion3d_(c, Tg, Cpg, variant=variant, boxes=box, halo_z=True, **KW)
        torch.cuda.synchronize()
        mask = torch.zeros(shape, dtype=torch.bool, device=gpu)
        mask[1:-1, 1:-1, 2:-1] = True
        assert (c[~mask] == -7.0).all(), (shape, variant)
        assert torch.equal(c[mask], a[mask]), (shape, variant)
