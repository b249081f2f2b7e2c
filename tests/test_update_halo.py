"""Port of test/test_update_halo.jl for CPU tensors (single process): argument
checks, buffer allocation/reinterpretation, send/recv ranges, face pack/unpack,
and full halo updates with the bitwise coordinate-encoding oracle."""
import pytest
import torch

import igg
from igg import IGGError
from igg.parallel import halo as H
from tests.helpers import encode, expected_after_halo, has_halo, zero_boundaries

nx, ny, nz = 7, 5, 6


def _prod_sorted(t):
    s = sorted(t.shape)
    out = 1
    for v in s[1:]:
        out *= v
    return out


# --- 1. argument checks -------------------------------------------------------
def test_argument_checks():
    igg.init_global_grid(nx, ny, nz, quiet=True, init_MPI=False)
    P = torch.zeros(nx, ny, nz)
    Sxz = torch.zeros(nx - 2, ny - 1, nz - 2)
    A = torch.zeros(nx - 1, ny + 2, nz + 1)
    A2 = A
    Z = torch.zeros(nx - 1, ny + 2, nz + 1, dtype=torch.complex128)
    Z2 = Z
    with pytest.raises(IGGError, match="position 2 has no halo"):
        igg.update_halo_(P, Sxz, A)
    with pytest.raises(IGGError, match="positions 2 and 4 have no halo"):
        igg.update_halo_(P, Sxz, A, Sxz)
    with pytest.raises(IGGError, match="position 3 is a duplicate of the one at the position 2"):
        igg.update_halo_(P, A, A)
    with pytest.raises(IGGError, match="duplicate"):
        igg.update_halo_(P, A, A2)
    with pytest.raises(IGGError, match="duplicate"):
        igg.update_halo_(P, A, A, A2)
    with pytest.raises(IGGError, match="duplicate"):
        igg.update_halo_(Z, Z2)
    with pytest.raises(IGGError, match="position 2 is of different type"):
        igg.update_halo_(Z, P)
    with pytest.raises(IGGError, match="positions 2 and 3 are of different type"):
        igg.update_halo_(Z, P, A)
    with pytest.raises(IGGError, match="dense"):
        igg.update_halo_(torch.zeros(nx, ny, 2 * nz)[:, :, ::2])
    igg.finalize_global_grid(finalize_MPI=False)


def test_gpu_tensor_without_gpu_enabled():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU tensor")
    igg.init_global_grid(nx, ny, nz, quiet=True, init_MPI=False, device_type="CUDA")
    with pytest.raises(IGGError, match="AMDGPU is not enabled"):
        igg.update_halo_(torch.zeros(nx, ny, nz, device="cuda"))
    igg.finalize_global_grid(finalize_MPI=False)


# --- 2. buffer allocation -------------------------------------------------------
def test_buffer_allocation():
    igg.init_global_grid(nx, ny, nz, periodx=1, periody=1, periodz=1, quiet=True, init_MPI=False)
    P = torch.zeros(nx, ny, nz, dtype=torch.float64)
    A = torch.zeros(nx - 1, ny + 2, nz + 1, dtype=torch.float64)
    B = torch.zeros(nx + 1, ny + 2, nz + 3, dtype=torch.float32)
    C = torch.zeros(nx + 1, ny + 1, nz + 1, dtype=torch.float32)
    Z = torch.zeros(nx, ny, nz, dtype=torch.complex64)
    Y = torch.zeros(nx - 1, ny + 2, nz + 1, dtype=torch.complex64)
    # free buffers
    H.free_update_halo_buffers()
    assert H.get_sendbufs_raw() is None and H.get_recvbufs_raw() is None
    H.allocate_bufs(P)
    assert H.get_sendbufs_raw() is not None
    H.free_update_halo_buffers()
    assert H.get_sendbufs_raw() is None and H.get_recvbufs_raw() is None
    # allocate single (real and complex)
    for X in (P, Z):
        H.free_update_halo_buffers()
        H.allocate_bufs(X)
        for raw in (H.get_sendbufs_raw(), H.get_recvbufs_raw()):
            assert len(raw) == 1 and len(raw[0]) == 2
            for n in range(2):
                assert raw[0][n].numel() >= _prod_sorted(X)
                assert raw[0][n].numel() % 32 == 0
    # keep 1st, allocate 2nd
    for first, second in ((P, A), (Z, Y)):
        H.free_update_halo_buffers()
        H.allocate_bufs(first)
        H.allocate_bufs(second, first)
        for raw in (H.get_sendbufs_raw(), H.get_recvbufs_raw()):
            assert len(raw) == 2
            for n in range(2):
                assert raw[0][n].numel() >= _prod_sorted(second)
                assert raw[1][n].numel() >= _prod_sorted(first)
    # reinterpret (no allocation): float32 fields fit into the float64 buffers
    H.free_update_halo_buffers()
    H.allocate_bufs(A, P)
    ptrs = [H.engine().pool_ptrs(i, False) for i in range(2)]
    H.allocate_bufs(B, C)
    assert [H.engine().pool_ptrs(i, False) for i in range(2)] == ptrs  # no reallocation
    for raw in (H.get_sendbufs_raw(), H.get_recvbufs_raw()):
        assert len(raw) == 2
        for n in range(2):
            assert raw[0][n].numel() >= _prod_sorted(B)
            assert raw[1][n].numel() >= _prod_sorted(C)
        assert all(raw[i][n].dtype == torch.float32 for i in range(2) for n in range(2))
    # reinterpret to complex
    H.free_update_halo_buffers()
    H.allocate_bufs(A, P)
    H.allocate_bufs(Y, Z)
    for raw in (H.get_sendbufs_raw(), H.get_recvbufs_raw()):
        assert all(raw[i][n].dtype == torch.complex64 for i in range(2) for n in range(2))
    # sendbuf / recvbuf shapes
    H.free_update_halo_buffers()
    H.allocate_bufs(A, P)
    for i, X in ((1, A), (2, P)):
        for dim in range(1, 4):
            for n in (1, 2):
                hs = tuple(s for d, s in enumerate(X.shape) if d != dim - 1)
                assert tuple(H.sendbuf(n, dim, i, X).shape) == hs
                assert tuple(H.recvbuf(n, dim, i, X).shape) == hs
    igg.finalize_global_grid(finalize_MPI=False)


def test_buffers_grow_only():
    igg.init_global_grid(nx, ny, nz, periodx=1, quiet=True, init_MPI=False)
    H.allocate_bufs(torch.zeros(nx, ny, nz))
    cap = H.engine().pool_capacity(0, False)
    H.allocate_bufs(torch.zeros(nx, 2, 2))  # smaller: keeps capacity
    assert H.engine().pool_capacity(0, False) == cap
    H.allocate_bufs(torch.zeros(nx, 3 * ny, nz))  # larger: grows
    assert H.engine().pool_capacity(0, False) > cap
    igg.finalize_global_grid(finalize_MPI=False)


# --- 3. data transfer components --------------------------------------------------
def test_send_recv_ranges():
    igg.init_global_grid(nx, ny, nz, periodx=1, periody=1, periodz=1, overlapz=3, quiet=True, init_MPI=False)
    P = torch.zeros(nx, ny, nz)
    A = torch.zeros(nx - 1, ny + 2, nz + 1)
    s = P.shape
    R = lambda a, b: range(a, b + 1)  # noqa: E731  (Julia a:b)
    assert H.sendranges(1, 1, P) == [R(2, 2), R(1, s[1]), R(1, s[2])]
    assert H.sendranges(2, 1, P) == [R(s[0] - 1, s[0] - 1), R(1, s[1]), R(1, s[2])]
    assert H.sendranges(1, 2, P) == [R(1, s[0]), R(2, 2), R(1, s[2])]
    assert H.sendranges(2, 2, P) == [R(1, s[0]), R(s[1] - 1, s[1] - 1), R(1, s[2])]
    assert H.sendranges(1, 3, P) == [R(1, s[0]), R(1, s[1]), R(3, 3)]
    assert H.sendranges(2, 3, P) == [R(1, s[0]), R(1, s[1]), R(s[2] - 2, s[2] - 2)]
    assert H.recvranges(1, 1, P) == [R(1, 1), R(1, s[1]), R(1, s[2])]
    assert H.recvranges(2, 1, P) == [R(s[0], s[0]), R(1, s[1]), R(1, s[2])]
    assert H.recvranges(1, 3, P) == [R(1, s[0]), R(1, s[1]), R(1, 1)]
    assert H.recvranges(2, 3, P) == [R(1, s[0]), R(1, s[1]), R(s[2], s[2])]
    a = A.shape
    with pytest.raises(IGGError):
        H.sendranges(1, 1, A)
    with pytest.raises(IGGError):
        H.sendranges(2, 1, A)
    assert H.sendranges(1, 2, A) == [R(1, a[0]), R(4, 4), R(1, a[2])]
    assert H.sendranges(2, 2, A) == [R(1, a[0]), R(a[1] - 3, a[1] - 3), R(1, a[2])]
    assert H.sendranges(1, 3, A) == [R(1, a[0]), R(1, a[1]), R(4, 4)]
    assert H.sendranges(2, 3, A) == [R(1, a[0]), R(1, a[1]), R(a[2] - 3, a[2] - 3)]
    with pytest.raises(IGGError):
        H.recvranges(1, 1, A)
    assert H.recvranges(1, 2, A) == [R(1, a[0]), R(1, 1), R(1, a[2])]
    assert H.recvranges(2, 2, A) == [R(1, a[0]), R(a[1], a[1]), R(1, a[2])]
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_write_read_face(device):
    if device == "cuda" and not torch.cuda.is_available():
        pytest.skip("no GPU")
    igg.init_global_grid(nx, ny, nz, quiet=True, init_MPI=False, select_device=False)
    i = torch.arange(1, nx + 1, dtype=torch.float64).view(-1, 1, 1)
    j = torch.arange(1, ny + 1, dtype=torch.float64).view(1, -1, 1)
    k = torch.arange(1, nz + 1, dtype=torch.float64).view(1, 1, -1)
    P = (k * 1e2 + j * 1e1 + i).to(device)
    P2 = torch.zeros_like(P)
    cases = [(1, [range(2, 3), range(1, ny + 1), range(1, nz + 1)]),
             (2, [range(1, nx + 1), range(3, 4), range(1, nz + 1)]),
             (3, [range(1, nx + 1), range(1, ny + 1), range(4, 5)])]
    for dim, ranges in cases:
        hs = tuple(s for d, s in enumerate(P.shape) if d != dim - 1)
        buf = torch.zeros(hs, dtype=torch.float64, device=device)
        H.write_face(buf, P, ranges, dim)
        sl = tuple(slice(r.start - 1, r.stop - 1) for r in ranges)
        assert torch.equal(buf.reshape(-1).cpu(), P[sl].reshape(-1).cpu())
        H.read_face(buf, P2, ranges, dim)
        assert torch.equal(P2[sl].reshape(-1).cpu(), buf.reshape(-1).cpu())
    igg.finalize_global_grid(finalize_MPI=False)


# --- 4. full halo updates ---------------------------------------------------------
def _full(shape_or_tensor, grid_kw, dtype=torch.float64, complex_factor=None):
    """Run the oracle with both exchange schedules (they must agree bitwise)."""
    igg.init_global_grid(*grid_kw.pop("n"), quiet=True, init_MPI=False, **grid_kw)
    gg = igg.get_global_grid()
    A = torch.zeros(shape_or_tensor, dtype=dtype)
    encode(A, complex_factor=complex_factor)
    ref = expected_after_halo(A, has_halo(A, gg), gg.neighbors.tolist())
    for mode in ("sequential", "onephase"):
        H.set_halo_mode(mode)
        X = zero_boundaries(A.clone())
        assert not torch.equal(X, A)
        igg.update_halo_(X)
        assert torch.equal(X, ref), mode
    igg.finalize_global_grid(finalize_MPI=False)
    return X, A


def test_basic_1d():
    X, A = _full((nx,), dict(n=(nx, 1, 1), periodx=1))
    assert torch.equal(X, A)


def test_basic_2d():
    X, A = _full((nx, ny), dict(n=(nx, ny, 1), periodx=1, periody=1))
    assert torch.equal(X, A)


def test_basic_3d():
    X, A = _full((nx, ny, nz), dict(n=(nx, ny, nz), periodx=1, periody=1, periodz=1))
    assert torch.equal(X, A)


def test_basic_3d_non_default_overlap():
    X, A = _full((nx, ny, nz), dict(n=(nx, ny, nz), periodx=1, periody=1, periodz=1, overlapx=4, overlapz=3))
    assert torch.equal(X, A)


def test_basic_3d_not_periodic():
    X, A = _full((nx, ny, nz), dict(n=(nx, ny, nz)))
    assert torch.equal(X[1:-1, 1:-1, 1:-1], A[1:-1, 1:-1, 1:-1])
    for d in range(3):
        for idx in (0, -1):
            sl = [slice(None)] * 3
            sl[d] = idx
            assert (X[tuple(sl)] == 0).all()


@pytest.mark.parametrize("shape,n,kw", [
    ((nx + 1,), (nx, 1, 1), dict(periodx=1)),
    ((nx, ny + 1), (nx, ny, 1), dict(periodx=1, periody=1)),
    ((nx, ny, nz + 1), (nx, ny, nz), dict(periodx=1, periody=1, periodz=1)),
    ((nx + 1, ny, nz), (nx, ny, nz), dict(periodx=1, periody=1, periodz=1, overlapx=3, overlapz=3)),
])
def test_staggered_periodic(shape, n, kw):
    X, A = _full(shape, dict(n=n, **kw))
    assert torch.equal(X, A)


def test_staggered_not_periodic():
    _full((nx, ny, nz + 1), dict(n=(nx, ny, nz)))


def test_no_halo_in_one_dim_2d():
    X, A = _full((nx - 1, ny + 2), dict(n=(nx, ny, 1), periodx=1, periody=1))
    assert torch.equal(X[1:-1, :], A[1:-1, :])
    assert (X[[0, -1], :] == 0).all()


def test_no_halo_in_one_dim_3d():
    X, A = _full((nx + 2, ny - 1, nz + 1), dict(n=(nx, ny, nz), periodx=1, periody=1, periodz=1))
    assert torch.equal(X[:, 1:-1, :], A[:, 1:-1, :])
    assert (X[:, [0, -1], :] == 0).all()


@pytest.mark.parametrize("dtype", [torch.complex64, torch.complex128, torch.float16, torch.bfloat16, torch.int16])
def test_other_element_types(dtype):
    cf = (1 + 1j) if dtype.is_complex else None
    X, A = _full((nx, ny, nz + 1), dict(n=(nx, ny, nz), periodx=1, periody=1, periodz=1), dtype=dtype,
                 complex_factor=cf)
    assert torch.equal(X, A)


@pytest.mark.parametrize("mode", ["sequential", "onephase"])
def test_two_fields_simultaneously(mode):
    igg.init_global_grid(nx, ny, nz, periodx=1, periody=1, periodz=1, quiet=True, init_MPI=False)
    H.set_halo_mode(mode)
    Vz = encode(torch.zeros(nx, ny, nz + 1, dtype=torch.float64))
    Vx = encode(torch.zeros(nx + 1, ny, nz, dtype=torch.float64))
    Vz_ref, Vx_ref = Vz.clone(), Vx.clone()
    zero_boundaries(Vz)
    zero_boundaries(Vx)
    igg.update_halo_(Vz, Vx)
    assert torch.equal(Vz, Vz_ref) and torch.equal(Vx, Vx_ref)
    igg.finalize_global_grid(finalize_MPI=False)


def test_onephase_message_counts():
    igg.init_global_grid(nx, ny, nz, periodx=1, periody=1, periodz=1, quiet=True, init_MPI=False)
    H.set_halo_mode("onephase")
    igg.update_halo_(torch.zeros(nx, ny, nz))
    assert H.engine().last_message_count == 26  # 6 faces + 12 edges + 8 corners (all to self)
    igg.update_halo_(torch.zeros(nx - 1, ny, nz))  # no halo in x: 4 faces + 4 edges
    assert H.engine().last_message_count == 8
    H.set_halo_mode("auto")
    assert H.halo_mode() == "auto"
    igg.finalize_global_grid(finalize_MPI=False)


def test_changing_datatype_between_calls():
    """The reference leaves this commented out (test_update_halo.jl:953-1028);
    byte-typed grow-only buffers make it work here."""
    igg.init_global_grid(nx, ny, nz, periodx=1, periody=1, periodz=1, quiet=True, init_MPI=False)
    for dtype in (torch.float64, torch.float32, torch.complex128, torch.float64):
        V = encode(torch.zeros(nx + 1, ny, nz, dtype=dtype))
        ref = V.clone()
        zero_boundaries(V)
        igg.update_halo_(V)
        assert torch.equal(V, ref)
    igg.finalize_global_grid(finalize_MPI=False)


def test_fortran_order_layout():
    igg.init_global_grid(nx, ny, nz, periodx=1, periody=1, periodz=1, quiet=True, init_MPI=False)
    A = torch.zeros(nz, ny, nx, dtype=torch.float64).permute(2, 1, 0)
    encode(A)
    ref = A.clone()
    zero_boundaries(A)
    igg.update_halo_(A)
    assert torch.equal(A, ref)
    igg.finalize_global_grid(finalize_MPI=False)


def test_plan_summary_reports_zero_copy():
    igg.init_global_grid(8, 6, 4, periodx=1, quiet=True, init_MPI=False)
    s = H.halo_plan_summary(torch.zeros(8, 6, 4))
    assert s[0]["faces"] and all(f["zero_copy"] for f in s[0]["faces"])  # x-faces of C-order arrays
    assert s[1]["faces"] == [] and s[2]["faces"] == []
    igg.finalize_global_grid(finalize_MPI=False)


def test_debug_sync_mode_runs(monkeypatch):
    """IGG_DEBUG_SYNC=1: the engine drains/checks after every phase (host path
    here: a no-op on CPU fields, but the flag is parsed and the update exact)."""
    monkeypatch.setenv("IGG_DEBUG_SYNC", "1")
    igg.init_global_grid(5, 4, 3, periodx=1, periody=1, periodz=1, quiet=True, init_MPI=False)
    from tests.helpers import encode, zero_boundaries

    A = encode(torch.zeros(5, 4, 3, dtype=torch.float64))
    ref = A.clone()
    X = zero_boundaries(A.clone())
    igg.update_halo_(X)
    assert torch.equal(X, ref)
    igg.finalize_global_grid(finalize_MPI=False)
