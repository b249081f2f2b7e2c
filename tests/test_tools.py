"""Port of test/test_tools.jl (exact vectors) and the x_g doctests
(src/tools.jl:66-96), plus tic/toc."""
import os

import numpy as np
import pytest
import torch

import igg
from igg.parallel import grid as G


def _vec(f, d, A, n):
    return [f(i, d, A) for i in range(1, n + 1)]


def test_doctest_x_g():
    lx, nx = 4, 3
    igg.init_global_grid(nx, nx, nx, quiet=True, init_MPI=False)
    dx = lx / (igg.nx_g() - 1)
    assert dx == 2.0
    A = torch.zeros(nx, nx, nx)
    Vx = torch.zeros(nx + 1, nx, nx)
    Vy = torch.zeros(nx, nx + 1, nx)
    Vz = torch.zeros(nx, nx, nx + 1)
    assert _vec(igg.x_g, dx, A, 3) == [0.0, 2.0, 4.0]
    assert _vec(igg.x_g, dx, Vx, 4) == [-1.0, 1.0, 3.0, 5.0]
    assert _vec(igg.y_g, dx, Vy, 4) == [-1.0, 1.0, 3.0, 5.0]
    assert _vec(igg.z_g, dx, Vz, 4) == [-1.0, 1.0, 3.0, 5.0]
    igg.finalize_global_grid(finalize_MPI=False)


def test_g_functions():
    lx = ly = lz = 8
    nx = ny = nz = 5
    P = torch.zeros(nx, ny, nz)
    Vx = torch.zeros(nx + 1, ny, nz)
    Vz = torch.zeros(nx, ny, nz + 1)
    A = torch.zeros(nx, ny, nz + 2)
    Sxz = torch.zeros(nx - 2, ny - 1, nz - 2)
    igg.init_global_grid(nx, ny, nz, dimx=1, dimy=1, dimz=1, periodz=1, quiet=True, init_MPI=False)
    assert igg.nx_g() == nx and igg.ny_g() == ny and igg.nz_g() == nz - 2
    dx, dy, dz = lx / (igg.nx_g() - 1), ly / (igg.ny_g() - 1), lz / (igg.nz_g() - 1)
    assert _vec(igg.x_g, dx, P, 5) == [0.0, 2.0, 4.0, 6.0, 8.0]
    assert _vec(igg.y_g, dy, P, 5) == [0.0, 2.0, 4.0, 6.0, 8.0]
    assert _vec(igg.z_g, dz, P, 5) == [8.0, 0.0, 4.0, 8.0, 0.0]
    assert _vec(igg.x_g, dx, Vx, 6) == [-1.0, 1.0, 3.0, 5.0, 7.0, 9.0]
    assert _vec(igg.y_g, dy, Vx, 5) == [0.0, 2.0, 4.0, 6.0, 8.0]
    assert _vec(igg.z_g, dz, Vx, 5) == [8.0, 0.0, 4.0, 8.0, 0.0]
    assert _vec(igg.x_g, dx, Vz, 5) == [0.0, 2.0, 4.0, 6.0, 8.0]
    assert _vec(igg.y_g, dy, Vz, 5) == [0.0, 2.0, 4.0, 6.0, 8.0]
    assert _vec(igg.z_g, dz, Vz, 6) == [6.0, 10.0, 2.0, 6.0, 10.0, 2.0]
    assert _vec(igg.x_g, dx, A, 5) == [0.0, 2.0, 4.0, 6.0, 8.0]
    assert _vec(igg.y_g, dy, A, 5) == [0.0, 2.0, 4.0, 6.0, 8.0]
    assert _vec(igg.z_g, dz, A, 7) == [4.0, 8.0, 0.0, 4.0, 8.0, 0.0, 4.0]
    assert _vec(igg.x_g, dx, Sxz, 3) == [2.0, 4.0, 6.0]
    assert _vec(igg.y_g, dy, Sxz, 4) == [1.0, 3.0, 5.0, 7.0]
    assert _vec(igg.z_g, dz, Sxz, 3) == [0.0, 4.0, 8.0]
    # array-size-aware global sizes
    assert igg.nx_g(Vx) == nx + 1 and igg.nz_g(Vz) == nz - 2 + 1 and igg.ny_g(Sxz) == ny - 1
    igg.finalize_global_grid(finalize_MPI=False)


def test_g_functions_non_default_overlap():
    lx = ly = lz = 8
    nx, ny, nz = 5, 5, 8
    P = torch.zeros(nx, ny, nz)
    Vz = torch.zeros(nx, ny, nz + 1)
    A = torch.zeros(nx, ny, nz + 2)
    Sxz = torch.zeros(nx - 2, ny - 1, nz - 2)
    igg.init_global_grid(nx, ny, nz, dimx=1, dimy=1, dimz=1, periodz=1, overlapx=3, overlapz=3, quiet=True,
                         init_MPI=False)
    assert igg.nx_g() == nx and igg.ny_g() == ny and igg.nz_g() == nz - 3
    dx, dy, dz = lx / (igg.nx_g() - 1), ly / (igg.ny_g() - 1), lz / (igg.nz_g() - 1)
    assert _vec(igg.x_g, dx, P, 5) == [0.0, 2.0, 4.0, 6.0, 8.0]
    assert _vec(igg.z_g, dz, P, 8) == [8.0, 0.0, 2.0, 4.0, 6.0, 8.0, 0.0, 2.0]
    assert _vec(igg.z_g, dz, Vz, 9) == [7.0, 9.0, 1.0, 3.0, 5.0, 7.0, 9.0, 1.0, 3.0]
    assert _vec(igg.z_g, dz, A, 10) == [6.0, 8.0, 0.0, 2.0, 4.0, 6.0, 8.0, 0.0, 2.0, 4.0]
    assert _vec(igg.x_g, dx, Sxz, 3) == [2.0, 4.0, 6.0]
    assert _vec(igg.y_g, dy, Sxz, 4) == [1.0, 3.0, 5.0, 7.0]
    assert _vec(igg.z_g, dz, Sxz, 6) == [0.0, 2.0, 4.0, 6.0, 8.0, 0.0]
    igg.finalize_global_grid(finalize_MPI=False)


def test_g_functions_simulated_3x3x3():
    lx, ly, lz = 20, 20, 16
    nx = ny = nz = 5
    P = torch.zeros(nx, ny, nz)
    A = torch.zeros(nx + 1, ny - 2, nz + 2)
    igg.init_global_grid(nx, ny, nz, dimx=1, dimy=1, dimz=1, periodz=1, quiet=True, init_MPI=False)
    gg = G.global_grid()
    dims = np.array([3, 3, 3])
    nxyz_g = dims * (gg.nxyz - gg.overlaps) + gg.overlaps * (gg.periods == 0)
    gg.dims[:] = dims
    gg.nxyz_g[:] = nxyz_g
    assert [igg.nx_g(), igg.ny_g(), igg.nz_g()] == list(nxyz_g)
    dx, dy, dz = lx / (igg.nx_g() - 1), ly / (igg.ny_g() - 1), lz / (igg.nz_g() - 1)
    c = gg.coords
    exp_P = {
        0: [[0.0, 2.0, 4.0, 6.0, 8.0], [6.0, 8.0, 10.0, 12.0, 14.0], [12.0, 14.0, 16.0, 18.0, 20.0]],
        1: [[0.0, 2.0, 4.0, 6.0, 8.0], [6.0, 8.0, 10.0, 12.0, 14.0], [12.0, 14.0, 16.0, 18.0, 20.0]],
        2: [[16.0, 0.0, 2.0, 4.0, 6.0], [4.0, 6.0, 8.0, 10.0, 12.0], [10.0, 12.0, 14.0, 16.0, 0.0]],
    }
    exp_A = {
        0: [[-1.0, 1.0, 3.0, 5.0, 7.0, 9.0], [5.0, 7.0, 9.0, 11.0, 13.0, 15.0], [11.0, 13.0, 15.0, 17.0, 19.0, 21.0]],
        1: [[2.0, 4.0, 6.0], [8.0, 10.0, 12.0], [14.0, 16.0, 18.0]],
        2: [[14.0, 16.0, 0.0, 2.0, 4.0, 6.0, 8.0], [2.0, 4.0, 6.0, 8.0, 10.0, 12.0, 14.0],
            [8.0, 10.0, 12.0, 14.0, 16.0, 0.0, 2.0]],
    }
    fns = (igg.x_g, igg.y_g, igg.z_g)
    ds = (dx, dy, dz)
    for d in range(3):
        for k in range(3):
            c[d] = k
            assert _vec(fns[d], ds[d], P, P.shape[d]) == exp_P[d][k]
            assert _vec(fns[d], ds[d], A, A.shape[d]) == exp_A[d][k]
    igg.finalize_global_grid(finalize_MPI=False)


def test_coords_g_vectorised_matches_scalar():
    igg.init_global_grid(7, 6, 5, periodx=1, quiet=True, init_MPI=False)
    A = torch.zeros(8, 6, 4)
    for d, f in enumerate((igg.x_g, igg.y_g, igg.z_g)):
        v = igg.coords_g(d, 0.3, A).tolist()
        assert v == [f(i + 1, 0.3, A) for i in range(A.shape[d])]
    igg.finalize_global_grid(finalize_MPI=False)


def test_tic_toc():
    igg.init_global_grid(4, 4, 4, quiet=True, init_MPI=False)
    t0 = igg.tic()
    assert isinstance(t0, float)
    t = igg.toc()
    assert isinstance(t, float) and 0 <= t < 5
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.parametrize("per", [0, 1])
def test_coords_g_vectorised_matches_x_g_bitwise(per):
    from igg.utils.tools import coords_g, x_g, y_g, z_g

    igg.init_global_grid(13, 9, 7, periodx=per, periody=per, periodz=per, quiet=True, init_MPI=False)
    for shape in [(13, 9, 7), (14, 9, 7), (12, 10, 8)]:
        A = torch.empty(shape, device="meta")
        for dim, f in ((0, x_g), (1, y_g), (2, z_g)):
            v = coords_g(dim, 0.37, A, device="cpu")
            ref = torch.tensor([f(i + 1, 0.37, A) for i in range(shape[dim])], dtype=torch.float64)
            assert torch.equal(v, ref)
    igg.finalize_global_grid(finalize_MPI=False)


def test_api_docs_up_to_date():
    """docs/api.md is generated from the docstrings (tools/gen_api_docs.py)."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "gen_api_docs.py"), "--check"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
