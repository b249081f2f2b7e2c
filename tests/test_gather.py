"""Port of test/test_gather.jl (single process; multi-rank cases live in
test_multiprocess.py)."""
import pytest
import torch

import igg
from igg import IGGError

nx, ny, nz = 7, 5, 6


def test_size_errors():
    igg.init_global_grid(nx, ny, nz, quiet=True, init_MPI=False)
    P = torch.zeros(nx, ny, nz)
    with pytest.raises(IGGError, match="can't be `nothing` on the root"):
        igg.gather_(P, None)
    with pytest.raises(IGGError, match="must be of length nprocs"):
        igg.gather_(P, torch.zeros(nx, ny, nz + 1))
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.parametrize("shape", [(nx,), (nx, ny), (nx, ny, nz)])
def test_gather_1d_2d_3d(shape):
    n = list(shape) + [1] * (3 - len(shape))
    igg.init_global_grid(*n, quiet=True, init_MPI=False)
    P = torch.arange(torch.tensor(shape).prod().item(), dtype=torch.float64).view(shape) * 1.5
    G = torch.zeros(shape, dtype=torch.float64)
    igg.gather_(P, G)
    assert torch.equal(G, P)
    igg.finalize_global_grid(finalize_MPI=False)


def test_gather_mixed_dims_and_growing_buffer():
    igg.init_global_grid(nx, ny, nz, quiet=True, init_MPI=False)
    A = torch.arange(nx, dtype=torch.float64)
    G = torch.zeros(nx, 1, 1, dtype=torch.float64)
    igg.gather_(A, G)   # 1-D A into a 3-D A_global
    assert torch.equal(G.view(-1), A)
    B = torch.rand(nx, ny, nz, dtype=torch.float64)
    GB = torch.zeros(nx, ny, nz, dtype=torch.float64)
    igg.gather_(B, GB)  # larger: internal buffer grows
    assert torch.equal(GB, B)
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.int16, torch.complex64])
def test_gather_dtypes(dtype):
    igg.init_global_grid(nx, ny, nz, quiet=True, init_MPI=False)
    P = (torch.arange(nx * ny * nz) % 100).view(nx, ny, nz).to(dtype)
    G = torch.zeros(nx, ny, nz, dtype=dtype)
    igg.gather_(P, G)
    assert torch.equal(G, P)
    igg.finalize_global_grid(finalize_MPI=False)


def test_dtype_mismatch_error():
    igg.init_global_grid(nx, ny, nz, quiet=True, init_MPI=False)
    with pytest.raises(IGGError):
        igg.gather_(torch.zeros(nx, ny, nz), torch.zeros(nx, ny, nz, dtype=torch.float64))
    igg.finalize_global_grid(finalize_MPI=False)


def test_gather_async_single_process_completes():
    """One process (or host tensors): gather_async_ completes synchronously."""
    igg.init_global_grid(4, 3, 2, quiet=True, init_MPI=False)
    A = torch.arange(24, dtype=torch.float64).view(4, 3, 2)
    G = torch.zeros(4, 3, 2, dtype=torch.float64)
    h = igg.gather_async_(A, G)
    assert h.done
    h.wait()
    assert torch.equal(G, A)
    igg.finalize_global_grid(finalize_MPI=False)
