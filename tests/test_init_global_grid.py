"""Port of test/test_init_global_grid.jl (single process; the pre-MPI_Init and
init_MPI semantics run in fresh subprocesses, see test_lifecycle.py)."""
import numpy as np
import pytest

import igg
from igg import IGGError
from igg.parallel import grid as G

p0 = igg.PROC_NULL
nx, ny, nz = 4, 4, 1


def test_initialization_values():
    me, dims, nprocs, coords, comm_cart = igg.init_global_grid(nx, ny, nz, dimx=1, dimy=1, dimz=1, quiet=True,
                                                               init_MPI=False)
    assert G.grid_is_initialized()
    assert me == 0
    assert list(dims) == [1, 1, 1]
    assert nprocs == 1
    assert list(coords) == [0, 0, 0]
    gg = G.global_grid()
    assert list(gg.nxyz_g) == [nx, ny, nz]
    assert list(gg.nxyz) == [nx, ny, nz]
    assert list(gg.dims) == list(dims)
    assert list(gg.overlaps) == [2, 2, 2]
    assert gg.nprocs == nprocs
    assert gg.me == me
    assert list(gg.coords) == list(coords)
    assert gg.neighbors.tolist() == [[p0, p0, p0], [p0, p0, p0]]
    assert list(gg.periods) == [0, 0, 0]
    assert gg.disp == 1
    assert gg.reorder == 1
    assert gg.comm == comm_cart
    assert gg.quiet is True
    igg.finalize_global_grid(finalize_MPI=False)


def test_initialization_preinitialized_runtime():
    igg.init_global_grid(nx, ny, nz, quiet=True, init_MPI=False)
    assert G.grid_is_initialized()
    igg.finalize_global_grid(finalize_MPI=False)


def test_initialization_periodic():
    nz_ = 4
    igg.init_global_grid(nx, ny, nz_, dimx=1, dimy=1, dimz=1, periodx=1, periodz=1, quiet=True, init_MPI=False)
    gg = G.global_grid()
    assert list(gg.nxyz_g) == [nx - 2, ny, nz_ - 2]
    assert list(gg.nxyz) == [nx, ny, nz_]
    assert gg.neighbors.tolist() == [[0, p0, 0], [0, p0, 0]]
    assert list(gg.periods) == [1, 0, 1]
    igg.finalize_global_grid(finalize_MPI=False)


def test_initialization_overlaps_one_periodic():
    nz_, olz, olx = 8, 3, 3
    igg.init_global_grid(nx, ny, nz_, dimx=1, dimy=1, dimz=1, periodz=1, overlapx=olx, overlapz=olz, quiet=True,
                         init_MPI=False)
    gg = G.global_grid()
    assert list(gg.nxyz_g) == [nx, ny, nz_ - olz]  # olx has no effect: 1 process, not periodic
    assert list(gg.nxyz) == [nx, ny, nz_]
    assert gg.neighbors.tolist() == [[p0, p0, 0], [p0, p0, 0]]
    assert list(gg.periods) == [0, 0, 1]
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.parametrize("args,kw", [
    ((1, 4, 4), {}),                          # nx == 1
    ((4, 1, 4), {}),                          # ny == 1 while nz > 1
    ((4, 4, 1), {"dimz": 3}),                 # dimz > 1 while nz == 1
    ((4, 4, 1), {"periodz": 1}),              # periodz while nz == 1
    ((4, 4, 4), {"periody": 1, "overlapy": 3}),  # periodic with ny < 2*overlapy-1
    ((4, 4, 4), {"device_type": "TPU"}),      # invalid device type
])
def test_argument_errors(args, kw):
    with pytest.raises(IGGError):
        igg.init_global_grid(*args, quiet=True, init_MPI=False, **kw)
    assert not G.grid_is_initialized()


def test_runtime_already_initialized_error():
    with pytest.raises(IGGError, match="already initialized"):
        igg.init_global_grid(4, 4, 4, quiet=True)  # init_MPI=True but runtime is up


def test_already_initialized_error():
    igg.init_global_grid(4, 4, 4, quiet=True, init_MPI=False)
    with pytest.raises(IGGError, match="already been initialized"):
        igg.init_global_grid(4, 4, 4, quiet=True, init_MPI=False)
    igg.finalize_global_grid(finalize_MPI=False)


def test_summary_line(capsys):
    igg.init_global_grid(6, 5, 4, periodx=1, init_MPI=False)
    out = capsys.readouterr().out
    assert "Global grid: 4x5x4 (nprocs: 1, dims: 1x1x1)" in out
    igg.finalize_global_grid(finalize_MPI=False)


def test_get_global_grid_is_deep_copy():
    igg.init_global_grid(6, 5, 4, quiet=True, init_MPI=False)
    c = igg.get_global_grid()
    c.dims[:] = 7
    assert list(G.global_grid().dims) == [1, 1, 1]
    assert c.comm is G.global_grid().comm
    igg.finalize_global_grid(finalize_MPI=False)


def test_hip_is_the_only_gpu_backend():
    igg.init_global_grid(6, 5, 4, quiet=True, init_MPI=False, device_type="CUDA")
    gg = G.global_grid()
    assert gg.cuda_enabled is False and gg.amdgpu_enabled is False
    igg.finalize_global_grid(finalize_MPI=False)
    igg.init_global_grid(6, 5, 4, quiet=True, init_MPI=False, device_type="AMDGPU", select_device=False)
    assert G.global_grid().amdgpu_enabled == (igg.native.device_count() > 0)
    igg.finalize_global_grid(finalize_MPI=False)


def test_env_flags_are_recorded(monkeypatch):
    monkeypatch.setenv("IGG_ROCMAWARE_MPI_DIMY", "1")
    monkeypatch.setenv("IGG_LOOPVECTORIZATION", "1")
    monkeypatch.setenv("IGG_LOOPVECTORIZATION_DIMZ", "0")
    igg.init_global_grid(6, 5, 4, quiet=True, init_MPI=False)
    gg = G.global_grid()
    assert gg.amdgpuaware_MPI == [False, True, False]
    assert gg.loopvectorization == [True, True, False]
    assert gg.cudaaware_MPI == [False, False, False]
    igg.finalize_global_grid(finalize_MPI=False)


def test_pack_mode_env_parsing():
    from igg.utils import config

    assert config.pack_modes({}) == ["kernel"] * 3
    assert config.pack_modes({"IGG_PACK": "memcpy2d"}) == ["memcpy2d"] * 3
    assert config.pack_modes({"IGG_PACK": "memcpy2d", "IGG_PACK_DIMX": "kernel"}) == ["kernel", "memcpy2d", "memcpy2d"]
    assert config.pack_modes({"IGG_PACK_DIMZ": "memcpy2d"}) == ["kernel", "kernel", "memcpy2d"]
    with pytest.raises(ValueError):
        config.pack_modes({"IGG_PACK": "dma"})


def test_pack_mode_setter_cpu():
    import torch

    from igg.parallel import halo as H

    igg.init_global_grid(6, 5, 4, quiet=True, init_MPI=False, device_type="none")
    assert [H.pack_mode(d) for d in (1, 2, 3)] == ["kernel"] * 3
    H.set_pack_mode("memcpy2d", dims=(False, True, True))
    assert [H.pack_mode(d) for d in (1, 2, 3)] == ["kernel", "memcpy2d", "memcpy2d"]
    A = torch.zeros(6, 5, 4)
    igg.update_halo_(A)  # host fields ignore the device pack mode
    igg.finalize_global_grid(finalize_MPI=False)
