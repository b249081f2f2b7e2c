"""Native Cartesian topology (the MPI_Dims_create / Cart_* replacement) and the
environment-flag precedence rules of src/init_global_grid.jl:51-68."""
import itertools

import pytest

import igg
from igg import IGGError
from igg._native import native
from igg.utils import config

P = igg.PROC_NULL


@pytest.mark.parametrize("n,dims,exp", [
    (8, [0, 0, 0], [2, 2, 2]), (4, [0, 0, 1], [2, 2, 1]), (6, [0, 0, 0], [3, 2, 1]), (2, [0, 0, 0], [2, 1, 1]),
    (1, [0, 0, 0], [1, 1, 1]), (12, [0, 0, 0], [3, 2, 2]), (16, [0, 0, 0], [4, 2, 2]), (8, [0, 2, 0], [2, 2, 2]),
    (8, [0, 1, 1], [8, 1, 1]), (7, [0, 0, 0], [7, 1, 1]), (64, [0, 0, 0], [4, 4, 4]), (24, [0, 0, 2], [4, 3, 2]),
    (4, [1, 0, 1], [1, 4, 1]), (5120, [0, 0, 0], [20, 16, 16]),
])
def test_dims_create(n, dims, exp):
    assert native.dims_create(n, dims) == exp


def test_dims_create_errors():
    with pytest.raises(IGGError):
        native.dims_create(8, [3, 0, 0])
    with pytest.raises(IGGError):
        native.dims_create(8, [2, 2, 1])


@pytest.mark.parametrize("dims", [[2, 2, 2], [3, 2, 1], [1, 4, 1], [5, 1, 3]])
def test_cart_coords_roundtrip_row_major(dims):
    ranks = range(dims[0] * dims[1] * dims[2])
    coords = [native.cart_coords(r, dims) for r in ranks]
    assert coords == [list(c) for c in itertools.product(*(range(d) for d in dims))]  # last dim fastest
    assert [native.cart_rank(c, dims) for c in coords] == list(ranks)


def test_cart_shift():
    dims = [2, 3, 1]
    # rank 0 = (0,0,0)
    assert native.cart_shift(0, 0, 1, dims, [0, 0, 0]) == [P, native.cart_rank([1, 0, 0], dims)]
    assert native.cart_shift(0, 0, 1, dims, [1, 0, 0]) == [3, 3]       # dims==2 periodic: same peer
    assert native.cart_shift(0, 1, 1, dims, [0, 1, 0]) == [2, 1]
    assert native.cart_shift(0, 2, 1, dims, [0, 0, 1]) == [0, 0]       # self (periodic, dims==1)
    assert native.cart_shift(0, 2, 1, dims, [0, 0, 0]) == [P, P]
    assert native.cart_shift(4, 1, 2, dims, [0, 1, 0]) == [5, 3]       # (1,1,0): disp 2 wraps both ways


def test_global_size():
    assert native.global_size([512] * 3, [2, 2, 2], [2] * 3, [0] * 3) == [1022] * 3
    assert native.global_size([4, 4, 8], [1, 1, 1], [3, 2, 3], [0, 0, 1]) == [4, 4, 5]


def test_coord_g_matches_python():
    assert native.coord_g(0, 2.0, 4, 3, 2, 0, 3, False) == -1.0
    assert native.coord_g(1, 2.0, 5, 5, 2, 0, 3, True) == 0.0


def test_env_precedence():
    assert config.parse_aware_flags("ROCMAWARE_MPI", {}) == [False] * 3
    assert config.parse_aware_flags("ROCMAWARE_MPI", {"IGG_ROCMAWARE_MPI": "1"}) == [True] * 3
    # per-dim honoured only if the global one left all dims false
    assert config.parse_aware_flags("ROCMAWARE_MPI", {"IGG_ROCMAWARE_MPI": "0", "IGG_ROCMAWARE_MPI_DIMZ": "1"}) == [False, False, True]
    assert config.parse_aware_flags("ROCMAWARE_MPI", {"IGG_ROCMAWARE_MPI": "1", "IGG_ROCMAWARE_MPI_DIMZ": "0"}) == [True] * 3
    # loopvectorization: per-dim only honoured if the global one set all dims true
    assert config.parse_loopvectorization({"IGG_LOOPVECTORIZATION_DIMX": "1"}) == [False] * 3
    assert config.parse_loopvectorization({"IGG_LOOPVECTORIZATION": "1", "IGG_LOOPVECTORIZATION_DIMX": "0"}) == [False, True, True]
    assert config.transport_choice({}) == "auto"
    assert config.transport_choice({"IGG_TRANSPORT": "PUT"}) == "put"
    with pytest.raises(ValueError):
        config.transport_choice({"IGG_TRANSPORT": "mpi"})
