"""Transport selection (parallel/transport_select.py): the probe payload and
the IGG_TRANSPORT=auto configuration (CPU; the GPU selection itself runs in
tests/test_multiprocess.py::test_auto_transport_shared_gpu and the multigpu tier)."""
import pytest
import torch

from igg.parallel import transport_select as ts
from igg.utils import config


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16, torch.float32, torch.float64, torch.uint8,
                                   torch.int8, torch.int16, torch.int32, torch.complex64, torch.complex128])
def test_probe_exact_and_rank_distinct(dtype):
    """Every probe value is an exact integer of the dtype, ranks' values are
    disjoint and distinct within a rank's span, and the poison (0) is no
    rank's value (float16/bfloat16 rounded neighbouring positions
    together, unsigned dtypes overflowed on the old -7 poison)."""
    shape, nranks = (9, 7, 40), 8
    A = torch.empty(shape, dtype=dtype)
    seen = set()
    for r in range(nranks):
        X = ts._probe(A, r, nranks)
        assert X.dtype == dtype and X.shape == A.shape
        inner = X[1:-1, 1:-1, 1:-1]
        vals = (inner.real if dtype.is_complex else inner).to(torch.float64)
        assert torch.equal(vals, vals.round())  # integers
        ints = vals.to(torch.int64).flatten()
        u = set(ints.tolist())
        assert 0 not in u
        assert not (u & seen), f"rank {r} shares probe values with a lower rank"
        seen |= u
        # the boundary planes carry the poison
        for d in range(3):
            for i in (0, shape[d] - 1):
                p = X.select(d, i)
                assert torch.equal(p, torch.zeros_like(p))
        # along the fastest dim neighbouring interior positions differ
        assert bool((inner[..., 1:] != inner[..., :-1]).any())


def test_exact_limits():
    assert ts._exact_limit(torch.float16) == 2048
    assert ts._exact_limit(torch.bfloat16) == 256
    assert ts._exact_limit(torch.float32) == 1 << 24
    assert ts._exact_limit(torch.uint8) == 256
    assert ts._exact_limit(torch.int16) == 32768
    assert ts._exact_limit(torch.complex64) == 1 << 24


def test_transport_default_is_auto():
    assert config.transport_choice({}) == "auto"
    for t in ("auto", "put", "rccl", "staged", "torch"):
        assert config.transport_choice({"IGG_TRANSPORT": t}) == t
    with pytest.raises(ValueError):
        config.transport_choice({"IGG_TRANSPORT": "mpi"})


def test_auto_is_off_on_single_process_and_cpu_grids():
    import igg
    from igg.parallel import halo as H

    igg.init_global_grid(8, 6, 5, periodx=1, quiet=True, init_MPI=False, device_type="none")
    try:
        assert not H.auto_transport()
        A = torch.arange(8 * 6 * 5, dtype=torch.float64).view(8, 6, 5)
        igg.update_halo_(A)
        assert H.tuned_transports() == []
    finally:
        igg.finalize_global_grid(finalize_MPI=False)
