"""pytest configuration: the ``gpu`` marker and the shared distributed runtime.

Like the reference suite (test/runtests.jl), most tests run with one process;
multi-rank tests spawn their own ``gloo`` worker processes
(tests/_mp.py). The distributed runtime (the MPI.Init equivalent) is
initialised once per session; tests call init_global_grid(..., init_MPI=False)
and finalize_global_grid(finalize_MPI=False).
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs an MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running test")
    config.addinivalue_line("markers", "multigpu: needs several MI355X, one rank per device (tests/test_multigpu.py)")


def _have_gpu() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    # ``slow``: redundant or long cases outside the driver's GPU tier budget
    # (<= 300 s on one GPU); IGG_TEST_SLOW=1 runs them.
    if os.environ.get("IGG_TEST_SLOW", "0") != "1":
        slow = pytest.mark.skip(reason="slow: IGG_TEST_SLOW=1 runs it")
        for it in items:
            if "slow" in it.keywords:
                it.add_marker(slow)
    if _have_gpu():
        return
    skip = pytest.mark.skip(reason="no GPU available")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session", autouse=True)
def runtime():
    import igg
    from igg.parallel import comm

    if not comm.runtime_initialized():
        comm.init_runtime()
    yield
    from igg.parallel import grid

    if grid.grid_is_initialized():
        igg.finalize_global_grid(finalize_MPI=False)


@pytest.fixture
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", torch.cuda.current_device())


@pytest.fixture(autouse=True)
def _clean_grid():
    """Never leak an initialised grid from a failing test into the next one."""
    yield
    from igg.parallel import grid
    import igg

    if grid.grid_is_initialized():
        igg.finalize_global_grid(finalize_MPI=False)
