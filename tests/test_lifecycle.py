"""Lifecycle semantics that need a fresh process (test/test_init_global_grid.jl:
"pre-MPI_Init-exception", "initialization including MPI"; and
test/test_finalize_global_grid.jl). Each case runs in its own interpreter, like
the reference driver runs each test file in a fresh Julia process
(test/runtests.jl:8-31)."""
import os
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(code: str):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["PYTHONPATH"] = ROOT
    r = subprocess.run([sys.executable, "-c", textwrap.dedent(code)], env=env, capture_output=True, text=True,
                       timeout=180, cwd=ROOT)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_pre_init_error_and_full_lifecycle():
    out = _run("""
        import igg
        from igg.parallel import grid as G, comm as C
        # 1. pre-init: init_MPI=False while the runtime is not initialised
        try:
            igg.init_global_grid(4, 4, 1, quiet=True, init_MPI=False); raise SystemExit("no error")
        except igg.IGGError as e:
            assert "has not been initialized" in str(e)
        assert not G.grid_is_initialized()
        # 2. initialization including the runtime
        me, dims, nprocs, coords, comm = igg.init_global_grid(4, 4, 1, dimx=1, dimy=1, dimz=1, quiet=True)
        assert G.grid_is_initialized() and C.runtime_initialized()
        assert (me, list(dims), nprocs, list(coords)) == (0, [1, 1, 1], 1, [0, 0, 0])
        igg.finalize_global_grid()
        assert not G.grid_is_initialized() and not C.runtime_initialized()
        # finalize before init / twice
        try:
            igg.finalize_global_grid(); raise SystemExit("no error")
        except igg.IGGError as e:
            assert "before init_global_grid()" in str(e)
        print("LIFECYCLE OK")
    """)
    assert "LIFECYCLE OK" in out


def test_finalize_resets_and_blocks_api():
    out = _run("""
        import torch, igg
        from igg.parallel import grid as G
        igg.init_global_grid(6, 5, 4, quiet=True)
        A = torch.zeros(6, 5, 4)
        igg.finalize_global_grid()
        assert G.get_global_grid().nprocs == -1
        for f in (lambda: igg.update_halo_(A), lambda: igg.nx_g(), lambda: igg.x_g(1, 1.0, A),
                  lambda: igg.tic(), lambda: igg.gather_(A, A)):
            try:
                f(); raise SystemExit("no error")
            except igg.IGGError as e:
                assert "No function of the module can be called" in str(e)
        # re-init after finalize works (fresh runtime)
        igg.init_global_grid(6, 5, 4, quiet=True)
        igg.finalize_global_grid()
        print("FINALIZE OK")
    """)
    assert "FINALIZE OK" in out


def test_finalize_without_runtime_finalization():
    out = _run("""
        import igg
        from igg.parallel import comm as C
        igg.init_global_grid(6, 5, 4, quiet=True)
        igg.finalize_global_grid(finalize_MPI=False)
        assert C.runtime_initialized()
        igg.init_global_grid(6, 5, 4, quiet=True, init_MPI=False)
        igg.finalize_global_grid()
        assert not C.runtime_initialized()
        print("NOFIN OK")
    """)
    assert "NOFIN OK" in out


def test_ipc_paths_need_one_node():
    """Ranks on several nodes: the put transport refuses with a clear error on
    every rank before entering any collective (IPC handles cannot be opened
    on another node); RCCL / staged stay available."""
    import pytest

    from igg.parallel.comm import Communicator
    from igg._native import IGGError

    one = Communicator(rank=0, size=2, local_size=2)
    two = Communicator(rank=0, size=2, local_size=1)
    assert one.one_node and not two.one_node
    with pytest.raises(IGGError, match="one node"):
        two.device_transport("put")
