"""Multi-process launcher for tests: N local ranks over torch.distributed
(gloo, rendezvous at 127.0.0.1), each running ``tests/mp_worker.py``.

Mirrors how the reference's suite is meant to be run under ``mpiexec -n N``
(test/test_update_halo.jl:1-3) — here without MPI.
"""
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_ranks(nprocs: int, scenario: str, *args, timeout: float = 240.0, env_extra=None) -> list[str]:
    port = free_port()
    procs = []
    for r in range(nprocs):
        env = dict(os.environ)
        env.update({
            "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(r), "WORLD_SIZE": str(nprocs),
            "LOCAL_RANK": str(r), "LOCAL_WORLD_SIZE": str(nprocs), "OMP_NUM_THREADS": "1",
            "IGG_HOST_THREADS": "2", "PYTHONPATH": ROOT + os.pathsep + env.get("PYTHONPATH", ""),
        })
        if env_extra:
            env.update(env_extra)
        procs.append(subprocess.Popen(
            [sys.executable, os.path.join(ROOT, "tests", "mp_worker.py"), scenario, *map(str, args)],
            env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, cwd=ROOT))
    outs, failed = [], []
    for r, p in enumerate(procs):
        try:
            out, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise AssertionError(f"rank {r} timed out in scenario {scenario}")
        outs.append(out)
        if p.returncode != 0:
            failed.append((r, p.returncode, out[-4000:]))
    if failed:
        msg = "\n".join(f"--- rank {r} rc={rc}\n{o}" for r, rc, o in failed)
        raise AssertionError(f"scenario {scenario} failed:\n{msg}")
    return outs
