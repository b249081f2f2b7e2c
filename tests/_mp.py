"""Multi-process launcher for tests: N local ranks over torch.distributed
(gloo, rendezvous at 127.0.0.1), each running ``tests/mp_worker.py``.

Mirrors how the reference's suite is meant to be run under ``mpiexec -n N``
(test/test_update_halo.jl:1-3) — here without MPI.
"""
import os
import socket
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


# Every multi-rank test ends within this many seconds: below the GPU box's
# 180 s no-output limit, so a hang fails its test (with every rank's output)
# instead of getting the whole run killed silently.
MAX_TIMEOUT = 170.0


class TierBudget:
    """Wall budget of a tier of multi-rank launches (tests/test_multigpu.py):
    each launch gets ``min(MAX_TIMEOUT, what is left)`` and none starts with
    less than ``min_launch`` seconds left (it is skipped instead), so the
    tier's worst case - every launch hitting its bound - is ``seconds`` plus
    the teardown of the last launch, whatever the number of launches. The
    clock starts at the first launch (collection and the single-GPU tests
    before the tier do not count)."""

    def __init__(self, seconds: float, min_launch: float = 30.0, clock=time.monotonic):
        self.seconds, self.min_launch, self.clock = float(seconds), float(min_launch), clock
        self.t0 = None

    def next_timeout(self) -> float | None:
        """The bound of the next launch, or None when the budget is spent."""
        if self.t0 is None:
            self.t0 = self.clock()
        left = self.seconds - (self.clock() - self.t0)
        if left < self.min_launch:
            return None
        return min(MAX_TIMEOUT, left)


def run_ranks(nprocs: int, scenario: str, *args, timeout: float = 150.0, env_extra=None) -> list[str]:
    """Run ``scenario`` on ``nprocs`` ranks. Fail-fast: the first rank that
    exits non-zero stops the others (a dead rank would otherwise leave its
    peers blocked in a collective until the timeout); on a timeout every
    rank's output tail is reported. A rendezvous whose port was taken between
    free_port() and rank 0's listen (EADDRINUSE: nothing ran yet) is retried
    on a new port, twice at most."""
    for attempt in range(3):
        try:
            return _run_ranks_once(nprocs, scenario, *args, timeout=timeout, env_extra=env_extra)
        except _PortTaken:
            if attempt == 2:
                raise AssertionError(f"scenario {scenario}: rendezvous port taken three times (EADDRINUSE)")
    raise AssertionError("unreachable")


class _PortTaken(Exception):
    pass


def _run_ranks_once(nprocs: int, scenario: str, *args, timeout: float, env_extra) -> list[str]:
    timeout = min(timeout, MAX_TIMEOUT)
    port = free_port()
    procs, logs = [], []
    for r in range(nprocs):
        env = dict(os.environ)
        env.update({
            "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(r), "WORLD_SIZE": str(nprocs),
            "LOCAL_RANK": str(r), "LOCAL_WORLD_SIZE": str(nprocs), "OMP_NUM_THREADS": "1",
            "IGG_HOST_THREADS": "2", "PYTHONPATH": ROOT + os.pathsep + env.get("PYTHONPATH", ""),
        })
        if env_extra:
            env.update(env_extra)
        log = tempfile.TemporaryFile(mode="w+")
        logs.append(log)
        procs.append(subprocess.Popen(
            [sys.executable, os.path.join(ROOT, "tests", "mp_worker.py"), scenario, *map(str, args)],
            env=env, stdout=log, stderr=subprocess.STDOUT, text=True, cwd=ROOT))
    deadline = time.monotonic() + timeout
    first_bad = None
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [r for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                first_bad = bad[0]
                break
            if all(c == 0 for c in codes) or time.monotonic() > deadline:
                break
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        for p in procs:
            p.wait()
    outs = []
    for log in logs:
        log.seek(0)
        outs.append(log.read())
        log.close()
    codes = [p.returncode for p in procs]
    if first_bad is not None:
        if "EADDRINUSE" in outs[first_bad] and "init_process_group" in outs[first_bad]:
            raise _PortTaken()
        raise AssertionError(f"scenario {scenario}: rank {first_bad} failed (rc={codes[first_bad]}), "
                             f"the others were stopped:\n{outs[first_bad][-4000:]}")
    if any(c != 0 for c in codes):
        msg = "\n".join(f"--- rank {r} rc={c}\n{o[-1500:]}" for r, (c, o) in enumerate(zip(codes, outs)))
        raise AssertionError(f"scenario {scenario} timed out after {timeout:.0f} s:\n{msg}")
    return outs
