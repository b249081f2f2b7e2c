"""Local multi-process launcher, the role ``mpiexec -n N julia app.jl`` plays for
the reference (README.md of ImplicitGlobalGrid.jl; test/test_update_halo.jl:1-3):

    python -m igg.utils.launch -n 8 app.py [args...]

starts N ranks of ``app.py`` with the torch.distributed environment
(``RANK``, ``WORLD_SIZE``, ``LOCAL_RANK``, ``LOCAL_WORLD_SIZE``,
``MASTER_ADDR=127.0.0.1``, ``MASTER_PORT``) that ``init_global_grid`` reads, tags
every output line with its rank, and when a rank fails stops the others and
exits with that rank's code. Single node only (one process per MI355X);
``torchrun`` works as well. The launcher itself never touches the GPU.
"""
from __future__ import annotations

import argparse
import os
import socket
import subprocess
import sys
import threading
import time


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _pump(stream, rank: int, out, lock: threading.Lock) -> None:
    for line in iter(stream.readline, ""):
        with lock:
            out.write(f"[{rank}] {line}")
            out.flush()
    stream.close()


def launch(nprocs: int, cmd: list[str], *, port: int | None = None, env: dict | None = None, tag: bool = True,
           grace: float = 10.0, out=None) -> int:
    """Run ``cmd`` as ``nprocs`` ranks; return 0 or the first failing rank's exit code."""
    if nprocs < 1:
        raise ValueError("launch: nprocs must be >= 1")
    out = sys.stdout if out is None else out
    port = port or _free_port()
    lock = threading.Lock()
    procs, pumps = [], []
    for r in range(nprocs):
        e = dict(os.environ if env is None else env)
        e.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), WORLD_SIZE=str(nprocs),
                 LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(nprocs))
        if tag:
            p = subprocess.Popen(cmd, env=e, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, bufsize=1)
            t = threading.Thread(target=_pump, args=(p.stdout, r, out, lock), daemon=True)
            t.start()
            pumps.append(t)
        else:
            p = subprocess.Popen(cmd, env=e)
        procs.append(p)
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            time.sleep(0.05)
    except KeyboardInterrupt:
        rc = 130
    if rc != 0:  # stop the ranks this launcher started (exact processes, never by pattern)
        for p in procs:
            if p.poll() is None:
                p.terminate()
        t0 = time.time()
        for p in procs:
            try:
                p.wait(timeout=max(0.1, grace - (time.time() - t0)))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    for t in pumps:
        t.join(timeout=5)
    return rc


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(prog="python -m igg.utils.launch", description=__doc__.split("\n\n")[0])
    ap.add_argument("-n", "--nproc", type=int, required=True, help="number of ranks")
    ap.add_argument("--port", type=int, default=None, help="rendezvous port (default: a free one)")
    ap.add_argument("--no-tag", action="store_true", help="do not prefix output lines with the rank")
    ap.add_argument("program", help="a .py script (run with this interpreter) or an executable")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    cmd = ([sys.executable] if a.program.endswith(".py") else []) + [a.program] + a.args
    return launch(a.nproc, cmd, port=a.port, tag=not a.no_tag)


if __name__ == "__main__":
    sys.exit(main())
