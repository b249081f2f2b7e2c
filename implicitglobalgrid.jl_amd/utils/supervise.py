"""Fail-soft job supervision: phases, deadlines and relaunch with exclusions.

Reference: a failing rank aborts the whole MPI job (MPI.Init in
src/init_global_grid.jl:80-92; every error of the library is fatal). That is
the right contract for a library call, but a *job* whose first contact with a
second GPU hangs - an RCCL bootstrap that never completes, an IPC mapping
that never returns - should lose the path that hung, not its result. This
module gives a multi-rank program (the benchmark) that property without ever
touching the GPU itself:

* the worker ranks announce what they are doing (:class:`Phases`): a phase
  name, the **exclusion key** of the path the phase exercises (``rccl``,
  ``put``, ``fused``, ``fused-inkernel``, ``graph``, ...) and a deadline;
* a supervisor (one per node-local worker under ``torchrun``, coordinated
  over the launcher's TCP store; or one parent for all ranks in a self
  launch) watches the workers' phase files and exit codes;
* when a worker dies, stalls past its phase deadline, or asks for it
  (:meth:`Phases.relaunch`, exit code :data:`RELAUNCH_EXIT` after a bounded
  call had to be abandoned), every worker of the attempt is stopped and a
  **fresh** set of worker processes is started with that key excluded
  (``IGG_EXCLUDE`` = JSON ``{key: reason}``). Processes are replaced, never
  reused: a process with a thread stuck inside the HIP runtime is not safe to
  continue with.

The decision is a pure function (:func:`decide`) so it is unit-tested on the
CPU; ``tests/test_supervise.py`` and ``tests/test_bench.py`` inject hangs
(``IGG_INJECT_PHASE_HANG=phase@rank``) and check that the run still reports,
with the excluded path listed.
"""
from __future__ import annotations

import json
import os
import signal
import socket
import subprocess
import sys
import tempfile
import time

RELAUNCH_EXIT = 3  # a worker asks for fresh processes without some path
DEFAULT_DEADLINE = 600.0


# ----------------------------------------------------------------- worker side
def excluded(env=None) -> dict:
    """{key: reason} of the paths this process must not use (``IGG_EXCLUDE``)."""
    env = os.environ if env is None else env
    raw = env.get("IGG_EXCLUDE", "").strip()
    if not raw:
        return {}
    try:
        d = json.loads(raw)
        return {str(k): str(v) for k, v in d.items()}
    except ValueError:  # plain "a,b,c"
        return {k.strip(): "excluded by IGG_EXCLUDE" for k in raw.split(",") if k.strip()}


def is_excluded(key: str, env=None) -> bool:
    return key in excluded(env)


class Phases:
    """Worker-side phase announcements (no-op without a supervisor).

    ``enter(name, key, deadline)`` records that this rank now runs phase
    ``name``, which exercises the path ``key`` (None: nothing to exclude) and
    should end within ``deadline`` seconds. The record is a small JSON file
    (``IGG_PHASE_FILE``), replaced atomically."""

    def __init__(self, rank: int | None = None):
        self.path = os.environ.get("IGG_PHASE_FILE")
        self.supervised = self.path is not None
        self.rank = int(os.environ.get("RANK", "0")) if rank is None else rank
        self.attempt = int(os.environ.get("IGG_SUP_ATTEMPT", "0"))
        self.scale = float(os.environ.get("IGG_PHASE_DEADLINE_SCALE", "1"))
        self.cur = None

    def _write(self, rec: dict) -> None:
        if not self.path:
            return
        tmp = f"{self.path}.tmp"
        with open(tmp, "w") as f:
            json.dump(rec, f)
        os.replace(tmp, self.path)

    def enter(self, name: str, key: str | None = None, deadline: float = DEFAULT_DEADLINE) -> None:
        self.cur = {"phase": name, "key": key, "since": time.time(), "deadline": float(deadline) * self.scale,
                    "pid": os.getpid()}
        self._write(self.cur)
        if self.rank == 0 and self.path:  # progress on stderr (and never a silent minute)
            print(f"[phase] {name}" + (f" (path {key})" if key else ""), file=sys.stderr, flush=True)
        self._maybe_hang(name)

    def printed(self) -> None:
        """The result line is out: a later stall (teardown) does not lose it."""
        if self.cur is not None:
            self.cur["printed"] = True
            self._write(self.cur)

    def relaunch(self, keys: dict, code: int = RELAUNCH_EXIT) -> None:
        """Ask the supervisor for fresh processes without ``keys`` ({key:
        reason}) and exit (every rank of the attempt should do the same)."""
        rec = dict(self.cur or {"phase": "?", "since": time.time(), "deadline": DEFAULT_DEADLINE})
        rec["relaunch"] = {str(k): str(v) for k, v in keys.items()}
        self._write(rec)
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(code)

    def _maybe_hang(self, name: str) -> None:
        """Fault injection (tests): ``IGG_INJECT_PHASE_HANG=phase@rank[,...]``
        blocks this rank forever on entering a phase whose name starts with
        ``phase`` - first attempt only, so the relaunch can succeed."""
        spec = os.environ.get("IGG_INJECT_PHASE_HANG", "")
        if not spec or self.attempt != 0:
            return
        for item in spec.split(","):
            ph, _, r = item.partition("@")
            if ph and name.startswith(ph) and r in (str(self.rank), "*"):
                print(f"rank {self.rank}: injected hang in phase {name}", file=sys.stderr, flush=True)
                while True:
                    time.sleep(3600)


# ------------------------------------------------------------- decision logic
def decide(statuses: list, now: float, excl: dict, attempts_left: int) -> dict | None:
    """What to do with an attempt, from every rank's status.

    ``statuses[r]``: {"phase", "key", "since", "deadline", "exit", "exit_t",
    "relaunch", "printed"} (missing entries = not reported yet). Returns None
    (keep waiting) or {"action": "done"} / {"action": "retry", "exclude":
    {key: reason}} / {"action": "fail", "why": str}."""

    def retry_or_fail(keys: dict, why: str) -> dict:
        new = {k: v for k, v in keys.items() if k and k not in excl}
        if new and attempts_left > 0:
            return {"action": "retry", "exclude": new, "why": why}
        if new:
            return {"action": "fail", "why": f"{why}; no relaunch attempts left"}
        return {"action": "fail", "why": f"{why}; nothing left to exclude"}

    if statuses and all(s.get("exit") == 0 for s in statuses):
        return {"action": "done"}
    dead = [(s.get("exit_t", now), r, s) for r, s in enumerate(statuses) if s.get("exit") not in (None, 0)]
    asks = [(t, r, s) for t, r, s in dead if s.get("exit") == RELAUNCH_EXIT and s.get("relaunch")]
    if asks:
        keys = {}
        for _t, r, s in sorted(asks):
            for k, v in s["relaunch"].items():
                keys.setdefault(k, f"rank {r}: {v}")
        return retry_or_fail(keys, f"rank {sorted(asks)[0][1]} asked for a relaunch without {sorted(keys)}")
    if dead:
        t, r, s = min(dead)
        printed = statuses[0].get("printed") if statuses else False
        if printed and s.get("phase") == "finalize":  # died in teardown after the result line
            return {"action": "done"}
        why = f"rank {r} exited with {s.get('exit')} in phase {s.get('phase')!r}"
        return retry_or_fail({s.get("key"): why} if s.get("key") else {}, why)
    # A stall is charged to the LAGGARD: the running rank that entered its
    # current phase first. A hung rank stays in its phase while its peers move
    # on and block in the next collective; their later phases must not take
    # the blame (nor time out before the laggard's own, possibly longer,
    # deadline has passed).
    running = [(float(s["since"]), r, s) for r, s in enumerate(statuses)
               if s.get("exit") is None and s.get("since") is not None]
    if running:
        since, r, s = min(running)
        over = now - since
        if over > float(s.get("deadline", DEFAULT_DEADLINE)):
            if statuses[0].get("printed") and s.get("phase") == "finalize":
                return {"action": "done"}
            why = f"rank {r} stalled in phase {s.get('phase')!r} for {over:.0f} s"
            return retry_or_fail({s.get("key"): why} if s.get("key") else {}, why)
    return None


def _read_phase(path: str) -> dict:
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def free_port(host: str = "127.0.0.1") -> int:
    with socket.socket() as sk:
        sk.bind((host, 0))
        return sk.getsockname()[1]


def _stop(procs: list, grace: float = 10.0) -> None:
    """Stop exact child process groups (never by pattern)."""
    procs = list(procs)
    for p in procs:
        if p is not None and p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except OSError:
                pass
    t0 = time.monotonic()
    for p in procs:
        if p is None:
            continue
        try:
            p.wait(timeout=max(0.1, grace - (time.monotonic() - t0)))
        except subprocess.TimeoutExpired:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except OSError:
                pass
            p.wait()
    for p in procs:
        if p in _LIVE:
            _LIVE.remove(p)


_LIVE: list = []  # worker processes of this supervisor (stopped if it is terminated)


def _on_term(signum, frame) -> None:
    """A supervisor that is told to stop (the launcher tearing the job down,
    a driver timeout) first stops its workers: they run in their own process
    groups and would otherwise keep the GPU."""
    _stop(_LIVE, grace=5.0)
    raise SystemExit(128 + signum)


def _install_term_handler() -> None:
    for sig in (signal.SIGTERM, signal.SIGHUP):
        try:
            signal.signal(sig, _on_term)
        except (ValueError, OSError):  # not the main thread
            pass


def _spawn(argv: list, env: dict, out) -> subprocess.Popen:
    p = subprocess.Popen(argv, env=env, stdout=out, stderr=None, start_new_session=True)
    _LIVE.append(p)
    return p


def _result_line(out) -> tuple[str | None, list]:
    out.seek(0)
    rec, other = None, []
    for ln in out.read().splitlines():
        if ln.startswith("{") and '"metric"' in ln:
            rec = ln
        else:
            other.append(ln)
    return rec, other


def _log(msg: str) -> None:
    print(f"[igg supervise] {msg}", file=sys.stderr, flush=True)


# --------------------------------------------------------- self-launch parent
def run_local(argv: list, n: int, base_env: dict, *, max_attempts: int = 4, timeout: float = 1800.0,
              env_for_rank=None, poll: float = 0.1) -> tuple[int, str | None, dict]:
    """Start ``n`` worker ranks of ``argv`` on this node and supervise them.

    Returns (exit code, rank 0's result line or None, {key: reason} excluded).
    ``env_for_rank(r, env)`` may adjust a rank's environment."""
    _install_term_handler()
    try:
        return _run_local(argv, n, base_env, max_attempts, timeout, env_for_rank, poll)
    finally:
        _stop(_LIVE)  # whatever ended the supervision, no worker outlives it


def _run_local(argv, n, base_env, max_attempts, timeout, env_for_rank, poll):
    excl = excluded(base_env)
    t_end = time.monotonic() + timeout
    tmp = tempfile.mkdtemp(prefix="igg_sup_")
    for attempt in range(max_attempts + 1):
        port = free_port()
        procs, outs, files = [], [], []
        for r in range(n):
            env = dict(base_env)
            env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), IGG_SUP_ATTEMPT=str(attempt),
                       IGG_PHASE_FILE=os.path.join(tmp, f"a{attempt}.r{r}.json"), IGG_SUP_CHILD="1")
            env.pop("TORCHELASTIC_USE_AGENT_STORE", None)
            if excl:
                env["IGG_EXCLUDE"] = json.dumps(excl)
            if env_for_rank is not None:
                env_for_rank(r, env)
            files.append(env["IGG_PHASE_FILE"])
            out = tempfile.TemporaryFile(mode="w+")
            outs.append(out)
            procs.append(_spawn(argv, env, out))
        exit_t = [None] * n
        t_start = time.time()  # a rank that never wrote a phase is "starting" since the launch
        verdict = None
        try:
            while verdict is None:
                now = time.time()
                st = []
                for r in range(n):
                    s = _read_phase(files[r])
                    c = procs[r].poll()
                    if c is not None:
                        if exit_t[r] is None:
                            exit_t[r] = now
                        s.update(exit=c, exit_t=exit_t[r])
                    else:
                        s["exit"] = None
                        s.setdefault("phase", "start")
                        s.setdefault("since", t_start)
                        s.setdefault("deadline", DEFAULT_DEADLINE)
                    st.append(s)
                verdict = decide(st, now, excl, max_attempts - attempt)
                if verdict is None and time.monotonic() > t_end:
                    verdict = {"action": "fail", "why": f"timed out after {timeout:.0f} s"}
                if verdict is None:
                    time.sleep(poll)
        except KeyboardInterrupt:
            verdict = {"action": "fail", "why": "interrupted"}
        _stop(procs)
        rec, other = _result_line(outs[0])
        for ln in other:
            print(ln, file=sys.stderr)
        for o in outs:
            o.close()
        if verdict["action"] == "done":
            return 0, rec, excl
        if verdict["action"] == "retry":
            _log(f"attempt {attempt}: {verdict['why']}; relaunching without {sorted(verdict['exclude'])}")
            excl.update(verdict["exclude"])
            continue
        _log(f"attempt {attempt}: {verdict['why']}")
        return 1, None, excl
    return 1, None, excl


# ------------------------------------------------------ torchrun supervisors
class _StoreGroup:
    """Supervisors of one job (one per launcher rank) over a TCP store."""

    def __init__(self, rank: int, size: int):
        import datetime

        import torch.distributed as dist

        host = os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = int(os.environ["MASTER_PORT"])
        to = datetime.timedelta(seconds=float(os.environ.get("IGG_SUP_STORE_TIMEOUT", "900")))
        if os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True":  # torchrun's agent hosts it
            base = dist.TCPStore(host, port, size, False, timeout=to)
        else:  # plain env launcher: rank 0 hosts it (as env:// would)
            base = dist.TCPStore(host, port, size, rank == 0, timeout=to)
        self.store = dist.PrefixStore("igg_supervise", base)
        self.rank, self.size = rank, size

    def set(self, k: str, v: dict) -> None:
        self.store.set(k, json.dumps(v))

    def get(self, k: str) -> dict | None:
        if not self.store.check([k]):
            return None
        return json.loads(self.store.get(k))

    def wait(self, k: str) -> dict:
        self.store.wait([k])
        return json.loads(self.store.get(k))


def run_torchrun(argv: list, *, max_attempts: int = 4, timeout: float = 1800.0, poll: float = 0.2,
                 env_adjust=None) -> int:
    """Supervisor of ONE worker rank under a launcher (``torchrun``): this
    process (which never touches the GPU) starts the worker with the same
    rank/world and a per-attempt rendezvous port, and agrees with the other
    supervisors over the launcher's TCP store on done / relaunch / fail.
    Supervisor 0 decides; rank 0's supervisor prints the result line."""
    _install_term_handler()
    try:
        return _run_torchrun(argv, max_attempts, timeout, poll, env_adjust)
    finally:
        _stop(_LIVE)


def _run_torchrun(argv, max_attempts, timeout, poll, env_adjust):
    rank, size = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    g = _StoreGroup(rank, size)
    excl = excluded()
    t_end = time.monotonic() + timeout
    tmp = tempfile.mkdtemp(prefix="igg_sup_")
    for attempt in range(max_attempts + 1):
        if rank == 0:
            g.set(f"a{attempt}/port", {"port": free_port(os.environ.get("MASTER_ADDR", "127.0.0.1")),
                                       "exclude": excl})
        info = g.wait(f"a{attempt}/port")
        excl = dict(info["exclude"])
        env = dict(os.environ)
        env.update(MASTER_PORT=str(info["port"]), IGG_SUP_ATTEMPT=str(attempt), IGG_SUP_CHILD="1",
                   IGG_PHASE_FILE=os.path.join(tmp, f"a{attempt}.json"))
        env.pop("TORCHELASTIC_USE_AGENT_STORE", None)
        if excl:
            env["IGG_EXCLUDE"] = json.dumps(excl)
        else:
            env.pop("IGG_EXCLUDE", None)
        if env_adjust is not None:
            env_adjust(env)
        out = tempfile.TemporaryFile(mode="w+")
        p = _spawn(argv, env, out)
        exit_t, last_pub, verdict = None, None, None
        t_start = time.time()
        while verdict is None:
            now = time.time()
            s = _read_phase(env["IGG_PHASE_FILE"])
            c = p.poll()
            if c is not None:
                exit_t = exit_t or now
                s.update(exit=c, exit_t=exit_t)
            else:
                s["exit"] = None
                if "since" not in s:  # no phase written yet: starting since the launch
                    s.update(phase="start", since=t_start, deadline=DEFAULT_DEADLINE)
            pub = json.dumps(s, sort_keys=True)
            if pub != last_pub:
                g.set(f"a{attempt}/s{rank}", s)
                last_pub = pub
            if rank == 0:
                st = []
                for r in range(size):
                    x = g.get(f"a{attempt}/s{r}")
                    if x is None:  # not reported yet: running since the attempt began (as in _run_local)
                        x = {"exit": None, "phase": "start", "since": t_start, "deadline": DEFAULT_DEADLINE}
                    st.append(x)
                verdict = decide(st, now, excl, max_attempts - attempt)
                if verdict is None and time.monotonic() > t_end:
                    verdict = {"action": "fail", "why": f"timed out after {timeout:.0f} s"}
                if verdict is not None:
                    g.set(f"a{attempt}/verdict", verdict)
            else:
                verdict = g.get(f"a{attempt}/verdict")
            if verdict is None:
                time.sleep(poll)
        _stop([p])
        g.set(f"a{attempt}/stopped{rank}", {"ok": True})
        rec, other = _result_line(out)
        out.close()
        for ln in other:
            print(ln, file=sys.stderr)
        if verdict["action"] == "done":
            if rank == 0 and rec is not None:
                print(rec, flush=True)
            return 0 if (rank != 0 or rec is not None) else 1
        if verdict["action"] == "retry":
            # every worker of this attempt is gone before the next one starts
            for r in range(size):
                g.wait(f"a{attempt}/stopped{r}")
            if rank == 0:
                _log(f"attempt {attempt}: {verdict['why']}; relaunching without {sorted(verdict['exclude'])}")
                excl.update(verdict["exclude"])
            continue
        if rank == 0:
            _log(f"attempt {attempt}: {verdict['why']}")
        return 1
    return 1
