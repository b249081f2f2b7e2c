"""Fail-soft supervision (igg/utils/supervise.py): the decision function, and
the benchmark surviving an injected hang or a relaunch request by excluding
the path that failed (CPU plumbing mode, gloo ranks).

Reference: a failing rank aborts the MPI job (src/init_global_grid.jl:80-92);
here the job loses the failing path, not its result."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")
sys.path.insert(0, ROOT)

from igg.utils import supervise as S  # noqa: E402


def st(phase="x", key=None, since=0.0, deadline=10.0, exit=None, **kw):
    d = {"phase": phase, "key": key, "since": since, "deadline": deadline, "exit": exit}
    d.update(kw)
    return d


def test_decide_done_and_wait():
    assert S.decide([st(exit=0), st(exit=0)], 5.0, {}, 3) == {"action": "done"}
    assert S.decide([st(exit=0), st()], 5.0, {}, 3) is None


def test_decide_stall_excludes_the_phase_key():
    v = S.decide([st(since=5.0), st(phase="validate:rccl-sequential", key="rccl", since=0.0, deadline=10.0)], 11.0,
                 {}, 3)
    assert v["action"] == "retry" and list(v["exclude"]) == ["rccl"]
    assert "rank 1 stalled" in v["exclude"]["rccl"]


def test_decide_charges_a_stall_to_the_laggard():
    """Rank 0 hangs in 'model' (long deadline); rank 1 moved on and waits in a
    collective of 'validate:put' (short deadline): not a put failure."""
    sts = [st(phase="model", since=0.0, deadline=100.0), st(phase="validate:put", key="put", since=5.0, deadline=10.0)]
    assert S.decide(sts, 50.0, {}, 3) is None  # the laggard's deadline has not passed
    v = S.decide(sts, 101.0, {}, 3)
    assert v["action"] == "fail" and "rank 0 stalled in phase 'model'" in v["why"]


def test_decide_fails_when_nothing_is_left_to_exclude():
    # no key, the key already excluded, or no attempts left: fail
    assert S.decide([st(phase="init", since=0, deadline=1)], 2.0, {}, 3)["action"] == "fail"
    assert S.decide([st(key="put", since=0, deadline=1)], 2.0, {"put": "x"}, 3)["action"] == "fail"
    assert S.decide([st(key="put", since=0, deadline=1)], 2.0, {}, 0)["action"] == "fail"


def test_decide_death_uses_the_first_dead_ranks_phase():
    v = S.decide([st(key="fused", exit=1, exit_t=5.0), st(key="rccl", exit=-9, exit_t=4.0)], 6.0, {}, 2)
    assert v["action"] == "retry" and list(v["exclude"]) == ["rccl"]


def test_decide_relaunch_request():
    v = S.decide([st(exit=S.RELAUNCH_EXIT, relaunch={"put": "ipc open abandoned"}), st(exit=S.RELAUNCH_EXIT,
                  relaunch={"put": "x"})], 1.0, {}, 2)
    assert v["action"] == "retry" and list(v["exclude"]) == ["put"]


def test_decide_teardown_after_the_result_is_done():
    v = S.decide([st(phase="finalize", printed=True, since=0, deadline=1), st(exit=0)], 5.0, {}, 0)
    assert v == {"action": "done"}


def test_excluded_parses_json_and_lists():
    assert S.excluded({"IGG_EXCLUDE": '{"rccl": "hang"}'}) == {"rccl": "hang"}
    assert set(S.excluded({"IGG_EXCLUDE": "put, fused"})) == {"put", "fused"}
    assert S.excluded({}) == {}


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT",
                                                             "IGG_EXCLUDE")}
    env.update(OMP_NUM_THREADS="1", IGG_HOST_THREADS="2", **kw)
    return env


def _json(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) <= 1, stdout
    return json.loads(lines[0]) if lines else None


ARGS = ["--device", "cpu", "--n", "20", "--steps", "3", "--warmup", "1"]


def test_self_launch_survives_an_injected_hang():
    """Rank 1 hangs forever in the validation of the order-only host matching:
    the supervisor stops the attempt at the phase deadline, relaunches fresh
    ranks without that path, and the run still reports - naming the
    exclusion."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", *ARGS], capture_output=True, text=True, timeout=240,
                       env=_env(IGG_INJECT_PHASE_HANG="validate:host-ordered@1", IGG_PHASE_DEADLINE_SCALE="0.05"),
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json(r.stdout)
    c = rec["config"]
    assert rec["n_gpus"] == 2
    assert "host-ordered" in c["excluded"] and "stalled" in c["excluded"]["host-ordered"], c["excluded"]
    assert c["supervisor_attempt"] == 1
    assert c["validation"]["host-ordered"].startswith("excluded")
    assert c["post_validation"]["result"] == "ok"
    assert "relaunching without ['host-ordered']" in r.stderr


def test_relaunch_request_after_an_abandoned_call():
    """A rank whose bounded first-contact call had to be abandoned makes every
    rank ask for fresh processes without that path (exit code 3)."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", *ARGS], capture_output=True, text=True, timeout=240,
                       env=_env(IGG_BENCH_INJECT="abandon-host-ordered"), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    c = _json(r.stdout)["config"]
    assert "host-ordered" in c["excluded"] and "abandoned" in c["excluded"]["host-ordered"], c["excluded"]


def test_unexcludable_hang_fails_without_a_number():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", *ARGS], capture_output=True, text=True, timeout=240,
                       env=_env(IGG_INJECT_PHASE_HANG="model@0", IGG_PHASE_DEADLINE_SCALE="0.02"), cwd=ROOT)
    assert r.returncode != 0
    assert _json(r.stdout) is None
    assert "stalled in phase 'model'" in r.stderr and "nothing left to exclude" in r.stderr


def test_torchrun_supervisors_survive_an_injected_hang():
    """The driver's launch form: one supervisor per torchrun rank, agreeing
    over the launcher's TCP store, relaunches its worker without the hung
    path."""
    from tests._mp import free_port

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), BENCH, "--gpus", "2",
           *[a.replace("--n", "--local-n") if a == "--n" else a for a in ARGS]]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT,
                       env=_env(IGG_INJECT_PHASE_HANG="validate:host-ordered@0", IGG_PHASE_DEADLINE_SCALE="0.05"))
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json(r.stdout)
    assert rec["n_gpus"] == 2 and rec["config"]["self_launched"] is False
    assert "host-ordered" in rec["config"]["excluded"]
    assert rec["config"]["supervisor_attempt"] == 1


def test_terminated_supervisor_stops_its_workers():
    """The launcher (or a driver timeout) terminating the self-launch parent
    must not leave its worker ranks running - they hold the GPU."""
    import signal
    import time
    import uuid

    marker = uuid.uuid4().hex
    p = subprocess.Popen([sys.executable, BENCH, "--gpus", "2", *ARGS], stdout=subprocess.DEVNULL,
                         stderr=subprocess.DEVNULL, cwd=ROOT,
                         env=_env(IGG_INJECT_PHASE_HANG="model@0", IGG_TEST_MARKER=marker))

    def workers():
        out = []
        for pid in os.listdir("/proc"):
            if not pid.isdigit() or int(pid) == p.pid:
                continue
            try:
                with open(f"/proc/{pid}/environ", "rb") as f:
                    if f"IGG_TEST_MARKER={marker}".encode() in f.read() and b"IGG_SUP_CHILD=1" in open(
                            f"/proc/{pid}/environ", "rb").read():
                        out.append(int(pid))
            except OSError:
                pass
        return out

    t0 = time.monotonic()
    while len(workers()) < 2 and time.monotonic() - t0 < 60:
        time.sleep(0.5)
    assert len(workers()) == 2, "the workers did not start"
    p.send_signal(signal.SIGTERM)
    p.wait(timeout=60)
    t1 = time.monotonic()
    while workers() and time.monotonic() - t1 < 20:
        time.sleep(0.5)
    assert workers() == [], "workers outlived their terminated supervisor"
