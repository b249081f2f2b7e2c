"""bench.py contract: ``--gpus N`` without a launcher starts N ranks itself and
reports n_gpus == N; a --gpus/WORLD_SIZE mismatch or a failing rank is an error,
never a silent 1-process number. Runs the CPU (gloo) plumbing mode."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(OMP_NUM_THREADS="1", IGG_HOST_THREADS="2", **kw)
    return env


def _run(args, timeout=150, **env):
    r = subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True, timeout=timeout,
                       env=_env(**env), cwd=ROOT)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, (json.loads(lines[-1]) if lines else None)


@pytest.mark.parametrize("n", [1, 2])
def test_metric_label_says_what_value_is(n):
    """The metric label states the value's semantics (whole-job aggregate), and
    the value is n_gpus x the per-GPU T_eff (also at N=1)."""
    r, rec = _run(["--gpus", str(n), "--device", "cpu", "--n", "20", "--steps", "3", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-3000:]
    assert rec["metric"].startswith("effective GB/s per GPU + weak-scaling parallel efficiency")  # BASELINE.json
    assert "whole-job aggregate" in rec["metric"] and "sum of the per-GPU T_eff" in rec["metric"]
    assert "aggregate" in rec["unit"]
    assert abs(rec["value"] - n * rec["config"]["t_eff_per_gpu_GBs"]) <= 1e-3 * rec["value"] + 0.01
    if n > 1:  # the post-timing validation ran on every multi-rank run
        assert rec["config"]["post_validation"]["result"] == "ok", rec["config"]["post_validation"]
    else:
        assert rec["config"]["post_validation"] is None


def test_post_validation_fails_closed():
    """A mismatch in the post-timing validation (injected on rank 0) leaves no
    schedule to fall back to in the CPU plumbing mode: the bench fails and
    prints no number."""
    r, rec = _run(["--gpus", "2", "--device", "cpu", "--n", "20", "--steps", "3", "--warmup", "1"],
                  IGG_BENCH_INJECT="post_validation")
    assert r.returncode != 0
    assert rec is None
    assert "post-timing validation failed" in r.stderr


@pytest.mark.parametrize("n", [1, 2])
def test_stencil_post_check_fails_closed(n):
    """After the timed region the same K steps are recomputed from the saved
    starting state (on a GPU through a second compiled stencil variant) and
    compared bitwise: a mismatch (injected on rank 0) means no result line,
    at N = 1 too."""
    r, rec = _run(["--gpus", str(n), "--device", "cpu", "--n", "20", "--steps", "3", "--warmup", "1"],
                  IGG_BENCH_INJECT="stencil_post")
    assert r.returncode != 0
    assert rec is None
    assert "post-timing stencil check failed" in r.stderr


def test_stencil_post_check_recorded_at_n1():
    r, rec = _run(["--gpus", "1", "--device", "cpu", "--n", "20", "--steps", "3", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-3000:]
    sp = rec["config"]["stencil_post_check"]
    assert sp["result"] == "ok" and sp["steps"] == 3


@pytest.mark.parametrize("n", [2, 4])
def test_self_launch_reports_n_gpus(n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--device", "cpu", "--n", "24", "--steps", "4",
                        "--warmup", "1"], capture_output=True, text=True, timeout=150, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == n and rec["steps"] == 4 and rec["warmup"] == 1
    assert rec["config"]["self_launched"] is True
    assert rec["config"]["finite"] is True
    # whole-job aggregate = n x per-GPU T_eff
    assert abs(rec["value"] - n * rec["config"]["t_eff_per_gpu_GBs"]) <= 1e-3 * rec["value"] + 0.01
    assert rec["ms_per_step"] == rec["config"]["t_it_ms"]


def test_share_gpu_self_launch_forces_one_hw_queue():
    """--share-gpu with > 2 ranks runs every rank with one hardware queue, even
    when the environment exports more (the GPU boxes export 4: N x 4 queues on
    one device are time-sliced, profiles/r2_reh8/)."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--share-gpu", "--device", "cpu", "--n", "20",
                        "--steps", "2", "--warmup", "1"], capture_output=True, text=True, timeout=150,
                       env=_env(GPU_MAX_HW_QUEUES="4"), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert rec["n_gpus"] == 3 and rec["config"]["hw_queues"] == "1"


def test_world_size_mismatch_is_an_error():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--device", "cpu", "--n", "16", "--steps", "1",
                        "--warmup", "0"], capture_output=True, text=True, timeout=60,
                       env=_env(WORLD_SIZE="1", RANK="0"), cwd=ROOT)
    assert r.returncode != 0
    assert "refusing" in r.stderr
    assert not any(ln.startswith("{") for ln in r.stdout.splitlines())


def test_failing_rank_fails_the_launch():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--device", "cpu", "--n", "1", "--steps", "1",
                        "--warmup", "0"], capture_output=True, text=True, timeout=120, env=_env(), cwd=ROOT)
    assert r.returncode != 0
    assert "self-launch" in r.stderr
    assert not any(ln.startswith("{") for ln in r.stdout.splitlines())


def test_driver_torchrun_launch_form():
    """The driver's N-rank command (torch.distributed.run, one rank per GPU,
    127.0.0.1 rendezvous) prints exactly one JSON line, from rank 0, with
    n_gpus == N and not self-launched (CPU plumbing mode)."""
    sys.path.insert(0, ROOT)
    from tests._mp import free_port

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), BENCH,
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--device", "cpu", "--local-n", "20"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=150, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["steps"] == 3 and rec["warmup"] == 1
    assert rec["config"]["self_launched"] is False
    assert rec["config"]["parallelism"] == "spatial 2x1x1"


@pytest.mark.gpu
@pytest.mark.timeout(420)  # subprocess bound 280 s + import/launch headroom (pytest.ini: a timeout aborts the session)
@pytest.mark.parametrize("inject", ["", "fused_post"])
def test_share_gpu_post_timing_checks(inject):
    """Two ranks on one GPU (put transport, fused exchange): the JSON carries
    the post-timing transport validation and the post-timing fused check; an
    injected fused mismatch fails closed (fused dropped, region re-timed on the
    update_halo_ path, the result still validated)."""
    r, rec = _run(["--gpus", "2", "--share-gpu", "--fused", "on", "--n", "96", "--steps", "20", "--warmup", "2",
                   "--launch-timeout", "240"], timeout=280, IGG_BENCH_INJECT=inject,
                  IGG_FUSED_CANDIDATES="0/8/3,42/12/2", IGG_STENCIL_VARIANT="0")
    assert r.returncode == 0, r.stderr[-3000:]
    c = rec["config"]
    assert c["post_validation"]["result"] == "ok", c["post_validation"]
    assert c["post_validation"]["transport"] == c["transport"]
    fp = c["fused_post_check"]
    assert fp is not None and fp["steps"] >= 200, (c.get("fused_ab_ms"), r.stderr[-3000:])
    if inject:
        assert fp["result"] == "mismatch" and "fallback" in fp
        assert c["fused_halo"] is False
    else:
        assert fp["result"] == "ok" and c["fused_halo"] is True


@pytest.mark.parametrize("n", [1, 2])
def test_efficiency_measured_in_the_same_job(n):
    """config.efficiency: interleaved pairs of the 1-GPU run's local problem
    (plain stencil, no exchange) and the real step, on the same processes;
    value = median t_local / median t_step, with per-rank numbers."""
    r, rec = _run(["--gpus", str(n), "--device", "cpu", "--n", "20", "--steps", "4", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-3000:]
    e = rec["config"]["efficiency"]
    assert e is not None and e["pairs"] >= 5 and e["steps"] % 2 == 0
    assert len(e["local_ms_samples"]) == e["pairs"] == len(e["step_ms_samples"])
    assert abs(e["value"] - e["t_local_ms"] / e["t_step_ms"]) <= 1e-3 * e["value"] + 1e-4
    assert len(e["per_rank_local_ms"]) == n == len(e["per_rank_efficiency"])
    # the pair order alternates (local-first in every pair
    # biased the N=1 value), and min/median/max are reported for both forms
    assert e["pair_order"] == ["local,step" if i % 2 == 0 else "step,local" for i in range(e["pairs"])]
    for key in ("local_ms", "step_ms"):
        assert e[key]["min"] <= e[key]["median"] <= e[key]["max"]
    # per-rank efficiency: each rank's local time over its OWN step time
    for a, s, x in zip(e["per_rank_local_ms"], e["per_rank_step_ms"], e["per_rank_efficiency"]):
        assert abs(x - a / s) <= 1e-3 * x + 1e-4


def test_nothing_between_warm_load_and_bracket():
    """The post-check snapshot (allocation + copy) is taken BEFORE the warm
    load, and the timed region's bracket follows the warm load directly (round
    4 lost 2.9 % of the driver's 20-step number to a snapshot in between); the
    stencil post check replays the warm load + the timed steps."""
    r, rec = _run(["--gpus", "1", "--device", "cpu", "--n", "20", "--steps", "4", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-3000:]
    order = rec["config"]["stage_order"]
    i = order.index("timed")
    assert order[i - 1] == "warm_load", order
    assert order[i - 2] == "snapshot", order
    assert "efficiency" in order[:i - 2], order
    sp = rec["config"]["stencil_post_check"]
    assert sp["result"] == "ok" and sp["timed_steps"] == 4 and sp["steps"] >= 4


def test_ab_budget_orders_and_truncates():
    """The A/B budget is collective and the fused candidates are tried in the
    order of their win record (a spent budget drops the never-winners)."""
    import importlib.util as ilu

    spec = ilu.spec_from_file_location("bench_mod", BENCH)
    b = ilu.module_from_spec(spec)
    spec.loader.exec_module(b)
    cands = [(0, 0, 3), (42, 12, 2), (9, 8, 3), (50, 1, 2)]
    assert b._win_order(cands) == [(9, 8, 3), (42, 12, 2), (0, 0, 3), (50, 1, 2)]

    class _C:
        size = 1

    bud = b._ABBudget(_C(), seconds=0.0)
    import time as _t

    _t.sleep(0.01)
    assert not bud.left()
    assert b._ABBudget(_C(), seconds=100.0).left()


@pytest.mark.parametrize("model", ["acoustic", "diffusion"])
def test_efficiency_phase_leaves_a_consistent_state(model):
    """The efficiency phase's local steps (no exchange) are undone for the
    timed region: the acoustic model's state is restored bitwise (its
    staggered fields have planes computed on two ranks that drift apart), the
    diffusion model's halos are re-exchanged (periodic: halo = wrapped
    interior)."""
    import importlib.util as ilu

    import torch

    import igg

    spec = ilu.spec_from_file_location("bench_mod", BENCH)
    b = ilu.module_from_spec(spec)
    spec.loader.exec_module(b)

    class _C:
        size = 1

        def barrier(self):
            pass

    b._BRACKET["gpu"] = False
    if model == "acoustic":
        from igg.models.acoustic2d import Acoustic2D

        igg.init_global_grid(20, 16, 1, periodx=1, periody=1, quiet=True, init_MPI=False)
        m = Acoustic2D(dtype=torch.float64)
    else:
        from igg.models.diffusion3d import Diffusion3D

        igg.init_global_grid(12, 10, 8, periodx=1, periody=1, periodz=1, quiet=True, init_MPI=False)
        m = Diffusion3D(dtype=torch.float64)
    try:
        m.run(3)
        before = {n: getattr(m, n).clone() for n in b._state(m)}
        e = b.measure_efficiency(m, _C(), lambda s: None, False, 4)
        assert e is not None and e["steps"] == b.EFF_MIN_STEPS
        if model == "acoustic":
            assert all(torch.equal(before[n], getattr(m, n)) for n in before)
            assert m._entry
        else:
            T = m.T
            assert not torch.equal(before["T"], T)  # the phase's real steps advanced it
            for d in range(3):
                lo, hi = T.select(d, 0), T.select(d, T.shape[d] - 1)
                assert torch.equal(lo, T.select(d, T.shape[d] - 2)) and torch.equal(hi, T.select(d, 1))
    finally:
        igg.finalize_global_grid(finalize_MPI=False)
