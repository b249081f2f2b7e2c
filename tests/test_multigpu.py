"""Real multi-GPU tier: ONE RANK PER DISTINCT MI355X (LOCAL_RANK = device).

Only these tests exercise what single-GPU runs cannot: RCCL point-to-point
between devices over xGMI, IPC mappings of another device's memory (put
transport, fused exchange, gather pulls) and cross-device memory ordering
(docs/COHERENCE.md). Every test is skipped when fewer GPUs than ranks are
visible, so the tier collects and skips cleanly on a 1-GPU box; run it on a
node with ``python -m pytest tests -m multigpu``.

First-run-proof budget: the checks are chained into suites, one launch of the
ranks per suite (tests/mp_worker.py scenario_suite: one torch import and one
rendezvous per launch, the grid re-initialised per item). The WHOLE tier has
one wall budget (tests/_mp.py TierBudget, IGG_MGPU_TIER_BUDGET, default
480 s): each launch is bounded by min(170 s, what is left) and a launch that
would start with < 30 s left is skipped, so the tier's worst case is the
budget, not launches x 170 s; with the single-GPU tests (<= 300 s) that
stays inside the driver's 900 s step cap. The launches run in the order of
their value, so a spent budget drops the least essential ones:

    1  8-rank halo oracle (RCCL sequential / one-phase / auto, put) + ring + select_transport
       + the IGG_TRANSPORT=auto first-exchange choice
    1b 8-rank direct-z fused soak
    2  2-rank suite (left == right periodic neighbour: same-peer ordering)
    3  4-rank suite (2x2x1)
    4  8-rank gather (pull and RCCL paths, roots 0 and 7) + gather_async + collectives
    5  8-rank fused exchange forms (z unpack with the in-kernel step sync included)
       + diffusion vs the global-grid run
    6, 7  bench.py --gpus 2 / --gpus 8 self-launch (validation + post-timing checks)
    9, 10 2- and 4-rank direct-z fused soak

A launch the budget drops is skipped with a PytestWarning in the summary.

Expected on a healthy node: about 3-4 min (each suite item takes seconds).

Reference counterparts: test/test_update_halo.jl (halo oracle incl. dims=2
periodic, where left == right neighbour), :697-743 (ring), test/test_gather.jl
:126-137 (gather to root 0 / last rank).
"""
import json
import os
import subprocess
import sys
import warnings

import pytest

from tests._mp import ROOT, TierBudget, run_ranks

pytestmark = [pytest.mark.gpu, pytest.mark.multigpu]


def _ngpus() -> int:
    try:
        import torch

        return torch.cuda.device_count()  # does not initialise HIP on this image
    except Exception:
        return 0


def need(n: int):
    if _ngpus() < n:
        pytest.skip(f"needs {n} GPUs (one rank per device), {_ngpus()} visible")


MGPU = "IGG_TEST_DEV=mgpu"
RCCL = f"{MGPU};IGG_TRANSPORT=rccl"
PUT = f"{MGPU};IGG_TRANSPORT=put;IGG_PUT_TIMEOUT=20"


def fused(v, mode, *cfg, rounds=None):
    """Fused exchange (stencil stores its send planes over xGMI) vs stencil +
    update_halo_ (RCCL), bitwise on every rank."""
    r = f";IGG_TEST_FUSED_ROUNDS={rounds}" if rounds else ""
    return f"diffusion_fused:{':'.join(map(str, cfg))}|{RCCL};IGG_PUT_TIMEOUT=20;IGG_TEST_VARIANT={v};" \
           f"IGG_TEST_FUSED_MODE={mode}{r}"


def soak(v, mode, rounds=40, per=40):
    return f"fused_soak:20:18:32:{rounds}:{per}|{PUT};IGG_PUT_TIMEOUT=30;IGG_TEST_VARIANT={v};" \
           f"IGG_TEST_FUSED_MODE={mode}"


def halo(cfg, env):
    return f"halo:mgpu:{':'.join(map(str, cfg))}:f64|{env}"


TIER = TierBudget(float(os.environ.get("IGG_MGPU_TIER_BUDGET", "480")))


def _launch_timeout() -> float:
    t = TIER.next_timeout()
    if t is None:
        # not silent: a spent budget means the tier ran slow
        warnings.warn(f"multigpu tier budget ({TIER.seconds:.0f} s) spent: launch skipped; "
                      "raise IGG_MGPU_TIER_BUDGET to run it", pytest.PytestWarning)
        pytest.skip(f"multigpu tier budget ({TIER.seconds:.0f} s) spent")
    return t


def suite(nprocs, *items):
    need(nprocs)
    outs = run_ranks(nprocs, "suite", *items, timeout=_launch_timeout())
    for o in outs:
        assert f"suite OK ({len(items)} items" in o, o[-3000:]


# 1. halo oracle (every boundary plane, edges and corners, bitwise)
def test_halo_and_ring_8_ranks():
    items = []
    for cfg in ((7, 5, 6, 0, 0, 0), (7, 5, 6, 1, 1, 1)):
        for mode in ("sequential", "onephase", "auto"):
            items.append(halo(cfg, f"{RCCL};IGG_HALO_MODE={mode}"))
    items.append(halo((7, 5, 6, 1, 1, 1), PUT))
    items.append(f"ring:mgpu|{RCCL}")
    items.append(f"select_transport:mgpu|{MGPU}")
    items.append(f"auto_transport:mgpu:fastest|{MGPU};IGG_TRANSPORT=auto;IGG_PUT_TIMEOUT=20")
    suite(8, *items)


# 1b. the direct-z fused soak (direct z: the z faces land in the halo
#    column of the neighbour's next field; random host skew between rounds),
#    early in the tier so a spent budget never drops it
def test_direct_z_fused_soak_8_ranks():
    suite(8, soak(40, 4), soak(42, 12), soak(0, 1))


# 2. two ranks: periodic dims=2 makes left == right (same-peer ordering)
def test_suite_2_ranks():
    suite(2,
          *[halo((7, 5, 6, 1, 1, 1), f"{RCCL};IGG_HALO_MODE={m}") for m in ("sequential", "onephase", "auto")],
          halo((7, 5, 6, 0, 0, 0), RCCL),
          halo((7, 5, 6, 1, 1, 1), PUT),
          f"ring:mgpu|{RCCL}",
          f"gather:mgpu:f64|{RCCL}",
          f"gather_async|{PUT}",
          f"collectives:mgpu|{RCCL}",
          # COHERENCE fact 4 across devices: warm reader L2s, writer on the other GPU
          f"coherence:mgpu:kernel:{4 << 20}:30|{MGPU};IGG_PUT_TIMEOUT=20",
          f"coherence:mgpu:inkernel:{4 << 20}:30|{MGPU};IGG_PUT_TIMEOUT=20",
          fused(0, 0, 24, 20, 64, 6, 0, 0),
          fused(40, 4, 24, 20, 64, 6, 1, 0),
          fused(42, 12, 40, 66, 136, 6, 1, 0))


# 3. four ranks (2x2x1)
def test_suite_4_ranks():
    suite(4,
          *[halo((9, 6, 5, 1, 0, 1), f"{RCCL};IGG_HALO_MODE={m}") for m in ("sequential", "onephase", "auto")],
          halo((9, 6, 5, 1, 0, 1), PUT),
          f"ring:mgpu|{RCCL}",
          f"gather:mgpu:f64|{RCCL}",
          fused(9, 1, 20, 22, 32, 5, 1, 1),
          f"diffusion:mgpu:24:20:18:5:0|{RCCL}")


# 4. gather (pull path and RCCL path, roots 0 and N-1), gather_async, collectives
def test_gather_and_collectives_8_ranks():
    suite(8,
          f"gather:mgpu:f64|{RCCL}",
          f"gather:mgpu:f64|{RCCL};IGG_GATHER_PULL=0",
          f"gather_async|{PUT}",
          f"collectives:mgpu|{RCCL}")


# 5. fused exchange forms and the 8-rank diffusion vs one global array
def test_fused_forms_and_diffusion_8_ranks():
    suite(8,
          fused(0, 1, 18, 20, 40, 7, 0, 0),
          fused(0, 0, 16, 18, 24, 6, 1, 1),
          fused(42, 4, 18, 20, 136, 5, 0, 1),
          fused(0, 5, 16, 18, 24, 6, 1, 1),
          fused(40, 8, 34, 66, 136, 5, 1, 1),
          fused(44, 4, 18, 20, 136, 4, 1, 0),
          fused(9, 72, 18, 20, 136, 5, 0, 1),
          fused(9, 0, 18, 20, 136, 5, 0, 0, rounds=2),
          fused(9, 8, 34, 66, 136, 5, 0, 0, rounds=2),
          fused(42, 64, 16, 18, 136, 5, 1, 1),
          # z unpack with the in-kernel step sync (bit 16): the copy kernel's
          # CopyWait spin on the neighbours' ARRIVED flags across devices
          fused(9, 88, 18, 20, 136, 5, 0, 1),
          fused(42, 80, 16, 18, 136, 5, 1, 0),
          f"diffusion:mgpu:24:20:18:7:0|{RCCL}",
          f"diffusion:mgpu:24:20:18:7:0|{PUT}")


# 6, 7. the bench on N distinct GPUs
@pytest.mark.parametrize("nprocs", [2, 8])
def test_bench_self_launch_validates_every_transport(nprocs):
    """bench.py --gpus N (self-launched, one rank per GPU) validates RCCL
    sequential / one-phase and put bitwise against the host-staged path before
    timing, checks the timed schedule (and the fused exchange, if kept) after
    timing, and reports n_gpus == N."""
    need(nprocs)
    t = _launch_timeout()
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["IGG_BENCH_AB_BUDGET"] = "40"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(nprocs), "--n", "128",
                        "--steps", "20", "--warmup", "2", "--launch-timeout", str(max(20, int(t) - 20))],
                       capture_output=True, text=True, timeout=t, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    c = rec["config"]
    assert rec["n_gpus"] == nprocs
    assert c["validation"] == {"rccl-sequential": "ok", "rccl-onephase": "ok", "put": "ok"}, rec
    assert c["post_validation"]["result"] == "ok", c["post_validation"]
    if c["fused_halo"]:
        assert c["fused_post_check"]["result"] == "ok", c["fused_post_check"]
    assert c["finite"]


# 9, 10. direct-z soak at 2 and 4 ranks
@pytest.mark.parametrize("nprocs", [2, 4])
def test_direct_z_fused_soak_small(nprocs):
    suite(nprocs, soak(40, 4, rounds=30), soak(0, 5, rounds=30))
