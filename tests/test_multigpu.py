"""Real multi-GPU tier: ONE RANK PER DISTINCT MI355X (LOCAL_RANK = device).

Only these tests exercise what single-GPU runs cannot: RCCL point-to-point
between devices over xGMI, IPC mappings of another device's memory (put
transport, fused exchange, async gather pulls) and cross-device memory
ordering. Every test is skipped when fewer GPUs than ranks are visible, so the
tier collects and skips cleanly on a 1-GPU box; run it on a node with
``python -m pytest tests -m multigpu``.

Reference counterparts: test/test_update_halo.jl (halo oracle incl. dims=2
periodic, where left == right neighbour), :697-743 (ring), test/test_gather.jl
:126-137 (gather to root 0 / last rank).
"""
import json
import os
import subprocess
import sys

import pytest

from tests._mp import ROOT, run_ranks

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


MGPU = {"IGG_TEST_DEV": "mgpu"}
RCCL = {**MGPU, "IGG_TRANSPORT": "rccl"}
PUT = {**MGPU, "IGG_TRANSPORT": "put", "IGG_PUT_TIMEOUT": "20"}


@pytest.mark.parametrize("mode", ["sequential", "onephase", "auto"])
@pytest.mark.parametrize("nprocs,cfg", [
    (2, (7, 5, 6, 1, 1, 1)),   # 2x1x1 periodic: left == right neighbour (same-peer ordering)
    (2, (7, 5, 6, 0, 0, 0)),
    (4, (9, 6, 5, 1, 0, 1)),   # 2x2x1
    (8, (7, 5, 6, 0, 0, 0)),   # 2x2x2
    (8, (7, 5, 6, 1, 1, 1)),   # 2x2x2 periodic: every direction is a neighbour (edges, corners)
])
def test_halo_rccl_across_devices(nprocs, cfg, mode):
    need(nprocs)
    run_ranks(nprocs, "halo", "mgpu", *cfg, "f64", env_extra={**RCCL, "IGG_HALO_MODE": mode})


@pytest.mark.parametrize("nprocs,cfg", [(2, (7, 5, 6, 1, 1, 1)), (4, (9, 6, 5, 1, 0, 1)), (8, (7, 5, 6, 1, 1, 1))])
def test_halo_put_across_devices(nprocs, cfg):
    need(nprocs)
    run_ranks(nprocs, "halo", "mgpu", *cfg, "f64", env_extra=PUT)


@pytest.mark.parametrize("nprocs", [2, 4, 8])
def test_ring_rccl(nprocs):
    need(nprocs)
    run_ranks(nprocs, "ring", "mgpu", env_extra=RCCL)


@pytest.mark.parametrize("nprocs", [2, 4, 8])
def test_gather_rccl_root_first_and_last(nprocs):
    need(nprocs)
    run_ranks(nprocs, "gather", "mgpu", "f64", env_extra=RCCL)


@pytest.mark.parametrize("nprocs", [2, 8])
def test_gather_async_across_devices(nprocs):
    need(nprocs)
    run_ranks(nprocs, "gather_async", env_extra=PUT)


@pytest.mark.parametrize("transport", ["rccl", "put"])
def test_diffusion_8_ranks_matches_global(transport):
    """The 8-rank run (2x2x2) equals the same physics on one global array."""
    need(8)
    run_ranks(8, "diffusion", "mgpu", 24, 20, 18, 7, 0, env_extra=RCCL if transport == "rccl" else PUT)


@pytest.mark.parametrize("nprocs,cfg,kernel", [(2, (24, 20, 64, 6, 0, 0), ("0", "0")),
                                               (4, (20, 22, 32, 5, 1, 1), ("9", "1")),
                                               (8, (18, 20, 40, 7, 0, 0), ("0", "1")),
                                               (8, (16, 18, 24, 6, 1, 1), ("11", "0")),
                                               # direct z (mode bit 4): z faces stored over xGMI into
                                               # the halo column of the neighbour's next field
                                               (2, (24, 20, 64, 6, 1, 0), ("40", "4")),
                                               (8, (18, 20, 136, 5, 0, 1), ("42", "4")),
                                               (8, (16, 18, 24, 6, 1, 1), ("0", "5")),
                                               # peeled x planes (mode bit 8)
                                               (2, (40, 66, 136, 6, 1, 0), ("42", "12")),
                                               (8, (34, 66, 136, 5, 1, 1), ("40", "8"))])
def test_fused_exchange_across_devices(nprocs, cfg, kernel):
    """Stencil kernel stores its send planes into the neighbours' arenas over
    xGMI: bitwise equal to stencil + update_halo_ (RCCL) on every rank."""
    need(nprocs)
    env = {**RCCL, "IGG_PUT_TIMEOUT": "20", "IGG_TEST_VARIANT": kernel[0], "IGG_TEST_FUSED_MODE": kernel[1]}
    run_ranks(nprocs, "diffusion_fused", *cfg, env_extra=env, timeout=170)


@pytest.mark.parametrize("nprocs,kernel", [(4, ("0", "1")), (8, ("0", "1")), (8, ("40", "4"))])
def test_fused_soak_across_devices(nprocs, kernel):
    need(nprocs)
    env = {**PUT, "IGG_PUT_TIMEOUT": "30", "IGG_TEST_VARIANT": kernel[0], "IGG_TEST_FUSED_MODE": kernel[1]}
    run_ranks(nprocs, "fused_soak", 20, 18, 32, 40, 40, env_extra=env, timeout=170)


@pytest.mark.parametrize("nprocs", [2, 8])
def test_tensor_collectives_gpu(nprocs):
    need(nprocs)
    run_ranks(nprocs, "collectives", "mgpu", env_extra=RCCL)


@pytest.mark.parametrize("nprocs", [2, 8])
def test_bench_self_launch_validates_every_transport(nprocs):
    """bench.py --gpus N (self-launched, one rank per GPU) validates RCCL
    sequential / one-phase and put bitwise against the host-staged path and
    reports n_gpus == N."""
    need(nprocs)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(nprocs), "--n", "128",
                        "--steps", "20", "--warmup", "2", "--launch-timeout", "150"],
                       capture_output=True, text=True, timeout=170, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert rec["n_gpus"] == nprocs
    assert rec["config"]["validation"] == {"rccl-sequential": "ok", "rccl-onephase": "ok", "put": "ok"}, rec
    assert rec["config"]["finite"]
