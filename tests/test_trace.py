"""Observability hooks: roctx ranges (dlopen'ed only with IGG_TRACE=1) and the
hipEvent phase timer."""
import os
import subprocess
import sys

import pytest
import torch

from tests._mp import ROOT


def test_trace_disabled_by_default_is_noop():
    from igg.utils.trace import PhaseTimer, trace_range, tracing

    if os.environ.get("IGG_TRACE"):
        pytest.skip("IGG_TRACE set in the environment")
    assert tracing() is False
    with trace_range("x"):
        pass
    t = PhaseTimer()
    with t.phase("a"):
        pass
    assert isinstance(t.summary(), dict)


def test_trace_enabled_loads_roctx():
    code = ("import igg; from igg.utils.trace import trace_range, tracing\n"
            "with trace_range('igg.test'):\n    pass\n"
            "igg.native.trace_mark('m')\nprint(tracing())")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=ROOT,
                       env=dict(os.environ, IGG_TRACE="1", PYTHONPATH=ROOT), timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    have = any(os.path.exists(os.path.join("/opt/rocm/lib", n))
               for n in ("librocprofiler-sdk-roctx.so.1", "libroctx64.so.4"))
    assert r.stdout.strip().splitlines()[-1] == ("True" if have else "False")


@pytest.mark.gpu
def test_phase_timer_on_model(gpu):
    import igg
    from igg.models.diffusion3d import Diffusion3D
    from igg.parallel import halo as H
    from igg.utils.trace import PhaseTimer

    igg.init_global_grid(64, 64, 64, periodx=1, periody=1, periodz=1, quiet=True, init_MPI=False)
    H.enable_loopback()
    m = Diffusion3D(dtype=torch.float64)
    m.timer = PhaseTimer()
    m.run(4)
    s = m.timer.summary()
    assert s["stencil"]["calls"] == 4 and s["update_halo"]["mean_ms"] > 0
    igg.finalize_global_grid(finalize_MPI=False)
