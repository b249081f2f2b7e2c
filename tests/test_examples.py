"""The example scripts run end to end (CPU variants; 1 and 4 processes)."""
import os
import subprocess
import sys

import pytest

from tests._mp import ROOT, free_port

EX = os.path.join(ROOT, "examples")


def _run(args, nprocs=1, timeout=240):
    if nprocs == 1:
        cmd = [sys.executable] + args
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nprocs}",
               "--master-addr", "127.0.0.1", "--master-port", str(free_port())] + args
    env = dict(os.environ, OMP_NUM_THREADS="1", IGG_HOST_THREADS="2")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return r.stdout


def test_diffusion_multicpu_novis():
    out = _run([os.path.join(EX, "diffusion3D_multicpu_novis.py"), "--nx", "16", "--nt", "10"])
    assert "ms/step" in out


def test_diffusion_vis_cpu(tmp_path):
    gif = str(tmp_path / "d.gif")
    out = _run([os.path.join(EX, "diffusion3D_multigpu.py"), "--cpu", "--nx", "12", "--nt", "20", "--vis-every", "5",
                "--out", gif], nprocs=4)
    assert "4 frames" in out and os.path.getsize(gif) > 0


def test_acoustic_multicpu(tmp_path):
    gif = str(tmp_path / "a.gif")
    out = _run([os.path.join(EX, "acoustic2D_multigpu.py"), "--cpu", "--nx", "24", "--nt", "10", "--vis-every", "5",
                "--out", gif], nprocs=4)
    assert "[2, 2, 1]" in out and os.path.getsize(gif) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("extra", [[], ["--fused"]])
def test_diffusion_multigpu_novis(extra):
    out = _run([os.path.join(EX, "diffusion3D_multigpu_novis.py"), "--nx", "64", "--nt", "20"] + extra)
    assert "T_eff" in out
