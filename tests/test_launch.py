"""igg.utils.launch: the mpiexec-style local launcher."""
import io
import os
import subprocess
import sys

from igg.utils.launch import launch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_launch_runs_every_rank_with_the_distributed_env(tmp_path):
    s = tmp_path / "w.py"
    s.write_text("import os\nprint('rank', os.environ['RANK'], 'of', os.environ['WORLD_SIZE'], "
                 "os.environ['MASTER_ADDR'], os.environ['LOCAL_RANK'])\n")
    out = io.StringIO()
    assert launch(3, [sys.executable, str(s)], out=out) == 0
    lines = sorted(out.getvalue().splitlines())
    assert lines == [f"[{r}] rank {r} of 3 127.0.0.1 {r}" for r in range(3)]


def test_launch_stops_the_others_when_a_rank_fails(tmp_path):
    s = tmp_path / "f.py"
    s.write_text("import os, sys, time\nif os.environ['RANK'] == '1':\n    sys.exit(3)\ntime.sleep(60)\n")
    out = io.StringIO()
    import time

    t0 = time.time()
    assert launch(3, [sys.executable, str(s)], out=out, grace=5) == 3
    assert time.time() - t0 < 30


def test_launch_cli_runs_an_example_on_two_cpu_ranks():
    env = dict(os.environ, OMP_NUM_THREADS="1", IGG_HOST_THREADS="2",
               PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    r = subprocess.run([sys.executable, "-m", "igg.utils.launch", "-n", "2",
                        os.path.join(ROOT, "examples", "diffusion3D_multicpu_novis.py"), "--nx", "12", "--nt", "4"],
                       capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "[0]" in r.stdout and "ms/step" in r.stdout
