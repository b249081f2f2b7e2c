import sys
sys.path.insert(0, "/root/repo")
from tests._mp import run_ranks
env = {"IGG_TRANSPORT": "staged", "IGG_PUT_TIMEOUT": "20", "GPU_MAX_HW_QUEUES": "1"}
for nprocs, n, per, graph in [(4, 512, 0, 0), (4, 512, 0, 1), (2, 512, 0, 0), (4, 64, 0, 0), (4, 512, 1, 0)]:
    try:
        outs = run_ranks(nprocs, "acoustic_fused_soak", n, n, 200, per, graph, env_extra=env, timeout=120)
        print(nprocs, n, per, graph, "OK")
    except AssertionError as e:
        lines = [l for l in str(e).splitlines() if "first divergence" in l or "diverged" in l]
        print(nprocs, n, per, graph, "FAIL", lines[:4] if lines else str(e)[-800:])
