import sys
sys.path.insert(0, "/root/repo")
from tests._mp import run_ranks
for nprocs, n, graph in [(4, 64, 0), (4, 64, 1), (2, 64, 1), (4, 512, 1)]:
    try:
        outs = run_ranks(nprocs, "put_after_model", n, graph, 21, env_extra={"IGG_TRANSPORT": "staged", "IGG_PUT_TIMEOUT": "20", "GPU_MAX_HW_QUEUES": "1"}, timeout=100)
        print(nprocs, n, graph, "OK")
    except AssertionError as e:
        print(nprocs, n, graph, "FAIL", str(e)[-1500:])
