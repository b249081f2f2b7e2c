import sys
sys.path.insert(0, ".")
from tests._mp import run_ranks
cases = [("auto", {}, 1), ("one", {"IGG_HALO_MODE": "onephase"}, 1), ("auto", {}, 1), ("one", {"IGG_HALO_MODE": "onephase"}, 1),
         ("auto_noov", {}, 0), ("one_noov", {"IGG_HALO_MODE": "onephase"}, 0), ("auto", {}, 1)]
for name, env, ov in cases:
    try:
        run_ranks(8, "diffusion", "gpu", 24, 20, 18, 5, ov, env_extra={"IGG_TRANSPORT": "staged", **env}, timeout=100)
        print(name, "OK", flush=True)
    except AssertionError as e:
        lines = [l.split("mismatch")[1] for l in str(e).splitlines() if "mismatch" in l and "AssertionError" in l]
        print(name, "FAIL", lines[:8], flush=True)
