#!/usr/bin/env python3
"""Time update_halo_ alone on one GPU in loopback mode (interior-rank workload).

Usage: [IGG_TRANSPORT=put|rccl] [IGG_HALO_MODE=...] [IGG_PACK=kernel|memcpy2d]
       python benchmarks/halo_only.py [--n 512] [--reps 50] [--self]
(--self: no loopback, the in-place self-periodic exchange of a 1-process grid)
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import igg  # noqa: E402
from igg.parallel import halo as H  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--dims", default="1,1,1", help="loopback dims (x,y,z)")
    ap.add_argument("--self", action="store_true")
    a = ap.parse_args()
    n = a.n
    igg.init_global_grid(n, n, n, periodx=1, periody=1, periodz=1, quiet=True)
    if not a.self:
        H.enable_loopback(tuple(bool(int(v)) for v in a.dims.split(",")))
    T = torch.rand(n, n, n, dtype=torch.float64, device="cuda")
    for _ in range(3):
        igg.update_halo_(T)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        igg.update_halo_(T)
    e1.record()
    e1.synchronize()
    print(f"transport={H.engine().transport_name(True)} mode={H.halo_mode()} "
          f"pack={','.join(H.pack_mode(d) for d in (1, 2, 3))} self={a.self} "
          f"msgs={H.engine().last_message_count} halo_us={e0.elapsed_time(e1) / a.reps * 1e3:.1f}", flush=True)
    igg.finalize_global_grid()


if __name__ == "__main__":
    main()
