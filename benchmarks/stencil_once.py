#!/usr/bin/env python3
"""Run selected stencil variants a few times on n^3 (for rocprofv3 counters)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import igg  # noqa: E402
from igg._native import native  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=512)
ap.add_argument("--variants", default="0")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--dtype", default="float64")
ap.add_argument("--rounds", default="0", help="grid residency rounds per launch (list; 0 = default)")
ap.add_argument("--calib", action="store_true", help="also run T2.copy_(T) (known bytes) for counter calibration")
ap.add_argument("--placement", action="store_true",
                help="fields on the fastest of the placement probe's candidate carves (utils/placement.py)")
a = ap.parse_args()
dt = getattr(torch, a.dtype)
n = a.n
if a.placement:
    from igg.models import diffusion3d as D
    from igg.utils import placement as PL

    class _G:
        nprocs = 1

    nb = n ** 3 * torch.empty(0, dtype=dt).element_size()
    (T, Cp, T2), rec = PL.placed(lambda: [torch.empty((n, n, n), dtype=dt, device="cuda") for _ in range(3)],
                                 PL.candidate_count(_G(), nb, 3 * nb, torch.device("cuda")),
                                 lambda c: D._time_placements(c, dt))
    print(f"placement: chosen {rec['chosen']} of {rec['candidates']}: {min(rec['ms']):.5f} .. {max(rec['ms']):.5f} ms",
          flush=True)
    g = torch.Generator(device="cpu").manual_seed(0)
    T.copy_(torch.rand((n, n, n), generator=g, dtype=torch.float64).to(dt))
    Cp.copy_(1 + torch.rand((n, n, n), generator=g, dtype=torch.float64).to(dt))
    T2.copy_(T)
else:
    T = torch.rand((n, n, n), dtype=dt, device="cuda")
    Cp = 1 + torch.rand((n, n, n), dtype=dt, device="cuda")
    T2 = T.clone()
s = torch.cuda.current_stream().cuda_stream
for v in [int(x) for x in a.variants.split(",")]:
    for gr in [int(x) for x in a.rounds.split(",")]:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            native.diffusion3d(T2.data_ptr(), T.data_ptr(), Cp.data_ptr(), [n, n, n], [1.0, 1.0, 1.0], 0.01,
                               T.element_size(), [((1, 1, 1), (n - 1, n - 1, n - 1))], True, v, s, gr)
        e1.record()
        e1.synchronize()
        print(f"variant {v} rounds {gr}: {e0.elapsed_time(e1) / a.reps:.5f} ms per launch", flush=True)
if a.calib:
    for _ in range(a.reps):
        T2.copy_(T)  # reads n^3 and writes n^3 elements
torch.cuda.synchronize()
print("done")
