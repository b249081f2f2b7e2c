#!/usr/bin/env python3
"""Run a few overlapped loopback diffusion steps for a kernel-trace timeline
(use under `rocprofv3 --kernel-trace --output-format csv`), then analyse with
benchmarks/timeline.py."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import igg  # noqa: E402
from igg.models.diffusion3d import Diffusion3D  # noqa: E402
from igg.parallel import halo as H  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=512)
ap.add_argument("--steps", type=int, default=6)
ap.add_argument("--ir", type=int, default=-2)
ap.add_argument("--hv", type=int, default=18)
ap.add_argument("--hr", type=int, default=-1)
ap.add_argument("--interior-first", type=int, default=0)
ap.add_argument("--no-loopback", action="store_true")
ap.add_argument("--cu", type=int, default=0)
a = ap.parse_args()
igg.init_global_grid(a.n, a.n, a.n, quiet=True)
if not a.no_loopback:
    H.enable_loopback()
m = Diffusion3D(dtype=torch.float64, overlap=True, interior_rounds=a.ir, halo_variant=a.hv, halo_rounds=a.hr, reserve_cus=a.cu)
m.interior_first = bool(a.interior_first)
for _ in range(3):
    m.step()
torch.cuda.synchronize()
for _ in range(a.steps):
    m.step()
torch.cuda.synchronize()
print("done")
igg.finalize_global_grid()
