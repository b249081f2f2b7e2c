#!/usr/bin/env python3
"""Time the diffusion kernel on individual boxes (slab decomposition study)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import igg  # noqa: E402
from igg._native import native  # noqa: E402
from igg.ops import stencil  # noqa: E402


def t(fn, reps=10):
    s = torch.cuda.current_stream()
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    e1.synchronize()
    return round(e0.elapsed_time(e1) / reps, 4)


n = 512
T = torch.rand((n, n, n), dtype=torch.float64, device="cuda")
Cp = 1 + torch.rand((n, n, n), dtype=torch.float64, device="cuda")
T2 = T.clone()
res = {}
import argparse  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--variants", default="11,0")
ap.add_argument("--zw", default="tile", help="z slab width: 'tile' (tile-1) or an integer")
ap.add_argument("--rounds", default="0,-4")
a = ap.parse_args()
for v in [int(x) for x in a.variants.split(",")]:
    W = native.diffusion3d_variant_tile(v)
    zw = W - 1 if a.zw == "tile" else int(a.zw)
    slabs, interior = stencil.split_boundary((n, n, n), [1, 1, 1], (1, 1, zw))
    names = ["x_lo", "x_hi", "y_lo", "y_hi", "z_lo", "z_hi"]
    for rounds in [int(x) for x in a.rounds.split(",")]:
        def run(boxes):
            return lambda: native.diffusion3d(T2.data_ptr(), T.data_ptr(), Cp.data_ptr(), [n, n, n], [1.0] * 3, 0.01,
                                              8, boxes, True, v, torch.cuda.current_stream().cuda_stream, rounds)
        r = {nm: t(run([b])) for nm, b in zip(names, slabs)}
        r["all_slabs"] = t(run(slabs))
        r["sum_separate"] = round(sum(r[nm] for nm in names), 4)
        r["interior"] = t(run([interior]))
        r["full"] = t(run([((1, 1, 1), (n - 1, n - 1, n - 1))]))
        res[f"v{v}_r{rounds}"] = r
print(json.dumps(res, indent=1))
