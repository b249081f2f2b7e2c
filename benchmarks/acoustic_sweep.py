#!/usr/bin/env python3
"""Time the 2-D acoustic kernel variants / marching chunk lengths at 8192^2 f32."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import igg  # noqa: E402
from igg._native import native  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
dt = getattr(torch, sys.argv[2]) if len(sys.argv) > 2 else torch.float32
P = torch.rand(n, n, dtype=dt, device="cuda")
Vx = torch.rand(n + 1, n, dtype=dt, device="cuda")
Vy = torch.rand(n, n + 1, dtype=dt, device="cuda")
P2, Vx2, Vy2 = torch.empty_like(P), torch.empty_like(Vx), torch.empty_like(Vy)
s = torch.cuda.current_stream()


def run():
    native.acoustic2d(P2.data_ptr(), Vx2.data_ptr(), Vy2.data_ptr(), P.data_ptr(), Vx.data_ptr(), Vy.data_ptr(), n, n,
                      0.01, 0.01, 10.0, 10.0, P.element_size(), True, s.cuda_stream)


res = {}
chs = [int(x) for x in os.environ.get("CHS", "8,16,32,64").split(",")]
for v, ch in [(0, 0)] + [(1, c) for c in chs] + [(2, c) for c in chs]:
    native.acoustic2d_set_variant(v)
    native.acoustic2d_set_chunk(ch)
    run()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(10):
            run()
        e1.record(s)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / 10)
    ms = sorted(ts)[2]
    res[f"v{v}_ch{ch}"] = {"ms": round(ms, 4), "GBs": round(2 * (P.numel() + Vx.numel() + Vy.numel()) * P.element_size() / ms / 1e6, 1)}
native.acoustic2d_set_variant(2)
native.acoustic2d_set_chunk(0)
print(json.dumps(res))
