#!/usr/bin/env python3
"""Interleaved timing of stencil variants x grid rounds on the 512^3 inner box
(the model autotune's measurement, over an arbitrary candidate list)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import igg  # noqa: E402, F401
from igg.ops import stencil  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=512)
ap.add_argument("--variants", default="11,21,23,24,25,26,27,28,29,30,31")
ap.add_argument("--rounds", default="1,2,3")
ap.add_argument("--dtype", default="float64")
ap.add_argument("--repeat", type=int, default=3)
a = ap.parse_args()
n, dt = a.n, getattr(torch, a.dtype)
T = torch.rand(n, n, n, dtype=dt, device="cuda")
Cp, T2 = T + 1, T.clone()
boxes = [([1, 1, 1], [n - 1, n - 1, n - 1])]
cands = [(int(v), int(r)) for v in a.variants.split(",") for r in a.rounds.split(",")]
names = stencil.variants()
acc = {c: [] for c in cands}
for _ in range(a.repeat):
    t = stencil.time_variants(T2, T, Cp, [1.0] * 3, 1e-4, boxes, cands, reps=5, rounds=3)
    for c, v in t.items():
        acc[c].append(v)
for c in sorted(cands, key=lambda c: sorted(acc[c])[len(acc[c]) // 2]):
    ms = sorted(acc[c])[len(acc[c]) // 2]
    print(f"{c[0]:3d} {names[c[0]]:<24s} r{c[1]}  {ms:.4f} ms  {3 * n**3 * T.element_size() / ms / 1e6:7.0f} GB/s")
