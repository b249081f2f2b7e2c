#!/usr/bin/env python3
"""Price the stencil's tile-edge re-fetch (timing probe; probe results are wrong
on purpose): tiling 40 (v2_by4_ry8, lane-distributed z-segment edges, one
workgroup per CU) as is (124), without its z-segment edge loads (130), without
its y-halo row loads (131), and without both (132). Ping-pong launches on two
512^3 f64 buffers, interleaved, median of rounds.

Usage: python profiles/r2_refetch/refetch_probe.py [--n 512] [--rounds-grid 2,3]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import igg  # noqa: E402,F401
from igg._native import native  # noqa: E402

NAMES = {124: "tiling 40", 130: "no z-edge loads", 131: "no y-halo loads", 132: "neither"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--rounds-grid", default="2,3")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--repeat", type=int, default=5)
    a = ap.parse_args()
    n = a.n
    T = torch.rand(n, n, n, dtype=torch.float64, device="cuda")
    T2 = T.clone()
    Cp = T + 1
    s = torch.cuda.current_stream()
    cands = [(t, int(r)) for r in a.rounds_grid.split(",") for t in NAMES]
    res = {c: [] for c in cands}

    def run(c):
        t, r = c
        for k in range(a.steps):
            src, dst = (T, T2) if k % 2 == 0 else (T2, T)
            native.diffusion3d_hx_tiling(dst.data_ptr(), src.data_ptr(), Cp.data_ptr(), [n] * 3, [1.0] * 3, 1e-4, 8,
                                         t, s.cuda_stream, r)

    for c in cands:
        run(c)
    torch.cuda.synchronize()
    for _ in range(a.repeat):
        for c in cands:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run(c)
            e1.record()
            e1.synchronize()
            res[c].append(e0.elapsed_time(e1) / a.steps)
    for (t, r), v in sorted(res.items(), key=lambda kv: (kv[0][1], kv[0][0])):
        v = sorted(v)
        print(f"rounds {r} tiling {t:3d} {NAMES[t]:17s} {v[len(v) // 2]:.4f} ms (min {v[0]:.4f})", flush=True)


if __name__ == "__main__":
    main()
