#!/usr/bin/env python3
"""Ping-pong timing of restrict-form plain tilings (fused_kernels.hip
dispatch_plain ids) on the model's own 512^3 f64 buffers, interleaved, median
of repeats; each tiling's result is checked bitwise against tiling 11 first.

Usage: python profiles/r2_fullrow/tiling_probe.py --tilings 11,124,140,141 [--rounds-grid 1,2,3]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import igg  # noqa: E402
from igg._native import native  # noqa: E402
from igg.models.diffusion3d import Diffusion3D  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--tilings", default="11,124,140,141,142,143,144,145")
    ap.add_argument("--rounds-grid", default="1,2,3")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--repeat", type=int, default=5)
    a = ap.parse_args()
    n = a.n
    igg.init_global_grid(n, n, n, quiet=True)
    m = Diffusion3D(dtype=torch.float64)
    T, T2, Cp = m.T, m.T2, m.Cp
    T2.copy_(T)
    s = torch.cuda.current_stream()
    rd2 = [1.0 / (m.dx * m.dx), 1.0 / (m.dy * m.dy), 1.0 / (m.dz * m.dz)]
    dtlam = m.dt * m.lam

    def launch(t, dst, src, r):
        native.diffusion3d_hx_tiling(dst.data_ptr(), src.data_ptr(), Cp.data_ptr(), [n] * 3, rd2, dtlam, 8, t,
                                     s.cuda_stream, r)

    tilings = [int(x) for x in a.tilings.split(",")]
    ref = T.clone()
    launch(11, ref, T, 3)
    for t in tilings:
        B = T.clone()
        launch(t, B, T, 3)
        torch.cuda.synchronize()
        print(f"bitwise tiling {t} vs 11: {torch.equal(B, ref)}", flush=True)
        del B
    del ref
    cands = [(t, int(r)) for r in a.rounds_grid.split(",") for t in tilings]
    res = {c: [] for c in cands}

    def run(c):
        t, r = c
        for k in range(a.steps):
            src, dst = (T, T2) if k % 2 == 0 else (T2, T)
            launch(t, dst, src, r)

    backup = T.clone()
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
    T.copy_(backup)
    for (t, r), v in sorted(res.items(), key=lambda kv: (kv[0][1], kv[0][0])):
        v = sorted(v)
        print(f"rounds {r} tiling {t:3d} {v[len(v) // 2]:.4f} ms/step (min {v[0]:.4f})", flush=True)
    igg.finalize_global_grid()


if __name__ == "__main__":
    main()
