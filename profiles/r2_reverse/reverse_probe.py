#!/usr/bin/env python3
"""Alternating march direction in the ping-pong loop (FEAT 65536, fused_impl.hpp
hx_sweep): every other step runs its chunks from the top x down and marches each
chunk from high x to low, so it starts on the planes the previous step touched
last (still in the memory-side Infinity Cache if it keeps them). Forward/forward
vs forward/reversed pairs of the same tiling, on the model's own buffers
(Diffusion3D placement), interleaved, median of repeats; plus a bitwise check of
the reversed sweep against the forward one.

Usage: python profiles/r2_reverse/reverse_probe.py [--n 512] [--rounds-grid 2,3]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import igg  # noqa: E402
from igg._native import native  # noqa: E402
from igg.models.diffusion3d import Diffusion3D  # noqa: E402

# forward restrict-form tiling -> its reversed-march instantiation
PAIRS = {0: 200, 11: 211, 100: 300, 124: 324, 411: 611}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--rounds-grid", default="2,3")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--repeat", type=int, default=7)
    ap.add_argument("--tilings", default="0,11,100,124,411")
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

    # bitwise: reversed sweep == forward sweep (same arithmetic order)
    for f, rv in PAIRS.items():
        A, B = torch.empty_like(T), torch.empty_like(T)
        A.copy_(T)
        B.copy_(T)
        launch(f, A, T, 3)
        launch(rv, B, T, 3)
        torch.cuda.synchronize()
        print(f"bitwise tiling {f} vs reversed {rv}: {torch.equal(A, B)}", flush=True)
        del A, B

    tilings = [int(x) for x in a.tilings.split(",")]
    cands = [(t, alt, int(r)) for r in a.rounds_grid.split(",") for t in tilings for alt in (False, True)]
    res = {c: [] for c in cands}

    def run(c):
        t, alt, r = c
        for k in range(a.steps):
            src, dst = (T, T2) if k % 2 == 0 else (T2, T)
            launch(PAIRS[t] if (alt and k % 2 == 1) else t, dst, src, r)

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
    # per-direction times: an event between every launch (T2 = f(T) steps vs T = f(T2) steps)
    per = {c: ([], []) for c in cands}
    for _ in range(3):
        for c in cands:
            t, alt, r = c
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
            ev[0].record()
            for k in range(a.steps):
                src, dst = (T, T2) if k % 2 == 0 else (T2, T)
                launch(PAIRS[t] if (alt and k % 2 == 1) else t, dst, src, r)
                ev[k + 1].record()
            ev[-1].synchronize()
            for k in range(a.steps):
                per[c][k % 2].append(ev[k].elapsed_time(ev[k + 1]))
    T.copy_(backup)
    for c, v in sorted(res.items(), key=lambda kv: (kv[0][2], kv[0][0], kv[0][1])):
        t, alt, r = c
        v = sorted(v)
        e, o = (sorted(x)[len(x) // 2] for x in per[c])
        print(f"rounds {r} tiling {t:3d} {'fwd/rev' if alt else 'fwd/fwd'} {v[len(v) // 2]:.4f} ms/step "
              f"(min {v[0]:.4f}); T2=f(T) {e:.4f}, T=f(T2) {o:.4f}", flush=True)
    m.close() if hasattr(m, "close") else None
    igg.finalize_global_grid()


if __name__ == "__main__":
    main()
