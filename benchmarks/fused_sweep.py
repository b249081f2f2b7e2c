#!/usr/bin/env python3
"""Cost of the fused halo exchange per stencil variant (1 GPU, self as peer).

For each fused-capable variant: plain inner-box stencil, fused stencil + sync
with 6 active sides (interior rank of a periodic 3-D decomposition) and with 3
active sides (low side of every dim: a corner rank of 2x2x2), and the sync
kernel alone. The 3-side case reads its halos from arena regions nobody writes
(timing only). Times are CUDA-event medians per step.

Usage: python benchmarks/fused_sweep.py [--n 512] [--reps 20] [--variants 0,2,9,11,14]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import igg  # noqa: E402
from igg._native import native  # noqa: E402


# fused-only tilings -> the plain stencil variant with the same tiling
PLAIN_OF = {50: 0, 55: 0, 41: 40, 42: 40}


def timed(fn, reps):
    s = torch.cuda.current_stream()
    fn()
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            fn()
        e1.record(s)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / reps)
    return sorted(ts)[1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--variants", default="0,2,9,11,14")
    ap.add_argument("--dtype", default="float64")
    ap.add_argument("--grid", action="store_true",
                    help="grid search: rounds x send mode for fused3/fused6 of each variant")
    a = ap.parse_args()
    n = a.n
    igg.init_global_grid(n, n, n, periodx=1, periody=1, periodz=1, quiet=True)
    dt = getattr(torch, a.dtype)
    T = torch.rand(n, n, n, dtype=dt, device="cuda")
    T2 = T.clone()
    Cp = torch.rand(n, n, n, dtype=dt, device="cuda") + 1
    rd2 = [1.0, 1.0, 1.0]
    eb = T.element_size()
    s = torch.cuda.current_stream().cuda_stream
    inner = [([1, 1, 1], [n - 1, n - 1, n - 1])]
    mesh = native.PeerMesh(0, 1, lambda b: [bytes(b)])
    fh6 = native.FusedHalo(mesh, [n, n, n], eb, [[0, 0], [0, 0], [0, 0]])
    fh3 = native.FusedHalo(mesh, [n, n, n], eb, [[0, -1], [0, -1], [0, -1]])
    fh0 = native.FusedHalo(mesh, [n, n, n], eb, [[-1, -1], [-1, -1], [-1, -1]])
    fhx = {d: native.FusedHalo(mesh, [n, n, n], eb, [[0, -1] if k == d else [-1, -1] for k in range(3)])
           for d in range(3)}
    print(f"n={n}^3 {a.dtype}, ms per step (median of 3 x {a.reps})")
    print("sync kernel alone: %.4f ms" % timed(lambda: fh6.sync(s), a.reps))
    k = [0]

    def fused(fh, v, rounds=0, mode=0):
        def f():
            fh.step(T2.data_ptr(), T.data_ptr(), Cp.data_ptr(), rd2, 1e-4, v, k[0], True, s, rounds, mode)
            k[0] += 1
        return f

    if a.grid:
        for v in (int(x) for x in a.variants.split(",")):
            pv = PLAIN_OF.get(v, v)
            for rounds in (1, 2, 3, 4):
                base = timed(lambda: native.diffusion3d(T2.data_ptr(), T.data_ptr(), Cp.data_ptr(), [n, n, n], rd2,
                                                        1e-4, eb, inner, True, pv, s, rounds), a.reps)
                row = [f"plain {base:.4f}"]
                for mode in (0, 1):
                    t0 = timed(fused(fh0, v, rounds, mode), a.reps)
                    t3 = timed(fused(fh3, v, rounds, mode), a.reps)
                    t6 = timed(fused(fh6, v, rounds, mode), a.reps)
                    row.append(f"m{mode}: none {t0:.4f} f3 {t3:.4f} f6 {t6:.4f}")
                print(f"variant {v:2d} rounds {rounds}: " + " | ".join(row), flush=True)
        mesh.check_error()
        igg.finalize_global_grid()
        return

    for v in (int(x) for x in a.variants.split(",")):
        base = timed(lambda: native.diffusion3d(T2.data_ptr(), T.data_ptr(), Cp.data_ptr(), [n, n, n], rd2, 1e-4, eb,
                                                inner, True, v, s), a.reps)
        t0 = timed(fused(fh0, v), a.reps)
        t6 = timed(fused(fh6, v), a.reps)
        t3 = timed(fused(fh3, v), a.reps)
        tx = [timed(fused(fhx[d], v), a.reps) for d in range(3)]
        print(f"variant {v:2d} {native.diffusion3d_variants()[v]:<20s} plain {base:.4f}  no-role +{(t0 - base) * 1e3:.1f} us  fused6 {t6:.4f} "
              f"(+{(t6 - base) * 1e3:.1f} us)  fused3 {t3:.4f} (+{(t3 - base) * 1e3:.1f} us)  "
              f"x-only +{(tx[0] - base) * 1e3:.1f}  y-only +{(tx[1] - base) * 1e3:.1f}  z-only +{(tx[2] - base) * 1e3:.1f} us",
              flush=True)
    mesh.check_error()
    igg.finalize_global_grid()


if __name__ == "__main__":
    main()
