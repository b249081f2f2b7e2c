#!/usr/bin/env python3
"""A/B of the plain stencil's z-edge stores (1 GPU, no exchange).

The z-edge lanes of a tile (z = 0..VZ-1 and n2-VZ..n2-1) hold one halo element
each, which the plain kernel does not write: their stores cover 8 (f64) or 12
(f32) of 16 bytes, so one cache line per row and z edge is written partially.
``halo_z=True`` (DiffusionArgs::halo_z) makes those lanes store the whole vector,
writing t's value into t2's z halo element. Timed interleaved in the time
loop's ping-pong shape, median of rounds; the fields are compared bitwise
after the same number of steps with both forms (t2's z halo equals t's here,
as in the time loop: T2 = T.clone() and nothing else writes the boundary).

Usage: python benchmarks/halo_z_ab.py [--n 512] [--dtype float64] [--variants 11,0,9,14]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from igg._native import native  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--dtype", default="float64", choices=["float64", "float32"])
    ap.add_argument("--variants", default="11,0,9,14,2,40,43,26,21")
    ap.add_argument("--rounds-list", default="1,2,3")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=7)
    a = ap.parse_args()
    n, dt = a.n, getattr(torch, a.dtype)
    g = torch.Generator(device="cpu").manual_seed(0)
    T0 = torch.rand(n, n, n, generator=g, dtype=torch.float64).to(dt).cuda()
    Cp = (torch.rand(n, n, n, generator=g, dtype=torch.float64) + 1).to(dt).cuda()
    T, T2 = T0.clone(), T0.clone()
    s = torch.cuda.current_stream()
    inner = [([1, 1, 1], [n - 1, n - 1, n - 1])]
    rd2 = [1.0, 1.0, 1.0]
    bufs = [T, T2]
    compiled = [v for v in (int(x) for x in a.variants.split(",")) if native.diffusion3d_variant_compiled(v)]

    def run(v, r, halo, k):
        for i in range(k):
            src, dst = bufs[i & 1], bufs[(i + 1) & 1]
            native.diffusion3d(dst.data_ptr(), src.data_ptr(), Cp.data_ptr(), [n, n, n], rd2, 1e-4,
                               T.element_size(), inner, True, v, s.cuda_stream, r, halo)

    # bitwise: same steps with and without
    for v in compiled:
        outs = []
        for halo in (False, True):
            T.copy_(T0)
            T2.copy_(T0)
            run(v, 1, halo, 6)
            torch.cuda.synchronize()
            outs.append((T.clone(), T2.clone()))
        same = torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
        print(f"v{v}: bitwise equal with and without the z-halo stores: {same}", flush=True)
        if not same:
            return 1
    res = {}
    for v in compiled:
        for r in (int(x) for x in a.rounds_list.split(",")):
            for halo in (False, True):
                run(v, r, halo, 4)
            times = {False: [], True: []}
            for _ in range(a.reps):
                for halo in (False, True):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    run(v, r, halo, a.steps)
                    e1.record(s)
                    e1.synchronize()
                    times[halo].append(e0.elapsed_time(e1) / a.steps)
            med = {h: sorted(t)[len(t) // 2] for h, t in times.items()}
            res[(v, r)] = med
            print(f"v{v} r{r}: partial-line z edges {med[False]:.4f} ms, whole-vector z edges {med[True]:.4f} ms "
                  f"({(med[True] / med[False] - 1) * 100:+.2f} %)", flush=True)
    best_off = min(res.items(), key=lambda kv: kv[1][False])
    best_on = min(res.items(), key=lambda kv: kv[1][True])
    print(f"best without: v{best_off[0][0]} r{best_off[0][1]} {best_off[1][False]:.4f} ms; "
          f"best with: v{best_on[0][0]} r{best_on[0][1]} {best_on[1][True]:.4f} ms", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
