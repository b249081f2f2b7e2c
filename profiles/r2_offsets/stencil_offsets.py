#!/usr/bin/env python3
"""Does the relative placement of T, Cp and T2 in HBM change the stencil time?

All three arrays are carved from one allocation with configurable byte gaps
(channel/bank alignment study); variants are timed interleaved, median of rounds.

Usage: python profiles/r2_offsets/stencil_offsets.py [--n 512] [--variants 0,11] [--gaps 0,4096,65536,...]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import igg  # noqa: E402
from igg._native import native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--variants", default="0,11")
    ap.add_argument("--gaps", default="0,4096,8192,65536,266240,1052672,2101248")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--pingpong", action="store_true",
                    help="alternate T2=f(T) and T=f(T2) like the time loop (default: T2=f(T) only)")
    ap.add_argument("--grid-rounds", type=int, default=0, help="grid residency rounds of each launch")
    a = ap.parse_args()
    n = a.n
    numel = n ** 3
    gaps = [int(g) for g in a.gaps.split(",")]
    variants = [int(v) for v in a.variants.split(",")]
    maxgap = max(gaps)
    buf = torch.empty(3 * numel * 8 + 3 * maxgap + 4096, dtype=torch.uint8, device="cuda")
    base = buf.data_ptr()
    res = {}
    s = torch.cuda.current_stream()
    for g in gaps:
        offs = [0, numel * 8 + g, 2 * (numel * 8 + g)]
        views = [buf[o:o + numel * 8].view(torch.float64).view(n, n, n) for o in offs]
        T, Cp, T2 = views
        T.uniform_()
        Cp.fill_(1.5)
        for v in variants:
            k = [0]

            def run():
                src, dst = (T2, T) if (a.pingpong and k[0] % 2) else (T, T2)
                k[0] += 1
                native.diffusion3d(dst.data_ptr(), src.data_ptr(), Cp.data_ptr(), [n, n, n], [1.0] * 3, 1e-4, 8,
                                   [((1, 1, 1), (n - 1, n - 1, n - 1))], True, v, s.cuda_stream, a.grid_rounds)
            run()
            ts = []
            for _ in range(a.rounds):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(a.reps):
                    run()
                e1.record(s)
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) / a.reps)
            res[f"gap{g}_v{v}"] = round(statistics.median(ts), 4)
    print(json.dumps({"base_mod_2M": base % (1 << 21), "ms": res}))


if __name__ == "__main__":
    main()
