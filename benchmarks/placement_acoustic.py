#!/usr/bin/env python3
"""Field placement lottery of the 2-D acoustic model (8192^2 f32, six fields in
one fine-grained carve): K models, each keeping the allocation it gets, timed
by graph replays interleaved over reps (profiles/r6_placement/).

Usage: python benchmarks/placement_acoustic.py [--n 8192] [--k 12] [--steps 400] [--reps 3]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--k", type=int, default=12)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    os.environ["IGG_FIELD_PLACEMENT"] = "1"  # each model keeps the carve it gets
    import torch

    import igg
    from igg.models.acoustic2d import Acoustic2D

    igg.init_global_grid(args.n, args.n, 1, quiet=True)
    models = [Acoustic2D() for _ in range(args.k)]
    for m in models:
        m.capture()
    res = [[] for _ in models]
    for _ in range(args.reps):
        for i, m in enumerate(models):
            m.run(100)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            m.run(args.steps)
            b.record()
            b.synchronize()
            res[i].append(a.elapsed_time(b) / args.steps)
    for i, m in enumerate(models):
        print(f"#{i} P at {m.P.data_ptr():#x}: best {min(res[i]):.5f} median {sorted(res[i])[len(res[i]) // 2]:.5f} "
              f"ms/step", flush=True)
    igg.finalize_global_grid()


if __name__ == "__main__":
    main()
