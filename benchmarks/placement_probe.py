#!/usr/bin/env python3
"""Field placement lottery: K Diffusion3D models (each keeps the allocation it
gets, IGG_FIELD_PLACEMENT=1), each timed with several probe kernels
(models/diffusion3d.py _time_placements) and with the model's own captured
step, to see which probe separates the fast placements from the slow ones.

Usage: python benchmarks/placement_probe.py [--n 512] [--dtype float64] [--k 8]
       [--probes 43:3:0,43:3:1,40:4:1] [--variant 43] [--grid-rounds 3]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--dtype", default="float64")
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--probes", default="43:3:0,43:3:1,40:4:1")
    ap.add_argument("--variant", type=int, default=43)
    ap.add_argument("--grid-rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=200)
    args = ap.parse_args()
    os.environ["IGG_FIELD_PLACEMENT"] = "1"
    import torch

    import igg
    from igg.models import diffusion3d as D

    igg.init_global_grid(args.n, args.n, args.n, quiet=True)
    dtype = getattr(torch, args.dtype)
    models = []
    for i in range(args.k):
        m = D.Diffusion3D(dtype=dtype, variant=args.variant)
        m.rounds = args.grid_rounds
        models.append(m)
    probes = [tuple(int(x) for x in p.split(":")) for p in args.probes.split(",")]
    rows = {i: {} for i in range(args.k)}
    for p in probes:
        ms = D._time_placements([(m.T, m.Cp, m.T2) for m in models], dtype, v=p[0], rounds=p[1], halo_z=bool(p[2]))
        for i, t in enumerate(ms):
            rows[i][f"probe {p[0]}/r{p[1]}/hz{p[2]}"] = t
    # the model's own step (fields re-initialised by the probes: timing only)
    for m in models:
        m.capture()
    for rep in range(2):
        for i, m in enumerate(models):
            m.run(100)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            m.run(args.steps)
            b.record()
            b.synchronize()
            rows[i].setdefault("model", []).append(a.elapsed_time(b) / args.steps)
    for i in range(args.k):
        r = rows[i]
        r["model"] = min(r["model"])
        print(f"#{i} T at {models[i].T.data_ptr():#x}: " + "  ".join(f"{k} {v:.5f}" for k, v in r.items()), flush=True)
    igg.finalize_global_grid()


if __name__ == "__main__":
    main()
