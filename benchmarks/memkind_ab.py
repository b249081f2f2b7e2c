#!/usr/bin/env python3
"""A/B: the plain diffusion sweep on fields in torch's coarse-grained memory vs
native fine-grained memory (Diffusion3D(field_memory=...)).

The direct-z fused exchange stores into the neighbours' fields while their
kernels run, which HIP defines for fine-grained memory only
(docs/COHERENCE.md); this measures what keeping the fields there costs the
1-GPU step. Interleaved rounds, hipGraph replays, CUDA-event timing.

Usage: python benchmarks/memkind_ab.py [--n 512] [--variant 43] [--rounds 3] [--reps 3] [--steps 200]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--variant", type=int, default=43)
    ap.add_argument("--grid-rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--dtype", default="float64")
    args = ap.parse_args()
    import torch

    import igg
    from igg.models.diffusion3d import Diffusion3D

    igg.init_global_grid(args.n, args.n, args.n, quiet=True)
    dtype = getattr(torch, args.dtype)
    models = {}
    for kind in ("torch", "fine"):
        m = Diffusion3D(dtype=dtype, variant=args.variant, field_memory=kind)
        m.rounds = args.grid_rounds
        m.capture()
        models[kind] = m
    res = {k: [] for k in models}
    for rep in range(args.reps):
        for kind, m in models.items():
            m.run(100)  # warm (>40 ms of load)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            a.record()
            m.run(args.steps)
            b.record()
            torch.cuda.synchronize()
            ms = a.elapsed_time(b) / args.steps
            res[kind].append(ms)
            print(f"rep {rep} {kind:5s}: {ms:.5f} ms/step  {m.a_eff_bytes / ms / 1e6:.1f} GB/s", flush=True)
    for kind, v in res.items():
        print(f"{kind:5s}: best {min(v):.5f} median {sorted(v)[len(v) // 2]:.5f} ms/step", flush=True)
    ref = models["torch"].T.clone()
    # same physics on both memories: run both from the same state, compare bitwise
    f = models["fine"]
    f.T.copy_(models["torch"].T)
    f.T2.copy_(models["torch"].T2)
    models["torch"].run(10)
    f.run(10)
    torch.cuda.synchronize()
    print("bitwise equal after 10 more steps:", bool(torch.equal(models["torch"].T, f.T)), flush=True)
    del ref
    igg.finalize_global_grid()


if __name__ == "__main__":
    main()
