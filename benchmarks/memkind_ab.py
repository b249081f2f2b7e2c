#!/usr/bin/env python3
"""A/B: the plain diffusion sweep on fields in torch's coarse-grained memory vs
native fine-grained memory vs HIP VMM memory (Diffusion3D(field_memory=...)).

The direct-z fused exchange stores into the neighbours' fields while their
kernels run, which HIP defines for fine-grained memory only
(docs/COHERENCE.md); this measures what keeping the fields there costs the
1-GPU step. Interleaved rounds, hipGraph replays, CUDA-event timing.

Round 6: VMM kinds carry the allocator's placement knobs (csrc/vmm.cpp):
"vmm:GRAN:ALIGN_MIB" sets IGG_VMM_GRAN (min|rec) and IGG_VMM_ALIGN_MIB for
that model's allocation ("vmm" = the defaults).

Usage: python benchmarks/memkind_ab.py [--n 512] [--variant 43] [--rounds 3] [--reps 3] [--steps 200]
       [--kinds torch,fine,vmm,vmm:min:0]
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
    ap.add_argument("--kinds", default="torch,fine")
    args = ap.parse_args()
    # every model keeps the allocation it gets (the lottery this measures;
    # Diffusion3D's placement probe would pick among candidates)
    os.environ.setdefault("IGG_FIELD_PLACEMENT", "1")
    import torch

    import igg
    from igg.models.diffusion3d import Diffusion3D

    igg.init_global_grid(args.n, args.n, args.n, quiet=True)
    dtype = getattr(torch, args.dtype)
    models = {}
    for i, kind in enumerate(args.kinds.split(",")):
        parts = kind.split(":")
        if len(parts) == 3:
            os.environ["IGG_VMM_GRAN"], os.environ["IGG_VMM_ALIGN_MIB"] = parts[1], parts[2]
        else:
            os.environ.pop("IGG_VMM_GRAN", None)
            os.environ.pop("IGG_VMM_ALIGN_MIB", None)
        m = Diffusion3D(dtype=dtype, variant=args.variant, field_memory=parts[0])
        kind = f"{kind}#{i}"
        print(f"{kind}: T at {m.T.data_ptr():#x}", flush=True)
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
            print(f"rep {rep} {kind:12s}: {ms:.5f} ms/step  {m.a_eff_bytes / ms / 1e6:.1f} GB/s", flush=True)
    for kind, v in res.items():
        print(f"{kind:12s}: best {min(v):.5f} median {sorted(v)[len(v) // 2]:.5f} ms/step", flush=True)
    ref = models["torch"].T.clone()
    # same physics on every memory: run all from the same state, compare bitwise
    first, *rest = models.values()
    for f in rest:
        f.T.copy_(first.T)
        f.T2.copy_(first.T2)
    for m in models.values():
        m.run(10)
    torch.cuda.synchronize()
    print("bitwise equal after 10 more steps:", all(torch.equal(first.T, f.T) for f in rest), flush=True)
    del ref
    igg.finalize_global_grid()


if __name__ == "__main__":
    main()
