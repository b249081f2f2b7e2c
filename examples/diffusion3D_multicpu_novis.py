#!/usr/bin/env python3
"""3-D heat diffusion on multiple CPU processes, no visualisation.

Counterpart of the reference's examples/diffusion3D_multicpu_novis.jl: the same
application code as the GPU example on host tensors (device_type="none"): the
fused stencil runs as the native C++ host kernel, halos move over gloo.

    torchrun --standalone --local-addr 127.0.0.1 --nproc-per-node 8 \\
        examples/diffusion3D_multicpu_novis.py --nx 32 --nt 100
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import igg  # noqa: E402
from igg.models.diffusion3d import Diffusion3D, t_eff_gbs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nx", type=int, default=32)
    ap.add_argument("--nt", type=int, default=100)
    a = ap.parse_args()
    import torch

    me, dims, nprocs, coords, comm = igg.init_global_grid(a.nx, a.nx, a.nx, device_type="none")
    model = Diffusion3D(dtype=torch.float64, device="cpu")
    igg.tic()
    model.run(a.nt)
    t = igg.toc()
    # Global maximum over the ranks through the grid's communicator (the
    # reference apps call MPI.Allreduce on comm_cart for such diagnostics).
    t_max = comm.allreduce_(model.T.max().reshape(1).clone(), "max")
    if me == 0:
        t_it = t / a.nt
        print(f"{nprocs} process(es) {dims.tolist()}: {t:.3f} s, {t_it * 1e3:.3f} ms/step, "
              f"T_eff = {t_eff_gbs(model, t_it):.2f} GB/s per process, global T_max = {float(t_max):.6f}")
    igg.finalize_global_grid()


if __name__ == "__main__":
    main()
